/* ORACLE — test infrastructure, NOT product code.
 *
 * A single-environment fp64 CPU restatement of the reference hot path:
 *   PickPlaceGymEnv.step (mujoco_manip/gym_env.py:536-581)
 *     -> decode_action (gym_env.py:252-281, pose_utils.py:85-209)
 *     -> 16 x (IKController.compute controller.py:87-137 ; mujoco.mj_step env.py:119-121)
 *     -> mujoco.mj_forward (gym_env.py:560) -> reward (gym_env.py:352-470) -> obs (gym_env.py:283-339)
 *   plus reset / randomization (gym_env.py:477-534, randomization.py:11-98) and the FSM expert
 *   (pick_and_place.py:167-291).
 *
 * mj_step / mj_forward / mj_jac live in the un-vendored third-party library
 * mujoco==3.5.0 (uv.lock:985-986).  Its published algorithm (MuJoCo documentation,
 * "Computation" chapter) is restated here: kinematics, CRBA, RNE, tendon/actuation,
 * passive damping, collision (plane-box, plane-convex, box-box, GJK/EPA), soft
 * constraints (solref/solimp impedance, pyramidal cones, invweight0 regularizer),
 * the primal Newton solver with exact line search, and the implicitfast integrator.
 * Physics parity against MuJoCo itself is UNPINNED (MuJoCo is absent in this image);
 * the pure-math parts are pinned against golden vectors generated from the reference
 * Python (tests/golden/).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 */
#ifndef ORACLE_H
#define ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAXCON 96
#define OR_MAXEFC 640

typedef struct or_env or_env;

/* lifecycle */
or_env* or_create(int action_mode, int reward_type, int max_episode_steps, int randomize,
                  const double* spawn_x, const double* spawn_y, int image_size);
void or_destroy(or_env* e);
void or_set_task_pool(or_env* e, int n, const int* obj_idx, const int* bin_idx);
void or_set_fixed_task(or_env* e, int obj, int bin); /* -1,-1 clears */

/* gym API: seed_given=0 keeps the RNG stream (gym semantics).  task_obj/bin = -1: no override */
int or_reset(or_env* e, int seed_given, uint64_t seed, int task_obj, int task_bin, float* obs85); /* -1: sampling exhausted */
/* returns reward; writes terminated/truncated/success flags and reward_components[6] */
double or_step(or_env* e, const float* action, float* obs85, int* terminated, int* truncated,
               int* success, float* reward_components);

/* physics-level */
void or_reset_keyframe(or_env* e);           /* mj_resetDataKeyframe + mj_forward */
void or_mj_step(or_env* e);                  /* one mj_step */
void or_mj_forward(or_env* e);               /* mj_forward */
void or_ik_compute(or_env* e, const double* target, double* q_target); /* controller.py:87-137 */
int or_ik_reached(or_env* e, const double* target);                    /* controller.py:139-145 */
void or_set_arm_ctrl(or_env* e, const double* q);
void or_set_gripper(or_env* e, int open);

/* FSM expert (pick_and_place.py) */
void or_fsm_init(or_env* e, int n_tasks, const int* obj_idx, const int* bin_idx);
int or_fsm_plan(or_env* e, int n_steps);     /* returns state after plan */
void or_fsm_actuate(or_env* e);
void or_fsm_get(or_env* e, int* state, int* task_index, int* settle, double* target, int* gripper_open);

/* state access (arrays sized nq/nv/nu) */
void or_get_state(or_env* e, double* qpos, double* qvel, double* ctrl, double* qacc_ws);
void or_set_state(or_env* e, const double* qpos, const double* qvel, const double* ctrl, const double* qacc_ws);
void or_get_body(or_env* e, int body, double* xpos, double* xmat);
int or_ncon(or_env* e);
int or_nefc(or_env* e);
void or_get_contact(or_env* e, int i, int* geom, double* dist, double* pos, double* frame);
void or_get_efc_force(or_env* e, double* f);
double or_solver_residual(or_env* e);
/* Newton tolerance / iteration cap (defaults 1e-13 / 200 for the parity tests; MuJoCo's defaults
 * are 1e-8 / 100, which the CPU baseline uses) and (solves, iterations) counted since creation */
void or_set_solver(or_env* e, double tol, int maxiter);
/* MuJoCo's convergence tests at opt.tolerance mj_tol (0 = off, the default): after each Newton
 * iteration stop when scale * (cost decrease) < mj_tol or scale * |gradient| < mj_tol, scale =
 * 1 / (meaninertia * nv) (mj_solNewton, recorded per iteration in mjSolverStat.improvement /
 * .gradient) */
void or_set_solver_mj(or_env* e, double mj_tol);
void or_solver_stats(or_env* e, long* calls, long* iters);
/* constraint rows of the last solve: type (0 equality, 1 limit, 2 contact edge), pos, R, aref;
 * returns nefc (NULL skips a field; arrays hold OR_MAXEFC) */
int or_get_efc(or_env* e, int* type, double* pos, double* R, double* aref);
void or_get_qacc(or_env* e, double* qacc);
void or_get_mass_matrix(or_env* e, double* M); /* qM (dense NV x NV, CRBA + armature) of the last forward */
void or_get_smooth(or_env* e, double* bias, double* act, double* passive, double* qacc_smooth, double* constraint,
                   double* act_force); /* smooth-force terms of the last forward */
void or_get_obs(or_env* e, float* obs85);
void or_get_initial_ee(or_env* e, double* T16);
int or_step_count(or_env* e);
void or_get_task(or_env* e, int* obj, int* bin);
void or_get_hwm(or_env* e, double* hwm5);

/* pure math (golden-vector checks) */
void or_orientation_error(const double* R_cur, const double* R_tgt, double* err3);
void or_ik_math(const double* J6x7, const double* ee_pos, const double* ee_xmat, const double* q7,
                const double* target, const double* jnt_range7x2, double* q_out);
void or_rotmat_to_quat_xyzw(const double* R, double* q);
void or_quat_xyzw_to_rotmat(const double* q, double* R);
void or_rotmat_from_6d(const double* d6, double* R);
void or_decode_action(int mode, const float* action, const double* T_init, double* target, double* grip);

/* numpy-compatible RNG (gymnasium np_random = Generator(PCG64(SeedSequence(seed)))) */
typedef struct { uint64_t s_hi, s_lo, i_hi, i_lo; int has32; uint32_t buf32; } or_pcg64;
void or_seedseq_state(const uint32_t* entropy, int n_entropy, const uint32_t* spawn_key, int n_spawn,
                      uint32_t* out, int n_out);
void or_pcg64_seed(or_pcg64* r, uint64_t seed);
uint64_t or_pcg64_next64(or_pcg64* r);
double or_pcg64_double(or_pcg64* r);
int64_t or_pcg64_integers(or_pcg64* r, int64_t high);
uint32_t or_episode_seed(uint64_t root_seed, int index); /* SeedSequence(root).spawn(N)[i].generate_state(1)[0] */
int or_sample_positions(or_pcg64* r, const double* xr, const double* yr, double min_sep, double* xy6);

/* test hooks (golden-trace replay) */
void or_debug_set_xpos(or_env* e, int body, const double* p);
void or_debug_set_contacts(or_env* e, int n, const int* pairs);
void or_debug_set_episode(or_env* e, int obj, int bin, const double* T16);
double or_debug_reward(or_env* e, int* success);

#ifdef __cplusplus
}
#endif
#endif
