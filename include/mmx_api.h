/* mmx_api.h — C-ABI of the MI355X batched pick-and-place simulator (libmmx.so).
 *
 * The reference path sits behind the Gymnasium Env API of PickPlaceGymEnv
 * (mujoco_manip/gym_env.py:39-602) and, below it, the MuJoCo C API reached through
 * pybind11 (mujoco.mj_step env.py:121, mj_forward gym_env.py:560, mj_jac controller.py:101).
 * This header is the boundary a host binding (ctypes here; cgo/JNI/N-API elsewhere) binds
 * to.  Plain C: no C++ or torch types, plain pointers and sizes.
 *
 * Conventions
 *  - every function returns 0 on success or a negative MMX_E* code and never aborts;
 *    mmx_last_error() gives a message;
 *  - device buffers are fp32/int32, env-major (one contiguous record per env, matching a
 *    torch [N, F] tensor): element (env i, field f) is at ptr[i * F + f];
 *  - sim-owned buffers returned by mmx_get_buffers stay valid until mmx_destroy;
 *  - all launches are asynchronous on the sim's stream (cfg.stream, or the null stream);
 *  - one sim per host thread at a time (not re-entrant); per-env faults go to the
 *    env_error buffer, never to return codes, except the reference's one raising case, spawn
 *    sampling exhaustion (MMX_ESAMPLING);
 *  - every entry point makes the sim's device (cfg.device) current for its HIP calls and
 *    restores the caller's current device before returning.
 */
#ifndef MMX_API_H
#define MMX_API_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMX_OK 0
#define MMX_EINVAL (-1)   /* bad argument (ValueError in the reference) */
#define MMX_EDEVICE (-2)  /* HIP runtime error */
#define MMX_ENOMEM (-3)   /* device allocation failed */
#define MMX_ESAMPLING (-4) /* object spawn sampling exhausted its 1000 attempts (RuntimeError in the
                              reference, randomization.py:84-87); reported by the synchronous
                              mmx_reset, and for autoresets inside steps / rollouts / the episode queue
                              by the next mmx_synchronize; the env's env_error carries bit 8 */

/* action modes, gym_env.py:30-36 */
enum { MMX_ACTION_ABS_POS = 0, MMX_ACTION_EE_POS_QUAT_G = 1, MMX_ACTION_EE_POS_ROT6D_G = 2,
       MMX_ACTION_EE_POS_QUAT_G_REL = 3, MMX_ACTION_EE_POS_ROT6D_G_REL = 4 };
/* reward types, gym_env.py:86 */
enum { MMX_REWARD_DENSE = 0, MMX_REWARD_SPARSE = 1, MMX_REWARD_STAGED = 2 };

typedef struct mmx_sim mmx_sim;

/* Constructor arguments of PickPlaceGymEnv (gym_env.py:62-75) plus batching knobs. */
typedef struct {
  int32_t num_envs;
  int32_t device;               /* HIP device ordinal */
  int32_t action_mode;          /* MMX_ACTION_* */
  int32_t reward_type;          /* MMX_REWARD_* */
  int32_t max_episode_steps;    /* truncation limit (constants.py:27) */
  int32_t randomize_objects;    /* randomization.py on reset */
  double spawn_x_range[2];      /* fp64: the spawn draws are numpy-identical fp64 */
  double spawn_y_range[2];
  int32_t n_tasks;              /* task pool (constants.py:11-25), objects/bins 0=red 1=green 2=blue */
  int8_t task_obj[9];
  int8_t task_bin[9];
  int32_t fixed_task_obj;       /* -1: sample from the pool (gym_env.py:511-517) */
  int32_t fixed_task_bin;
  int32_t image_size;           /* camera image side (any, <= 1024; sides that are multiples of 16 write
                                   whole dwords); 0 = no rendering */
  int32_t autoreset;            /* same-step autoreset on terminated/truncated/FSM done */
  int32_t solver_iterations;    /* Newton iteration cap (default 30) */
  float solver_tolerance;       /* relative gradient-norm tolerance (default 1e-6) */
  void* stream;                 /* hipStream_t, NULL = default stream */
} mmx_config;

/* Env-major device buffers (sim-owned): [N][F]. */
typedef struct {
  int32_t num_envs;
  float* qpos;               /* [N][30] */
  float* qvel;               /* [N][27] */
  float* ctrl;               /* [N][8]  */
  float* qacc_warmstart;     /* [N][27] */
  float* obs;                /* [N][85] numeric observation, gym_env.py:295-339 order */
  float* reward;             /* [N] */
  int32_t* done;             /* [N][3] terminated, truncated, success */
  float* reward_components;  /* [N][6] staged breakdown (gym_env.py:568-573) */
  int32_t* episode_i;        /* [N][18] obj, bin, step_count, flags, fsm_state, fsm_task_index,
                                fsm_settle, fsm_gripper_open, fsm_has_target, env_error, ncon, nefc,
                                episodes (resets so far), rng_has32, then sticky counters never
                                cleared by a reset: successes (episodes that ended with
                                info["success"] under autoreset), placed (episodes that ended with
                                the target cube in the target bin), error_resets (autoresets forced by
                                a diverged state: NaN / Inf / |qvel| or |qacc| >= 1e10, reported
                                as truncated), and fsm_phases (bitmask of the FSM states visited
                                since the last reset) */
  float* episode_f;          /* [N][28] T_init(12), hwm(5), target_kp(4), fsm_target(3), transit(3), return */
  float* kin;                /* [N][63] hand pos/mat, arm joint axes/anchors and cube positions of the
                                last position stage (what data.xpos holds after mj_step) */
  float* stats;              /* [N][19] sum nefc, sum ncon, sum solver iterations, substeps, max residual,
                                then shader-clock cycles spent per phase: ik, kinematics, dynamics,
                                collision, constraints, solver, integrate, step end (reward/obs/reset),
                                4 sub-phase probes (cycle fields: diagnostic build only, else 0), then
                                the substeps whose solve ended above the tolerance: by no progress
                                (step < 1e-9, an fp32 stall), by the iteration cap */
  float* contacts;           /* [N][64][13] dist, pos3, normal3, mu3 (slide, spin, roll), dim, geom1, geom2
                                (last substep) */
  uint8_t* images;           /* [N][2][S][S][3] RGB of the overhead and wrist cameras (S = image_size),
                                rendered after every reset / step / forward; NULL when image_size = 0 */
  uint8_t* seg;              /* [N][2][S][S] segment ids: 0 sky, 1 floor, 2 table, 3-5 bins (red, green,
                                blue), 6-8 cubes (red, green, blue), 9 robot; NULL when image_size = 0 */
  float* target;             /* [N][4] decoded EE target (IKController.compute's target_pos) + gripper
                                value of the current step; writable for physics-level harnesses */
} mmx_buffers;

void mmx_config_default(mmx_config* cfg);

/* PickPlaceGymEnv.__init__ (gym_env.py:62-208) for num_envs environments. */
int mmx_create(const mmx_config* cfg, mmx_sim** out);
void mmx_destroy(mmx_sim* sim);
const char* mmx_last_error(const mmx_sim* sim);

/* PickPlaceGymEnv.reset (gym_env.py:477-534) for the envs selected by env_mask (host,
 * N bytes, NULL = all).  seeds: host, N entries, or NULL to continue each env's stream
 * (gym semantics: reset(seed=None)).  seed_given: host, N bytes, NULL = all seeds valid.
 * task_override: host, N entries of (obj << 4 | bin), -1 = none (options["task"]).
 * Synchronous.  Returns MMX_ESAMPLING when an env's spawn sampling (randomize_objects) found no
 * separated placement in 1000 attempts: as where the reference raises, that env's cubes stay at the
 * keyframe and its task is not redrawn (its random stream stays the reference's); the others reset. */
int mmx_reset(mmx_sim* sim, const uint64_t* seeds, const uint8_t* seed_given, const int32_t* task_override,
              const uint8_t* env_mask);

/* PickPlaceGymEnv.step (gym_env.py:536-581): action_dev is a device pointer to [N][action_dim]
 * fp32 (row-major, env-major).  Runs decode -> 16 x (IK + mj_step) -> mj_forward -> reward -> obs. */
int mmx_step(mmx_sim* sim, const float* action_dev, int32_t action_dim);

/* Host helper of the dataset path (dataset.py collect_episodes, generate_dataset.py:250-260's
 * per-frame PNG files): copies n byte ranges, len[k] bytes from host address src[k] to dst[k]
 * (ranges must not overlap); returns the bytes copied, -1 on bad arguments (nothing copied).  One
 * call per camera and step appends every slot's new PNG file to its episode's buffer straight out of
 * the pinned copy of the step, with no Python object per frame (ctypes releases the GIL for the call). */
int64_t mmx_copy_ranges(int64_t n, const uint64_t* src, const uint64_t* dst, const int64_t* len);

/* PickAndPlaceTask.plan(n_steps) (pick_and_place.py:167-277) for every env; writes the
 * abs_pos action [N][4] = (target_xyz, gripper_val) to action_dev_out (may be NULL). */
int mmx_expert_plan(mmx_sim* sim, int32_t n_steps, float* action_dev_out);

/* Expert rollout driver (scripts/generate_dataset.py:140-196): n_env_steps x (plan(16) ->
 * step(abs_pos)); envs whose FSM is done auto-reset when cfg.autoreset is set.
 * Requires action_mode == MMX_ACTION_ABS_POS. */
int mmx_rollout_expert(mmx_sim* sim, int32_t n_env_steps);

/* Batched PNG encoder (dataset emission, generate_dataset.py:250-260: LeRobot embeds image
 * features as PNG files).  Encodes n RGB8 images (device, image i at rgb_dev + i * img_stride,
 * rows of 3 * width bytes, height <= 1024, width <= MMX_PNG_MAX_WIDTH: the encoder's row-above match
 * uses deflate distance 3 * width + 1, capped at 32768) into complete PNG files: image i's file is written at
 * out_dev + i * out_stride (out_stride >= mmx_png_bound(width, height)) and its byte size to
 * sizes_dev[i] (int32).  scratch_dev: n * mmx_png_scratch(width, height) bytes of device memory.
 * mmx_png_pack copies the n files back to back into packed_dev at offsets_dev[i] (int64, device).
 * Asynchronous on the sim's stream; bounds return -1 for unsupported sizes. */
#define MMX_PNG_MAX_WIDTH 10922
int64_t mmx_png_bound(int32_t width, int32_t height);
int64_t mmx_png_scratch(int32_t width, int32_t height);
int mmx_png_encode(mmx_sim* sim, const uint8_t* rgb_dev, int64_t img_stride, int32_t n, int32_t width,
                   int32_t height, uint8_t* out_dev, int64_t out_stride, int32_t* sizes_dev, void* scratch_dev);
int mmx_png_pack(mmx_sim* sim, const uint8_t* out_dev, int64_t out_stride, const int32_t* sizes_dev,
                 const int64_t* offsets_dev, int32_t n, uint8_t* packed_dev);

/* Per-image channel statistics of n RGB8 images (device, image i at rgb_dev + i * img_stride, rows
 * of 3 * width bytes, width and height <= 4096): out_dev[i] = int64 [min R G B, max R G B, sum R G B,
 * sum of squares R G B] over every pixel (LeRobot's image feature statistics, which the dataset
 * writer scales to [0, 1]; generate_dataset.py:250-260).  Asynchronous on the sim's stream. */
int mmx_image_stats(mmx_sim* sim, const uint8_t* rgb_dev, int64_t img_stride, int32_t n, int32_t width,
                    int32_t height, int64_t* out_dev);

/* Physics-level entry points (parity harnesses): n x mujoco.mj_step with the current ctrl
 * (env.py:119-121), optionally preceded by IKController.compute toward the decoded target
 * each substep; and the mj_forward position stage (kinematics + IK cache). */
int mmx_physics_step(mmx_sim* sim, int32_t n, int32_t with_ik);
int mmx_forward(mmx_sim* sim);

/* Per-physics-step expert loop (main.py:65-91; tests/test_pick_and_place.py:147-166):
 * n x (PickAndPlaceTask.update() = plan(1) + _actuate() (pick_and_place.py:279-304) ;
 * mujoco.mj_step), the FSM reading data.xpos as the previous mj_step left it.  No gym
 * bookkeeping (no reward, observation or autoreset); the FSM state is in episode_i. */
int mmx_expert_physics(mmx_sim* sim, int32_t n_physics_steps);

/* Reward-layer parity harness (gym_env.py:341-470, 562-573).  For every env: the object at
 * obj_dev[N][3], the EE at ee_dev[N][3], gripper ctrl ctrl7_dev[N] and this step's contacts as
 * geom-id pairs pairs_dev[N][max_pairs][2] (int32, a negative id ends the list; geom ids as in the
 * compiled model = MuJoCo's).  Evaluates _compute_reward, updating the sticky flags and
 * high-water marks like a step, and writes reward, reward_components, done[0] (terminated) and
 * done[2] (success).  All pointers are device pointers. */
int mmx_eval_reward(mmx_sim* sim, const float* obj_dev, const float* ee_dev, const float* ctrl7_dev,
                    const int32_t* pairs_dev, int32_t max_pairs);

int mmx_get_buffers(mmx_sim* sim, mmx_buffers* out);
/* Waits for the sim's stream; MMX_ESAMPLING when an autoreset since the last check (mmx_reset or
 * mmx_synchronize) exhausted its spawn sampling (that env's env_error has bit 8). */
int mmx_synchronize(mmx_sim* sim);

/* Host copies of the core state (host arrays of [N][field] fp32). NULL skips a field. */
int mmx_get_state(mmx_sim* sim, float* qpos, float* qvel, float* ctrl, float* qacc_warmstart);
int mmx_set_state(mmx_sim* sim, const float* qpos, const float* qvel, const float* ctrl, const float* qacc_warmstart);

/* Device-side episode queue of dataset generation (scripts/generate_dataset.py:140-198 runs
 * run_episode per episode with seeds / tasks from :263-277): n_episodes episodes stream through the
 * N env slots with no host synchronisation per step.  mmx_queue_init uploads every episode's task
 * (host, n_episodes entries of obj << 4 | bin, -1 = the env's own draw) and, when seeds (host,
 * n_episodes entries) is non-NULL, its PCG64(SeedSequence(seed)) state; no slot holds an episode
 * yet (synchronous; replaces a previous queue).  mmx_queue_advance, asynchronous on the sim's
 * stream: every slot that holds no episode or whose episode's FSM reached DONE takes the next
 * episode, in ascending slot order, and is reset (PickPlaceGymEnv.reset with the episode's seed
 * and task, gym_env.py:477-534) and re-rendered; slot_ep_dev (device int32 [N], may be NULL)
 * receives each slot's episode afterwards (-1: none left) and fin_ep_dev (device int32 [N], may be
 * NULL) the episode that ended in the slot at this call (-1: none).  MMX_EINVAL without a queue. */
int mmx_queue_init(mmx_sim* sim, int32_t n_episodes, const uint64_t* seeds, const int32_t* tasks);
int mmx_queue_advance(mmx_sim* sim, int32_t* slot_ep_dev, int32_t* fin_ep_dev);

/* Host helper: SeedSequence(root).spawn(n)[index].generate_state(1)[0]
 * (scripts/generate_dataset.py:263-268). */
uint32_t mmx_episode_seed(uint64_t root_seed, int32_t index);

/* Measurement and tuning entry points (launch shape, layout, dispatch order, per-launch timing) have
 * no reference counterpart and are declared in mmx_tuning.h; a reference-side binding needs none. */

#ifdef __cplusplus
}
#endif
#endif
