/* ORACLE internal state (test infrastructure only). */
#ifndef OR_INTERNAL_H
#define OR_INTERNAL_H
#include "oracle.h"
#include "oracle_model_gen.h"
#include "or_math.h"

#define NB OM_NBODY
#define NJ OM_NJNT
#define NQ OM_NQ
#define NV OM_NV
#define NG OM_NGEOM
#define NU OM_NU
#define NC OM_NCAM
#define MINVAL 1e-15
#define OR_IMPRATIO 1.0 /* MuJoCo default <option impratio>; the model does not set it */

enum { EFC_EQUALITY = 0, EFC_LIMIT = 1, EFC_CONTACT = 2 };

typedef struct {
  int geom[2];
  double dist;
  double pos[3];
  double frame[9];
  double friction[5];
  int dim;
  double solref[2], solimp[5];
} or_contact;

struct or_env {
  /* configuration (gym_env.py:62-75) */
  int action_mode, reward_type, max_episode_steps, randomize, image_size;
  double spawn_x[2], spawn_y[2];
  int ntask, task_obj[9], task_bin[9];
  int fixed_obj, fixed_bin;
  /* simulation state (mjData qpos/qvel/ctrl/qacc_warmstart) */
  double qpos[NQ], qvel[NV], ctrl[NU], qacc_ws[NV];
  /* position-dependent */
  double xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3];
  double janchor[NJ][3], jaxis[NJ][3];
  double cdof[NV][6]; /* motion subspace, world-origin Plucker coordinates (ang, lin) */
  double gxpos[NG][3], gxmat[NG][9];
  double camxpos[NC][3], camxmat[NC][9];
  double M[NV * NV];
  double ten_len, ten_moment[NV];
  int ncon;
  or_contact con[OR_MAXCON];
  int nefc;
  double efc_J[OR_MAXEFC][NV];
  double efc_pos[OR_MAXEFC], efc_aref[OR_MAXEFC], efc_R[OR_MAXEFC], efc_D[OR_MAXEFC];
  double efc_force[OR_MAXEFC], efc_vel[OR_MAXEFC];
  int efc_type[OR_MAXEFC];
  /* velocity / force dependent */
  double qfrc_bias[NV], qfrc_passive[NV], act_force[NU], act_raw[NU], qfrc_act[NV];
  double qfrc_smooth[NV], qacc_smooth[NV], qacc[NV], qfrc_constraint[NV];
  double solver_res;
  int solver_iter;
  double solver_tol;       /* Newton: relative gradient tolerance (default 1e-13: parity tests) */
  int solver_maxiter;      /* iteration cap (default 200) */
  double solver_mj_tol;    /* MuJoCo's opt.tolerance convergence tests, 0 = off (parity tests) */
  long solver_calls, solver_iters_total;
  /* gym episode state */
  or_pcg64 rng;
  int obj, bin, step_count;
  double T_init[16];
  int has_grasped, has_lifted, above_target, has_placed, hwm_valid;
  double hwm[5];
  float tgt_obj_kp[2], tgt_bin_kp[2];
  /* FSM expert state (pick_and_place.py:100-105) */
  int fsm_state, fsm_task_index, fsm_settle, fsm_gripper_open, fsm_has_target;
  double fsm_target[3], fsm_transit_end[3];
  int fsm_ntasks, fsm_obj[9], fsm_bin[9];
};

/* physics */
void or_kinematics(or_env* e);
void or_collision(or_env* e);
void or_point_jac(or_env* e, int body, const double* point, double* jacp, double* jacr);

#endif
