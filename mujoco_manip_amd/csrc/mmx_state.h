// Device-resident batch state for the MI355X pick-and-place simulator.
//
// Layout: structure-of-arrays with the environment index fastest, i.e. field f of env i
// lives at ptr[f * N + i].  One env is owned by one wavefront lane, so every per-field
// access of a wave is a 256-byte coalesced transaction.  Shared by mmx_kernels.hip (device)
// and mmx_api.cpp (host allocation / C-ABI); no torch types anywhere.
#ifndef MMX_STATE_H
#define MMX_STATE_H
#include <stdint.h>

#define MMX_NQ_ 30
#define MMX_NV_ 27
#define MMX_NU_ 8
#define MMX_NOBS 85
#define MMX_MAXCON 40
#define MMX_MAXEFC 264
#define MMX_NSUBSTEP 16

// stale kinematics cache read by the IK (controller.py:99-108 reads data.xpos / mj_jac
// outputs left by the previous mj_step's position stage)
enum {
  KIN_HAND_POS = 0,   // 3
  KIN_HAND_MAT = 3,   // 9 (row-major)
  KIN_AXIS = 12,      // 7 x 3 arm joint axes (world)
  KIN_ANCHOR = 33,    // 7 x 3 arm joint anchors (world)
  KIN_N = 54
};

// per-env integer episode / FSM state
enum {
  EPI_OBJ = 0, EPI_BIN, EPI_STEP, EPI_FLAGS, EPI_FSM_STATE, EPI_FSM_TASKIDX, EPI_FSM_SETTLE,
  EPI_FSM_GRIP, EPI_FSM_HASTGT, EPI_ERROR, EPI_NCON, EPI_NEFC, EPI_EPISODES, EPI_RNG_HAS32,
  EPI_N
};
// per-env float episode / FSM state
enum {
  EPF_TINIT = 0,       // 12: R (row-major 9) + p (3)
  EPF_HWM = 12,        // 5
  EPF_TGTKP = 17,      // 4
  EPF_FSM_TARGET = 21, // 3
  EPF_FSM_TRANSIT = 24,// 3
  EPF_EP_RETURN = 27,
  EPF_N = 28
};
// staged-reward sticky flags (gym_env.py:129-132)
enum { FLAG_GRASPED = 1, FLAG_LIFTED = 2, FLAG_ABOVE = 4, FLAG_PLACED = 8, FLAG_HWM_VALID = 16 };
// env_error bits
enum { ERR_CON_OVERFLOW = 1, ERR_EFC_OVERFLOW = 2, ERR_NAN = 4, ERR_SAMPLING = 8 };

// contact record fields
enum { CON_DIST = 0, CON_POS = 1, CON_N = 4, CON_MU0 = 7, CON_MU1, CON_MU2, CON_DIM, CON_G1, CON_G2, CON_F };
// constraint row fields
enum { EFC_J = 0, EFC_MJ = 15, EFC_AREF = 30, EFC_R = 31, EFC_DINV = 32, EFC_FORCE = 33, EFC_BLK = 34, EFC_F = 35 };
// statistics accumulated per env (over substeps since the last clear)
enum { STAT_NEFC = 0, STAT_NCON, STAT_PGS_ITER, STAT_SUBSTEPS, STAT_RESID, STAT_N };

struct MMXState {
  int N;
  // configuration (gym_env.py:62-75 constructor arguments)
  int action_mode, reward_type, max_episode_steps, randomize, image_size, autoreset;
  float spawn_x0, spawn_x1, spawn_y0, spawn_y1;
  int ntask, task_obj[9], task_bin[9], fixed_obj, fixed_bin;
  int pgs_max_iter;
  float pgs_tol;
  // state
  float *qpos, *qvel, *ctrl, *qacc_ws;
  float *kin, *target;
  int* epi;
  float* epf;
  unsigned long long* rng;  // [4][N]: state hi, state lo, inc hi, inc lo
  unsigned int* rng32;      // [N]: buffered upper half of the last 64-bit draw
  // outputs
  float *obs, *reward, *reward_components;
  int* done;  // [3][N]: terminated, truncated, success
  // scratch
  float* con;
  float* efc;
  float* stats;
};

#endif
