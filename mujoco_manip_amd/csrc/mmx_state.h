// Device-resident batch state for the MI355X pick-and-place simulator.
//
// Layout: env-major ("array of per-env records"): field f of env i lives at ptr[i * F + f].
// One environment is owned by one 64-lane workgroup for the whole env step, so an env's record
// is one contiguous, coalesced read at kernel start and one write at kernel end; everything in
// between (16 substeps) stays in that workgroup's LDS.  Shared by mmx_kernels.hip (device) and
// mmx_api.cpp (host allocation / C-ABI); no torch types anywhere.
#ifndef MMX_STATE_H
#define MMX_STATE_H
#include <stdint.h>

#define MMX_NQ_ 30
#define MMX_NV_ 27
#define MMX_NU_ 8
#define MMX_NOBS 85
#define MMX_MAXCON 64
// constraint rows (basis rows: 4 per contact + equality / limits padded to 4; <= 64 x 4 + 20)
#define MMX_MAXEFC 320
// constraint rows [0, MMX_LDSEFC) live in the workgroup's LDS, rows [MMX_LDSEFC, MMX_MAXEFC) in the
// env's HBM overflow block (efc_ovf); 128 rows keep the env's LDS within 12,800 B (twelve envs per CU:
// the LDS is allocated in 1,280-byte blocks, tools/calib/lds_occ.hip; r05: 14,080 B, 11 per CU; r01-r04:
// 192 rows, 20 KB, 8 per CU)
#ifndef MMX_LDSEFC
#define MMX_LDSEFC 128
#endif
#define MMX_OVFEFC (MMX_MAXEFC - MMX_LDSEFC)
// persistent broadphase list entries (pair indices, in the env's overflow block; a longer list is not
// kept: the full prune runs)
#ifndef MMX_CAND_CAP  // (test builds lower it with MMX_COL_LIST: tests/test_overflow_kat.py)
#define MMX_CAND_CAP 256
#endif
// the env's HBM overflow block, in floats: J rows [OVFEFC][16], then D, NC [OVFEFC], then the general
// Cholesky's 27 x 27 transpose (+3: 16-byte aligned blocks), then the overflow rows' headers (bytes)
// and the broadphase list (16-bit pair indices)
#define MMX_OVF_ARROW_AT(efc) (18 * (MMX_MAXEFC - (efc)))
#define MMX_OVF_HDR_AT(efc) (MMX_OVF_ARROW_AT(efc) + 27 * 27 + 3)
#define MMX_OVF_CAND_AT(efc) (MMX_OVF_HDR_AT(efc) + (MMX_MAXEFC - (efc) + 3) / 4)
#define MMX_OVF_F_AT(efc) ((MMX_OVF_CAND_AT(efc) + (MMX_CAND_CAP + 1) / 2 + 3) / 4 * 4)  // (16-byte env blocks)
#define MMX_OVF_F MMX_OVF_F_AT(MMX_LDSEFC)
#define MMX_NSUBSTEP 16

// stale kinematics cache read by the IK (controller.py:99-108 reads data.xpos / mj_jac
// outputs left by the previous mj_step's position stage)
enum {
  KIN_HAND_POS = 0,    // 3
  KIN_HAND_MAT = 3,    // 9 (row-major)
  KIN_AXIS = 12,       // 7 x 3 arm joint axes (world)
  KIN_ANCHOR = 33,     // 7 x 3 arm joint anchors (world)
  KIN_OBJ = 54,        // 3 x 3 cube positions (data.xpos of obj_red/green/blue: the per-physics-step
                       // FSM reads them stale, pick_and_place.py:167-277 via env.get_body_pos)
  KIN_N = 63
};

// per-env integer episode / FSM state
enum {
  EPI_OBJ = 0, EPI_BIN, EPI_STEP, EPI_FLAGS, EPI_FSM_STATE, EPI_FSM_TASKIDX, EPI_FSM_SETTLE,
  EPI_FSM_GRIP, EPI_FSM_HASTGT, EPI_ERROR, EPI_NCON, EPI_NEFC, EPI_EPISODES, EPI_RNG_HAS32,
  // sticky counters (never cleared by a reset): episodes that ended with info["success"], episodes
  // that ended with the target cube in the target bin (the success test of gym_env.py:436-447:
  // xy < 0.05 and z < bin z + 0.06), and autoresets forced by a diverged state (ERR_NAN: NaN / Inf
  // / |qvel| or |qacc| >= 1e10, MuJoCo's mj_checkVel / mj_checkAcc); then the bitmask of the FSM
  // states visited since the last reset
  EPI_NSUCCESS, EPI_NPLACED, EPI_NERROR, EPI_PHASES,
  EPI_N
};
// per-env float episode / FSM state
enum {
  EPF_TINIT = 0,        // 12: R (row-major 9) + p (3)
  EPF_HWM = 12,         // 5
  EPF_TGTKP = 17,       // 4
  EPF_FSM_TARGET = 21,  // 3
  EPF_FSM_TRANSIT = 24, // 3
  EPF_EP_RETURN = 27,
  EPF_N = 28
};
// staged-reward sticky flags (gym_env.py:129-132)
enum { FLAG_GRASPED = 1, FLAG_LIFTED = 2, FLAG_ABOVE = 4, FLAG_PLACED = 8, FLAG_HWM_VALID = 16 };
// env_error bits
enum { ERR_CON_OVERFLOW = 1, ERR_EFC_OVERFLOW = 2, ERR_NAN = 4, ERR_SAMPLING = 8 };

// contact record fields
enum { CON_DIST = 0, CON_POS = 1, CON_N = 4, CON_MU0 = 7, CON_MU1, CON_MU2, CON_DIM, CON_G1, CON_G2, CON_F };
// statistics accumulated per env (over substeps since the last clear)
// (STAT_T_*: shader-clock cycles per phase, read with s_memtime and summed over substeps; only the
//  diagnostic build libmmx_prof.so, compiled with -DMMX_PHASE_CLOCK, fills them)
enum {
  STAT_NEFC = 0, STAT_NCON, STAT_SOLVER_ITER, STAT_SUBSTEPS, STAT_RESID,
  STAT_T_IK, STAT_T_KIN, STAT_T_DYN, STAT_T_COL, STAT_T_CON, STAT_T_SOLVE, STAT_T_INT, STAT_T_END,
  STAT_T_AUX0, STAT_T_AUX1, STAT_T_AUX2, STAT_T_AUX3,  // sub-phase probes (see the kernel source)
  // substeps whose Newton solve ended above the tolerance: no progress (step < 1e-9, an fp32 stall)
  // / the iteration cap
  STAT_EXIT_STALL, STAT_EXIT_CAP,
  STAT_N
};

enum { MMX_SOLVER_NEWTON = 0, MMX_SOLVER_PGS = 1 };

struct MMXState {
  int N;
  // configuration (gym_env.py:62-75 constructor arguments)
  int action_mode, reward_type, max_episode_steps, randomize, image_size, autoreset;
  double spawn_x0, spawn_x1, spawn_y0, spawn_y1;
  int ntask, task_obj[9], task_bin[9], fixed_obj, fixed_bin;
  int solver, solver_max_iter;
  float solver_tol;
  // state, env-major
  float* qpos;     // [N][30]
  float* qvel;     // [N][27]
  float* ctrl;     // [N][8]
  float* qacc_ws;  // [N][27]
  float* kin;      // [N][54]
  float* target;   // [N][4] decoded EE target + gripper command
  int* epi;        // [N][EPI_N]
  float* epf;      // [N][EPF_N]
  unsigned long long* rng;  // [N][4]: state hi, state lo, inc hi, inc lo
  unsigned int* rng32;      // [N]: buffered upper half of the last 64-bit draw
  // outputs
  float* obs;                // [N][85]
  float* reward;             // [N]
  float* reward_components;  // [N][6]
  int* done;                 // [N][3]: terminated, truncated, success
  // diagnostics
  float* con;    // [N][MAXCON][CON_F] contacts of the last substep
  float* stats;  // [N][STAT_N]
  float* efc_ovf;  // [N][MMX_OVF_F] constraint rows past the LDS ones (scratch, rarely touched)
  int* fault;      // [1] sim-level sticky error bits: ERR_SAMPLING of any reset since the host last checked
  // camera images (image_size > 0 only, else null)
  float* rpose;            // [N][14][12] body poses (R row-major, p) of the last position stage
  unsigned char* images;   // [N][2][S][S][3] overhead, wrist RGB
  unsigned char* seg;      // [N][2][S][S] segment ids (0 sky, 1 floor, 2 table, 3-5 bins, 6-8 cubes, 9 robot)
  unsigned int* bg_overhead;  // [Sg][Sg] the fixed overhead camera's background (packed RGB | seg << 24)
};

#endif
