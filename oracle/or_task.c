/* ORACLE (test infrastructure only) — fp64 restatement of the reference's task layer:
 *   IKController.compute/_orientation_error/reached   controller.py:21-145
 *   PickAndPlaceTask.plan/_actuate                     pick_and_place.py:167-291
 *   PickPlaceGymEnv decode_action/_get_obs/rewards/reset/step   gym_env.py:252-581
 *   pose codecs                                        pose_utils.py:48-209
 *   keypoint projection                                cameras.py:56-130
 *   randomization (rejection sampling)                 randomization.py:11-98
 *   gymnasium seeding Generator(PCG64(SeedSequence(s))) and numpy's uniform / bounded
 *   integers (numpy 2.x, restated from its published algorithm). */
#include <stdlib.h>
#include <stdio.h>
#include "or_internal.h"

static const double HOME_QPOS[7] = {1.5708, -0.2, 0.0, -2.1, 0.0, 1.8, 0.785}; /* controller.py:8 */
static const double TARGET_ORI[9] = {0, 1, 0, 1, 0, 0, 0, 0, -1};                /* controller.py:12-18 */

/* ======================================================================= pose utils */
void or_rotmat_to_quat_xyzw(const double* R, double* q) { /* pose_utils.py:48-82 */
  double tr = R[0] + R[4] + R[8], s, w, x, y, z;
  if (tr > 0) {
    s = 2.0 * sqrt(tr + 1.0);
    w = 0.25 * s; x = (R[7] - R[5]) / s; y = (R[2] - R[6]) / s; z = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    s = 2.0 * sqrt(1.0 + R[0] - R[4] - R[8]);
    w = (R[7] - R[5]) / s; x = 0.25 * s; y = (R[1] + R[3]) / s; z = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    s = 2.0 * sqrt(1.0 + R[4] - R[0] - R[8]);
    w = (R[2] - R[6]) / s; x = (R[1] + R[3]) / s; y = 0.25 * s; z = (R[5] + R[7]) / s;
  } else {
    s = 2.0 * sqrt(1.0 + R[8] - R[0] - R[4]);
    w = (R[3] - R[1]) / s; x = (R[2] + R[6]) / s; y = (R[5] + R[7]) / s; z = 0.25 * s;
  }
  q[0] = x; q[1] = y; q[2] = z; q[3] = w;
}

void or_quat_xyzw_to_rotmat(const double* q, double* R) { /* pose_utils.py:85-101 (no normalisation) */
  double x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}

void or_rotmat_from_6d(const double* d6, double* R) { /* pose_utils.py:121-146 */
  double b1[3], b2[3], b3[3], a2[3];
  v3_copy(b1, d6);
  double n1 = v3_norm(b1);
  v3_scl(b1, b1, 1.0 / (n1 > 1e-12 ? n1 : 1e-12));
  v3_copy(a2, d6 + 3);
  double d = v3_dot(b1, a2);
  v3_addscl(b2, a2, b1, -d);
  double n2 = v3_norm(b2);
  v3_scl(b2, b2, 1.0 / (n2 > 1e-12 ? n2 : 1e-12));
  v3_cross(b3, b1, b2);
  v3_copy(R, b1); v3_copy(R + 3, b2); v3_copy(R + 6, b3);
}

/* decode_action (gym_env.py:252-281); action already float32 (gym_env.py:547) */
void or_decode_action(int mode, const float* a, const double* T_init, double* target, double* grip) {
  double p[3] = {a[0], a[1], a[2]};
  switch (mode) {
    case 0: v3_copy(target, p); *grip = a[3]; return;
    case 1: v3_copy(target, p); *grip = a[7]; return;
    case 2: v3_copy(target, p); *grip = a[9]; return;
    default: {
      /* T_abs = T_init @ T_rel: translation = R_init p_rel + p_init */
      for (int i = 0; i < 3; i++)
        target[i] = T_init[4 * i] * p[0] + T_init[4 * i + 1] * p[1] + T_init[4 * i + 2] * p[2] + T_init[4 * i + 3];
      *grip = mode == 3 ? a[7] : a[9];
    }
  }
}

/* ======================================================================= IK */
void or_orientation_error(const double* Rc, const double* Rt, double* err) { /* controller.py:21-43 */
  double E[9];
  /* R_err = R_target @ R_current^T */
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) E[3 * i + j] = Rt[3 * i] * Rc[3 * j] + Rt[3 * i + 1] * Rc[3 * j + 1] + Rt[3 * i + 2] * Rc[3 * j + 2];
  double tv = (E[0] + E[4] + E[8] - 1) / 2;
  if (tv < -1) tv = -1;
  if (tv > 1) tv = 1;
  double ang = acos(tv);
  if (ang < 1e-6) { err[0] = err[1] = err[2] = 0; return; }
  double s = 2 * sin(ang);
  err[0] = (E[7] - E[5]) / s * ang;
  err[1] = (E[2] - E[6]) / s * ang;
  err[2] = (E[3] - E[1]) / s * ang;
}

static void inv6_spd(const double* A, double* Ainv) {
  double L[36];
  memcpy(L, A, sizeof(L));
  chol_factor(L, 6);
  for (int c = 0; c < 6; c++) {
    double x[6] = {0};
    x[c] = 1;
    chol_solve(L, 6, x);
    for (int r = 0; r < 6; r++) Ainv[6 * r + c] = x[r];
  }
}

/* damped least squares with nullspace bias, given J (6x7, row-major) */
void or_ik_math(const double* J, const double* ee_pos, const double* ee_xmat, const double* q, const double* target,
                const double* rng, double* q_out) {
  double e6[6], ori[3];
  for (int k = 0; k < 3; k++) e6[k] = 1.0 * (target[k] - ee_pos[k]);
  or_orientation_error(ee_xmat, TARGET_ORI, ori);
  for (int k = 0; k < 3; k++) e6[3 + k] = 1.0 * ori[k];
  double JJT[36], inv[36], Jp[42];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) {
      double s = 0;
      for (int k = 0; k < 7; k++) s += J[7 * i + k] * J[7 * j + k];
      JJT[6 * i + j] = s + (i == j ? 1e-3 : 0);
    }
  inv6_spd(JJT, inv);
  for (int i = 0; i < 7; i++)
    for (int j = 0; j < 6; j++) {
      double s = 0;
      for (int k = 0; k < 6; k++) s += J[7 * k + i] * inv[6 * k + j];
      Jp[6 * i + j] = s;
    }
  double dq[7], bias[7];
  for (int i = 0; i < 7; i++) {
    double s = 0;
    for (int k = 0; k < 6; k++) s += Jp[6 * i + k] * e6[k];
    dq[i] = s;
    bias[i] = 0.5 * (HOME_QPOS[i] - q[i]);
  }
  for (int i = 0; i < 7; i++) {
    double s = bias[i];
    for (int j = 0; j < 7; j++) {
      double PJ = 0;
      for (int k = 0; k < 6; k++) PJ += Jp[6 * i + k] * J[7 * k + j];
      s -= PJ * bias[j];
    }
    dq[i] += s;
  }
  double n = 0;
  for (int i = 0; i < 7; i++) n += dq[i] * dq[i];
  n = sqrt(n);
  if (n > 5.0)
    for (int i = 0; i < 7; i++) dq[i] *= 5.0 / n;
  for (int i = 0; i < 7; i++) {
    double t = q[i] + dq[i];
    double lo = rng[2 * i], hi = rng[2 * i + 1];
    if (lo < hi) {
      if (t < lo) t = lo;
      if (t > hi) t = hi;
    }
    q_out[i] = t;
  }
}

void or_ik_compute(or_env* e, const double* target, double* q_target) { /* controller.py:87-137 */
  const int hand = OM_BODY_HAND;
  double ee[3], jacp[3 * NV], jacr[3 * NV], J[42], rng[14];
  v3_copy(ee, e->xpos[hand]);
  or_point_jac(e, hand, ee, jacp, jacr);
  for (int k = 0; k < 3; k++)
    for (int d = 0; d < 7; d++) {
      J[7 * k + d] = jacp[k * NV + d];
      J[7 * (3 + k) + d] = jacr[k * NV + d];
    }
  for (int j = 0; j < 7; j++) {
    rng[2 * j] = OM_jnt_range[2 * j];
    rng[2 * j + 1] = OM_jnt_range[2 * j + 1];
  }
  or_ik_math(J, ee, e->xmat[hand], e->qpos, target, rng, q_target);
}

int or_ik_reached(or_env* e, const double* target) { /* controller.py:139-145 */
  double d[3];
  v3_sub(d, e->xpos[OM_BODY_HAND], target);
  return v3_norm(d) < 0.02;
}

void or_set_arm_ctrl(or_env* e, const double* q) {
  for (int i = 0; i < 7; i++) e->ctrl[i] = q[i];
}
void or_set_gripper(or_env* e, int open) { e->ctrl[7] = open ? 255.0 : 0.0; }

/* ======================================================================= FSM */
enum { S_IDLE, S_PRE_GRASP, S_GRASP, S_CLOSE_GRIPPER, S_LIFT, S_MOVE_TO_BIN, S_SETTLE_AT_BIN, S_LOWER_TO_BIN,
       S_RELEASE, S_RETREAT, S_DONE };
static const int OBJ_BODY[3] = {OM_BODY_OBJ_RED, OM_BODY_OBJ_GREEN, OM_BODY_OBJ_BLUE};
static const int BIN_BODY[3] = {OM_BODY_BIN_RED, OM_BODY_BIN_GREEN, OM_BODY_BIN_BLUE};

void or_fsm_init(or_env* e, int n, const int* obj, const int* bin) {
  e->fsm_state = S_IDLE;
  e->fsm_task_index = 0;
  e->fsm_settle = 0;
  e->fsm_gripper_open = 1;
  e->fsm_has_target = 0;
  e->fsm_ntasks = n;
  for (int i = 0; i < n; i++) {
    e->fsm_obj[i] = obj[i];
    e->fsm_bin[i] = bin[i];
  }
}

int or_fsm_plan(or_env* e, int n) { /* pick_and_place.py:167-277 */
  double* t = e->fsm_target;
  int ti = e->fsm_task_index;
  const double* oxy = ti < e->fsm_ntasks ? e->xpos[OBJ_BODY[e->fsm_obj[ti]]] : NULL;
  const double* bxy = ti < e->fsm_ntasks ? e->xpos[BIN_BODY[e->fsm_bin[ti]]] : NULL;
  switch (e->fsm_state) {
    case S_IDLE:
      if (ti >= e->fsm_ntasks) { e->fsm_state = S_DONE; break; }
      e->fsm_gripper_open = 1;
      v3_set(t, oxy[0], oxy[1], 0.44);
      e->fsm_has_target = 1;
      e->fsm_state = S_PRE_GRASP;
      break;
    case S_PRE_GRASP:
      if (or_ik_reached(e, t)) { v3_set(t, oxy[0], oxy[1], 0.36); e->fsm_state = S_GRASP; }
      break;
    case S_GRASP:
      if (or_ik_reached(e, t)) { e->fsm_gripper_open = 0; e->fsm_settle = 150; e->fsm_state = S_CLOSE_GRIPPER; }
      break;
    case S_CLOSE_GRIPPER:
      e->fsm_settle -= n;
      if (e->fsm_settle <= 0) { v3_set(t, oxy[0], oxy[1], 0.55); e->fsm_state = S_LIFT; }
      break;
    case S_LIFT:
      if (or_ik_reached(e, t)) { v3_set(e->fsm_transit_end, bxy[0], bxy[1], 0.55); e->fsm_state = S_MOVE_TO_BIN; }
      break;
    case S_MOVE_TO_BIN: {
      double diff[3];
      v3_sub(diff, e->fsm_transit_end, t);
      double dist = v3_norm(diff);
      double step = 0.001 * n;
      if (dist > step) v3_addscl(t, t, diff, step / dist);
      else v3_copy(t, e->fsm_transit_end);
      if (dist <= 0.02) { e->fsm_settle = 100; e->fsm_state = S_SETTLE_AT_BIN; }
      break;
    }
    case S_SETTLE_AT_BIN:
      e->fsm_settle -= n;
      if (e->fsm_settle <= 0) { v3_set(t, bxy[0], bxy[1], 0.45); e->fsm_state = S_LOWER_TO_BIN; }
      break;
    case S_LOWER_TO_BIN:
      if (or_ik_reached(e, t)) { e->fsm_gripper_open = 1; e->fsm_settle = 150; e->fsm_state = S_RELEASE; }
      break;
    case S_RELEASE:
      e->fsm_settle -= n;
      if (e->fsm_settle <= 0) { v3_set(t, 0.0, 0.3, 0.55); e->fsm_state = S_RETREAT; }
      break;
    case S_RETREAT:
      if (or_ik_reached(e, t)) { e->fsm_task_index++; e->fsm_state = S_IDLE; }
      break;
    default: break;
  }
  return e->fsm_state;
}

void or_fsm_actuate(or_env* e) { /* pick_and_place.py:279-291 */
  or_set_gripper(e, e->fsm_gripper_open);
  if (e->fsm_has_target) {
    double q[7];
    or_ik_compute(e, e->fsm_target, q);
    or_set_arm_ctrl(e, q);
  }
}

void or_fsm_get(or_env* e, int* state, int* task_index, int* settle, double* target, int* gripper_open) {
  *state = e->fsm_state;
  *task_index = e->fsm_task_index;
  *settle = e->fsm_settle;
  v3_copy(target, e->fsm_target);
  *gripper_open = e->fsm_gripper_open;
}

/* ======================================================================= RNG */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t v, uint32_t* hc) {
  v ^= *hc;
  *hc *= SS_MULT_A;
  v *= *hc;
  v ^= v >> 16;
  return v;
}
static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  r ^= r >> 16;
  return r;
}

/* numpy SeedSequence(entropy, spawn_key).generate_state(n_out, uint32) */
void or_seedseq_state(const uint32_t* ent, int nent, const uint32_t* spawn, int nspawn, uint32_t* out, int nout) {
  uint32_t arr[64];
  int n = 0;
  for (int i = 0; i < nent; i++) arr[n++] = ent[i];
  if (nspawn > 0 && nent < 4)
    for (int i = nent; i < 4; i++) arr[n++] = 0;
  for (int i = 0; i < nspawn; i++) arr[n++] = spawn[i];
  uint32_t pool[4];
  uint32_t hc = SS_INIT_A;
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n ? arr[i] : 0, &hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
  for (int s = 4; s < n; s++)
    for (int d = 0; d < 4; d++) pool[d] = ss_mix(pool[d], ss_hashmix(arr[s], &hc));
  uint32_t hb = SS_INIT_B;
  for (int i = 0; i < nout; i++) {
    uint32_t v = pool[i % 4];
    v ^= hb;
    hb *= SS_MULT_B;
    v *= hb;
    v ^= v >> 16;
    out[i] = v;
  }
}

static int seed_words(uint64_t seed, uint32_t* w) {
  w[0] = (uint32_t)seed;
  w[1] = (uint32_t)(seed >> 32);
  return w[1] ? 2 : 1;
}

typedef unsigned __int128 u128;
static const u128 PCG_MULT = (((u128)0x2360ED051FC65DA4ull) << 64) | 0x4385DF649FCCF645ull;
static u128 st128(const or_pcg64* r) { return ((u128)r->s_hi << 64) | r->s_lo; }
static u128 inc128(const or_pcg64* r) { return ((u128)r->i_hi << 64) | r->i_lo; }
static void put_st(or_pcg64* r, u128 s) { r->s_hi = (uint64_t)(s >> 64); r->s_lo = (uint64_t)s; }

void or_pcg64_seed(or_pcg64* r, uint64_t seed) {
  uint32_t w[2], st[8];
  int n = seed_words(seed, w);
  or_seedseq_state(w, n, NULL, 0, st, 8);
  uint64_t v[4];
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)st[2 * i] | ((uint64_t)st[2 * i + 1] << 32);
  u128 initstate = ((u128)v[0] << 64) | v[1];
  u128 initseq = ((u128)v[2] << 64) | v[3];
  u128 inc = (initseq << 1) | 1;
  r->i_hi = (uint64_t)(inc >> 64);
  r->i_lo = (uint64_t)inc;
  u128 s = 0;
  s = s * PCG_MULT + inc;
  s += initstate;
  s = s * PCG_MULT + inc;
  put_st(r, s);
  r->has32 = 0;
  r->buf32 = 0;
}

uint64_t or_pcg64_next64(or_pcg64* r) {
  u128 s = st128(r) * PCG_MULT + inc128(r);
  put_st(r, s);
  uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
  unsigned rot = (unsigned)(s >> 122);
  uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((-rot) & 63));
}

static uint32_t pcg64_next32(or_pcg64* r) {
  if (r->has32) { r->has32 = 0; return r->buf32; }
  uint64_t v = or_pcg64_next64(r);
  r->has32 = 1;
  r->buf32 = (uint32_t)(v >> 32);
  return (uint32_t)v;
}

double or_pcg64_double(or_pcg64* r) { return (double)(or_pcg64_next64(r) >> 11) * (1.0 / 9007199254740992.0); }

/* Generator.integers(high) for 1 <= high <= 2^32: buffered 32-bit Lemire (numpy) */
int64_t or_pcg64_integers(or_pcg64* r, int64_t high) {
  uint32_t rng = (uint32_t)(high - 1);
  if (rng == 0) return 0;
  uint32_t rng_excl = rng + 1;
  uint64_t m = (uint64_t)pcg64_next32(r) * rng_excl;
  uint32_t left = (uint32_t)m;
  if (left < rng_excl) {
    uint32_t thr = (uint32_t)(0xFFFFFFFFu - rng) % rng_excl;
    while (left < thr) {
      m = (uint64_t)pcg64_next32(r) * rng_excl;
      left = (uint32_t)m;
    }
  }
  return (int64_t)(m >> 32);
}

uint32_t or_episode_seed(uint64_t root, int index) { /* generate_dataset.py:263-268 */
  uint32_t w[2], out[1], key[1] = {(uint32_t)index};
  int n = seed_words(root, w);
  or_seedseq_state(w, n, key, 1, out, 1);
  return out[0];
}

/* randomization.py:70-98 ; returns attempts used, -1 on exhaustion */
int or_sample_positions(or_pcg64* r, const double* xr, const double* yr, double min_sep, double* xy) {
  for (int att = 0; att < 1000; att++) {
    double xs[3], ys[3];
    for (int i = 0; i < 3; i++) xs[i] = xr[0] + (xr[1] - xr[0]) * or_pcg64_double(r);
    for (int i = 0; i < 3; i++) ys[i] = yr[0] + (yr[1] - yr[0]) * or_pcg64_double(r);
    int ok = 1;
    for (int i = 0; i < 3 && ok; i++)
      for (int j = i + 1; j < 3; j++) {
        double dx = xs[i] - xs[j], dy = ys[i] - ys[j];
        if (dx * dx + dy * dy < min_sep * min_sep) { ok = 0; break; }
      }
    if (ok) {
      for (int i = 0; i < 3; i++) { xy[2 * i] = xs[i]; xy[2 * i + 1] = ys[i]; }
      return att + 1;
    }
  }
  return -1;
}

/* ======================================================================= gym env */
or_env* or_create(int action_mode, int reward_type, int max_episode_steps, int randomize, const double* sx,
                  const double* sy, int image_size) {
  or_env* e = (or_env*)calloc(1, sizeof(or_env));
  e->action_mode = action_mode;
  e->reward_type = reward_type;
  e->max_episode_steps = max_episode_steps;
  e->randomize = randomize;
  e->image_size = image_size;
  e->spawn_x[0] = sx ? sx[0] : -0.20; e->spawn_x[1] = sx ? sx[1] : 0.20;
  e->spawn_y[0] = sy ? sy[0] : 0.30; e->spawn_y[1] = sy ? sy[1] : 0.45;
  e->ntask = 9;
  for (int i = 0; i < 9; i++) { e->task_obj[i] = i / 3; e->task_bin[i] = i % 3; }
  e->fixed_obj = e->fixed_bin = -1;
  e->solver_tol = 1e-13;
  e->solver_maxiter = 200;
  e->solver_mj_tol = 0;
  or_pcg64_seed(&e->rng, 0);
  or_reset_keyframe(e);
  return e;
}
void or_destroy(or_env* e) { free(e); }
void or_set_task_pool(or_env* e, int n, const int* o, const int* b) {
  e->ntask = n;
  for (int i = 0; i < n; i++) { e->task_obj[i] = o[i]; e->task_bin[i] = b[i]; }
}
void or_set_fixed_task(or_env* e, int o, int b) { e->fixed_obj = o; e->fixed_bin = b; }

static void project(const or_env* e, int cam, const double* p, float* out) { /* cameras.py:56-104 */
  double fovy = OM_cam_fovy[cam] * M_PI / 180.0;
  double S = e->image_size;
  double f = (S / 2.0) / tan(fovy / 2.0);
  double rel[3], cc[3];
  v3_sub(rel, p, e->camxpos[cam]);
  m3_mulTv(cc, e->camxmat[cam], rel); /* rel @ cam_mat */
  double depth = cc[2];
  if (fabs(depth) < 1e-6) depth = 1e-6;
  double px = f * cc[0] / depth + S / 2.0;
  double py = -f * cc[1] / depth + S / 2.0;
  out[0] = (float)(px / S);
  out[1] = (float)(py / S);
}

static void se3_inv_mul(const double* Ti, const double* T, double* out) {
  /* out = inv(Ti) @ T, Ti rigid */
  double R[9], p[3], Rt[9], q[3];
  for (int i = 0; i < 3; i++) { for (int j = 0; j < 3; j++) R[3 * i + j] = Ti[4 * i + j]; p[i] = Ti[4 * i + 3]; }
  m3_transpose(Rt, R);
  memset(out, 0, 16 * sizeof(double));
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += Rt[3 * i + k] * T[4 * k + j];
      out[4 * i + j] = s;
    }
  for (int i = 0; i < 3; i++) q[i] = T[4 * i + 3] - p[i];
  double r[3];
  m3_mulv(r, Rt, q);
  for (int i = 0; i < 3; i++) out[4 * i + 3] = r[i];
  out[15] = 1;
}

static void enc_pose(const double* T, float g, float* q8, float* r10) { /* pose_utils.py:154-181 */
  double R[9], q[4];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = T[4 * i + j];
  or_rotmat_to_quat_xyzw(R, q);
  for (int i = 0; i < 3; i++) { q8[i] = (float)T[4 * i + 3]; r10[i] = (float)T[4 * i + 3]; }
  for (int i = 0; i < 4; i++) q8[3 + i] = (float)q[i];
  q8[7] = g;
  for (int i = 0; i < 6; i++) r10[3 + i] = (float)R[i];
  r10[9] = g;
}

void or_get_obs(or_env* e, float* o) { /* gym_env.py:283-339 (numeric part) */
  const int hand = OM_BODY_HAND;
  float g = (float)(e->ctrl[7] / 255.0);
  for (int i = 0; i < 3; i++) o[i] = (float)e->xpos[hand][i];
  o[3] = g;
  for (int i = 0; i < 7; i++) o[4 + i] = (float)e->qpos[i];
  double T[16] = {0};
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) T[4 * i + j] = e->xmat[hand][3 * i + j];
    T[4 * i + 3] = e->xpos[hand][i];
  }
  T[15] = 1;
  double Tr[16];
  se3_inv_mul(e->T_init, T, Tr);
  enc_pose(T, g, o + 11, o + 19);
  enc_pose(Tr, g, o + 29, o + 37);
  for (int i = 0; i < 3; i++) { o[47 + i] = (float)(i == e->bin); o[50 + i] = (float)(i == e->obj); }
  static const int KP[7] = {OM_BODY_OBJ_RED, OM_BODY_OBJ_GREEN, OM_BODY_OBJ_BLUE, OM_BODY_BIN_RED,
                            OM_BODY_BIN_GREEN, OM_BODY_BIN_BLUE, OM_BODY_HAND};
  for (int k = 0; k < 7; k++) {
    project(e, OM_CAM_OVERHEAD, e->xpos[KP[k]], o + 53 + 2 * k);
    project(e, OM_CAM_WRIST, e->xpos[KP[k]], o + 67 + 2 * k);
  }
  o[81] = e->tgt_obj_kp[0]; o[82] = e->tgt_obj_kp[1];
  o[83] = e->tgt_bin_kp[0]; o[84] = e->tgt_bin_kp[1];
}

/* returns 0, or -1 when the spawn sampling is exhausted: randomization.py:84-87 raises RuntimeError
 * there, leaving the env at the keyframe with step_count 0 (gym_env.py:492-501), no task drawn */
int or_reset(or_env* e, int seed_given, uint64_t seed, int tobj, int tbin, float* obs) { /* gym_env.py:477-534 */
  if (seed_given) or_pcg64_seed(&e->rng, seed);
  or_reset_keyframe(e);
  e->step_count = 0;
  if (e->randomize) { /* env.py:148-162 */
    double xy[6];
    if (or_sample_positions(&e->rng, e->spawn_x, e->spawn_y, 0.08, xy) < 0) return -1;
    for (int k = 0; k < 3; k++) {
      int qa = 9 + 7 * k;
      e->qpos[qa] = xy[2 * k]; e->qpos[qa + 1] = xy[2 * k + 1]; e->qpos[qa + 2] = 0.26;
      e->qpos[qa + 3] = 1; e->qpos[qa + 4] = e->qpos[qa + 5] = e->qpos[qa + 6] = 0;
    }
    or_mj_forward(e);
  }
  const int hand = OM_BODY_HAND;
  memset(e->T_init, 0, sizeof(e->T_init));
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) e->T_init[4 * i + j] = e->xmat[hand][3 * i + j];
    e->T_init[4 * i + 3] = e->xpos[hand][i];
  }
  e->T_init[15] = 1;
  e->has_grasped = e->has_lifted = e->above_target = e->has_placed = 0;
  e->hwm_valid = 0;
  memset(e->hwm, 0, sizeof(e->hwm));
  if (tobj >= 0) { e->obj = tobj; e->bin = tbin; }
  else if (e->fixed_obj >= 0) { e->obj = e->fixed_obj; e->bin = e->fixed_bin; }
  else {
    int idx = (int)or_pcg64_integers(&e->rng, e->ntask);
    e->obj = e->task_obj[idx];
    e->bin = e->task_bin[idx];
  }
  project(e, OM_CAM_OVERHEAD, e->xpos[OBJ_BODY[e->obj]], e->tgt_obj_kp);
  project(e, OM_CAM_OVERHEAD, e->xpos[BIN_BODY[e->bin]], e->tgt_bin_kp);
  if (obs) or_get_obs(e, obs);
  return 0;
}

static int robot_collision(const or_env* e) { /* gym_env.py:341-350 */
  for (int i = 0; i < e->ncon; i++) {
    int c1 = OM_geom_class[e->con[i].geom[0]], c2 = OM_geom_class[e->con[i].geom[1]];
    if ((c1 == 1 && c2 == 2) || (c1 == 2 && c2 == 1)) return 1;
  }
  return 0;
}

static double dmin1(double a, double b) { return a < b ? a : b; }
static double dmax1(double a, double b) { return a > b ? a : b; }

static double staged_reward(or_env* e, int* done) { /* gym_env.py:352-434 */
  const double DMAX = 0.5, GRASP_Z = 0.35, LIFT_Z = 0.42;
  const double* obj = e->xpos[OBJ_BODY[e->obj]];
  const double* bin = e->xpos[BIN_BODY[e->bin]];
  const double* ee = e->xpos[OM_BODY_HAND];
  int closed = e->ctrl[7] == 0.0;
  if (!e->has_grasped && obj[2] > GRASP_Z && closed) e->has_grasped = 1;
  if (!e->has_lifted && obj[2] > LIFT_Z && closed) e->has_lifted = 1;
  double xy = hypot(obj[0] - bin[0], obj[1] - bin[1]);
  if (!e->above_target && e->has_lifted && xy < 0.06) e->above_target = 1;
  int placed = xy < 0.05 && obj[2] < bin[2] + 0.06;
  if (!e->has_placed && placed) e->has_placed = 1;
  double d[3], r[5];
  v3_sub(d, ee, obj);
  r[0] = e->has_grasped ? 1.0 : 1.0 - dmin1(v3_norm(d) / DMAX, 1.0);
  if (!e->has_grasped) r[1] = 0;
  else if (e->has_lifted) r[1] = 1;
  else r[1] = dmax1(0.0, dmin1((obj[2] - 0.30) / (LIFT_Z - 0.30), 1.0));
  if (!e->has_lifted) r[2] = 0;
  else if (e->above_target) r[2] = 1;
  else r[2] = 1.0 - dmin1(xy / DMAX, 1.0);
  if (!e->above_target) r[3] = 0;
  else if (e->has_placed) r[3] = 1;
  else r[3] = 1.0 - dmax1(0.0, dmin1((obj[2] - bin[2]) / 0.25, 1.0));
  if (!e->has_placed) r[4] = 0;
  else {
    double ip[3] = {e->T_init[3], e->T_init[7], e->T_init[11]};
    v3_sub(d, ee, ip);
    r[4] = 1.0 - dmin1(v3_norm(d) / DMAX, 1.0);
  }
  if (!e->hwm_valid) { memset(e->hwm, 0, sizeof(e->hwm)); e->hwm_valid = 1; }
  for (int k = 0; k < 5; k++) e->hwm[k] = dmax1(e->hwm[k], r[k]);
  if (robot_collision(e)) { *done = 1; return -1.0; }
  double s = 0;
  int all = 1;
  for (int k = 0; k < 5; k++) { s += e->hwm[k]; all &= e->hwm[k] >= 0.90; }
  *done = all;
  return s / 5.0;
}

static double compute_reward(or_env* e, int* success) { /* gym_env.py:436-470 */
  const double* obj = e->xpos[OBJ_BODY[e->obj]];
  const double* bin = e->xpos[BIN_BODY[e->bin]];
  const double* ee = e->xpos[OM_BODY_HAND];
  double xy = hypot(obj[0] - bin[0], obj[1] - bin[1]);
  int succ = xy < 0.05 && obj[2] < bin[2] + 0.06;
  if (e->reward_type == 1) { *success = succ; return succ ? 1.0 : 0.0; }
  if (e->reward_type == 2) return staged_reward(e, success);
  double d[3], r = 0;
  v3_sub(d, ee, obj);
  r -= v3_norm(d);
  if (obj[2] > 0.30) {
    r += 2.0;
    v3_sub(d, obj, bin);
    r -= v3_norm(d);
  }
  if (succ) r += 10.0;
  *success = succ;
  return r;
}

double or_step(or_env* e, const float* action, float* obs, int* terminated, int* truncated, int* success,
               float* rc) { /* gym_env.py:536-581 */
  double target[3], grip;
  or_decode_action(e->action_mode, action, e->T_init, target, &grip);
  or_set_gripper(e, grip > 0.5);
  for (int s = 0; s < 16; s++) {
    double q[7];
    or_ik_compute(e, target, q);
    or_set_arm_ctrl(e, q);
    or_mj_step(e);
  }
  or_mj_forward(e);
  e->step_count++;
  int succ = 0;
  double reward = compute_reward(e, &succ);
  if (e->reward_type == 2) {
    *terminated = reward < 0 || succ;
    *success = succ && reward >= 0;
    if (rc) {
      double s = 0;
      for (int k = 0; k < 5; k++) s += e->hwm[k] / 5.0;
      rc[0] = (float)s;
      for (int k = 0; k < 5; k++) rc[1 + k] = (float)(e->hwm[k] / 5.0);
    }
  } else {
    *terminated = succ;
    *success = succ;
    if (rc) memset(rc, 0, 6 * sizeof(float));
  }
  *truncated = e->step_count >= e->max_episode_steps;
  if (obs) or_get_obs(e, obs);
  return reward;
}

void or_get_initial_ee(or_env* e, double* T16) { memcpy(T16, e->T_init, sizeof(e->T_init)); }
int or_step_count(or_env* e) { return e->step_count; }
void or_get_task(or_env* e, int* o, int* b) { *o = e->obj; *b = e->bin; }
void or_get_hwm(or_env* e, double* h) { memcpy(h, e->hwm, sizeof(e->hwm)); }

/* ======================================================================= test hooks
 * Overwrite derived quantities so golden traces generated with scripted body positions
 * (tests/golden/make_golden.py) can be replayed through the same task-layer code. */
void or_debug_set_xpos(or_env* e, int body, const double* p) { v3_copy(e->xpos[body], p); }
void or_debug_set_contacts(or_env* e, int n, const int* pairs) {
  e->ncon = n;
  for (int i = 0; i < n; i++) { e->con[i].geom[0] = pairs[2 * i]; e->con[i].geom[1] = pairs[2 * i + 1]; }
}
void or_debug_set_episode(or_env* e, int obj, int bin, const double* T16) {
  e->obj = obj;
  e->bin = bin;
  memcpy(e->T_init, T16, sizeof(e->T_init));
  e->has_grasped = e->has_lifted = e->above_target = e->has_placed = 0;
  e->hwm_valid = 0;
  memset(e->hwm, 0, sizeof(e->hwm));
}
double or_debug_reward(or_env* e, int* success) { return compute_reward(e, success); }
