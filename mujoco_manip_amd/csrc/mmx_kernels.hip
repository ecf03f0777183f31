// MI355X (gfx950) kernels for the batched pick-and-place simulator.
//
// Hot path replaced (reference): PickPlaceGymEnv.step (mujoco_manip/gym_env.py:536-581)
//   = decode_action -> 16 x (IKController.compute controller.py:87-137 ; mujoco.mj_step env.py:121)
//     -> mujoco.mj_forward (gym_env.py:560) -> reward (gym_env.py:352-470) -> obs (gym_env.py:283-339)
// plus reset/randomization (gym_env.py:477-534, randomization.py:11-98) and the FSM expert
// (pick_and_place.py:167-291).
//
// Execution model: one environment per wavefront lane, 64-lane workgroups (one wave each).
// All persistent state is SoA in HBM (field-major, env fastest: coalesced 256 B per wave per
// field).  Per-substep body poses, arm motion subspaces and the PGS acceleration vector live in
// LDS ([field][lane], conflict-free); constraint rows stream through a SoA scratch buffer in HBM.
// Physics follows MuJoCo's documented pipeline (see oracle/ for the fp64 restatement used as
// the checker): kinematics, CRBA + Cholesky, RNE, affine actuators + tendon, collision
// (plane-box, plane-convex, box-box SAT/clipping, GJK + EPA), soft constraints with
// solref/solimp impedance and pyramidal friction cones, a projected Gauss-Seidel dual solver,
// and the implicitfast integrator.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MMX_MODEL_QUAL static __constant__
#include "mmx_model_gen.h"
#include "mmx_device.h"
#include "mmx_state.h"

#define WG 64
#define LANE (threadIdx.x)
#define GF(ptr, f) (ptr)[(size_t)(f) * S.N + i]

// ---------------------------------------------------------------------------- LDS layout
#define NSLOT 14  // arm bodies 1..11 -> slots 0..10, cubes 16..18 -> slots 11..13
#define OFF_BX 0
#define OFF_BR (OFF_BX + NSLOT * 3 * WG)
#define OFF_S (OFF_BR + NSLOT * 9 * WG)
#define OFF_QACC (OFF_S + 9 * 6 * WG)
#define SH_TOTAL (OFF_QACC + 27 * WG)
#define SBX(slot, k) sh[OFF_BX + ((slot)*3 + (k)) * WG + LANE]
#define SBR(slot, k) sh[OFF_BR + ((slot)*9 + (k)) * WG + LANE]
#define SS(d, k) sh[OFF_S + ((d)*6 + (k)) * WG + LANE]
#define SQ(d) sh[OFF_QACC + (d)*WG + LANE]

static constexpr float kDt = 0.002f;
static constexpr float kHome[7] = {1.5708f, -0.2f, 0.0f, -2.1f, 0.0f, 1.8f, 0.785f};  // controller.py:8
static constexpr int kObjBody[3] = {MMX_BODY_OBJ_RED, MMX_BODY_OBJ_GREEN, MMX_BODY_OBJ_BLUE};
static constexpr int kBinBody[3] = {MMX_BODY_BIN_RED, MMX_BODY_BIN_GREEN, MMX_BODY_BIN_BLUE};

enum { GT_PLANE = 0, GT_CYL = 5, GT_BOX = 6, GT_MESH = 7 };

DEV int body_slot(int b) { return b <= 11 ? b - 1 : b - 5; }
// block of a body: 0 = arm (9 dofs), 1+k = cube k (6 dofs), -1 = static
DEV int body_block(int b) { return (b >= 2 && b <= 11) ? 0 : (b >= 16 ? b - 15 : -1); }
DEV int block_size(int blk) { return blk == 0 ? 9 : 6; }
DEV int block_dof0(int blk) { return blk == 0 ? 0 : 9 + 6 * (blk - 1); }
// is arm dof d an ancestor-or-self dof of arm body b
DEV bool arm_anc(int d, int b) { return d <= 6 ? (b >= d + 2 && b <= 11) : (d == 7 ? b == 10 : b == 11); }

DEV V3 ldv(const float* p) { return V3{p[0], p[1], p[2]}; }
DEV V3 body_x(const float* sh, int b) {
  if (MMX_body_static[b]) return V3{0.f, 0.f, 0.f};
  int s = body_slot(b);
  return V3{SBX(s, 0), SBX(s, 1), SBX(s, 2)};
}
DEV M3 body_R(const float* sh, int b) {
  M3 R;
  int s = body_slot(b);
#pragma unroll
  for (int k = 0; k < 9; k++) R.m[k] = SBR(s, k);
  return R;
}

// =========================================================================== kinematics
// mj_kinematics + motion subspaces for the arm (world-origin Plucker coordinates).  Writes body
// poses of the 10 moving arm bodies and 3 cubes to LDS.  All joint anchors of this model are at
// the body origin (jnt_pos = 0), asserted by the model compiler's output.
DEV void kinematics(float* sh, const float* qpos) {
  V3 px[12];
  Q4 pq[12];
  px[0] = V3{0.f, 0.f, 0.f};
  pq[0] = Q4{1.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 1; b <= 11; b++) {
    const int p = MMX_body_parent[b];
    M3 Rp = qmat(pq[p]);
    V3 pos = px[p] + mul(Rp, V3{MMX_body_pos[3 * b], MMX_body_pos[3 * b + 1], MMX_body_pos[3 * b + 2]});
    Q4 q = qmul(pq[p], Q4{MMX_body_quat[4 * b], MMX_body_quat[4 * b + 1], MMX_body_quat[4 * b + 2], MMX_body_quat[4 * b + 3]});
    const int j = MMX_body_jnt[b];
    if (j >= 0) {
      V3 axl = V3{MMX_jnt_axis[3 * j], MMX_jnt_axis[3 * j + 1], MMX_jnt_axis[3 * j + 2]};
      M3 R0 = qmat(qnormalize(q));
      V3 axw = mul(R0, axl);
      float qv = qpos[j];
      if (MMX_jnt_type[j] == 3) {  // hinge
        q = qmul(q, qaxisangle(axl, qv));
        SS(j, 0) = axw.x; SS(j, 1) = axw.y; SS(j, 2) = axw.z;
        V3 lin = cross(pos, axw);
        SS(j, 3) = lin.x; SS(j, 4) = lin.y; SS(j, 5) = lin.z;
      } else {  // slide
        SS(j, 0) = 0.f; SS(j, 1) = 0.f; SS(j, 2) = 0.f;
        SS(j, 3) = axw.x; SS(j, 4) = axw.y; SS(j, 5) = axw.z;
        pos = pos + axw * qv;
      }
    }
    q = qnormalize(q);
    px[b] = pos;
    pq[b] = q;
    M3 R = qmat(q);
    const int s = b - 1;
    SBX(s, 0) = pos.x; SBX(s, 1) = pos.y; SBX(s, 2) = pos.z;
#pragma unroll
    for (int k = 0; k < 9; k++) SBR(s, k) = R.m[k];
  }
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int qa = 9 + 7 * c;
    Q4 q = qnormalize(Q4{qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]});
    M3 R = qmat(q);
    const int s = 11 + c;
    SBX(s, 0) = qpos[qa]; SBX(s, 1) = qpos[qa + 1]; SBX(s, 2) = qpos[qa + 2];
#pragma unroll
    for (int k = 0; k < 9; k++) SBR(s, k) = R.m[k];
  }
}

DEV SV load_S(const float* sh, int d) { return SV{V3{SS(d, 0), SS(d, 1), SS(d, 2)}, V3{SS(d, 3), SS(d, 4), SS(d, 5)}}; }

// stale-kinematics cache for the next IK call (controller.py:99-110 reads xpos/xmat/mj_jac)
DEV void write_kin_cache(const MMXState& S, int i, const float* sh) {
  V3 hx = body_x(sh, MMX_BODY_HAND);
  M3 hR = body_R(sh, MMX_BODY_HAND);
  GF(S.kin, KIN_HAND_POS + 0) = hx.x; GF(S.kin, KIN_HAND_POS + 1) = hx.y; GF(S.kin, KIN_HAND_POS + 2) = hx.z;
#pragma unroll
  for (int k = 0; k < 9; k++) GF(S.kin, KIN_HAND_MAT + k) = hR.m[k];
#pragma unroll
  for (int d = 0; d < 7; d++) {
    V3 ax = V3{SS(d, 0), SS(d, 1), SS(d, 2)};
    V3 an = body_x(sh, d + 2);
    GF(S.kin, KIN_AXIS + 3 * d + 0) = ax.x; GF(S.kin, KIN_AXIS + 3 * d + 1) = ax.y; GF(S.kin, KIN_AXIS + 3 * d + 2) = ax.z;
    GF(S.kin, KIN_ANCHOR + 3 * d + 0) = an.x; GF(S.kin, KIN_ANCHOR + 3 * d + 1) = an.y; GF(S.kin, KIN_ANCHOR + 3 * d + 2) = an.z;
  }
}

// =========================================================================== arm dynamics
DEV RI body_inertia(const float* sh, int b) {
  V3 x = body_x(sh, b);
  M3 R = body_R(sh, b);
  const float m = MMX_body_mass[b];
  V3 c = x + mul(R, V3{MMX_body_ipos[3 * b], MMX_body_ipos[3 * b + 1], MMX_body_ipos[3 * b + 2]});
  // I_c = R Ib R^T
  M3 Ib;
#pragma unroll
  for (int k = 0; k < 9; k++) Ib.m[k] = MMX_body_inertia[9 * b + k];
  M3 T = mul(R, Ib);
  float Ic[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int cc = 0; cc < 3; cc++) Ic[3 * r + cc] = T.m[3 * r] * R.m[3 * cc] + T.m[3 * r + 1] * R.m[3 * cc + 1] + T.m[3 * r + 2] * R.m[3 * cc + 2];
  RI I;
  I.m = m;
  I.h = c * m;
  float cc2 = dot(c, c);
  I.J[0] = Ic[0] + m * (cc2 - c.x * c.x);
  I.J[1] = Ic[4] + m * (cc2 - c.y * c.y);
  I.J[2] = Ic[8] + m * (cc2 - c.z * c.z);
  I.J[3] = Ic[1] - m * c.x * c.y;
  I.J[4] = Ic[2] - m * c.x * c.z;
  I.J[5] = Ic[5] - m * c.y * c.z;
  return I;
}

// packed lower-triangular 9x9 index
#define LT(r, c) ((r) * ((r) + 1) / 2 + (c))

// CRBA for the 9 arm dofs (bodies 2..11) + armature; RNE bias for the arm.  Returns M (packed).
DEV void arm_dynamics(const float* sh, const float* qvel, float* Mp, float* bias) {
  RI Ib[12];
#pragma unroll
  for (int b = 2; b <= 11; b++) Ib[b] = body_inertia(sh, b);
  // ---- RNE (recursive Newton-Euler), base acceleration = -gravity
  SV vel[12], acc[12], frc[12];
  vel[1] = SV{V3{0.f, 0.f, 0.f}, V3{0.f, 0.f, 0.f}};
  acc[1] = SV{V3{0.f, 0.f, 0.f}, V3{0.f, 0.f, -MMX_GRAVITY_Z}};
#pragma unroll
  for (int b = 2; b <= 11; b++) {
    const int p = MMX_body_parent[b];
    const int j = MMX_body_jnt[b];
    vel[b] = vel[p];
    acc[b] = acc[p];
    if (j >= 0) {
      SV vj = load_S(sh, j) * qvel[j];
      acc[b] = acc[b] + cross_motion(vel[p], vj);
      vel[b] = vel[b] + vj;
    }
    frc[b] = rimul(Ib[b], acc[b]) + cross_force(vel[b], rimul(Ib[b], vel[b]));
  }
#pragma unroll
  for (int b = 11; b >= 3; b--) {
    const int p = MMX_body_parent[b];
    frc[p] = frc[p] + frc[b];
  }
  // ---- composite inertias
  RI Ic[12];
#pragma unroll
  for (int b = 2; b <= 11; b++) Ic[b] = Ib[b];
#pragma unroll
  for (int b = 11; b >= 3; b--) riadd(Ic[MMX_body_parent[b]], Ic[b]);
  SV Sd[9];
#pragma unroll
  for (int d = 0; d < 9; d++) Sd[d] = load_S(sh, d);
#pragma unroll
  for (int d = 0; d < 9; d++) {
    const int bd = MMX_jnt_body[d];
    bias[d] = sdot(Sd[d], frc[bd]);
    SV F = rimul(Ic[bd], Sd[d]);
#pragma unroll
    for (int e = 0; e <= d; e++) {
      const bool anc = (e == d) || (e <= 6 && (d <= 6 || true));
      float v = anc ? sdot(Sd[e], F) : 0.f;
      if (d == 8 && e == 7) v = 0.f;  // fingers are siblings
      Mp[LT(d, e)] = v;
    }
    Mp[LT(d, d)] += MMX_dof_armature[d];
  }
}

DEV bool chol9(float* L) {
#pragma unroll
  for (int j = 0; j < 9; j++) {
    float s = L[LT(j, j)];
#pragma unroll
    for (int k = 0; k < j; k++) s -= L[LT(j, k)] * L[LT(j, k)];
    s = fmaxf(s, 1e-12f);
    float d = sqrtf(s), inv = 1.0f / d;
    L[LT(j, j)] = d;
#pragma unroll
    for (int r = j + 1; r < 9; r++) {
      float t = L[LT(r, j)];
#pragma unroll
      for (int k = 0; k < j; k++) t -= L[LT(r, k)] * L[LT(j, k)];
      L[LT(r, j)] = t * inv;
    }
  }
  return true;
}
DEV void chol9_solve(const float* L, float* x) {
#pragma unroll
  for (int r = 0; r < 9; r++) {
    float s = x[r];
#pragma unroll
    for (int k = 0; k < r; k++) s -= L[LT(r, k)] * x[k];
    x[r] = s / L[LT(r, r)];
  }
#pragma unroll
  for (int r = 8; r >= 0; r--) {
    float s = x[r];
#pragma unroll
    for (int k = r + 1; k < 9; k++) s -= L[LT(k, r)] * x[k];
    x[r] = s / L[LT(r, r)];
  }
}

// =========================================================================== collision
struct Geom {
  V3 x;
  M3 R;
  int type, g;
};
DEV Geom geom_pose(const float* sh, int g) {
  Geom G;
  G.g = g;
  G.type = MMX_geom_type[g];
  const int b = MMX_geom_body[g];
  if (MMX_body_static[b]) {
    G.x = V3{MMX_geom_static_xpos[3 * g], MMX_geom_static_xpos[3 * g + 1], MMX_geom_static_xpos[3 * g + 2]};
#pragma unroll
    for (int k = 0; k < 9; k++) G.R.m[k] = MMX_geom_static_xmat[9 * g + k];
  } else {
    V3 bx = body_x(sh, b);
    M3 bR = body_R(sh, b);
    G.x = bx + mul(bR, V3{MMX_geom_pos[3 * g], MMX_geom_pos[3 * g + 1], MMX_geom_pos[3 * g + 2]});
    M3 L;
#pragma unroll
    for (int k = 0; k < 9; k++) L.m[k] = MMX_geom_lmat[9 * g + k];
    G.R = mul(bR, L);
  }
  return G;
}

DEV V3 support(const Geom& G, V3 dir) {
  V3 dl = mulT(G.R, dir), sl;
  const int g = G.g;
  if (G.type == GT_BOX) {
    sl = V3{dl.x >= 0.f ? MMX_geom_size[3 * g] : -MMX_geom_size[3 * g], dl.y >= 0.f ? MMX_geom_size[3 * g + 1] : -MMX_geom_size[3 * g + 1],
            dl.z >= 0.f ? MMX_geom_size[3 * g + 2] : -MMX_geom_size[3 * g + 2]};
  } else if (G.type == GT_CYL) {
    float r = MMX_geom_size[3 * g], hh = MMX_geom_size[3 * g + 1];
    float n = sqrtf(dl.x * dl.x + dl.y * dl.y);
    sl = n > 1e-12f ? V3{r * dl.x / n, r * dl.y / n, 0.f} : V3{r, 0.f, 0.f};
    sl.z = dl.z >= 0.f ? hh : -hh;
  } else {
    const int m = MMX_geom_mesh[g];
    const int a = MMX_mesh_vertadr[m], nvert = MMX_mesh_vertnum[m];
    float best = -3.0e38f;
    int bi = a;
    for (int v = a; v < a + nvert; v++) {
      float s = MMX_mesh_vert[3 * v] * dl.x + MMX_mesh_vert[3 * v + 1] * dl.y + MMX_mesh_vert[3 * v + 2] * dl.z;
      if (s > best) { best = s; bi = v; }
    }
    sl = V3{MMX_mesh_vert[3 * bi], MMX_mesh_vert[3 * bi + 1], MMX_mesh_vert[3 * bi + 2]};
  }
  return G.x + mul(G.R, sl);
}

DEV bool obb_overlap(const Geom& A, const Geom& B) {
  const float* ha = &MMX_geom_aabb[3 * A.g];
  const float* hb = &MMX_geom_aabb[3 * B.g];
  V3 d = B.x - A.x;
#pragma unroll
  for (int s = 0; s < 2; s++) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      V3 L = col(s ? B.R : A.R, k);
      float r1 = ha[0] * fabsf(dot(L, col(A.R, 0))) + ha[1] * fabsf(dot(L, col(A.R, 1))) + ha[2] * fabsf(dot(L, col(A.R, 2)));
      float r2 = hb[0] * fabsf(dot(L, col(B.R, 0))) + hb[1] * fabsf(dot(L, col(B.R, 1))) + hb[2] * fabsf(dot(L, col(B.R, 2)));
      if (fabsf(dot(d, L)) > r1 + r2) return false;
    }
  }
  return true;
}

struct ConSink {
  const MMXState* S;
  int i;
  int n;
  bool overflow;
  bool robot_obstacle;  // staged reward: any robot<->table/bin contact (gym_env.py:341-350)
};

DEV void add_contact(ConSink& cs, int g1, int g2, float dist, V3 pos, V3 nrm) {
  const int c1 = MMX_geom_class[g1], c2 = MMX_geom_class[g2];
  if ((c1 == 1 && c2 == 2) || (c1 == 2 && c2 == 1)) cs.robot_obstacle = true;
  if (cs.S == nullptr) return;
  if (cs.n >= MMX_MAXCON) { cs.overflow = true; return; }
  const MMXState& S = *cs.S;
  const int i = cs.i;
  float* base = S.con + (size_t)cs.n * CON_F * S.N;
#define CW(f) base[(size_t)(f) * S.N + i]
  nrm = normalize(nrm);
  CW(CON_DIST) = dist;
  CW(CON_POS + 0) = pos.x; CW(CON_POS + 1) = pos.y; CW(CON_POS + 2) = pos.z;
  CW(CON_N + 0) = nrm.x; CW(CON_N + 1) = nrm.y; CW(CON_N + 2) = nrm.z;
  CW(CON_MU0) = fmaxf(MMX_geom_friction[3 * g1], MMX_geom_friction[3 * g2]);
  CW(CON_MU1) = fmaxf(MMX_geom_friction[3 * g1 + 1], MMX_geom_friction[3 * g2 + 1]);
  CW(CON_MU2) = fmaxf(MMX_geom_friction[3 * g1 + 2], MMX_geom_friction[3 * g2 + 2]);
  CW(CON_DIM) = (float)max(MMX_geom_condim[g1], MMX_geom_condim[g2]);
  CW(CON_G1) = (float)g1;
  CW(CON_G2) = (float)g2;
#undef CW
  cs.n++;
}

DEV void plane_box(ConSink& cs, const Geom& P, const Geom& B) {
  V3 nz = col(P.R, 2);
  const float* h = &MMX_geom_size[3 * B.g];
  float depth[8];
  V3 pts[8];
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    V3 l = V3{(k & 1) ? h[0] : -h[0], (k & 2) ? h[1] : -h[1], (k & 4) ? h[2] : -h[2]};
    V3 w = B.x + mul(B.R, l);
    float d = dot(w - P.x, nz);
    if (d <= 0.f) {
      depth[cnt] = d;
      pts[cnt] = w - nz * (0.5f * d);
      cnt++;
    }
  }
  for (int k = 0; k < cnt && k < 4; k++) {
    int bi = k;
    for (int m = k + 1; m < cnt; m++)
      if (depth[m] < depth[bi]) bi = m;
    float td = depth[k]; depth[k] = depth[bi]; depth[bi] = td;
    V3 tp = pts[k]; pts[k] = pts[bi]; pts[bi] = tp;
    add_contact(cs, P.g, B.g, depth[k], pts[k], nz);
  }
}

DEV void plane_convex(ConSink& cs, const Geom& P, const Geom& C) {
  V3 nz = col(P.R, 2);
  V3 s = support(C, -nz);
  float d = dot(s - P.x, nz);
  if (d <= 0.f) add_contact(cs, P.g, C.g, d, s - nz * (0.5f * d), nz);
}

DEV int clip_poly(const V3* in, int n, V3* out, V3 a, float b) {
  int m = 0;
  for (int k = 0; k < n; k++) {
    V3 p = in[k], q = in[(k + 1) % n];
    float dp = dot(p, a) - b, dq = dot(q, a) - b;
    if (dp <= 0.f) out[m++] = p;
    if ((dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f)) {
      float t = dp / (dp - dq);
      out[m++] = p + (q - p) * t;
    }
  }
  return m;
}

// box-box: separating axis test over 15 axes; face contacts clip the incident face against the
// reference face (up to 8 points), edge-edge contacts give one point.
DEV void box_box(ConSink& cs, const Geom& G1, const Geom& G2) {
  const float* h1 = &MMX_geom_size[3 * G1.g];
  const float* h2 = &MMX_geom_size[3 * G2.g];
  V3 A[3] = {col(G1.R, 0), col(G1.R, 1), col(G1.R, 2)};
  V3 B[3] = {col(G2.R, 0), col(G2.R, 1), col(G2.R, 2)};
  V3 d = G2.x - G1.x;
  float best_face = 3e38f, best_edge = 3e38f;
  int face_axis = 0, ei = -1, ej = -1;
  V3 eL = V3{0.f, 0.f, 0.f};
#pragma unroll
  for (int ax = 0; ax < 6; ax++) {
    V3 L = ax < 3 ? A[ax] : B[ax - 3];
    float r1 = h1[0] * fabsf(dot(L, A[0])) + h1[1] * fabsf(dot(L, A[1])) + h1[2] * fabsf(dot(L, A[2]));
    float r2 = h2[0] * fabsf(dot(L, B[0])) + h2[1] * fabsf(dot(L, B[1])) + h2[2] * fabsf(dot(L, B[2]));
    float s = r1 + r2 - fabsf(dot(d, L));
    if (s < 0.f) return;
    if (s < best_face) { best_face = s; face_axis = ax; }
  }
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 3; b++) {
      V3 L = cross(A[a], B[b]);
      float ln = norm(L);
      if (ln < 1e-6f) continue;
      L = L * (1.0f / ln);
      float r1 = h1[0] * fabsf(dot(L, A[0])) + h1[1] * fabsf(dot(L, A[1])) + h1[2] * fabsf(dot(L, A[2]));
      float r2 = h2[0] * fabsf(dot(L, B[0])) + h2[1] * fabsf(dot(L, B[1])) + h2[2] * fabsf(dot(L, B[2]));
      float s = r1 + r2 - fabsf(dot(d, L));
      if (s < 0.f) return;
      if (s < best_edge) { best_edge = s; ei = a; ej = b; eL = L; }
    }
  if (ei >= 0 && best_edge < 0.95f * best_face - 1e-9f) {
    V3 L = dot(eL, d) < 0.f ? -eL : eL;
    V3 ca = G1.x, cb = G2.x;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k != ei) ca = ca + A[k] * (dot(A[k], L) >= 0.f ? h1[k] : -h1[k]);
      if (k != ej) cb = cb + B[k] * (dot(B[k], L) >= 0.f ? -h2[k] : h2[k]);
    }
    V3 ua = A[ei], ub = B[ej], w = ca - cb;
    float bb = dot(ua, ub), dd = dot(ua, w), ee = dot(ub, w);
    float den = 1.f - bb * bb;
    float ta = den > 1e-9f ? (bb * ee - dd) / den : 0.f;
    float tb = den > 1e-9f ? (ee - bb * dd) / den : 0.f;
    ta = fminf(fmaxf(ta, -h1[ei]), h1[ei]);
    tb = fminf(fmaxf(tb, -h2[ej]), h2[ej]);
    V3 pos = ((ca + ua * ta) + (cb + ub * tb)) * 0.5f;
    add_contact(cs, G1.g, G2.g, -best_edge, pos, L);
    return;
  }
  const bool ref1 = face_axis < 3;
  const int k = ref1 ? face_axis : face_axis - 3;
  const V3* Rr = ref1 ? A : B;
  const V3* Ri = ref1 ? B : A;
  const float* hr = ref1 ? h1 : h2;
  const float* hi = ref1 ? h2 : h1;
  V3 pr = ref1 ? G1.x : G2.x, pi = ref1 ? G2.x : G1.x;
  V3 nref = Rr[k];
  if (dot(nref, pi - pr) < 0.f) nref = -nref;
  int bj = 0;
  float bdot = 0.f;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    float t = fabsf(dot(Ri[j], nref));
    if (t > bdot) { bdot = t; bj = j; }
  }
  V3 ni = Ri[bj];
  if (dot(ni, nref) > 0.f) ni = -ni;
  V3 ci = pi + ni * hi[bj];
  const int u = (bj + 1) % 3, v = (bj + 2) % 3;
  V3 poly[16], tmp[16];
  int np = 4;
  poly[0] = ci + Ri[u] * hi[u] + Ri[v] * hi[v];
  poly[1] = ci - Ri[u] * hi[u] + Ri[v] * hi[v];
  poly[2] = ci - Ri[u] * hi[u] - Ri[v] * hi[v];
  poly[3] = ci + Ri[u] * hi[u] - Ri[v] * hi[v];
  V3 cr = pr + nref * hr[k];
  const int ru = (k + 1) % 3, rv = (k + 2) % 3;
  V3 ax0 = Rr[ru], ax1 = Rr[rv];
  np = clip_poly(poly, np, tmp, ax0, dot(ax0, cr) + hr[ru]);
  np = clip_poly(tmp, np, poly, -ax0, dot(-ax0, cr) + hr[ru]);
  np = clip_poly(poly, np, tmp, ax1, dot(ax1, cr) + hr[rv]);
  np = clip_poly(tmp, np, poly, -ax1, dot(-ax1, cr) + hr[rv]);
  V3 nout = ref1 ? nref : -nref;
  for (int c = 0; c < np; c++) {
    float depth = -dot(poly[c] - cr, nref);
    if (depth >= 0.f) add_contact(cs, G1.g, G2.g, -depth, poly[c] + nref * (0.5f * depth), nout);
  }
}

// ---- GJK + EPA (nativeccd-style convex path, one contact per pair)
struct SVx {
  V3 w, a, b;
};
DEV SVx mk_sv(const Geom& A, const Geom& B, V3 dir) {
  SVx s;
  s.a = support(A, dir);
  s.b = support(B, -dir);
  s.w = s.a - s.b;
  return s;
}

DEV bool gjk_line(SVx* S, int& n, V3& dir) {
  V3 ab = S[1].w - S[0].w, ao = -S[0].w;
  if (dot(ab, ao) > 0.f) {
    dir = cross(cross(ab, ao), ab);
    n = 2;
    return norm(dir) < 1e-12f * (1.f + dot(ab, ab));
  }
  n = 1;
  dir = ao;
  return false;
}
DEV bool gjk_tri(SVx* S, int& n, V3& dir) {
  V3 ab = S[1].w - S[0].w, ac = S[2].w - S[0].w, ao = -S[0].w;
  V3 abc = cross(ab, ac);
  if (dot(cross(abc, ac), ao) > 0.f) {
    if (dot(ac, ao) > 0.f) {
      S[1] = S[2];
      n = 2;
      dir = cross(cross(ac, ao), ac);
      return false;
    }
    n = 2;
    return gjk_line(S, n, dir);
  }
  if (dot(cross(ab, abc), ao) > 0.f) {
    n = 2;
    return gjk_line(S, n, dir);
  }
  float dd = dot(abc, ao);
  n = 3;
  if (fabsf(dd) < 1e-12f * (1.f + dot(abc, abc))) return true;
  if (dd > 0.f) dir = abc;
  else {
    SVx t = S[1]; S[1] = S[2]; S[2] = t;
    dir = -abc;
  }
  return false;
}
DEV bool gjk_tet(SVx* S, int& n, V3& dir) {
  V3 ao = -S[0].w;
  const int F[3][3] = {{0, 1, 2}, {0, 2, 3}, {0, 3, 1}};
  const int O[3] = {3, 1, 2};
  for (int f = 0; f < 3; f++) {
    V3 nn = cross(S[F[f][1]].w - S[0].w, S[F[f][2]].w - S[0].w);
    if (dot(nn, S[O[f]].w - S[0].w) > 0.f) nn = -nn;
    if (dot(nn, ao) > 0.f) {
      SVx t0 = S[F[f][0]], t1 = S[F[f][1]], t2 = S[F[f][2]];
      S[0] = t0; S[1] = t1; S[2] = t2;
      n = 3;
      return gjk_tri(S, n, dir);
    }
  }
  n = 4;
  return true;
}

DEV bool gjk(const Geom& A, const Geom& B, SVx* S, int& n) {
  V3 dir = A.x - B.x;
  if (norm(dir) < 1e-9f) dir = V3{1.f, 0.f, 0.f};
  S[0] = mk_sv(A, B, dir);
  n = 1;
  dir = -S[0].w;
  for (int it = 0; it < 48; it++) {
    if (norm(dir) < 1e-12f) return true;
    SVx P = mk_sv(A, B, dir);
    if (dot(P.w, dir) < 0.f) return false;
    for (int k = n; k > 0; k--) S[k] = S[k - 1];
    S[0] = P;
    n++;
    bool hit = n == 2 ? gjk_line(S, n, dir) : (n == 3 ? gjk_tri(S, n, dir) : gjk_tet(S, n, dir));
    if (hit) return true;
  }
  return norm(dir) < 1e-12f;
}

#define EPA_MAXV 40
#define EPA_MAXF 80
struct EFace {
  int v0, v1, v2;
  V3 n;
  float d;
};
DEV bool epa_face(const SVx* V, EFace& f, int a, int b, int c) {
  f.v0 = a; f.v1 = b; f.v2 = c;
  V3 n = cross(V[b].w - V[a].w, V[c].w - V[a].w);
  float ln = norm(n);
  if (ln < 1e-20f) return false;
  f.n = n * (1.f / ln);
  f.d = dot(f.n, V[a].w);
  return true;
}

DEV bool epa(const Geom& A, const Geom& B, SVx* V, int nv, V3& nrm, float& depth, V3& pa, V3& pb) {
  EFace F[EPA_MAXF];
  int nf = 0;
  const V3 dirs[6] = {V3{1.f, 0.f, 0.f}, V3{-1.f, 0.f, 0.f}, V3{0.f, 1.f, 0.f}, V3{0.f, -1.f, 0.f}, V3{0.f, 0.f, 1.f}, V3{0.f, 0.f, -1.f}};
  if (nv == 1) {
    for (int k = 0; k < 6 && nv < 2; k++) {
      V[nv] = mk_sv(A, B, dirs[k]);
      if (norm(V[nv].w - V[0].w) > 1e-7f) nv++;
    }
  }
  if (nv == 2) {
    V3 ab = V[1].w - V[0].w;
    V3 ax = fabsf(ab.x) <= fabsf(ab.y) && fabsf(ab.x) <= fabsf(ab.z) ? V3{1.f, 0.f, 0.f} : (fabsf(ab.y) <= fabsf(ab.z) ? V3{0.f, 1.f, 0.f} : V3{0.f, 0.f, 1.f});
    V3 t = normalize(cross(ab, ax));
    V[2] = mk_sv(A, B, t);
    if (norm(cross(V[2].w - V[0].w, ab)) < 1e-10f) V[2] = mk_sv(A, B, -t);
    nv = 3;
  }
  if (nv == 3) {
    V3 n = normalize(cross(V[1].w - V[0].w, V[2].w - V[0].w));
    V[3] = mk_sv(A, B, n);
    if (fabsf(dot(V[3].w - V[0].w, n)) < 1e-9f) V[3] = mk_sv(A, B, -n);
    nv = 4;
  }
  const int T[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
  V3 cen = (V[0].w + V[1].w + V[2].w + V[3].w) * 0.25f;
  for (int k = 0; k < 4; k++) {
    if (!epa_face(V, F[nf], T[k][0], T[k][1], T[k][2])) continue;
    if (dot(F[nf].n, V[T[k][0]].w - cen) < 0.f) epa_face(V, F[nf], T[k][0], T[k][2], T[k][1]);
    nf++;
  }
  int best = -1;
  for (int it = 0; it < 32; it++) {
    best = -1;
    float bd = 3e38f;
    for (int k = 0; k < nf; k++)
      if (F[k].d < bd) { bd = F[k].d; best = k; }
    if (best < 0) return false;
    SVx P = mk_sv(A, B, F[best].n);
    float dist = dot(P.w, F[best].n);
    if (dist - F[best].d < 1e-6f * (1.f + fabsf(dist)) || nv >= EPA_MAXV) break;
    int edges[EPA_MAXF * 3][2];
    int ne = 0;
    int m = 0;
    for (int k = 0; k < nf; k++) {
      EFace f = F[k];
      if (dot(f.n, P.w - V[f.v0].w) > 1e-9f) {
        int vv[3] = {f.v0, f.v1, f.v2};
        for (int e = 0; e < 3; e++) {
          int a = vv[e], b = vv[(e + 1) % 3];
          int found = -1;
          for (int q = 0; q < ne; q++)
            if (edges[q][0] == b && edges[q][1] == a) { found = q; break; }
          if (found >= 0) { edges[found][0] = edges[ne - 1][0]; edges[found][1] = edges[ne - 1][1]; ne--; }
          else if (ne < EPA_MAXF * 3) { edges[ne][0] = a; edges[ne][1] = b; ne++; }
        }
      } else {
        F[m++] = f;
      }
    }
    nf = m;
    const int pi = nv++;
    V[pi] = P;
    for (int q = 0; q < ne && nf < EPA_MAXF; q++)
      if (epa_face(V, F[nf], edges[q][0], edges[q][1], pi)) nf++;
  }
  if (best < 0) return false;
  const EFace& f = F[best];
  V3 p = f.n * f.d;
  V3 v0 = V[f.v1].w - V[f.v0].w, v1 = V[f.v2].w - V[f.v0].w, v2 = p - V[f.v0].w;
  float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
  float den = d00 * d11 - d01 * d01;
  float lv = den > 1e-30f ? (d11 * d20 - d01 * d21) / den : 0.f;
  float lw = den > 1e-30f ? (d00 * d21 - d01 * d20) / den : 0.f;
  float lu = 1.f - lv - lw;
  pa = V[f.v0].a * lu + V[f.v1].a * lv + V[f.v2].a * lw;
  pb = V[f.v0].b * lu + V[f.v1].b * lv + V[f.v2].b * lw;
  nrm = f.n;
  depth = f.d;
  return true;
}

DEV void convex_convex(ConSink& cs, const Geom& A, const Geom& B) {
  SVx V[EPA_MAXV];
  int n = 0;
  if (!gjk(A, B, V, n)) return;
  V3 nrm, pa, pb;
  float depth;
  if (!epa(A, B, V, n, nrm, depth, pa, pb)) return;
  if (depth < 0.f) return;
  add_contact(cs, A.g, B.g, -depth, (pa + pb) * 0.5f, nrm);
}

// broadphase over body pairs (bounding spheres), then geom pairs (spheres + OBB), narrowphase.
// only_robot_obstacle: evaluate just robot<->obstacle body pairs (staged-reward contact scan).
DEV void collide(ConSink& cs, const float* sh, bool only_robot_obstacle) {
  for (int bp = 0; bp < MMX_NBODYPAIR; bp++) {
    const int b1 = MMX_bodypair[4 * bp], b2 = MMX_bodypair[4 * bp + 1];
    const int start = MMX_bodypair[4 * bp + 2], cnt = MMX_bodypair[4 * bp + 3];
    if (only_robot_obstacle) {
      const int c1 = MMX_geom_class[MMX_bodypair_geoms[2 * start]], c2 = MMX_geom_class[MMX_bodypair_geoms[2 * start + 1]];
      if (!((c1 == 1 && c2 == 2) || (c1 == 2 && c2 == 1))) continue;
    }
    // body-level sphere test (world body = floor plane at z = 0 handled per geom below)
    if (b1 != 0 && b2 != 0) {
      V3 c1, c2;
      const float r1 = MMX_body_bsphere[4 * b1 + 3], r2 = MMX_body_bsphere[4 * b2 + 3];
      V3 l1 = V3{MMX_body_bsphere[4 * b1], MMX_body_bsphere[4 * b1 + 1], MMX_body_bsphere[4 * b1 + 2]};
      V3 l2 = V3{MMX_body_bsphere[4 * b2], MMX_body_bsphere[4 * b2 + 1], MMX_body_bsphere[4 * b2 + 2]};
      c1 = MMX_body_static[b1] ? l1 : body_x(sh, b1) + mul(body_R(sh, b1), l1);
      c2 = MMX_body_static[b2] ? l2 : body_x(sh, b2) + mul(body_R(sh, b2), l2);
      V3 dd = c2 - c1;
      if (dot(dd, dd) > (r1 + r2) * (r1 + r2)) continue;
    } else {
      const int bo = b1 == 0 ? b2 : b1;
      V3 l = V3{MMX_body_bsphere[4 * bo], MMX_body_bsphere[4 * bo + 1], MMX_body_bsphere[4 * bo + 2]};
      V3 c = body_x(sh, bo) + mul(body_R(sh, bo), l);
      if (c.z > MMX_body_bsphere[4 * bo + 3]) continue;
    }
    for (int p = start; p < start + cnt; p++) {
      int g1 = MMX_bodypair_geoms[2 * p], g2 = MMX_bodypair_geoms[2 * p + 1];
      int t1 = MMX_geom_type[g1], t2 = MMX_geom_type[g2];
      if (t1 > t2) { int t = g1; g1 = g2; g2 = t; t = t1; t1 = t2; t2 = t; }
      Geom A = geom_pose(sh, g1), B = geom_pose(sh, g2);
      if (t1 == GT_PLANE) {
        if (dot(B.x - A.x, col(A.R, 2)) > MMX_geom_rbound[g2]) continue;
        if (t2 == GT_BOX) plane_box(cs, A, B);
        else if (t2 == GT_MESH) plane_convex(cs, A, B);
        continue;
      }
      V3 dd = B.x - A.x;
      const float rb = MMX_geom_rbound[g1] + MMX_geom_rbound[g2];
      if (dot(dd, dd) > rb * rb) continue;
      if (!obb_overlap(A, B)) continue;
      if (t1 == GT_BOX && t2 == GT_BOX) box_box(cs, A, B);
      else convex_convex(cs, A, B);
    }
  }
}

// =========================================================================== constraints
DEV float impedance(const float* si, float pos) {
  float dmin = fminf(fmaxf(si[0], 1e-4f), 0.9999f), dmax = fminf(fmaxf(si[1], 1e-4f), 0.9999f);
  const float width = si[2], mid = si[3], power = si[4];
  if (dmin == dmax || width <= 1e-15f) return 0.5f * (dmin + dmax);
  float x = fabsf(pos / width);
  if (x >= 1.f) return dmax;
  if (x <= 0.f) return dmin;
  float y;
  if (power == 1.f) y = x;
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1.f);
  else y = 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
  return dmin + y * (dmax - dmin);
}

struct RowCtx {
  const MMXState* S;
  int i;
  int n;
  bool overflow;
  const float* L;      // arm Cholesky factor (packed)
  const float* qvel;   // [27]
  float mdiag[18];     // cube mass-matrix diagonal
};

// Write one row given its block-format Jacobian (slot layout: first block, then second block).
DEV void add_row(RowCtx& rc, int blk0, int blk1, const float* J, float pos, float diag, const float* solref,
                 const float* solimp) {
  if (rc.n >= MMX_MAXEFC) { rc.overflow = true; return; }
  const MMXState& S = *rc.S;
  const int i = rc.i;
  float* base = S.efc + (size_t)rc.n * EFC_F * S.N;
#define EW(f) base[(size_t)(f) * S.N + i]
  float MJ[15];
  int off = 0;
  float vel = 0.f, Aii = 0.f;
  for (int bk = 0; bk < 2; bk++) {
    const int blk = bk == 0 ? blk0 : blk1;
    if (blk < 0) continue;
    const int d0 = block_dof0(blk);
    if (blk == 0) {
      float x[9];
#pragma unroll
      for (int k = 0; k < 9; k++) x[k] = J[off + k];
      chol9_solve(rc.L, x);
#pragma unroll
      for (int k = 0; k < 9; k++) {
        MJ[off + k] = x[k];
        vel += J[off + k] * rc.qvel[k];
        Aii += J[off + k] * x[k];
      }
      off += 9;
    } else {
      const int c = blk - 1;
      for (int k = 0; k < 6; k++) {
        const float x = J[off + k] / rc.mdiag[6 * c + k];
        MJ[off + k] = x;
        vel += J[off + k] * rc.qvel[d0 + k];
        Aii += J[off + k] * x;
      }
      off += 6;
    }
  }
  for (int k = 0; k < off; k++) {
    EW(EFC_J + k) = J[k];
    EW(EFC_MJ + k) = MJ[k];
  }
  const float imp = impedance(solimp, pos);
  const float dmax = fminf(fmaxf(solimp[1], 1e-4f), 0.9999f);
  const float tc = fmaxf(solref[0], 2.f * kDt), dr = solref[1];
  const float K = 1.f / (dmax * dmax * tc * tc * dr * dr), Bd = 2.f / (dmax * tc);
  const float R = fmaxf((1.f - imp) / imp * diag, 1e-15f);
  EW(EFC_AREF) = -Bd * vel - K * imp * pos;
  EW(EFC_R) = R;
  EW(EFC_DINV) = 1.f / (Aii + R);
  EW(EFC_BLK) = __int_as_float((blk0 + 1) | ((blk1 + 1) << 4));
#undef EW
  rc.n++;
}

// Jacobian columns of a point on body b projected on (u: linear, w: angular), accumulated with
// sign sg into the block slots.  Arm bodies use the LDS motion subspaces; cubes use their pose.
DEV void body_jac_proj(const float* sh, int b, V3 p, V3 u, V3 w, float sg, float* Jb) {
  if (body_block(b) == 0) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
      if (!arm_anc(d, b)) continue;
      SV s = load_S(sh, d);
      V3 lin = s.v + cross(s.w, p);
      Jb[d] += sg * (dot(u, lin) + dot(w, s.w));
    }
  } else if (body_block(b) > 0) {
    V3 x = body_x(sh, b);
    M3 R = body_R(sh, b);
    Jb[0] += sg * u.x; Jb[1] += sg * u.y; Jb[2] += sg * u.z;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      V3 r = col(R, k);
      Jb[3 + k] += sg * (dot(u, cross(r, p - x)) + dot(w, r));
    }
  }
}

DEV void make_constraints(RowCtx& rc, const float* sh, const float* qpos) {
  const float def_ref[2] = {0.02f, 1.0f};
  const float def_imp[5] = {0.9f, 0.95f, 0.001f, 0.5f, 2.0f};
  float J[15];
  // equality finger_joint1 == finger_joint2 (panda.xml:261)
  {
#pragma unroll
    for (int k = 0; k < 15; k++) J[k] = 0.f;
    J[7] = 1.f; J[8] = -1.f;
    add_row(rc, 0, -1, J, qpos[7] - qpos[8], MMX_dof_invweight0[7] + MMX_dof_invweight0[8], MMX_eq_solref, MMX_eq_solimp);
  }
  // joint limits
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const float q = qpos[j];
    const float lo = MMX_jnt_range[2 * j], hi = MMX_jnt_range[2 * j + 1];
    for (int side = 0; side < 2; side++) {
      const float dist = side == 0 ? q - lo : hi - q;
      if (dist < 0.f) {
        for (int k = 0; k < 15; k++) J[k] = 0.f;
        J[j] = side == 0 ? 1.f : -1.f;
        add_row(rc, 0, -1, J, dist, MMX_dof_invweight0[j], def_ref, def_imp);
      }
    }
  }
  // contacts -> pyramidal rows J_n +/- mu_k J_k
  const MMXState& S = *rc.S;
  const int i = rc.i;
  const int ncon = min(S.epi[(size_t)EPI_NCON * S.N + i], MMX_MAXCON);
  for (int c = 0; c < ncon; c++) {
    const float* base = S.con + (size_t)c * CON_F * S.N;
#define CR(f) base[(size_t)(f) * S.N + i]
    const float dist = CR(CON_DIST);
    const V3 p = V3{CR(CON_POS), CR(CON_POS + 1), CR(CON_POS + 2)};
    const V3 n = V3{CR(CON_N), CR(CON_N + 1), CR(CON_N + 2)};
    const float mu[3] = {CR(CON_MU0), CR(CON_MU0), CR(CON_MU1)};
    const int dim = (int)CR(CON_DIM);
    const int g1 = (int)CR(CON_G1), g2 = (int)CR(CON_G2);
#undef CR
    const int b1 = MMX_geom_body[g1], b2 = MMX_geom_body[g2];
    int k1 = body_block(b1), k2 = body_block(b2);
    // slot assignment: arm block first, merge equal blocks
    int blk0 = k1 >= 0 ? k1 : k2, blk1 = (k1 >= 0 && k2 >= 0 && k2 != k1) ? k2 : -1;
    if (blk1 >= 0 && blk1 < blk0) { int t = blk0; blk0 = blk1; blk1 = t; }
    const int off1 = blk0 >= 0 ? block_size(blk0) : 0;
    // tangent frame (mju_makeFrame semantics)
    V3 y = (n.y < 0.5f && n.y > -0.5f) ? V3{0.f, 1.f, 0.f} : V3{0.f, 0.f, 1.f};
    V3 t1 = normalize(y - n * dot(n, y));
    V3 t2 = cross(n, t1);
    float solref[2], solimp[5];
#pragma unroll
    for (int k = 0; k < 2; k++) solref[k] = 0.5f * (MMX_geom_solref[2 * g1 + k] + MMX_geom_solref[2 * g2 + k]);
#pragma unroll
    for (int k = 0; k < 5; k++) solimp[k] = 0.5f * (MMX_geom_solimp[5 * g1 + k] + MMX_geom_solimp[5 * g2 + k]);
    const float tran = MMX_body_invweight0[2 * b1] + MMX_body_invweight0[2 * b2];
    const float rot = MMX_body_invweight0[2 * b1 + 1] + MMX_body_invweight0[2 * b2 + 1];
    const int nrows = dim == 1 ? 1 : 2 * (dim - 1);
    for (int r = 0; r < nrows; r++) {
      V3 u = n, w = V3{0.f, 0.f, 0.f};
      float diag = tran;
      if (dim > 1) {
        const int k = r >> 1;
        const float sg = (r & 1) ? -mu[k] : mu[k];
        if (k == 0) u = n + t1 * sg;
        else if (k == 1) u = n + t2 * sg;
        else w = n * sg;
        diag = tran + mu[k] * mu[k] * (k < 2 ? tran : rot);
      }
      float Jb1[9], Jb2[9];
#pragma unroll
      for (int k = 0; k < 9; k++) { Jb1[k] = 0.f; Jb2[k] = 0.f; }
      // J = J(b2) - J(b1); route each body's columns into its slot
      float* dst1 = (k1 >= 0 && k1 == blk0) ? Jb1 : Jb2;
      float* dst2 = (k2 >= 0 && k2 == blk0) ? Jb1 : Jb2;
      body_jac_proj(sh, b1, p, u, w, -1.f, dst1);
      body_jac_proj(sh, b2, p, u, w, 1.f, dst2);
#pragma unroll
      for (int k = 0; k < 15; k++) J[k] = 0.f;
      for (int k = 0; k < off1; k++) J[k] = Jb1[k];
      if (blk1 >= 0)
        for (int k = 0; k < 6; k++) J[off1 + k] = Jb2[k];
      add_row(rc, blk0, blk1, J, dist, diag, solref, solimp);
    }
  }
}

// projected Gauss-Seidel on the dual (MuJoCo's PGS formulation), matrix-free:
// qacc is kept consistent with f through the per-row M^-1 J^T columns.
DEV int pgs_solve(const MMXState& S, int i, float* sh, int nefc, const float* qacc_smooth, int max_iter, float tol,
                  float& resid) {
#pragma unroll
  for (int d = 0; d < 27; d++) SQ(d) = qacc_smooth[d];
  // warm start: f = proj(-(J qacc_ws - aref)/R)
  for (int r = 0; r < nefc; r++) {
    float* base = S.efc + (size_t)r * EFC_F * S.N;
#define EW(f) base[(size_t)(f) * S.N + i]
    const int bp = __float_as_int(EW(EFC_BLK));
    const int blk0 = (bp & 15) - 1, blk1 = (bp >> 4) - 1;
    float jq = 0.f;
    int off = 0;
    for (int bk = 0; bk < 2; bk++) {
      const int blk = bk == 0 ? blk0 : blk1;
      if (blk < 0) continue;
      const int d0 = block_dof0(blk), ns = block_size(blk);
      for (int k = 0; k < ns; k++) jq += EW(EFC_J + off + k) * GF(S.qacc_ws, d0 + k);
      off += ns;
    }
    float f = -(jq - EW(EFC_AREF)) / EW(EFC_R);
    const bool eq = (r == 0);
    if (!eq) f = fmaxf(f, 0.f);
    EW(EFC_FORCE) = f;
    off = 0;
    for (int bk = 0; bk < 2; bk++) {
      const int blk = bk == 0 ? blk0 : blk1;
      if (blk < 0) continue;
      const int d0 = block_dof0(blk), ns = block_size(blk);
      for (int k = 0; k < ns; k++) SQ(d0 + k) += f * EW(EFC_MJ + off + k);
      off += ns;
    }
  }
  int it = 0;
  bool conv = nefc == 0;
  resid = 0.f;
  while (it < max_iter && !conv) {
    float dmax = 0.f, fmax = 1e-6f;
    for (int r = 0; r < nefc; r++) {
      float* base = S.efc + (size_t)r * EFC_F * S.N;
      const int bp = __float_as_int(EW(EFC_BLK));
      const int blk0 = (bp & 15) - 1, blk1 = (bp >> 4) - 1;
      const float f = EW(EFC_FORCE);
      float g = EW(EFC_R) * f - EW(EFC_AREF);
      int off = 0;
      for (int bk = 0; bk < 2; bk++) {
        const int blk = bk == 0 ? blk0 : blk1;
        if (blk < 0) continue;
        const int d0 = block_dof0(blk), ns = block_size(blk);
        for (int k = 0; k < ns; k++) g += EW(EFC_J + off + k) * SQ(d0 + k);
        off += ns;
      }
      float fn = f - g * EW(EFC_DINV);
      if (r != 0) fn = fmaxf(fn, 0.f);
      const float df = fn - f;
      if (df != 0.f) {
        EW(EFC_FORCE) = fn;
        off = 0;
        for (int bk = 0; bk < 2; bk++) {
          const int blk = bk == 0 ? blk0 : blk1;
          if (blk < 0) continue;
          const int d0 = block_dof0(blk), ns = block_size(blk);
          for (int k = 0; k < ns; k++) SQ(d0 + k) += df * EW(EFC_MJ + off + k);
          off += ns;
        }
      }
      dmax = fmaxf(dmax, fabsf(df));
      fmax = fmaxf(fmax, fabsf(fn));
    }
#undef EW
    it++;
    resid = dmax / fmax;
    conv = resid < tol;
  }
  return it;
}

// =========================================================================== IK (controller.py:87-137)
DEV void orientation_error(const M3& Rc, V3& err) {
  // R_err = TARGET_ORI @ Rc^T, TARGET_ORI = [[0,1,0],[1,0,0],[0,0,-1]]
  float E[9];
  const float T[9] = {0.f, 1.f, 0.f, 1.f, 0.f, 0.f, 0.f, 0.f, -1.f};
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) E[3 * r + c] = T[3 * r] * Rc.m[3 * c] + T[3 * r + 1] * Rc.m[3 * c + 1] + T[3 * r + 2] * Rc.m[3 * c + 2];
  V3 v = V3{E[7] - E[5], E[2] - E[6], E[3] - E[1]};
  float cs = fminf(fmaxf((E[0] + E[4] + E[8] - 1.f) * 0.5f, -1.f), 1.f);
  float sn = 0.5f * norm(v);
  float ang = atan2f(sn, cs);  // == arccos(cs) on [0, pi], well conditioned near 0
  if (ang < 1e-6f || sn < 1e-12f) { err = V3{0.f, 0.f, 0.f}; return; }
  err = v * (ang / (2.f * sn));
}

DEV void chol6_solve(const float* A, float* x) {  // A packed lower (21), SPD
  float L[21];
#pragma unroll
  for (int k = 0; k < 21; k++) L[k] = A[k];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    float s = L[LT(j, j)];
#pragma unroll
    for (int k = 0; k < j; k++) s -= L[LT(j, k)] * L[LT(j, k)];
    float d = sqrtf(fmaxf(s, 1e-20f)), inv = 1.f / d;
    L[LT(j, j)] = d;
#pragma unroll
    for (int r = j + 1; r < 6; r++) {
      float t = L[LT(r, j)];
#pragma unroll
      for (int k = 0; k < j; k++) t -= L[LT(r, k)] * L[LT(j, k)];
      L[LT(r, j)] = t * inv;
    }
  }
#pragma unroll
  for (int r = 0; r < 6; r++) {
    float s = x[r];
#pragma unroll
    for (int k = 0; k < r; k++) s -= L[LT(r, k)] * x[k];
    x[r] = s / L[LT(r, r)];
  }
#pragma unroll
  for (int r = 5; r >= 0; r--) {
    float s = x[r];
#pragma unroll
    for (int k = r + 1; k < 6; k++) s -= L[LT(k, r)] * x[k];
    x[r] = s / L[LT(r, r)];
  }
}

// DLS IK with nullspace bias on the stale kinematics cache; writes ctrl[0:7]
DEV void ik_compute(const MMXState& S, int i, V3 tgt) {
  V3 ee = V3{GF(S.kin, KIN_HAND_POS), GF(S.kin, KIN_HAND_POS + 1), GF(S.kin, KIN_HAND_POS + 2)};
  M3 Rc;
#pragma unroll
  for (int k = 0; k < 9; k++) Rc.m[k] = GF(S.kin, KIN_HAND_MAT + k);
  float J[6][7];
#pragma unroll
  for (int d = 0; d < 7; d++) {
    V3 ax = V3{GF(S.kin, KIN_AXIS + 3 * d), GF(S.kin, KIN_AXIS + 3 * d + 1), GF(S.kin, KIN_AXIS + 3 * d + 2)};
    V3 an = V3{GF(S.kin, KIN_ANCHOR + 3 * d), GF(S.kin, KIN_ANCHOR + 3 * d + 1), GF(S.kin, KIN_ANCHOR + 3 * d + 2)};
    V3 jp = cross(ax, ee - an);
    J[0][d] = jp.x; J[1][d] = jp.y; J[2][d] = jp.z;
    J[3][d] = ax.x; J[4][d] = ax.y; J[5][d] = ax.z;
  }
  V3 ori;
  orientation_error(Rc, ori);
  float e6[6] = {tgt.x - ee.x, tgt.y - ee.y, tgt.z - ee.z, ori.x, ori.y, ori.z};
  float A[21];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c <= r; c++) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 7; k++) s += J[r][k] * J[c][k];
      A[LT(r, c)] = s + (r == c ? 1e-3f : 0.f);
    }
  float q[7], b[7], dq[7];
#pragma unroll
  for (int k = 0; k < 7; k++) {
    q[k] = GF(S.qpos, k);
    b[k] = 0.5f * (kHome[k] - q[k]);
  }
  // dq = J^T A^-1 e ;  N b = b - J^T A^-1 (J b)
  float y[6], z[6];
#pragma unroll
  for (int r = 0; r < 6; r++) {
    y[r] = e6[r];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 7; k++) s += J[r][k] * b[k];
    z[r] = s;
  }
  chol6_solve(A, y);
  chol6_solve(A, z);
  float n2 = 0.f;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    float s = b[k];
#pragma unroll
    for (int r = 0; r < 6; r++) s += J[r][k] * (y[r] - z[r]);
    dq[k] = s;
    n2 += s * s;
  }
  const float nrm = sqrtf(n2);
  const float scl = nrm > 5.0f ? 5.0f / nrm : 1.0f;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    float t = q[k] + dq[k] * scl;
    const float lo = MMX_jnt_range[2 * k], hi = MMX_jnt_range[2 * k + 1];
    if (lo < hi) t = fminf(fmaxf(t, lo), hi);
    GF(S.ctrl, k) = t;
  }
}

// =========================================================================== mj_step
DEV void mj_step_lane(const MMXState& S, int i, float* sh) {
  float qpos[30], qvel[27], ctrl[8];
#pragma unroll
  for (int k = 0; k < 30; k++) qpos[k] = GF(S.qpos, k);
#pragma unroll
  for (int k = 0; k < 27; k++) qvel[k] = GF(S.qvel, k);
#pragma unroll
  for (int k = 0; k < 8; k++) ctrl[k] = GF(S.ctrl, k);
  // ---- position stage
  kinematics(sh, qpos);
  write_kin_cache(S, i, sh);
  float M[45], L[45], bias[9];
  arm_dynamics(sh, qvel, M, bias);
#pragma unroll
  for (int k = 0; k < 45; k++) L[k] = M[k];
  chol9(L);
  ConSink cs{&S, i, 0, false, false};
  collide(cs, sh, false);
  GF(S.epi, EPI_NCON) = cs.n;
  RowCtx rc;
  rc.S = &S; rc.i = i; rc.n = 0; rc.overflow = false; rc.L = L; rc.qvel = qvel;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int b = 16 + c;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      rc.mdiag[6 * c + k] = MMX_body_mass[b];
      rc.mdiag[6 * c + 3 + k] = MMX_body_inertia[9 * b + 4 * k];
    }
  }
  make_constraints(rc, sh, qpos);
  GF(S.epi, EPI_NEFC) = rc.n;
  if (cs.overflow) GF(S.epi, EPI_ERROR) |= ERR_CON_OVERFLOW;
  if (rc.overflow) GF(S.epi, EPI_ERROR) |= ERR_EFC_OVERFLOW;
  // ---- velocity / actuation stage
  float qfrc[27];
  float tlen = MMX_tendon_coef[0] * qpos[7] + MMX_tendon_coef[1] * qpos[8];
  float tvel = MMX_tendon_coef[0] * qvel[7] + MMX_tendon_coef[1] * qvel[8];
  bool act_unclamped[8];
#pragma unroll
  for (int d = 0; d < 9; d++) qfrc[d] = -MMX_dof_damping[d] * qvel[d] - bias[d];
#pragma unroll
  for (int a = 0; a < 8; a++) {
    const float c = fminf(fmaxf(ctrl[a], MMX_act_ctrlrange[2 * a]), MMX_act_ctrlrange[2 * a + 1]);
    const int j = MMX_act_trn_joint[a];
    const float len = j >= 0 ? qpos[j] : tlen, vel = j >= 0 ? qvel[j] : tvel;
    float f = MMX_act_gain[a] * c + MMX_act_bias[3 * a] + MMX_act_bias[3 * a + 1] * len + MMX_act_bias[3 * a + 2] * vel;
    act_unclamped[a] = f > MMX_act_forcerange[2 * a] && f < MMX_act_forcerange[2 * a + 1];
    f = fminf(fmaxf(f, MMX_act_forcerange[2 * a]), MMX_act_forcerange[2 * a + 1]);
    if (j >= 0) qfrc[j] += f;
    else {
      qfrc[7] += MMX_tendon_coef[0] * f;
      qfrc[8] += MMX_tendon_coef[1] * f;
    }
  }
  float qacc_s[27];
#pragma unroll
  for (int d = 0; d < 9; d++) qacc_s[d] = qfrc[d];
  chol9_solve(L, qacc_s);
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int b = 16 + c;
    const float m = MMX_body_mass[b];
    // free body with com at the origin: bias = gravity + w x (I w) (body frame)
    const float I0 = MMX_body_inertia[9 * b], I1 = MMX_body_inertia[9 * b + 4], I2 = MMX_body_inertia[9 * b + 8];
    const int da = 9 + 6 * c;
    V3 w = V3{qvel[da + 3], qvel[da + 4], qvel[da + 5]};
    V3 gyro = cross(w, V3{I0 * w.x, I1 * w.y, I2 * w.z});
    qfrc[da] = 0.f; qfrc[da + 1] = 0.f; qfrc[da + 2] = MMX_GRAVITY_Z * m;
    qfrc[da + 3] = -gyro.x; qfrc[da + 4] = -gyro.y; qfrc[da + 5] = -gyro.z;
    qacc_s[da] = 0.f; qacc_s[da + 1] = 0.f; qacc_s[da + 2] = MMX_GRAVITY_Z;
    qacc_s[da + 3] = qfrc[da + 3] / I0; qacc_s[da + 4] = qfrc[da + 4] / I1; qacc_s[da + 5] = qfrc[da + 5] / I2;
  }
  // ---- constraint solve
  float resid = 0.f;
  const int iters = pgs_solve(S, i, sh, rc.n, qacc_s, S.pgs_max_iter, S.pgs_tol, resid);
  GF(S.stats, STAT_NEFC) += (float)rc.n;
  GF(S.stats, STAT_NCON) += (float)cs.n;
  GF(S.stats, STAT_PGS_ITER) += (float)iters;
  GF(S.stats, STAT_SUBSTEPS) += 1.f;
  GF(S.stats, STAT_RESID) = fmaxf(GF(S.stats, STAT_RESID), resid);
  float qacc[27];
#pragma unroll
  for (int d = 0; d < 27; d++) qacc[d] = SQ(d);
  // ---- implicitfast: (M - h qDeriv) qacc = qfrc_smooth + qfrc_constraint (arm block)
  float rhs[9], MD[45];
  {
    float dqa[9];
#pragma unroll
    for (int d = 0; d < 9; d++) dqa[d] = qacc[d] - qacc_s[d];
    // qfrc_constraint = M (qacc - qacc_smooth)
#pragma unroll
    for (int r = 0; r < 9; r++) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 9; c++) s += M[r >= c ? LT(r, c) : LT(c, r)] * dqa[c];
      rhs[r] = qfrc[r] + s;
    }
  }
#pragma unroll
  for (int k = 0; k < 45; k++) MD[k] = M[k];
#pragma unroll
  for (int d = 0; d < 9; d++) MD[LT(d, d)] += kDt * MMX_dof_damping[d];
#pragma unroll
  for (int a = 0; a < 7; a++)
    if (act_unclamped[a]) MD[LT(a, a)] -= kDt * MMX_act_bias[3 * a + 2];
  if (act_unclamped[7]) {
    const float bv = MMX_act_bias[3 * 7 + 2];
    const float c0 = MMX_tendon_coef[0], c1 = MMX_tendon_coef[1];
    MD[LT(7, 7)] -= kDt * bv * c0 * c0;
    MD[LT(8, 8)] -= kDt * bv * c1 * c1;
    MD[LT(8, 7)] -= kDt * bv * c0 * c1;
  }
  chol9(MD);
  chol9_solve(MD, rhs);
  // warm start stores the solver's qacc
#pragma unroll
  for (int d = 0; d < 27; d++) GF(S.qacc_ws, d) = qacc[d];
#pragma unroll
  for (int d = 0; d < 9; d++) qacc[d] = rhs[d];
  // ---- mj_advance
  bool bad = false;
#pragma unroll
  for (int d = 0; d < 27; d++) {
    qvel[d] += kDt * qacc[d];
    bad |= !(fabsf(qvel[d]) < 1e10f);
  }
#pragma unroll
  for (int d = 0; d < 9; d++) qpos[d] += kDt * qvel[d];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int qa = 9 + 7 * c, da = 9 + 6 * c;
    qpos[qa] += kDt * qvel[da];
    qpos[qa + 1] += kDt * qvel[da + 1];
    qpos[qa + 2] += kDt * qvel[da + 2];
    V3 w = V3{qvel[da + 3], qvel[da + 4], qvel[da + 5]};
    const float wn = norm(w);
    Q4 q = qnormalize(Q4{qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]});
    if (wn > 0.f) q = qmul(q, qaxisangle(w * (1.f / wn), wn * kDt));
    q = qnormalize(q);
    qpos[qa + 3] = q.w; qpos[qa + 4] = q.x; qpos[qa + 5] = q.y; qpos[qa + 6] = q.z;
  }
  if (bad) GF(S.epi, EPI_ERROR) |= ERR_NAN;
#pragma unroll
  for (int k = 0; k < 30; k++) GF(S.qpos, k) = qpos[k];
#pragma unroll
  for (int k = 0; k < 27; k++) GF(S.qvel, k) = qvel[k];
}

// =========================================================================== RNG (numpy PCG64)
struct Pcg {
  unsigned long long shi, slo, ihi, ilo;
};
DEV unsigned long long pcg_next64(Pcg& r) {
  const unsigned long long MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  unsigned long long lo = r.slo * ML;
  unsigned long long hi = __umul64hi(r.slo, ML) + r.slo * MH + r.shi * ML;
  unsigned long long nlo = lo + r.ilo;
  hi += r.ihi + (nlo < lo ? 1ull : 0ull);
  r.slo = nlo;
  r.shi = hi;
  unsigned long long x = hi ^ nlo;
  unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
DEV double pcg_double(Pcg& r) { return (double)(pcg_next64(r) >> 11) * (1.0 / 9007199254740992.0); }
DEV Pcg load_rng(const MMXState& S, int i) {
  return Pcg{S.rng[(size_t)0 * S.N + i], S.rng[(size_t)1 * S.N + i], S.rng[(size_t)2 * S.N + i], S.rng[(size_t)3 * S.N + i]};
}
DEV void store_rng(const MMXState& S, int i, const Pcg& r) {
  S.rng[(size_t)0 * S.N + i] = r.shi;
  S.rng[(size_t)1 * S.N + i] = r.slo;
}
// Generator.integers(high): buffered 32-bit Lemire on next_uint32 (low half first)
DEV int pcg_integers(const MMXState& S, int i, Pcg& r, int high) {
  const unsigned rng = (unsigned)(high - 1);
  if (rng == 0) return 0;
  auto next32 = [&]() -> unsigned {
    if (GF(S.epi, EPI_RNG_HAS32)) {
      GF(S.epi, EPI_RNG_HAS32) = 0;
      return S.rng32[i];
    }
    unsigned long long v = pcg_next64(r);
    GF(S.epi, EPI_RNG_HAS32) = 1;
    S.rng32[i] = (unsigned)(v >> 32);
    return (unsigned)v;
  };
  const unsigned excl = rng + 1;
  unsigned long long m = (unsigned long long)next32() * excl;
  unsigned left = (unsigned)m;
  if (left < excl) {
    const unsigned thr = (0xFFFFFFFFu - rng) % excl;
    while (left < thr) {
      m = (unsigned long long)next32() * excl;
      left = (unsigned)m;
    }
  }
  return (int)(m >> 32);
}

// =========================================================================== task layer
DEV V3 hand_pos(const MMXState& S, int i) { return V3{GF(S.kin, KIN_HAND_POS), GF(S.kin, KIN_HAND_POS + 1), GF(S.kin, KIN_HAND_POS + 2)}; }
DEV V3 obj_pos(const MMXState& S, int i, int o) { return V3{GF(S.qpos, 9 + 7 * o), GF(S.qpos, 10 + 7 * o), GF(S.qpos, 11 + 7 * o)}; }
DEV V3 bin_pos(int bn) {
  const int b = kBinBody[bn];
  // bins are static: their body origin is the constant body pos (parent = world)
  return V3{MMX_body_pos[3 * b], MMX_body_pos[3 * b + 1], MMX_body_pos[3 * b + 2]};
}

DEV void project(V3 p, V3 cx, const M3& cR, float fovy_deg, float* out) {  // cameras.py:56-104
  const float t = tanf(fovy_deg * (3.14159265358979f / 180.f) * 0.5f);
  V3 cc = mulT(cR, p - cx);
  float depth = cc.z;
  if (fabsf(depth) < 1e-6f) depth = 1e-6f;
  // px/S = f x / (depth S) + 1/2 with f = (S/2)/tan(fovy/2): independent of S
  out[0] = cc.x / (depth * 2.f * t) + 0.5f;
  out[1] = -cc.y / (depth * 2.f * t) + 0.5f;
}

DEV void camera_pose(int cam, V3 hx, const M3& hR, V3& cx, M3& cR) {
  Q4 q = Q4{MMX_cam_quat[4 * cam], MMX_cam_quat[4 * cam + 1], MMX_cam_quat[4 * cam + 2], MMX_cam_quat[4 * cam + 3]};
  M3 lq = qmat(q);
  V3 lp = V3{MMX_cam_pos[3 * cam], MMX_cam_pos[3 * cam + 1], MMX_cam_pos[3 * cam + 2]};
  if (MMX_cam_body[cam] == 0) {
    cx = lp;
    cR = lq;
  } else {
    cx = hx + mul(hR, lp);
    cR = mul(hR, lq);
  }
}

DEV void rotmat_to_quat_xyzw(const float* R, float* q) {  // pose_utils.py:48-82 (branch-exact)
  const float tr = R[0] + R[4] + R[8];
  float s, w, x, y, z;
  if (tr > 0.f) {
    s = 2.f * sqrtf(tr + 1.f);
    w = 0.25f * s; x = (R[7] - R[5]) / s; y = (R[2] - R[6]) / s; z = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    s = 2.f * sqrtf(1.f + R[0] - R[4] - R[8]);
    w = (R[7] - R[5]) / s; x = 0.25f * s; y = (R[1] + R[3]) / s; z = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    s = 2.f * sqrtf(1.f + R[4] - R[0] - R[8]);
    w = (R[2] - R[6]) / s; x = (R[1] + R[3]) / s; y = 0.25f * s; z = (R[5] + R[7]) / s;
  } else {
    s = 2.f * sqrtf(1.f + R[8] - R[0] - R[4]);
    w = (R[3] - R[1]) / s; x = (R[2] + R[6]) / s; y = (R[5] + R[7]) / s; z = 0.25f * s;
  }
  q[0] = x; q[1] = y; q[2] = z; q[3] = w;
}

DEV void write_obs(const MMXState& S, int i) {  // gym_env.py:283-339 (numeric part, 85 floats)
  V3 hx = hand_pos(S, i);
  M3 hR;
#pragma unroll
  for (int k = 0; k < 9; k++) hR.m[k] = GF(S.kin, KIN_HAND_MAT + k);
  float o[MMX_NOBS];
  const float g = GF(S.ctrl, 7) / 255.f;
  o[0] = hx.x; o[1] = hx.y; o[2] = hx.z; o[3] = g;
#pragma unroll
  for (int k = 0; k < 7; k++) o[4 + k] = GF(S.qpos, k);
  // T_rel = inv(T_init) T_cur
  float Ri[9];
  V3 pi;
#pragma unroll
  for (int k = 0; k < 9; k++) Ri[k] = GF(S.epf, EPF_TINIT + k);
  pi = V3{GF(S.epf, EPF_TINIT + 9), GF(S.epf, EPF_TINIT + 10), GF(S.epf, EPF_TINIT + 11)};
  float Rr[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) Rr[3 * r + c] = Ri[r] * hR.m[c] + Ri[3 + r] * hR.m[3 + c] + Ri[6 + r] * hR.m[6 + c];
  V3 dpp = hx - pi;
  V3 pr = V3{Ri[0] * dpp.x + Ri[3] * dpp.y + Ri[6] * dpp.z, Ri[1] * dpp.x + Ri[4] * dpp.y + Ri[7] * dpp.z,
             Ri[2] * dpp.x + Ri[5] * dpp.y + Ri[8] * dpp.z};
  for (int rel = 0; rel < 2; rel++) {
    const float* R = rel ? Rr : hR.m;
    V3 p = rel ? pr : hx;
    float* q8 = o + (rel ? 29 : 11);
    float* r10 = o + (rel ? 37 : 19);
    float q[4];
    rotmat_to_quat_xyzw(R, q);
    q8[0] = p.x; q8[1] = p.y; q8[2] = p.z;
    q8[3] = q[0]; q8[4] = q[1]; q8[5] = q[2]; q8[6] = q[3]; q8[7] = g;
    r10[0] = p.x; r10[1] = p.y; r10[2] = p.z;
#pragma unroll
    for (int k = 0; k < 6; k++) r10[3 + k] = R[k];
    r10[9] = g;
  }
  const int ob = GF(S.epi, EPI_OBJ), bn = GF(S.epi, EPI_BIN);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    o[47 + k] = (k == bn) ? 1.f : 0.f;
    o[50 + k] = (k == ob) ? 1.f : 0.f;
  }
  V3 kp[7] = {obj_pos(S, i, 0), obj_pos(S, i, 1), obj_pos(S, i, 2), bin_pos(0), bin_pos(1), bin_pos(2), hx};
  V3 cx;
  M3 cR;
  camera_pose(MMX_CAM_OVERHEAD, hx, hR, cx, cR);
#pragma unroll
  for (int k = 0; k < 7; k++) project(kp[k], cx, cR, MMX_cam_fovy[MMX_CAM_OVERHEAD], o + 53 + 2 * k);
  camera_pose(MMX_CAM_WRIST, hx, hR, cx, cR);
#pragma unroll
  for (int k = 0; k < 7; k++) project(kp[k], cx, cR, MMX_cam_fovy[MMX_CAM_WRIST], o + 67 + 2 * k);
#pragma unroll
  for (int k = 0; k < 4; k++) o[81 + k] = GF(S.epf, EPF_TGTKP + k);
#pragma unroll
  for (int k = 0; k < MMX_NOBS; k++) GF(S.obs, k) = o[k];
}

// reset one env (gym_env.py:477-534); seeded RNG state already in S.rng when requested
DEV void reset_lane(const MMXState& S, int i, float* sh, int task_override) {
#pragma unroll
  for (int k = 0; k < 30; k++) GF(S.qpos, k) = MMX_key_qpos[k];
#pragma unroll
  for (int k = 0; k < 27; k++) { GF(S.qvel, k) = 0.f; GF(S.qacc_ws, k) = 0.f; }
#pragma unroll
  for (int k = 0; k < 8; k++) GF(S.ctrl, k) = MMX_key_ctrl[k];
  Pcg r = load_rng(S, i);
  if (S.randomize) {  // randomization.py:70-98
    double xs[3] = {0, 0, 0}, ys[3] = {0, 0, 0};
    bool ok = false;
    for (int att = 0; att < 1000 && !ok; att++) {
      for (int k = 0; k < 3; k++) xs[k] = (double)S.spawn_x0 + ((double)S.spawn_x1 - (double)S.spawn_x0) * pcg_double(r);
      for (int k = 0; k < 3; k++) ys[k] = (double)S.spawn_y0 + ((double)S.spawn_y1 - (double)S.spawn_y0) * pcg_double(r);
      ok = true;
      for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++) {
          double dx = xs[a] - xs[b], dy = ys[a] - ys[b];
          if (dx * dx + dy * dy < 0.08 * 0.08) ok = false;
        }
    }
    if (!ok) GF(S.epi, EPI_ERROR) |= ERR_SAMPLING;
    for (int k = 0; k < 3; k++) {
      const int qa = 9 + 7 * k;
      GF(S.qpos, qa) = (float)xs[k]; GF(S.qpos, qa + 1) = (float)ys[k]; GF(S.qpos, qa + 2) = 0.26f;
      GF(S.qpos, qa + 3) = 1.f; GF(S.qpos, qa + 4) = 0.f; GF(S.qpos, qa + 5) = 0.f; GF(S.qpos, qa + 6) = 0.f;
    }
  }
  float qpos[30];
#pragma unroll
  for (int k = 0; k < 30; k++) qpos[k] = GF(S.qpos, k);
  kinematics(sh, qpos);
  write_kin_cache(S, i, sh);
  V3 hx = hand_pos(S, i);
#pragma unroll
  for (int k = 0; k < 9; k++) GF(S.epf, EPF_TINIT + k) = GF(S.kin, KIN_HAND_MAT + k);
  GF(S.epf, EPF_TINIT + 9) = hx.x; GF(S.epf, EPF_TINIT + 10) = hx.y; GF(S.epf, EPF_TINIT + 11) = hx.z;
  GF(S.epi, EPI_STEP) = 0;
  GF(S.epi, EPI_FLAGS) = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) GF(S.epf, EPF_HWM + k) = 0.f;
  GF(S.epf, EPF_EP_RETURN) = 0.f;
  int ob, bn;
  if (task_override >= 0) { ob = task_override >> 4; bn = task_override & 15; }
  else if (S.fixed_obj >= 0) { ob = S.fixed_obj; bn = S.fixed_bin; }
  else {
    const int idx = pcg_integers(S, i, r, S.ntask);
    ob = S.task_obj[idx]; bn = S.task_bin[idx];
  }
  store_rng(S, i, r);
  GF(S.epi, EPI_OBJ) = ob;
  GF(S.epi, EPI_BIN) = bn;
  // constant target keypoints (overhead camera, world-fixed)
  V3 cx;
  M3 cR, hR;
#pragma unroll
  for (int k = 0; k < 9; k++) hR.m[k] = GF(S.kin, KIN_HAND_MAT + k);
  camera_pose(MMX_CAM_OVERHEAD, hx, hR, cx, cR);
  float kp[2];
  project(obj_pos(S, i, ob), cx, cR, MMX_cam_fovy[MMX_CAM_OVERHEAD], kp);
  GF(S.epf, EPF_TGTKP) = kp[0]; GF(S.epf, EPF_TGTKP + 1) = kp[1];
  project(bin_pos(bn), cx, cR, MMX_cam_fovy[MMX_CAM_OVERHEAD], kp);
  GF(S.epf, EPF_TGTKP + 2) = kp[0]; GF(S.epf, EPF_TGTKP + 3) = kp[1];
  // FSM expert for this episode's task (generate_dataset.py:112-117 builds it after reset)
  GF(S.epi, EPI_FSM_STATE) = 0;
  GF(S.epi, EPI_FSM_TASKIDX) = 0;
  GF(S.epi, EPI_FSM_SETTLE) = 0;
  GF(S.epi, EPI_FSM_GRIP) = 1;
  GF(S.epi, EPI_FSM_HASTGT) = 0;
  GF(S.epi, EPI_EPISODES) += 1;
  write_obs(S, i);
}

// reward (gym_env.py:352-470); returns reward, writes success / done flags
DEV float compute_reward(const MMXState& S, int i, bool robot_obstacle, int& success, int& done_staged) {
  const int ob = GF(S.epi, EPI_OBJ), bn = GF(S.epi, EPI_BIN);
  V3 o = obj_pos(S, i, ob), b = bin_pos(bn), ee = hand_pos(S, i);
  const float xy = sqrtf((o.x - b.x) * (o.x - b.x) + (o.y - b.y) * (o.y - b.y));
  const bool succ = xy < 0.05f && o.z < b.z + 0.06f;
  done_staged = 0;
  if (S.reward_type == 1) { success = succ; return succ ? 1.f : 0.f; }
  if (S.reward_type == 2) {
    const float DM = 0.5f, GZ = 0.35f, LZ = 0.42f;
    int fl = GF(S.epi, EPI_FLAGS);
    const bool closed = GF(S.ctrl, 7) == 0.f;
    if (!(fl & FLAG_GRASPED) && o.z > GZ && closed) fl |= FLAG_GRASPED;
    if (!(fl & FLAG_LIFTED) && o.z > LZ && closed) fl |= FLAG_LIFTED;
    if (!(fl & FLAG_ABOVE) && (fl & FLAG_LIFTED) && xy < 0.06f) fl |= FLAG_ABOVE;
    if (!(fl & FLAG_PLACED) && succ) fl |= FLAG_PLACED;
    float r[5];
    r[0] = (fl & FLAG_GRASPED) ? 1.f : 1.f - fminf(norm(ee - o) / DM, 1.f);
    r[1] = !(fl & FLAG_GRASPED) ? 0.f : ((fl & FLAG_LIFTED) ? 1.f : fmaxf(0.f, fminf((o.z - 0.30f) / (LZ - 0.30f), 1.f)));
    r[2] = !(fl & FLAG_LIFTED) ? 0.f : ((fl & FLAG_ABOVE) ? 1.f : 1.f - fminf(xy / DM, 1.f));
    r[3] = !(fl & FLAG_ABOVE) ? 0.f : ((fl & FLAG_PLACED) ? 1.f : 1.f - fmaxf(0.f, fminf((o.z - b.z) / 0.25f, 1.f)));
    V3 ip = V3{GF(S.epf, EPF_TINIT + 9), GF(S.epf, EPF_TINIT + 10), GF(S.epf, EPF_TINIT + 11)};
    r[4] = !(fl & FLAG_PLACED) ? 0.f : 1.f - fminf(norm(ee - ip) / DM, 1.f);
    fl |= FLAG_HWM_VALID;
    GF(S.epi, EPI_FLAGS) = fl;
    float sum = 0.f;
    bool all = true;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const float h = fmaxf(GF(S.epf, EPF_HWM + k), r[k]);
      GF(S.epf, EPF_HWM + k) = h;
      sum += h;
      all &= h >= 0.90f;
    }
    if (robot_obstacle) { success = 1; done_staged = 1; return -1.f; }
    success = all;
    return sum / 5.f;
  }
  float rew = -norm(ee - o);
  if (o.z > 0.30f) rew += 2.f - norm(o - b);
  if (succ) rew += 10.f;
  success = succ;
  return rew;
}

// =========================================================================== kernels
extern "C" __global__ void __launch_bounds__(WG) mmx_reset_kernel(MMXState S, const unsigned char* mask, const int* task_override) {
  __shared__ float sh[SH_TOTAL];
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  if (mask && !mask[i]) return;
  GF(S.epi, EPI_ERROR) = 0;
  reset_lane(S, i, sh, task_override ? task_override[i] : -1);
#pragma unroll
  for (int k = 0; k < 3; k++) S.done[(size_t)k * S.N + i] = 0;
}

// decode_action (gym_env.py:252-281) + gripper command (gym_env.py:550-553). action: [N][A] row-major.
extern "C" __global__ void __launch_bounds__(WG) mmx_step_begin_kernel(MMXState S, const float* action, int adim) {
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  const float* a = action + (size_t)i * adim;
  V3 p = V3{a[0], a[1], a[2]};
  float g;
  switch (S.action_mode) {
    case 0: g = a[3]; break;
    case 1: g = a[7]; break;
    case 2: g = a[9]; break;
    default: {
      float R[9];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = GF(S.epf, EPF_TINIT + k);
      V3 t = V3{GF(S.epf, EPF_TINIT + 9), GF(S.epf, EPF_TINIT + 10), GF(S.epf, EPF_TINIT + 11)};
      p = V3{R[0] * a[0] + R[1] * a[1] + R[2] * a[2] + t.x, R[3] * a[0] + R[4] * a[1] + R[5] * a[2] + t.y,
             R[6] * a[0] + R[7] * a[1] + R[8] * a[2] + t.z};
      g = S.action_mode == 3 ? a[7] : a[9];
    }
  }
  GF(S.target, 0) = p.x; GF(S.target, 1) = p.y; GF(S.target, 2) = p.z;
  GF(S.ctrl, 7) = g > 0.5f ? 255.f : 0.f;
}

// one substep: IK on the stale kinematics (controller.py:87-137) + one mj_step (env.py:121)
extern "C" __global__ void __launch_bounds__(WG) mmx_substep_kernel(MMXState S, int do_ik) {
  __shared__ float sh[SH_TOTAL];
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  if (do_ik) ik_compute(S, i, V3{GF(S.target, 0), GF(S.target, 1), GF(S.target, 2)});
  mj_step_lane(S, i, sh);
}

// mj_forward position stage (gym_env.py:560) + reward + flags + obs (+ optional autoreset)
extern "C" __global__ void __launch_bounds__(WG) mmx_step_end_kernel(MMXState S, int expert_autoreset) {
  __shared__ float sh[SH_TOTAL];
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  float qpos[30];
#pragma unroll
  for (int k = 0; k < 30; k++) qpos[k] = GF(S.qpos, k);
  kinematics(sh, qpos);
  write_kin_cache(S, i, sh);
  ConSink cs{nullptr, i, 0, false, false};
  if (S.reward_type == 2) collide(cs, sh, true);
  GF(S.epi, EPI_STEP) += 1;
  int success = 0, done_staged = 0;
  const float r = compute_reward(S, i, cs.robot_obstacle, success, done_staged);
  int terminated, succ_flag;
  if (S.reward_type == 2) {
    terminated = (r < 0.f) || success;
    succ_flag = success && r >= 0.f;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const float h = GF(S.epf, EPF_HWM + k) / 5.f;
      GF(S.reward_components, 1 + k) = h;
      sum += h;
    }
    GF(S.reward_components, 0) = sum;
  } else {
    terminated = success;
    succ_flag = success;
#pragma unroll
    for (int k = 0; k < 6; k++) GF(S.reward_components, k) = 0.f;
  }
  const int truncated = GF(S.epi, EPI_STEP) >= S.max_episode_steps;
  S.reward[i] = r;
  S.done[(size_t)0 * S.N + i] = terminated;
  S.done[(size_t)1 * S.N + i] = truncated;
  S.done[(size_t)2 * S.N + i] = succ_flag;
  GF(S.epf, EPF_EP_RETURN) += r;
  write_obs(S, i);
  const bool fsm_done = GF(S.epi, EPI_FSM_STATE) == 10;
  const bool err = GF(S.epi, EPI_ERROR) & (ERR_NAN);
  if (S.autoreset && (terminated || truncated || err || (expert_autoreset && fsm_done))) {
    GF(S.epi, EPI_ERROR) = 0;
    reset_lane(S, i, sh, -1);
  }
}

// FSM expert plan(n_steps) (pick_and_place.py:167-277) -> abs_pos action [N][4]
// (generate_dataset.py:142-148: action = float32([*target_pos, gripper_val]))
extern "C" __global__ void __launch_bounds__(WG) mmx_expert_kernel(MMXState S, int n, float* action) {
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  int st = GF(S.epi, EPI_FSM_STATE), ti = GF(S.epi, EPI_FSM_TASKIDX), settle = GF(S.epi, EPI_FSM_SETTLE);
  int grip = GF(S.epi, EPI_FSM_GRIP), has = GF(S.epi, EPI_FSM_HASTGT);
  V3 t = V3{GF(S.epf, EPF_FSM_TARGET), GF(S.epf, EPF_FSM_TARGET + 1), GF(S.epf, EPF_FSM_TARGET + 2)};
  V3 te = V3{GF(S.epf, EPF_FSM_TRANSIT), GF(S.epf, EPF_FSM_TRANSIT + 1), GF(S.epf, EPF_FSM_TRANSIT + 2)};
  const int ob = GF(S.epi, EPI_OBJ), bn = GF(S.epi, EPI_BIN);
  V3 o = obj_pos(S, i, ob), b = bin_pos(bn), ee = hand_pos(S, i);
  auto reached = [&](V3 p) { return norm(ee - p) < 0.02f; };
  switch (st) {
    case 0:
      if (ti >= 1) { st = 10; break; }
      grip = 1; t = V3{o.x, o.y, 0.44f}; has = 1; st = 1; break;
    case 1: if (reached(t)) { t = V3{o.x, o.y, 0.36f}; st = 2; } break;
    case 2: if (reached(t)) { grip = 0; settle = 150; st = 3; } break;
    case 3: settle -= n; if (settle <= 0) { t = V3{o.x, o.y, 0.55f}; st = 4; } break;
    case 4: if (reached(t)) { te = V3{b.x, b.y, 0.55f}; st = 5; } break;
    case 5: {
      V3 diff = te - t;
      const float dist = norm(diff), step = 0.001f * n;
      if (dist > step) t = t + diff * (step / dist);
      else t = te;
      if (dist <= 0.02f) { settle = 100; st = 6; }
      break;
    }
    case 6: settle -= n; if (settle <= 0) { t = V3{b.x, b.y, 0.45f}; st = 7; } break;
    case 7: if (reached(t)) { grip = 1; settle = 150; st = 8; } break;
    case 8: settle -= n; if (settle <= 0) { t = V3{0.f, 0.3f, 0.55f}; st = 9; } break;
    case 9: if (reached(t)) { ti += 1; st = 0; } break;
    default: break;
  }
  GF(S.epi, EPI_FSM_STATE) = st; GF(S.epi, EPI_FSM_TASKIDX) = ti; GF(S.epi, EPI_FSM_SETTLE) = settle;
  GF(S.epi, EPI_FSM_GRIP) = grip; GF(S.epi, EPI_FSM_HASTGT) = has;
  GF(S.epf, EPF_FSM_TARGET) = t.x; GF(S.epf, EPF_FSM_TARGET + 1) = t.y; GF(S.epf, EPF_FSM_TARGET + 2) = t.z;
  GF(S.epf, EPF_FSM_TRANSIT) = te.x; GF(S.epf, EPF_FSM_TRANSIT + 1) = te.y; GF(S.epf, EPF_FSM_TRANSIT + 2) = te.z;
  if (action) {
    float* a = action + (size_t)i * 4;
    // before the first plan the reference has no target; the action keeps the EE in place
    V3 tgt = has ? t : ee;
    a[0] = tgt.x; a[1] = tgt.y; a[2] = tgt.z; a[3] = grip ? 1.f : 0.f;
  }
}

// physics-only entry points used by parity harnesses: one mj_step / one position-stage refresh
extern "C" __global__ void __launch_bounds__(WG) mmx_forward_pos_kernel(MMXState S) {
  __shared__ float sh[SH_TOTAL];
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  float qpos[30];
#pragma unroll
  for (int k = 0; k < 30; k++) qpos[k] = GF(S.qpos, k);
  kinematics(sh, qpos);
  write_kin_cache(S, i, sh);
}

// =========================================================================== host launchers
static inline dim3 grid_for(int n) { return dim3((n + WG - 1) / WG); }

extern "C" hipError_t mmx_launch_reset(const MMXState* S, const unsigned char* mask, const int* task, hipStream_t st) {
  hipLaunchKernelGGL(mmx_reset_kernel, grid_for(S->N), dim3(WG), 0, st, *S, mask, task);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_step(const MMXState* S, const float* action, int adim, int expert_autoreset,
                                      hipStream_t st) {
  hipLaunchKernelGGL(mmx_step_begin_kernel, grid_for(S->N), dim3(WG), 0, st, *S, action, adim);
  for (int k = 0; k < MMX_NSUBSTEP; k++)
    hipLaunchKernelGGL(mmx_substep_kernel, grid_for(S->N), dim3(WG), 0, st, *S, 1);
  hipLaunchKernelGGL(mmx_step_end_kernel, grid_for(S->N), dim3(WG), 0, st, *S, expert_autoreset);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_expert(const MMXState* S, int n, float* action, hipStream_t st) {
  hipLaunchKernelGGL(mmx_expert_kernel, grid_for(S->N), dim3(WG), 0, st, *S, n, action);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_physics(const MMXState* S, int n, int with_ik, hipStream_t st) {
  for (int k = 0; k < n; k++) hipLaunchKernelGGL(mmx_substep_kernel, grid_for(S->N), dim3(WG), 0, st, *S, with_ik);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_forward(const MMXState* S, hipStream_t st) {
  hipLaunchKernelGGL(mmx_forward_pos_kernel, grid_for(S->N), dim3(WG), 0, st, *S);
  return hipGetLastError();
}
