// MI355X (gfx950) kernels for the batched pick-and-place simulator.
//
// Hot path replaced (reference): PickPlaceGymEnv.step (mujoco_manip/gym_env.py:536-581)
//   = decode_action -> 16 x (IKController.compute controller.py:87-137 ; mujoco.mj_step env.py:121)
//     -> mujoco.mj_forward (gym_env.py:560) -> reward (gym_env.py:352-470) -> obs (gym_env.py:283-339)
// plus reset/randomization (gym_env.py:477-534, randomization.py:11-98) and the FSM expert
// (pick_and_place.py:167-291).
//
// Execution model: ONE ENVIRONMENT PER 64-LANE WORKGROUP (one wavefront).  The env record is
// read from HBM once per env step (coalesced, env-major), the 16 substeps run entirely out of
// the workgroup's LDS (state, body poses, mass matrix, contacts, constraint rows, Newton
// Hessian), and the record + observation are written back once.  Inside a substep the wave
// splits the work by phase:
//   serial tree recursions (kinematics, RNE, composite inertia, IK, integration): lane 0;
//   CRBA entries, body-pair/geom-pair broadphase + narrowphase, constraint-row assembly,
//   Newton gradient / Hessian / Cholesky / line search: all 64 lanes, joined by wave shuffles.
// Physics follows MuJoCo's documented pipeline (the fp64 oracle in oracle/ is the checker).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>

#include <type_traits>

#define MMX_MODEL_QUAL static __constant__
#include "mmx_model_gen.h"
#include "mmx_device.h"
#include "mmx_clock.h"
#include "mmx_geom.h"
#include "mmx_state.h"

#define WG 64  // lanes of the wave that runs a phase
// lane within the wave (a workgroup is one wave: one env)
// Lane id re-materialised per use (an opaque copy of threadIdx.x): nothing lane-derived (lane masks,
// per-lane dof / row indices) is hoisted to a function's entry and kept live across it.  In the
// Newton solver, where the substep's register peak sits, that frees registers: the substep's
// callee-saved save area 592 -> 436 B per lane and most SGPR spills go, for fewer instructions
// overall (C3 +2.4 % in the A/B); applied everywhere it costs more re-materialisation than it saves
// (-0.6 %), and in the constraint / collision / integrate + IK sections as well -0.8 to -1.7 %.
DEV int lane_opaque() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t & 63;
}
#define LANE ((int)(threadIdx.x & 63))
// SYNC: wave-local LDS ordering (a phase runs on ONE wave: its lanes exchange data through LDS,
// whose operations a wave issues and completes in order, so no s_barrier / waitcnt is needed,
// only a compiler fence).  XSYNC: the workgroup barrier (s_barrier + memory fence) between env steps.
DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#define SYNC() wave_sync()
#define XSYNC() __syncthreads()

static constexpr float kDt = 0.002f;
static constexpr float kHome[7] = {1.5708f, -0.2f, 0.0f, -2.1f, 0.0f, 1.8f, 0.785f};  // controller.py:8
static constexpr int kBinBody[3] = {MMX_BODY_BIN_RED, MMX_BODY_BIN_GREEN, MMX_BODY_BIN_BLUE};

#define NSLOT 14  // arm bodies 1..11 -> slots 0..10, cubes 16..18 -> slots 11..13
#define MMX_CAND_MARGIN 0.08f  // m: the list's inflation of the sphere / plane test (A/B: 0.04 +0.2 %, 0.08 +0.8 %, 0.15 -0.6 %)
#define LD 28     // padded row stride for 27-wide rows

// ============================================================================ per-env LDS
// LDS contact record: distance, position, normal and one int (bits): the 15-bit order key (pair x 8 +
// local order, the sort key) | geom 1 << 16 | geom 2 << 22 (the bodies are the geoms' bodies)
enum { CL_DIST = 0, CL_POS = 1, CL_N = 4, CL_KEY = 7, CL_F };
static_assert(MMX_NGEOM <= 64 && MMX_NPAIR * 8 < 65536, "contact key packing");
// contact c's record in the field-major array E.con[field][contact] (a lane reading its own contact
// reads consecutive words: no LDS bank conflicts at the 8-float record size)
struct CRec {
  const float* b;
  int c;
  DEV float operator[](int k) const { return b[k * MMX_MAXCON + c]; }
};
struct CRecW {
  float* b;
  int c;
  DEV float& operator[](int k) const { return b[k * MMX_MAXCON + c]; }
};
// a contact record held in registers (the row build: lane c holds contact c)
struct CReg {
  float v[CL_F];
  DEV float operator[](int k) const { return v[k]; }
};
template <class R>
DEV int con_key(const R& c) { return __float_as_int(c[CL_KEY]); }
template <class R>
DEV int con_g1(const R& c) { return (con_key(c) >> 16) & 63; }
template <class R>
DEV int con_g2(const R& c) { return (con_key(c) >> 22) & 63; }
// Hessian staging tile row stride: 17, so the dof lanes' reads of different tile rows (tile_gather)
// fall on different banks (a 16-float stride put rows sd and sd + 2 on one bank: up to 5-way; with the
// polygon stride below, LDS bank conflicts 0.31 -> 0.12 per LDS-active cycle, +0.2 % in the A/B)
#define GST 17
struct EnvSh {
  float qpos[30], qvel[28], ctrl[8];
  float target[4];
  float bx[NSLOT][3], bR[NSLOT][9];
  float S[9][6];
  // mass matrix: the arm's 9 x 9 block (the 3 free cubes are separate trees whose 6 x 6 blocks are
  // diagonal: mass x3, principal inertia x3, centre of mass at the joint)
  float M9[9][9];
  // x: the Newton solution; between solves it holds the warm start for the next one (MuJoCo's
  // qacc_warmstart: the record's qacc_ws is loaded into it and stored from it)
  float qfrc[LD], qacc_s[LD], x[LD], p[LD];
  // constraint rows in block format: a row touches at most two dof blocks (arm = 9 dofs,
  // cube k = 6 dofs); J[i][0..n0) holds block b0's columns, J[i][n0..n0+n1) block b1's;
  // J doubles as the contact-sort scratch in collide_wave (rows are built after it).
  // Rows come in aligned groups of 4: the equality / joint-limit rows (padded to a multiple of 4),
  // then per contact its 4 BASIS rows (normal, tangent 1, tangent 2, torsion; rows the contact's
  // condim does not use are zero rows).  MuJoCo's pyramid edges J_n +/- mu_k J_k are never
  // stored: the solver forms them from the basis rows (2/3 of the storage and MFMA steps).
  // Rows past MMX_LDSEFC (a pile of contacts) live in the env's HBM overflow block `ovf` (J rows,
  // then D, then NC): lane-owned row q >= LDSEFC / 64 is always an HBM row.
  // Chunk-major (r04): chunk q (slots 4q..4q+3) of row i at J[q][i], a chunk-row stride of
  // MMX_LDSEFC + 1 chunks.  A row-per-lane read of chunk q is one ds_read_b128 at an immediate
  // offset with consecutive lanes on consecutive 16-byte bank quads (conflict-free); the Hessian
  // staging's reads of one row's slot (lane & 15) land on 16 different banks.  Row-major 64-byte
  // rows put lanes 4 apart on one bank (4-way): LDS bank conflicts 0.71 -> 0.31 cycles per
  // LDS-active cycle, +0.75 % env steps/s at unchanged VALU (A/B).
  alignas(16) float J[4][MMX_LDSEFC + 1][4];  // J[k >> 2][i][k & 3] = slot k of row i (past the width 0; 15 = aref)
  unsigned char hdr[MMX_LDSEFC];  // b0 | b1 << 4 (block 15 = none); row 0 is the equality (rows past: ovf)
  // D: the row's 1 / R while the rows are built (doubling as the row -> contact map before) and in
  // the solver's setup; then per Newton iteration the diagonal entry of the group's edge-weight
  // matrix C (C_kk; a single row's active weight).  NC: C_nk, the row's coupling to its contact's
  // normal row (0 for single and normal rows).
  alignas(16) float D[MMX_LDSEFC];
  alignas(16) float NC[MMX_LDSEFC];
  // the Newton Hessian's 16 x 16 staging tile (row stride GST); the collision scratch before the rows
  alignas(16) float G[16 * GST];
  float* ovf;  // this env's overflow block (S.efc_ovf + i * MMX_OVF_F): rows past LDSEFC, headers, list
  int ncon, nefc, flags;
  int nsingle;  // rows [0, nsingle): equality + limit rows (+ zero padding); contact groups after
  int nefc_mj;  // MuJoCo's row count (pyramid edges + equality + limits), for the statistics
  int ncls[3];    // collision candidates per narrowphase class (plane, box-box, GJK)
  int tbase[11];  // rows are grouped by block-pair type: type t owns rows [tbase[t], tbase[t+1])
  int act_free;  // bit a: actuator a's force is inside its forcerange (its kv enters qDeriv)
  float stats[STAT_N];  // lane 0 accumulates; loaded / stored with the env record
  // persistent broadphase list (collide_prune; its entries in the overflow block, cand_of): the pairs
  // within MMX_CAND_MARGIN of contact when it was built, in pair order; valid while the bodies'
  // accumulated displacement bound stays under half the margin.  ncand < 0: no valid list (every
  // record load invalidates it).
  float cdisp;     // bound on any geom's displacement since the build (x 2: a pair's relative one)
  float crad;      // max over moving geoms of |geom centre - body origin| + bounding radius
  float cva, cwa;  // this substep's max arm-body origin speed and angular speed (from the RNE)
  int ncand;
};
// The workgroup's env lives in one file-scope LDS object: the non-inlined substep function below
// reaches it by symbol (LDS address space), not through a generic pointer.
static __shared__ EnvSh g_E;
// twelve workgroups (envs) per CU share its 160 KiB of LDS, allocated in 1,280-byte blocks (measured:
// tools/calib/lds_occ.hip, profiles/r05_lds_residency.json): the occupancy the kernel is tuned for (r06;
// r05: eleven; with 192 LDS rows, MMX_LDSEFC=192, four, each with a helper wave).  Twelve waves are three per SIMD, the
// 168-VGPR budget of amdgpu_waves_per_eu(3).
static_assert(MMX_LDSEFC != 128 || (sizeof(EnvSh) + 1279) / 1280 * 1280 * 12 <= 160 * 1024,
              "EnvSh no longer fits 12 envs per CU");
static_assert((sizeof(EnvSh) + 1279) / 1280 * 1280 * 8 <= 160 * 1024, "EnvSh no longer fits 8 envs per CU");

// The scratch region: E.J, E.hdr, E.D, E.NC and E.G (contiguous in EnvSh) hold the phases' scratch
// outside the constraint build + Newton solve (rows are rebuilt every substep): the collision layout
// below (geom records, candidates, the contacts, the narrowphase work space), the position stage's chain
// scan, the IK system, the RNE / composite-inertia / actuator scratch of the dynamics (at COL_WORK) and
// the observation of the step end.  The contacts live here from the narrowphase to the row build, whose
// lanes take them into registers (lane c: contact c) before the first row is written; the Newton
// Hessian staging tile is E.G.
// r06: the contacts out of their own LDS array (into this region, then registers), the rows' mu passed
// to the solver in registers, the overflow rows' headers and the broadphase list in the HBM overflow
// block: 12,640 B of LDS, twelve envs per CU (r05: 14,080 B with its own contact array, eleven; r04:
// 20,432 B with 192 rows, eight); rows past 128 go to the HBM overflow block.
#define GXS 17        // geom record: world pose (x 3, R 9), rbound, type, box half extents (3)
#define GX_RB 12
#define GX_TYPE 13
#define GX_HALF 14
#define COL_GX 0      // [NGEOM][GXS]
#define COL_CAND ((MMX_NGEOM * GXS + 15) & ~15)  // [COL_LIST] candidate pairs after the sphere test, then by class
#ifndef MMX_COL_LIST
#define MMX_COL_LIST 320  // more survivors of the sphere test than this: the rest are dropped, SHF_CON_OVF
#endif
#define COL_LIST MMX_COL_LIST
#define COL_CON (COL_CAND + COL_LIST)   // the contacts, field-major [CL_F][MMX_MAXCON] (crec)
#define COL_WORK (COL_CON + CL_F * MMX_MAXCON)  // narrowphase work space: box-box polygons, the EPA polytope
#define COL_POLY 49                     // (GJK pass), then the contact sort (49: the quads' polygons
                                        // start on different banks; 48 put quads 2 apart on one)
#define COL_PLANES 16                   // box-box lane quads per pass: one polygon each
#define COL_EPA COL_WORK
static_assert(offsetof(EnvSh, hdr) == offsetof(EnvSh, J) + sizeof(EnvSh::J) &&
                  offsetof(EnvSh, D) == offsetof(EnvSh, hdr) + sizeof(EnvSh::hdr) &&
                  offsetof(EnvSh, NC) == offsetof(EnvSh, D) + sizeof(EnvSh::D) &&
                  offsetof(EnvSh, G) == offsetof(EnvSh, NC) + sizeof(EnvSh::NC),
              "the scratch region must be contiguous");
#define SCR_FLOATS ((int)((offsetof(EnvSh, G) + sizeof(EnvSh::G) - offsetof(EnvSh, J)) / 4))
static_assert(COL_EPA + EPA_SCRATCH_FLOATS <= SCR_FLOATS, "EPA scratch exceeds the scratch region");
static_assert(COL_WORK + MMX_MAXCON * CL_F <= SCR_FLOATS, "contact sort exceeds the scratch region");
static_assert(COL_CON % 4 == 0 && COL_WORK % 4 == 0, "16-byte aligned collision scratch blocks");
static_assert(COL_WORK + COL_PLANES * COL_POLY <= SCR_FLOATS, "box-box polygons exceed the scratch region");
static_assert(MMX_CAND_CAP <= COL_LIST && MMX_NPAIR < 4096, "collision scratch layout");

// The 192-row build (one env per CU quarter, C2's batches) gives each env a second wave, the
// "helper": per substep it runs the IK beside the env wave's kinematics, then the dynamics (RNE, CRBA,
// smooth forces) beside the broadphase, then the GJK / EPA pairs beside the plane and box-box pairs
// (mj_step_wave).  Its scratch (IK system, dynamics, EPA polytope, one after the other) sits past
// everything the env wave's collision uses (the 192-row scratch region has the room); the 128-row build
// runs the phases in turn on one wave and keeps them in the narrowphase work space.
#ifndef MMX_STEP_HELPER
#define MMX_STEP_HELPER (MMX_LDSEFC == 192)
#endif
#if MMX_STEP_HELPER
#define COL_END (COL_WORK + EPA_SCRATCH_FLOATS)  // the collision's scratch ends here (asserted below)
static_assert(COL_WORK + COL_PLANES * COL_POLY <= COL_END && COL_WORK + MMX_MAXCON * CL_F <= COL_END,
              "the narrowphase work space exceeds COL_END");
#define SCR_DYN ((COL_END + 3) & ~3)
#define SCR_IKW SCR_DYN  // the IK system [72] (before the dynamics, on the helper)
#define SCR_EPA SCR_DYN  // the helper's EPA polytope (after the dynamics)
#else
#define SCR_DYN COL_WORK
#define SCR_IKW 0
#define SCR_EPA COL_EPA
#endif
// SCR_DYN: RNE frc + inertia [12][16], subtree force [12][6] (264), then:
#define SCR_IC (SCR_DYN + 272)     // composite inertias [12][10]
#define SCR_AF (SCR_IC + 120)      // actuator forces [8]
#define SCR_BIAS (SCR_AF + 8)      // RNE bias force of the arm dofs [9]
#define SCR_OBS COL_WORK           // observation (step end after its contact scan, reset, forward)
#define SCR_ACT (COL_WORK + 96)    // raw action of the step (lane 0, before the substeps)
static_assert(SCR_BIAS + 9 <= SCR_FLOATS && SCR_OBS + MMX_NOBS <= SCR_ACT && SCR_ACT + 12 <= SCR_FLOATS &&
                  SCR_EPA + EPA_SCRATCH_FLOATS <= SCR_FLOATS && SCR_IKW + 72 <= SCR_FLOATS,
              "scratch layout");
DEV float* scr_of(EnvSh& E) { return reinterpret_cast<float*>(&E.J); }
DEV const float* scr_of(const EnvSh& E) { return reinterpret_cast<const float*>(&E.J); }
DEV float* obs_of(EnvSh& E) { return scr_of(E) + SCR_OBS; }
DEV const float* obs_of(const EnvSh& E) { return scr_of(E) + SCR_OBS; }
// the contacts (from the narrowphase to the row build, which takes them into registers)
DEV float* con_of(EnvSh& E) { return scr_of(E) + COL_CON; }
DEV CRec crec(const EnvSh& E, int c) { return CRec{scr_of(E) + COL_CON, c}; }
DEV float* lrow_of(EnvSh& E) { return E.G; }  // the Hessian staging tile
// the general (cube-cube coupled) Cholesky's 27 x 27 transpose: rare, so in the env's HBM overflow
// block after the overflow rows, not in LDS
DEV float* arrow_of(EnvSh& E) { return E.ovf + MMX_OVF_ARROW_AT(MMX_LDSEFC); }
// the persistent broadphase list (16-bit pair indices) in the overflow block
DEV unsigned short* cand_of(const EnvSh& E) { return reinterpret_cast<unsigned short*>(E.ovf + MMX_OVF_CAND_AT(MMX_LDSEFC)); }
// Constraint row i: J in E.J[.][i] (chunk-major) and D in E.D[i] for i < MMX_LDSEFC, else in the env's HBM
// overflow block (J rows [OVFEFC][16], then D [OVFEFC]).  For a lane-owned row i = LANE + 64 q the
// test folds at compile time (LANE's known bits), so the unrolled loops carry no branch.
static_assert(MMX_LDSEFC % WG == 0 && MMX_LDSEFC <= MMX_MAXEFC, "LDS rows: whole lane slices");
DEV float* ovf_j(const EnvSh& E, int i) { return E.ovf + 16 * (i - MMX_LDSEFC); }
DEV float* ovf_d(const EnvSh& E, int i) { return E.ovf + 16 * MMX_OVFEFC + (i - MMX_LDSEFC); }
DEV float* ovf_nc(const EnvSh& E, int i) { return E.ovf + 17 * MMX_OVFEFC + (i - MMX_LDSEFC); }
DEV float& jlds(EnvSh& E, int i, int k) { return E.J[k >> 2][i][k & 3]; }
DEV const float& jlds(const EnvSh& E, int i, int k) { return E.J[k >> 2][i][k & 3]; }
DEV float4 jrow4(const EnvSh& E, int i, int q) {
  if (i >= MMX_LDSEFC) return reinterpret_cast<const float4*>(ovf_j(E, i))[q];
  return *reinterpret_cast<const float4*>(E.J[q][i]);
}
DEV float jget(const EnvSh& E, int i, int k) { return i < MMX_LDSEFC ? jlds(E, i, k) : ovf_j(E, i)[k]; }
DEV void jset(EnvSh& E, int i, int k, float v) {
  if (i < MMX_LDSEFC) jlds(E, i, k) = v;
  else ovf_j(E, i)[k] = v;
}
DEV float dget(const EnvSh& E, int i) { return i < MMX_LDSEFC ? E.D[i] : *ovf_d(E, i); }
DEV void dset(EnvSh& E, int i, float v) {
  if (i < MMX_LDSEFC) E.D[i] = v;
  else *ovf_d(E, i) = v;
}
DEV float ncget(const EnvSh& E, int i) { return i < MMX_LDSEFC ? E.NC[i] : *ovf_nc(E, i); }
// row headers: LDS for the LDS rows, the overflow block's byte array for the rest
DEV unsigned char* ovf_hdr(const EnvSh& E) { return reinterpret_cast<unsigned char*>(E.ovf + MMX_OVF_HDR_AT(MMX_LDSEFC)); }
DEV int hdr_get(const EnvSh& E, int i) { return i < MMX_LDSEFC ? E.hdr[i] : ovf_hdr(E)[i - MMX_LDSEFC]; }
DEV void hdr_set(EnvSh& E, int i, int h) {
  if (i < MMX_LDSEFC) E.hdr[i] = (unsigned char)h;
  else ovf_hdr(E)[i - MMX_LDSEFC] = (unsigned char)h;
}
DEV void ncset(EnvSh& E, int i, float v) {
  if (i < MMX_LDSEFC) E.NC[i] = v;
  else *ovf_nc(E, i) = v;
}
// rows written by one lane and read by another: HBM rows need the wave's stores complete first
// (workgroup scope = s_waitcnt vmcnt(0); the CU's L1 is shared by the wave).  Uniform branch.
DEV void ovf_fence(int nefc) {
  if (nefc > MMX_LDSEFC) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}
// the last substep's contacts (diagnostic copy, mmx_buffers.contacts), stored before the row build
// overwrites the scratch region that holds them
DEV void store_contacts(float* dst, const EnvSh& E) {
  const int n = E.ncon;
  for (int c = LANE; c < MMX_MAXCON; c += WG) {  // the 13-field record (CON_*) of LDS contact c
    float* o = dst + (size_t)c * CON_F;
    const CRec l = crec(E, c);
    const int g1 = c < n ? con_g1(l) : 0, g2 = c < n ? con_g2(l) : 0;
    o[CON_DIST] = c < n ? l[CL_DIST] : 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      o[CON_POS + k] = c < n ? l[CL_POS + k] : 0.f;
      o[CON_N + k] = c < n ? l[CL_N + k] : 0.f;
      o[CON_MU0 + k] = c < n ? fmaxf(MMX_geom_friction[3 * g1 + k], MMX_geom_friction[3 * g2 + k]) : 0.f;
    }
    o[CON_DIM] = c < n ? (float)max(MMX_geom_condim[g1], MMX_geom_condim[g2]) : 0.f;
    o[CON_G1] = c < n ? (float)g1 : 0.f;
    o[CON_G2] = c < n ? (float)g2 : 0.f;
  }
}
DEV float* contacts_dst(const MMXState& S, int i) { return S.con + (size_t)i * MMX_MAXCON * CON_F; }
enum { SHF_ROBOT_OBST = 1, SHF_CON_OVF = 2, SHF_EFC_OVF = 4, SHF_NAN = 8 };

DEV int body_slot(int b) { return b <= 11 ? b - 1 : b - 5; }
// The IK's kinematics cache (KIN_*: hand pose, arm joint axes and anchors, cube positions of the
// last position stage, the HBM record's kin[]) is not a separate LDS array: its entries ARE the
// position stage's outputs (hand slot of bx / bR, angular part of S, joint and cube bodies' bx), which stay
// untouched from one position stage to the next IK.  load_env scatters the record into them,
// store_env gathers it back.
DEV float& kin_ref(EnvSh& E, int k) {
  if (k < KIN_HAND_MAT) return E.bx[body_slot(MMX_BODY_HAND)][k - KIN_HAND_POS];
  if (k < KIN_AXIS) return E.bR[body_slot(MMX_BODY_HAND)][k - KIN_HAND_MAT];
  if (k < KIN_ANCHOR) return E.S[(k - KIN_AXIS) / 3][(k - KIN_AXIS) % 3];
  if (k < KIN_OBJ) return E.bx[body_slot(MMX_jnt_body[(k - KIN_ANCHOR) / 3])][(k - KIN_ANCHOR) % 3];
  return E.bx[11 + (k - KIN_OBJ) / 3][(k - KIN_OBJ) % 3];
}
DEV float kin_get(const EnvSh& E, int k) { return kin_ref(const_cast<EnvSh&>(E), k); }
DEV int body_block(int b) { return (b >= 2 && b <= 11) ? 0 : (b >= 16 ? b - 15 : -1); }
#define BLK_NONE 15
DEV int blk_size(int b) { return b == 0 ? 9 : (b == BLK_NONE ? 0 : 6); }
DEV int blk_d0(int b) { return b == 0 ? 0 : 9 + 6 * (b - 1); }
DEV int dof_blk(int a) { return a < 9 ? 0 : 1 + (a - 9) / 6; }
// slot of dof a in a row with header h, or -1 if the row does not touch a
DEV int row_slot(int h, int a) {
  const int b0 = h & 15, b1 = (h >> 4) & 15, ba = dof_blk(a);
  if (ba == b0) return a - blk_d0(b0);
  if (ba == b1) return blk_size(b0) + a - blk_d0(b1);
  return -1;
}
// block-pair row types: (0,-) (0,1) (0,2) (0,3) (1,-) (1,2) (1,3) (2,-) (2,3) (3,-)
#define NTYPE 10
static constexpr int kTB0[NTYPE] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
static constexpr int kTB1[NTYPE] = {15, 1, 2, 3, 15, 2, 3, 15, 3, 15};
DEV int row_type(int b0, int b1) {
  return b0 == 0 ? (b1 == BLK_NONE ? 0 : b1) : (b0 == 1 ? (b1 == BLK_NONE ? 4 : 3 + b1) : (b0 == 2 ? (b1 == BLK_NONE ? 7 : 8) : 9));
}
DEV bool arm_anc(int d, int b) { return d <= 6 ? (b >= d + 2 && b <= 11) : (d == 7 ? b == 10 : b == 11); }
// the arm dofs on body b's root path as a 9-bit mask (bit d = arm_anc(d, b)): the chain dofs
// 0..min(b - 2, 6), plus finger dof 7 / 8 for the finger bodies 10 / 11
DEV unsigned anc_mask(int b) {
  return b >= 2 && b <= 11 ? ((1u << min(b - 1, 7)) - 1u) | (b == 10 ? 0x80u : 0u) | (b == 11 ? 0x100u : 0u) : 0u;
}
DEV V3 body_x(const EnvSh& E, int b) {
  if (MMX_body_static[b]) return V3{0.f, 0.f, 0.f};
  const int s = body_slot(b);
  return V3{E.bx[s][0], E.bx[s][1], E.bx[s][2]};
}
DEV M3 body_R(const EnvSh& E, int b) {
  M3 R;
  const int s = body_slot(b);
#pragma unroll
  for (int k = 0; k < 9; k++) R.m[k] = E.bR[s][k];
  return R;
}
DEV SV load_S(const EnvSh& E, int d) { return SV{V3{E.S[d][0], E.S[d][1], E.S[d][2]}, V3{E.S[d][3], E.S[d][4], E.S[d][5]}}; }

// ---------------------------------------------------------------- wave primitives
// wave64 sum: DPP butterflies inside each row of 16 lanes, then the four row sums in a fixed
// order (bit-identical in every lane, no LDS traffic)
// (update_dpp with old = 0 and bound_ctrl: every control used here reads a valid lane, so the value
// is the same as mov_dpp's, but LLVM's DPP combiner only folds this form into the consuming VOP2
// op: v_add_f32_dpp instead of v_mov_b32_dpp + v_add_f32)
template <int CTRL>
DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
DEV float wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}
DEV float readlane_max0(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)); }
DEV float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return fmaxf(fmaxf(readlane_max0(v), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
}
// wave64 inclusive prefix sum: DPP row_shr butterflies inside each row of 16 lanes, then the
// row totals (v_readlane) are added to the rows above
DEV int wave_scan_incl(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = LANE >> 4;
  return v + (row == 0 ? 0 : (row == 1 ? r0 : (row == 2 ? r0 + r1 : r0 + r1 + r2)));
}
// triangular index e -> (a, b) with a >= b, e = a(a+1)/2 + b
DEV void tri_index(int e, int& a, int& b) {
  int aa = (int)((sqrtf(8.f * (float)e + 1.f) - 1.f) * 0.5f);
  while ((aa + 1) * (aa + 2) / 2 <= e) aa++;
  while (aa * (aa + 1) / 2 > e) aa--;
  a = aa;
  b = e - aa * (aa + 1) / 2;
}

// ============================================================================ kinematics (lane 0)
// mj_kinematics + arm motion subspaces (world-origin Plucker).  All joint anchors of this model
// sit at the body origin (jnt_pos = 0).  Also refreshes the IK's kinematics cache.
DEV void kinematics_lane0(EnvSh& E) {
  V3 px[12];
  Q4 pq[12];
  px[0] = V3{0.f, 0.f, 0.f};
  pq[0] = Q4{1.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 1; b <= 11; b++) {
    const int p = MMX_body_parent[b];
    const M3 Rp = qmat(pq[p]);
    V3 pos = px[p] + mul(Rp, V3{MMX_body_pos[3 * b], MMX_body_pos[3 * b + 1], MMX_body_pos[3 * b + 2]});
    Q4 q = qmul(pq[p], Q4{MMX_body_quat[4 * b], MMX_body_quat[4 * b + 1], MMX_body_quat[4 * b + 2], MMX_body_quat[4 * b + 3]});
    const int j = MMX_body_jnt[b];
    if (j >= 0) {
      const V3 axl = V3{MMX_jnt_axis[3 * j], MMX_jnt_axis[3 * j + 1], MMX_jnt_axis[3 * j + 2]};
      const V3 axw = mul(qmat(qnormalize(q)), axl);
      const float qv = E.qpos[j];
      if (MMX_jnt_type[j] == 3) {  // hinge
        q = qmul(q, qaxisangle(axl, qv));
        const V3 lin = cross(pos, axw);
        E.S[j][0] = axw.x; E.S[j][1] = axw.y; E.S[j][2] = axw.z;
        E.S[j][3] = lin.x; E.S[j][4] = lin.y; E.S[j][5] = lin.z;
      } else {  // slide
        E.S[j][0] = 0.f; E.S[j][1] = 0.f; E.S[j][2] = 0.f;
        E.S[j][3] = axw.x; E.S[j][4] = axw.y; E.S[j][5] = axw.z;
        pos = pos + axw * qv;
      }
    }
    q = qnormalize(q);
    px[b] = pos;
    pq[b] = q;
    const M3 R = qmat(q);
    const int s = b - 1;
    E.bx[s][0] = pos.x; E.bx[s][1] = pos.y; E.bx[s][2] = pos.z;
#pragma unroll
    for (int k = 0; k < 9; k++) E.bR[s][k] = R.m[k];
  }
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int qa = 9 + 7 * c;
    const M3 R = qmat(qnormalize(Q4{E.qpos[qa + 3], E.qpos[qa + 4], E.qpos[qa + 5], E.qpos[qa + 6]}));
    const int s = 11 + c;
    E.bx[s][0] = E.qpos[qa]; E.bx[s][1] = E.qpos[qa + 1]; E.bx[s][2] = E.qpos[qa + 2];
#pragma unroll
    for (int k = 0; k < 9; k++) E.bR[s][k] = R.m[k];
  }
}

// Wave form of kinematics_lane0: one lane per body.  Each arm body first builds its local
// transform (static offset x joint), then the chain is composed by pointer jumping (4 rounds
// cover the 10-deep finger chain): T_b <- T_anc(b) o T_b, anc(b) <- anc(anc(b)).  Cubes read their
// free joints directly.  Results equal kinematics_lane0 up to fp32 association order.
DEV void kinematics_wave(EnvSh& E) {
  float* T = scr_of(E);  // [12][8] scan scratch: q (4), p (3), ancestor
  const int b = LANE + 1;    // lanes 0..10 -> arm bodies 1..11
  Q4 q = Q4{1.f, 0.f, 0.f, 0.f};
  V3 p = V3{0.f, 0.f, 0.f};
  int anc = 0;
  if (LANE < 11) {
    p = V3{MMX_body_pos[3 * b], MMX_body_pos[3 * b + 1], MMX_body_pos[3 * b + 2]};
    q = Q4{MMX_body_quat[4 * b], MMX_body_quat[4 * b + 1], MMX_body_quat[4 * b + 2], MMX_body_quat[4 * b + 3]};
    const int j = MMX_body_jnt[b];
    if (j >= 0) {
      const V3 axl = V3{MMX_jnt_axis[3 * j], MMX_jnt_axis[3 * j + 1], MMX_jnt_axis[3 * j + 2]};
      const float qv = E.qpos[j];
      if (MMX_jnt_type[j] == 3) q = qmul(q, qaxisangle(axl, qv));  // hinge
      else p = p + mul(qmat(qnormalize(q)), axl) * qv;             // slide along the joint axis
    }
    anc = MMX_body_parent[b];
  }
#pragma unroll
  for (int round = 0; round < 4; round++) {
    if (LANE < 11) {
      float* t = T + 8 * b;
      t[0] = q.w; t[1] = q.x; t[2] = q.y; t[3] = q.z;
      t[4] = p.x; t[5] = p.y; t[6] = p.z;
      t[7] = __int_as_float(anc);
    }
    SYNC();
    if (LANE < 11 && anc != 0) {
      const float* t = T + 8 * anc;
      const Q4 qa = Q4{t[0], t[1], t[2], t[3]};
      const V3 pa = V3{t[4], t[5], t[6]};
      const int aa = __float_as_int(t[7]);
      p = pa + mul(qmat(qa), p);
      q = qnormalize(qmul(qa, q));
      anc = aa;
    }
    SYNC();
  }
  if (LANE < 11) {
    q = qnormalize(q);
    const M3 R = qmat(q);
    const int s = b - 1;
    E.bx[s][0] = p.x; E.bx[s][1] = p.y; E.bx[s][2] = p.z;
#pragma unroll
    for (int k = 0; k < 9; k++) E.bR[s][k] = R.m[k];
    const int j = MMX_body_jnt[b];
    if (j >= 0) {
      const V3 axw = mul(R, V3{MMX_jnt_axis[3 * j], MMX_jnt_axis[3 * j + 1], MMX_jnt_axis[3 * j + 2]});
      if (MMX_jnt_type[j] == 3) {
        const V3 lin = cross(p, axw);
        E.S[j][0] = axw.x; E.S[j][1] = axw.y; E.S[j][2] = axw.z;
        E.S[j][3] = lin.x; E.S[j][4] = lin.y; E.S[j][5] = lin.z;
      } else {
        E.S[j][0] = 0.f; E.S[j][1] = 0.f; E.S[j][2] = 0.f;
        E.S[j][3] = axw.x; E.S[j][4] = axw.y; E.S[j][5] = axw.z;
      }
    }
  } else if (LANE < 14) {  // cubes: free joints
    const int c = LANE - 11, qa = 9 + 7 * c;
    const M3 R = qmat(qnormalize(Q4{E.qpos[qa + 3], E.qpos[qa + 4], E.qpos[qa + 5], E.qpos[qa + 6]}));
    const int s = 11 + c;
    E.bx[s][0] = E.qpos[qa]; E.bx[s][1] = E.qpos[qa + 1]; E.bx[s][2] = E.qpos[qa + 2];
#pragma unroll
    for (int k = 0; k < 9; k++) E.bR[s][k] = R.m[k];
  }
  SYNC();
}

// ============================================================================ dynamics
DEV RI body_inertia(const EnvSh& E, int b) {
  const V3 x = body_x(E, b);
  const M3 R = body_R(E, b);
  const float m = MMX_body_mass[b];
  const V3 c = x + mul(R, V3{MMX_body_ipos[3 * b], MMX_body_ipos[3 * b + 1], MMX_body_ipos[3 * b + 2]});
  M3 Ib;
#pragma unroll
  for (int k = 0; k < 9; k++) Ib.m[k] = MMX_body_inertia[9 * b + k];
  const M3 T = mul(R, Ib);
  float Ic[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int cc = 0; cc < 3; cc++) Ic[3 * r + cc] = T.m[3 * r] * R.m[3 * cc] + T.m[3 * r + 1] * R.m[3 * cc + 1] + T.m[3 * r + 2] * R.m[3 * cc + 2];
  RI I;
  I.m = m;
  I.h = c * m;
  const float cc2 = dot(c, c);
  I.J[0] = Ic[0] + m * (cc2 - c.x * c.x);
  I.J[1] = Ic[4] + m * (cc2 - c.y * c.y);
  I.J[2] = Ic[8] + m * (cc2 - c.z * c.z);
  I.J[3] = Ic[1] - m * c.x * c.y;
  I.J[4] = Ic[2] - m * c.x * c.z;
  I.J[5] = Ic[5] - m * c.y * c.z;
  return I;
}
DEV void ri_store(float* d, const RI& I) {
  d[0] = I.m; d[1] = I.h.x; d[2] = I.h.y; d[3] = I.h.z;
#pragma unroll
  for (int k = 0; k < 6; k++) d[4 + k] = I.J[k];
}
DEV RI ri_load(const float* d) {
  RI I;
  I.m = d[0];
  I.h = V3{d[1], d[2], d[3]};
#pragma unroll
  for (int k = 0; k < 6; k++) I.J[k] = d[4 + k];
  return I;
}

#define LT(r, c) ((r) * ((r) + 1) / 2 + (c))

// RNE bias of the arm + composite inertias (for CRBA), one lane per moving arm body (2..11).  A
// body's velocity and acceleration are running sums over the joints on its root path (arm_anc),
// its force is local.  Lane l < 10 holds body b = 11 - l (the fingers 11, 10, then the chain 9..2),
// so a body's subtree (bodies >= b for b <= 9, itself for a finger) is an inclusive prefix over
// lanes 0..l: the backward pass and the composite inertias are 16 DPP row_shr scans in registers.
// Scratch at SCR_DYN: subtree force (6) per body at 16 * 12, composite inertias at SCR_IC.
DEV float shr_add_scan(float v) {  // inclusive prefix sum over the lanes of each 16-lane row
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));  // row_shr:1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false));  // row_shr:2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false));  // row_shr:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, false));  // row_shr:8
  return v;
}
DEV void rne_wave(EnvSh& E) {
  float* F = scr_of(E) + SCR_DYN;
  const int b = 11 - LANE;
  float fi[16];  // the body's force (6), then its inertia (m, h, J: 10)
#pragma unroll
  for (int m = 0; m < 16; m++) fi[m] = 0.f;
  float vmax = 0.f, wmax = 0.f;  // for collide_prune's displacement bound
  if (LANE < 10) {
    const RI Ib = body_inertia(E, b);
    SV vel = SV{V3{0.f, 0.f, 0.f}, V3{0.f, 0.f, 0.f}};
    SV acc = SV{V3{0.f, 0.f, 0.f}, V3{0.f, 0.f, -MMX_GRAVITY_Z}};  // base acceleration = -gravity
#pragma unroll
    for (int d = 0; d < 9; d++) {
      if (arm_anc(d, b)) {
        const SV vj = load_S(E, d) * E.qvel[d];
        acc = acc + cross_motion(vel, vj);
        vel = vel + vj;
      }
    }
    const SV f = rimul(Ib, acc) + cross_force(vel, rimul(Ib, vel));
    vmax = norm(vel.v + cross(vel.w, body_x(E, b)));  // speed of the body origin
    wmax = norm(vel.w);
    fi[0] = f.w.x; fi[1] = f.w.y; fi[2] = f.w.z; fi[3] = f.v.x; fi[4] = f.v.y; fi[5] = f.v.z;
    ri_store(fi + 6, Ib);
  }
#pragma unroll
  for (int m = 0; m < 16; m++) {  // subtree sums (lanes >= 10 hold zeros and come after)
    const float sm = shr_add_scan(fi[m]);
    fi[m] = LANE == 1 ? fi[m] : sm;  // finger 10: its own subtree only (finger 11 sits before it)
  }
  if (LANE < 10) {
#pragma unroll
    for (int m = 0; m < 10; m++) (scr_of(E) + SCR_IC)[10 * b + m] = fi[6 + m];
    float* o = F + 16 * 12 + 6 * b;
#pragma unroll
    for (int m = 0; m < 6; m++) o[m] = fi[m];
  }
  SYNC();
  if (LANE < 9) {
    const float* o = F + 16 * 12 + 6 * MMX_jnt_body[LANE];
    (scr_of(E) + SCR_BIAS)[LANE] = sdot(load_S(E, LANE), SV{V3{o[0], o[1], o[2]}, V3{o[3], o[4], o[5]}});
  }
  vmax = wave_max(vmax);
  wmax = wave_max(wmax);
  if (LANE == 0) {
    E.cva = vmax;
    E.cwa = wmax;
  }
  SYNC();
}

// DPP row_newbcast:K, the value of lane K of each 16-lane row in every lane of that row
template <int K>
DEV float row_bcast_t(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + K, 0xF, 0xF, true));
}
// k is a constant of a fully unrolled loop at every call: the switch folds to one DPP move
DEV float row_bcast(float v, int k) {
  switch (k) {
    case 0: return row_bcast_t<0>(v);
    case 1: return row_bcast_t<1>(v);
    case 2: return row_bcast_t<2>(v);
    case 3: return row_bcast_t<3>(v);
    case 4: return row_bcast_t<4>(v);
    case 5: return row_bcast_t<5>(v);
    case 6: return row_bcast_t<6>(v);
    case 7: return row_bcast_t<7>(v);
    default: return row_bcast_t<8>(v);
  }
}
// broadcast of lane k's value (k < 16) to the lanes of DPP row 0 that hold the small system: one
// row_newbcast (a VGPR result, no SGPR round trip and its hazard nops; v_readlane measured slower)
DEV float small_bcast(float v, int k) { return row_bcast(v, k); }

// (A^{-1} v)_j in lane j for a small SPD A given by rows (lane j holds row j in arow[0..N), N <= 9:
// the rows sit in DPP row 0; lanes of rows 1..3 compute values nobody reads).  Right-looking
// Cholesky with lane broadcasts; lane k keeps column k of L (selects) for the transposed solve.
// eps: pivot floor.  The arithmetic is the same in either broadcast form (bit-identical results).
template <int N>
DEV float chol_solve_small(const float* arow, float v, float eps) {
  static_assert(N <= 9, "row_bcast covers lanes 0..8");
  const int j = LANE & 15;
  float h[N], c[N], dinv[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    h[i] = arow[i];
    c[i] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float d = fmaxf(small_bcast(h[k], k), eps);
    const float inv = __builtin_amdgcn_rsqf(d), sd = d * inv;
    dinv[k] = inv;
    const float l = j == k ? sd : h[k] * inv;
    h[k] = l;
    c[k] = j == k ? sd : c[k];
#pragma unroll
    for (int i = k + 1; i < N; i++) {
      const float li = small_bcast(l, i);
      h[i] = fmaf(-li, l, h[i]);
      c[i] = j == k ? li : c[i];
    }
  }
  float y = j < N ? v : 0.f;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float yk = small_bcast(y, k) * dinv[k];
    y = j == k ? yk : (j > k ? fmaf(-h[k], yk, y) : y);
  }
#pragma unroll
  for (int k = N - 1; k >= 0; k--) {
    const float zk = small_bcast(y, k) * dinv[k];
    y = j == k ? zk : (j < k ? fmaf(-c[k], zk, y) : y);
  }
  return y;
}

// whole wave: mass matrix (CRBA entries in parallel), smooth forces, qacc_smooth
DEV void dynamics_wave(EnvSh& E) {
  float* stats = E.stats;
  CLK_DECL;
  rne_wave(E);
  PROBE(11, stats, STAT_T_AUX0);
  if (LANE < 45) {
    int d, e;
    tri_index(LANE, d, e);
    float v = 0.f;
    if (e == d || (e <= 6 && !(d == 8 && e == 7))) {  // fingers 7, 8 are siblings
      const RI Ic = ri_load(scr_of(E) + SCR_IC + 10 * MMX_jnt_body[d]);
      v = sdot(load_S(E, e), rimul(Ic, load_S(E, d)));
    }
    if (d == e) v += MMX_dof_armature[d];
    E.M9[d][e] = v;
    E.M9[e][d] = v;
  }  // (the cubes' diagonal blocks are model constants: mass_cube)
  SYNC();
  PROBE(11, stats, STAT_T_AUX1);
  // smooth force: passive damping - bias + actuation (arm; one lane per actuator, then per dof),
  // gravity + gyroscopic (cubes, one lane each); arm qacc_smooth = M_arm^{-1} qfrc by a register
  // Cholesky (rows in lanes 0..8)
  float* af = scr_of(E) + SCR_AF;  // actuator forces
  bool unclamped = false;
  if (LANE < 8) {
    const int a = LANE;
    const float c = fminf(fmaxf(E.ctrl[a], MMX_act_ctrlrange[2 * a]), MMX_act_ctrlrange[2 * a + 1]);
    const int j = MMX_act_trn_joint[a];
    const float tlen = MMX_tendon_coef[0] * E.qpos[7] + MMX_tendon_coef[1] * E.qpos[8];
    const float tvel = MMX_tendon_coef[0] * E.qvel[7] + MMX_tendon_coef[1] * E.qvel[8];
    const float len = j >= 0 ? E.qpos[j] : tlen, vel = j >= 0 ? E.qvel[j] : tvel;
    float f = MMX_act_gain[a] * c + MMX_act_bias[3 * a] + MMX_act_bias[3 * a + 1] * len + MMX_act_bias[3 * a + 2] * vel;
    unclamped = f > MMX_act_forcerange[2 * a] && f < MMX_act_forcerange[2 * a + 1];
    af[a] = fminf(fmaxf(f, MMX_act_forcerange[2 * a]), MMX_act_forcerange[2 * a + 1]);
  }
  const unsigned free_mask = (unsigned)__ballot(unclamped);
  if (LANE == 0) E.act_free = (int)free_mask;
  SYNC();
  float qf = 0.f;
  if (LANE < 9) {
    const int d = LANE;
    qf = -MMX_dof_damping[d] * E.qvel[d] - (scr_of(E) + SCR_BIAS)[d];
#pragma unroll
    for (int a = 0; a < 8; a++) {  // actuator order as the serial accumulation
      const int j = MMX_act_trn_joint[a];
      if (j >= 0) qf += j == d ? af[a] : 0.f;
      else qf += d == 7 ? MMX_tendon_coef[0] * af[a] : (d == 8 ? MMX_tendon_coef[1] * af[a] : 0.f);
    }
    E.qfrc[d] = qf;
  } else if (LANE < 12) {  // free body with com at the origin: gravity + w x (I w)
    const int c = LANE - 9, b = 16 + c, da = 9 + 6 * c;
    const float I0 = MMX_body_inertia[9 * b], I1 = MMX_body_inertia[9 * b + 4], I2 = MMX_body_inertia[9 * b + 8];
    const V3 w = V3{E.qvel[da + 3], E.qvel[da + 4], E.qvel[da + 5]};
    const V3 gyro = cross(w, V3{I0 * w.x, I1 * w.y, I2 * w.z});
    const float m = MMX_body_mass[b];
    E.qfrc[da] = 0.f; E.qfrc[da + 1] = 0.f; E.qfrc[da + 2] = MMX_GRAVITY_Z * m;
    E.qfrc[da + 3] = -gyro.x; E.qfrc[da + 4] = -gyro.y; E.qfrc[da + 5] = -gyro.z;
    E.qacc_s[da] = 0.f; E.qacc_s[da + 1] = 0.f; E.qacc_s[da + 2] = MMX_GRAVITY_Z;
    E.qacc_s[da + 3] = -gyro.x / I0; E.qacc_s[da + 4] = -gyro.y / I1; E.qacc_s[da + 5] = -gyro.z / I2;
  }
  float arow[9];
  const int jr = min(LANE, 8);
#pragma unroll
  for (int e = 0; e < 9; e++) arow[e] = E.M9[jr][e];
  PROBE(11, stats, STAT_T_AUX2);
  const float xs = chol_solve_small<9>(arow, qf, 1e-12f);
  if (LANE < 9) E.qacc_s[LANE] = xs;
  SYNC();
  PROBE(11, stats, STAT_T_AUX3);
}

// ============================================================================ collision (wave)
DEV Geom geom_pose(const EnvSh& E, int g) {
  Geom G;
  G.g = g;
  G.type = MMX_geom_type[g];
  const int b = MMX_geom_body[g];
  if (MMX_body_static[b]) {
    G.x = V3{MMX_geom_static_xpos[3 * g], MMX_geom_static_xpos[3 * g + 1], MMX_geom_static_xpos[3 * g + 2]};
#pragma unroll
    for (int k = 0; k < 9; k++) G.R.m[k] = MMX_geom_static_xmat[9 * g + k];
  } else {
    const V3 bx = body_x(E, b);
    const M3 bR = body_R(E, b);
    G.x = bx + mul(bR, V3{MMX_geom_pos[3 * g], MMX_geom_pos[3 * g + 1], MMX_geom_pos[3 * g + 2]});
    M3 Lm;
#pragma unroll
    for (int k = 0; k < 9; k++) Lm.m[k] = MMX_geom_lmat[9 * g + k];
    G.R = mul(bR, Lm);
  }
  return G;
}

// appends contacts to the env's LDS list; key = pair index * 8 + local sequence gives a
// deterministic contact order independent of lane timing
struct WaveSink {
  EnvSh* E;
  int key;
  bool store;
  bool ro;
  int geoms;  // the geoms packed above the order key: g1 << 16 | g2 << 22
  int key0;
  DEV WaveSink(EnvSh* e, int p, bool st, int g1, int g2) : E(e), key(p * 8), store(st) {
    key0 = p * 8;
    geoms = (g1 << 16) | (g2 << 22);
    const int c1 = MMX_geom_class[g1], c2 = MMX_geom_class[g2];
    ro = (c1 == 1 && c2 == 2) || (c1 == 2 && c2 == 1);
  }
  DEV void add(int g1, int g2, float dist, V3 pos, V3 nrm) { put(reserve(1), g1, g2, dist, pos, nrm); }
  // contact `order` of the pair (its key = pair * 8 + order, as the sequential put would give it)
  // into a reserved slot: the lane-group form of the box-box narrowphase puts a pair's contacts
  // from several lanes at once
  DEV void put_at(int slot, int order, int g1, int g2, float dist, V3 pos, V3 nrm) {
    key = key0 + order;
    put(slot, g1, g2, dist, pos, nrm);
  }
  // n consecutive contact slots with one LDS atomic (a pair's corners / clipped points are
  // counted first, then reserved together); returns the first slot, MMX_MAXCON when none is kept
  DEV int reserve(int n) {
    if (n <= 0) return MMX_MAXCON;
    if (ro) atomicOr(&E->flags, (int)SHF_ROBOT_OBST);
    if (!store) return MMX_MAXCON;
    const int slot = atomicAdd(&E->ncon, n);
    if (slot + n > MMX_MAXCON) atomicOr(&E->flags, (int)SHF_CON_OVF);
    return slot;
  }
  // contact into a reserved slot (slots past the list are dropped); keys follow the call order
  DEV void put(int slot, int g1, int g2, float dist, V3 pos, V3 nrm) {
    if (slot >= MMX_MAXCON) return;
    nrm = normalize(nrm);
    const CRecW c{scr_of(*E) + COL_CON, slot};
    c[CL_DIST] = dist;
    c[CL_POS] = pos.x; c[CL_POS + 1] = pos.y; c[CL_POS + 2] = pos.z;
    c[CL_N] = nrm.x; c[CL_N + 1] = nrm.y; c[CL_N + 2] = nrm.z;
    c[CL_KEY] = __int_as_float((key++) | geoms);
  }
};

DEV V3 geom_half(const float* gx, int g) {
  const float* o = gx + GXS * g;
  return V3{o[GX_HALF], o[GX_HALF + 1], o[GX_HALF + 2]};
}
DEV Geom geom_lds(const float* gx, int g) {
  const float* o = gx + GXS * g;
  Geom G;
  G.g = g;
  G.type = __float_as_int(o[GX_TYPE]);
  G.x = V3{o[0], o[1], o[2]};
#pragma unroll
  for (int k = 0; k < 9; k++) G.R.m[k] = o[3 + k];
  return G;
}
// MMX_pair_packed[p]: the geoms of pair p ordered by type (plane first), as the narrowphase dispatch
// expects (pre-sorted by the model compiler).  A candidate entry carries the pair index and both geom ids (p | g1 << 12 | g2 << 18), so the
// passes after the sphere test decode them from LDS instead of gathering MMX_pair_packed (a
// per-lane global-memory load) again.  Classes go above bit 24 (collide_prune's regrouping).
static_assert(MMX_NPAIR < 4096 && MMX_NGEOM <= 64, "candidate entry packing");
DEV int cand_pack(int p, int pk) { return p | ((pk & 255) << 12) | ((pk >> 8) << 18); }
DEV void cand_unpack(int e, int& p, int& g1, int& g2) {
  p = e & 4095;
  g1 = (e >> 12) & 63;
  g2 = (e >> 18) & 63;
}
DEV bool robot_obstacle(int g1, int g2) {
  const int c1 = MMX_geom_class[g1], c2 = MMX_geom_class[g2];
  return (c1 == 1 && c2 == 2) || (c1 == 2 && c2 == 1);
}
// stream compaction of one wave's flags into list[base...]; returns the new length
DEV int wave_compact(bool keep, int* list, int base, int val) {
  const unsigned long long m = __ballot(keep);
  const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
  if (keep) list[base + pos] = val;
  return base + __popcll(m);
}

// Collision in coherent stages: (1) world poses of all geoms into LDS, one lane per geom;
// (2) bounding-sphere / plane-distance prune of all pairs, compacted with ballots; (3) OBB prune,
// split by narrowphase class into per-class lists (E.ncls); (4) one pass per class (plane-convex
// / box lane per pair, box-box one pair per lane quad, GJK/EPA one pair per wave), so lanes of a
// pass run the same code; (5) deterministic rank sort of the contacts by pair key.  Every prune is
// conservative, so the contact set equals the all-pairs narrowphase.
DEV void collide_prune(EnvSh& E, bool only_ro) {
  float* stats = E.stats;
  CLK_DECL;
  if (LANE == 0) {
    E.ncon = 0;
    E.flags &= ~SHF_ROBOT_OBST;  // (SHF_CON_OVF is sticky from the record load to the fold: any substep's overflow counts)
  }
  float* scr = scr_of(E);
  float* gx = scr + COL_GX;
  int* cand = reinterpret_cast<int*>(scr + COL_CAND);
  // (2) runs over the persistent list when it is still valid: its pairs were within
  // MMX_CAND_MARGIN of contact at the build, and no pair has since closed by more than the bound
  // cdisp = sum over substeps of 2 dt (max body-origin speed + max angular speed x crad) (x 1.25
  // for the integrators' second-order terms).  The list is in pair order, so the exact test below
  // keeps the same candidates, in the same order, as the all-pairs pass.
  bool use_list = false;
  if (!only_ro && E.ncand >= 0) {
    float vc = 0.f;
    if (LANE < 3) {
      const int da = 9 + 6 * LANE;
      vc = norm(V3{E.qvel[da], E.qvel[da + 1], E.qvel[da + 2]}) +
           norm(V3{E.qvel[da + 3], E.qvel[da + 4], E.qvel[da + 5]}) * E.crad;
    }
    vc = fmaxf(fmaxf(readlane_max0(vc), __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vc), 1))),
               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vc), 2)));
    const float inc = 1.25f * 2.f * kDt * fmaxf(fmaf(E.cwa, E.crad, E.cva), vc) + 1e-5f;
    use_list = E.cdisp + inc < 0.5f * MMX_CAND_MARGIN;
    SYNC();
    if (LANE == 0) E.cdisp = use_list ? E.cdisp + inc : E.cdisp;
  }
  const bool rebuild = !only_ro && !use_list;
  if (LANE < MMX_NGEOM) {
    const Geom G = geom_pose(E, LANE);
    float* o = gx + GXS * LANE;
    o[0] = G.x.x; o[1] = G.x.y; o[2] = G.x.z;
#pragma unroll
    for (int k = 0; k < 9; k++) o[3 + k] = G.R.m[k];
    o[GX_RB] = MMX_geom_rbound[LANE];
    o[GX_TYPE] = __int_as_float(G.type);
    o[GX_HALF] = MMX_geom_aabb[3 * LANE];  // bounding-box half extents in the geom frame (= size for boxes)
    o[GX_HALF + 1] = MMX_geom_aabb[3 * LANE + 1];
    o[GX_HALF + 2] = MMX_geom_aabb[3 * LANE + 2];
  }
  if (rebuild) {  // uniform: the moving geoms' extent about their body origins (rigid: any pose)
    float ext = 0.f;
    if (LANE < MMX_NGEOM) {
      const int b = MMX_geom_body[LANE];
      if (!MMX_body_static[b]) ext = norm(V3{gx[GXS * LANE], gx[GXS * LANE + 1], gx[GXS * LANE + 2]} - body_x(E, b)) +
                                     MMX_geom_rbound[LANE];
    }
    ext = wave_max(ext);
    if (LANE == 0) E.crad = ext;
  }
  SYNC();
  PROBE(2, stats, STAT_T_AUX0);
  // (2) sphere / plane-distance prune
  auto sphere_test = [&](int p, int pk, float infl) {
    const int g1 = pk & 255, g2 = pk >> 8;
    if (only_ro && !robot_obstacle(g1, g2)) return false;
    const float* o1 = gx + GXS * g1;
    const float* o2 = gx + GXS * g2;
    const V3 d = V3{o2[0] - o1[0], o2[1] - o1[1], o2[2] - o1[2]};
    if (__float_as_int(o1[GX_TYPE]) == GT_PLANE) return d.x * o1[5] + d.y * o1[8] + d.z * o1[11] <= o2[GX_RB] + infl;
    const float rb = o1[GX_RB] + o2[GX_RB] + infl;
    return dot(d, d) <= rb * rb;
  };
  int nc = 0;
  if (use_list) {  // uniform: the list's pairs only (<= MMX_CAND_CAP, pair order; in the overflow block)
    const int n = E.ncand;
    constexpr int NLP = (MMX_CAND_CAP + WG - 1) / WG;
    int lp[NLP], lk[NLP];  // every pass's pair-table gather in flight at once
    const unsigned short* cl = cand_of(E);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the rebuild's stores (below)
#pragma unroll
    for (int q = 0; q < NLP; q++) {
      const int k = q * WG + LANE;
      lp[q] = k < n ? (int)cl[k] : 0;
      lk[q] = WG * q < n ? MMX_pair_packed[lp[q]] : 0;
    }
#pragma unroll
    for (int q = 0; q < NLP; q++) {
      if (WG * q >= n) break;  // uniform
      const int k = q * WG + LANE;
      const bool keep = k < n && sphere_test(lp[q], lk[q], 0.f);
      nc = wave_compact(keep, cand, nc, cand_pack(lp[q], lk[q]));
    }
  } else {
  // all pairs: unrolled so the pair-table loads issue together
  constexpr int NPASS = (MMX_NPAIR + WG - 1) / WG;
  int pg[NPASS];  // all pair-table loads in flight at once
#pragma unroll
  for (int q = 0; q < NPASS; q++) {
    const int p = min(q * WG + LANE, MMX_NPAIR - 1);
    pg[q] = MMX_pair_packed[p];
  }
  // all tests first (ballot masks in SGPRs), compaction stores after: no LDS store between the
  // passes' gathers, so the compiler may keep several passes' loads in flight
  unsigned long long km[NPASS], ki[NPASS];
#pragma unroll
  for (int q = 0; q < NPASS; q++) {
    const int p = q * WG + LANE;
    km[q] = __ballot(p < MMX_NPAIR && sphere_test(p, pg[q], 0.f));
    ki[q] = rebuild ? __ballot(p < MMX_NPAIR && sphere_test(p, pg[q], MMX_CAND_MARGIN)) : 0ull;
  }
  int ni = 0;
#pragma unroll
  for (int q = 0; q < NPASS; q++) {
    const unsigned long long m = km[q];
    if ((m >> LANE) & 1ull) {
      const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      if (nc + pos < COL_LIST) cand[nc + pos] = cand_pack(q * WG + LANE, pg[q]);
    }
    nc += __popcll(m);
    if (rebuild) {  // the inflated set -> the persistent list (pair order)
      const unsigned long long mi = ki[q];
      const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(mi >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mi, 0u));
      if (((mi >> LANE) & 1ull) && ni + pos < MMX_CAND_CAP) cand_of(E)[ni + pos] = (unsigned short)(q * WG + LANE);
      ni += __popcll(mi);
    }
  }
  if (rebuild) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the list's stores complete before its next read
    if (LANE == 0) {
      E.ncand = ni <= MMX_CAND_CAP ? ni : -1;
      E.cdisp = 0.f;
    }
  }
  if (nc > COL_LIST) {  // uniform: more sphere-test survivors than the list holds (flagged; none in C3)
    if (LANE == 0) E.flags |= SHF_CON_OVF;
    nc = COL_LIST;
  }
  }
  SYNC();
  PROBE(2, stats, STAT_T_AUX1);
  // (3) OBB prune and class (0 plane, 1 box-box, 2 GJK, 3 pruned); then the candidates are
  // regrouped in place as [plane | box-box | GJK], each group in candidate (pair) order
  constexpr int NCP = (COL_LIST + WG - 1) / WG;
  int ce[NCP];
  int ncls[3] = {0, 0, 0};
#pragma unroll
  for (int q = 0; q < NCP; q++) {
    const int k = q * WG + LANE;
    int c = 3, p = 0;
    if (q * WG < nc) {
      if (k < nc) {
        p = cand[k];
        int pp, g1, g2;
        cand_unpack(p, pp, g1, g2);
        const Geom A = geom_lds(gx, g1), B = geom_lds(gx, g2);
        if (A.type == GT_PLANE) c = 0;
        else if (obb_overlap(A, B, geom_half(gx, g1), geom_half(gx, g2))) c = (A.type == GT_BOX && B.type == GT_BOX) ? 1 : 2;
      }
#pragma unroll
      for (int t = 0; t < 3; t++) ncls[t] += __popcll(__ballot(c == t));
    }
    ce[q] = p | (c << 24);  // (p: the packed candidate entry, 24 bits)
  }
  SYNC();
  int base[3] = {0, ncls[0], ncls[0] + ncls[1]};
#pragma unroll
  for (int q = 0; q < NCP; q++) {
    if (q * WG < nc) {
      const int c = ce[q] >> 24;
#pragma unroll
      for (int t = 0; t < 3; t++) base[t] = wave_compact(c == t, cand, base[t], ce[q] & 0xFFFFFF);
    }
  }
  if (LANE == 0) {
    E.ncls[0] = ncls[0];
    E.ncls[1] = ncls[1];
    E.ncls[2] = ncls[2];
  }
  SYNC();
  if (MMX_PROBE == 4 && LANE == 0) {
    stats[STAT_T_AUX0] += (float)nc;
    stats[STAT_T_AUX1] += (float)ncls[1];
    stats[STAT_T_AUX2] += (float)ncls[2];
    stats[STAT_T_AUX3] += (float)ncls[0];
  }
  // probe set 13: per collision pass of a substep, the full 780-pair prunes (no
  // valid persistent list), the list rebuilds that then kept no list (more than MMX_CAND_CAP pairs),
  // and the box-box / GJK candidates after the OBB prune
  if (MMX_PROBE == 13 && LANE == 0 && !only_ro) {
    stats[STAT_T_AUX0] += use_list ? 0.f : 1.f;
    stats[STAT_T_AUX1] += (rebuild && E.ncand < 0) ? 1.f : 0.f;
    stats[STAT_T_AUX2] += (float)ncls[1];
    stats[STAT_T_AUX3] += (float)ncls[2];
  }
  PROBE(2, stats, STAT_T_AUX2);
  PROBE(5, stats, STAT_T_AUX3);
}

// (4) narrowphase over the class lists of collide_prune: which & 1 = plane pairs and box-box
// pairs (lane per pair), which & 2 = GJK/EPA pairs (the whole wave on one pair at a time, EPA
// polytope in LDS beside the box-box polygons)
DEV void collide_pairs(EnvSh& E, bool only_ro, int which) {
  float* stats = E.stats;
  CLK_DECL;
  float* scr = scr_of(E);
  const float* gx = scr + COL_GX;
  const int* cand = reinterpret_cast<const int*>(scr + COL_CAND);
  const int n0 = E.ncls[0], n1 = E.ncls[1], n2 = E.ncls[2];
  if (which & 1) {
    for (int k = LANE; k < n0; k += WG) {  // plane-box / plane-convex
      int p, g1, g2;
      cand_unpack(cand[k], p, g1, g2);
      const Geom A = geom_lds(gx, g1), B = geom_lds(gx, g2);
      WaveSink cs(&E, p, !only_ro, g1, g2);
      if (B.type == GT_BOX) plane_box(cs, A, B, geom_half(gx, g2));
      else if (B.type == GT_MESH) plane_convex(cs, A, B);
    }
    SYNC();
    PROBE(5, stats, STAT_T_AUX0);
    // box-box, one pair per lane quad (16 pairs per pass): the clip's vertices split over the quad
    V3* poly = reinterpret_cast<V3*>(scr + COL_WORK + COL_POLY * (LANE >> 2));
    for (int k0 = 0; k0 < n1; k0 += WG / 4) {
      const int k = k0 + (LANE >> 2);
      if (k < n1) {
        int p, g1, g2;
        cand_unpack(cand[n0 + k], p, g1, g2);
        const Geom A = geom_lds(gx, g1), B = geom_lds(gx, g2);
        WaveSink cs(&E, p, !only_ro, g1, g2);
        box_box_quad(cs, A, B, geom_half(gx, g1), geom_half(gx, g2), poly, poly + 8);
      }
    }
    SYNC();
    PROBE(5, stats, STAT_T_AUX1);
  }
  if (which & 2) {
    for (int k = 0; k < n2; k++) {  // GJK / EPA
      int p, g1, g2;
      cand_unpack(cand[n0 + n1 + k], p, g1, g2);
      const Geom A = geom_lds(gx, g1), B = geom_lds(gx, g2);
      WaveSink cs(&E, p, !only_ro, g1, g2);
      convex_convex(cs, A, B, scr + SCR_EPA);
    }
    SYNC();
    PROBE(5, stats, STAT_T_AUX2);
  }
}

// (5) deterministic order: rank sort of the contacts by their 16-bit pair/order key
DEV void collide_sort(EnvSh& E) {
  float* stats = E.stats;
  CLK_DECL;
  float* scr = scr_of(E);
  const int n = min(E.ncon, MMX_MAXCON);
  float* tmp = scr + COL_WORK;
  int kb = 0, rank = 0;
  if (LANE < n) {  // rank by the order key (the key word, with the geoms, travels with the record)
    kb = con_key(crec(E, LANE));
    const int key = kb & 0xFFFF;
    for (int j = 0; j < n; j++) rank += (con_key(crec(E, j)) & 0xFFFF) < key;
#pragma unroll
    for (int f = 0; f < CL_F; f++) tmp[f * MMX_MAXCON + rank] = con_of(E)[f * MMX_MAXCON + LANE];
  }
  SYNC();
  for (int k = LANE; k < MMX_MAXCON * CL_F; k += WG) con_of(E)[k] = tmp[k];
  if (LANE == 0) E.ncon = n;
  SYNC();
  PROBE(5, stats, STAT_T_AUX3);
}

DEV void collide_wave(EnvSh& E, bool only_ro) {
  collide_prune(E, only_ro);
  collide_pairs(E, only_ro, 3);
  if (!only_ro) collide_sort(E);
}

// ============================================================================ constraints (wave)
// Soft-constraint reference terms of a row: K, B from solref, impedance from solimp (MuJoCo
// mj_makeImpedance); D = 1 / R with R = (1 - imp) / imp * diag.
DEV void row_ref(const float* solref, const float* solimp, float pos, float& imp_ratio, float& kid, float& B) {
  const float imp = impedance(solimp, pos);
  const float dmax = fminf(fmaxf(solimp[1], 1e-4f), 0.9999f);
  const float tc = fmaxf(solref[0], 2.f * kDt), dr = solref[1];
  const float K = 1.f / (dmax * dmax * tc * tc * dr * dr);
  B = 2.f / (dmax * tc);
  imp_ratio = (1.f - imp) / imp;
  kid = K * imp * pos;
}
DEV void store_row(EnvSh& E, int row, const float* jv, int hdr, float vel, float imp_ratio, float kid, float B,
                   float diag) {
  const float aref = -B * vel - kid;  // slot 15
  if (row < MMX_LDSEFC) {
#pragma unroll
    for (int q = 0; q < 3; q++)
      *reinterpret_cast<float4*>(E.J[q][row]) = make_float4(jv[4 * q], jv[4 * q + 1], jv[4 * q + 2], jv[4 * q + 3]);
    *reinterpret_cast<float4*>(E.J[3][row]) = make_float4(jv[12], jv[13], jv[14], aref);
  } else {
    float4* Jr = reinterpret_cast<float4*>(ovf_j(E, row));
#pragma unroll
    for (int q = 0; q < 3; q++) Jr[q] = make_float4(jv[4 * q], jv[4 * q + 1], jv[4 * q + 2], jv[4 * q + 3]);
    Jr[3] = make_float4(jv[12], jv[13], jv[14], aref);
  }
  hdr_set(E, row, hdr);
  dset(E, row, 1.f / fmaxf(imp_ratio * diag, 1e-15f));
}

// A contact's mixed parameters (MuJoCo: friction and condim the max of the two geoms', solref /
// solimp their mean) and reference terms: computed by each of its basis rows' lanes from the
// 9-float LDS record (the rows of one contact are built by up to four lanes; the same inputs and
// arithmetic give each the same values)
struct ConPar {
  int dim;
  float mu0, mu1, kid, B, idiag;
};
template <class R>
DEV ConPar contact_params(const R& cc) {
  const int g1 = con_g1(cc), g2 = con_g2(cc);
  ConPar P;
  P.dim = max(MMX_geom_condim[g1], MMX_geom_condim[g2]);
  P.mu0 = fmaxf(MMX_geom_friction[3 * g1], MMX_geom_friction[3 * g2]);
  P.mu1 = fmaxf(MMX_geom_friction[3 * g1 + 1], MMX_geom_friction[3 * g2 + 1]);
  float solref[2], solimp[5];
#pragma unroll
  for (int k = 0; k < 2; k++) solref[k] = 0.5f * (MMX_geom_solref[2 * g1 + k] + MMX_geom_solref[2 * g2 + k]);
#pragma unroll
  for (int k = 0; k < 5; k++) solimp[k] = 0.5f * (MMX_geom_solimp[5 * g1 + k] + MMX_geom_solimp[5 * g2 + k]);
  float impr;
  row_ref(solref, solimp, cc[CL_DIST], impr, P.kid, P.B);
  const int b1 = MMX_geom_body[g1], b2 = MMX_geom_body[g2];
  const float tran = MMX_body_invweight0[2 * b1] + MMX_body_invweight0[2 * b2];
  const float it = impr * tran;  // (the pyramid's common R needs only the translational invweight)
  // pyramidal cone: one R for every edge, A_hat = 2 mu0^2 (tran + mu0^2 tran) / impratio (impratio
  // = 1), R = (1 - d) / d A_hat; pinned by the closed-form scenes of tests/test_physics_kat.py
  P.idiag = P.dim > 1 ? 2.f * P.mu0 * P.mu0 * (it + P.mu0 * P.mu0 * it) : it;
  return P;
}
DEV V3 contact_t1(V3 n) {  // mju_makeFrame's first tangent
  const V3 y = (n.y < 0.5f && n.y > -0.5f) ? V3{0.f, 1.f, 0.f} : V3{0.f, 0.f, 1.f};
  return normalize(y - n * dot(n, y));
}

// Basis row rr of contact c, built straight into block format: rr 0 = normal, 1 / 2 = tangents
// t1 / t2 (mju_makeFrame), 3 = rotation about the normal (torsion, condim 4).  MuJoCo's pyramid
// edges of the contact are J_n +/- mu_k J_k (k = t1, t2 with the sliding mu, torsion with the
// torsional mu) and their aref = aref_n +/- mu_k aref_k with aref_k = -B J_k qvel (the position
// term belongs to the normal); the solver forms them from these rows.  An arm block entry is the
// motion subspace of dof d seen at the contact point, a cube block the free-body Jacobian.  Rows the
// contact's condim does not use are zero rows with D = 0.  Returns the row's mu (-1: no edges).
DEV float contact_row(EnvSh& E, int row, const CReg& cc, int rr, const ConPar& P) {
  const V3 p = V3{cc[CL_POS], cc[CL_POS + 1], cc[CL_POS + 2]};
  const V3 n = V3{cc[CL_N], cc[CL_N + 1], cc[CL_N + 2]};
  const int b1 = MMX_geom_body[con_g1(cc)], b2 = MMX_geom_body[con_g2(cc)];
  const int dim = P.dim;
  const bool used = rr == 0 || (rr < 3 && dim >= 3) || (rr == 3 && dim >= 4);
  const V3 t1 = contact_t1(n);
  const V3 u = rr == 0 ? n : (rr == 1 ? t1 : (rr == 2 ? cross(n, t1) : V3{0.f, 0.f, 0.f}));
  const V3 w = rr == 3 ? n : V3{0.f, 0.f, 0.f};
  const float idiag = P.idiag;  // impedance ratio x diagApprox
  const int k1 = body_block(b1), k2 = body_block(b2);
  int rb0 = k1 >= 0 ? k1 : k2, rb1 = (k1 >= 0 && k2 >= 0 && k2 != k1) ? k2 : BLK_NONE;
  if (rb1 != BLK_NONE && rb1 < rb0) {
    const int t = rb0;
    rb0 = rb1;
    rb1 = t;
  }
  // arm block: coefficient +1 / -1 / 0 of dof d from the two bodies' ancestor-dof masks
  const unsigned am1 = anc_mask(b1), am2 = anc_mask(b2);
  float vel = 0.f;
  float arm[9];
  // u . (v_d + w_d x p) + w . w_d = u . v_d + w_d . (p x u + w): one cross product per row
  const V3 pu = cross(p, u) + w;
#pragma unroll
  for (int d = 0; d < 9; d++) {  // body 2 counts +, body 1 counts -
    const float coef = (float)((int)((am2 >> d) & 1u) - (int)((am1 >> d) & 1u));
    const SV sd = load_S(E, d);
    arm[d] = coef * (dot(u, sd.v) + dot(sd.w, pu));
    vel = fmaf(arm[d], E.qvel[d], vel);
  }
  float cubeA[6], cubeB[6];  // blocks rb0 (when a cube) and rb1
  // each body's free-body columns (zero unless it is a cube), velocity summed in body order; block
  // A (rb0) is body 1's unless body 1 is not rb0
  float cvs[2][6];
#pragma unroll
  for (int side = 0; side < 2; side++) {
    const int b = side ? b2 : b1, blk = side ? k2 : k1;
#pragma unroll
    for (int j = 0; j < 6; j++) cvs[side][j] = 0.f;
    if (blk > 0) {
      const float sg = side ? 1.f : -1.f;
      const V3 x = body_x(E, b);
      const M3 R = body_R(E, b);
      cvs[side][0] = sg * u.x;
      cvs[side][1] = sg * u.y;
      cvs[side][2] = sg * u.z;
      const V3 ru = cross(p - x, u) + w;  // u . (r_k x (p - x)) + w . r_k = r_k . ((p - x) x u + w)
#pragma unroll
      for (int k = 0; k < 3; k++) cvs[side][3 + k] = sg * dot(col(R, k), ru);
      const int d0 = blk_d0(blk);
#pragma unroll
      for (int j = 0; j < 6; j++) vel = fmaf(cvs[side][j], E.qvel[d0 + j], vel);
    }
  }
  const bool swap = k1 != rb0;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    cubeA[j] = swap ? cvs[1][j] : cvs[0][j];
    cubeB[j] = swap ? cvs[0][j] : cvs[1][j];
  }
  float jv[16];
  const bool armrow = rb0 == 0;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const float va = j < 9 ? arm[j] : (j < 15 ? cubeB[j - 9] : 0.f);
    const float vc = j < 6 ? cubeA[j] : (j < 12 ? cubeB[j - 6] : 0.f);
    jv[j] = armrow ? va : vc;
  }
  store_row(E, row, jv, rb0 | (rb1 << 4), vel, 1.f, rr == 0 ? P.kid : 0.f, P.B, idiag);
  if (!used) dset(E, row, 0.f);  // (its J is zero as well: u = w = 0)
  return !used || rr == 0 ? (rr == 0 ? 0.f : -1.f) : (rr < 3 ? P.mu0 : P.mu1);
}

// Constraint rows in MuJoCo's order per lane scan: finger equality (lane 0), joint limits
// (lanes 0..8), contacts (lane c = contact c, 4 basis rows each).  Equality and limit rows are
// written by their lanes; contact rows are spread over all lanes through a row -> (contact, basis
// row) map.  Rows are grouped by block-pair type in aligned groups of 4 (type 0 starts with the
// equality / limit rows, padded with zero rows to a multiple of 4); the rows' mu (the solver's
// edge coefficients) go to the solver in registers (mu_out, the lane's rows LANE + 64 q).
DEV void make_constraints_wave(EnvSh& E, float* mu_out) {
  float* stats = E.stats;
  CLK_DECL;
  const float def_ref[2] = {0.02f, 1.0f};
  const float def_imp[5] = {0.9f, 0.95f, 0.001f, 0.5f, 2.0f};
  const int ncon = E.ncon;
  // the lane's own contact into registers (lane c: contact c): the rows overwrite the scratch region
  // that holds the contacts, and each row's lane reads its contact's fields from lane c (ds_bpermute)
  CReg own;
#pragma unroll
  for (int k = 0; k < CL_F; k++) own.v[k] = LANE < ncon ? crec(E, LANE)[k] : 0.f;
  // row -> (contact, basis row) map, -1 for the equality / limit / padding rows; it lives in the
  // rows' D (dset / dget), so the equality / limit rows (whose store_row writes D) are stored after
  // the contact rows
  auto rowmap_set = [&](int r, int m) { dset(E, r, __int_as_float(m)); };
  int nlim = 0, tc = -1, nedge = 0;
  bool lo_act = false, hi_act = false;
  if (LANE < 9) {
    const float q = E.qpos[LANE];
    lo_act = q - MMX_jnt_range[2 * LANE] < 0.f;
    hi_act = MMX_jnt_range[2 * LANE + 1] - q < 0.f;
    nlim = (int)lo_act + (int)hi_act;
  }
  if (LANE < ncon) {
    const int g1 = con_g1(own), g2 = con_g2(own);
    const int dim = max(MMX_geom_condim[g1], MMX_geom_condim[g2]);
    nedge = dim == 1 ? 1 : 2 * (dim - 1);
    const int k1 = body_block(MMX_geom_body[g1]), k2 = body_block(MMX_geom_body[g2]);
    int rb0 = k1 >= 0 ? k1 : k2, rb1 = (k1 >= 0 && k2 >= 0 && k2 != k1) ? k2 : BLK_NONE;
    if (rb1 != BLK_NONE && rb1 < rb0) {
      const int t = rb0;
      rb0 = rb1;
      rb1 = t;
    }
    tc = row_type(rb0, rb1);
  }
  // single rows (equality + limits), then per type the contact groups
  const int acnt = (LANE == 0 ? 1 : 0) + nlim;
  // acnt <= 3: its two bits as ballots give the exclusive prefix and the total without a scan
  const unsigned long long a0 = __ballot(acnt & 1), a1 = __ballot(acnt & 2);
  const int nsingle_raw = __popcll(a0) + 2 * __popcll(a1);
  const int arow = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(a0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)a0, 0u)) +
                   2 * (int)__builtin_amdgcn_mbcnt_hi((unsigned)(a1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)a1, 0u));
  const int nsingle = (nsingle_raw + 3) & ~3;
  int brow = 0, base = 0;
  // per type: one ballot of the contacts (lanes) of that type; a lane's rows start at the type's
  // base plus 4 x the contacts of its type in lower lanes (mbcnt), so no prefix scans
#pragma unroll
  for (int t = 0; t < NTYPE; t++) {
    const unsigned long long m = __ballot(tc == t);
    const int first = base + (t == 0 ? nsingle : 0);  // type 0: the single rows come first
    if (tc == t) brow = first + 4 * (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    if (LANE == 0) E.tbase[t] = min(base, MMX_MAXEFC);
    base = first + 4 * __popcll(m);
  }
  const int total = base;
  const int nefc = min(total, MMX_MAXEFC);
  const int nefc_mj = nsingle_raw + __popcll(__ballot(nedge & 1)) + 2 * __popcll(__ballot(nedge & 2)) +
                      4 * __popcll(__ballot(nedge & 4));  // nedge <= 6
  if (LANE == 0) {
    E.tbase[NTYPE] = nefc;
    E.nefc = nefc;
    E.nefc_mj = nefc_mj;
    E.nsingle = nsingle;
    if (total > MMX_MAXEFC) E.flags |= SHF_EFC_OVF;
  }
  PROBE(3, stats, STAT_T_AUX0);
  if (LANE < 4 && nsingle_raw + LANE < nsingle) rowmap_set(nsingle_raw + LANE, -1);  // padding
  int row = arow;
  if (LANE == 0 && row < MMX_MAXEFC) rowmap_set(row++, -1);  // finger equality
  if (LANE < 9) {
#pragma unroll
    for (int side = 0; side < 2; side++)
      if ((side == 0 ? lo_act : hi_act) && row < MMX_MAXEFC) rowmap_set(row++, -1);  // joint limits
  }
  PROBE(3, stats, STAT_T_AUX1);
  // each contact's parameters computed once, by its lane, and read by its rows' lanes over ds_bpermute
  // (computing them per row measured -1.3 %)
  ConPar Pc{1, 0.f, 0.f, 0.f, 0.f, 1.f};
  if (LANE < ncon) Pc = contact_params(own);
  if (LANE < ncon) {  // the contact's 4 basis rows in the row -> (contact, basis row) map
#pragma unroll
    for (int rr = 0; rr < 4; rr++)
      if (brow + rr < MMX_MAXEFC) rowmap_set(brow + rr, LANE | (rr << 8));
  }
  ovf_fence(nefc);
  SYNC();
  PROBE(3, stats, STAT_T_AUX3);
  constexpr int RPB = (MMX_MAXEFC + WG - 1) / WG;
  float mu[RPB];
#pragma unroll
  for (int q = 0; q < RPB; q++) {
    const int r = LANE + WG * q;
    mu[q] = 0.f;
    if (WG * q >= nefc) continue;  // uniform: no row in this slice
    const int m = r < nefc ? __float_as_int(dget(E, r)) : -1;
    const int c = m >= 0 ? (m & 255) : 0;
    ConPar P;  // contact c's parameters from lane c (every lane takes part in the exchange)
    P.dim = __shfl(Pc.dim, c);
    P.mu0 = __shfl(Pc.mu0, c);
    P.mu1 = __shfl(Pc.mu1, c);
    P.kid = __shfl(Pc.kid, c);
    P.B = __shfl(Pc.B, c);
    P.idiag = __shfl(Pc.idiag, c);
    CReg cc;  // contact c's position, normal and geoms from lane c
    cc.v[CL_DIST] = 0.f;
#pragma unroll
    for (int k = CL_POS; k < CL_F; k++) cc.v[k] = __shfl(own.v[k], c);
    if (m >= 0) mu[q] = contact_row(E, r, cc, m >> 8, P);
  }
  row = arow;
  float jv[16];
  if (LANE == 0 && row < MMX_MAXEFC) {  // finger equality (panda.xml:261)
#pragma unroll
    for (int j = 0; j < 16; j++) jv[j] = j == 7 ? 1.f : (j == 8 ? -1.f : 0.f);
    float ir, kid, B;
    row_ref(MMX_eq_solref, MMX_eq_solimp, E.qpos[7] - E.qpos[8], ir, kid, B);
    store_row(E, row, jv, 0 | (BLK_NONE << 4), E.qvel[7] - E.qvel[8], ir, kid, B,
              MMX_dof_invweight0[7] + MMX_dof_invweight0[8]);
    row++;
  }
  if (LANE < 9) {  // joint limits (MuJoCo default solref / solimp)
    const float q = E.qpos[LANE];
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const bool act = side == 0 ? lo_act : hi_act;
      if (act && row < MMX_MAXEFC) {
        const float sg = side == 0 ? 1.f : -1.f;
#pragma unroll
        for (int j = 0; j < 16; j++) jv[j] = j == LANE ? sg : 0.f;
        const float dist = side == 0 ? q - MMX_jnt_range[2 * LANE] : MMX_jnt_range[2 * LANE + 1] - q;
        float ir, kid, B;
        row_ref(def_ref, def_imp, dist, ir, kid, B);
        store_row(E, row, jv, 0 | (BLK_NONE << 4), sg * E.qvel[LANE], ir, kid, B, MMX_dof_invweight0[LANE]);
        row++;
      }
    }
  }
  if (LANE < 4 && nsingle_raw + LANE < nsingle) {  // zero padding rows (weight 0)
#pragma unroll
    for (int j = 0; j < 16; j++) jv[j] = 0.f;
    store_row(E, nsingle_raw + LANE, jv, 0 | (BLK_NONE << 4), 0.f, 1.f, 0.f, 0.f, 1.f);
    dset(E, nsingle_raw + LANE, 0.f);
  }
  ovf_fence(nefc);
  SYNC();  // every row is built; the rows' mu go to the solver in registers
#pragma unroll
  for (int q = 0; q < RPB; q++) mu_out[q] = mu[q];
  PROBE(3, stats, STAT_T_AUX2);
}

#undef LANE
#define LANE lane_opaque()  // the Newton solver section (see lane_opaque)
// ============================================================================ Newton solver (wave)
// Primal Newton with exact line search (MuJoCo's default solver): minimise
//   0.5 (x - xs)' M (x - xs) + sum_i s_i(J_i x - aref_i),  s_i = 0.5 D_i r^2 on active rows.
// Lane l owns constraint rows l + 64 q (q < RPL): their residual, search-direction projection,
// D and equality flag stay in registers through the line search.  The Hessian and gradient come
// from one MFMA pass (hess_grad_mfma) straight into registers; the Cholesky factorisation and
// both triangular solves run in registers (chol_solve).
#define RPL ((MMX_MAXEFC + WG - 1) / WG)

DEV float readlane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

// Newton lane layout: the solver's dof-space values (Hessian rows, gradient, search direction,
// M v) sit with arm dof d in lane d (DPP row 0 of the wave's four 16-lane rows) and cube b's dof k
// in lane 16 b + k (row b), so each dof block owns one DPP row: the block Cholesky broadcasts a
// pivot to its block with one row_newbcast.  Lanes 9..15, 16 b + 6..15 hold no dof (-1).
DEV int newton_dof(int L) {
  const int r = L >> 4, k = L & 15;
  return r == 0 ? (k < 9 ? k : -1) : (k < 6 ? 9 + 6 * (r - 1) + k : -1);
}
__host__ __device__ constexpr int newton_lane(int d) { return d < 9 ? d : 16 * (1 + (d - 9) / 6) + (d - 9) % 6; }

// J_i . x for a block-format row (slots past the row's width hold zeros)
DEV float row_dot16(const EnvSh& E, int i, const float* x) {
  const int h = hdr_get(E, i), b0 = h & 15, b1 = (h >> 4) & 15;
  const int n0 = blk_size(b0), o0 = blk_d0(b0), o1 = (b1 == BLK_NONE ? 0 : blk_d0(b1)) - n0;
  float jv[16];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const float4 v = jrow4(E, i, q);
    jv[4 * q] = v.x;
    jv[4 * q + 1] = v.y;
    jv[4 * q + 2] = v.z;
    jv[4 * q + 3] = v.w;
  }
  // slot k holds dof k + o0 below n0 and dof k + o1 from n0 on (n0 = 9 for an arm block, 6 for a
  // cube), so slots 0..5 read from one base, 6..8 from the base n0 selects, 9..11 from the second
  // one: LDS reads with immediate offsets instead of a per-slot index select.  Slots 12..14 are
  // clamped to dof 26 (past the row's width they hold zeros; the clamp keeps the read in x).
  const float* x0 = x + o0;
  const float* x1 = x + o1;
  const float* x2 = n0 == 9 ? x0 : x1;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    const float v = k < 6 ? x0[k] : (k < 9 ? x2[k] : (k < 12 ? x1[k] : x[min(o1 + k, 26)]));
    s = fmaf(jv[k], v, s);
  }
  return s;
}

// the cubes' diagonal mass matrix entry of free dof k (0..17: cube k / 6, mass x3 then principal
// inertia x3): model constants, not per env
DEV float mass_cube(int k) {
  const int b = 16 + k / 6, rr = k % 6;
  return rr < 3 ? MMX_body_mass[b] : MMX_body_inertia[9 * b + 4 * (rr - 3)];
}
// (M v) of the lane's dof (Newton lane layout; arm rows: the 9 x 9 block; cube rows: the diagonal)
DEV float mass_mul(const EnvSh& E, const float* v) {
  const int nd = newton_dof(LANE);
  if (LANE < 9) {
    float m = 0.f;
#pragma unroll
    for (int b = 0; b < 9; b++) m = fmaf(E.M9[LANE][b], v[b], m);
    return m;
  }
  return nd >= 0 ? mass_cube(nd - 9) * v[nd] : 0.f;
}
// (M (xa - xb)) of the lane's dof, same layout
DEV float mass_mul_diff(const EnvSh& E, const float* xa, const float* xb) {
  const int nd = newton_dof(LANE);
  if (LANE < 9) {
    float m = 0.f;
#pragma unroll
    for (int b = 0; b < 9; b++) m = fmaf(E.M9[LANE][b], xa[b] - xb[b], m);
    return m;
  }
  return nd >= 0 ? mass_cube(nd - 9) * (xa[nd] - xb[nd]) : 0.f;
}

// Pyramid edges from basis rows.  Lane l owns rows l + 64 q; rows are 4-aligned groups, so a
// group's rows sit in one DPP quad (lanes 4m..4m+3).  A row's role: single (equality / limit /
// padding row: one edge, itself), normal row of a contact (no edge of its own), basis row k >= 1 of
// a contact (the two edges J_n +/- mu_k J_k; mu < 0: unused row, no edge).  Edge e of the lane's
// row is a_e (normal row value) + b_e (own value), for residuals and for J p alike.
struct EdgeCoef {
  float a0, b0, a1, b1;  // edge 0: a0 n + b0 own, edge 1: a1 n + b1 own; all 0 for a missing edge
};
// (no boolean per edge: a missing edge has zero coefficients, so its value is 0 and never
// active; only the finger equality, row 0 = lane 0 of slice 0, is active at any sign)
DEV EdgeCoef edge_coef(int i, int nefc, int nsingle, float mu) {
  EdgeCoef c;
  const bool valid = i < nefc;
  const bool single = valid && i < nsingle;
  const bool krow = valid && !single && (i & 3) != 0 && mu >= 0.f;
  c.a0 = krow ? 1.f : 0.f;
  c.b0 = krow ? mu : (single ? 1.f : 0.f);
  c.a1 = c.a0;
  c.b1 = krow ? -mu : 0.f;
  return c;
}
// the finger equality row (always active): row 0, owned by lane 0 in slice 0
#define EQROW(q) ((q) == 0 && LANE == 0)
// value held by the first lane of the caller's DPP quad (the group's normal row)
DEV float quad_first(float v) { return dpp_f<0x00>(v); }  // quad_perm [0,0,0,0]
DEV float quad_sum(float v) {
  v += dpp_f<0xB1>(v);  // quad_perm [1,0,3,2]
  return v + dpp_f<0x4E>(v);  // quad_perm [2,3,0,1]
}

// cost at two candidate points (warm start, qacc_smooth) in one pass; also returns, per lane,
// the basis-row residuals J x - aref of the rows it owns and (M (x - xs))_lane for both
// candidates, so the Newton loop starts from them and then only updates them (r += a J p,
// M dx += a M p).  Edge cost 0.5 D e^2 on active edges (e < 0, or the equality).
DEV void cost2_wave(const EnvSh& E, const float* xa, const float* xb, const float* mu, const float* dd, float& ca,
                    float& cb, float* va, float* vb, float& ma, float& mb) {
  float c0 = 0.f, c1 = 0.f;
  ma = 0.f;
  mb = 0.f;
  const int nd = newton_dof(LANE);
  if (nd >= 0) {
    ma = mass_mul_diff(E, xa, E.qacc_s);
    mb = mass_mul_diff(E, xb, E.qacc_s);
    c0 = 0.5f * (xa[nd] - E.qacc_s[nd]) * ma;
    c1 = 0.5f * (xb[nd] - E.qacc_s[nd]) * mb;
  }
  const int nefc = E.nefc, nsingle = E.nsingle;
#pragma unroll
  for (int q = 0; q < RPL; q++) {
    const int i = LANE + WG * q;
    va[q] = 0.f;
    vb[q] = 0.f;
    if (WG * q >= nefc) continue;  // uniform: the slice holds no row
    if (i < nefc) {
      const float aref = jget(E, i, 15);
      va[q] = row_dot16(E, i, xa) - aref;
      vb[q] = row_dot16(E, i, xb) - aref;
    }
    const float na = quad_first(va[q]), nb = quad_first(vb[q]);
    const EdgeCoef ec = edge_coef(i, nefc, nsingle, mu[q]);
    const float ea0 = fmaf(ec.a0, na, ec.b0 * va[q]), ea1 = fmaf(ec.a1, na, ec.b1 * va[q]);
    const float eb0 = fmaf(ec.a0, nb, ec.b0 * vb[q]), eb1 = fmaf(ec.a1, nb, ec.b1 * vb[q]);
    const float h = 0.5f * dd[q];
    c0 += (EQROW(q) || ea0 < 0.f ? h * ea0 * ea0 : 0.f) + (ea1 < 0.f ? h * ea1 * ea1 : 0.f);
    c1 += (EQROW(q) || eb0 < 0.f ? h * eb0 * eb0 : 0.f) + (eb1 < 0.f ? h * eb1 * eb1 : 0.f);
  }
  ca = wave_sum(c0);
  cb = wave_sum(c1);
}

// J'WJ and J'W r on the matrix cores, one block-pair row type at a time.  Rows of a type share
// their slot -> dof map, so in slot space the type's contribution is a 16 x 16 tile.  Over the
// pyramid edges J_e = c_e' B of a 4-row group B (c_e = e_n +/- mu_k e_k), sum_e w_e J_e' J_e =
// B' C B with the group's 4 x 4 edge-weight matrix C = sum_e w_e c_e c_e' (an arrow: C_nn, C_nk,
// C_kk), and sum_e w_e r_e J_e' = B' g.  So G = sum_groups B' [C B | g]:
// v_mfma_f32_16x16x4_f32 with A[slot i][row k] = B[k][i] and B-operand[row k][slot j] =
// (C B)[k][j] = C_kk B[k][j] + (k == n ? sum_m C_nm B[m][j] : C_nk B[n][j]), where slot 15
// (always 0 in J) carries g_k instead, so G[:, 15] is the type's gradient.  Single rows form
// groups with a diagonal C (their active weights).  Lane l supplies row (l >> 4) of the step's
// group at slot l & 15: contiguous reads of the block-format rows.  Each tile is staged in LDS and gathered by the
// dof lanes into their Hessian row (static columns) and gradient.  Returns, in lane j < 27,
// row j of H = M + J'WJ in hrow[0..27) and g_j = (M (x - xs) + J'W r)_j.
typedef float f32x4 __attribute__((ext_vector_type(4)));
// groups (MFMA steps) per trip, their loads issued together (3 or 4: -1.3 / -0.7 % in the r03 A/B)
#define MMX_HESS_U 2
// gather one row type's staged 16 x 16 tile into the dof lanes' Hessian rows: dof lane d reads row
// sd of the tile; the type's two blocks land on static columns of hrow (uniform branches over the
// 4 possible blocks keep every register index static); slot 15 is the type's gradient
DEV void tile_gather(const float* G, int t, int bd, int od, float* hrow, float& gacc) {
  const int b0 = kTB0[t], b1 = kTB1[t];
  const int n0 = blk_size(b0);
  const int sd = bd == b0 ? od : (bd == b1 ? n0 + od : -1);
  if (sd >= 0) {
    const float* Gr = G + GST * sd;
#pragma unroll
    for (int B = 0; B < 4; B++) {
      const int nb = B == 0 ? 9 : 6, dB = B == 0 ? 0 : 9 + 6 * (B - 1);
      if (B == b0) {
#pragma unroll
        for (int k = 0; k < nb; k++) hrow[dB + k] += Gr[k];
      } else if (B == b1) {
#pragma unroll
        for (int k = 0; k < nb; k++) hrow[dB + k] += Gr[n0 + k];
      }
    }
    gacc += Gr[15];
  }
}
// row types staged per barrier round (E.con holds up to three 16 x 16 tiles; 3 measured -1.3 % in the
// r03 A/B: the unrolled rounds grow the substep's register save area)
#define HESS_TILES 1
static_assert(HESS_TILES * 16 * GST <= MMX_MAXCON * CL_F, "Hessian staging tiles exceed E.con");
DEV float hess_grad_mfma(EnvSh& E, int nefc, float* hrow, float mdx) {
  float* stats = E.stats;
  CLK_DECL;
  float* G = lrow_of(E);  // 16 x 16 staging tile (the factor's space is free until the Cholesky)
  const int col = LANE & 15, rk = LANE >> 4;
  // the lane's dof (Newton lane layout): block LANE >> 4, offset LANE & 15 in it
  const int nd = newton_dof(LANE), d = max(nd, 0);
  const int bd = nd >= 0 ? LANE >> 4 : -2, od = LANE & 15;
#pragma unroll
  for (int i = 0; i < 27; i++) hrow[i] = d < 9 ? (i < 9 ? E.M9[d][i] : 0.f) : (i == d ? mass_cube(d - 9) : 0.f);
  float gacc = 0.f;
  PROBE(6, stats, STAT_T_AUX3);
  // The non-empty row types go in rounds of up to HESS_TILES: each type's tile is staged in its
  // own 16 x 16 slot of E.con (free until the Cholesky), then one barrier, then the dof lanes
  // gather every tile of the round (in type order, so the sums are the same as one type at a time)
  unsigned tmask = 0;  // non-empty row types (uniform)
  for (int t = 0; t < NTYPE; t++) tmask |= E.tbase[t + 1] > E.tbase[t] ? 1u << t : 0u;
  tmask = __builtin_amdgcn_readfirstlane(tmask);
  int nst = 0, tyslots = 0;  // tiles staged in this round and their row types (4 bits each)
  auto flush = [&]() {
    if (nst == 0) return;
    SYNC();
#pragma unroll
    for (int j = 0; j < HESS_TILES; j++)
      if (j < nst) tile_gather(G + 16 * GST * j, (tyslots >> (4 * j)) & 15, bd, od, hrow, gacc);
    SYNC();
    nst = 0;
    tyslots = 0;
    PROBE(6, stats, STAT_T_AUX1);
  };
  while (tmask) {
    {
      const int t = __builtin_ctz(tmask);
      tmask &= tmask - 1u;
      const int r0 = E.tbase[t], r1 = E.tbase[t + 1];
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      // MMX_HESS_U MFMA steps (one 4-row group each) per trip, loads first; the steps alternate
      // between the two accumulators, so each sums the same groups in the same order for any
      // MMX_HESS_U.  Types span whole groups (tbase and MMX_LDSEFC are multiples of 4), so every step
      // is full.  The LDS groups and the (rare) HBM overflow groups run in separate loops: one
      // address space per loop, no generic (flat) loads in the hot one.
      const float m_[4] = {rk == 0 ? 1.f : 0.f, rk == 1 ? 1.f : 0.f, rk == 2 ? 1.f : 0.f, rk == 3 ? 1.f : 0.f};
      const float c15 = col == 15 ? 1.f : 0.f;  // slot 15 carries g, not C B
      auto groups = [&](auto from_lds, int g_begin, int g_end) {
        constexpr bool LDS = decltype(from_lds)::value;
        float jg_[MMX_HESS_U][4], nc_[MMX_HESS_U][4], dr_[MMX_HESS_U];
        auto load_trip = [&](int s0) {
  #pragma unroll
          for (int u = 0; u < MMX_HESS_U; u++) {
            const int g0 = min(s0 + 4 * u, g_end - 4), r = g0 + rk;
            if (LDS) {
              const float4 n4 = *reinterpret_cast<const float4*>(&E.NC[g0]);  // one broadcast read
              nc_[u][0] = n4.x; nc_[u][1] = n4.y; nc_[u][2] = n4.z; nc_[u][3] = n4.w;
  #pragma unroll
              for (int m = 0; m < 4; m++) jg_[u][m] = jlds(E, g0 + m, col);  // slot 15 holds g
              dr_[u] = E.D[r];
            } else {
  #pragma unroll
              for (int m = 0; m < 4; m++) {
                jg_[u][m] = ovf_j(E, g0 + m)[col];
                nc_[u][m] = *ovf_nc(E, g0 + m);
              }
              dr_[u] = *ovf_d(E, r);
            }
          }
        };
        for (int s0 = g_begin; s0 < g_end; s0 += 4 * MMX_HESS_U) {
          float a[MMX_HESS_U], b[MMX_HESS_U];
          load_trip(s0);
  #pragma unroll
          for (int u = 0; u < MMX_HESS_U; u++) {
            // arithmetic selects over the lane's row rk (0 / 1 masks): no divergent branches
            const float live = s0 + 4 * u < g_end ? 1.f : 0.f;  // uniform
            const float* jg = jg_[u];
            const float* nc = nc_[u];
            const float own = fmaf(m_[0], jg[0], fmaf(m_[1], jg[1], fmaf(m_[2], jg[2], m_[3] * jg[3])));
            const float ncr = fmaf(m_[1], nc[1], fmaf(m_[2], nc[2], m_[3] * nc[3]));  // C_nk of row rk (0 for n)
            const float s123 = fmaf(nc[1], jg[1], fmaf(nc[2], jg[2], nc[3] * jg[3]));
            const float cpl = fmaf(ncr, jg[0], m_[0] * s123);
            a[u] = live * own;  // (slot 15 only feeds G's unused row 15)
            b[u] = live * fmaf(c15, own - fmaf(dr_[u], own, cpl), fmaf(dr_[u], own, cpl));
          }
  #pragma unroll
          for (int u = 0; u < MMX_HESS_U; u++) {
            if (u & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc1, 0, 0, 0);
            else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc0, 0, 0, 0);
          }
        }
      };
      const int split = min(max(r0, MMX_LDSEFC), r1);
      groups(std::true_type{}, r0, split);
      if (split < r1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the overflow rows' stores (ovf_fence)
        // group k of the type (from r0) goes to accumulator k & 1 in either loop, so the sums do not
        // depend on where the LDS rows end (the 128- and 192-row layouts are bit-identical)
        const bool odd = ((split - r0) >> 2) & 1;  // uniform
        auto swap_acc = [&]() {
          const f32x4 t = acc0;
          acc0 = acc1;
          acc1 = t;
        };
        if (odd) swap_acc();
        groups(std::false_type{}, split, r1);
        if (odd) swap_acc();
      }
      PROBE(6, stats, STAT_T_AUX0);
      // stage: lane l holds G[4 (l >> 4) + q][l & 15]
#pragma unroll
      for (int q = 0; q < 4; q++) G[16 * GST * nst + GST * (4 * rk + q) + col] = acc0[q] + acc1[q];
      tyslots |= t << (4 * nst);
      if (++nst == HESS_TILES) flush();
    }
  }
  flush();
  PROBE(6, stats, STAT_T_AUX2);
  return nd >= 0 ? gacc + mdx : 0.f;
}

// Incremental form of hess_grad_mfma for the Newton iterations after the first.  Over a line
// search only the edges whose active state flipped change their weight, so with Delta C the
// groups' change of edge-weight matrix (nonzero only in groups holding a flipped edge):
//   H_new = H_old + sum_groups B' dC B,   g_new = g_old + a H_old p + sum_groups B' dC r_new
// (g = M (x - xs) + sum B' C r; B' C_old r_new = B' C_old r_old + a B' C_old B p).  E.D / E.NC /
// slot 15 hold dC_kk, dC_nk and dC r_new (newton_wave's weight pass in delta mode); gm[q] bit 4m
// marks group m of row slice q as changed (wave-uniform).  Only the changed groups' MFMA steps run,
// and only the row types holding one are staged and gathered, LDS and HBM overflow rows alike (r05:
// with 128 LDS rows the grasp phases' rows spill; the full pass whenever rows spill, as in r02-r04,
// measured slower).  Adds into hrow; returns sum B' dC r in lane j < 27.
#define HESS_LQ (MMX_LDSEFC / WG)  // row slices held in LDS
#define HESS_NQ RPL                // row slices the delta pass covers
DEV float hess_grad_delta(EnvSh& E, float* hrow, const unsigned long long* gm) {
  float* G = lrow_of(E);
  const int col = LANE & 15, rk = LANE >> 4;
  const int nd = newton_dof(LANE);
  const int bd = nd >= 0 ? LANE >> 4 : -2, od = LANE & 15;
  const float m_[4] = {rk == 0 ? 1.f : 0.f, rk == 1 ? 1.f : 0.f, rk == 2 ? 1.f : 0.f, rk == 3 ? 1.f : 0.f};
  const float c15 = col == 15 ? 1.f : 0.f;
  float gacc = 0.f;
  int nst = 0, tyslots = 0;  // tiles staged in this round and their row types (4 bits each)
  auto flush = [&]() {
    if (nst == 0) return;
    SYNC();
#pragma unroll
    for (int j = 0; j < HESS_TILES; j++)
      if (j < nst) tile_gather(G + 16 * GST * j, (tyslots >> (4 * j)) & 15, bd, od, hrow, gacc);
    SYNC();
    nst = 0;
    tyslots = 0;
  };
  for (int t = 0; t < NTYPE; t++) {
    const int r0 = E.tbase[t], r1 = E.tbase[t + 1];
    if (r1 <= r0) continue;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    bool any = false;
#pragma unroll
    for (int q = 0; q < HESS_NQ; q++) {
      if (64 * q >= r1 || 64 * (q + 1) <= r0) continue;  // uniform
      const int lo = max(r0 - 64 * q, 0), hi = min(r1 - 64 * q, 64);
      unsigned long long m = gm[q] & (hi >= 64 ? ~0ull : ((1ull << hi) - 1ull)) & (~0ull << lo);
      if (q >= HESS_LQ && m) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the HBM rows' stores
      while (m) {  // uniform: the type's changed groups, one MFMA step each
        const int g0 = 64 * q + __builtin_ctzll(m);
        m &= m - 1ull;
        any = true;
        float4 n4;
        float jg[4], dr;
        if (q < HESS_LQ) {  // (static per unrolled slice: LDS or HBM rows)
          n4 = *reinterpret_cast<const float4*>(&E.NC[g0]);
#pragma unroll
          for (int mm = 0; mm < 4; mm++) jg[mm] = jlds(E, g0 + mm, col);  // slot 15 holds dC r
          dr = E.D[g0 + rk];
        } else {
          n4 = make_float4(*ovf_nc(E, g0), *ovf_nc(E, g0 + 1), *ovf_nc(E, g0 + 2), *ovf_nc(E, g0 + 3));
#pragma unroll
          for (int mm = 0; mm < 4; mm++) jg[mm] = ovf_j(E, g0 + mm)[col];
          dr = *ovf_d(E, g0 + rk);
        }
        const float own = fmaf(m_[0], jg[0], fmaf(m_[1], jg[1], fmaf(m_[2], jg[2], m_[3] * jg[3])));
        const float ncr = fmaf(m_[1], n4.y, fmaf(m_[2], n4.z, m_[3] * n4.w));
        const float s123 = fmaf(n4.y, jg[1], fmaf(n4.z, jg[2], n4.w * jg[3]));
        const float cpl = fmaf(ncr, jg[0], m_[0] * s123);
        const float b = fmaf(c15, own - fmaf(dr, own, cpl), fmaf(dr, own, cpl));
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(own, b, acc, 0, 0, 0);
      }
    }
    if (!any) continue;
    // stage into the round's next tile; a full round (or the last type) is gathered in type order
#pragma unroll
    for (int q = 0; q < 4; q++) G[16 * GST * nst + GST * (4 * rk + q) + col] = acc[q];
    tyslots |= t << (4 * nst);
    if (++nst == HESS_TILES) flush();
  }
  flush();
  return nd >= 0 ? gacc : 0.f;
}

// ---------------------------------------------------------------- Cholesky solves of H p = v
// H is 27 x 27 and block-structured: the arm block (9 dofs) and three cube blocks (6 dofs each),
// coupled only where a constraint row spans two blocks (cpl: 4 x 4 bit mask of block pairs).
// Lanes hold rows in the Newton lane layout (hrow[i] = H[dof][i], columns in dof order); the
// solution comes back in the same layout.

// Block form (no cube-cube coupling): every cube block factors inside its own DPP row, pivots
// broadcast with row_newbcast.  Without any coupling the four blocks factor in lockstep (9 pivot
// steps for all of H; cube rows meet identity rows on their dummy lanes 6..8).  With arm-cube
// coupling the arrow order holds: the three cube blocks first (6 lockstep steps), the arm lanes
// forming their coupling columns L[arm][cube] and the Schur complement of the arm block as each
// cube pivot passes (v_readlane of the cube rows' values), then the arm block (9 steps in row 0).
// Each pivot lane collects the column of L that the transposed solve needs (c[m] = L[m][own],
// block-relative; cx[i] = L[arm i][own] for a coupled cube lane) with one select per value it
// reads anyway, so no LDS transpose.
// block-relative row of the lane: its entries in its own block's columns (dummy lanes: identity)
DEV void block_row(const float* hrow, float* hb) {
  const int r = LANE >> 4, kk = LANE & 15;
  const bool valid = r != 0 ? kk < 6 : kk < 9;
  // 0/1 masks, not selects: a select chain over hrow[m + 6 r ...] is turned into a lane-indexed
  // load, which moves hrow to scratch
  const float m0 = r == 0 ? 1.f : 0.f, m1 = r == 1 ? 1.f : 0.f, m2 = r == 2 ? 1.f : 0.f, m3 = r == 3 ? 1.f : 0.f;
#pragma unroll
  for (int m = 0; m < 9; m++) {
    const float vv = m < 6 ? fmaf(m3, hrow[21 + m], fmaf(m2, hrow[15 + m], fmaf(m1, hrow[9 + m], m0 * hrow[m]))) : m0 * hrow[m];
    hb[m] = valid ? vv : (m == kk ? 1.f : 0.f);
  }
}
// no coupling at all: the four blocks factor in lockstep (9 pivot steps; cube rows meet identity
// rows on their dummy lanes 6..8), forward solve riding along
DEV float chol_block_free(const float* hrow, float v) {
  const int r = LANE >> 4, kk = LANE & 15;
  const bool valid = r != 0 ? kk < 6 : kk < 9;
  float hb[9], c[9], dinv[9];
  block_row(hrow, hb);
#pragma unroll
  for (int m = 0; m < 9; m++) c[m] = 0.f;
  float y = valid ? v : 0.f;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const float d = fmaxf(row_bcast(hb[k], k), 1e-20f);
    const float inv = __builtin_amdgcn_rsqf(d), sd = d * inv;
    dinv[k] = inv;
    const float l = kk == k ? sd : hb[k] * inv;  // lanes after the pivot: L[own][k]
    hb[k] = l;
    const float yk = row_bcast(y, k) * inv;
    y = kk == k ? yk : (kk > k ? fmaf(-l, yk, y) : y);
#pragma unroll
    for (int m = k + 1; m < 9; m++) {
      const float lm = row_bcast(l, m);
      hb[m] = fmaf(-lm, l, hb[m]);
      c[m] = kk == k ? lm : c[m];
    }
  }
#pragma unroll
  for (int k = 8; k >= 0; k--) {  // L' z = y
    const float zk = row_bcast(y, k) * dinv[k];
    y = kk == k ? zk : (kk < k ? fmaf(-c[k], zk, y) : y);
  }
  return valid ? y : 0.f;
}
// arm-cube coupling (a grasp), no cube-cube coupling: arrow order, the three cube blocks first (6
// lockstep steps) with the arm lanes forming their coupling columns L[arm][cube] and the arm
// block's Schur complement as each cube pivot passes (v_readlane of the cube rows' values), then
// the arm block (9 steps in row 0); the transposed solve in reverse order
DEV float chol_block_arm(const float* hrow, float v, int cpla) {
  const int L = LANE, r = L >> 4, kk = L & 15;
  const bool cube = r != 0;
  const bool valid = cube ? kk < 6 : kk < 9;
  float hb[9], c[9], cx[9], dinv[9], hx[18];
  block_row(hrow, hb);
#pragma unroll
  for (int m = 0; m < 9; m++) {
    c[m] = 0.f;
    cx[m] = 0.f;
  }
#pragma unroll
  for (int m = 0; m < 18; m++) hx[m] = hrow[9 + m];  // arm lanes: the coupling columns
  float y = valid ? v : 0.f;
#pragma unroll
  for (int k = 0; k < 6; k++) {  // the cube blocks (arm lanes: l = 0, untouched)
    const float d = fmaxf(row_bcast(hb[k], k), 1e-20f);
    const float inv = __builtin_amdgcn_rsqf(d), sd = d * inv;
    dinv[k] = inv;
    const float l = cube ? (kk == k ? sd : hb[k] * inv) : 0.f;
    hb[k] = cube ? l : hb[k];
    const float yk = row_bcast(y, k) * inv;
    y = cube ? (kk == k ? yk : (kk > k ? fmaf(-l, yk, y) : y)) : y;
#pragma unroll
    for (int m = k + 1; m < 6; m++) {
      const float lm = row_bcast(l, m);
      hb[m] = fmaf(-lm, l, hb[m]);
      c[m] = cube && kk == k ? lm : c[m];
    }
#pragma unroll
    for (int b = 1; b < 4; b++) {
      if (!((cpla >> b) & 1)) continue;  // uniform
      const float invb = readlane_f(inv, 16 * b);
      const float la = cube ? 0.f : hx[6 * (b - 1) + k] * invb;  // arm lane j: L[j][cube pivot]
      hx[6 * (b - 1) + k] = la;
#pragma unroll
      for (int m = k + 1; m < 6; m++) hx[6 * (b - 1) + m] = fmaf(-readlane_f(l, 16 * b + m), la, hx[6 * (b - 1) + m]);
#pragma unroll
      for (int i = 0; i < 9; i++) {  // Schur complement of the arm block
        const float li = readlane_f(la, i);
        hb[i] = fmaf(-li, la, hb[i]);
        cx[i] = L == 16 * b + k ? li : cx[i];
      }
      y = fmaf(-la, readlane_f(y, 16 * b + k), y);  // the cube pivot's y is final
    }
  }
  if (!cube) {
#pragma unroll
    for (int k = 0; k < 9; k++) {  // the arm block, row 0
      const float d = fmaxf(row_bcast(hb[k], k), 1e-20f);
      const float inv = __builtin_amdgcn_rsqf(d), sd = d * inv;
      dinv[k] = inv;
      const float l = kk == k ? sd : hb[k] * inv;
      hb[k] = l;
      const float yk = row_bcast(y, k) * inv;
      y = kk == k ? yk : (kk > k ? fmaf(-l, yk, y) : y);
#pragma unroll
      for (int m = k + 1; m < 9; m++) {
        const float lm = row_bcast(l, m);
        hb[m] = fmaf(-lm, l, hb[m]);
        c[m] = kk == k ? lm : c[m];
      }
    }
#pragma unroll
    for (int k = 8; k >= 0; k--) {  // L' z = y: the arm block (eliminated last) first
      const float zk = row_bcast(y, k) * dinv[k];
      y = kk == k ? zk : (kk < k ? fmaf(-c[k], zk, y) : y);
    }
  }
  // the coupled cube rows take the arm's final z: the arm lanes' y no longer changes here (cx = 0 off
  // the coupled cubes), so the 9 reads are independent of the updates and issue back to back
  float za[9];
#pragma unroll
  for (int i = 0; i < 9; i++) za[i] = readlane_f(y, i);
#pragma unroll
  for (int i = 0; i < 9; i++) y = fmaf(-cx[i], za[i], y);
#pragma unroll
  for (int k = 5; k >= 0; k--) {
    const float zk = row_bcast(y, k) * dinv[k];
    y = cube ? (kk == k ? zk : (kk < k ? fmaf(-c[k], zk, y) : y)) : y;
  }
  return valid ? y : 0.f;
}

// General arrow-ordered register Cholesky (any coupling, incl. cube-cube): pivots in the order
// cube 1, cube 2, cube 3, arm, and a pivot only updates the blocks it is coupled to (cpl plus the
// fill-in eliminating a block creates among the blocks after it); cross-lane values by
// v_readlane from the dof's lane, columns of L for the transposed solve through an LDS transpose.
DEV float chol_solve_arrow(EnvSh& E, const float* hrow, float v, int cpl) {
  const int j = newton_dof(LANE);
  const int pj = j < 0 ? 1000 : (j < 9 ? j + 18 : j - 9);  // elimination position of dof j
  float h[27], dinv[27];
#pragma unroll
  for (int i = 0; i < 27; i++) h[i] = hrow[i];
#pragma unroll
  for (int pi = 0; pi < 27; pi++) {
    const int p = pi < 18 ? pi + 9 : pi - 18;
    const int bp = p < 9 ? 0 : 1 + (p - 9) / 6;
    const float d = fmaxf(readlane_f(h[p], newton_lane(p)), 1e-20f);
    const float inv = __builtin_amdgcn_rsqf(d), sd = d * inv;  // one transcendental per pivot
    dinv[p] = inv;
    const float l = j == p ? sd : h[p] * inv;  // lanes after p: L[j][p]
    h[p] = l;
#pragma unroll
    for (int B = 0; B < 4; B++) {
      const int dB = B == 0 ? 0 : 9 + 6 * (B - 1), nB = B == 0 ? 9 : 6;
      const int lastpos = B == 0 ? 26 : 6 * B - 1;  // position of the block's last pivot
      if (lastpos <= pi) continue;                    // block already eliminated (static)
      if (B == bp || ((cpl >> (4 * bp + B)) & 1)) {
#pragma unroll
        for (int k = 0; k < nB; k++) {
          const int i = dB + k;
          const int qi = i < 9 ? i + 18 : i - 9;
          if (qi > pi) h[i] = fmaf(-readlane_f(l, newton_lane(i)), l, h[i]);
        }
      }
    }
    const bool last_of_block = pi == 5 || pi == 11 || pi == 17;
    if (last_of_block) {  // fill-in among the blocks eliminated later (cubes after bp, then arm)
#pragma unroll
      for (int x = 0; x < 4; x++)
#pragma unroll
        for (int yb = 0; yb < 4; yb++) {
          const bool later_x = x == 0 || x > bp, later_y = yb == 0 || yb > bp;
          if (x != yb && later_x && later_y && x != bp && yb != bp && ((cpl >> (4 * bp + x)) & 1) &&
              ((cpl >> (4 * bp + yb)) & 1))
            cpl |= 1 << (4 * x + yb);
        }
    }
  }
  float y = j >= 0 ? v : 0.f;
#pragma unroll
  for (int pi = 0; pi < 27; pi++) {  // L y = v in elimination order
    const int p = pi < 18 ? pi + 9 : pi - 18;
    const float yk = readlane_f(y, newton_lane(p)) * dinv[p];
    y = j == p ? yk : (pj > pi ? fmaf(-h[p], yk, y) : y);
  }
  const int jc = max(j, 0);
  if (j >= 0) {
#pragma unroll
    for (int m = 0; m < 27; m++) arrow_of(E)[27 * j + m] = h[m];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // (HBM: the stores complete before the reads)
  SYNC();
  float c[27];
#pragma unroll
  for (int k = 0; k < 27; k++) c[k] = arrow_of(E)[27 * k + jc];  // L[k][j]
#pragma unroll
  for (int pi = 26; pi >= 0; pi--) {  // L' z = y
    const int p = pi < 18 ? pi + 9 : pi - 18;
    const float zk = readlane_f(y, newton_lane(p)) * dinv[p];
    y = j == p ? zk : (pj < pi ? fmaf(-c[p], zk, y) : y);
  }
  SYNC();
  return j >= 0 ? y : 0.f;
}

// H^{-1} v: the block form unless two cubes are coupled (a cube resting on or pushing another)
DEV float chol_solve(EnvSh& E, const float* hrow, float v, int cpl) {
  float* stats = E.stats;
  CLK_DECL;
  const bool cube_cube = (cpl & 0x6AC0) != 0;  // bits 4 x + y with x, y in 1..3, x != y
  const float y = cube_cube ? chol_solve_arrow(E, hrow, v, cpl)
                            : ((cpl & 0xE) ? chol_block_arm(hrow, v, cpl & 0xE) : chol_block_free(hrow, v));
  // probe set 9: cycles of the uncoupled / arm-coupled / cube-cube solves; AUX3 counts the
  // arm-coupled solves + 1000 x the cube-cube ones
  PROBE(9, stats, cube_cube ? STAT_T_AUX1 : ((cpl & 0xE) ? STAT_T_AUX2 : STAT_T_AUX0));
  if (MMX_PROBE == 9 && LANE == 0) stats[STAT_T_AUX3] += cube_cube ? 1000.f : ((cpl & 0xE) ? 1.f : 0.f);
  return y;
}

// exit: 0 converged (gradient below tol), 1 no progress (step below 1e-9 with the gradient above
// tol: an fp32 stall), 2 iteration cap reached above tol
DEV int newton_wave(EnvSh& E, int max_iter, float tol, float& resid, int& exit, const float* mu_in) {
  float* stats = E.stats;
  CLK_DECL;
  const int nefc = E.nefc, nsingle = E.nsingle;
  // per owned row: D (1/R; the contact's common pyramid R), mu (from the row build, in registers) and
  // the edge coefficients
  float dd[RPL], mu[RPL];
#pragma unroll
  for (int q = 0; q < RPL; q++) {
    const int i = LANE + WG * q;
    dd[q] = i < nefc ? dget(E, i) : 0.f;
    mu[q] = i < nefc ? mu_in[q] : 0.f;
  }
  // start from the cheaper of the warm start and qacc_smooth (as MuJoCo does)
  float c_ws, c_s, ra[RPL], rs[RPL], mws, ms;
  cost2_wave(E, E.x, E.qacc_s, mu, dd, c_ws, c_s, ra, rs, mws, ms);
  const bool from_ws = c_ws < c_s;
  const int nd = newton_dof(LANE);  // the lane's dof in the Newton lane layout (-1: none)
  if (nd >= 0) E.x[nd] = from_ws ? E.x[nd] : E.qacc_s[nd];
  float mdx = from_ws ? mws : ms;  // (M (x - xs))_lane, kept current through the iterations
  float scale = nd >= 0 ? E.qfrc[nd] * E.qfrc[nd] : 0.f;
  scale = sqrtf(wave_sum(scale)) + 1.f;
  float rr[RPL], jp[RPL];  // basis-row residuals J x - aref and J p
#pragma unroll
  for (int q = 0; q < RPL; q++) {
    rr[q] = from_ws ? ra[q] : rs[q];
    jp[q] = 0.f;
  }
  int cpl = 0;  // block pairs that share constraint rows (uniform)
  for (int t = 0; t < NTYPE; t++)
    if (kTB1[t] != BLK_NONE && E.tbase[t + 1] > E.tbase[t]) cpl |= (1 << (4 * kTB0[t] + kTB1[t])) | (1 << (4 * kTB1[t] + kTB0[t]));
  cpl = __builtin_amdgcn_readfirstlane(cpl);
  SYNC();
  int it = 0;
  resid = 0.f;
  exit = 2;
  // Hessian rows and gradient persist across iterations: after the first full pass each later one
  // adds only the groups whose edge weights changed (hess_grad_delta); act holds the lane's edge
  // active bits (bit 2q: edge 0 of slice q, bit 2q + 1: edge 1) the current H was built from
  float hrow[32];
  float gpred = 0.f;  // g_old + a H_old p: the gradient at the new point before the weight change
  int act = 0;
  PROBE(1, stats, STAT_T_AUX3);
  for (; it < max_iter; it++) {
    // per group: the edge-weight matrix C (C_kk -> D, C_nk -> NC) and g = sum_e w_e r_e c_e
    // (-> slot 15), from the active edges of the current residuals; a contact's normal row
    // collects its edges' normal parts over the DPP quad.  Delta mode: the same with the change
    // of each edge's weight (+-D where its active state flipped, else 0), and a mask of the
    // groups holding a flipped edge.
    const bool delta = it > 0;  // uniform
    unsigned long long gm[HESS_NQ];
#pragma unroll
    for (int q = 0; q < HESS_NQ; q++) gm[q] = 0ull;
#pragma unroll
    for (int q = 0; q < RPL; q++) {
      if (WG * q >= nefc) break;  // uniform: no rows past this slice
      const int i = LANE + WG * q;
      const EdgeCoef ec = edge_coef(i, nefc, nsingle, mu[q]);
      const float rn = quad_first(rr[q]);
      const float e0 = fmaf(ec.a0, rn, ec.b0 * rr[q]), e1 = fmaf(ec.a1, rn, ec.b1 * rr[q]);
      const bool on0 = EQROW(q) || e0 < 0.f, on1 = e1 < 0.f;  // (missing edges: coefficients 0)
      const bool was0 = (act >> (2 * q)) & 1, was1 = (act >> (2 * q + 1)) & 1;
      act = (act & ~(3 << (2 * q))) | ((on0 ? 1 : 0) << (2 * q)) | ((on1 ? 2 : 0) << (2 * q));
      float w0 = on0 ? dd[q] : 0.f, w1 = on1 ? dd[q] : 0.f;
      if (delta) {
        w0 = on0 == was0 ? 0.f : (on0 ? dd[q] : -dd[q]);
        w1 = on1 == was1 ? 0.f : (on1 ? dd[q] : -dd[q]);
        if (q < HESS_NQ) {
          const unsigned long long bm = __ballot(w0 != 0.f || w1 != 0.f);
          gm[q < HESS_NQ ? q : 0] = (bm | (bm >> 1) | (bm >> 2) | (bm >> 3)) & 0x1111111111111111ull;
        }
      }
      const float ckk = fmaf(w0 * ec.b0, ec.b0, w1 * ec.b1 * ec.b1);
      const float cnk = fmaf(w0 * ec.a0, ec.b0, w1 * ec.a1 * ec.b1);
      const float gk = fmaf(w0 * e0, ec.b0, w1 * e1 * ec.b1);
      const float cnn = quad_sum(fmaf(w0 * ec.a0, ec.a0, w1 * ec.a1 * ec.a1));
      const float gn = quad_sum(fmaf(w0 * e0, ec.a0, w1 * e1 * ec.a1));
      const bool nrow = i >= nsingle && (i & 3) == 0;
      if (i < nefc) {
        jset(E, i, 15, nrow ? gn : gk);  // g for the gradient (the row's aref slot is dead after the setup)
        dset(E, i, nrow ? cnn : ckk);    // C diagonal (D itself is in registers since the setup)
        ncset(E, i, nrow ? 0.f : cnk);
      }
    }
    ovf_fence(nefc);
    SYNC();
    PROBE(1, stats, STAT_T_AUX0);
    float g;
    if (delta) {
      g = gpred + hess_grad_delta(E, hrow, gm);
    } else {
      g = hess_grad_mfma(E, nefc, hrow, mdx);
    }
    resid = sqrtf(wave_sum(g * g)) / scale;
    PROBE(1, stats, STAT_T_AUX1);
    if (resid < tol) {
      exit = 0;
      break;
    }
    const float pj = chol_solve(E, hrow, -g, cpl);
    if (nd >= 0) E.p[nd] = pj;
    SYNC();
    float hp = 0.f;  // (H p)_lane: the gradient's change per unit step while no edge changes state
#pragma unroll
    for (int m = 0; m < 27; m++) hp = fmaf(hrow[m], E.p[m], hp);
    PROBE(1, stats, STAT_T_AUX2);
    // exact line search on phi(a) = cost(x + a p): phi' is piecewise linear and increasing; per
    // owned row its (up to two) edges e(a) = e + a je
    float e0[RPL], e1[RPL], j0[RPL], j1[RPL];
#pragma unroll
    for (int q = 0; q < RPL; q++) {
      e0[q] = e1[q] = j0[q] = j1[q] = 0.f;
      jp[q] = 0.f;
      if (WG * q >= nefc) continue;  // uniform: the slice holds no row
      const int i = LANE + WG * q;
      jp[q] = i < nefc ? row_dot16(E, i, E.p) : 0.f;
      const EdgeCoef ec = edge_coef(i, nefc, nsingle, mu[q]);
      const float rn = quad_first(rr[q]), pn = quad_first(jp[q]);
      e0[q] = fmaf(ec.a0, rn, ec.b0 * rr[q]);
      e1[q] = fmaf(ec.a1, rn, ec.b1 * rr[q]);
      j0[q] = fmaf(ec.a0, pn, ec.b0 * jp[q]);
      j1[q] = fmaf(ec.a1, pn, ec.b1 * jp[q]);
    }
    PROBE(10, stats, STAT_T_AUX0);
    float c0 = 0.f, c1 = 0.f, mp = 0.f;
    if (nd >= 0) {
      mp = mass_mul(E, E.p);
      c0 = mp * (E.x[nd] - E.qacc_s[nd]);
      c1 = mp * pj;
    }
    c0 = wave_sum(c0);
    c1 = wave_sum(c1);
    PROBE(10, stats, STAT_T_AUX1);
    // the lane's edge active bits at step a, laid out like `act` (bit 2q: edge 0 of slice q, with
    // the equality row always on; bit 2q + 1: edge 1)
    auto act_at = [&](float a) {
      int b = 0;
#pragma unroll
      for (int q = 0; q < RPL; q++) {
        if (WG * q >= nefc) break;  // uniform
        b |= ((EQROW(q) || fmaf(a, j0[q], e0[q]) < 0.f) ? 1 : 0) << (2 * q);
        b |= (fmaf(a, j1[q], e1[q]) < 0.f ? 2 : 0) << (2 * q);
      }
      return b;
    };
    // phi' is linear on any interval over which no edge changes state (each edge is linear in a),
    // so a Newton root of phi' whose active set equals the set of the point it was taken from is
    // the minimiser and needs no confirming evaluation (which would only move it by rounding).  The
    // first evaluation, at the full step a = 1, always runs: it corrects the step length for the
    // fp32 error of the Cholesky solve p (accepting a = 1 unevaluated moved whole C3 episodes by
    // up to 7e-4 m against the solver at MuJoCo's tolerance).
    float alpha = 1.f, lo = 0.f, hi = 3e38f;
    int bcur = act_at(1.f);
    bool exact = false;  // (+1.0 % env steps/s in the A/B)
    for (int ls = 0; ls < 24 && !exact; ls++) {
      if (MMX_PROBE == 10 && LANE == 0) stats[STAT_T_AUX3] += 1.f;  // line-search steps
      float d1 = 0.f, d2 = 0.f;
#pragma unroll
      for (int q = 0; q < RPL; q++) {
        if (WG * q >= nefc) break;  // uniform
        const float a0 = fmaf(alpha, j0[q], e0[q]), a1 = fmaf(alpha, j1[q], e1[q]);
        const float s0 = EQROW(q) || a0 < 0.f ? dd[q] * j0[q] : 0.f;
        const float s1 = a1 < 0.f ? dd[q] * j1[q] : 0.f;
        d1 = fmaf(s0, a0, fmaf(s1, a1, d1));
        d2 = fmaf(s0, j0[q], fmaf(s1, j1[q], d2));
      }
      d1 = wave_sum(d1) + c0 + alpha * c1;
      d2 = wave_sum(d2) + c1;
      if (d1 < 0.f) lo = alpha;
      else hi = alpha;
      float na = alpha - d1 / fmaxf(d2, 1e-30f);
      const bool newton = na >= lo && na <= hi;
      if (!newton) na = hi < 3e38f ? 0.5f * (lo + hi) : 2.f * alpha;
      if (fabsf(na - alpha) <= 1e-6f * fabsf(alpha) + 1e-12f) {
        alpha = na;
        break;
      }
      const int bn = act_at(na);
      exact = newton && __ballot(bn != bcur) == 0ull;
      bcur = bn;
      alpha = na;
    }
    PROBE(1, stats, STAT_T_AUX3);
    PROBE(10, stats, STAT_T_AUX2);
    float stepn = 0.f;
    if (nd >= 0) {
      E.x[nd] += alpha * pj;
      stepn = alpha * alpha * pj * pj;
    }
    mdx = fmaf(alpha, mp, mdx);
    bool flip = false;  // an edge changed active state over the step
#pragma unroll
    for (int q = 0; q < RPL; q++) {
      if (WG * q >= nefc) break;  // uniform
      const float a0 = fmaf(alpha, j0[q], e0[q]), a1 = fmaf(alpha, j1[q], e1[q]);
      flip |= !EQROW(q) && ((a0 < 0.f) != (e0[q] < 0.f));
      flip |= (a1 < 0.f) != (e1[q] < 0.f);
      rr[q] = fmaf(alpha, jp[q], rr[q]);
    }
    SYNC();
    stepn = sqrtf(wave_sum(stepn));
    if (stepn < 1e-9f) {
      it++;
      exit = 1;
      break;
    }
    gpred = nd >= 0 ? fmaf(alpha, hp, g) : 0.f;
    if (__ballot(flip) == 0ull) {
      // same active set: H is unchanged, so g(x + a p) = g + a H p exactly; when that already
      // meets the tolerance the confirming Hessian pass is skipped
      const float rn = sqrtf(wave_sum(gpred * gpred)) / scale;
      if (rn < tol) {
        resid = rn;
        it++;
        exit = 0;
        break;
      }
    }
  }
  SYNC();
  return it;
}

#undef LANE
#define LANE ((int)(threadIdx.x & 63))
// ============================================================================ implicitfast + advance (wave)
// Arm: (M - h qDeriv) qacc = qfrc_smooth + qfrc_constraint with qfrc_constraint = M (x - qacc_s),
// qDeriv = -(damping + actuator kv where the force is unclamped), solved by a register Cholesky
// (rows in lanes 0..8); free bodies take the solver's qacc.  Then semi-implicit Euler and
// free-joint quaternion integration (one lane per cube).
DEV void integrate_wave(EnvSh& E) {
  const int d = min(LANE, 8);
  float arow[9];
  float rhs = E.qfrc[d];
#pragma unroll
  for (int c = 0; c < 9; c++) {
    arow[c] = E.M9[d][c];
    rhs += E.M9[d][c] * (E.x[c] - E.qacc_s[c]);
  }
#pragma unroll
  for (int c = 0; c < 9; c++) {
    float a = arow[c];
    if (c == d) {
      a += kDt * MMX_dof_damping[d];
      if (d < 7 && ((E.act_free >> d) & 1)) a -= kDt * MMX_act_bias[3 * d + 2];
    }
    if (((E.act_free >> 7) & 1) && d >= 7 && c >= 7) {  // tendon actuator kv on the finger pair
      const float bv = MMX_act_bias[3 * 7 + 2];
      a -= kDt * bv * MMX_tendon_coef[d - 7] * MMX_tendon_coef[c - 7];
    }
    arow[c] = a;
  }
  const float qa_arm = chol_solve_small<9>(arow, rhs, 1e-12f);
  bool bad = false;
  if (LANE < 27) {
    const float qa = LANE < 9 ? qa_arm : E.x[LANE];
    // (E.x stays: it is the next solve's warm start, MuJoCo's qacc_warmstart)
    const float v = E.qvel[LANE] + kDt * qa;
    E.qvel[LANE] = v;
    // |v| or |qacc| >= 1e10, Inf or NaN (MuJoCo's mj_checkVel / mj_checkAcc bound mjMAXVAL): an
    // integer test of the bits.  The values pass through an opaque register copy first: the device
    // code is built without NaN / Inf semantics (-ffinite-math-only), under which the compiler may
    // treat a NaN or Inf result of the fp ops above as impossible and fold a test it can see through
    // (ADVICE r04); behind the copy the test reads whatever bits the ALU produced.
    unsigned vb = __float_as_uint(v), qb = __float_as_uint(qa);
    asm volatile("" : "+v"(vb), "+v"(qb));
    bad = (vb & 0x7fffffffu) >= 0x501502F9u || (qb & 0x7fffffffu) >= 0x501502F9u;
    if (LANE < 9) E.qpos[LANE] += kDt * v;
  }
  if (__ballot(bad) != 0ull && LANE == 0) E.flags |= SHF_NAN;
  SYNC();
  if (LANE < 3) {
    const int c = LANE, qa = 9 + 7 * c, da = 9 + 6 * c;
    E.qpos[qa] += kDt * E.qvel[da];
    E.qpos[qa + 1] += kDt * E.qvel[da + 1];
    E.qpos[qa + 2] += kDt * E.qvel[da + 2];
    const V3 w = V3{E.qvel[da + 3], E.qvel[da + 4], E.qvel[da + 5]};
    const float wn = norm(w);
    Q4 q = qnormalize(Q4{E.qpos[qa + 3], E.qpos[qa + 4], E.qpos[qa + 5], E.qpos[qa + 6]});
    if (wn > 0.f) q = qmul(q, qaxisangle(w * (1.f / wn), wn * kDt));
    q = qnormalize(q);
    E.qpos[qa + 3] = q.w; E.qpos[qa + 4] = q.x; E.qpos[qa + 5] = q.y; E.qpos[qa + 6] = q.z;
  }
  SYNC();
}

// ============================================================================ implicitfast + advance (lane 0)

// ============================================================================ IK (lane 0)
DEV void orientation_error(const M3& Rc, V3& err) {  // controller.py:21-43, atan2 form for fp32
  float Em[9];
  const float T[9] = {0.f, 1.f, 0.f, 1.f, 0.f, 0.f, 0.f, 0.f, -1.f};
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) Em[3 * r + c] = T[3 * r] * Rc.m[3 * c] + T[3 * r + 1] * Rc.m[3 * c + 1] + T[3 * r + 2] * Rc.m[3 * c + 2];
  const V3 v = V3{Em[7] - Em[5], Em[2] - Em[6], Em[3] - Em[1]};
  const float cs = fminf(fmaxf((Em[0] + Em[4] + Em[8] - 1.f) * 0.5f, -1.f), 1.f);
  const float sn = 0.5f * norm(v);
  const float ang = atan2f(sn, cs);
  if (ang < 1e-6f || sn < 1e-12f) {
    err = V3{0.f, 0.f, 0.f};
    return;
  }
  err = v * (ang / (2.f * sn));
}

DEV void chol6_solve(const float* A, float* x) {
  float L[21];
#pragma unroll
  for (int k = 0; k < 21; k++) L[k] = A[k];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    float s = L[LT(j, j)];
#pragma unroll
    for (int k = 0; k < j; k++) s -= L[LT(j, k)] * L[LT(j, k)];
    const float d = sqrtf(fmaxf(s, 1e-20f)), inv = 1.f / d;
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

// DLS IK with nullspace bias on the stale kinematics cache -> ctrl[0:7]
DEV void ik_lane0(EnvSh& E) {
  const V3 tgt = V3{E.target[0], E.target[1], E.target[2]};
  const V3 ee = V3{kin_get(E, KIN_HAND_POS), kin_get(E, KIN_HAND_POS + 1), kin_get(E, KIN_HAND_POS + 2)};
  M3 Rc;
#pragma unroll
  for (int k = 0; k < 9; k++) Rc.m[k] = kin_get(E, KIN_HAND_MAT + k);
  float J[6][7];
#pragma unroll
  for (int d = 0; d < 7; d++) {
    const V3 ax = V3{kin_get(E, KIN_AXIS + 3 * d), kin_get(E, KIN_AXIS + 3 * d + 1), kin_get(E, KIN_AXIS + 3 * d + 2)};
    const V3 an = V3{kin_get(E, KIN_ANCHOR + 3 * d), kin_get(E, KIN_ANCHOR + 3 * d + 1), kin_get(E, KIN_ANCHOR + 3 * d + 2)};
    const V3 jp = cross(ax, ee - an);
    J[0][d] = jp.x; J[1][d] = jp.y; J[2][d] = jp.z;
    J[3][d] = ax.x; J[4][d] = ax.y; J[5][d] = ax.z;
  }
  V3 ori;
  orientation_error(Rc, ori);
  const float e6[6] = {tgt.x - ee.x, tgt.y - ee.y, tgt.z - ee.z, ori.x, ori.y, ori.z};
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
  float q[7], b[7];
#pragma unroll
  for (int k = 0; k < 7; k++) {
    q[k] = E.qpos[k];
    b[k] = 0.5f * (kHome[k] - q[k]);
  }
  float y[6], z[6];  // dq = J' A^-1 e + (b - J' A^-1 J b)
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
  float dq[7], n2 = 0.f;
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
    E.ctrl[k] = t;
  }
}

// Wave form of ik_lane0: J columns one lane per arm joint, the 6 x 6 DLS system one lane per row
// (register Cholesky), dq = b + J' A^{-1} (e - J b) with b the null-space pull toward home
// (= J' A^{-1} e + (I - J' A^{-1} J) b of controller.py:111-124).  Scratch: E.J (free here).
DEV void ik_wave(EnvSh& E) {
  float* W = scr_of(E) + SCR_IKW;  // J [6][8] at 0, b [8] at 48, e [8] at 56, u [8] at 64
  const V3 ee = V3{kin_get(E, KIN_HAND_POS), kin_get(E, KIN_HAND_POS + 1), kin_get(E, KIN_HAND_POS + 2)};
  if (LANE < 7) {
    const int d = LANE;
    const V3 ax = V3{kin_get(E, KIN_AXIS + 3 * d), kin_get(E, KIN_AXIS + 3 * d + 1), kin_get(E, KIN_AXIS + 3 * d + 2)};
    const V3 an = V3{kin_get(E, KIN_ANCHOR + 3 * d), kin_get(E, KIN_ANCHOR + 3 * d + 1), kin_get(E, KIN_ANCHOR + 3 * d + 2)};
    const V3 jp = cross(ax, ee - an);
    W[0 * 8 + d] = jp.x; W[1 * 8 + d] = jp.y; W[2 * 8 + d] = jp.z;
    W[3 * 8 + d] = ax.x; W[4 * 8 + d] = ax.y; W[5 * 8 + d] = ax.z;
    W[48 + d] = 0.5f * (kHome[d] - E.qpos[d]);
  } else if (LANE == 7) {
    M3 Rc;
#pragma unroll
    for (int k = 0; k < 9; k++) Rc.m[k] = kin_get(E, KIN_HAND_MAT + k);
    V3 ori;
    orientation_error(Rc, ori);
    W[56] = E.target[0] - ee.x; W[57] = E.target[1] - ee.y; W[58] = E.target[2] - ee.z;
    W[59] = ori.x; W[60] = ori.y; W[61] = ori.z;
  }
  SYNC();
  const int r = min(LANE, 5);
  float arow[6], rhs = W[56 + r];
#pragma unroll
  for (int c = 0; c < 6; c++) arow[c] = r == c ? 1e-3f : 0.f;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const float jr = W[8 * r + k];
#pragma unroll
    for (int c = 0; c < 6; c++) arow[c] = fmaf(jr, W[8 * c + k], arow[c]);
    rhs = fmaf(-jr, W[48 + k], rhs);
  }
  const float u = chol_solve_small<6>(arow, rhs, 1e-20f);
  if (LANE < 6) W[64 + LANE] = u;
  SYNC();
  float dq = 0.f;
  if (LANE < 7) {
    dq = W[48 + LANE];
#pragma unroll
    for (int rr = 0; rr < 6; rr++) dq = fmaf(W[8 * rr + LANE], W[64 + rr], dq);
  }
  const float nrm = sqrtf(wave_sum(dq * dq));
  const float scl = nrm > 5.0f ? 5.0f / nrm : 1.0f;
  if (LANE < 7) {
    float t = E.qpos[LANE] + dq * scl;
    const float lo = MMX_jnt_range[2 * LANE], hi = MMX_jnt_range[2 * LANE + 1];
    if (lo < hi) t = fminf(fmaxf(t, lo), hi);
    E.ctrl[LANE] = t;
  }
  SYNC();
}

// ============================================================================ one mj_step
DEV void mj_step_wave(int max_iter, float tol, EnvSh& E, float* con_dst) {
  float* stats = E.stats;
  CLK_DECL;
#if MMX_STEP_HELPER
  // the env wave and the helper wave (the kernel's helper loop mirrors these workgroup barriers)
  __syncthreads();  // C: the previous substep's state is in LDS; the helper runs the IK
  kinematics_wave(E);
  CLK(stats, STAT_T_KIN);
  __syncthreads();  // A: the kinematics; the helper runs the dynamics beside the broadphase
  collide_prune(E, false);
  __syncthreads();  // P: the class lists (and the dynamics); the helper takes the GJK / EPA pairs
  collide_pairs(E, false, 1);
  __syncthreads();  // Q: the helper's contacts (the rank sort orders them by key)
  collide_sort(E);
#else
  kinematics_wave(E);
  CLK(stats, STAT_T_KIN);
  dynamics_wave(E);
  CLK(stats, STAT_T_DYN);
  collide_wave(E, false);
#endif
  CLK(stats, STAT_T_COL);
  if (con_dst) store_contacts(con_dst, E);  // before the row build reuses contact fields
  float mu[RPL];  // the lane's rows' mu (LANE + 64 q), from the row build to the solver
  make_constraints_wave(E, mu);
  CLK(stats, STAT_T_CON);
  float resid = 0.f;
  int exit = 0;
  const int it = newton_wave(E, max_iter, tol, resid, exit, mu);
  CLK(stats, STAT_T_SOLVE);
  integrate_wave(E);
  CLK(stats, STAT_T_INT);
  if (LANE == 0) {
    stats[STAT_NEFC] += (float)E.nefc_mj;  // MuJoCo's rows (pyramid edges), not the stored basis rows
    stats[STAT_NCON] += (float)E.ncon;
    stats[STAT_SOLVER_ITER] += (float)it;
    stats[STAT_SUBSTEPS] += 1.f;
    stats[STAT_RESID] = fmaxf(stats[STAT_RESID], resid);
    // solver exits above tolerance, by cause (no progress in fp32 / iteration cap)
    stats[STAT_EXIT_STALL] += exit == 1 ? 1.f : 0.f;
    stats[STAT_EXIT_CAP] += exit == 2 ? 1.f : 0.f;
#ifdef MMX_PHASE_CLOCK
    if (MMX_PROBE == 12) {  // row / contact count distribution (sizes the LDS row capacity)
      stats[STAT_T_AUX0] = fmaxf(stats[STAT_T_AUX0], (float)E.nefc);  // stored (basis) rows
      stats[STAT_T_AUX1] = fmaxf(stats[STAT_T_AUX1], (float)E.ncon);
      stats[STAT_T_AUX2] += E.nefc > MMX_LDSEFC ? 1.f : 0.f;
      stats[STAT_T_AUX3] += E.nefc > 160 ? 1.f : 0.f;
    }
#endif
  }
  SYNC();
}

// ============================================================================ RNG (numpy PCG64)
struct Pcg {
  unsigned long long shi, slo, ihi, ilo;
};
DEV unsigned long long pcg_next64(Pcg& r) {
  const unsigned long long MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  const unsigned long long lo = r.slo * ML;
  unsigned long long hi = __umul64hi(r.slo, ML) + r.slo * MH + r.shi * ML;
  const unsigned long long nlo = lo + r.ilo;
  hi += r.ihi + (nlo < lo ? 1ull : 0ull);
  r.slo = nlo;
  r.shi = hi;
  const unsigned long long x = hi ^ nlo;
  const unsigned rot = (unsigned)(hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
DEV double pcg_double(Pcg& r) { return (double)(pcg_next64(r) >> 11) * (1.0 / 9007199254740992.0); }

// Generator.integers(high): buffered 32-bit Lemire on next_uint32 (low half first)
DEV int pcg_integers(Pcg& r, int& has32, unsigned& buf32, int high) {
  const unsigned rng = (unsigned)(high - 1);
  if (rng == 0) return 0;
  auto next32 = [&]() -> unsigned {
    if (has32) {
      has32 = 0;
      return buf32;
    }
    const unsigned long long v = pcg_next64(r);
    has32 = 1;
    buf32 = (unsigned)(v >> 32);
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

// ============================================================================ task layer (lane 0)
#define EPI(f) S.epi[(size_t)i * EPI_N + (f)]
#define EPF(f) S.epf[(size_t)i * EPF_N + (f)]

DEV V3 obj_pos(const EnvSh& E, int o) { return V3{E.qpos[9 + 7 * o], E.qpos[10 + 7 * o], E.qpos[11 + 7 * o]}; }
DEV V3 bin_pos(int bn) {
  const int b = kBinBody[bn];  // static bins: body origin = constant body pos (parent = world)
  return V3{MMX_body_pos[3 * b], MMX_body_pos[3 * b + 1], MMX_body_pos[3 * b + 2]};
}
DEV V3 hand_pos(const EnvSh& E) { return V3{kin_get(E, KIN_HAND_POS), kin_get(E, KIN_HAND_POS + 1), kin_get(E, KIN_HAND_POS + 2)}; }
DEV M3 hand_R(const EnvSh& E) {
  M3 R;
#pragma unroll
  for (int k = 0; k < 9; k++) R.m[k] = kin_get(E, KIN_HAND_MAT + k);
  return R;
}

DEV void project(V3 p, V3 cx, const M3& cR, float fovy_deg, float* out) {  // cameras.py:56-104
  const float t = tanf(fovy_deg * (3.14159265358979f / 180.f) * 0.5f);
  const V3 cc = mulT(cR, p - cx);
  float depth = cc.z;
  if (fabsf(depth) < 1e-6f) depth = 1e-6f;
  // px / S = f x / (depth S) + 1/2 with f = (S/2) / tan(fovy/2): independent of the image size
  out[0] = cc.x / (depth * 2.f * t) + 0.5f;
  out[1] = -cc.y / (depth * 2.f * t) + 0.5f;
}
DEV void camera_pose(int cam, V3 hx, const M3& hR, V3& cx, M3& cR) {
  const M3 lq = qmat(Q4{MMX_cam_quat[4 * cam], MMX_cam_quat[4 * cam + 1], MMX_cam_quat[4 * cam + 2], MMX_cam_quat[4 * cam + 3]});
  const V3 lp = V3{MMX_cam_pos[3 * cam], MMX_cam_pos[3 * cam + 1], MMX_cam_pos[3 * cam + 2]};
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

// numeric observation (gym_env.py:283-339, 85 floats) into E.obs
DEV void obs_lane0(const MMXState& S, int i, EnvSh& E) {
  const V3 hx = hand_pos(E);
  const M3 hR = hand_R(E);
  float* o = obs_of(E);
  const float g = E.ctrl[7] / 255.f;
  o[0] = hx.x; o[1] = hx.y; o[2] = hx.z; o[3] = g;
#pragma unroll
  for (int k = 0; k < 7; k++) o[4 + k] = E.qpos[k];
  float Ri[9];
#pragma unroll
  for (int k = 0; k < 9; k++) Ri[k] = EPF(EPF_TINIT + k);
  const V3 pi = V3{EPF(EPF_TINIT + 9), EPF(EPF_TINIT + 10), EPF(EPF_TINIT + 11)};
  float Rr[9];  // T_rel = inv(T_init) T_cur
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) Rr[3 * r + c] = Ri[r] * hR.m[c] + Ri[3 + r] * hR.m[3 + c] + Ri[6 + r] * hR.m[6 + c];
  const V3 dp = hx - pi;
  const V3 pr = V3{Ri[0] * dp.x + Ri[3] * dp.y + Ri[6] * dp.z, Ri[1] * dp.x + Ri[4] * dp.y + Ri[7] * dp.z,
                   Ri[2] * dp.x + Ri[5] * dp.y + Ri[8] * dp.z};
  for (int rel = 0; rel < 2; rel++) {
    const float* R = rel ? Rr : hR.m;
    const V3 p = rel ? pr : hx;
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
  const int ob = EPI(EPI_OBJ), bn = EPI(EPI_BIN);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    o[47 + k] = (k == bn) ? 1.f : 0.f;
    o[50 + k] = (k == ob) ? 1.f : 0.f;
  }
  const V3 kp[7] = {obj_pos(E, 0), obj_pos(E, 1), obj_pos(E, 2), bin_pos(0), bin_pos(1), bin_pos(2), hx};
  V3 cx;
  M3 cR;
  camera_pose(MMX_CAM_OVERHEAD, hx, hR, cx, cR);
#pragma unroll
  for (int k = 0; k < 7; k++) project(kp[k], cx, cR, MMX_cam_fovy[MMX_CAM_OVERHEAD], o + 53 + 2 * k);
  camera_pose(MMX_CAM_WRIST, hx, hR, cx, cR);
#pragma unroll
  for (int k = 0; k < 7; k++) project(kp[k], cx, cR, MMX_cam_fovy[MMX_CAM_WRIST], o + 67 + 2 * k);
#pragma unroll
  for (int k = 0; k < 4; k++) o[81 + k] = EPF(EPF_TGTKP + k);
}

// reset (gym_env.py:477-534) of the env in E; S.rng may just have been re-seeded by the host
DEV void reset_lane0(const MMXState& S, int i, EnvSh& E, int task_override) {
#pragma unroll
  for (int k = 0; k < 30; k++) E.qpos[k] = MMX_key_qpos[k];
#pragma unroll
  for (int k = 0; k < 27; k++) {
    E.qvel[k] = 0.f;
    E.x[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) E.ctrl[k] = MMX_key_ctrl[k];
  Pcg r = Pcg{S.rng[4 * (size_t)i], S.rng[4 * (size_t)i + 1], S.rng[4 * (size_t)i + 2], S.rng[4 * (size_t)i + 3]};
  int has32 = EPI(EPI_RNG_HAS32);
  unsigned buf32 = S.rng32[i];
  bool ok = true;  // the spawn sampling succeeded (or did not run)
  if (S.randomize) {  // randomization.py:70-98 (fp64 draws, numpy-identical stream)
    double xs[3] = {0, 0, 0}, ys[3] = {0, 0, 0};
    ok = false;
    for (int att = 0; att < 1000 && !ok; att++) {
      for (int k = 0; k < 3; k++) xs[k] = (double)S.spawn_x0 + ((double)S.spawn_x1 - (double)S.spawn_x0) * pcg_double(r);
      for (int k = 0; k < 3; k++) ys[k] = (double)S.spawn_y0 + ((double)S.spawn_y1 - (double)S.spawn_y0) * pcg_double(r);
      ok = true;
      for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++) {
          const double dx = xs[a] - xs[b], dy = ys[a] - ys[b];
          if (dx * dx + dy * dy < 0.08 * 0.08) ok = false;
        }
    }
    // exhausted (randomization.py:84-87 raises RuntimeError before touching qpos or drawing the task):
    // the cubes stay at the keyframe, the task draw is skipped (the stream stays the reference's), the
    // env's error bit and the sim's fault word are set; mmx_reset / mmx_synchronize turn the fault into
    // MMX_ESAMPLING and the facades into the reference's RuntimeError
    if (!ok) {
      EPI(EPI_ERROR) |= ERR_SAMPLING;
      atomicOr(S.fault, (int)ERR_SAMPLING);
    }
    for (int k = 0; k < 3 && ok; k++) {
      const int qa = 9 + 7 * k;
      E.qpos[qa] = (float)xs[k]; E.qpos[qa + 1] = (float)ys[k]; E.qpos[qa + 2] = 0.26f;
      E.qpos[qa + 3] = 1.f; E.qpos[qa + 4] = 0.f; E.qpos[qa + 5] = 0.f; E.qpos[qa + 6] = 0.f;
    }
  }
  kinematics_lane0(E);
  const V3 hx = hand_pos(E);
#pragma unroll
  for (int k = 0; k < 9; k++) EPF(EPF_TINIT + k) = kin_get(E, KIN_HAND_MAT + k);
  EPF(EPF_TINIT + 9) = hx.x; EPF(EPF_TINIT + 10) = hx.y; EPF(EPF_TINIT + 11) = hx.z;
  EPI(EPI_STEP) = 0;
  EPI(EPI_FLAGS) = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) EPF(EPF_HWM + k) = 0.f;
  EPF(EPF_EP_RETURN) = 0.f;
  int ob, bn;
  if (task_override >= 0) {
    ob = task_override >> 4;
    bn = task_override & 15;
  } else if (S.fixed_obj >= 0) {
    ob = S.fixed_obj;
    bn = S.fixed_bin;
  } else if (!ok) {  // (the reference raised before its task draw)
    ob = EPI(EPI_OBJ);
    bn = EPI(EPI_BIN);
  } else {
    const int idx = pcg_integers(r, has32, buf32, S.ntask);
    ob = S.task_obj[idx];
    bn = S.task_bin[idx];
  }
  S.rng[4 * (size_t)i] = r.shi;
  S.rng[4 * (size_t)i + 1] = r.slo;
  EPI(EPI_RNG_HAS32) = has32;
  S.rng32[i] = buf32;
  EPI(EPI_OBJ) = ob;
  EPI(EPI_BIN) = bn;
  V3 cx;
  M3 cR;
  camera_pose(MMX_CAM_OVERHEAD, hx, hand_R(E), cx, cR);
  float kp[2];
  project(obj_pos(E, ob), cx, cR, MMX_cam_fovy[MMX_CAM_OVERHEAD], kp);
  EPF(EPF_TGTKP) = kp[0]; EPF(EPF_TGTKP + 1) = kp[1];
  project(bin_pos(bn), cx, cR, MMX_cam_fovy[MMX_CAM_OVERHEAD], kp);
  EPF(EPF_TGTKP + 2) = kp[0]; EPF(EPF_TGTKP + 3) = kp[1];
  // FSM expert for this episode's task (scripts/generate_dataset.py:112-117)
  EPI(EPI_FSM_STATE) = 0;
  EPI(EPI_FSM_TASKIDX) = 0;
  EPI(EPI_FSM_SETTLE) = 0;
  EPI(EPI_FSM_GRIP) = 1;
  EPI(EPI_FSM_HASTGT) = 0;
  EPI(EPI_PHASES) = 1;  // IDLE
  EPI(EPI_EPISODES) += 1;
  obs_lane0(S, i, E);
}

// the target cube inside the target bin (the success test of gym_env.py:436-447)
DEV bool in_target_bin(const MMXState& S, int i, const EnvSh& E) {
  const V3 o = obj_pos(E, EPI(EPI_OBJ)), b = bin_pos(EPI(EPI_BIN));
  return sqrtf((o.x - b.x) * (o.x - b.x) + (o.y - b.y) * (o.y - b.y)) < 0.05f && o.z < b.z + 0.06f;
}

// reward (gym_env.py:352-470); returns reward, sets success (staged: all HWM >= 0.9)
DEV float reward_lane0(const MMXState& S, int i, const EnvSh& E, bool robot_obstacle, int& success) {
  const int ob = EPI(EPI_OBJ), bn = EPI(EPI_BIN);
  const V3 o = obj_pos(E, ob), b = bin_pos(bn), ee = hand_pos(E);
  const float xy = sqrtf((o.x - b.x) * (o.x - b.x) + (o.y - b.y) * (o.y - b.y));
  const bool succ = xy < 0.05f && o.z < b.z + 0.06f;
  if (S.reward_type == 1) {
    success = succ;
    return succ ? 1.f : 0.f;
  }
  if (S.reward_type == 2) {
    const float DM = 0.5f, GZ = 0.35f, LZ = 0.42f;
    int fl = EPI(EPI_FLAGS);
    const bool closed = E.ctrl[7] == 0.f;
    if (!(fl & FLAG_GRASPED) && o.z > GZ && closed) fl |= FLAG_GRASPED;
    if (!(fl & FLAG_LIFTED) && o.z > LZ && closed) fl |= FLAG_LIFTED;
    if (!(fl & FLAG_ABOVE) && (fl & FLAG_LIFTED) && xy < 0.06f) fl |= FLAG_ABOVE;
    if (!(fl & FLAG_PLACED) && succ) fl |= FLAG_PLACED;
    float rr[5];
    rr[0] = (fl & FLAG_GRASPED) ? 1.f : 1.f - fminf(norm(ee - o) / DM, 1.f);
    rr[1] = !(fl & FLAG_GRASPED) ? 0.f : ((fl & FLAG_LIFTED) ? 1.f : fmaxf(0.f, fminf((o.z - 0.30f) / (LZ - 0.30f), 1.f)));
    rr[2] = !(fl & FLAG_LIFTED) ? 0.f : ((fl & FLAG_ABOVE) ? 1.f : 1.f - fminf(xy / DM, 1.f));
    rr[3] = !(fl & FLAG_ABOVE) ? 0.f : ((fl & FLAG_PLACED) ? 1.f : 1.f - fmaxf(0.f, fminf((o.z - b.z) / 0.25f, 1.f)));
    const V3 ip = V3{EPF(EPF_TINIT + 9), EPF(EPF_TINIT + 10), EPF(EPF_TINIT + 11)};
    rr[4] = !(fl & FLAG_PLACED) ? 0.f : 1.f - fminf(norm(ee - ip) / DM, 1.f);
    fl |= FLAG_HWM_VALID;
    EPI(EPI_FLAGS) = fl;
    float sum = 0.f;
    bool all = true;
#pragma unroll
    for (int k = 0; k < 5; k++) {
      const float h = fmaxf(EPF(EPF_HWM + k), rr[k]);
      EPF(EPF_HWM + k) = h;
      sum += h;
      all &= h >= 0.90f;
    }
    if (robot_obstacle) {
      success = 1;
      return -1.f;
    }
    success = all;
    return sum / 5.f;
  }
  float rew = -norm(ee - o);
  if (o.z > 0.30f) rew += 2.f - norm(o - b);
  if (succ) rew += 10.f;
  success = succ;
  return rew;
}

// FSM expert plan(n) (pick_and_place.py:167-277) -> abs_pos action (generate_dataset.py:142-148).
// ee / object positions come from the last position stage (consistent after mj_forward).
// PickAndPlaceTask.plan(n) (pick_and_place.py:167-277) in branch-free form: every transition
// condition is evaluated, then each FSM field takes its new value through selects.  (Two
// switch-statement forms of this function, called from one-lane-per-env divergent code, were
// miscompiled: the LOWER_TO_BIN target's z and then the emitted action's z came out wrong.)
DEV void expert_plan(const MMXState& S, int i, V3 o, V3 ee, int n, float* act4) {
  const int s = EPI(EPI_FSM_STATE), ti = EPI(EPI_FSM_TASKIDX), settle = EPI(EPI_FSM_SETTLE);
  const int grip = EPI(EPI_FSM_GRIP), has = EPI(EPI_FSM_HASTGT);
  const V3 t = V3{EPF(EPF_FSM_TARGET), EPF(EPF_FSM_TARGET + 1), EPF(EPF_FSM_TARGET + 2)};
  const V3 te = V3{EPF(EPF_FSM_TRANSIT), EPF(EPF_FSM_TRANSIT + 1), EPF(EPF_FSM_TRANSIT + 2)};
  const V3 b = bin_pos(EPI(EPI_BIN));
  const bool r = norm(ee - t) < 0.02f;  // controller.reached (controller.py:139-145)
  const int sn = settle - n;
  const bool idle_done = s == 0 && ti >= 1;  // single-task FSM: one pick and place, then DONE
  const bool go1 = s == 0 && ti < 1;          // IDLE -> PRE_GRASP
  const bool go2 = s == 1 && r;               // PRE_GRASP -> GRASP
  const bool go3 = s == 2 && r;               // GRASP -> CLOSE_GRIPPER
  const bool go4 = s == 3 && sn <= 0;         // CLOSE_GRIPPER -> LIFT
  const bool go5 = s == 4 && r;               // LIFT -> MOVE_TO_BIN
  const V3 diff = te - t;                     // MOVE_TO_BIN: advance 0.001 n toward the transit end
  const float dist = norm(diff), step = 0.001f * n;
  const V3 tmove = dist > step ? t + diff * (step / dist) : te;
  const bool go6 = s == 5 && dist <= 0.02f;   // (pre-move distance) -> SETTLE_AT_BIN
  const bool go7 = s == 6 && sn <= 0;         // SETTLE_AT_BIN -> LOWER_TO_BIN
  const bool go8 = s == 7 && r;               // LOWER_TO_BIN -> RELEASE
  const bool go9 = s == 8 && sn <= 0;         // RELEASE -> RETREAT
  const bool go0 = s == 9 && r;               // RETREAT -> IDLE (next task)
  float tx = t.x, ty = t.y, tz = t.z;
  tx = go1 || go2 || go4 ? o.x : tx;
  ty = go1 || go2 || go4 ? o.y : ty;
  tz = go1 ? 0.44f : (go2 ? 0.36f : (go4 ? 0.55f : tz));
  tx = s == 5 ? tmove.x : tx;
  ty = s == 5 ? tmove.y : ty;
  tz = s == 5 ? tmove.z : tz;
  tx = go7 ? b.x : (go9 ? 0.f : tx);
  ty = go7 ? b.y : (go9 ? 0.3f : ty);
  tz = go7 ? 0.45f : (go9 ? 0.55f : tz);
  const int ns = idle_done ? 10 : go1 ? 1 : go2 ? 2 : go3 ? 3 : go4 ? 4 : go5 ? 5 : go6 ? 6 : go7 ? 7
               : go8 ? 8 : go9 ? 9 : go0 ? 0 : s;
  int nset = (s == 3 || s == 6 || s == 8) ? sn : settle;
  nset = go3 || go8 ? 150 : (go6 ? 100 : nset);
  const int ng = go1 || go8 ? 1 : (go3 ? 0 : grip);
  const int nhas = go1 ? 1 : has;
  EPI(EPI_FSM_STATE) = ns; EPI(EPI_FSM_TASKIDX) = go0 ? ti + 1 : ti; EPI(EPI_FSM_SETTLE) = nset;
  EPI(EPI_PHASES) |= 1 << ns;
  EPI(EPI_FSM_GRIP) = ng; EPI(EPI_FSM_HASTGT) = nhas;
  EPF(EPF_FSM_TARGET) = tx; EPF(EPF_FSM_TARGET + 1) = ty; EPF(EPF_FSM_TARGET + 2) = tz;
  if (go5) {
    EPF(EPF_FSM_TRANSIT) = b.x; EPF(EPF_FSM_TRANSIT + 1) = b.y; EPF(EPF_FSM_TRANSIT + 2) = 0.55f;
  }
  // before the first plan the reference has no target and commands the current EE position
  act4[0] = nhas ? tx : ee.x; act4[1] = nhas ? ty : ee.y; act4[2] = nhas ? tz : ee.z;
  act4[3] = ng ? 1.f : 0.f;
}

// decode_action (gym_env.py:252-281) + gripper command (gym_env.py:550-553)
DEV void decode_lane0(const MMXState& S, int i, EnvSh& E, const float* a) {
  V3 p = V3{a[0], a[1], a[2]};
  float g;
  switch (S.action_mode) {
    case 0: g = a[3]; break;
    case 1: g = a[7]; break;
    case 2: g = a[9]; break;
    default: {
      float R[9];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = EPF(EPF_TINIT + k);
      const V3 t = V3{EPF(EPF_TINIT + 9), EPF(EPF_TINIT + 10), EPF(EPF_TINIT + 11)};
      p = V3{R[0] * a[0] + R[1] * a[1] + R[2] * a[2] + t.x, R[3] * a[0] + R[4] * a[1] + R[5] * a[2] + t.y,
             R[6] * a[0] + R[7] * a[1] + R[8] * a[2] + t.z};
      g = S.action_mode == 3 ? a[7] : a[9];
    }
  }
  E.target[0] = p.x; E.target[1] = p.y; E.target[2] = p.z; E.target[3] = g;
  E.ctrl[7] = g > 0.5f ? 255.f : 0.f;
}

// ============================================================================ record I/O
DEV void load_env(const MMXState& S, int i, EnvSh& E) {
  if (LANE < 30) E.qpos[LANE] = S.qpos[(size_t)i * 30 + LANE];
  if (LANE < 27) {
    E.qvel[LANE] = S.qvel[(size_t)i * 27 + LANE];
    E.x[LANE] = S.qacc_ws[(size_t)i * 27 + LANE];
  }
  if (LANE < 8) E.ctrl[LANE] = S.ctrl[(size_t)i * 8 + LANE];
  if (LANE < KIN_N) kin_ref(E, LANE) = S.kin[(size_t)i * KIN_N + LANE];
  if (LANE < 4) E.target[LANE] = S.target[(size_t)i * 4 + LANE];
  if (LANE < STAT_N) E.stats[LANE] = S.stats[(size_t)i * STAT_N + LANE];
  if (LANE == 0) {
    E.ovf = S.efc_ovf + (size_t)i * MMX_OVF_F;
    E.flags = 0;
    E.ncon = 0;
    E.nefc = 0;
    E.nefc_mj = 0;
    E.ncand = -1;  // positions come from the record: rebuild the broadphase list
    E.cva = 3e38f;
    E.cwa = 3e38f;
  }
  SYNC();
}
DEV void store_env(const MMXState& S, int i, const EnvSh& E) {
  SYNC();
  if (LANE < 30) S.qpos[(size_t)i * 30 + LANE] = E.qpos[LANE];
  if (LANE < 27) {
    S.qvel[(size_t)i * 27 + LANE] = E.qvel[LANE];
    S.qacc_ws[(size_t)i * 27 + LANE] = E.x[LANE];
  }
  if (LANE < 8) S.ctrl[(size_t)i * 8 + LANE] = E.ctrl[LANE];
  if (LANE < KIN_N) S.kin[(size_t)i * KIN_N + LANE] = kin_get(E, LANE);
  if (LANE < 4) S.target[(size_t)i * 4 + LANE] = E.target[LANE];
  if (LANE < STAT_N) S.stats[(size_t)i * STAT_N + LANE] = E.stats[LANE];
  if (S.rpose)  // body poses for the camera renderer (mmx_render.hip)
    for (int k = LANE; k < NSLOT * 12; k += WG) {
      const int sl = k / 12, c = k % 12;
      S.rpose[(size_t)i * NSLOT * 12 + k] = c < 9 ? E.bR[sl][c] : E.bx[sl][c - 9];
    }
}
DEV void store_obs(const MMXState& S, int i, const EnvSh& E) {
  SYNC();
  for (int k = LANE; k < MMX_NOBS; k += WG) S.obs[(size_t)i * MMX_NOBS + k] = obs_of(E)[k];
}

// ============================================================================ kernels
// One env per 64-lane workgroup.  mmx_env_step_kernel (below) is the product path: a whole gym
// step per launch.  mmx_substep_kernel runs ONE substep per launch (the physics-level parity
// harness, mmx_physics_step, and a gym step split over 16 launches when mode has SS_GYM): the
// first launch decodes the action (or runs the FSM expert's plan(16)), the last runs the
// mj_forward position stage, reward, observation and autoreset (gym_env.py:536-581).
enum { SS_FIRST = 1, SS_LAST = 2, SS_EXPERT = 4, SS_IK = 8, SS_GYM = 16 };

DEV void fold_flags(const MMXState& S, int i, const EnvSh& E) {  // lane 0
  if (E.flags & SHF_CON_OVF) EPI(EPI_ERROR) |= ERR_CON_OVERFLOW;
  if (E.flags & SHF_EFC_OVF) EPI(EPI_ERROR) |= ERR_EFC_OVERFLOW;
  if (E.flags & SHF_NAN) EPI(EPI_ERROR) |= ERR_NAN;
}

// reward, termination and info of the current state (gym_env.py:562-573): writes the reward and
// the reward components, adds the reward to the episode return; lane 0
DEV void reward_outputs(const MMXState& S, int i, EnvSh& E, bool robot_obstacle, int& terminated, int& succ_flag) {
  int success = 0;
  const float r = reward_lane0(S, i, E, robot_obstacle, success);
  float* rc = S.reward_components + (size_t)i * 6;
  if (S.reward_type == 2) {
    terminated = (r < 0.f) || success;
    succ_flag = success && r >= 0.f;
    float sum = 0.f;
    for (int k = 0; k < 5; k++) {
      const float h = EPF(EPF_HWM + k) / 5.f;
      rc[1 + k] = h;
      sum += h;
    }
    rc[0] = sum;
  } else {
    terminated = success;
    succ_flag = success;
    for (int k = 0; k < 6; k++) rc[k] = 0.f;
  }
  S.reward[i] = r;
  EPF(EPF_EP_RETURN) += r;
}

// end of PickPlaceGymEnv.step: position stage, staged-penalty contact scan, reward, obs, autoreset
DEV void step_end(const MMXState& S, int i, EnvSh& E) {
  float* stats = E.stats;
  CLK_DECL;
  // mj_forward position stage (gym_env.py:560): kinematics + contacts for the staged penalty
  if (LANE == 0) {
    EPI(EPI_NCON) = E.ncon;
    EPI(EPI_NEFC) = E.nefc_mj;
  }
  kinematics_wave(E);
  if (S.reward_type == 2) collide_wave(E, true);
  if (LANE == 0) {
    EPI(EPI_STEP) += 1;
    int terminated, succ_flag;
    reward_outputs(S, i, E, (E.flags & SHF_ROBOT_OBST) != 0, terminated, succ_flag);
    const int truncated = EPI(EPI_STEP) >= S.max_episode_steps;
    S.done[3 * (size_t)i] = terminated;
    S.done[3 * (size_t)i + 1] = truncated;
    S.done[3 * (size_t)i + 2] = succ_flag;
    fold_flags(S, i, E);
    obs_lane0(S, i, E);
    // the FSM state only moves when the expert plans (mmx_expert_plan, or inside the rollout's
    // step launch), so host-action steps never see DONE: expert_plan + step autoresets exactly like
    // the fused rollout
    const bool fsm_done = EPI(EPI_FSM_STATE) == 10;
    const bool err = (EPI(EPI_ERROR) & ERR_NAN) != 0;
    if (S.autoreset && (terminated || truncated || err || fsm_done)) {
      if (err) {  // a diverged env ends its episode as truncated, not as a silent reset
        S.done[3 * (size_t)i + 1] = 1;
        S.done[3 * (size_t)i + 2] = 0;
        EPI(EPI_NERROR) += 1;
      } else {
        // an episode ended by the expert's FSM alone (no termination, no time limit) is reported as
        // truncated, so every autoreset carries a done flag (ended outside the MDP, like a time limit)
        if (!terminated) S.done[3 * (size_t)i + 1] = 1;
        EPI(EPI_NSUCCESS) += succ_flag;
        EPI(EPI_NPLACED) += in_target_bin(S, i, E) ? 1 : 0;
      }
      EPI(EPI_ERROR) = 0;
      reset_lane0(S, i, E, -1);
    }
    CLK(stats, STAT_T_END);
  }
  store_obs(S, i, E);
}

// The env-step kernel is built twice (mmx_step_l192.hip): MMX_STEP_ONLY compiles only it and its
// launcher, under names with the MMX_STEP_SUFFIX suffix; every other kernel comes from this file's
// own build.
#ifndef MMX_STEP_ONLY
extern "C" __global__ void __launch_bounds__(WG) mmx_substep_kernel(MMXState S, const float* action, int adim, int mode) {
  EnvSh& E = g_E;
  float* act = scr_of(E) + SCR_ACT;  // lane 0's decoded action (E.J is free before the substeps)
  const int i = blockIdx.x;
  if (i >= S.N) return;
  load_env(S, i, E);
  if ((mode & SS_FIRST) && (mode & SS_GYM) && LANE == 0) {
    if (mode & SS_EXPERT) expert_plan(S, i, obj_pos(E, EPI(EPI_OBJ)), hand_pos(E), MMX_NSUBSTEP, act);
    else
      for (int k = 0; k < adim && k < 12; k++) act[k] = action[(size_t)i * adim + k];
    decode_lane0(S, i, E, act);
  }
  SYNC();
  {
    float* stats = E.stats;
    CLK_DECL;
    if (mode & SS_IK) ik_wave(E);  // IK on the kinematics of the previous position stage
    SYNC();
    CLK(stats, STAT_T_IK);
  }
  mj_step_wave(S.solver_max_iter, S.solver_tol, E, (mode & SS_LAST) ? contacts_dst(S, i) : nullptr);
  if ((mode & SS_LAST) && (mode & SS_GYM)) {
    step_end(S, i, E);
  } else {
    if (LANE == 0) {
      fold_flags(S, i, E);
      if (mode & SS_LAST) {
        EPI(EPI_NCON) = E.ncon;
        EPI(EPI_NEFC) = E.nefc_mj;
      }
    }
  }
  store_env(S, i, E);
}

#endif  // MMX_STEP_ONLY

// One substep = IK + mj_step, kept out of line: nothing is hoisted across the 16 iterations of
// the env-step loop (hoisted invariants would pin registers for the whole kernel and serialise
// the phases' LDS loads); the price is the callee-saved register spill / fill per call.
//
// (Measured and removed: splitting one env over two waves, wave 1 running the collision prune and
// the plane / box-box pairs beside wave 0's dynamics and GJK/EPA: register-bound at 4 workgroups per
// CU, 1.11 M env steps/s against 1.21 M for one wave at 5 / CU, before the LDS shrink to 8 / CU.)
__device__ __attribute__((noinline)) void substep(int max_iter, float tol, float* con_dst) {
  EnvSh& E = g_E;
  float* stats = E.stats;
  CLK_DECL;
#if !MMX_STEP_HELPER  // (the helper wave's, beside the kinematics: mj_step_wave)
  ik_wave(E);  // IK on the kinematics left by the previous position stage
#endif
  CLK(stats, STAT_T_IK);
  mj_step_wave(max_iter, tol, E, con_dst);
}

// The whole PickPlaceGymEnv.step in ONE launch (product path): the 16 substeps loop inside the
// workgroup, so per-env cost variation averages out over the step instead of stretching 16
// separate launch tails (measured: one launch per substep ran 40 % slower).  With the on-device
// FSM expert (expert = 1) a launch may also run `nsteps` consecutive env steps of its env: each
// iteration is exactly one launch's body (record loaded, stepped, stored), so the trajectory is
// bit-identical to nsteps single-step launches, minus nsteps - 1 launch tails.
// The step's prologue (record load, FSM plan, action decode) and epilogue (position stage, reward,
// observation, autoreset, record store) are out of line like the substep: inlined into the fused
// step loop they kept ~280 VGPRs of hoisted values live across iterations (scratch spills).
__device__ __attribute__((noinline)) void step_begin(const MMXState& S, int i, const float* action, int adim,
                                                     int expert) {
  EnvSh& E = g_E;
  float* act = scr_of(E) + SCR_ACT;  // lane 0's decoded action (E.J is free before the substeps)
  load_env(S, i, E);
  if (LANE == 0) {
    if (expert) expert_plan(S, i, obj_pos(E, EPI(EPI_OBJ)), hand_pos(E), MMX_NSUBSTEP, act);
    else
      for (int k = 0; k < adim && k < 12; k++) act[k] = action[(size_t)i * adim + k];
    decode_lane0(S, i, E, act);
  }
  SYNC();
}
__device__ __attribute__((noinline)) void step_finish(const MMXState& S, int i) {
  EnvSh& E = g_E;
  step_end(S, i, E);
  store_env(S, i, E);
}
#ifdef MMX_PHASE_CLOCK
// Diagnostic build only: per FSM state of the env step (the state the step's action was planned
// in), the sums over env steps of the shader cycles of each phase (STAT_T_IK .. STAT_T_END), of
// the whole step, of the solver iterations / MuJoCo rows / contacts, the whole step's constant-rate
// wall clock (100 MHz ticks: the slot time an env step holds, and with FSMP_STEP the shader clock) and
// the env-step count (tools/gpu_probe.py fsm_profile).  Lane 0 of each env adds with global atomics.
enum { FSMP_PHASES = STAT_T_AUX3 - STAT_T_IK + 1, FSMP_STEP = FSMP_PHASES, FSMP_ITER, FSMP_NEFC, FSMP_NCON,
       FSMP_RT, FSMP_COUNT, FSMP_N };
#ifdef MMX_STEP_ONLY
static __device__ double g_fsm_prof[11 * FSMP_N];  // (this build's copy is not read out)
#else
__device__ double g_fsm_prof[11 * FSMP_N];
extern "C" hipError_t mmx_fsm_profile(double* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fsm_prof), sizeof(g_fsm_prof));
  if (e == hipSuccess && reset) {
    static double z[11 * FSMP_N];
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_fsm_prof), z, sizeof(z));
  }
  return e;
}
extern "C" int mmx_fsm_profile_fields() { return FSMP_N; }
#endif  // MMX_STEP_ONLY
#endif

// waves per SIMD the step kernel's register allocation is made for: 3 for the 128-row layout (168
// VGPRs: twelve envs per CU); 2 for the 192-row layout, the one for batches that leave CU slots empty
// (C2's 1024 envs are four per CU, each an env wave and its helper wave: eight waves per CU, 248 VGPRs;
// C2 1.29 -> 1.52 M, profiles/r06_ab_c2_helper.json; without the helper it ran one wave per SIMD)
#ifndef MMX_STEP_WAVES
#define MMX_STEP_WAVES (MMX_LDSEFC == 128 ? 3 : (MMX_STEP_HELPER ? 2 : 1))
#endif
#define MMX_STEP_THREADS (MMX_STEP_HELPER ? 128 : 64)  // the env's wave (+ the helper wave)
#ifndef MMX_STEP_SUFFIX
#define MMX_STEP_SUFFIX
#endif
#define MMX_CAT2_(a, b) a##b
#define MMX_CAT_(a, b) MMX_CAT2_(a, b)
#define MMX_STEP_SYM(name) MMX_CAT_(name, MMX_STEP_SUFFIX)
extern "C" __global__ void __launch_bounds__(MMX_STEP_THREADS) __attribute__((amdgpu_waves_per_eu(MMX_STEP_WAVES, MMX_STEP_WAVES)))
MMX_STEP_SYM(mmx_env_step_kernel)(MMXState S, const float* action, int adim, int expert, int base, int nsteps,
                                  const int* order) {
  // order (optional): the launch's envs in dispatch order, the grasp-carrying ones first (mmx_order_kernel)
  const int i = order ? order[blockIdx.x] : base + blockIdx.x;
  if (i >= S.N) return;
#if MMX_STEP_HELPER
  if (threadIdx.x >= 64) {  // the helper wave: the same workgroup barriers as the env's wave below
    for (int k = 0; k < nsteps; k++) {
      if (k) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        XSYNC();
      }
      XSYNC();  // step_begin's record load
      for (int sub = 0; sub < MMX_NSUBSTEP; sub++) {  // mj_step_wave's barriers C, A, P, Q
        __syncthreads();
        ik_wave(g_E);
        __syncthreads();
        dynamics_wave(g_E);
        __syncthreads();
        collide_pairs(g_E, false, 2);
        __syncthreads();
      }
    }
    return;
  }
#endif
  for (int k = 0; k < nsteps; k++) {
    if (k) {  // the previous step's record stores complete before this step reloads it
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      XSYNC();
    }
#ifdef MMX_PHASE_CLOCK
    const unsigned long long rt_step = wall_clock64();  // (the record load and the plan included)
#endif
    step_begin(S, i, action, adim, expert);
    XSYNC();
#ifdef MMX_PHASE_CLOCK
    float snap[FSMP_N];
    const int fsm = EPI(EPI_FSM_STATE);
    const unsigned long long t_step = clk_now();
    if (LANE == 0) {
      for (int j = 0; j < FSMP_PHASES; j++) snap[j] = g_E.stats[STAT_T_IK + j];
      snap[FSMP_ITER] = g_E.stats[STAT_SOLVER_ITER];
      snap[FSMP_NEFC] = g_E.stats[STAT_NEFC];
      snap[FSMP_NCON] = g_E.stats[STAT_NCON];
    }
#endif
    for (int sub = 0; sub < MMX_NSUBSTEP; sub++)
      substep(S.solver_max_iter, S.solver_tol, sub == MMX_NSUBSTEP - 1 ? contacts_dst(S, i) : nullptr);
#ifdef MMX_PHASE_CLOCK
    // (read before step_finish stores the record: an autoreset does not clear stats)
    if (LANE == 0) {
      double* g = g_fsm_prof + FSMP_N * min(max(fsm, 0), 10);
      for (int j = 0; j < FSMP_PHASES; j++) atomicAdd(g + j, (double)(g_E.stats[STAT_T_IK + j] - snap[j]));
      atomicAdd(g + FSMP_ITER, (double)(g_E.stats[STAT_SOLVER_ITER] - snap[FSMP_ITER]));
      atomicAdd(g + FSMP_NEFC, (double)(g_E.stats[STAT_NEFC] - snap[FSMP_NEFC]));
      atomicAdd(g + FSMP_NCON, (double)(g_E.stats[STAT_NCON] - snap[FSMP_NCON]));
    }
#endif
    step_finish(S, i);
#ifdef MMX_PHASE_CLOCK
    if (LANE == 0) {
      double* g = g_fsm_prof + FSMP_N * min(max(fsm, 0), 10);
      atomicAdd(g + STAT_T_END - STAT_T_IK, (double)(g_E.stats[STAT_T_END] - snap[STAT_T_END - STAT_T_IK]));
      atomicAdd(g + FSMP_STEP, (double)(clk_now() - t_step));
      atomicAdd(g + FSMP_RT, (double)(wall_clock64() - rt_step));
      atomicAdd(g + FSMP_COUNT, 1.0);
    }
#endif
  }
}

#ifndef MMX_STEP_ONLY
// mj_forward position stage only (kinematics -> IK cache) + observation refresh
extern "C" __global__ void __launch_bounds__(WG) mmx_forward_kernel(MMXState S) {
  EnvSh& E = g_E;
  const int i = blockIdx.x;
  if (i >= S.N) return;
  load_env(S, i, E);
  if (LANE == 0) {
    kinematics_lane0(E);
    obs_lane0(S, i, E);
  }
  store_env(S, i, E);
  store_obs(S, i, E);
}

extern "C" __global__ void __launch_bounds__(WG) mmx_reset_kernel(MMXState S, const unsigned char* mask, const int* task) {
  EnvSh& E = g_E;
  const int i = blockIdx.x;
  if (i >= S.N) return;
  if (mask && !mask[i]) return;
  load_env(S, i, E);
  if (LANE == 0) {
    EPI(EPI_ERROR) = 0;
    reset_lane0(S, i, E, task ? task[i] : -1);
    S.done[3 * (size_t)i] = 0;
    S.done[3 * (size_t)i + 1] = 0;
    S.done[3 * (size_t)i + 2] = 0;
  }
  store_env(S, i, E);
  store_obs(S, i, E);
}

// Per-physics-step expert loop (main.py:65-91, tests/test_pick_and_place.py:147-166): n x
// (PickAndPlaceTask.update() = plan(1) + _actuate() (pick_and_place.py:279-304) ; mj_step).  plan
// reads data.xpos as the previous mj_step left it: the hand pose and cube positions of
// the last position stage (the kin cache), not the integrated qpos.  No gym bookkeeping.
extern "C" __global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2, 2)))
mmx_expert_physics_kernel(MMXState S, int n) {
  EnvSh& E = g_E;
  const int i = blockIdx.x;
  if (i >= S.N) return;
  load_env(S, i, E);
  for (int k = 0; k < n; k++) {
    if (LANE == 0) {
      float act[4];
      const int ob = EPI(EPI_OBJ);
      expert_plan(S, i, V3{E.bx[11 + ob][0], E.bx[11 + ob][1], E.bx[11 + ob][2]}, hand_pos(E), 1, act);
      // _actuate: gripper open / closed, then IK toward the target once there is one
      E.ctrl[7] = EPI(EPI_FSM_GRIP) ? 255.f : 0.f;
      E.target[0] = EPF(EPF_FSM_TARGET);
      E.target[1] = EPF(EPF_FSM_TARGET + 1);
      E.target[2] = EPF(EPF_FSM_TARGET + 2);
      E.target[3] = EPI(EPI_FSM_HASTGT) ? act[3] : -1.f;  // < 0: no target yet, no IK
    }
    SYNC();
    if (E.target[3] >= 0.f) ik_wave(E);
    SYNC();
    mj_step_wave(S.solver_max_iter, S.solver_tol, E, k == n - 1 ? contacts_dst(S, i) : nullptr);
  }
  if (LANE == 0) fold_flags(S, i, E);
  store_env(S, i, E);
}

// Reward-layer parity harness (gym_env.py:341-470, 562-573): the reward of every env at the given
// object / EE positions and gripper command, with the step's contacts given as geom-id pairs (-1
// ends a list; robot x obstacle pairs are classified by the same geom classes as the collision
// scan).  Updates the sticky flags / high-water marks like a step; writes reward, reward
// components, terminated and success.
extern "C" __global__ void __launch_bounds__(WG) mmx_reward_kernel(MMXState S, const float* obj, const float* ee,
                                                                  const float* ctrl7, const int* pairs, int max_pairs) {
  EnvSh& E = g_E;
  const int i = blockIdx.x;
  if (i >= S.N || LANE != 0) return;
  const int ob = EPI(EPI_OBJ);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    E.qpos[9 + 7 * ob + k] = obj[3 * (size_t)i + k];
    kin_ref(E, KIN_HAND_POS + k) = ee[3 * (size_t)i + k];
  }
  E.ctrl[7] = ctrl7[i];
  bool ro = false;
  for (int p = 0; p < max_pairs; p++) {
    const int g1 = pairs[2 * ((size_t)i * max_pairs + p)], g2 = pairs[2 * ((size_t)i * max_pairs + p) + 1];
    if (g1 < 0 || g2 < 0 || g1 >= MMX_NGEOM || g2 >= MMX_NGEOM) break;
    const int c1 = MMX_geom_class[g1], c2 = MMX_geom_class[g2];
    ro |= (c1 == 1 && c2 == 2) || (c1 == 2 && c2 == 1);
  }
  int terminated, succ_flag;
  reward_outputs(S, i, E, ro, terminated, succ_flag);
  S.done[3 * (size_t)i] = terminated;
  S.done[3 * (size_t)i + 1] = 0;
  S.done[3 * (size_t)i + 2] = succ_flag;
}

// FSM expert plan(n) for every env -> abs_pos action [N][4] (one lane per env: tiny)
extern "C" __global__ void __launch_bounds__(WG) mmx_expert_kernel(MMXState S, int n, float* action) {
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= S.N) return;
  const int ob = EPI(EPI_OBJ);
  const float* q = S.qpos + (size_t)i * 30;
  const float* kn = S.kin + (size_t)i * KIN_N;
  float a[4];
  expert_plan(S, i, V3{q[9 + 7 * ob], q[10 + 7 * ob], q[11 + 7 * ob]}, V3{kn[0], kn[1], kn[2]}, n, a);
  if (action)
    for (int k = 0; k < 4; k++) action[(size_t)i * 4 + k] = a[k];
}

// ============================================================================ episode queue
// Device-side slot reassignment of the dataset loop (scripts/generate_dataset.py:140-198 runs one
// episode per env; here E episodes stream through the N env slots, mmx_queue_advance).  One
// workgroup scans the slots in order and hands episodes next, next + 1, ... to the slots that need
// one (no episode yet, or their FSM reached DONE = state 10, pick_and_place.py:167-277), staging the
// reset: mask, task and the episode's PCG64(SeedSequence(seed_e)) state (generate_dataset.py:263-277).
// The slot -> episode order is the host loop's (finished slots in ascending order).
struct MMXQueue {
  int* slot;                      // [N] episode running in the slot, -1: none
  int* next;                      // [1] next episode to hand out
  int n_ep;                       // E
  const unsigned long long* rng;  // [E][4] initial PCG64 state per episode, or null (no reseed)
  const int* task;                // [E] obj << 4 | bin, -1: the env's own draw
};
#define QWG 1024
extern "C" __global__ void __launch_bounds__(QWG) mmx_queue_kernel(MMXState S, MMXQueue Q, unsigned char* mask, int* task,
                                                                  int* slot_out, int* fin_out) {
  __shared__ int scan[QWG];
  const int t = threadIdx.x, N = S.N;
  const int c = (N + QWG - 1) / QWG, s0 = min(N, t * c), s1 = min(N, s0 + c);  // contiguous slots per thread
  int cnt = 0;
  for (int s = s0; s < s1; s++) cnt += Q.slot[s] < 0 || S.epi[(size_t)s * EPI_N + EPI_FSM_STATE] == 10;
  scan[t] = cnt;
  __syncthreads();
  for (int off = 1; off < QWG; off <<= 1) {  // inclusive scan of the per-thread counts
    const int v = t >= off ? scan[t - off] : 0;
    __syncthreads();
    scan[t] += v;
    __syncthreads();
  }
  const int base = *Q.next;
  int e = base + scan[t] - cnt;
  for (int s = s0; s < s1; s++) {
    const int cur = Q.slot[s];
    const bool ended = cur >= 0 && S.epi[(size_t)s * EPI_N + EPI_FSM_STATE] == 10;
    int now = cur;
    unsigned char m = 0;
    if (cur < 0 || ended) {
      now = e < Q.n_ep ? e : -1;
      if (now >= 0) {
        m = 1;
        task[s] = Q.task[now];
        if (Q.rng) {
#pragma unroll
          for (int k = 0; k < 4; k++) S.rng[4 * (size_t)s + k] = Q.rng[4 * (size_t)now + k];
          S.epi[(size_t)s * EPI_N + EPI_RNG_HAS32] = 0;
        }
      }
      e++;
      Q.slot[s] = now;
    }
    mask[s] = m;
    if (slot_out) slot_out[s] = now;
    if (fin_out) fin_out[s] = ended ? cur : -1;
  }
  __syncthreads();
  if (t == 0) *Q.next = min(Q.n_ep, base + scan[QWG - 1]);
}

// Dispatch order of an env range for the step kernel, longest first.  An env step's cycles follow its
// FSM phase (profiles/r06_fsm_profile.json, cycles per env step at twelve per CU): lift / move to bin /
// lower to bin ~2.5 M, close gripper / settle ~2.2 M, release / retreat ~1.7 M, the rest ~1.4-1.5 M.  A counting
// sort over those four classes (refined by rows, below) puts the long ones at the front of order[],
// so the launch's last workgroups are short ones (C3 +2.0 %, C5 +3.8 %).  One workgroup of any size (a single
// wave beside running step launches: it then fits a CU the step kernel fills); the order within a
// class is whatever the atomics give (the envs are independent: results do not depend on it).
DEV int step_cost_class(int fsm_state) {
  switch (fsm_state) {
    case 4: case 5: case 7: return 0;  // lift, move to bin, lower to bin (the object held)
    case 3: case 6: return 1;          // close gripper, settle at bin
    case 8: case 9: return 2;          // release, retreat
    default: return 3;
  }
}
// the sort key: the phase class first, then within a class the env's constraint rows of its last
// substep (MuJoCo's count, EPI_NEFC) in 32-row steps, more rows first (C5 +1.0 %, C3 unchanged; rows
// alone: C5 +0.5 %, C3 -1.1 %: a fused launch's steps follow the phase more than the last rows)
#define ORD_NB 24
DEV int step_order_bucket(const MMXState& S, int i) {
  const int c = step_cost_class(S.epi[(size_t)i * EPI_N + EPI_FSM_STATE]);
  return 6 * c + 5 - min(5, S.epi[(size_t)i * EPI_N + EPI_NEFC] >> 5);
}
extern "C" __global__ void __launch_bounds__(1024) mmx_order_kernel(MMXState S, int base, int count, int* order) {
  __shared__ int cnt[ORD_NB], off[ORD_NB];
  if (threadIdx.x < ORD_NB) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int k = threadIdx.x; k < count; k += blockDim.x) atomicAdd(&cnt[step_order_bucket(S, base + k)], 1);
  __syncthreads();
  if (threadIdx.x == 0)
    for (int b = 0, o = 0; b < ORD_NB; b++) off[b] = o, o += cnt[b];
  __syncthreads();
  for (int k = threadIdx.x; k < count; k += blockDim.x) {
    const int i = base + k;
    order[atomicAdd(&off[step_order_bucket(S, i)], 1)] = i;
  }
}

// =========================================================================== host launchers
// threads: 1024 when the launch has the GPU to itself, 64 beside other streams' step launches (a
// 1,024-lane workgroup waited ~0.35 ms for a CU to drain there: profiles/archive/r05_c3_kernel_stats.csv)
extern "C" hipError_t mmx_launch_order(const MMXState* S, int base, int count, int* order, int threads, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  if (threads != 64 && threads != 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mmx_order_kernel, dim3(1), dim3(threads), 0, st, *S, base, count, order);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_queue(const MMXState* S, int* slot, int* next, int n_ep, const unsigned long long* rng,
                                       const int* qtask, unsigned char* mask, int* task, int* slot_out, int* fin_out,
                                       hipStream_t st) {
  const MMXQueue Q{slot, next, n_ep, rng, qtask};
  hipLaunchKernelGGL(mmx_queue_kernel, dim3(1), dim3(QWG), 0, st, *S, Q, mask, task, slot_out, fin_out);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_reset(const MMXState* S, const unsigned char* mask, const int* task, hipStream_t st) {
  hipLaunchKernelGGL(mmx_reset_kernel, dim3(S->N), dim3(WG), 0, st, *S, mask, task);
  return hipGetLastError();
}
#endif  // MMX_STEP_ONLY
// Occupancy probe (diagnostics only, never set by the product): MMX_LDS_PAD bytes of dynamic LDS
// per step-kernel workgroup lower the envs per CU (tools/occupancy_probe.sh).
static size_t step_lds_pad() {
  static const size_t pad = [] {
    const char* v = std::getenv("MMX_LDS_PAD");
    return v ? (size_t)std::max(0, std::atoi(v)) : (size_t)0;
  }();
  return pad;
}
// envs [base, base+count): independent env ranges may run on separate streams
extern "C" hipError_t MMX_STEP_SYM(mmx_launch_step)(const MMXState* S, const float* action, int adim, int expert, int base,
                                                    int count, int nsteps, hipStream_t st, const int* order) {
  if (count <= 0 || nsteps <= 0) return hipSuccess;
  if (nsteps > 1 && !expert) return hipErrorInvalidValue;  // host actions: one env step per launch
  hipLaunchKernelGGL(MMX_STEP_SYM(mmx_env_step_kernel), dim3(count), dim3(MMX_STEP_THREADS), step_lds_pad(), st, *S, action, adim, expert, base,
                     nsteps, order);
  return hipGetLastError();
}
#ifndef MMX_STEP_ONLY
extern "C" hipError_t mmx_launch_expert(const MMXState* S, int n, float* action, hipStream_t st) {
  hipLaunchKernelGGL(mmx_expert_kernel, dim3((S->N + WG - 1) / WG), dim3(WG), 0, st, *S, n, action);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_physics(const MMXState* S, int n, int with_ik, hipStream_t st) {
  for (int sub = 0; sub < n; sub++) {
    const int mode = (with_ik ? SS_IK : 0) | (sub == n - 1 ? SS_LAST : 0);
    hipLaunchKernelGGL(mmx_substep_kernel, dim3(S->N), dim3(WG), 0, st, *S, nullptr, 0, mode);
  }
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_expert_physics(const MMXState* S, int n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(mmx_expert_physics_kernel, dim3(S->N), dim3(WG), 0, st, *S, n);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_reward(const MMXState* S, const float* obj, const float* ee, const float* ctrl7,
                                        const int* pairs, int max_pairs, hipStream_t st) {
  hipLaunchKernelGGL(mmx_reward_kernel, dim3(S->N), dim3(WG), 0, st, *S, obj, ee, ctrl7, pairs, max_pairs);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_forward(const MMXState* S, hipStream_t st) {
  hipLaunchKernelGGL(mmx_forward_kernel, dim3(S->N), dim3(WG), 0, st, *S);
  return hipGetLastError();
}
#endif  // MMX_STEP_ONLY
