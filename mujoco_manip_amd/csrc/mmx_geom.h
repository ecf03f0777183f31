// Narrowphase geometry for the MI355X kernels (fp32, one geom pair per lane).
//
// Restates MuJoCo's collision functions for the pair classes of this scene:
// plane-box (corners), plane-convex (support point), box-box (separating-axis test with
// reference-face clipping, up to 8 points), and the general convex path GJK + EPA (one contact,
// as MuJoCo 3.x nativeccd without multiccd).  Contacts are emitted through Sink::add(g1, g2,
// dist, pos, normal) with the normal pointing from geom1 to geom2.
#ifndef MMX_GEOM_H
#define MMX_GEOM_H
#include "mmx_device.h"
#include "mmx_state.h"
#include "mmx_clock.h"

enum { GT_PLANE = 0, GT_CYL = 5, GT_BOX = 6, GT_MESH = 7 };

struct Geom {
  V3 x;
  M3 R;
  int type, g;
};

DEV V3 support(const Geom& G, V3 dir) {
  V3 dl = mulT(G.R, dir), sl;
  const int g = G.g;
  if (G.type == GT_BOX) {
    sl = V3{dl.x >= 0.f ? MMX_geom_size[3 * g] : -MMX_geom_size[3 * g],
            dl.y >= 0.f ? MMX_geom_size[3 * g + 1] : -MMX_geom_size[3 * g + 1],
            dl.z >= 0.f ? MMX_geom_size[3 * g + 2] : -MMX_geom_size[3 * g + 2]};
  } else if (G.type == GT_CYL) {
    const float r = MMX_geom_size[3 * g], hh = MMX_geom_size[3 * g + 1];
    const float n = sqrtf(dl.x * dl.x + dl.y * dl.y);
    sl = n > 1e-12f ? V3{r * dl.x / n, r * dl.y / n, 0.f} : V3{r, 0.f, 0.f};
    sl.z = dl.z >= 0.f ? hh : -hh;
  } else {  // convex hull of a collision mesh (brute-force support over hull vertices)
    const int m = MMX_geom_mesh[g];
    const int a = MMX_mesh_vertadr[m], nvert = MMX_mesh_vertnum[m];
    float best = -3.0e38f;
    int bi = a;
    for (int v = a; v < a + nvert; v++) {
      const float s = MMX_mesh_vert[3 * v] * dl.x + MMX_mesh_vert[3 * v + 1] * dl.y + MMX_mesh_vert[3 * v + 2] * dl.z;
      if (s > best) {
        best = s;
        bi = v;
      }
    }
    sl = V3{MMX_mesh_vert[3 * bi], MMX_mesh_vert[3 * bi + 1], MMX_mesh_vert[3 * bi + 2]};
  }
  return G.x + mul(G.R, sl);
}

// Oriented-box overlap on the six face axes (a conservative prune), in the relative-rotation
// form: R = A'B, t = A'd, u = B'd, so each axis costs a 3-term sum instead of two projections.
DEV bool obb_overlap(const Geom& A, const Geom& B, V3 ha, V3 hb) {
  const V3 d = B.x - A.x;
  float Rm[3][3], aR[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      Rm[i][j] = dot(col(A.R, i), col(B.R, j));
      aR[i][j] = fabsf(Rm[i][j]);
    }
  const float hA[3] = {ha.x, ha.y, ha.z}, hB[3] = {hb.x, hb.y, hb.z};
  bool sep = false;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float t = dot(d, col(A.R, i));
    sep |= fabsf(t) > hA[i] + hB[0] * aR[i][0] + hB[1] * aR[i][1] + hB[2] * aR[i][2];
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const float u = dot(d, col(B.R, j));
    sep |= fabsf(u) > hB[j] + hA[0] * aR[0][j] + hA[1] * aR[1][j] + hA[2] * aR[2][j];
  }
  (void)Rm;
  return !sep;
}

template <class Sink>
DEV void plane_box(Sink& cs, const Geom& P, const Geom& B, V3 hb) {
  const V3 nz = col(P.R, 2);
  const float h[3] = {hb.x, hb.y, hb.z};
  // penetrating corners compacted in corner order, then a selection sort of the 4 deepest, as
  // the oracle does it; every index is static (select chains), so nothing lands in scratch
  float cd[8];
  V3 cp[8];
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    cd[k] = 0.f;
    cp[k] = V3{0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const V3 l = V3{(k & 1) ? h[0] : -h[0], (k & 2) ? h[1] : -h[1], (k & 4) ? h[2] : -h[2]};
    const V3 w = B.x + mul(B.R, l);
    const float d = dot(w - P.x, nz);
    if (d <= 0.f) {
      const V3 pw = w - nz * (0.5f * d);
#pragma unroll
      for (int q = 0; q <= k; q++)
        if (q == cnt) {
          cd[q] = d;
          cp[q] = pw;
        }
      cnt++;
    }
  }
  const int base = cs.reserve(cnt < 4 ? cnt : 4);  // one slot reservation for the pair
#pragma unroll
  for (int k = 0; k < 4; k++) {  // keep the 4 deepest corners
    if (k >= cnt) break;
    int bi = k;
    float bd = cd[k];
    V3 bp = cp[k];
#pragma unroll
    for (int m = k + 1; m < 8; m++)
      if (m < cnt && cd[m] < bd) {
        bi = m;
        bd = cd[m];
        bp = cp[m];
      }
    const float td = cd[k];
    const V3 tp = cp[k];
    cd[k] = bd;
    cp[k] = bp;
#pragma unroll
    for (int m = k + 1; m < 8; m++)
      if (m == bi) {
        cd[m] = td;
        cp[m] = tp;
      }
    cs.put(base + k, P.g, B.g, cd[k], cp[k], nz);
  }
}

template <class Sink>
DEV void plane_convex(Sink& cs, const Geom& P, const Geom& C) {
  const V3 nz = col(P.R, 2);
  const V3 s = support(C, -nz);
  const float d = dot(s - P.x, nz);
  if (d <= 0.f) cs.add(P.g, C.g, d, s - nz * (0.5f * d), nz);
}

DEV int clip_poly(const V3* in, int n, V3* out, V3 a, float b) {
  int m = 0;
  for (int k = 0; k < n; k++) {
    const V3 p = in[k], q = in[k + 1 == n ? 0 : k + 1];
    const float dp = dot(p, a) - b, dq = dot(q, a) - b;
    if (dp <= 0.f) out[m++] = p;
    if ((dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f)) {
      const float t = dp / (dp - dq);
      out[m++] = p + (q - p) * t;
    }
  }
  return m;
}

DEV V3 sel3(V3 a0, V3 a1, V3 a2, int k) { return k == 0 ? a0 : (k == 1 ? a1 : a2); }
DEV float self3(float a0, float a1, float a2, int k) { return k == 0 ? a0 : (k == 1 ? a1 : a2); }

// box-box, split in parts (used by the lane-quad form box_box_quad below):
// the 15-axis SAT, the edge-edge contact and the face-contact setup (reference / incident faces).
struct BoxSat {
  V3 A[3], B[3], d;
  float h1[3], h2[3];
  float best_face, best_edge;
  int face_axis, ei, ej;
  bool sep;
};
DEV void box_sat(const Geom& G1, const Geom& G2, V3 hb1, V3 hb2, BoxSat& S) {
  S.h1[0] = hb1.x; S.h1[1] = hb1.y; S.h1[2] = hb1.z;
  S.h2[0] = hb2.x; S.h2[1] = hb2.y; S.h2[2] = hb2.z;
  const float* h1 = S.h1;
  const float* h2 = S.h2;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    S.A[k] = col(G1.R, k);
    S.B[k] = col(G2.R, k);
  }
  const V3* A = S.A;
  const V3* B = S.B;
  const V3 d = G2.x - G1.x;
  S.d = d;
  // SAT in the relative-rotation form (R = A'B, t = A'd, u = B'd): face axes of box 1, of box 2,
  // then the 9 edge-edge axes A_i x B_j, whose projections are again entries of R (unit axes;
  // depths divided by |A_i x B_j|).  Same axes, order and strict-minimum tie rule as the
  // explicit form.
  float Rm[3][3], aR[3][3], t[3], tu[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    t[i] = dot(d, A[i]);
    tu[i] = dot(d, B[i]);
#pragma unroll
    for (int j = 0; j < 3; j++) {
      Rm[i][j] = dot(A[i], B[j]);
      aR[i][j] = fabsf(Rm[i][j]);
    }
  }
  float best_face = 3e38f, best_edge = 3e38f;
  int face_axis = 0, ei = -1, ej = -1;
  bool sep = false;
#pragma unroll
  for (int ax = 0; ax < 6; ax++) {
    const float s = ax < 3 ? h1[ax] + h2[0] * aR[ax][0] + h2[1] * aR[ax][1] + h2[2] * aR[ax][2] - fabsf(t[ax])
                           : h2[ax - 3] + h1[0] * aR[0][ax - 3] + h1[1] * aR[1][ax - 3] + h1[2] * aR[2][ax - 3] -
                                 fabsf(tu[ax - 3]);
    sep |= s < 0.f;
    if (s < best_face) {
      best_face = s;
      face_axis = ax;
    }
  }
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 3; b++) {
      const int a1 = (a + 1) % 3, a2 = (a + 2) % 3, b1 = (b + 1) % 3, b2 = (b + 2) % 3;
      // A_a x B_b = R[a1][b] A_a2 - R[a2][b] A_a1
      const float ln = sqrtf(Rm[a1][b] * Rm[a1][b] + Rm[a2][b] * Rm[a2][b]);
      if (ln < 1e-6f) continue;
      const float ra = h1[a1] * aR[a2][b] + h1[a2] * aR[a1][b];
      const float rb = h2[b1] * aR[a][b2] + h2[b2] * aR[a][b1];
      const float s = (ra + rb - fabsf(t[a2] * Rm[a1][b] - t[a1] * Rm[a2][b])) / ln;
      sep |= s < 0.f;
      if (s < best_edge) {
        best_edge = s;
        ei = a;
        ej = b;
      }
    }
  S.best_face = best_face;
  S.best_edge = best_edge;
  S.face_axis = face_axis;
  S.ei = ei;
  S.ej = ej;
  S.sep = sep;
}
DEV bool box_edge_contact(const BoxSat& S) { return S.ei >= 0 && S.best_edge < 0.95f * S.best_face - 1e-9f; }
// edge-edge: one point at the midpoint of the closest points of the two edges
template <class Sink>
DEV void box_edge(Sink& cs, const Geom& G1, const Geom& G2, const BoxSat& S) {
  const V3* A = S.A;
  const V3* B = S.B;
  const float* h1 = S.h1;
  const float* h2 = S.h2;
  const int ei = S.ei, ej = S.ej;
  const V3 eL = normalize(cross(sel3(A[0], A[1], A[2], ei), sel3(B[0], B[1], B[2], ej)));
  const V3 L = dot(eL, S.d) < 0.f ? -eL : eL;
  V3 ca = G1.x, cb = G2.x;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (k != ei) ca = ca + A[k] * (dot(A[k], L) >= 0.f ? h1[k] : -h1[k]);
    if (k != ej) cb = cb + B[k] * (dot(B[k], L) >= 0.f ? -h2[k] : h2[k]);
  }
  const V3 ua = sel3(A[0], A[1], A[2], ei), ub = sel3(B[0], B[1], B[2], ej), w = ca - cb;
  const float bb = dot(ua, ub), dd = dot(ua, w), ee = dot(ub, w);
  const float den = 1.f - bb * bb;
  float ta = den > 1e-9f ? (bb * ee - dd) / den : 0.f;
  float tb = den > 1e-9f ? (ee - bb * dd) / den : 0.f;
  ta = fminf(fmaxf(ta, -self3(h1[0], h1[1], h1[2], ei)), self3(h1[0], h1[1], h1[2], ei));
  tb = fminf(fmaxf(tb, -self3(h2[0], h2[1], h2[2], ej)), self3(h2[0], h2[1], h2[2], ej));
  cs.add(G1.g, G2.g, -S.best_edge, ((ca + ua * ta) + (cb + ub * tb)) * 0.5f, L);
}
// face contact setup: the incident face's corners q[0..3] (in the clip order), the reference
// face's centre cr, its normal nref (toward the incident box), its two side axes and half extents,
// and the contact normal from geom 1 to geom 2.  Every per-axis pick is a select over the three
// axes (no dynamically indexed private arrays -> no scratch).
struct BoxFace {
  V3 q[4], cr, nref, ax0, ax1, nout;
  float hru, hrv;
};
DEV void box_face(const Geom& G1, const Geom& G2, const BoxSat& S, BoxFace& F) {
  const V3* A = S.A;
  const V3* B = S.B;
  const float* h1 = S.h1;
  const float* h2 = S.h2;
  const bool ref1 = S.face_axis < 3;
  const int k = ref1 ? S.face_axis : S.face_axis - 3;
  const V3 Rr0 = ref1 ? A[0] : B[0], Rr1 = ref1 ? A[1] : B[1], Rr2 = ref1 ? A[2] : B[2];
  const V3 Ri0 = ref1 ? B[0] : A[0], Ri1 = ref1 ? B[1] : A[1], Ri2 = ref1 ? B[2] : A[2];
  const float hr0 = ref1 ? h1[0] : h2[0], hr1 = ref1 ? h1[1] : h2[1], hr2 = ref1 ? h1[2] : h2[2];
  const float hi0 = ref1 ? h2[0] : h1[0], hi1 = ref1 ? h2[1] : h1[1], hi2 = ref1 ? h2[2] : h1[2];
  const V3 pr = ref1 ? G1.x : G2.x, pi = ref1 ? G2.x : G1.x;
  V3 nref = sel3(Rr0, Rr1, Rr2, k);
  if (dot(nref, pi - pr) < 0.f) nref = -nref;
  int bj = 0;
  float bdot = 0.f;
  {
    const float t0 = fabsf(dot(Ri0, nref)), t1 = fabsf(dot(Ri1, nref)), t2 = fabsf(dot(Ri2, nref));
    if (t0 > bdot) { bdot = t0; bj = 0; }
    if (t1 > bdot) { bdot = t1; bj = 1; }
    if (t2 > bdot) { bdot = t2; bj = 2; }
  }
  V3 ni = sel3(Ri0, Ri1, Ri2, bj);
  if (dot(ni, nref) > 0.f) ni = -ni;
  const V3 ci = pi + ni * self3(hi0, hi1, hi2, bj);
  const int u = bj == 2 ? 0 : bj + 1, v = bj == 0 ? 2 : bj - 1;
  const V3 Ru = sel3(Ri0, Ri1, Ri2, u) * self3(hi0, hi1, hi2, u);
  const V3 Rv = sel3(Ri0, Ri1, Ri2, v) * self3(hi0, hi1, hi2, v);
  F.q[0] = ci + Ru + Rv;
  F.q[1] = ci - Ru + Rv;
  F.q[2] = ci - Ru - Rv;
  F.q[3] = ci + Ru - Rv;
  F.cr = pr + nref * self3(hr0, hr1, hr2, k);
  const int ru = k == 2 ? 0 : k + 1, rv = k == 0 ? 2 : k - 1;
  F.ax0 = sel3(Rr0, Rr1, Rr2, ru);
  F.ax1 = sel3(Rr0, Rr1, Rr2, rv);
  F.hru = self3(hr0, hr1, hr2, ru);
  F.hrv = self3(hr0, hr1, hr2, rv);
  F.nref = nref;
  F.nout = ref1 ? nref : -nref;
}

// ---- lane-quad form: one pair per 4 consecutive lanes (a DPP quad), 16 pairs per wave pass
template <int CTRL>
DEV int qdpp_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
// the quad's lanes where b holds, as bits 0..3
DEV int qpop(unsigned m) { return (int)__popc(m); }
DEV unsigned quad_bits(bool b) {
  const unsigned long long m = __ballot(b);
  return (unsigned)(m >> ((threadIdx.x & 63) & ~3)) & 0xFu;
}
// one pair on the lane quad (every lane of the quad calls it with the same pair): the SAT and the
// face setup redundantly, then the incident corners one per lane ("inside" case) or the
// Sutherland-Hodgman clip with polygon vertices ql and ql + 4 per lane and plane (quad prefix
// counts keep the sequential vertex order, and every vertex and intersection is computed with the
// sequential clip's expression), contacts put with the keys and slots the sequential clip gives
// them, i.e. the same contact list in the same order as the oracle's sequential box_box.  (r03
// checked it bit-identical to the then lane-per-pair form on 24,576 C3 states under strict fp
// evaluation order; the step kernel has since been compiled with -fassociative-math, so that
// bit-for-bit claim no longer holds or is re-checked.  What is enforced now: the box-box scenes of
// tests/test_collision_kat.py against geometry, depth 2e-6 m and the exact contact counts, and the
// oracle parity tests' qpos / qvel tolerances.)  poly, tmp: 8 V3 each of the quad's LDS scratch.
template <class Sink>
DEV void box_box_quad(Sink& cs, const Geom& G1, const Geom& G2, V3 hb1, V3 hb2, V3* poly, V3* tmp) {
  CLK_DECL;
  const int ql = threadIdx.x & 3;
  const unsigned below = (1u << ql) - 1u;
  BoxSat S;
  box_sat(G1, G2, hb1, hb2, S);
  if (S.sep) return;  // (quad-uniform from here on: every lane has the same pair)
  PROBEF(8, cs.E->stats, STAT_T_AUX0);
  if (box_edge_contact(S)) {
    if (ql == 0) box_edge(cs, G1, G2, S);
    return;
  }
  BoxFace F;
  box_face(G1, G2, S, F);
  const V3 cr = F.cr, nref = F.nref, nout = F.nout;
  const V3 pa[4] = {F.ax0, -F.ax0, F.ax1, -F.ax1};
  const float pb[4] = {dot(F.ax0, cr) + F.hru, dot(-F.ax0, cr) + F.hru, dot(F.ax1, cr) + F.hrv, dot(-F.ax1, cr) + F.hrv};
  const V3 qc = ql == 0 ? F.q[0] : (ql == 1 ? F.q[1] : (ql == 2 ? F.q[2] : F.q[3]));
  const bool in_c = dot(qc, pa[0]) - pb[0] <= 0.f && dot(qc, pa[1]) - pb[1] <= 0.f && dot(qc, pa[2]) - pb[2] <= 0.f &&
                    dot(qc, pa[3]) - pb[3] <= 0.f;
  PROBEF(8, cs.E->stats, STAT_T_AUX1);
  if (quad_bits(in_c) == 0xFu) {  // incident face inside the reference face: the 4 corners
    const float dep = -dot(qc - cr, nref);
    const unsigned km = quad_bits(dep >= 0.f);
    int slot = ql == 0 ? cs.reserve(qpop(km)) : 0;
    slot = qdpp_i<0x00>(slot);  // quad_perm [0,0,0,0]: lane 0's reservation
    if (dep >= 0.f) {
      const int rank = qpop(km & below);
      cs.put_at(slot + rank, rank, G1.g, G2.g, -dep, qc + nref * (0.5f * dep), nout);
    }
    PROBEF(8, cs.E->stats, STAT_T_AUX2);
    return;
  }
  // clip: 4 planes, the polygon in the quad's LDS scratch, vertex k in lane k & 3 (slot k >> 2)
  poly[ql] = qc;
  __builtin_amdgcn_wave_barrier();
  int np = 4;
  V3* src = poly;
  V3* dst = tmp;
#pragma unroll
  for (int st = 0; st < 4; st++) {
    V3 p[2], q[2];
    float dp[2], dq[2];
    bool keep[2], crs[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int k = ql + 4 * h;
      const bool have = k < np;
      p[h] = src[have ? k : 0];
      q[h] = src[have ? (k + 1 == np ? 0 : k + 1) : 0];
      dp[h] = dot(p[h], pa[st]) - pb[st];
      dq[h] = dot(q[h], pa[st]) - pb[st];
      keep[h] = have && dp[h] <= 0.f;
      crs[h] = have && ((dp[h] < 0.f && dq[h] > 0.f) || (dp[h] > 0.f && dq[h] < 0.f));
    }
    const unsigned k0 = quad_bits(keep[0]), c0 = quad_bits(crs[0]), k1 = quad_bits(keep[1]), c1 = quad_bits(crs[1]);
    const int tot0 = qpop(k0) + qpop(c0);
    int pos[2] = {qpop(k0 & below) + qpop(c0 & below), tot0 + qpop(k1 & below) + qpop(c1 & below)};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (keep[h]) dst[pos[h]] = p[h];
      if (crs[h]) {
        const float t = dp[h] / (dp[h] - dq[h]);
        dst[pos[h] + (keep[h] ? 1 : 0)] = p[h] + (q[h] - p[h]) * t;
      }
    }
    np = tot0 + qpop(k1) + qpop(c1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    V3* sw = src;
    src = dst;
    dst = sw;
  }
  PROBEF(8, cs.E->stats, STAT_T_AUX3);
  float dep[2];
  bool kv[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int k = ql + 4 * h;
    dep[h] = k < np ? -dot(src[k] - cr, nref) : -1.f;
    kv[h] = k < np && dep[h] >= 0.f;
  }
  const unsigned m0 = quad_bits(kv[0]), m1 = quad_bits(kv[1]);
  int slot = ql == 0 ? cs.reserve(qpop(m0) + qpop(m1)) : 0;
  slot = qdpp_i<0x00>(slot);
  const int r[2] = {qpop(m0 & below), qpop(m0) + qpop(m1 & below)};
#pragma unroll
  for (int h = 0; h < 2; h++)
    if (kv[h]) {
      const int k = ql + 4 * h;
      cs.put_at(slot + r[h], r[h], G1.g, G2.g, -dep[h], src[k] + nref * (0.5f * dep[h]), nout);
    }
}

// ---------------------------------------------------------------- GJK + EPA (wave-cooperative)
// One geom pair at a time per wave: every lane runs the same, uniform GJK/EPA control flow; the
// mesh support query is split over the lanes (hull vertices strided by lane, then a DPP arg-max
// whose ties resolve to the lowest vertex index, as the serial scan does); the EPA polytope lives
// in LDS scratch supplied by the caller.  Must be called with all 64 lanes active.
template <int CTRL>
DEV float gdpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
DEV int gdpp_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
DEV void argmax_merge(float& v, int& i, float v2, int i2) {
  const bool take = v2 > v || (v2 == v && i2 < i);
  v = take ? v2 : v;
  i = take ? i2 : i;
}
template <int CTRL>
DEV void argmax_dpp(float& v, int& i) {
  argmax_merge(v, i, gdpp_f<CTRL>(v), gdpp_i<CTRL>(i));
}
DEV void wave_argmax(float& v, int& i) {
  argmax_dpp<0xB1>(v, i);   // quad_perm [1,0,3,2]
  argmax_dpp<0x4E>(v, i);   // quad_perm [2,3,0,1]
  argmax_dpp<0x141>(v, i);  // row_half_mirror
  argmax_dpp<0x140>(v, i);  // row_mirror
  float bv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
  for (int r = 1; r < 4; r++)
    argmax_merge(bv, bi, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16 * r)),
                 __builtin_amdgcn_readlane(i, 16 * r));
  v = bv;
  i = bi;
}
// Mesh support query over the wave: the hull's vertices strided by lane (each lane keeps the best of
// its own and that vertex's coordinates), the wave arg-max (ties: the lowest index, as the serial
// scan), then the winner's coordinates by v_readlane from its lane (r06: no dependent reload of the
// winning vertex from the constant tables).  Caching the hull in registers for the whole GJK / EPA
// pair measured no faster (the extra live registers cost spill slots, CHANGELOG r06).
DEV V3 support_wave(const Geom& G, V3 dir) {
  if (G.type != GT_MESH) return support(G, dir);
  const V3 dl = mulT(G.R, dir);
  const int m = MMX_geom_mesh[G.g];
  const int a = MMX_mesh_vertadr[m], nvert = MMX_mesh_vertnum[m];
  float best = -3.0e38f, bx = 0.f, by = 0.f, bz = 0.f;
  int bi = 0x7fffffff;
  for (int v = (int)(threadIdx.x & 63); v < nvert; v += 64) {
    const int q = 3 * (a + v);
    const float x = MMX_mesh_vert[q], y = MMX_mesh_vert[q + 1], z = MMX_mesh_vert[q + 2];
    const float s = x * dl.x + y * dl.y + z * dl.z;
    if (s > best) {
      best = s;
      bi = v;
      bx = x;
      by = y;
      bz = z;
    }
  }
  wave_argmax(best, bi);
  const int wl = bi & 63;  // the winner's lane holds its coordinates as its own best
  const V3 p = V3{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(bx), wl)),
                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(by), wl)),
                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bz), wl))};
  return G.x + mul(G.R, p);
}

struct SVx {
  V3 w, a, b;
};
// the pair's geoms
struct GPair {
  const Geom& A;
  const Geom& B;
};
DEV SVx mk_sv(const GPair& P, V3 dir) {
  SVx s;
  s.a = support_wave(P.A, dir);
  s.b = support_wave(P.B, -dir);
  s.w = s.a - s.b;
  return s;
}
// GJK simplex in named registers (s0 = newest point): every case below is a fixed permutation,
// so no simplex element is ever indexed at run time (that spilled the simplex to scratch).
DEV bool gjk_line(const SVx& s0, const SVx& s1, int& n, V3& dir) {
  const V3 ab = s1.w - s0.w, ao = -s0.w;
  if (dot(ab, ao) > 0.f) {
    dir = cross(cross(ab, ao), ab);
    n = 2;
    return norm(dir) < 1e-12f * (1.f + dot(ab, ab));
  }
  n = 1;
  dir = ao;
  return false;
}
DEV bool gjk_tri(const SVx& s0, SVx& s1, SVx& s2, int& n, V3& dir) {
  const V3 ab = s1.w - s0.w, ac = s2.w - s0.w, ao = -s0.w;
  const V3 abc = cross(ab, ac);
  if (dot(cross(abc, ac), ao) > 0.f) {
    if (dot(ac, ao) > 0.f) {
      s1 = s2;
      n = 2;
      dir = cross(cross(ac, ao), ac);
      return false;
    }
    n = 2;
    return gjk_line(s0, s1, n, dir);
  }
  if (dot(cross(ab, abc), ao) > 0.f) {
    n = 2;
    return gjk_line(s0, s1, n, dir);
  }
  const float dd = dot(abc, ao);
  n = 3;
  if (fabsf(dd) < 1e-12f * (1.f + dot(abc, abc))) return true;
  if (dd > 0.f) dir = abc;
  else {
    const SVx t = s1;
    s1 = s2;
    s2 = t;
    dir = -abc;
  }
  return false;
}
// face (s0, b, c) with the fourth vertex o opposite: does the origin lie beyond it?
DEV bool gjk_face_out(const SVx& s0, const SVx& b, const SVx& c, const SVx& o) {
  V3 nn = cross(b.w - s0.w, c.w - s0.w);
  if (dot(nn, o.w - s0.w) > 0.f) nn = -nn;
  return dot(nn, -s0.w) > 0.f;
}
DEV bool gjk_tet(const SVx& s0, SVx& s1, SVx& s2, SVx& s3, int& n, V3& dir) {
  n = 3;
  if (gjk_face_out(s0, s1, s2, s3)) return gjk_tri(s0, s1, s2, n, dir);  // face (0,1,2)
  if (gjk_face_out(s0, s2, s3, s1)) {                                     // face (0,2,3)
    s1 = s2;
    s2 = s3;
    return gjk_tri(s0, s1, s2, n, dir);
  }
  if (gjk_face_out(s0, s3, s1, s2)) {  // face (0,3,1)
    s2 = s1;
    s1 = s3;
    return gjk_tri(s0, s1, s2, n, dir);
  }
  n = 4;
  return true;
}
DEV bool gjk(const GPair& GP, SVx& s0, SVx& s1, SVx& s2, SVx& s3, int& n) {
  V3 dir = GP.A.x - GP.B.x;
  if (norm(dir) < 1e-9f) dir = V3{1.f, 0.f, 0.f};
  s0 = mk_sv(GP, dir);
  n = 1;
  dir = -s0.w;
  for (int it = 0; it < 48; it++) {
    if (norm(dir) < 1e-12f) return true;
    const SVx P = mk_sv(GP, dir);
    if (dot(P.w, dir) < 0.f) return false;
    s3 = s2;  // push P; entries beyond n are dead
    s2 = s1;
    s1 = s0;
    s0 = P;
    n++;
    const bool hit = n == 2 ? gjk_line(s0, s1, n, dir)
                            : (n == 3 ? gjk_tri(s0, s1, s2, n, dir) : gjk_tet(s0, s1, s2, s3, n, dir));
    if (hit) return true;
  }
  return norm(dir) < 1e-12f;
}

#define EPA_MAXV 38
#define EPA_MAXF 72  // 2 EPA_MAXV - 4: the faces of a closed polytope on EPA_MAXV vertices
// an EPA face: its three vertex indices packed in one word (8 bits each: EPA_MAXV < 256), unit
// normal and distance from the origin (5 words; the polytope fits the collision scratch beside the
// contacts)
struct EFace {
  int vv;
  V3 n;
  float d;
  DEV int v(int k) const { return (vv >> (8 * k)) & 255; }
};
static_assert(EPA_MAXV < 256, "EPA vertex indices are packed in bytes");
DEV bool epa_face(const SVx* V, EFace& f, int a, int b, int c) {
  f.vv = a | (b << 8) | (c << 16);
  const V3 n = cross(V[b].w - V[a].w, V[c].w - V[a].w);
  const float ln = norm(n);
  if (ln < 1e-20f) return false;
  f.n = n * (1.f / ln);
  f.d = dot(f.n, V[a].w);
  return true;
}
// wave-level ordering of the EPA's LDS arrays between its lane-parallel steps (one wave runs the pair)
DEV void epa_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
DEV int epa_lane() { return (int)(threadIdx.x & 63); }
DEV int epa_prefix(unsigned long long m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// V, F, edges: LDS scratch (EPA_MAXV SVx, EPA_MAXF EFace, 3 EPA_MAXF edges packed a | b << 8).
// The polytope's faces are handled one per lane (r06): the nearest face is a wave arg-min (ties to
// the lowest index, as the serial scan), the faces the new point sees are one ballot, the others
// are compacted in index order by ballot prefixes, and the horizon's new faces are formed one per
// lane and appended in edge order; the horizon edge list itself is built from the visible faces in
// index order with the serial add / cancel rule.  Every array ends each iteration exactly as the
// serial loops left it (same faces, same order, same arithmetic per face).
DEV bool epa(const GPair& GP, SVx* V, int nv, V3& nrm, float& depth, V3& pa, V3& pb, EFace* F, int* edges) {
  int nf = 0;
  if (nv == 1) {
    for (int k = 0; k < 6 && nv < 2; k++) {  // +x, -x, +y, -y, +z, -z
      const float sg = (k & 1) ? -1.f : 1.f;
      V[nv] = mk_sv(GP, V3{k < 2 ? sg : 0.f, (k >> 1) == 1 ? sg : 0.f, k >= 4 ? sg : 0.f});
      if (norm(V[nv].w - V[0].w) > 1e-7f) nv++;
    }
  }
  if (nv == 2) {
    const V3 ab = V[1].w - V[0].w;
    const V3 ax = fabsf(ab.x) <= fabsf(ab.y) && fabsf(ab.x) <= fabsf(ab.z)
                      ? V3{1.f, 0.f, 0.f}
                      : (fabsf(ab.y) <= fabsf(ab.z) ? V3{0.f, 1.f, 0.f} : V3{0.f, 0.f, 1.f});
    const V3 t = normalize(cross(ab, ax));
    V[2] = mk_sv(GP, t);
    if (norm(cross(V[2].w - V[0].w, ab)) < 1e-10f) V[2] = mk_sv(GP, -t);
    nv = 3;
  }
  if (nv == 3) {
    const V3 n = normalize(cross(V[1].w - V[0].w, V[2].w - V[0].w));
    V[3] = mk_sv(GP, n);
    if (fabsf(dot(V[3].w - V[0].w, n)) < 1e-9f) V[3] = mk_sv(GP, -n);
    nv = 4;
  }
  const int T[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
  const V3 cen = (V[0].w + V[1].w + V[2].w + V[3].w) * 0.25f;
  for (int k = 0; k < 4; k++) {
    if (!epa_face(V, F[nf], T[k][0], T[k][1], T[k][2])) continue;
    if (dot(F[nf].n, V[T[k][0]].w - cen) < 0.f) epa_face(V, F[nf], T[k][0], T[k][2], T[k][1]);
    nf++;
  }
  static_assert(EPA_MAXF <= 128, "two faces per lane");
  const int ln = epa_lane();
  int best = -1;
  for (int it = 0; it < 32; it++) {
    epa_sync();
    // nearest face: per lane its faces ln, ln + 64 (strict <: the lower index on ties), then the
    // wave's arg-max of -d (ties: the lowest index)
    float bd = -3e38f;
    int bi = 0x7fffffff;
    if (ln < nf && F[ln].d < 3e38f) {
      bd = -F[ln].d;
      bi = ln;
    }
    if (ln + 64 < nf && -F[ln + 64].d > bd) {
      bd = -F[ln + 64].d;
      bi = ln + 64;
    }
    wave_argmax(bd, bi);
    best = bi < nf ? bi : -1;
    if (best < 0) return false;
    const V3 fn = F[best].n;
    const float fd = F[best].d;
    const SVx P = mk_sv(GP, fn);
    const float dist = dot(P.w, fn);
    if (dist - fd < 1e-6f * (1.f + fabsf(dist)) || nv >= EPA_MAXV) break;
    // which faces P sees (lane ln: faces ln and ln + 64), the others kept in index order
    EFace f0, f1;
    bool vis0 = false, vis1 = false;
    if (ln < nf) {
      f0 = F[ln];
      vis0 = dot(f0.n, P.w - V[f0.v(0)].w) > 1e-9f;
    }
    if (ln + 64 < nf) {
      f1 = F[ln + 64];
      vis1 = dot(f1.n, P.w - V[f1.v(0)].w) > 1e-9f;
    }
    const unsigned long long mv0 = __ballot(vis0), mv1 = __ballot(vis1);
    const unsigned long long mk0 = __ballot(ln < nf && !vis0), mk1 = __ballot(ln + 64 < nf && !vis1);
    // horizon: the visible faces' edges in face order, an edge cancelling its reverse (serial rule)
    int ne = 0;
    for (int half = 0; half < 2; half++) {
      unsigned long long m = half ? mv1 : mv0;
      while (m) {
        const int k = 64 * half + __builtin_ctzll(m);
        m &= m - 1ull;
        const EFace f = F[k];
        for (int e = 0; e < 3; e++) {
          const int a = f.v(e), b = f.v((e + 1) % 3);
          int found = -1;
          for (int q0 = 0; q0 < ne && found < 0; q0 += 64) {  // the first (b, a) in the list
            const int q = q0 + ln;
            const unsigned long long hit = __ballot(q < ne && edges[q] == (b | (a << 8)));
            if (hit) found = q0 + __builtin_ctzll(hit);
          }
          epa_sync();
          if (found >= 0) {
            if (ln == 0) edges[found] = edges[ne - 1];
            ne--;
          } else if (ne < EPA_MAXF * 3) {
            if (ln == 0) edges[ne] = a | (b << 8);
            ne++;
          }
          epa_sync();
        }
      }
    }
    // kept faces compacted in index order (their records are in registers: no overlap hazard)
    epa_sync();
    const int nk0 = __popcll(mk0);
    if (ln < nf && !vis0) F[epa_prefix(mk0)] = f0;
    if (ln + 64 < nf && !vis1) F[nk0 + epa_prefix(mk1)] = f1;
    nf = nk0 + __popcll(mk1);
    const int pi = nv++;
    if (ln == 0) V[pi] = P;
    epa_sync();
    // the horizon's faces with P, appended in edge order while they fit (degenerate ones skipped)
    for (int q0 = 0; q0 < ne && nf < EPA_MAXF; q0 += 64) {
      const int q = q0 + ln;
      EFace g;
      const bool ok = q < ne && epa_face(V, g, edges[q] & 255, edges[q] >> 8, pi);
      const unsigned long long mo = __ballot(ok);
      const int pos = nf + epa_prefix(mo);
      if (ok && pos < EPA_MAXF) F[pos] = g;
      nf = min(EPA_MAXF, nf + __popcll(mo));
    }
  }
  epa_sync();
  if (best < 0) return false;
  const EFace& f = F[best];
  const V3 p = f.n * f.d;
  const V3 v0 = V[f.v(1)].w - V[f.v(0)].w, v1 = V[f.v(2)].w - V[f.v(0)].w, v2 = p - V[f.v(0)].w;
  const float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
  const float den = d00 * d11 - d01 * d01;
  const float lv = den > 1e-30f ? (d11 * d20 - d01 * d21) / den : 0.f;
  const float lw = den > 1e-30f ? (d00 * d21 - d01 * d20) / den : 0.f;
  const float lu = 1.f - lv - lw;
  pa = V[f.v(0)].a * lu + V[f.v(1)].a * lv + V[f.v(2)].a * lw;
  pb = V[f.v(0)].b * lu + V[f.v(1)].b * lv + V[f.v(2)].b * lw;
  nrm = f.n;
  depth = f.d;
  return true;
}

#define EPA_SCRATCH_FLOATS (9 * EPA_MAXV + 5 * EPA_MAXF + 3 * EPA_MAXF)
// scr: EPA_SCRATCH_FLOATS of LDS; emits at most one contact (lane 0)
template <class Sink>
DEV void convex_convex(Sink& cs, const Geom& A, const Geom& B, float* scr) {
  const GPair GP{A, B};
  SVx s0, s1, s2, s3;
  int n = 0;
  if (!gjk(GP, s0, s1, s2, s3, n)) return;
  SVx* V = reinterpret_cast<SVx*>(scr);
  EFace* F = reinterpret_cast<EFace*>(scr + 9 * EPA_MAXV);
  int* edges = reinterpret_cast<int*>(scr + 9 * EPA_MAXV + 5 * EPA_MAXF);
  V[0] = s0;
  if (n > 1) V[1] = s1;
  if (n > 2) V[2] = s2;
  if (n > 3) V[3] = s3;
  V3 nrm, pa, pb;
  float depth;
  if (!epa(GP, V, n, nrm, depth, pa, pb, F, edges)) return;
  if (depth < 0.f) return;
  // Minkowski A-B face normal n: translating B by +depth n separates -> normal A->B is n
  if ((threadIdx.x & 63) == 0) cs.add(A.g, B.g, -depth, (pa + pb) * 0.5f, nrm);
}

// soft-constraint impedance d(pos) (MuJoCo solimp: dmin, dmax, width, midpoint, power)
DEV float impedance(const float* si, float pos) {
  const float dmin = fminf(fmaxf(si[0], 1e-4f), 0.9999f), dmax = fminf(fmaxf(si[1], 1e-4f), 0.9999f);
  const float width = si[2], mid = si[3], power = si[4];
  if (dmin == dmax || width <= 1e-15f) return 0.5f * (dmin + dmax);
  const float x = fabsf(pos / width);
  if (x >= 1.f) return dmax;
  if (x <= 0.f) return dmin;
  float y;
  if (power == 1.f) y = x;
  else if (power == 2.f) y = x <= mid ? x * x / mid : 1.f - (1.f - x) * (1.f - x) / (1.f - mid);  // MuJoCo default
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1.f);
  else y = 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
  return dmin + y * (dmax - dmin);
}

#endif
