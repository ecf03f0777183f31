/* ORACLE (test infrastructure only) — fp64 restatement of MuJoCo's collision stage for
 * the pick-and-place model (inside mujoco.mj_step, env.py:121).  MuJoCo 3.5.0 is not
 * vendored; this follows its documented design:
 *   broadphase: the compiled candidate pair list (same-weld / parent-weld / exclude
 *               filtered, panda.xml:284-286) culled by bounding spheres and OBBs;
 *   narrowphase: plane-box (corners), plane-convex (support point), box-box (separating
 *               axis test + reference-face clipping), everything else through GJK + EPA
 *               (the "nativeccd" convex path: one contact per pair, multiccd off);
 *   contact parameters: condim = max, friction = element-wise max, solref/solimp = mean
 *               (solmix 1/1), margin = gap = 0; normal points from geom1 to geom2 with
 *               geom1 the lower geom type.
 * Physics parity with MuJoCo itself is unpinned (MuJoCo absent in this image). */
#include <stdlib.h>
#include "or_internal.h"

enum { GT_PLANE = 0, GT_CYLINDER = 5, GT_BOX = 6, GT_MESH = 7 };

static void add_contact(or_env* e, int g1, int g2, double dist, const double* pos, const double* normal) {
  if (e->ncon >= OR_MAXCON) return;
  or_contact* c = &e->con[e->ncon++];
  c->geom[0] = g1;
  c->geom[1] = g2;
  c->dist = dist;
  v3_copy(c->pos, pos);
  double n[3];
  v3_copy(n, normal);
  v3_normalize(n);
  make_frame(c->frame, n);
  int d1 = OM_geom_condim[g1], d2 = OM_geom_condim[g2];
  c->dim = d1 > d2 ? d1 : d2;
  double f[3];
  for (int k = 0; k < 3; k++) {
    double a = OM_geom_friction[3 * g1 + k], b = OM_geom_friction[3 * g2 + k];
    f[k] = a > b ? a : b;
  }
  c->friction[0] = f[0]; c->friction[1] = f[0]; c->friction[2] = f[1];
  c->friction[3] = f[2]; c->friction[4] = f[2];
  for (int k = 0; k < 2; k++) c->solref[k] = 0.5 * (OM_geom_solref[2 * g1 + k] + OM_geom_solref[2 * g2 + k]);
  for (int k = 0; k < 5; k++) c->solimp[k] = 0.5 * (OM_geom_solimp[5 * g1 + k] + OM_geom_solimp[5 * g2 + k]);
}

/* ------------------------------------------------------------------ support functions */
static void support(const or_env* e, int g, const double* dir, double* out) {
  const double* R = e->gxmat[g];
  const double* p = e->gxpos[g];
  double dl[3], sl[3];
  m3_mulTv(dl, R, dir);
  int type = OM_geom_type[g];
  if (type == GT_BOX) {
    const double* h = &OM_geom_size[3 * g];
    for (int k = 0; k < 3; k++) sl[k] = dl[k] >= 0 ? h[k] : -h[k];
  } else if (type == GT_CYLINDER) {
    double r = OM_geom_size[3 * g], hh = OM_geom_size[3 * g + 1];
    double n = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
    if (n > 1e-15) { sl[0] = r * dl[0] / n; sl[1] = r * dl[1] / n; }
    else { sl[0] = r; sl[1] = 0; }
    sl[2] = dl[2] >= 0 ? hh : -hh;
  } else { /* mesh hull */
    int m = OM_geom_mesh[g];
    const double* v = &OM_mesh_vert[3 * OM_mesh_vertadr[m]];
    int nv = OM_mesh_vertnum[m];
    double best = -1e300;
    int bi = 0;
    for (int i = 0; i < nv; i++) {
      double s = v3_dot(&v[3 * i], dl);
      if (s > best) { best = s; bi = i; }
    }
    v3_copy(sl, &v[3 * bi]);
  }
  m3_mulv(out, R, sl);
  v3_add(out, out, p);
}

/* ------------------------------------------------------------------ midphase */
static int obb_overlap(const or_env* e, int g1, int g2) {
  const double* R1 = e->gxmat[g1];
  const double* R2 = e->gxmat[g2];
  const double* h1 = &OM_geom_aabb[3 * g1];
  const double* h2 = &OM_geom_aabb[3 * g2];
  double d[3];
  v3_sub(d, e->gxpos[g2], e->gxpos[g1]);
  for (int s = 0; s < 2; s++) {
    const double* Ra = s ? R2 : R1;
    for (int k = 0; k < 3; k++) {
      double L[3] = {Ra[k], Ra[3 + k], Ra[6 + k]};
      double r1 = 0, r2 = 0;
      for (int i = 0; i < 3; i++) {
        r1 += h1[i] * fabs(L[0] * R1[i] + L[1] * R1[3 + i] + L[2] * R1[6 + i]);
        r2 += h2[i] * fabs(L[0] * R2[i] + L[1] * R2[3 + i] + L[2] * R2[6 + i]);
      }
      if (fabs(v3_dot(d, L)) > r1 + r2) return 0;
    }
  }
  return 1;
}

/* ------------------------------------------------------------------ plane-box */
static void plane_box(or_env* e, int gp, int gb) {
  const double* n = &e->gxmat[gp][0];
  double nz[3] = {e->gxmat[gp][2], e->gxmat[gp][5], e->gxmat[gp][8]};
  (void)n;
  const double* R = e->gxmat[gb];
  const double* h = &OM_geom_size[3 * gb];
  double depth[8], pts[8][3];
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    double l[3] = {(i & 1) ? h[0] : -h[0], (i & 2) ? h[1] : -h[1], (i & 4) ? h[2] : -h[2]};
    double w[3], rel[3];
    m3_mulv(w, R, l);
    v3_add(w, w, e->gxpos[gb]);
    v3_sub(rel, w, e->gxpos[gp]);
    double dist = v3_dot(rel, nz);
    if (dist <= 0) {
      depth[cnt] = dist;
      v3_addscl(pts[cnt], w, nz, -0.5 * dist);
      cnt++;
    }
  }
  /* keep the 4 deepest corners */
  for (int k = 0; k < cnt && k < 4; k++) {
    int bi = k;
    for (int i = k + 1; i < cnt; i++)
      if (depth[i] < depth[bi]) bi = i;
    double td = depth[k]; depth[k] = depth[bi]; depth[bi] = td;
    double tp[3]; v3_copy(tp, pts[k]); v3_copy(pts[k], pts[bi]); v3_copy(pts[bi], tp);
    add_contact(e, gp, gb, depth[k], pts[k], nz);
  }
}

/* ------------------------------------------------------------------ plane-convex */
static void plane_convex(or_env* e, int gp, int gc) {
  double nz[3] = {e->gxmat[gp][2], e->gxmat[gp][5], e->gxmat[gp][8]};
  double mn[3] = {-nz[0], -nz[1], -nz[2]};
  double s[3], rel[3];
  support(e, gc, mn, s);
  v3_sub(rel, s, e->gxpos[gp]);
  double dist = v3_dot(rel, nz);
  if (dist <= 0) {
    double pos[3];
    v3_addscl(pos, s, nz, -0.5 * dist);
    add_contact(e, gp, gc, dist, pos, nz);
  }
}

/* ------------------------------------------------------------------ box-box */
/* clip polygon (n pts) against plane  dot(x, a) <= b ; returns new count */
static int clip_poly(double (*in)[3], int n, double (*out)[3], const double* a, double b) {
  int m = 0;
  for (int i = 0; i < n; i++) {
    const double* p = in[i];
    const double* q = in[(i + 1) % n];
    double dp = v3_dot(p, a) - b, dq = v3_dot(q, a) - b;
    if (dp <= 0) v3_copy(out[m++], p);
    if ((dp < 0 && dq > 0) || (dp > 0 && dq < 0)) {
      double t = dp / (dp - dq);
      double r[3];
      for (int k = 0; k < 3; k++) r[k] = p[k] + t * (q[k] - p[k]);
      v3_copy(out[m++], r);
    }
  }
  return m;
}

static void box_box(or_env* e, int g1, int g2) {
  const double* p1 = e->gxpos[g1];
  const double* p2 = e->gxpos[g2];
  const double* R1 = e->gxmat[g1];
  const double* R2 = e->gxmat[g2];
  const double* h1 = &OM_geom_size[3 * g1];
  const double* h2 = &OM_geom_size[3 * g2];
  double A[3][3], B[3][3]; /* axes as rows */
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) {
      A[k][i] = R1[3 * i + k];
      B[k][i] = R2[3 * i + k];
    }
  double d[3];
  v3_sub(d, p2, p1);
  double best_face = 1e300, best_edge = 1e300;
  int face_axis = -1, edge_i = -1, edge_j = -1;
  double edge_L[3] = {0, 0, 0};
  for (int ax = 0; ax < 6; ax++) {
    const double* L = ax < 3 ? A[ax] : B[ax - 3];
    double r1 = 0, r2 = 0;
    for (int k = 0; k < 3; k++) {
      r1 += h1[k] * fabs(v3_dot(L, A[k]));
      r2 += h2[k] * fabs(v3_dot(L, B[k]));
    }
    double s = r1 + r2 - fabs(v3_dot(d, L));
    if (s < 0) return;
    if (s < best_face) { best_face = s; face_axis = ax; }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double L[3];
      v3_cross(L, A[i], B[j]);
      double ln = v3_norm(L);
      if (ln < 1e-6) continue;
      v3_scl(L, L, 1.0 / ln);
      double r1 = 0, r2 = 0;
      for (int k = 0; k < 3; k++) {
        r1 += h1[k] * fabs(v3_dot(L, A[k]));
        r2 += h2[k] * fabs(v3_dot(L, B[k]));
      }
      double s = r1 + r2 - fabs(v3_dot(d, L));
      if (s < 0) return;
      if (s < best_edge) { best_edge = s; edge_i = i; edge_j = j; v3_copy(edge_L, L); }
    }
  if (edge_i >= 0 && best_edge < 0.95 * best_face - 1e-9) {
    /* edge-edge: single contact at the midpoint of the closest points */
    double L[3];
    v3_copy(L, edge_L);
    if (v3_dot(L, d) < 0) v3_scl(L, L, -1);
    double ca[3], cb[3];
    v3_copy(ca, p1);
    v3_copy(cb, p2);
    for (int k = 0; k < 3; k++) {
      if (k != edge_i) v3_addscl(ca, ca, A[k], v3_dot(A[k], L) >= 0 ? h1[k] : -h1[k]);
      if (k != edge_j) v3_addscl(cb, cb, B[k], v3_dot(B[k], L) >= 0 ? -h2[k] : h2[k]);
    }
    const double* ua = A[edge_i];
    const double* ub = B[edge_j];
    double w[3];
    v3_sub(w, ca, cb);
    double a = 1, b = v3_dot(ua, ub), c = 1, dd = v3_dot(ua, w), ee = v3_dot(ub, w);
    double den = a * c - b * b;
    double ta = den > 1e-12 ? (b * ee - c * dd) / den : 0;
    double tb = den > 1e-12 ? (a * ee - b * dd) / den : 0;
    if (ta > h1[edge_i]) ta = h1[edge_i];
    if (ta < -h1[edge_i]) ta = -h1[edge_i];
    if (tb > h2[edge_j]) tb = h2[edge_j];
    if (tb < -h2[edge_j]) tb = -h2[edge_j];
    double qa[3], qb[3], pos[3];
    v3_addscl(qa, ca, ua, ta);
    v3_addscl(qb, cb, ub, tb);
    v3_add(pos, qa, qb);
    v3_scl(pos, pos, 0.5);
    add_contact(e, g1, g2, -best_edge, pos, L);
    return;
  }
  /* face contact: reference box owns face_axis */
  int ref_is_1 = face_axis < 3;
  int k = ref_is_1 ? face_axis : face_axis - 3;
  const double(*Rr)[3] = ref_is_1 ? A : B;
  const double(*Ri)[3] = ref_is_1 ? B : A;
  const double* hr = ref_is_1 ? h1 : h2;
  const double* hi = ref_is_1 ? h2 : h1;
  const double* pr = ref_is_1 ? p1 : p2;
  const double* pi = ref_is_1 ? p2 : p1;
  double nref[3]; /* reference face outward normal, pointing toward the incident box */
  v3_copy(nref, Rr[k]);
  double dri[3];
  v3_sub(dri, pi, pr);
  if (v3_dot(nref, dri) < 0) v3_scl(nref, nref, -1);
  /* incident face: most anti-parallel face of the incident box */
  int bj = 0;
  double bdot = 0;
  for (int j = 0; j < 3; j++) {
    double t = fabs(v3_dot(Ri[j], nref));
    if (t > bdot) { bdot = t; bj = j; }
  }
  double ni[3];
  v3_copy(ni, Ri[bj]);
  if (v3_dot(ni, nref) > 0) v3_scl(ni, ni, -1);
  double ci[3];
  v3_addscl(ci, pi, ni, hi[bj]);
  int u = (bj + 1) % 3, v = (bj + 2) % 3;
  double poly[16][3], tmp[16][3];
  int np = 4;
  for (int c = 0; c < 4; c++) {
    double su = (c == 0 || c == 3) ? 1 : -1;
    double sv = (c < 2) ? 1 : -1;
    double pt[3];
    v3_addscl(pt, ci, Ri[u], su * hi[u]);
    v3_addscl(pt, pt, Ri[v], sv * hi[v]);
    v3_copy(poly[c], pt);
  }
  double cr[3];
  v3_addscl(cr, pr, nref, hr[k]);
  int ru = (k + 1) % 3, rv = (k + 2) % 3;
  const double* axes[2] = {Rr[ru], Rr[rv]};
  double hh[2] = {hr[ru], hr[rv]};
  for (int a = 0; a < 2 && np > 0; a++) {
    double pa[3], na[3];
    v3_copy(pa, axes[a]);
    np = clip_poly(poly, np, tmp, pa, v3_dot(pa, cr) + hh[a]);
    v3_scl(na, pa, -1);
    np = clip_poly(tmp, np, poly, na, v3_dot(na, cr) + hh[a]);
  }
  double nout[3];
  v3_copy(nout, nref);
  if (!ref_is_1) v3_scl(nout, nout, -1); /* normal from geom1 to geom2 */
  for (int c = 0; c < np; c++) {
    double rel[3];
    v3_sub(rel, poly[c], cr);
    double depth = -v3_dot(rel, nref);
    if (depth >= 0) {
      double pos[3];
      v3_addscl(pos, poly[c], nref, 0.5 * depth);
      add_contact(e, g1, g2, -depth, pos, nout);
    }
  }
}

/* ------------------------------------------------------------------ GJK + EPA */
typedef struct { double w[3], a[3], b[3]; } sv;

static void mk_sv(const or_env* e, int g1, int g2, const double* dir, sv* s) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  support(e, g1, dir, s->a);
  support(e, g2, nd, s->b);
  v3_sub(s->w, s->a, s->b);
}

/* GJK boolean intersection on A - B (simplex cases, newest vertex first) */
static int gjk_line(sv* S, int* n, double* dir) {
  double ab[3], ao[3], t[3];
  v3_sub(ab, S[1].w, S[0].w);
  v3_scl(ao, S[0].w, -1);
  if (v3_dot(ab, ao) > 0) {
    v3_cross(t, ab, ao);
    v3_cross(dir, t, ab);
    *n = 2;
    if (v3_norm(dir) < 1e-14 * (1 + v3_norm(ab))) return 1; /* origin on the segment */
  } else {
    *n = 1;
    v3_copy(dir, ao);
  }
  return 0;
}

static int gjk_tri(sv* S, int* n, double* dir) {
  double ab[3], ac[3], ao[3], abc[3], t[3];
  v3_sub(ab, S[1].w, S[0].w);
  v3_sub(ac, S[2].w, S[0].w);
  v3_scl(ao, S[0].w, -1);
  v3_cross(abc, ab, ac);
  v3_cross(t, abc, ac);
  if (v3_dot(t, ao) > 0) {
    if (v3_dot(ac, ao) > 0) {
      S[1] = S[2];
      *n = 2;
      v3_cross(t, ac, ao);
      v3_cross(dir, t, ac);
      return 0;
    }
    *n = 2;
    return gjk_line(S, n, dir);
  }
  v3_cross(t, ab, abc);
  if (v3_dot(t, ao) > 0) {
    *n = 2;
    return gjk_line(S, n, dir);
  }
  double dd = v3_dot(abc, ao);
  *n = 3;
  if (fabs(dd) < 1e-14 * (1 + v3_dot(abc, abc))) return 1; /* origin inside the triangle */
  if (dd > 0) v3_copy(dir, abc);
  else {
    sv tmp = S[1]; S[1] = S[2]; S[2] = tmp;
    v3_scl(dir, abc, -1);
  }
  return 0;
}

static int gjk_tet(sv* S, int* n, double* dir) {
  double ao[3];
  v3_scl(ao, S[0].w, -1);
  /* faces containing the newest vertex a: (a,b,c), (a,c,d), (a,d,b) */
  int faces[3][3] = {{0, 1, 2}, {0, 2, 3}, {0, 3, 1}};
  int opp[3] = {3, 1, 2};
  for (int f = 0; f < 3; f++) {
    double e1[3], e2[3], nn[3], rel[3];
    v3_sub(e1, S[faces[f][1]].w, S[0].w);
    v3_sub(e2, S[faces[f][2]].w, S[0].w);
    v3_cross(nn, e1, e2);
    v3_sub(rel, S[opp[f]].w, S[0].w);
    if (v3_dot(nn, rel) > 0) v3_scl(nn, nn, -1); /* outward */
    if (v3_dot(nn, ao) > 0) {
      sv T[3] = {S[faces[f][0]], S[faces[f][1]], S[faces[f][2]]};
      S[0] = T[0]; S[1] = T[1]; S[2] = T[2];
      *n = 3;
      return gjk_tri(S, n, dir);
    }
  }
  *n = 4;
  return 1;
}

static int gjk(const or_env* e, int g1, int g2, sv* simplex, int* nsimp) {
  double dir[3];
  v3_sub(dir, e->gxpos[g1], e->gxpos[g2]);
  if (v3_norm(dir) < 1e-12) v3_set(dir, 1, 0, 0);
  sv S[4];
  int n = 1;
  mk_sv(e, g1, g2, dir, &S[0]);
  v3_scl(dir, S[0].w, -1);
  for (int it = 0; it < 64; it++) {
    if (v3_norm(dir) < 1e-14) break;
    sv P;
    mk_sv(e, g1, g2, dir, &P);
    if (v3_dot(P.w, dir) < 0) return 0; /* separating axis found */
    for (int i = n; i > 0; i--) S[i] = S[i - 1];
    S[0] = P;
    n++;
    int hit = n == 2 ? gjk_line(S, &n, dir) : n == 3 ? gjk_tri(S, &n, dir) : gjk_tet(S, &n, dir);
    if (hit) {
      *nsimp = n;
      for (int i = 0; i < n; i++) simplex[i] = S[i];
      return 1;
    }
  }
  if (v3_norm(dir) < 1e-14) {
    *nsimp = n;
    for (int i = 0; i < n; i++) simplex[i] = S[i];
    return 1;
  }
  return 0;
}

#define EPA_MAXV 128
#define EPA_MAXF 256
typedef struct { int v[3]; double n[3]; double d; int alive; } epa_face;

static int epa_make_face(sv* V, epa_face* f, int a, int b, int c) {
  f->v[0] = a; f->v[1] = b; f->v[2] = c;
  double ab[3], ac[3];
  v3_sub(ab, V[b].w, V[a].w);
  v3_sub(ac, V[c].w, V[a].w);
  v3_cross(f->n, ab, ac);
  double ln = v3_norm(f->n);
  if (ln < 1e-18) { f->alive = 0; return 0; }
  v3_scl(f->n, f->n, 1.0 / ln);
  f->d = v3_dot(f->n, V[a].w);
  f->alive = 1;
  return 1;
}

static int epa(const or_env* e, int g1, int g2, sv* simplex, int nsimp, double* normal, double* depth, double* pa,
               double* pb) {
  sv V[EPA_MAXV];
  epa_face F[EPA_MAXF];
  int nv = nsimp, nf = 0;
  for (int i = 0; i < nsimp; i++) V[i] = simplex[i];
  /* blow up degenerate simplices to a tetrahedron */
  static const double dirs[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
  if (nv == 1) {
    for (int k = 0; k < 6 && nv < 2; k++) {
      mk_sv(e, g1, g2, dirs[k], &V[nv]);
      double df[3];
      v3_sub(df, V[nv].w, V[0].w);
      if (v3_norm(df) > 1e-10) nv++;
    }
  }
  if (nv == 2) {
    double ab[3], t[3];
    v3_sub(ab, V[1].w, V[0].w);
    int bi = 0;
    double bm = 1e300;
    for (int k = 0; k < 3; k++)
      if (fabs(ab[k]) < bm) { bm = fabs(ab[k]); bi = k; }
    double ax[3] = {0, 0, 0};
    ax[bi] = 1;
    v3_cross(t, ab, ax);
    v3_normalize(t);
    mk_sv(e, g1, g2, t, &V[nv]);
    double df[3];
    v3_sub(df, V[nv].w, V[0].w);
    double cr[3];
    v3_cross(cr, df, ab);
    if (v3_norm(cr) > 1e-12) nv++;
    else {
      v3_scl(t, t, -1);
      mk_sv(e, g1, g2, t, &V[nv]);
      nv++;
    }
  }
  if (nv == 3) {
    double ab[3], ac[3], n[3];
    v3_sub(ab, V[1].w, V[0].w);
    v3_sub(ac, V[2].w, V[0].w);
    v3_cross(n, ab, ac);
    v3_normalize(n);
    mk_sv(e, g1, g2, n, &V[3]);
    double df[3];
    v3_sub(df, V[3].w, V[0].w);
    if (fabs(v3_dot(df, n)) < 1e-12) {
      v3_scl(n, n, -1);
      mk_sv(e, g1, g2, n, &V[3]);
    }
    nv = 4;
  }
  /* initial tetrahedron faces oriented outward */
  int tet[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
  double cen[3] = {0, 0, 0};
  for (int i = 0; i < 4; i++) v3_addscl(cen, cen, V[i].w, 0.25);
  for (int i = 0; i < 4; i++) {
    epa_make_face(V, &F[nf], tet[i][0], tet[i][1], tet[i][2]);
    double rel[3];
    v3_sub(rel, V[tet[i][0]].w, cen);
    if (v3_dot(F[nf].n, rel) < 0) epa_make_face(V, &F[nf], tet[i][0], tet[i][2], tet[i][1]);
    nf++;
  }
  int best = -1;
  for (int it = 0; it < 100; it++) {
    best = -1;
    double bd = 1e300;
    for (int i = 0; i < nf; i++)
      if (F[i].alive && F[i].d < bd) { bd = F[i].d; best = i; }
    if (best < 0) return 0;
    sv P;
    mk_sv(e, g1, g2, F[best].n, &P);
    double dist = v3_dot(P.w, F[best].n);
    if (dist - F[best].d < 1e-10 || nv >= EPA_MAXV) break;
    /* remove faces visible from P, collect horizon */
    int edges[EPA_MAXF * 3][2];
    int ne = 0;
    for (int i = 0; i < nf; i++) {
      if (!F[i].alive) continue;
      double rel[3];
      v3_sub(rel, P.w, V[F[i].v[0]].w);
      if (v3_dot(F[i].n, rel) > 1e-14) {
        F[i].alive = 0;
        for (int k = 0; k < 3; k++) {
          int a = F[i].v[k], b = F[i].v[(k + 1) % 3];
          int found = -1;
          for (int q = 0; q < ne; q++)
            if (edges[q][0] == b && edges[q][1] == a) { found = q; break; }
          if (found >= 0) { edges[found][0] = edges[ne - 1][0]; edges[found][1] = edges[ne - 1][1]; ne--; }
          else { edges[ne][0] = a; edges[ne][1] = b; ne++; }
        }
      }
    }
    int pi = nv++;
    V[pi] = P;
    /* compact faces */
    int m = 0;
    for (int i = 0; i < nf; i++)
      if (F[i].alive) F[m++] = F[i];
    nf = m;
    for (int q = 0; q < ne && nf < EPA_MAXF; q++)
      if (epa_make_face(V, &F[nf], edges[q][0], edges[q][1], pi)) nf++;
  }
  if (best < 0) return 0;
  epa_face* f = &F[best];
  /* barycentric coordinates of the origin's projection on the face */
  double p[3];
  v3_scl(p, f->n, f->d);
  const double* A = V[f->v[0]].w;
  const double* B = V[f->v[1]].w;
  const double* C = V[f->v[2]].w;
  double v0[3], v1[3], v2[3];
  v3_sub(v0, B, A);
  v3_sub(v1, C, A);
  v3_sub(v2, p, A);
  double d00 = v3_dot(v0, v0), d01 = v3_dot(v0, v1), d11 = v3_dot(v1, v1);
  double d20 = v3_dot(v2, v0), d21 = v3_dot(v2, v1);
  double den = d00 * d11 - d01 * d01;
  double lv = den > 1e-30 ? (d11 * d20 - d01 * d21) / den : 0;
  double lw = den > 1e-30 ? (d00 * d21 - d01 * d20) / den : 0;
  double lu = 1 - lv - lw;
  for (int k = 0; k < 3; k++) {
    pa[k] = lu * V[f->v[0]].a[k] + lv * V[f->v[1]].a[k] + lw * V[f->v[2]].a[k];
    pb[k] = lu * V[f->v[0]].b[k] + lv * V[f->v[1]].b[k] + lw * V[f->v[2]].b[k];
  }
  v3_copy(normal, f->n);
  *depth = f->d;
  return 1;
}

static void convex_convex(or_env* e, int g1, int g2) {
  sv simplex[4];
  int ns = 0;
  if (!gjk(e, g1, g2, simplex, &ns)) return;
  double n[3], depth, pa[3], pb[3];
  if (!epa(e, g1, g2, simplex, ns, n, &depth, pa, pb)) return;
  if (depth < 0) return;
  double pos[3];
  v3_add(pos, pa, pb);
  v3_scl(pos, pos, 0.5);
  /* Minkowski A-B face normal n: translating B by +depth*n separates -> normal A->B is n */
  add_contact(e, g1, g2, -depth, pos, n);
}

/* ------------------------------------------------------------------ driver */
void or_collision(or_env* e) {
  e->ncon = 0;
  for (int p = 0; p < OM_NPAIR; p++) {
    int g1 = OM_pair_geom[2 * p], g2 = OM_pair_geom[2 * p + 1];
    int t1 = OM_geom_type[g1], t2 = OM_geom_type[g2];
    if (t1 > t2) { int t = g1; g1 = g2; g2 = t; t = t1; t1 = t2; t2 = t; }
    if (t1 == GT_PLANE) {
      /* plane vs geom: bounding-sphere distance to the plane */
      double nz[3] = {e->gxmat[g1][2], e->gxmat[g1][5], e->gxmat[g1][8]};
      double rel[3];
      v3_sub(rel, e->gxpos[g2], e->gxpos[g1]);
      if (v3_dot(rel, nz) > OM_geom_rbound[g2]) continue;
      if (t2 == GT_BOX) plane_box(e, g1, g2);
      else if (t2 == GT_MESH) plane_convex(e, g1, g2);
      continue;
    }
    double d[3];
    v3_sub(d, e->gxpos[g2], e->gxpos[g1]);
    double rb = OM_geom_rbound[g1] + OM_geom_rbound[g2];
    if (v3_dot(d, d) > rb * rb) continue;
    if (!obb_overlap(e, g1, g2)) continue;
    if (t1 == GT_BOX && t2 == GT_BOX) box_box(e, g1, g2);
    else convex_convex(e, g1, g2);
  }
}
