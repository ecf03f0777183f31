/* ORACLE (test infrastructure only) — fp64 restatement of mujoco.mj_step / mj_forward
 * for the pick-and-place model (called at mujoco_manip/env.py:117,121,161 and
 * mujoco_manip/gym_env.py:560).  MuJoCo 3.5.0 is an un-vendored dependency
 * (uv.lock:985-986); this file restates its documented pipeline:
 *   fwdPosition:  kinematics, com/cdof, tendon, CRBA (+armature), collision, constraints
 *   fwdVelocity:  RNE bias, passive damping
 *   fwdActuation: clamped ctrl -> gain/bias -> clamped force -> moment^T force
 *   fwdConstraint: primal Newton solver with exact line search (MuJoCo's default solver)
 *   implicitfast: (M - h qDeriv) qacc = qfrc_smooth + qfrc_constraint ; mj_advance
 * Spatial algebra uses world-origin Plucker coordinates (an equivalent coordinate
 * choice to MuJoCo's com-based frames; qM and qfrc_bias are coordinate-free). */
#include <stdlib.h>
#include <stdio.h>
#include "or_internal.h"

/* ------------------------------------------------------------------ kinematics */
void or_kinematics(or_env* e) {
  v3_set(e->xpos[0], 0, 0, 0);
  e->xquat[0][0] = 1; e->xquat[0][1] = e->xquat[0][2] = e->xquat[0][3] = 0;
  q_to_mat(e->xmat[0], e->xquat[0]);
  v3_set(e->xipos[0], 0, 0, 0);
  for (int b = 1; b < NB; b++) {
    int p = OM_body_parent[b];
    double pos[3], quat[4], tmp[3];
    m3_mulv(tmp, e->xmat[p], &OM_body_pos[3 * b]);
    v3_add(pos, e->xpos[p], tmp);
    q_mul(quat, e->xquat[p], &OM_body_quat[4 * b]);
    int j = OM_body_jnt[b];
    if (j >= 0) {
      int qa = OM_jnt_qposadr[j];
      int type = OM_jnt_type[j];
      if (type == 0) { /* free */
        v3_copy(pos, &e->qpos[qa]);
        for (int k = 0; k < 4; k++) quat[k] = e->qpos[qa + 3 + k];
        q_normalize(quat);
        v3_copy(e->janchor[j], pos);
      } else {
        double R[9];
        q_normalize(quat);
        q_to_mat(R, quat);
        m3_mulv(tmp, R, &OM_jnt_pos[3 * j]);
        v3_add(e->janchor[j], pos, tmp);
        m3_mulv(e->jaxis[j], R, &OM_jnt_axis[3 * j]);
        double qv = e->qpos[qa] - OM_qpos0[qa];
        if (type == 3) { /* hinge: rotate about the local axis, keep the anchor fixed */
          double qloc[4];
          q_axis_angle(qloc, &OM_jnt_axis[3 * j], qv);
          q_mul(quat, quat, qloc);
          q_normalize(quat);
          q_to_mat(R, quat);
          m3_mulv(tmp, R, &OM_jnt_pos[3 * j]);
          v3_sub(pos, e->janchor[j], tmp);
        } else { /* slide */
          v3_addscl(pos, pos, e->jaxis[j], qv);
        }
      }
    }
    q_normalize(quat);
    v3_copy(e->xpos[b], pos);
    memcpy(e->xquat[b], quat, sizeof(quat));
    q_to_mat(e->xmat[b], quat);
    m3_mulv(tmp, e->xmat[b], &OM_body_ipos[3 * b]);
    v3_add(e->xipos[b], e->xpos[b], tmp);
  }
  for (int g = 0; g < NG; g++) {
    int b = OM_geom_body[g];
    double tmp[3], R[9];
    m3_mulv(tmp, e->xmat[b], &OM_geom_pos[3 * g]);
    v3_add(e->gxpos[g], e->xpos[b], tmp);
    q_to_mat(R, &OM_geom_quat[4 * g]);
    m3_mul(e->gxmat[g], e->xmat[b], R);
  }
  for (int c = 0; c < NC; c++) {
    int b = OM_cam_body[c];
    double tmp[3], R[9];
    m3_mulv(tmp, e->xmat[b], &OM_cam_pos[3 * c]);
    v3_add(e->camxpos[c], e->xpos[b], tmp);
    q_to_mat(R, &OM_cam_quat[4 * c]);
    m3_mul(e->camxmat[c], e->xmat[b], R);
  }
  /* motion subspaces */
  for (int j = 0; j < NJ; j++) {
    int da = OM_jnt_dofadr[j];
    int type = OM_jnt_type[j];
    if (type == 0) {
      int b = OM_jnt_body[j];
      for (int k = 0; k < 3; k++) {
        double* s = e->cdof[da + k];
        v3_set(s, 0, 0, 0);
        v3_set(s + 3, k == 0, k == 1, k == 2);
        double r[3] = {e->xmat[b][k], e->xmat[b][3 + k], e->xmat[b][6 + k]};
        double* sr = e->cdof[da + 3 + k];
        v3_copy(sr, r);
        v3_cross(sr + 3, e->xpos[b], r);
      }
    } else if (type == 3) {
      double* s = e->cdof[da];
      v3_copy(s, e->jaxis[j]);
      v3_cross(s + 3, e->janchor[j], e->jaxis[j]);
    } else {
      double* s = e->cdof[da];
      v3_set(s, 0, 0, 0);
      v3_copy(s + 3, e->jaxis[j]);
    }
  }
}

/* is body a an ancestor of (or equal to) body b */
static int is_ancestor(int a, int b) {
  while (b > 0) {
    if (b == a) return 1;
    b = OM_body_parent[b];
  }
  return a == 0;
}

/* 6x6 spatial inertia of body b at the world origin: [[Ic - m[c]^2, m[c]], [-m[c], m I]] */
static void body_spatial_inertia(const or_env* e, int b, double* I6) {
  memset(I6, 0, 36 * sizeof(double));
  double m = OM_body_mass[b];
  if (m <= 0) return;
  const double* c = e->xipos[b];
  double Ib[9], Ic[9], tmp[9];
  memcpy(Ib, &OM_body_inertia[9 * b], sizeof(Ib));
  m3_mul(tmp, e->xmat[b], Ib);
  double RT[9];
  m3_transpose(RT, e->xmat[b]);
  m3_mul(Ic, tmp, RT);
  double C[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
  double CC[9];
  m3_mul(CC, C, C);
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) {
      I6[6 * i + k] = Ic[3 * i + k] - m * CC[3 * i + k];
      I6[6 * i + 3 + k] = m * C[3 * i + k];
      I6[6 * (3 + i) + k] = -m * C[3 * i + k];
      I6[6 * (3 + i) + 3 + k] = (i == k) ? m : 0;
    }
}

static void mat6_vec(double* r, const double* A, const double* v) {
  for (int i = 0; i < 6; i++) {
    double s = 0;
    for (int k = 0; k < 6; k++) s += A[6 * i + k] * v[k];
    r[i] = s;
  }
}
static double sdot(const double* m, const double* f) {
  double s = 0;
  for (int i = 0; i < 6; i++) s += m[i] * f[i];
  return s;
}
/* motion cross: v x m = (w x mw, w x mv + vo x mw) */
static void cross_motion(double* r, const double* v, const double* m) {
  double a[3], b[3], c[3];
  v3_cross(a, v, m);
  v3_cross(b, v, m + 3);
  v3_cross(c, v + 3, m);
  v3_copy(r, a);
  v3_add(r + 3, b, c);
}
/* force cross: v x* f = (w x fn + vo x ff, w x ff) */
static void cross_force(double* r, const double* v, const double* f) {
  double a[3], b[3], c[3];
  v3_cross(a, v, f);
  v3_cross(b, v + 3, f + 3);
  v3_cross(c, v, f + 3);
  v3_add(r, a, b);
  v3_copy(r + 3, c);
}

static void crba(or_env* e) {
  double Ic[NB][36];
  for (int b = 0; b < NB; b++) body_spatial_inertia(e, b, Ic[b]);
  for (int b = NB - 1; b > 0; b--) {
    int p = OM_body_parent[b];
    for (int k = 0; k < 36; k++) Ic[p][k] += Ic[b][k];
  }
  memset(e->M, 0, sizeof(e->M));
  for (int i = 0; i < NV; i++) {
    int bi = OM_dof_body[i];
    double F[6];
    mat6_vec(F, Ic[bi], e->cdof[i]);
    for (int j = 0; j <= i; j++) {
      int bj = OM_dof_body[j];
      if (!is_ancestor(bj, bi)) continue;
      double v = sdot(e->cdof[j], F);
      e->M[i * NV + j] = v;
      e->M[j * NV + i] = v;
    }
    e->M[i * NV + i] += OM_dof_armature[i];
  }
}

static void rne(or_env* e) {
  double v[NB][6], a[NB][6], f[NB][6];
  memset(v[0], 0, sizeof(v[0]));
  memset(a[0], 0, sizeof(a[0]));
  a[0][5] = -OM_GRAVITY_Z; /* base acceleration = -gravity */
  for (int b = 1; b < NB; b++) {
    int p = OM_body_parent[b];
    memcpy(v[b], v[p], sizeof(v[b]));
    memcpy(a[b], a[p], sizeof(a[b]));
    int j = OM_body_jnt[b];
    if (j >= 0) {
      int da = OM_jnt_dofadr[j];
      int type = OM_jnt_type[j];
      if (type == 0) {
        double vt[6] = {0}, vr[6] = {0};
        for (int k = 0; k < 3; k++)
          for (int c = 0; c < 6; c++) {
            vt[c] += e->cdof[da + k][c] * e->qvel[da + k];
            vr[c] += e->cdof[da + 3 + k][c] * e->qvel[da + 3 + k];
          }
        for (int c = 0; c < 6; c++) v[b][c] += vt[c] + vr[c];
        /* translational axes fixed in world; rotational axes fixed in the body */
        double t[6];
        cross_motion(t, v[b], vr);
        for (int c = 0; c < 6; c++) a[b][c] += t[c];
      } else {
        double vj[6], t[6];
        for (int c = 0; c < 6; c++) vj[c] = e->cdof[da][c] * e->qvel[da];
        cross_motion(t, v[p], vj);
        for (int c = 0; c < 6; c++) {
          v[b][c] += vj[c];
          a[b][c] += t[c];
        }
      }
    }
    double I6[36], Iv[6], Ia[6], cf[6];
    body_spatial_inertia(e, b, I6);
    mat6_vec(Ia, I6, a[b]);
    mat6_vec(Iv, I6, v[b]);
    cross_force(cf, v[b], Iv);
    for (int c = 0; c < 6; c++) f[b][c] = Ia[c] + cf[c];
  }
  for (int b = NB - 1; b > 0; b--) {
    int p = OM_body_parent[b];
    for (int c = 0; c < 6; c++) f[p][c] += f[b][c];
  }
  for (int d = 0; d < NV; d++) e->qfrc_bias[d] = sdot(e->cdof[d], f[OM_dof_body[d]]);
}

/* point Jacobian (mj_jac): columns for ancestor dofs, v(p) = v_o + w x p */
void or_point_jac(or_env* e, int body, const double* point, double* jacp, double* jacr) {
  memset(jacp, 0, 3 * NV * sizeof(double));
  memset(jacr, 0, 3 * NV * sizeof(double));
  if (body <= 0) return;
  for (int d = 0; d < NV; d++) {
    if (!is_ancestor(OM_dof_body[d], body)) continue;
    const double* s = e->cdof[d];
    double wp[3];
    v3_cross(wp, s, point);
    for (int k = 0; k < 3; k++) {
      jacp[k * NV + d] = s[3 + k] + wp[k];
      jacr[k * NV + d] = s[k];
    }
  }
}

static void tendon(or_env* e) {
  memset(e->ten_moment, 0, sizeof(e->ten_moment));
  e->ten_len = 0;
  for (int k = 0; k < 2; k++) {
    int j = OM_tendon_jnt[k];
    e->ten_len += OM_tendon_coef[k] * e->qpos[OM_jnt_qposadr[j]];
    e->ten_moment[OM_jnt_dofadr[j]] += OM_tendon_coef[k];
  }
}

static void actuation(or_env* e) {
  memset(e->qfrc_act, 0, sizeof(e->qfrc_act));
  for (int i = 0; i < NU; i++) {
    double c = e->ctrl[i];
    const double* cr = &OM_act_ctrlrange[2 * i];
    if (c < cr[0]) c = cr[0];
    if (c > cr[1]) c = cr[1];
    double len, vel;
    int j = OM_act_trn_joint[i];
    if (j >= 0) {
      len = e->qpos[OM_jnt_qposadr[j]];
      vel = e->qvel[OM_jnt_dofadr[j]];
    } else {
      len = e->ten_len;
      vel = 0;
      for (int d = 0; d < NV; d++) vel += e->ten_moment[d] * e->qvel[d];
    }
    const double* bp = &OM_act_bias[3 * i];
    double f = OM_act_gain[i] * c + bp[0] + bp[1] * len + bp[2] * vel;
    e->act_raw[i] = f;
    const double* fr = &OM_act_forcerange[2 * i];
    if (f < fr[0]) f = fr[0];
    if (f > fr[1]) f = fr[1];
    e->act_force[i] = f;
    if (j >= 0) e->qfrc_act[OM_jnt_dofadr[j]] += f;
    else
      for (int d = 0; d < NV; d++) e->qfrc_act[d] += e->ten_moment[d] * f;
  }
}

/* ------------------------------------------------------------------ constraints */
static void impedance(const double* solimp, double pos, double* imp) {
  double dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (dmin < 1e-4) dmin = 1e-4;
  if (dmin > 0.9999) dmin = 0.9999;
  if (dmax < 1e-4) dmax = 1e-4;
  if (dmax > 0.9999) dmax = 0.9999;
  if (dmin == dmax || width <= MINVAL) { *imp = 0.5 * (dmin + dmax); return; }
  double x = fabs(pos / width);
  if (x >= 1) { *imp = dmax; return; }
  if (x <= 0) { *imp = dmin; return; }
  double y;
  if (power == 1) y = x;
  else if (x <= mid) y = pow(x, power) / pow(mid, power - 1);
  else y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  *imp = dmin + y * (dmax - dmin);
}

static void add_row(or_env* e, int type, const double* J, double pos, double diag, const double* solref,
                    const double* solimp) {
  if (e->nefc >= OR_MAXEFC) return;
  int i = e->nefc++;
  memcpy(e->efc_J[i], J, NV * sizeof(double));
  e->efc_type[i] = type;
  e->efc_pos[i] = pos;
  double vel = 0;
  for (int d = 0; d < NV; d++) vel += J[d] * e->qvel[d];
  e->efc_vel[i] = vel;
  double imp;
  impedance(solimp, pos, &imp);
  double dmax = solimp[1];
  if (dmax < 1e-4) dmax = 1e-4;
  if (dmax > 0.9999) dmax = 0.9999;
  double tc = solref[0], dr = solref[1];
  if (tc < 2 * OM_TIMESTEP) tc = 2 * OM_TIMESTEP;
  double K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
  double B = 2.0 / (dmax * tc);
  e->efc_aref[i] = -B * vel - K * imp * pos;
  double R = (1 - imp) / imp * diag;
  if (R < MINVAL) R = MINVAL;
  e->efc_R[i] = R;
  e->efc_D[i] = 1.0 / R;
}

static const double DEF_SOLREF[2] = {0.02, 1.0};
static const double DEF_SOLIMP[5] = {0.9, 0.95, 0.001, 0.5, 2.0};

static void make_constraints(or_env* e) {
  e->nefc = 0;
  double J[NV];
  /* equality: joint coupling finger_joint1 == finger_joint2 (panda.xml:261) */
  {
    int j1 = OM_eq_jnt[0], j2 = OM_eq_jnt[1];
    int d1 = OM_jnt_dofadr[j1], d2 = OM_jnt_dofadr[j2];
    memset(J, 0, sizeof(J));
    J[d1] = 1;
    J[d2] = -1;
    double pos = (e->qpos[OM_jnt_qposadr[j1]] - OM_qpos0[OM_jnt_qposadr[j1]]) -
                 (e->qpos[OM_jnt_qposadr[j2]] - OM_qpos0[OM_jnt_qposadr[j2]]);
    add_row(e, EFC_EQUALITY, J, pos, OM_dof_invweight0[d1] + OM_dof_invweight0[d2], OM_eq_solref, OM_eq_solimp);
  }
  /* joint limits */
  for (int j = 0; j < NJ; j++) {
    if (!OM_jnt_limited[j]) continue;
    int d = OM_jnt_dofadr[j];
    double q = e->qpos[OM_jnt_qposadr[j]];
    for (int side = 0; side < 2; side++) {
      double dist = side == 0 ? q - OM_jnt_range[2 * j] : OM_jnt_range[2 * j + 1] - q;
      if (dist < 0) {
        memset(J, 0, sizeof(J));
        J[d] = side == 0 ? 1 : -1;
        add_row(e, EFC_LIMIT, J, dist, OM_dof_invweight0[d], DEF_SOLREF, DEF_SOLIMP);
      }
    }
  }
  /* contacts: pyramidal cone, rows J_n +/- mu_k J_k */
  for (int c = 0; c < e->ncon; c++) {
    or_contact* con = &e->con[c];
    int b1 = OM_geom_body[con->geom[0]], b2 = OM_geom_body[con->geom[1]];
    double jp1[3 * NV], jr1[3 * NV], jp2[3 * NV], jr2[3 * NV];
    or_point_jac(e, b1, con->pos, jp1, jr1);
    or_point_jac(e, b2, con->pos, jp2, jr2);
    double Jt[3][NV], Jr[3][NV];
    for (int k = 0; k < 3; k++)
      for (int d = 0; d < NV; d++) {
        double dp[3] = {jp2[0 * NV + d] - jp1[0 * NV + d], jp2[1 * NV + d] - jp1[1 * NV + d],
                        jp2[2 * NV + d] - jp1[2 * NV + d]};
        double dr[3] = {jr2[0 * NV + d] - jr1[0 * NV + d], jr2[1 * NV + d] - jr1[1 * NV + d],
                        jr2[2 * NV + d] - jr1[2 * NV + d]};
        Jt[k][d] = v3_dot(&con->frame[3 * k], dp);
        Jr[k][d] = v3_dot(&con->frame[3 * k], dr);
      }
    double tran = OM_body_invweight0[2 * b1] + OM_body_invweight0[2 * b2];
    double rot = OM_body_invweight0[2 * b1 + 1] + OM_body_invweight0[2 * b2 + 1];
    if (con->dim == 1) {
      add_row(e, EFC_CONTACT, Jt[0], con->dist, tran, con->solref, con->solimp);
      continue;
    }
    /* Pyramidal regulariser (MuJoCo documentation, Computation / soft constraints: R = (1 - d) / d
     * * A_hat): every edge of a pyramidal contact shares A_hat = 2 mu0^2 (t + mu0^2 t) / impratio,
     * t = the bodies' translational invweight0, impratio = 1 (neither pick_and_place_scene.xml nor
     * panda.xml sets <option impratio>).  Checked by tests/test_physics_kat.py against closed-form
     * answers derived from these equations: the resting cubes' penetration (24 edges x D aref =
     * m g), every contact edge's R at that depth, and the first substep of a slow slide (the primal
     * problem with all 24 edges active), each on this oracle and on the HIP kernel. */
    (void)rot;
    const double mu0 = con->friction[0];
    const double diag = 2.0 * mu0 * mu0 / OR_IMPRATIO * (tran + mu0 * mu0 * tran);
    for (int k = 0; k < con->dim - 1; k++) {
      const double* Jk = k < 2 ? Jt[k + 1] : Jr[0];
      double mu = con->friction[k];
      for (int s = 0; s < 2; s++) {
        double sg = s == 0 ? 1 : -1;
        for (int d = 0; d < NV; d++) J[d] = Jt[0][d] + sg * mu * Jk[d];
        add_row(e, EFC_CONTACT, J, con->dist, diag, con->solref, con->solimp);
      }
    }
  }
}

/* ------------------------------------------------------------------ Newton solver */
static void Mmul(const or_env* e, const double* x, double* r) {
  for (int i = 0; i < NV; i++) {
    double s = 0;
    for (int k = 0; k < NV; k++) s += e->M[i * NV + k] * x[k];
    r[i] = s;
  }
}

static double cost_at(const or_env* e, const double* x) {
  double dx[NV], Mdx[NV];
  for (int i = 0; i < NV; i++) dx[i] = x[i] - e->qacc_smooth[i];
  Mmul(e, dx, Mdx);
  double c = 0;
  for (int i = 0; i < NV; i++) c += 0.5 * dx[i] * Mdx[i];
  for (int r = 0; r < e->nefc; r++) {
    double v = -e->efc_aref[r];
    for (int d = 0; d < NV; d++) v += e->efc_J[r][d] * x[d];
    if (e->efc_type[r] == EFC_EQUALITY || v < 0) c += 0.5 * e->efc_D[r] * v * v;
  }
  return c;
}

static int cmp_dbl_idx(const void* a, const void* b) {
  const double* x = (const double*)a;
  const double* y = (const double*)b;
  return (x[0] > y[0]) - (x[0] < y[0]);
}

/* Primal Newton with exact line search (MuJoCo's default solver, mj_solNewton), warm-started from
 * the cheaper of qacc_warmstart and qacc_smooth.  Convergence: the relative gradient test
 * |g| / (1 + |qfrc_smooth|) < solver_tol (the parity tests' fully converged solve, 1e-13), and, when
 * solver_mj_tol > 0, MuJoCo's own tests at opt.tolerance: after an iteration, stop when its cost
 * decrease or the gradient norm, both scaled by 1 / (meaninertia * nv) (mj_setConst's
 * stat.meaninertia: the mean diagonal of qM at qpos0), is below the tolerance (MuJoCo records the
 * two per iteration as mjSolverStat.improvement / .gradient). */
static void solve_newton(or_env* e) {
  int n = e->nefc;
  double x[NV];
  const double c_ws = cost_at(e, e->qacc_ws), c_s = cost_at(e, e->qacc_smooth);
  if (c_ws < c_s) memcpy(x, e->qacc_ws, sizeof(x));
  else memcpy(x, e->qacc_smooth, sizeof(x));
  const double mjscale = 1.0 / (OM_MEANINERTIA * NV);
  double cost_old = c_ws < c_s ? c_ws : c_s;
  double r[OR_MAXEFC], s[OR_MAXEFC], bp[OR_MAXEFC][2];
  double res = 0;
  int it;
  for (it = 0; it < e->solver_maxiter; it++) {
    double g[NV], dx[NV];
    for (int i = 0; i < NV; i++) dx[i] = x[i] - e->qacc_smooth[i];
    Mmul(e, dx, g);
    double H[NV * NV];
    memcpy(H, e->M, sizeof(H));
    for (int k = 0; k < n; k++) {
      double v = -e->efc_aref[k];
      for (int d = 0; d < NV; d++) v += e->efc_J[k][d] * x[d];
      r[k] = v;
      if (e->efc_type[k] == EFC_EQUALITY || v < 0) {
        double D = e->efc_D[k];
        for (int d = 0; d < NV; d++) {
          double Jd = e->efc_J[k][d];
          if (Jd == 0) continue;
          g[d] += D * v * Jd;
          for (int d2 = 0; d2 < NV; d2++) H[d * NV + d2] += D * Jd * e->efc_J[k][d2];
        }
      }
    }
    double gn = 0, sc = 0;
    for (int d = 0; d < NV; d++) {
      gn += g[d] * g[d];
      sc += e->qfrc_smooth[d] * e->qfrc_smooth[d];
    }
    res = sqrt(gn) / (1 + sqrt(sc));
    if (res < e->solver_tol) break;
    if (e->solver_mj_tol > 0 && it > 0 && mjscale * sqrt(gn) < e->solver_mj_tol) break;
    if (chol_factor(H, NV) != 0) break;
    double p[NV];
    for (int d = 0; d < NV; d++) p[d] = -g[d];
    chol_solve(H, NV, p);
    /* exact line search on the convex piecewise-quadratic cost */
    double Mp[NV];
    Mmul(e, p, Mp);
    double c0 = 0, c1 = 0;
    for (int d = 0; d < NV; d++) {
      c0 += Mp[d] * dx[d];
      c1 += Mp[d] * p[d];
    }
    int nb = 0;
    for (int k = 0; k < n; k++) {
      double sk = 0;
      for (int d = 0; d < NV; d++) sk += e->efc_J[k][d] * p[d];
      s[k] = sk;
      double D = e->efc_D[k];
      int eq = e->efc_type[k] == EFC_EQUALITY;
      int active0 = eq || r[k] < 0 || (r[k] == 0 && sk < 0);
      if (active0) {
        c0 += D * sk * r[k];
        c1 += D * sk * sk;
      }
      if (!eq && sk != 0) {
        double a = -r[k] / sk;
        if (a > 0) {
          bp[nb][0] = a;
          bp[nb][1] = k;
          nb++;
        }
      }
    }
    qsort(bp, nb, sizeof(bp[0]), cmp_dbl_idx);
    double alpha = c1 > 0 ? -c0 / c1 : 0;
    for (int q = 0; q < nb; q++) {
      if (c1 > 0 && -c0 / c1 <= bp[q][0]) break;
      int k = (int)bp[q][1];
      double D = e->efc_D[k], sk = s[k];
      int was_active = r[k] < 0 || (r[k] == 0 && sk < 0);
      if (was_active) { /* leaves the active set (sk>0) */
        c0 -= D * sk * r[k];
        c1 -= D * sk * sk;
      } else { /* enters (sk<0) */
        c0 += D * sk * r[k];
        c1 += D * sk * sk;
      }
      alpha = c1 > 0 ? -c0 / c1 : bp[q][0];
    }
    double step = 0;
    for (int d = 0; d < NV; d++) {
      x[d] += alpha * p[d];
      step += alpha * alpha * p[d] * p[d];
    }
    if (sqrt(step) < 1e-15) { it++; break; }
    if (e->solver_mj_tol > 0) {
      const double c = cost_at(e, x);
      const double improvement = mjscale * (cost_old - c);
      cost_old = c;
      if (improvement < e->solver_mj_tol) { it++; break; }
    }
  }
  e->solver_res = res;
  e->solver_iter = it;
  e->solver_calls++;
  e->solver_iters_total += it;
  memcpy(e->qacc, x, sizeof(x));
  memset(e->qfrc_constraint, 0, sizeof(e->qfrc_constraint));
  for (int k = 0; k < n; k++) {
    double v = -e->efc_aref[k];
    for (int d = 0; d < NV; d++) v += e->efc_J[k][d] * x[d];
    double f = 0;
    if (e->efc_type[k] == EFC_EQUALITY || v < 0) f = -e->efc_D[k] * v;
    e->efc_force[k] = f;
    for (int d = 0; d < NV; d++) e->qfrc_constraint[d] += e->efc_J[k][d] * f;
  }
}

/* ------------------------------------------------------------------ pipeline */
static void solve_M(const or_env* e, const double* rhs, double* x) {
  double L[NV * NV];
  memcpy(L, e->M, sizeof(L));
  chol_factor(L, NV);
  memcpy(x, rhs, NV * sizeof(double));
  chol_solve(L, NV, x);
}

void or_mj_forward(or_env* e) {
  or_kinematics(e);
  tendon(e);
  crba(e);
  or_collision(e);
  make_constraints(e);
  rne(e);
  for (int d = 0; d < NV; d++) e->qfrc_passive[d] = -OM_dof_damping[d] * e->qvel[d];
  actuation(e);
  for (int d = 0; d < NV; d++) e->qfrc_smooth[d] = e->qfrc_passive[d] - e->qfrc_bias[d] + e->qfrc_act[d];
  solve_M(e, e->qfrc_smooth, e->qacc_smooth);
  solve_newton(e);
}

static void implicitfast_advance(or_env* e) {
  const double h = OM_TIMESTEP;
  double MD[NV * NV];
  memcpy(MD, e->M, sizeof(MD));
  /* qDeriv = d(qfrc_passive + qfrc_actuator)/d qvel ; MD = M - h qDeriv */
  for (int d = 0; d < NV; d++) MD[d * NV + d] += h * OM_dof_damping[d];
  for (int i = 0; i < NU; i++) {
    const double* fr = &OM_act_forcerange[2 * i];
    if (e->act_raw[i] <= fr[0] || e->act_raw[i] >= fr[1]) continue; /* clamped: zero derivative */
    double bv = OM_act_bias[3 * i + 2];
    int j = OM_act_trn_joint[i];
    if (j >= 0) {
      int d = OM_jnt_dofadr[j];
      MD[d * NV + d] -= h * bv;
    } else {
      for (int a = 0; a < NV; a++)
        for (int b = 0; b < NV; b++)
          if (e->ten_moment[a] != 0 && e->ten_moment[b] != 0) MD[a * NV + b] -= h * bv * e->ten_moment[a] * e->ten_moment[b];
    }
  }
  double rhs[NV], qacc[NV];
  for (int d = 0; d < NV; d++) rhs[d] = e->qfrc_smooth[d] + e->qfrc_constraint[d];
  chol_factor(MD, NV);
  memcpy(qacc, rhs, sizeof(rhs));
  chol_solve(MD, NV, qacc);
  /* warm start keeps the constraint solver's qacc */
  memcpy(e->qacc_ws, e->qacc, sizeof(e->qacc_ws));
  for (int d = 0; d < NV; d++) e->qvel[d] += h * qacc[d];
  for (int j = 0; j < NJ; j++) {
    int qa = OM_jnt_qposadr[j], da = OM_jnt_dofadr[j];
    if (OM_jnt_type[j] == 0) {
      for (int k = 0; k < 3; k++) e->qpos[qa + k] += h * e->qvel[da + k];
      double w[3] = {e->qvel[da + 3], e->qvel[da + 4], e->qvel[da + 5]};
      double* q = &e->qpos[qa + 3];
      double ang = v3_normalize(w) * h;
      double qr[4];
      q_axis_angle(qr, w, ang);
      q_normalize(q);
      q_mul(q, q, qr);
      q_normalize(q);
    } else {
      e->qpos[qa] += h * e->qvel[da];
    }
  }
}

void or_mj_step(or_env* e) {
  or_mj_forward(e);
  implicitfast_advance(e);
}

void or_reset_keyframe(or_env* e) {
  for (int i = 0; i < NQ; i++) e->qpos[i] = OM_key_qpos[i];
  for (int i = 0; i < NU; i++) e->ctrl[i] = OM_key_ctrl[i];
  memset(e->qvel, 0, sizeof(e->qvel));
  memset(e->qacc_ws, 0, sizeof(e->qacc_ws));
  or_mj_forward(e);
}

/* ------------------------------------------------------------------ accessors */
void or_get_state(or_env* e, double* qpos, double* qvel, double* ctrl, double* qacc_ws) {
  if (qpos) memcpy(qpos, e->qpos, sizeof(e->qpos));
  if (qvel) memcpy(qvel, e->qvel, sizeof(e->qvel));
  if (ctrl) memcpy(ctrl, e->ctrl, sizeof(e->ctrl));
  if (qacc_ws) memcpy(qacc_ws, e->qacc_ws, sizeof(e->qacc_ws));
}
void or_set_state(or_env* e, const double* qpos, const double* qvel, const double* ctrl, const double* qacc_ws) {
  if (qpos) memcpy(e->qpos, qpos, sizeof(e->qpos));
  if (qvel) memcpy(e->qvel, qvel, sizeof(e->qvel));
  if (ctrl) memcpy(e->ctrl, ctrl, sizeof(e->ctrl));
  if (qacc_ws) memcpy(e->qacc_ws, qacc_ws, sizeof(e->qacc_ws));
}
void or_get_body(or_env* e, int body, double* xpos, double* xmat) {
  if (xpos) v3_copy(xpos, e->xpos[body]);
  if (xmat) memcpy(xmat, e->xmat[body], 9 * sizeof(double));
}
int or_ncon(or_env* e) { return e->ncon; }
int or_nefc(or_env* e) { return e->nefc; }
void or_get_contact(or_env* e, int i, int* geom, double* dist, double* pos, double* frame) {
  or_contact* c = &e->con[i];
  geom[0] = c->geom[0];
  geom[1] = c->geom[1];
  *dist = c->dist;
  v3_copy(pos, c->pos);
  memcpy(frame, c->frame, 9 * sizeof(double));
}
void or_get_efc_force(or_env* e, double* f) { memcpy(f, e->efc_force, e->nefc * sizeof(double)); }
double or_solver_residual(or_env* e) { return e->solver_res; }
void or_set_solver(or_env* e, double tol, int maxiter) {
  e->solver_tol = tol;
  e->solver_maxiter = maxiter;
}
void or_set_solver_mj(or_env* e, double mj_tol) { e->solver_mj_tol = mj_tol; }
void or_solver_stats(or_env* e, long* calls, long* iters) {
  *calls = e->solver_calls;
  *iters = e->solver_iters_total;
}
int or_get_efc(or_env* e, int* type, double* pos, double* R, double* aref) {
  for (int i = 0; i < e->nefc; i++) {
    if (type) type[i] = e->efc_type[i];
    if (pos) pos[i] = e->efc_pos[i];
    if (R) R[i] = e->efc_R[i];
    if (aref) aref[i] = e->efc_aref[i];
  }
  return e->nefc;
}
void or_get_qacc(or_env* e, double* qacc) { memcpy(qacc, e->qacc, sizeof(e->qacc)); }
void or_get_mass_matrix(or_env* e, double* M) { memcpy(M, e->M, sizeof(e->M)); }
/* the smooth-force terms of the last forward (tests/test_smooth_dynamics_kat.py pins them against
 * answers derived from the raw MJCF): qfrc_bias (RNE: Coriolis + gravity), qfrc_actuator, qfrc_passive,
 * qacc_smooth, qfrc_constraint (NV each) and the clamped actuator forces (NU) */
void or_get_smooth(or_env* e, double* bias, double* act, double* passive, double* qacc_smooth, double* constraint,
                   double* act_force) {
  memcpy(bias, e->qfrc_bias, NV * sizeof(double));
  memcpy(act, e->qfrc_act, NV * sizeof(double));
  memcpy(passive, e->qfrc_passive, NV * sizeof(double));
  memcpy(qacc_smooth, e->qacc_smooth, NV * sizeof(double));
  memcpy(constraint, e->qfrc_constraint, NV * sizeof(double));
  memcpy(act_force, e->act_force, NU * sizeof(double));
}
