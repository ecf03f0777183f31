/* ORACLE (test infrastructure only): small fp64 vector/matrix helpers.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * anything under oracle/.  Conventions follow MuJoCo: quaternions are (w,x,y,z),
 * 3x3 matrices row-major. */
#ifndef OR_MATH_H
#define OR_MATH_H
#include <math.h>
#include <string.h>

static inline void v3_set(double* r, double x, double y, double z) { r[0] = x; r[1] = y; r[2] = z; }
static inline void v3_copy(double* r, const double* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
static inline void v3_add(double* r, const double* a, const double* b) { r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
static inline void v3_sub(double* r, const double* a, const double* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
static inline void v3_scl(double* r, const double* a, double s) { r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
static inline void v3_addscl(double* r, const double* a, const double* b, double s) { r[0] = a[0] + b[0] * s; r[1] = a[1] + b[1] * s; r[2] = a[2] + b[2] * s; }
static inline double v3_dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline double v3_norm(const double* a) { return sqrt(v3_dot(a, a)); }
static inline void v3_cross(double* r, const double* a, const double* b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  v3_copy(r, t);
}
static inline double v3_normalize(double* a) {
  double n = v3_norm(a);
  if (n < 1e-15) { a[0] = 1; a[1] = 0; a[2] = 0; return 0; }
  v3_scl(a, a, 1.0 / n);
  return n;
}
/* r = M a  (M row-major 3x3) */
static inline void m3_mulv(double* r, const double* M, const double* a) {
  double t[3] = {M[0] * a[0] + M[1] * a[1] + M[2] * a[2], M[3] * a[0] + M[4] * a[1] + M[5] * a[2],
                 M[6] * a[0] + M[7] * a[1] + M[8] * a[2]};
  v3_copy(r, t);
}
/* r = M^T a */
static inline void m3_mulTv(double* r, const double* M, const double* a) {
  double t[3] = {M[0] * a[0] + M[3] * a[1] + M[6] * a[2], M[1] * a[0] + M[4] * a[1] + M[7] * a[2],
                 M[2] * a[0] + M[5] * a[1] + M[8] * a[2]};
  v3_copy(r, t);
}
static inline void m3_mul(double* R, const double* A, const double* B) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(R, t, sizeof(t));
}
/* R = A^T B */
static inline void m3_mulT(double* R, const double* A, const double* B) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[i] * B[j] + A[3 + i] * B[3 + j] + A[6 + i] * B[6 + j];
  memcpy(R, t, sizeof(t));
}
static inline void m3_transpose(double* R, const double* A) {
  double t[9] = {A[0], A[3], A[6], A[1], A[4], A[7], A[2], A[5], A[8]};
  memcpy(R, t, sizeof(t));
}
static inline void q_normalize(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < 1e-15) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static inline void q_mul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof(t));
}
static inline void q_to_mat(double* R, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}
static inline void q_axis_angle(double* q, const double* axis, double ang) {
  double s = sin(0.5 * ang);
  q[0] = cos(0.5 * ang); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
/* orthonormal frame with n as first row: MuJoCo mju_makeFrame semantics */
static inline void make_frame(double* f, const double* n) {
  double y[3];
  v3_copy(f, n);
  if (n[1] < 0.5 && n[1] > -0.5) v3_set(y, 0, 1, 0); else v3_set(y, 0, 0, 1);
  double d = v3_dot(n, y);
  v3_addscl(y, y, n, -d);
  v3_normalize(y);
  v3_copy(f + 3, y);
  v3_cross(f + 6, n, y);
}
/* dense Cholesky (lower, in place on a copy), returns 0 on success */
static inline int chol_factor(double* L, int n) {
  for (int j = 0; j < n; j++) {
    double s = L[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
    if (s <= 0) return -1;
    double d = sqrt(s);
    L[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = L[i * n + j];
      for (int k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = t / d;
    }
  }
  return 0;
}
static inline void chol_solve(const double* L, int n, double* x) {
  for (int i = 0; i < n; i++) {
    double s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}
#endif
