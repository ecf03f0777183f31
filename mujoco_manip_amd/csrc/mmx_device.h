// Device math helpers for the MI355X kernels (fp32, per-lane scalars).
#ifndef MMX_DEVICE_H
#define MMX_DEVICE_H
#include <hip/hip_runtime.h>

#define DEV __device__ __forceinline__

struct V3 {
  float x, y, z;
};
DEV V3 v3(float x, float y, float z) { return V3{x, y, z}; }
DEV V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
DEV V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
DEV V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
DEV V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
DEV V3 operator*(float s, V3 a) { return V3{a.x * s, a.y * s, a.z * s}; }
DEV float dot(V3 a, V3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
DEV V3 cross(V3 a, V3 b) {
  return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
DEV float norm(V3 a) { return sqrtf(dot(a, a)); }
DEV V3 normalize(V3 a) {
  float n = norm(a);
  return n > 1e-20f ? a * (1.0f / n) : V3{1.f, 0.f, 0.f};
}

// 3x3 row-major
struct M3 {
  float m[9];
};
DEV V3 mul(const M3& R, V3 a) {
  return V3{R.m[0] * a.x + R.m[1] * a.y + R.m[2] * a.z, R.m[3] * a.x + R.m[4] * a.y + R.m[5] * a.z,
            R.m[6] * a.x + R.m[7] * a.y + R.m[8] * a.z};
}
DEV V3 mulT(const M3& R, V3 a) {
  return V3{R.m[0] * a.x + R.m[3] * a.y + R.m[6] * a.z, R.m[1] * a.x + R.m[4] * a.y + R.m[7] * a.z,
            R.m[2] * a.x + R.m[5] * a.y + R.m[8] * a.z};
}
DEV M3 mul(const M3& A, const M3& B) {
  M3 C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
  return C;
}
DEV V3 col(const M3& R, int k) { return V3{R.m[k], R.m[3 + k], R.m[6 + k]}; }

struct Q4 {
  float w, x, y, z;
};
DEV Q4 qmul(Q4 a, Q4 b) {
  return Q4{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x, a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}
DEV Q4 qnormalize(Q4 q) {
  float n = sqrtf(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  if (n < 1e-20f) return Q4{1.f, 0.f, 0.f, 0.f};
  float s = 1.0f / n;
  return Q4{q.w * s, q.x * s, q.y * s, q.z * s};
}
DEV M3 qmat(Q4 q) {
  float w = q.w, x = q.x, y = q.y, z = q.z;
  M3 R;
  R.m[0] = 1 - 2 * (y * y + z * z); R.m[1] = 2 * (x * y - z * w); R.m[2] = 2 * (x * z + y * w);
  R.m[3] = 2 * (x * y + z * w); R.m[4] = 1 - 2 * (x * x + z * z); R.m[5] = 2 * (y * z - x * w);
  R.m[6] = 2 * (x * z - y * w); R.m[7] = 2 * (y * z + x * w); R.m[8] = 1 - 2 * (x * x + y * y);
  return R;
}
DEV Q4 qaxisangle(V3 a, float ang) {
  float s, c;
  sincosf(0.5f * ang, &s, &c);
  return Q4{c, a.x * s, a.y * s, a.z * s};
}

// spatial motion / force in world-origin Plucker coordinates: (angular, linear)
struct SV {
  V3 w, v;
};
DEV SV operator+(SV a, SV b) { return SV{a.w + b.w, a.v + b.v}; }
DEV SV operator*(SV a, float s) { return SV{a.w * s, a.v * s}; }
DEV float sdot(SV m, SV f) { return dot(m.w, f.w) + dot(m.v, f.v); }
DEV SV cross_motion(SV a, SV b) { return SV{cross(a.w, b.w), cross(a.w, b.v) + cross(a.v, b.w)}; }
DEV SV cross_force(SV a, SV f) { return SV{cross(a.w, f.w) + cross(a.v, f.v), cross(a.w, f.v)}; }

// rigid-body inertia at the world origin: mass, first moment h = m c, rotational J_o (sym)
struct RI {
  float m;
  V3 h;
  float J[6];  // xx yy zz xy xz yz
};
DEV V3 symmul(const float* J, V3 a) {
  return V3{J[0] * a.x + J[3] * a.y + J[4] * a.z, J[3] * a.x + J[1] * a.y + J[5] * a.z,
            J[4] * a.x + J[5] * a.y + J[2] * a.z};
}
DEV SV rimul(const RI& I, SV s) { return SV{symmul(I.J, s.w) + cross(I.h, s.v), s.v * I.m - cross(I.h, s.w)}; }
DEV void riadd(RI& a, const RI& b) {
  a.m += b.m;
  a.h = a.h + b.h;
#pragma unroll
  for (int k = 0; k < 6; k++) a.J[k] += b.J[k];
}

#endif
