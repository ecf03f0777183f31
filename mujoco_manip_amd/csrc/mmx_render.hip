// Batched camera renderer for gfx950: the overhead and wrist images of
// PickPlaceGymEnv's observation (gym_env.py:295-339 via cameras.py:9-53, mujoco.Renderer).
//
// One workgroup (512 lanes) renders two horizontal bands (up to 8192 px each) of one camera image
// of one env (two workgroups per CU: one rasterises while the other sets up); the bands share the
// setup and take turns in one LDS z-buffer:
//   1. body poses of the env (stored by the step / reset / forward kernels in S.rpose) and the
//      camera pose (overhead: fixed; wrist: on the hand, env.py:52-65) -> LDS;
//   2. all render vertices (tools/compile_render.py: table / bins / cubes as boxes and prisms, the
//      Panda's visual parts as convex pieces / clustered meshes) to camera space and, once
//      per vertex, to the screen (MuJoCo pinhole, fovy, row 0 at the top) -> LDS (screen x, y,
//      1 / depth: the camera-space point is recovered from them where the shading needs it);
//   3. triangles, one lane each: near cull, back-face cull, bounding box, flat face light, then
//      per band into one of two LDS queues by box area;
//   4. small boxes (<= 2048 px): one triangle per 8-lane group, walked column by column (edge
//      functions as planes, 3 FMAs per pixel); depth test = one 32-bit LDS atomicMax per covered
//      pixel on (inverse depth quantised over the camera's depth range : 20 bits | triangle : 12 bits);
//   5. large boxes (table top, bin walls, close-up links) and shading, fused per 16 x 16 tile: the
//      wave walks the large queue with its depth keys in registers, then shades 4 pixels per lane:
//      flat per-face light, MuJoCo's headlight (ambient 0.3, diffuse 0.6) + the scene's directional
//      (0.8) and point (0.4) lights (pick_and_place_scene.xml:6-9,33-36), the floor checker (0.1 m
//      squares), sky gradient elsewhere; RGB u8 and the segment id written as packed dwords.
// Not modelled (documented in DESIGN.md): shadows, specular, reflectance, bin transparency
// (alpha 0.4 -> opaque); the Panda's visual meshes are reduced per part (tools/compile_render.py:
// convex pieces for the links, clustered hand / fingers; robot-mask IoU vs the full meshes in
// tests/test_render.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MMX_MODEL_QUAL static __constant__
#include "mmx_model_gen.h"
#define MMR_QUAL static __constant__
#include "mmx_render_gen.h"
#include "mmx_device.h"
#include "mmx_state.h"

#ifndef MMR_WG
#define MMR_WG 512
#endif
#define RWG MMR_WG
#ifndef MMR_SKIP
#define MMR_SKIP 0  // diagnostic builds only: 1 small-triangle raster, 2 large-triangle raster, 4 shading
#endif
#define RNSLOT 14
static_assert(MMR_NTRI <= 4096, "triangle index must fit the 12-bit depth-key field");
#ifndef MMR_BAND_PX
#define MMR_BAND_PX 8192  // 32 KB z-buffer: LDS for two workgroups per CU
#endif
#ifndef MMR_SMALL_AREA
#define MMR_SMALL_AREA 2048  // measured: 256 -> 2048 px boxes on 16-lane groups, -8 % render time (4096: +9 %)
#endif
static constexpr int kBandPx = MMR_BAND_PX;      // z-buffer pixels per band
#ifndef MMR_ZPAD
// z-buffer row stride Sg + 4 (LDS banks, ds_max_u32 / ds_read_b128, MI355X_MICROARCH.md §LDS): an
// 8-lane group's column walk (w columns x 8 / w rows, w <= 8) then covers 8 distinct banks mod 32, and
// a tile read (16-lane groups of ds_read_b128, rows {r, r + 4, r + 8, r + 12}: kTileRow) 16 distinct
// 4-bank slots mod 64; stride Sg + 1 (r04) left both 2-way
#define MMR_ZPAD 4
#endif
static_assert((sizeof(float4) * MMR_NVERT + sizeof(float) * 19 * 12) % 16 == 0, "z-buffer 16-byte aligned in LDS");
static_assert(MMR_ZPAD % 4 == 0, "z-buffer rows 16-byte aligned: the tile walk reads 4 pixels with one ds_read_b128");
static constexpr int kZbWords = kBandPx + 64 * MMR_ZPAD;  // 64 rows of 128 + ZPAD at S = 128 (rend_band_rows)
static constexpr int kSmallArea = MMR_SMALL_AREA; // bounding boxes up to this many pixels: a 16-lane group
#ifndef MMR_GROUP
#define MMR_GROUP 8  // measured with the column walk: 8 lanes per triangle -3 % render time vs 16
#endif
static constexpr int kGroup = MMR_GROUP;         // lanes per small triangle
static constexpr int kMaxBig = 512;
#ifndef MMR_BIG_CACHE
#define MMR_BIG_CACHE 40  // large-triangle setups kept in LDS per band (what fits beside two workgroups per CU)
#endif
static constexpr int kBigCache = MMR_BIG_CACHE;  // per band; a full queue sends further large triangles to the small path
#ifndef MMR_BPW
#define MMR_BPW 2
#endif
static constexpr int kBPW = MMR_BPW;  // bands per workgroup: vertex and triangle setup shared by them
static_assert(kBPW >= 1 && kBPW <= 4, "nbig holds 3 counters per band");
#ifndef MMR_TINY
#define MMR_TINY 64  // small boxes up to this many pixels queue from the front, the others from the back
#endif
static constexpr int kTiny = MMR_TINY;  // (a wave's 8-lane groups then walk boxes of similar size)
static constexpr int kNbig = 12;        // [2 kb]: large, [2 kb + 1]: small (front), [8 + kb]: small (back)
#ifndef MMR_TPW
#define MMR_TPW 2
#endif
static constexpr int kTPW = MMR_TPW;
// MMR_CLOCK (diagnostic builds only): wave 0 of each workgroup adds its wall-clock ticks (100 MHz)
// per stage into g_rclk: 0 poses / camera / clear, 1 vertices, 2 triangle setup + queues, 3 small
// raster, 4 large triangles + shading, 5 workgroups; read by mmx_render_clock (tools/render_clock.py)
#ifdef MMR_CLOCK
__device__ unsigned long long g_rclk[8];
#define RCLK_DECL unsigned long long rclk_t = wall_clock64(), rclk_acc[5] = {0, 0, 0, 0, 0};
#define RCLK(k) do { const unsigned long long n_ = wall_clock64(); rclk_acc[k] += n_ - rclk_t; rclk_t = n_; } while (0)
#define RCLK_END if (tid == 0) { for (int k_ = 0; k_ < 5; k_++) atomicAdd(&g_rclk[k_], rclk_acc[k_]); atomicAdd(&g_rclk[5], 1ull); }
#else
#define RCLK_DECL
#define RCLK(k)
#define RCLK_END
#endif  // 16 x 16 tiles per wave and pass of the large-triangle queue

// rows per band: the image split into the fewest bands whose rows (stride S + ZPAD) fit the
// z-buffer, balanced
__host__ DEV int rend_band_rows(int S) {
  const int cap = kZbWords / (S + MMR_ZPAD);  // >= 8 for S <= 1024
  const int nb = (S + cap - 1) / cap;
  return (S + nb - 1) / nb;
}
// tile walk: lane quad q = lane / 4 takes tile row kTileRow(q), so that each 16-lane group of a
// ds_read_b128 ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, and + 32) holds rows r, r + 4, r + 8, r + 12
__host__ DEV constexpr int kTileRow(int q) { return (int)((0xFEAB6732DC894510ull >> (4 * q)) & 15); }

struct RTri {  // screen-space setup of one triangle
  float A[3], B[3], C[3];  // edge k (opposite vertex k) as the plane e_k(x, y) = A x + B y + C
  float w[3];              // depth-key weights: q = sum_k e_k w_k + q0 (1 / depth, scaled to [0, 1])
  int bx0, by0, bx1, by1;  // pixel bbox (inclusive), clipped to the rows asked for
};

// Edge function of a -> b as a plane, formed from the lower vertex id to the higher one and negated
// when the triangle walks the edge the other way: the two triangles of a shared edge hold exactly
// opposite coefficients and evaluate them with the same fused ops, so their values at a pixel
// centre are exact negatives and no centre on the edge is missed by both.  (The constant term
// cancels only to the rounding of x0 y1: ~1e-7 of the vertices' pixel coordinates, far below a
// pixel's distance resolution for any edge on screen.)
DEV void rend_edge_plane(float xa, float ya, int ia, float xb, float yb, int ib, float& A, float& B, float& C) {
  const bool fwd = ia < ib;
  const float x0 = fwd ? xa : xb, y0 = fwd ? ya : yb, x1 = fwd ? xb : xa, y1 = fwd ? yb : ya;
  const float sg = fwd ? 1.f : -1.f;
  A = sg * (y0 - y1);
  B = sg * (x1 - x0);
  C = sg * __fsub_rn(__fmul_rn(x0, y1), __fmul_rn(x1, y0));
}
// e_k(x, y) = B y + (A x + C): every path evaluates it in this one order (the x part can be hoisted
// out of a column walk without changing a bit)
DEV float rend_edge_x(const RTri& T, int k, float x) { return fmaf(T.A[k], x, T.C[k]); }
DEV float rend_edge_at(const RTri& T, int k, float x, float y) { return fmaf(T.B[k], y, rend_edge_x(T, k, x)); }
// depth key from the scaled inverse depth q of a covered pixel
DEV uint32_t rend_key_q(int t, float q) {
  const uint32_t d = 1u + (uint32_t)(fminf(fmaxf(q, 0.f), 1.f) * 1048574.f);  // 1 .. 2^20 - 1 (0 = empty)
  return (d << 12) | (uint32_t)t;
}
// depth key from the edge values of a covered pixel
DEV uint32_t rend_key(const RTri& T, int t, float e0, float e1, float e2, float q0) {
  return rend_key_q(t, fmaf(e0, T.w[0], fmaf(e1, T.w[1], fmaf(e2, T.w[2], q0))));
}

// camera-space vertex -> screen (sx, sy, 1 / depth, 1) or (0, 0, 0, 0) behind the near plane
DEV float4 rend_project(float4 c, float f, float half, float znear) {
  const float d = -c.z;
  if (d < znear) return make_float4(0.f, 0.f, 0.f, 0.f);
  const float iz = 1.f / d;
  return make_float4(half + f * c.x * iz, half - f * c.y * iz, iz, 1.f);
}

// the camera-space point of a projected vertex (inverse of rend_project)
DEV float4 rend_unproject(float sx, float sy, float iz, float f, float half) {
  const float d = 1.f / iz;
  return make_float4((sx - half) * d / f, (half - sy) * d / f, -d, 0.f);
}

// setup of triangle (a, b, c) for rows [row0, row1); false = culled (near plane, back face, no
// pixel centre in its box).  iz_scale: depth-key scale (1 / depth range).
DEV bool rend_setup_abc(const float4* vs, int a, int b, int c, int S, int row0, int row1, float iz_scale, RTri& T) {
  const float4 pa = vs[a], pb = vs[b], pc = vs[c];
  if (pa.w == 0.f || pb.w == 0.f || pc.w == 0.f) return false;  // a vertex behind the near plane
  // screen y points down: a counter-clockwise (outward) face has negative signed area
  const float area = (pb.x - pa.x) * (pc.y - pa.y) - (pc.x - pa.x) * (pb.y - pa.y);
  // area < -1e-12 as an integer test of the bits (negative finite values below -1e-12 lie strictly
  // between the bits of -1e-12 and of -Inf): NaN / Inf areas (a diverged env's poses reach the
  // renderer when autoreset is off) are culled whatever the fp-math flags let the compiler assume
  // about fp comparisons; the opaque copy keeps it from reasoning about the bits
  unsigned ab = __float_as_uint(area);
  asm volatile("" : "+v"(ab));
  if (!(ab > 0xAB8CBCCCu && ab < 0xFF800000u)) return false;
  const float mnx = fminf(pa.x, fminf(pb.x, pc.x)), mxx = fmaxf(pa.x, fmaxf(pb.x, pc.x));
  const float mny = fminf(pa.y, fminf(pb.y, pc.y)), mxy = fmaxf(pa.y, fmaxf(pb.y, pc.y));
  // pixel (i, j) has its centre at (i + 0.5, j + 0.5)
  T.bx0 = max(0, (int)ceilf(mnx - 0.5f));
  T.bx1 = min(S - 1, (int)floorf(mxx - 0.5f));
  T.by0 = max(row0, (int)ceilf(mny - 0.5f));
  T.by1 = min(row1 - 1, (int)floorf(mxy - 0.5f));
  rend_edge_plane(pb.x, pb.y, b, pc.x, pc.y, c, T.A[0], T.B[0], T.C[0]);
  rend_edge_plane(pc.x, pc.y, c, pa.x, pa.y, a, T.A[1], T.B[1], T.C[1]);
  rend_edge_plane(pa.x, pa.y, a, pb.x, pb.y, b, T.A[2], T.B[2], T.C[2]);
  const float s = iz_scale / area;  // barycentric e_k / area, times the key scale
  T.w[0] = pa.z * s;
  T.w[1] = pb.z * s;
  T.w[2] = pc.z * s;
  return T.bx0 <= T.bx1 && T.by0 <= T.by1;
}
DEV bool rend_setup(const float4* vs, int t, int S, int row0, int row1, float iz_scale, RTri& T) {
  return rend_setup_abc(vs, MMR_tri[3 * t], MMR_tri[3 * t + 1], MMR_tri[3 * t + 2], S, row0, row1, iz_scale, T);
}

// coverage + depth key of pixel (px, py) for triangle t; 0 = not covered.  q0 = -iz_lo * iz_scale.
DEV uint32_t rend_cover(const RTri& T, int t, int px, int py, float q0) {
  const float x = px + 0.5f, y = py + 0.5f;
  // front faces have negative screen area: inside = every edge function <= 0
  const float e0 = rend_edge_at(T, 0, x, y), e1 = rend_edge_at(T, 1, x, y), e2 = rend_edge_at(T, 2, x, y);
  if (fmaxf(e0, fmaxf(e1, e2)) > 0.f) return 0u;
  return rend_key(T, t, e0, e1, e2, q0);
}

// RGB8 of a colour in [0, 1]^3 (rounded) and a segment id, packed r | g << 8 | b << 16 | seg << 24
DEV uint32_t rend_pack(float r, float g, float b, uint32_t sid) {
  return (uint32_t)(r * 255.f + 0.5f) | ((uint32_t)(g * 255.f + 0.5f) << 8) | ((uint32_t)(b * 255.f + 0.5f) << 16) |
         (sid << 24);
}
// shading of 4 horizontally adjacent pixels (px .. px + 3, py) from their depth keys: a covered
// pixel takes its triangle's packed colour (tinfo: flat face light x material, set up once per
// triangle), an uncovered one the floor's checker where its ray meets the floor (per pixel: the
// floor's normal is world z, so its headlight / directional terms are constants of the camera and
// the point light's cosine is 1.5 / |(0.5, 0.5, 1.5) - p|), the sky gradient elsewhere; RGB u8
// (3 dwords) and segment ids (1 dword)
// background of a pixel no triangle covers, from its world ray dw: the floor's checker where the
// ray meets the floor (the floor's normal is world z, so its headlight / directional terms are
// constants of the camera and the point light's cosine is 1.5 / |(0.5, 0.5, 1.5) - p|), the sky
// gradient elsewhere
DEV uint32_t shade_bg(const V3& dw, const V3& cx, float floor_light0, const float* mrgb) {
  const float s0 = -cx.z / dw.z;  // ray parameter at the floor plane z = 0
  const float fx = cx.x + s0 * dw.x, fy = cx.y + s0 * dw.y;
  if (dw.z < 0.f && fabsf(fx) <= MMR_FLOOR_HALF && fabsf(fy) <= MMR_FLOOR_HALF) {
    const float* mt = mrgb + 8 * MMR_FLOOR_MAT;  // checker (0.1 m squares) under the face lights
    const float ddx = 0.5f - fx, ddy = 0.5f - fy;
    const float light = fminf(floor_light0 + 0.6f * rsqrtf(fmaf(ddx, ddx, fmaf(ddy, ddy, 2.25f))), 3.99f);
    const bool alt = ((int)floorf(fx / mt[6]) + (int)floorf(fy / mt[6])) & 1;
    const float* c = alt ? mt + 3 : mt;
    return rend_pack(fminf(c[0] * light, 1.f), fminf(c[1] * light, 1.f), fminf(c[2] * light, 1.f), (uint32_t)mt[7]);
  }
  const float sky = 0.5f * (dw.z * rsqrtf(dot(dw, dw)) + 1.f);  // skybox gradient (rgb1 top -> rgb2 bottom, scene.xml:17-18)
  return rend_pack(0.3f * sky, 0.5f * sky, 0.7f * sky, 0u);
}
// the world rays of 4 horizontally adjacent pixels (px0 .. px0 + 3, py): the first one's, then steps
// by the camera's x axis / f (one order for every caller: the background table is bit-identical to
// the per-pixel shading)
DEV void rays4(int px0, int py, float half, float f, const M3& cR, V3* dw4) {
  const float rf = 1.f / f;
  const V3 dx = col(cR, 0) * rf;
  V3 dw = mul(cR, V3{(px0 + 0.5f - half) * rf, -(py + 0.5f - half) * rf, -1.f});
  for (int u = 0; u < 4; u++, dw = dw + dx) dw4[u] = dw;
}
// bg: the camera's precomputed background row (fixed cameras), or null (computed per pixel)
DEV void shade4(const uint32_t* keys, int px0, int py, float half, float f, const M3& cR, const V3& cx,
                float floor_light0, const uint32_t* tinfo, const float* mrgb, const uint32_t* bg, uint32_t* rgb_out,
                uint32_t* seg_out, int nvalid) {
  uint32_t pix[4];
  if (bg) {
    for (int u = 0; u < 4; u++) pix[u] = keys[u] != 0u ? tinfo[keys[u] & 4095] : bg[px0 + u];
  } else {
    V3 dw4[4];
    rays4(px0, py, half, f, cR, dw4);
    for (int u = 0; u < 4; u++) pix[u] = keys[u] != 0u ? tinfo[keys[u] & 4095] : shade_bg(dw4[u], cx, floor_light0, mrgb);
  }
  const uint32_t rgbw[3] = {(pix[0] & 0xFFFFFFu) | (pix[1] << 24), ((pix[1] >> 8) & 0xFFFFu) | (pix[2] << 16),
                            ((pix[2] >> 16) & 0xFFu) | (pix[3] << 8)};
  const uint32_t segw = (pix[0] >> 24) | ((pix[1] >> 24) << 8) | ((pix[2] >> 24) << 16) | (pix[3] & 0xFF000000u);
  if (nvalid == 4) {  // the image side is a multiple of 16: 4 whole pixels, dword-aligned
    rgb_out[0] = rgbw[0]; rgb_out[1] = rgbw[1]; rgb_out[2] = rgbw[2];
    seg_out[0] = segw;
  } else {  // other sides: byte stores of the pixels inside the image
    unsigned char* rb = reinterpret_cast<unsigned char*>(rgb_out);
    unsigned char* sb = reinterpret_cast<unsigned char*>(seg_out);
    for (int u = 0; u < nvalid; u++) {
      for (int k = 0; k < 3; k++) rb[3 * u + k] = (unsigned char)(rgbw[(3 * u + k) >> 2] >> (8 * ((3 * u + k) & 3)));
      sb[u] = (unsigned char)(segw >> (8 * u));
    }
  }
}

extern "C" __global__ void __launch_bounds__(RWG) __attribute__((amdgpu_waves_per_eu(2 * RWG / 256, 2 * RWG / 256)))
mmx_render_kernel(MMXState S, int env_base, const unsigned char* mask) {  // two workgroups per CU (LDS), registers to match
  extern __shared__ __align__(16) unsigned char rsmem[];
  float4* vs = reinterpret_cast<float4*>(rsmem);                                 // [MMR_NVERT] screen
  float* bpose = reinterpret_cast<float*>(vs + MMR_NVERT);                        // [19][12]
  uint32_t* zb = reinterpret_cast<uint32_t*>(bpose + 19 * 12);                    // [rows][Zs]
  unsigned short* bigq = reinterpret_cast<unsigned short*>(zb + kZbWords);        // [kBPW][kMaxBig]
  int* nbig = reinterpret_cast<int*>(bigq + kBPW * kMaxBig);                      // [kNbig] queue counters
  float* cam = reinterpret_cast<float*>(nbig + kNbig);                            // R (9), p (3)
  uint32_t* tinfo = reinterpret_cast<uint32_t*>(cam + 12);                        // [MMR_NTRI]
  float* mrgb = reinterpret_cast<float*>(tinfo + MMR_NTRI);                       // [MMR_NMAT][8]
  unsigned short* smallq = reinterpret_cast<unsigned short*>(mrgb + 8 * MMR_NMAT); // [kBPW][MMR_NTRI]
  RTri* bigs = reinterpret_cast<RTri*>(smallq + kBPW * MMR_NTRI);                 // [kBigCache] setups

  const int tid = threadIdx.x;
  const int Sz = S.image_size;        // image side (projection, output)
  const int Sg = (Sz + 15) & ~15;     // raster grid side: bands, 16 x 16 tiles, z-buffer rows
  const bool whole = Sz == Sg;        // every tile lies inside the image
  const int rows = rend_band_rows(Sg);
  const int Zs = Sg + MMR_ZPAD;  // z-buffer row stride
  const int rowA = blockIdx.x * kBPW * rows, rowB = min(Sz, rowA + kBPW * rows);  // the workgroup's bands
  const int ci = blockIdx.y;  // 0 overhead, 1 wrist
  const int i = env_base + blockIdx.z;
  if (i >= S.N || rowA >= Sz || (mask && !mask[i])) return;  // mask: only the envs just reset
  const float* rp = S.rpose + (size_t)i * RNSLOT * 12;
  RCLK_DECL

  // 1. body poses (world, static scene bodies, moving bodies) and the camera
  if (tid < 19) {
    float* o = bpose + 12 * tid;
    const int b = tid;
    const int slot = b >= 1 && b <= 11 ? b - 1 : (b >= 16 ? b - 5 : -1);
    if (slot >= 0) {
      for (int k = 0; k < 12; k++) o[k] = rp[12 * slot + k];
    } else {  // world and the static table / bins: parent = world
      const M3 R = qmat(Q4{MMX_body_quat[4 * b], MMX_body_quat[4 * b + 1], MMX_body_quat[4 * b + 2],
                           MMX_body_quat[4 * b + 3]});
      for (int k = 0; k < 9; k++) o[k] = b == 0 ? (k % 4 == 0 ? 1.f : 0.f) : R.m[k];
      for (int k = 0; k < 3; k++) o[9 + k] = b == 0 ? 0.f : MMX_body_pos[3 * b + k];
    }
  }
  if (tid < kNbig) nbig[tid] = 0;
  if (tid == 32) {
    const int c = ci == 0 ? MMX_CAM_OVERHEAD : MMX_CAM_WRIST;
    const M3 lq = qmat(Q4{MMX_cam_quat[4 * c], MMX_cam_quat[4 * c + 1], MMX_cam_quat[4 * c + 2], MMX_cam_quat[4 * c + 3]});
    const V3 lp = V3{MMX_cam_pos[3 * c], MMX_cam_pos[3 * c + 1], MMX_cam_pos[3 * c + 2]};
    M3 R = lq;
    V3 p = lp;
    if (MMX_cam_body[c] != 0) {
      const int s = MMX_cam_body[c] - 1;  // the hand: an arm body slot
      M3 hR;
      for (int k = 0; k < 9; k++) hR.m[k] = rp[12 * s + k];
      const V3 hx = V3{rp[12 * s + 9], rp[12 * s + 10], rp[12 * s + 11]};
      R = mul(hR, lq);
      p = hx + mul(hR, lp);
    }
    for (int k = 0; k < 9; k++) cam[k] = R.m[k];
    cam[9] = p.x; cam[10] = p.y; cam[11] = p.z;
  }
  for (int k = tid; k < min(rows, rowB - rowA) * Zs; k += RWG) zb[k] = 0u;  // the first band's z-buffer
  if (tid < MMR_NMAT * 8) {  // rgb1, rgb2, checker square, segment id
    const int m = tid >> 3, k = tid & 7;
    mrgb[tid] = k < 6 ? MMR_mat_rgb[6 * m + k] : (k == 6 ? MMR_mat_checker[m] : (float)MMR_mat_seg[m]);
  }
  __syncthreads();
  RCLK(0);

  // 2. vertices to camera space and to the screen
  M3 cR;
  for (int k = 0; k < 9; k++) cR.m[k] = cam[k];
  const V3 cx = V3{cam[9], cam[10], cam[11]};
  const int c = ci == 0 ? MMX_CAM_OVERHEAD : MMX_CAM_WRIST;
  const float half = 0.5f * Sz;
  const float f = half / tanf(MMX_cam_fovy[c] * (3.14159265358979f / 360.f));
  // depth range of the camera: overhead 2 m above the floor, wrist from 1 cm
  const float znear = ci == 0 ? 0.5f : 0.01f, zfar = ci == 0 ? 2.5f : 4.0f;
  for (int v = tid; v < MMR_NVERT; v += RWG) {
    const float* o = bpose + 12 * MMR_vert_body[v];
    M3 R;
    for (int k = 0; k < 9; k++) R.m[k] = o[k];
    const V3 w = V3{o[9], o[10], o[11]} + mul(R, V3{MMR_vert[3 * v], MMR_vert[3 * v + 1], MMR_vert[3 * v + 2]});
    const V3 cv = mulT(cR, w - cx);
    vs[v] = rend_project(make_float4(cv.x, cv.y, cv.z, 0.f), f, half, znear);
  }
  __syncthreads();
  RCLK(1);

  // 3. rasterise
  const float iz_lo = 1.f / zfar, iz_scale = 1.f / (1.f / znear - 1.f / zfar), q0 = -iz_lo * iz_scale;
  const V3 l_top = mulT(cR, V3{0.f, 0.f, 1.f});  // toward the directional light (dir 0 0 -1)
  const V3 lp_cam = mulT(cR, V3{0.5f, 0.5f, 1.5f} - cx);
  const float floor_light0 = 0.3f + 0.6f * fmaxf(l_top.z, 0.f) + 0.8f;  // the floor's headlight + directional
  // the floor's triangles [0, MMR_FLOOR_TRIS) are not rasterised: it lies below everything, so a
  // pixel no triangle covers shows the floor where its ray meets z = 0 inside the plane, else sky
  // Each triangle is set up once for the workgroup's rows (cull, box, face light) and queued per
  // band its box meets.
  for (int t = MMR_FLOOR_TRIS + tid; t < MMR_NTRI; t += RWG) {
    RTri T;
    const int ta = MMR_tri[3 * t], tb = MMR_tri[3 * t + 1], tc = MMR_tri[3 * t + 2];
    if (!rend_setup_abc(vs, ta, tb, tc, Sz, rowA, rowB, iz_scale, T)) continue;
    {  // flat shading of the face, once: headlight + directional + point light (at the centroid)
      const float4 pa = vs[ta], pb = vs[tb], pcv = vs[tc];
      const float4 a = rend_unproject(pa.x, pa.y, pa.z, f, half), b = rend_unproject(pb.x, pb.y, pb.z, f, half),
                   cc = rend_unproject(pcv.x, pcv.y, pcv.z, f, half);
      const V3 n = normalize(cross(V3{b.x - a.x, b.y - a.y, b.z - a.z}, V3{cc.x - a.x, cc.y - a.y, cc.z - a.z}));
      const V3 pc = V3{(a.x + b.x + cc.x) * (1.f / 3.f), (a.y + b.y + cc.y) * (1.f / 3.f), (a.z + b.z + cc.z) * (1.f / 3.f)};
      const float light = 0.3f + 0.6f * fmaxf(n.z, 0.f) + 0.8f * fmaxf(dot(n, l_top), 0.f) +
                          0.4f * fmaxf(dot(n, normalize(lp_cam - pc)), 0.f);
      // the face's packed colour (light in steps of 2^-14; no rasterised material has a checker:
      // the floor, the only one, is shaded per pixel, tools/compile_render.py)
      const float lq = (float)(uint32_t)(fminf(light, 3.99f) * 16384.f) * (1.f / 16384.f);
      const float* mt = mrgb + 8 * MMR_tri_mat[t];
      tinfo[t] = rend_pack(fminf(mt[0] * lq, 1.f), fminf(mt[1] * lq, 1.f), fminf(mt[2] * lq, 1.f), (uint32_t)mt[7]);
    }
    for (int kb = 0; kb < kBPW; kb++) {
      const int r0 = rowA + kb * rows;
      const int by0 = max(T.by0, r0), by1 = min(T.by1, r0 + rows - 1);
      if (by0 > by1) continue;
      const int area = (T.bx1 - T.bx0 + 1) * (by1 - by0 + 1);
      int k = area > kSmallArea ? atomicAdd(nbig + 2 * kb, 1) : kMaxBig;
      if (k < kMaxBig) bigq[kb * kMaxBig + k] = (unsigned short)t;
      else if (area <= kTiny) smallq[kb * MMR_NTRI + atomicAdd(nbig + 2 * kb + 1, 1)] = (unsigned short)t;
      else smallq[kb * MMR_NTRI + MMR_NTRI - 1 - atomicAdd(nbig + 8 + kb, 1)] = (unsigned short)t;
    }
  }
  const int tcols = Sg >> 4;
  // the overhead camera is fixed: its background (floor / sky per pixel) is one table for every env
  // the per-sim background table holds a world-fixed camera's view: used only while the overhead
  // camera is attached to the world (a body-mounted one falls back to per-pixel shading)
  const uint32_t* bgtab = ci == 0 && MMX_cam_body[MMX_CAM_OVERHEAD] == 0 ? S.bg_overhead : nullptr;
  const int lane = tid & 63, lx = 4 * (lane & 3), ly = kTileRow(lane >> 2);
  unsigned char* img = S.images + ((size_t)i * 2 + ci) * Sz * Sz * 3;
  unsigned char* seg = S.seg + ((size_t)i * 2 + ci) * Sz * Sz;
  for (int kb = 0; kb < kBPW; kb++) {  // the bands one after the other through the one z-buffer
  const int row0 = rowA + kb * rows, row1 = min(Sz, row0 + rows);
  if (row0 >= Sz) break;
  if (kb) {
    __syncthreads();  // the previous band's tiles have read zb
    RCLK(4);
    for (int k = tid; k < (row1 - row0) * Zs; k += RWG) zb[k] = 0u;
  }
  __syncthreads();
  if (kb) RCLK(3); else RCLK(2);
  // the band's first kBigCache large triangles set up once for every wave's tile walk
  for (int q = tid; q < min((MMR_SKIP & 2) ? 0 : nbig[2 * kb], kBigCache); q += RWG)
    rend_setup(vs, bigq[kb * kMaxBig + q], Sz, row0, row1, iz_scale, bigs[q]);
  {  // small triangles: one per 8-lane group, walked column by column
    const int nsf = nbig[2 * kb + 1], ns = (MMR_SKIP & 1) ? 0 : nsf + nbig[8 + kb];
    // queue entry q: the tiny boxes [0, nsf) from the front, then the others from the back
    const unsigned short* sq = smallq + kb * MMR_NTRI;
    auto sq_at = [&](int q) { return (int)sq[q < nsf ? q : MMR_NTRI - 1 - (q - nsf)]; };
    // Group grp = tid / 8 (wave wv = tid / 64, group g = lane / 8 in it) walks the queue entries
    // q = grp + 64 k, k = 0, 1, ...  The setups are computed wave-wide, one lane per triangle:
    // for the 8 steps k = 8 r .. 8 r + 7 of a round, lane 8 j + g sets up group g's triangle of
    // step 8 r + j, and at step j each group fetches its setup from that lane (ds_bpermute)
    // instead of its 8 lanes all recomputing it (written for kGroup lanes per group).
    // (with G = 64 / kGroup groups per wave, a round is kGroup steps: lane j G + g sets up group
    // g's triangle of step j)
    constexpr int G = 64 / kGroup;
    static_assert(64 % kGroup == 0 && RWG % 64 == 0, "wave-wide setup: whole groups per wave");
    const int lane = tid & 63, wv = tid >> 6, g = lane / kGroup, gl = lane % kGroup;
    const int per_step = RWG / kGroup;  // groups in the workgroup: queue entries per step
    for (int r = 0; kGroup * r * per_step < ns; r++) {
      const int qs = (kGroup * r + lane / G) * per_step + G * wv + lane % G;  // this lane's setup
      RTri Ts;
      const int ts = qs < ns ? sq_at(qs) : MMR_FLOOR_TRIS;
      rend_setup(vs, ts, Sz, row0, row1, iz_scale, Ts);
      for (int j = 0; j < kGroup; j++) {
        const int k = kGroup * r + j;
        if (k * per_step + G * wv >= ns) break;  // uniform per wave: no group of it has an entry
        const int q = k * per_step + G * wv + g;
        const int src = G * j + g;  // the lane holding this group's setup
        RTri T;
#pragma unroll
        for (int e = 0; e < 3; e++) {
          T.A[e] = __shfl(Ts.A[e], src);
          T.B[e] = __shfl(Ts.B[e], src);
          T.C[e] = __shfl(Ts.C[e], src);
          T.w[e] = __shfl(Ts.w[e], src);
        }
        T.bx0 = __shfl(Ts.bx0, src);
        T.bx1 = __shfl(Ts.bx1, src);
        T.by0 = __shfl(Ts.by0, src);
        T.by1 = __shfl(Ts.by1, src);
        const int t = __shfl(ts, src);
        if (q >= ns) continue;
        const int w = T.bx1 - T.bx0 + 1;
        const float rw = 1.f / (float)w;
        const float qB = fmaf(T.B[0], T.w[0], fmaf(T.B[1], T.w[1], T.B[2] * T.w[2]));  // dq / dy
        // column walk: a box up to 8 wide gives each lane one column and a row phase (8 / w lanes
        // per column, rows strided by that), a wider one 8 columns per pass, rows one by one; the
        // edges' x parts are formed once per column, a pixel then costs 3 FMAs and a max
        const bool narrow = w <= kGroup;
        const int rstep = narrow ? (int)(((float)kGroup + 0.5f) * rw) : 1;  // kGroup / w (exact)
        const int rph = narrow ? (int)(((float)gl + 0.5f) * rw) : 0;        // gl / w
        const float rB[3] = {1.f / T.B[0], 1.f / T.B[1], 1.f / T.B[2]};  // (unused where B_k = 0)
        if (rph < rstep) {
          for (int col = narrow ? gl - rph * w : gl; col < w; col += kGroup) {
            const int px = T.bx0 + col;
            const float x = px + 0.5f;
            const float ex0 = rend_edge_x(T, 0, x), ex1 = rend_edge_x(T, 1, x), ex2 = rend_edge_x(T, 2, x);
            // the column's span inside the triangle: edge k bounds the row centres y = py + 0.5 from
            // above (B_k > 0: y <= -ex_k / B_k) or below (B_k < 0); widened by a row on each side, it
            // only narrows the walk, every pixel still takes the exact edge test
            float lo = (float)T.by0, hi = (float)T.by1;
            {
              const float ex[3] = {ex0, ex1, ex2};
              for (int e = 0; e < 3; e++) {
                const float yb = -ex[e] * rB[e] - 0.5f;  // the boundary in row-index units
                hi = T.B[e] > 0.f ? fminf(hi, yb + 1.f) : hi;
                lo = T.B[e] < 0.f ? fmaxf(lo, yb - 1.f) : lo;
              }
            }
            // (kept inside [by0, by1 + 1] / [by0 - 1, by1] before the integer conversion)
            const int pylo = (int)ceilf(fminf(lo, (float)(T.by1 + 1))), pyhi = (int)floorf(fmaxf(hi, (float)(T.by0 - 1)));
            // q is affine in y along the column: q = qB y + qx (one FMA per pixel)
            const float qx = fmaf(ex0, T.w[0], fmaf(ex1, T.w[1], fmaf(ex2, T.w[2], q0)));
            uint32_t* zc = zb + (pylo + rph - row0) * Zs + px;
            const float ystep = (float)rstep;
            float y = (float)(pylo + rph) + 0.5f;
            for (int py = pylo + rph; py <= pyhi; py += rstep, zc += rstep * Zs, y += ystep) {
              const float e0 = fmaf(T.B[0], y, ex0), e1 = fmaf(T.B[1], y, ex1), e2 = fmaf(T.B[2], y, ex2);
              if (fmaxf(e0, fmaxf(e1, e2)) <= 0.f) atomicMax(zc, rend_key_q(t, fmaf(qB, y, qx)));
            }
          }
        }
      }
    }
  }
  __syncthreads();
  RCLK(3);

  // 4. large triangles + shading, fused, per 16 x 16 tile (S is a multiple of 16): each wave owns
  // kTPW tiles at a time, lane l the 4 pixels (4 (l & 3) .. +3, l >> 2) of each.  A lane starts from
  // the small triangles' depth keys in zb, walks the large-triangle queue once per tile batch (the
  // setup uniform per wave: scalar table loads, LDS broadcasts), skips tiles outside a triangle's
  // box or wholly outside one of its edges (12 corner tests, one per lane, one ballot), keeps the
  // nearest key in registers and shades its pixels straight away: no depth atomics, no zb write
  // back, no barrier between the large-triangle raster and the shading.
  const int nb = (MMR_SKIP & 2) ? 0 : min(nbig[2 * kb], kMaxBig);
  const int ntiles = tcols * ((row1 - row0 + 15) >> 4);
  for (int tb = (tid >> 6) * kTPW; tb < ((MMR_SKIP & 4) ? 0 : ntiles); tb += (RWG / 64) * kTPW) {
    int tx[kTPW], ty[kTPW];
    uint32_t best[kTPW][4];
    for (int j = 0; j < kTPW; j++) {
      const int tile = min(tb + j, ntiles - 1);  // a batch's spare tiles repeat the last one (not stored)
      const int trow = tile / tcols;
      tx[j] = (tile - trow * tcols) * 16;
      ty[j] = row0 + trow * 16;
      const int py = ty[j] + ly;
      const uint4 z4 = py < row1 ? *reinterpret_cast<const uint4*>(zb + (py - row0) * Zs + tx[j] + lx) : uint4{0u, 0u, 0u, 0u};
      best[j][0] = z4.x; best[j][1] = z4.y; best[j][2] = z4.z; best[j][3] = z4.w;  // (x < Sg)
    }
    for (int q = 0; q < nb; q++) {
      const int t = __builtin_amdgcn_readfirstlane((int)bigq[kb * kMaxBig + q]);
      RTri T;
      if (q < kBigCache) T = bigs[q];  // uniform address: LDS broadcast
      else rend_setup(vs, t, Sz, row0, row1, iz_scale, T);
      for (int j = 0; j < kTPW; j++) {
        if (T.bx1 < tx[j] || T.bx0 > tx[j] + 15 || T.by1 < ty[j] || T.by0 > ty[j] + 15) continue;
        {  // lane 4e + c: edge e at tile corner c; a tile whose 4 corners all lie outside one edge
           // lies wholly outside the triangle (pixel centres of the tile's corner pixels)
          const int e = min(lane >> 2, 2), c = lane & 3;
          const float cx0 = tx[j] + ((c & 1) ? 15.5f : 0.5f), cy0 = ty[j] + ((c & 2) ? 15.5f : 0.5f);
          const float A = e == 0 ? T.A[0] : (e == 1 ? T.A[1] : T.A[2]), B = e == 0 ? T.B[0] : (e == 1 ? T.B[1] : T.B[2]);
          const float C = e == 0 ? T.C[0] : (e == 1 ? T.C[1] : T.C[2]);
          const uint64_t out = __ballot(lane < 12 && fmaf(B, cy0, fmaf(A, cx0, C)) > 0.f);
          if ((out & 0xFull) == 0xFull || (out & 0xF0ull) == 0xF0ull || (out & 0xF00ull) == 0xF00ull) continue;
        }
        for (int u = 0; u < 4; u++) {
          const uint32_t key = rend_cover(T, t, tx[j] + lx + u, ty[j] + ly, q0);
          best[j][u] = max(best[j][u], key);
        }
      }
    }
    for (int j = 0; j < kTPW; j++) {
      const int py = ty[j] + ly;
      if (tb + j >= ntiles || py >= row1) continue;
      const int nvalid = whole ? 4 : min(4, Sz - (tx[j] + lx));
      if (nvalid <= 0) continue;
      const size_t p0 = (size_t)py * Sz + tx[j] + lx;  // image pixel of the lane's first pixel
      shade4(best[j], tx[j] + lx, py, half, f, cR, cx, floor_light0, tinfo, mrgb, bgtab ? bgtab + (size_t)py * Sg : nullptr,
             reinterpret_cast<uint32_t*>(img + 3 * p0), reinterpret_cast<uint32_t*>(seg + p0), nvalid);
    }
  }
  }  // bands
  RCLK(4);
  RCLK_END
}
#ifdef MMR_CLOCK
extern "C" hipError_t mmx_render_clock(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rclk), sizeof(unsigned long long) * 8);
  if (e == hipSuccess && reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_rclk), z, sizeof(z));
  }
  return e;
}
#endif

// The fixed overhead camera's background: for every pixel of the Sg x Sg raster grid, the packed
// colour + segment id shade4 gives an uncovered pixel (same rays, same arithmetic), computed once per
// sim; the render kernel then reads it instead of intersecting the floor per pixel and env.
extern "C" __global__ void __launch_bounds__(256) mmx_render_bg_kernel(MMXState S, uint32_t* bg) {
  const int Sz = S.image_size, Sg = (Sz + 15) & ~15;
  const int g = blockIdx.x * 256 + threadIdx.x;  // 4-pixel group
  if (g >= Sg * Sg / 4) return;
  const int py = g / (Sg / 4), px0 = 4 * (g % (Sg / 4));
  const int c = MMX_CAM_OVERHEAD;
  const M3 cR = qmat(Q4{MMX_cam_quat[4 * c], MMX_cam_quat[4 * c + 1], MMX_cam_quat[4 * c + 2], MMX_cam_quat[4 * c + 3]});
  const V3 cx = V3{MMX_cam_pos[3 * c], MMX_cam_pos[3 * c + 1], MMX_cam_pos[3 * c + 2]};
  const float half = 0.5f * Sz;
  const float f = half / tanf(MMX_cam_fovy[c] * (3.14159265358979f / 360.f));
  const V3 l_top = mulT(cR, V3{0.f, 0.f, 1.f});
  const float floor_light0 = 0.3f + 0.6f * fmaxf(l_top.z, 0.f) + 0.8f;
  float mrgb[8 * MMR_NMAT];
  for (int k = 0; k < 8 * MMR_NMAT; k++) {
    const int m = k >> 3, j = k & 7;
    mrgb[k] = j < 6 ? MMR_mat_rgb[6 * m + j] : (j == 6 ? MMR_mat_checker[m] : (float)MMR_mat_seg[m]);
  }
  V3 dw4[4];
  rays4(px0, py, half, f, cR, dw4);
  for (int u = 0; u < 4; u++) bg[(size_t)py * Sg + px0 + u] = shade_bg(dw4[u], cx, floor_light0, mrgb);
}
extern "C" hipError_t mmx_launch_render_bg(const MMXState* S, hipStream_t st) {
  if (S->image_size <= 0 || !S->bg_overhead) return hipSuccess;
  const int Sg = (S->image_size + 15) & ~15;
  hipLaunchKernelGGL(mmx_render_bg_kernel, dim3((Sg * Sg / 4 + 255) / 256), dim3(256), 0, st, *S, S->bg_overhead);
  return hipGetLastError();
}

static_assert(sizeof(float4) * MMR_NVERT + sizeof(float) * 19 * 12 + sizeof(uint32_t) * kZbWords +
                  sizeof(unsigned short) * kBPW * kMaxBig + kNbig * sizeof(int) + 12 * sizeof(float) +
                  sizeof(uint32_t) * MMR_NTRI + sizeof(float) * 8 * MMR_NMAT + sizeof(unsigned short) * kBPW * MMR_NTRI +
                  sizeof(RTri) * kBigCache <= 80 * 1024,
              "render model too large for two workgroups per CU (LDS)");
extern "C" size_t mmx_render_lds_bytes() {
  return sizeof(float4) * MMR_NVERT + sizeof(float) * 19 * 12 + sizeof(uint32_t) * kZbWords +
         sizeof(unsigned short) * kBPW * kMaxBig + kNbig * sizeof(int) + 12 * sizeof(float) + sizeof(uint32_t) * MMR_NTRI +
         sizeof(float) * 8 * MMR_NMAT + sizeof(unsigned short) * kBPW * MMR_NTRI + sizeof(RTri) * kBigCache;
}

// envs [base, base + count); with a device mask (N bytes) only the envs whose byte is set
extern "C" hipError_t mmx_launch_render_masked(const MMXState* S, int base, int count, const unsigned char* mask,
                                               hipStream_t st) {
  if (count <= 0 || S->image_size <= 0) return hipSuccess;
  const int rows = rend_band_rows((S->image_size + 15) & ~15);
  const int bands = (S->image_size + rows - 1) / rows;
  hipLaunchKernelGGL(mmx_render_kernel, dim3((bands + kBPW - 1) / kBPW, 2, count), dim3(RWG), mmx_render_lds_bytes(), st, *S,
                     base, mask);
  return hipGetLastError();
}
extern "C" hipError_t mmx_launch_render(const MMXState* S, int base, int count, hipStream_t st) {
  return mmx_launch_render_masked(S, base, count, nullptr, st);
}
