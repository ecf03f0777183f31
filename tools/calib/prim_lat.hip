// Calibration micro-benchmark (not product code): the latency of the cross-lane primitives the
// step kernel's dependency chains are built from, measured as shader cycles (s_memtime) per link
// of a dependent chain, one wave per SIMD and two waves per SIMD (occupancy pinned by dynamic LDS).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define DEV __device__ __forceinline__
template <int CTRL>
DEV float dpp_f(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true)); }
DEV float readlane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
DEV float wave_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}
// full-wave sum through the gfx9 DPP broadcasts (row_bcast:15, row_bcast:31): the total lands in
// lane 63, one v_readlane hands it to every lane
DEV float wave_sum_bcast(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x114>(v);  // row_shr:4 (bound_ctrl: lanes without a source add 0)
  v += dpp_f<0x118>(v);  // row_shr:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));  // row_bcast:15
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));  // row_bcast:31
  return readlane_f(v, 63);
}
DEV void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

enum { P_FMA, P_READLANE, P_DPP_SHR, P_ROWBCAST, P_WAVESUM, P_RSQ, P_LDS_RT, P_BPERMUTE, P_BALLOT, P_SQRT_DIV,
       P_WAVESUM_BCAST, P_N };
static const char* kNames[P_N] = {"fma", "readlane_fma", "dpp_row_shr_add", "dpp_row_newbcast_fma", "wave_sum",
                                  "rsq_fma", "lds_write_sync_read", "ds_bpermute", "ballot_popc_cvt", "sqrt_div",
                                  "wave_sum_bcast"};

template <int P>
__global__ void __launch_bounds__(64) chain(float* out, int iters, unsigned long long* clk) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x;
  float v = 1.0f + lane * 1e-3f;
  const float a = 0.999f, b = 1e-3f;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      if (P == P_FMA) v = fmaf(v, a, b);
      if (P == P_READLANE) v = fmaf(readlane_f(v, (u * 7) & 63), a, v);
      if (P == P_DPP_SHR) v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));
      if (P == P_ROWBCAST) v = fmaf(dpp_f<0x153>(v), a, b);
      if (P == P_WAVESUM) v = fmaf(wave_sum(v), 1e-3f, v);
      if (P == P_RSQ) v = fmaf(__builtin_amdgcn_rsqf(v), a, 1.0f);
      if (P == P_LDS_RT) {
        lds[lane] = v;
        wsync();
        v = fmaf(lds[(lane + 1 + u) & 63], a, b);
        wsync();
      }
      if (P == P_BPERMUTE) v = fmaf(__shfl(v, (lane + 1 + u) & 63), a, b);
      if (P == P_BALLOT) v = v + (float)__popcll(__ballot(v > 1.0f)) * 1e-6f;
      if (P == P_SQRT_DIV) v = sqrtf(v) / (v + 1.0f) + 1.0f;
      if (P == P_WAVESUM_BCAST) v = fmaf(wave_sum_bcast(v), 1e-3f, v);
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (lane == 0) clk[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + lane] = v;
}

template <int P>
void run(int cus) {
  const int iters = 256;
  for (int wps : {1, 2}) {
    const int wg_per_cu = 4 * wps;
    const size_t lds = (size_t)(160 * 1024 / wg_per_cu) & ~(size_t)255;
    const int n = cus * wg_per_cu;
    float* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, n * 64 * sizeof(float));
    (void)hipMalloc(&clk, n * sizeof(unsigned long long));
    (void)hipFuncSetAttribute((const void*)chain<P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(chain<P>, dim3(n), dim3(64), lds, 0, out, 4, clk);
    hipLaunchKernelGGL(chain<P>, dim3(n), dim3(64), lds, 0, out, iters, clk);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> c(n);
    (void)hipMemcpy(c.data(), clk, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mc = 0;
    for (auto x : c) mc += (double)x;
    mc /= n;
    printf("{\"primitive\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_link\": %.2f}\n", kNames[P], wps,
           mc / (iters * 16.0));
    (void)hipFree(out);
    (void)hipFree(clk);
  }
}

__global__ void check_kernel(float* out) {
  const float v = (float)threadIdx.x;
  out[threadIdx.x] = wave_sum_bcast(v) - wave_sum(v);
}
int check_bcast() {
  float* d;
  (void)hipMalloc(&d, 64 * sizeof(float));
  hipLaunchKernelGGL(check_kernel, dim3(1), dim3(64), 0, 0, d);
  float h[64];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int k = 0; k < 64; k++) bad += h[k] != 0.f;
  printf("{\"wave_sum_bcast_check\": \"%s\"}\n", bad ? "MISMATCH" : "equal");
  (void)hipFree(d);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int c = p.multiProcessorCount;
  run<P_FMA>(c);
  run<P_READLANE>(c);
  run<P_DPP_SHR>(c);
  run<P_ROWBCAST>(c);
  run<P_WAVESUM>(c);
  run<P_RSQ>(c);
  run<P_LDS_RT>(c);
  run<P_BPERMUTE>(c);
  run<P_BALLOT>(c);
  run<P_SQRT_DIV>(c);
  run<P_WAVESUM_BCAST>(c);
  // correctness of wave_sum_bcast against the readlane form (one wave, lane values 0..63)
  return check_bcast();
}
