// Calibration micro-benchmark (not product code): how many wave64 VALU instructions one SIMD
// issues per cycle with 1..4 resident waves per SIMD, each wave running NCH independent FMA chains
// (NCH = 1: a dependent chain, latency-bound).  Occupancy is pinned with dynamic LDS (one 64-lane
// workgroup = one wave; the LDS per workgroup sets the workgroups per CU).  Built with
// -fno-slp-vectorize (scalar v_fma_f32, as the step kernel) and, as valu_peak_pk, without it (the
// compiler packs pairs into v_pk_fma_f32).  Prints per configuration the shader-clock cycles
// (s_memtime) per wave64 FMA instruction, per wave and per SIMD, and hipEvent TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int NCH>
__global__ void __launch_bounds__(64) fma_chains(float* out, int iters, unsigned long long* clk) {
  extern __shared__ float lds[];
  float a[NCH];
#pragma unroll
  for (int k = 0; k < NCH; k++) a[k] = threadIdx.x + k;
  const float m = 0.999f, c = 1e-3f;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 128 / NCH; u++)
#pragma unroll
      for (int k = 0; k < NCH; k++) a[k] = fmaf(a[k], m, c);
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; k++) s += a[k];
  if (threadIdx.x == 0) {
    lds[0] = s;
    clk[blockIdx.x] = t1 - t0;
  }
  out[blockIdx.x * 64 + threadIdx.x] = s + lds[0];
}

template <int NCH>
void run(int cus) {
  const int iters = 4096;  // 4096 x 128 FMAs per lane
  for (int wps : {1, 2, 3, 4}) {  // waves per SIMD
    const int wg_per_cu = 4 * wps;
    const size_t lds = (size_t)(160 * 1024 / wg_per_cu) & ~(size_t)255;
    const int n = cus * wg_per_cu;
    float* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, n * 64 * sizeof(float));
    (void)hipMalloc(&clk, n * sizeof(unsigned long long));
    (void)hipFuncSetAttribute((const void*)fma_chains<NCH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(fma_chains<NCH>, dim3(n), dim3(64), lds, 0, out, 16, clk);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(fma_chains<NCH>, dim3(n), dim3(64), lds, 0, out, iters, clk);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> c(n);
    (void)hipMemcpy(c.data(), clk, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mc = 0;
    for (auto v : c) mc += (double)v;
    mc /= n;
    const double fma_per_wave = (double)iters * 128;
    printf("{\"chains\": %d, \"waves_per_simd\": %d, \"lds_per_wg\": %zu, \"ms\": %.3f, \"tflops\": %.1f, "
           "\"clock_cycles_per_wave\": %.0f, \"cycles_per_fma_inst_per_wave\": %.3f, \"cycles_per_fma_inst_per_simd\": %.3f}\n",
           NCH, wps, lds, ms, 2.0 * fma_per_wave * 64 * n / (ms * 1e-3) / 1e12, mc, mc / fma_per_wave,
           mc / (wps * fma_per_wave));
    (void)hipFree(out);
    (void)hipFree(clk);
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  run<1>(p.multiProcessorCount);
  run<2>(p.multiProcessorCount);
  run<8>(p.multiProcessorCount);
  return 0;
}
