// Calibration micro-benchmark (not product code): how many 64-lane workgroups with B bytes of LDS
// each are resident on one CU at once, for B around the step kernel's footprints (the LDS
// allocation granularity decides it).  Every workgroup spins ~40 us; lane 0 records its CU (HW_ID:
// CU, SH, SE; XCC_ID) and its start / end shader clock.  The host finds, per CU, the largest number of
// workgroups whose [start, end) intervals overlap, and prints one JSON line per size.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

__global__ void __launch_bounds__(64) resident(unsigned* rec, unsigned long long spin) {
  extern __shared__ unsigned lds[];
  lds[threadIdx.x] = threadIdx.x;  // touch the allocation
  const unsigned long long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < spin) __builtin_amdgcn_s_sleep(1);
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) {
    // HW_REG_HW_ID (4): bits 8-11 CU, 12 SH, 13-15 SE; HW_REG_XCC_ID (20): bits 0-3
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
    unsigned* r = rec + 7 * blockIdx.x;
    r[0] = (hw >> 8) & 15;
    r[1] = (hw >> 12) & 1;
    r[2] = (hw >> 13) & 7;
    r[3] = xcc & 15;
    r[4] = (unsigned)(t0 & 0xffffffffu);
    r[5] = (unsigned)(t0 >> 32);
    r[6] = (unsigned)((t1 - t0) & 0xffffffffu);
    lds[0] += r[0];
  }
}

int main() {
  const int sizes[] = {12800, 13312, 13400, 13653, 13824, 14336, 14800, 14848, 14900, 15360, 15824, 16384,
                       19408, 20432, 20480, 20600};
  const int nwg = 256 * 24;
  unsigned* d;
  if (hipMalloc(&d, sizeof(unsigned) * 7 * nwg) != hipSuccess) return 1;
  std::vector<unsigned> h(7 * nwg);
  for (int B : sizes) {
    hipLaunchKernelGGL(resident, dim3(nwg), dim3(64), B, 0, d, 100000ull);  // ~40 us at 2.4 GHz
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpy(h.data(), d, sizeof(unsigned) * 7 * nwg, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    std::map<unsigned, std::vector<std::pair<long long, int>>> ev;  // CU key -> (time, +1 / -1)
    for (int w = 0; w < nwg; w++) {
      const unsigned* r = &h[7 * w];
      const unsigned key = r[0] | (r[1] << 4) | (r[2] << 5) | (r[3] << 8);
      const long long s = (long long)(((unsigned long long)r[5] << 32) | r[4]), e = s + r[6];
      ev[key].push_back({s, +1});
      ev[key].push_back({e, -1});
    }
    int best = 0, cus = 0;
    std::map<int, int> hist;
    for (auto& kv : ev) {
      auto& v = kv.second;
      std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
      int cur = 0, mx = 0;
      for (auto& p : v) mx = std::max(mx, cur += p.second);
      hist[mx]++;
      best = std::max(best, mx);
      cus++;
    }
    printf("{\"lds_bytes\": %d, \"cus_seen\": %d, \"max_resident_per_cu\": %d, \"histogram\": {", B, cus, best);
    bool first = true;
    for (auto& kv : hist) {
      printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
      first = false;
    }
    printf("}}\n");
  }
  return 0;
}
