// Phase clock of the diagnostic build (libmmx_prof.so, -DMMX_PHASE_CLOCK): CLK_DECL / CLK add
// the shader-clock cycles between stamps into a stats array (lane 0); PROBE(set, ...) is a CLK
// active only in the build whose MMX_PROBE equals set.  The product build compiles all of it away.
#ifndef MMX_CLOCK_H
#define MMX_CLOCK_H
#include <hip/hip_runtime.h>
// Built with -DMMX_PHASE_CLOCK (libmmx_prof.so) the kernels add the shader-clock cycles
// (s_memtime) of each phase into stats[STAT_T_*]; the product build compiles them away.
#ifdef MMX_PHASE_CLOCK
// volatile asm: the compiler may not move a stamp across the code it brackets
__device__ __forceinline__ unsigned long long clk_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define CLK_DECL unsigned long long clk_t0_ = clk_now()
#define CLK(st, k)                                                           \
  do {                                                                       \
    const unsigned long long clk_t1_ = clk_now();                            \
    if ((threadIdx.x & 63) == 0 && clk_t1_ > clk_t0_) (st)[k] += (float)(clk_t1_ - clk_t0_); \
    clk_t0_ = clk_t1_;                                                       \
  } while (0)
// variant for divergent code: the first active lane records
#define CLKF(st, k)                                                                        \
  do {                                                                                     \
    const unsigned long long clk_t1_ = clk_now();                                          \
    const unsigned long long act_ = __ballot(1);                                           \
    if ((int)(threadIdx.x & 63) == __ffsll((long long)act_) - 1 && clk_t1_ > clk_t0_)             \
      (st)[k] += (float)(clk_t1_ - clk_t0_);                                               \
    clk_t0_ = clk_t1_;                                                                     \
  } while (0)
#else
#define CLKF(st, k) \
  do {              \
  } while (0)
#define CLK_DECL \
  do {           \
  } while (0)
#define CLK(st, k) \
  do {             \
  } while (0)
#endif
// sub-phase probes into STAT_T_AUX0..3: MMX_PROBE selects the phase they instrument
// (1 solver, 2 collision, 3 constraints)
#ifndef MMX_PROBE
#define MMX_PROBE 1
#endif
#define PROBE(set, st, k)            \
  do {                               \
    if (MMX_PROBE == (set)) CLK(st, k); \
  } while (0)
#define PROBEF(set, st, k)            \
  do {                                \
    if (MMX_PROBE == (set)) CLKF(st, k); \
  } while (0)

#endif
