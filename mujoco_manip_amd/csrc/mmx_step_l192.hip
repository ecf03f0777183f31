// The env-step kernel and its launcher a second time, with 192 constraint rows in LDS (20,432 B per
// env, eight envs per CU, 248 VGPRs): mmx_env_step_kernel_l192 / mmx_launch_step_l192.  The 128-row
// build (ten per CU) is faster when the step kernel alone fills the chip (C3: +1.4 %); with cameras
// (render launches between the step launches, C5) and with fewer envs than slots (C2) this one is
// (+4.3 % C5).  mmx_api.cpp picks per sim (mmx_set_step_rows).  Same sources, same
// arithmetic: only where the rows past the LDS ones live and the register budget differ.
#undef MMX_LDSEFC
#define MMX_LDSEFC 192
#define MMX_STEP_ONLY 1
#define MMX_STEP_SUFFIX _l192
#include "mmx_kernels.hip"
