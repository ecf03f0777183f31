// The env-step kernel and its launcher a second time, with 192 constraint rows in LDS and two waves per
// env (the helper wave: MMX_STEP_HELPER in mmx_kernels.hip; four envs per CU, 248 VGPRs):
// mmx_env_step_kernel_l192 / mmx_launch_step_l192.  The 128-row build (twelve per CU) wins once the
// batch fills the workgroup slots; with four or fewer envs per CU each env's own speed is what counts
// and this one is faster (C2's 1024 envs: 1.52 M vs 1.29 M env steps/s).  mmx_api.cpp picks
// per sim from the batch size (mmx_set_step_rows, include/mmx_tuning.h).  Same sources, same arithmetic, bit-identical results: only where the rows past
// the LDS ones live and the register budget differ.
#undef MMX_LDSEFC
#define MMX_LDSEFC 192
#define MMX_STEP_ONLY 1
#define MMX_STEP_SUFFIX _l192
#include "mmx_kernels.hip"
// mmx_api.cpp allocates S.efc_ovf with the 128-row build's per-env stride, which must cover this one's
static_assert(MMX_OVF_F <= MMX_OVF_F_AT(128), "overflow block stride exceeds the allocation");
