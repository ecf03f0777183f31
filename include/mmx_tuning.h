/* mmx_tuning.h — measurement and tuning entry points of libmmx.so (no reference counterpart).
 *
 * The reference boundary is include/mmx_api.h; a host binding of PickPlaceGymEnv needs nothing from
 * this header.  These calls report or choose how the batch is launched (rollout lanes and launch
 * lengths, the env-step kernel's LDS layout, the dispatch order of env steps) and time the launches
 * for bench.py.  None of them changes a result: every choice here is bit-identical to the default
 * (tests/test_gpu.py: test_step_layouts_agree, test_step_order_bit_identical,
 * test_rollout_lanes_bit_identical, test_fused_rollout_bit_identical).  Same conventions as
 * mmx_api.h (0 or a negative MMX_E* code, never an abort). */
#ifndef MMX_TUNING_H
#define MMX_TUNING_H
#include "mmx_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Constraint rows the env-step kernel (mmx_step, mmx_rollout_expert) keeps in LDS: 128 (twelve envs
 * per CU: the fastest layout once the batch fills the GPU's workgroup slots, C3 / C5 / dataset
 * generation) or 192 (four envs per CU, each with a second "helper" wave that runs its IK, dynamics and
 * GJK / EPA pairs beside the env wave's kinematics, broadphase and box pairs: faster per env, for
 * batches of at most four envs per CU, e.g. C2's 1024).  mmx_create picks by the batch size (192 up to
 * four envs per CU); env MMX_STEP_ROWS overrides at create.  The rows past the LDS ones live in the env's HBM overflow block; the two layouts are
 * bit-identical (a performance choice only).  MMX_EINVAL for any other value. */
int mmx_set_step_rows(mmx_sim* sim, int32_t rows);
int mmx_step_rows(const mmx_sim* sim);

/* Dispatch order of env-step launches (mmx_step, mmx_rollout_expert): 1 (default) = each launch's
 * envs longest first by FSM phase (a one-workgroup counting sort before the launch: the envs holding
 * an object, then closing / settling, then releasing, then the rest; within a phase class more
 * constraint rows in the last substep first), 0 = env index order.  Env
 * MMX_STEP_ORDER=0 sets 0 at create.  Only the hardware's workgroup schedule changes: results are
 * bit-identical either way.  MMX_EINVAL for other values; mmx_step_order returns -1 for NULL. */
int mmx_set_step_order(mmx_sim* sim, int32_t on);
int mmx_step_order(const mmx_sim* sim);

/* The most launches any rollout lane makes in mmx_rollout_expert(sim, n_env_steps): a launch runs
 * len = min(steps_per_launch, ceil(n / 4)) consecutive steps (1 with cameras); lane l of L starts with
 * a launch of l * len / L steps, then launches of len, then the remainder, so the lanes' launch
 * boundaries (each launch ends with a drain) do not fall together.  0 for a null sim or n <= 0. */
int mmx_rollout_launches(const mmx_sim* sim, int32_t n_env_steps);

/* Number of independent env ranges a multi-step rollout runs concurrently (one internal stream
 * each, forked from and joined back to cfg.stream; env MMX_STREAMS overrides the default of one
 * range per 1024 envs, at most 4).  Single-step calls always run as one launch on cfg.stream. */
int mmx_rollout_lanes(const mmx_sim* sim);

/* Render launches per rollout step: 1 with cameras (the env-step launch of all envs, then one render
 * launch over all envs), 0 without. */
int mmx_rollout_render_launches(const mmx_sim* sim);

/* 1 when camera rollouts (mmx_rollout_expert, more than one env step) render step k on a stream of
 * their own beside the env-step launch of step k + 1, the body poses double-buffered (the default
 * with cameras; env MMX_RENDER_OVERLAP=0 at create: render, then the next step); 0 otherwise.
 * Timing only: images and states are bit-identical either way. */
int mmx_rollout_render_overlap(const mmx_sim* sim);

/* Upper bound of the env steps one mmx_env_step_kernel launch runs per env in mmx_rollout_expert: 1
 * with cameras (every step is rendered), else 32 (env MMX_FUSE overrides).  A fused launch runs its
 * envs' steps back to back inside each workgroup; the trajectories are bit-identical to one
 * launch per step.  0 for a null sim. */
int mmx_rollout_steps_per_launch(const mmx_sim* sim);

/* Per-launch kernel timing of mmx_rollout_expert (measurement): with enable = 1 every step-kernel
 * and render-kernel launch is bracketed by a HIP event pair on the stream it runs on (a new
 * collection starts); enable = 0 stops collecting.  mmx_kernel_times waits for the recorded events
 * and returns the summed launch durations (ms) and launch counts of each kernel; NULL skips a
 * field. */
int mmx_kernel_timing(mmx_sim* sim, int32_t enable);
int mmx_kernel_times(mmx_sim* sim, float* step_ms, int32_t* step_launches, float* render_ms,
                     int32_t* render_launches);

#ifdef __cplusplus
}
#endif
#endif
