// C-ABI implementation (include/mmx_api.h, include/mmx_tuning.h): device allocation, host-side seeding, launches.
//
// Host-side seeding restates numpy's SeedSequence / PCG64 initialisation (the reference seeds
// every episode through gymnasium: Generator(PCG64(SeedSequence(seed))), gym_env.py:491) so the
// device PCG64 streams are bit-identical to the reference's np_random streams.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/mmx_api.h"
#include "../../include/mmx_tuning.h"
#include "mmx_state.h"

extern "C" hipError_t mmx_launch_reset(const MMXState* S, const unsigned char* mask, const int* task, hipStream_t st);
extern "C" hipError_t mmx_launch_step(const MMXState* S, const float* action, int adim, int expert_autoreset,
                                      int base, int count, int nsteps, hipStream_t st, const int* order);
extern "C" hipError_t mmx_launch_step_l192(const MMXState* S, const float* action, int adim, int expert_autoreset,
                                           int base, int count, int nsteps, hipStream_t st, const int* order);
extern "C" hipError_t mmx_launch_order(const MMXState* S, int base, int count, int* order, int threads, hipStream_t st);
extern "C" hipError_t mmx_launch_expert(const MMXState* S, int n, float* action, hipStream_t st);
extern "C" hipError_t mmx_launch_physics(const MMXState* S, int n, int with_ik, hipStream_t st);
extern "C" hipError_t mmx_launch_forward(const MMXState* S, hipStream_t st);
extern "C" hipError_t mmx_launch_render(const MMXState* S, int base, int count, hipStream_t st);
extern "C" hipError_t mmx_launch_render_bg(const MMXState* S, hipStream_t st);
extern "C" hipError_t mmx_launch_render_masked(const MMXState* S, int base, int count, const unsigned char* mask,
                                               hipStream_t st);
extern "C" hipError_t mmx_launch_queue(const MMXState* S, int* slot, int* next, int n_ep, const unsigned long long* rng,
                                       const int* qtask, unsigned char* mask, int* task, int* slot_out, int* fin_out,
                                       hipStream_t st);
extern "C" hipError_t mmx_launch_png(const uint8_t* rgb, int64_t img_stride, int n, int W, int H, uint8_t* out,
                                     int64_t out_stride, int32_t* sizes, uint32_t* scratch, hipStream_t st);
extern "C" hipError_t mmx_launch_png_pack(const uint8_t* out, int64_t out_stride, const int32_t* sizes,
                                          const int64_t* offsets, int n, uint8_t* packed, hipStream_t st);
extern "C" hipError_t mmx_launch_image_stats(const uint8_t* rgb, int64_t img_stride, int n, int64_t npx, int64_t* out,
                                             hipStream_t st);
extern "C" int64_t mmx_png_bound_bytes(int width, int height);
extern "C" int64_t mmx_png_scratch_bytes(int width, int height);
extern "C" hipError_t mmx_launch_expert_physics(const MMXState* S, int n, hipStream_t st);
extern "C" hipError_t mmx_launch_reward(const MMXState* S, const float* obj, const float* ee, const float* ctrl7,
                                        const int* pairs, int max_pairs, hipStream_t st);

struct mmx_sim {
  MMXState S;
  mmx_config cfg;
  hipStream_t stream;
  std::string err;
  std::vector<void*> allocs;
  float* expert_action;  // [N][4]
  unsigned char* d_mask;
  int* d_task;
  int* d_order;  // [N] dispatch order of the rollout's step launches (MMX_STEP_ORDER)
  // Multi-step rollouts split the envs into `nlanes` independent ranges, each stepped on its own
  // stream (lane 0 = the caller's stream): the ranges never wait for each other between steps,
  // so one range's last-wave tail overlaps the next step of the others.
  static constexpr int kMaxLanes = 8;
  int nlanes = 1;
  // cap on the env steps per mmx_env_step_kernel launch in expert rollouts without cameras (MMX_FUSE
  // overrides): with the staggered lanes 32 beat 16 by 0.5 % and 8 lost 2.7 % on 512-step C3 windows
  // (profiles/r06_sweep_launch_shape.json)
  int fuse = 32;
  // constraint rows the env-step kernel keeps in LDS: 128 (twelve envs per CU) or 192 (four per CU, each
  // with a helper wave, mmx_step_l192.hip: faster when the batch leaves CU slots empty); chosen at create
  // from the batch size, mmx_set_step_rows / MMX_STEP_ROWS override
  int step_rows = 128;
  // env steps launched longest first (mmx_order_kernel; mmx_set_step_order, MMX_STEP_ORDER=0 at
  // create turns it off): the launch's order only, never its results
  int step_order = 1;
  hipStream_t lane[kMaxLanes] = {};
  hipEvent_t ev_fork = nullptr, ev_join[kMaxLanes] = {};
  // camera rollouts render step k on their own stream beside step k + 1 (MMX_RENDER_OVERLAP=0 at
  // create: serial): the body poses alternate between S.rpose and rpose_alt; ev_step = the step
  // launch done, ev_rend[k & 1] = render k done
  int render_overlap = 0;
  float* rpose_alt = nullptr;
  hipStream_t rstream = nullptr;
  hipEvent_t ev_step = nullptr, ev_rend[2] = {};
  // per-launch kernel timing (mmx_kernel_timing): an event pair around every step / render launch
  // on the stream it runs on; pairs come from a pool reused after each read-out
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<std::pair<size_t, size_t>> t_step, t_render;
  // device-side episode queue (mmx_queue_init / mmx_queue_advance): per-slot episode, next episode,
  // and the episodes' tasks / PCG64 states; q_n < 0: no queue
  int* q_slot = nullptr;
  int* q_next = nullptr;
  int* q_task = nullptr;
  unsigned long long* q_rng = nullptr;
  int q_n = -1;
};

namespace {

// ---------------------------------------------------------------- numpy SeedSequence / PCG64
constexpr uint32_t kInitA = 0x43b0d7e5u, kMultA = 0x931e8875u, kInitB = 0x8b51f9ddu, kMultB = 0x58f38dedu;
constexpr uint32_t kMixL = 0xca01f9ddu, kMixR = 0x4973f715u;

uint32_t hashmix(uint32_t v, uint32_t& hc) {
  v ^= hc;
  hc *= kMultA;
  v *= hc;
  v ^= v >> 16;
  return v;
}
uint32_t mix(uint32_t x, uint32_t y) {
  uint32_t r = kMixL * x - kMixR * y;
  return r ^ (r >> 16);
}
std::vector<uint32_t> seed_words(uint64_t s) {
  std::vector<uint32_t> w{static_cast<uint32_t>(s)};
  if (s >> 32) w.push_back(static_cast<uint32_t>(s >> 32));
  return w;
}
// SeedSequence(entropy, spawn_key).generate_state(n_out, uint32)
std::vector<uint32_t> seedseq(std::vector<uint32_t> ent, const std::vector<uint32_t>& spawn, int n_out) {
  if (!spawn.empty() && ent.size() < 4) ent.resize(4, 0u);
  ent.insert(ent.end(), spawn.begin(), spawn.end());
  uint32_t pool[4];
  uint32_t hc = kInitA;
  for (int i = 0; i < 4; i++) pool[i] = hashmix(i < static_cast<int>(ent.size()) ? ent[i] : 0u, hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], hc));
  for (size_t s = 4; s < ent.size(); s++)
    for (int d = 0; d < 4; d++) pool[d] = mix(pool[d], hashmix(ent[s], hc));
  std::vector<uint32_t> out(n_out);
  uint32_t hb = kInitB;
  for (int i = 0; i < n_out; i++) {
    uint32_t v = pool[i % 4];
    v ^= hb;
    hb *= kMultB;
    v *= hb;
    v ^= v >> 16;
    out[i] = v;
  }
  return out;
}

using u128 = unsigned __int128;
const u128 kPcgMult = (static_cast<u128>(0x2360ED051FC65DA4ull) << 64) | 0x4385DF649FCCF645ull;

// PCG64(SeedSequence(seed)) initial (state, inc)
void pcg64_seed(uint64_t seed, uint64_t out[4]) {
  std::vector<uint32_t> st = seedseq(seed_words(seed), {}, 8);
  uint64_t v[4];
  for (int i = 0; i < 4; i++) v[i] = static_cast<uint64_t>(st[2 * i]) | (static_cast<uint64_t>(st[2 * i + 1]) << 32);
  u128 initstate = (static_cast<u128>(v[0]) << 64) | v[1];
  u128 initseq = (static_cast<u128>(v[2]) << 64) | v[3];
  u128 inc = (initseq << 1) | 1;
  u128 s = 0;
  s = s * kPcgMult + inc;
  s += initstate;
  s = s * kPcgMult + inc;
  out[0] = static_cast<uint64_t>(s >> 64);
  out[1] = static_cast<uint64_t>(s);
  out[2] = static_cast<uint64_t>(inc >> 64);
  out[3] = static_cast<uint64_t>(inc);
}

// Makes the sim's device current for the duration of an entry point (NULL-stream launches and
// hipMemcpy go to the current device) and restores the caller's device afterwards.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(const mmx_sim* sim) {
    if (sim && hipGetDevice(&prev) == hipSuccess && prev != sim->cfg.device) {
      if (hipSetDevice(sim->cfg.device) != hipSuccess) prev = -1;
    } else {
      prev = -1;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int fail(mmx_sim* sim, int code, const std::string& msg) {
  if (sim) sim->err = msg;
  return code;
}
int hip_check(mmx_sim* sim, hipError_t e, const char* what) {
  if (e == hipSuccess) return MMX_OK;
  return fail(sim, MMX_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
// After a stream synchronisation: the sim's fault word (ERR_SAMPLING of a reset since the last check,
// set by the reset kernel or a step's autoreset) is read, cleared and returned as MMX_ESAMPLING with
// the message randomization.py:84-87 raises.
int check_fault(mmx_sim* sim, const char* what) {
  int f = 0;
  if (hipMemcpy(&f, sim->S.fault, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(sim, MMX_EDEVICE, std::string(what) + ": fault readback");
  if (!(f & ERR_SAMPLING)) return MMX_OK;
  if (hipMemset(sim->S.fault, 0, sizeof(int)) != hipSuccess) return fail(sim, MMX_EDEVICE, std::string(what) + ": fault clear");
  return fail(sim, MMX_ESAMPLING, "Failed to sample 3 positions with min_separation=0.08 in 1000 attempts");
}

template <typename T>
T* dalloc(mmx_sim* sim, size_t count) {
  void* p = nullptr;
  if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, count * sizeof(T)) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  sim->allocs.push_back(p);
  return static_cast<T*>(p);
}

}  // namespace

namespace {
static constexpr size_t kTimingPoolPresize = 2048;
// an event of the timing pool recorded on `st` (its index), or SIZE_MAX when the pool cannot grow
size_t timing_mark(mmx_sim* sim, hipStream_t st) {
  if (sim->ev_used == sim->ev_pool.size()) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return SIZE_MAX;
    sim->ev_pool.push_back(ev);
  }
  const size_t k = sim->ev_used;
  if (hipEventRecord(sim->ev_pool[k], st) != hipSuccess) return SIZE_MAX;
  sim->ev_used++;
  return k;
}
// launch `f` on `st`, bracketed by a timing event pair when timing is on
template <class F>
hipError_t timed(mmx_sim* sim, hipStream_t st, std::vector<std::pair<size_t, size_t>>& pairs, F f) {
  const size_t a = sim->timing ? timing_mark(sim, st) : SIZE_MAX;
  const hipError_t e = f();
  if (a != SIZE_MAX && e == hipSuccess) {
    const size_t b = timing_mark(sim, st);
    if (b != SIZE_MAX) pairs.emplace_back(a, b);
  }
  return e;
}
}  // namespace

extern "C" {

void mmx_config_default(mmx_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->num_envs = 1;
  c->action_mode = MMX_ACTION_EE_POS_QUAT_G_REL;  // gym_env.py:67
  c->reward_type = MMX_REWARD_DENSE;              // gym_env.py:68
  c->max_episode_steps = 500;                     // constants.py:27
  c->spawn_x_range[0] = -0.20;
  c->spawn_x_range[1] = 0.20;
  c->spawn_y_range[0] = 0.30;
  c->spawn_y_range[1] = 0.45;
  c->n_tasks = 9;  // "all" (constants.py:19)
  for (int k = 0; k < 9; k++) {
    c->task_obj[k] = static_cast<int8_t>(k / 3);
    c->task_bin[k] = static_cast<int8_t>(k % 3);
  }
  c->fixed_task_obj = -1;
  c->fixed_task_bin = -1;
  c->image_size = 224;  // constants.py:23
  c->solver_iterations = 30;
  c->solver_tolerance = 1e-6f;
}

int mmx_create(const mmx_config* cfg, mmx_sim** out) {
  if (!cfg || !out) return MMX_EINVAL;
  *out = nullptr;
  if (cfg->image_size < 0 || cfg->image_size > 1024) return MMX_EINVAL;
  if (cfg->num_envs <= 0 || cfg->action_mode < 0 || cfg->action_mode > 4 || cfg->reward_type < 0 ||
      cfg->reward_type > 2 || cfg->n_tasks < 1 || cfg->n_tasks > 9)
    return MMX_EINVAL;
  for (int k = 0; k < cfg->n_tasks; k++)
    if (cfg->task_obj[k] < 0 || cfg->task_obj[k] > 2 || cfg->task_bin[k] < 0 || cfg->task_bin[k] > 2) return MMX_EINVAL;
  mmx_sim* sim = new mmx_sim();
  sim->cfg = *cfg;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) {
    delete sim;
    return MMX_EDEVICE;
  }
  DeviceGuard guard(sim);  // allocations and streams on cfg->device; the caller's device restored
  sim->stream = static_cast<hipStream_t>(cfg->stream);
  const int N = cfg->num_envs;
  MMXState& S = sim->S;
  std::memset(&S, 0, sizeof(S));
  S.N = N;
  S.action_mode = cfg->action_mode;
  S.reward_type = cfg->reward_type;
  S.max_episode_steps = cfg->max_episode_steps;
  S.randomize = cfg->randomize_objects;
  S.image_size = cfg->image_size;
  S.autoreset = cfg->autoreset;
  S.spawn_x0 = cfg->spawn_x_range[0];
  S.spawn_x1 = cfg->spawn_x_range[1];
  S.spawn_y0 = cfg->spawn_y_range[0];
  S.spawn_y1 = cfg->spawn_y_range[1];
  S.ntask = cfg->n_tasks;
  for (int k = 0; k < 9; k++) {
    S.task_obj[k] = k < cfg->n_tasks ? cfg->task_obj[k] : 0;
    S.task_bin[k] = k < cfg->n_tasks ? cfg->task_bin[k] : 0;
  }
  S.fixed_obj = cfg->fixed_task_obj;
  S.fixed_bin = cfg->fixed_task_bin;
  S.solver = MMX_SOLVER_NEWTON;
  S.solver_max_iter = cfg->solver_iterations > 0 ? cfg->solver_iterations : 30;
  S.solver_tol = cfg->solver_tolerance > 0 ? cfg->solver_tolerance : 1e-6f;
  const size_t n = static_cast<size_t>(N);
  S.qpos = dalloc<float>(sim, MMX_NQ_ * n);
  S.qvel = dalloc<float>(sim, MMX_NV_ * n);
  S.ctrl = dalloc<float>(sim, MMX_NU_ * n);
  S.qacc_ws = dalloc<float>(sim, MMX_NV_ * n);
  S.kin = dalloc<float>(sim, KIN_N * n);
  S.target = dalloc<float>(sim, 4 * n);
  S.epi = dalloc<int>(sim, EPI_N * n);
  S.epf = dalloc<float>(sim, EPF_N * n);
  S.rng = dalloc<unsigned long long>(sim, 4 * n);
  S.rng32 = dalloc<unsigned int>(sim, n);
  S.obs = dalloc<float>(sim, MMX_NOBS * n);
  S.reward = dalloc<float>(sim, n);
  S.reward_components = dalloc<float>(sim, 6 * n);
  S.done = dalloc<int>(sim, 3 * n);
  S.con = dalloc<float>(sim, static_cast<size_t>(MMX_MAXCON) * CON_F * n);
  S.stats = dalloc<float>(sim, STAT_N * n);
  S.efc_ovf = dalloc<float>(sim, static_cast<size_t>(MMX_OVF_F) * n);
  S.fault = dalloc<int>(sim, 1);
  sim->expert_action = dalloc<float>(sim, 4 * n);
  sim->d_mask = dalloc<unsigned char>(sim, n);
  sim->d_task = dalloc<int>(sim, n);
  sim->d_order = dalloc<int>(sim, n);
  if (cfg->image_size > 0) {  // camera renderer (mmx_render.hip): poses + RGB + segment ids
    const size_t px = static_cast<size_t>(cfg->image_size) * cfg->image_size;
    S.rpose = dalloc<float>(sim, 14 * 12 * n);
    sim->rpose_alt = dalloc<float>(sim, 14 * 12 * n);
    S.images = dalloc<unsigned char>(sim, 2 * px * 3 * n);
    S.seg = dalloc<unsigned char>(sim, 2 * px * n);
    const size_t sg = static_cast<size_t>((cfg->image_size + 15) & ~15);
    S.bg_overhead = dalloc<unsigned int>(sim, sg * sg);
  }
  for (void* p : sim->allocs)
    if (!p) {
      mmx_destroy(sim);
      return MMX_ENOMEM;
    }
  if (!S.qpos || !S.con || !S.efc_ovf || !S.fault || !sim->d_task || !sim->d_order) {
    mmx_destroy(sim);
    return MMX_ENOMEM;
  }
  // gymnasium's lazily created np_random uses OS entropy when never seeded
  std::random_device rd;
  std::vector<unsigned long long> rng(4 * n);
  for (size_t i = 0; i < n; i++) {
    uint64_t st[4];
    pcg64_seed((static_cast<uint64_t>(rd()) << 32) ^ rd(), st);
    for (int k = 0; k < 4; k++) rng[4 * i + k] = st[k];
  }
  if (hipMemcpy(S.rng, rng.data(), rng.size() * sizeof(unsigned long long), hipMemcpyHostToDevice) != hipSuccess) {
    mmx_destroy(sim);
    return MMX_EDEVICE;
  }
  // rollout lanes: MMX_STREAMS overrides; by default one lane per 1024 envs, at most 4 (the
  // process's hardware queues: more lanes multiplex onto them and gain nothing, C5 8 vs 4 lanes
  // -0.8 %), at most kMaxLanes
  int lanes = std::min(N / 1024, 4);
  if (const char* v = std::getenv("MMX_STREAMS")) lanes = std::atoi(v);
  if (const char* v = std::getenv("MMX_FUSE")) sim->fuse = std::max(1, std::atoi(v));
  // the layout: 192 rows (one env wave + its helper wave, four envs per CU) while the batch fits the
  // chip at four per CU, where each env's own speed counts (C2's 1024 envs: 1.52 M vs 1.29 M env
  // steps/s); 128 rows (twelve per CU) for larger batches, where slots count
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess) cus = 0;
  sim->step_rows = cus > 0 && N <= 4 * cus ? 192 : 128;
  if (const char* v = std::getenv("MMX_STEP_ROWS")) {
    const int r = std::atoi(v);
    if (r == 128 || r == 192) sim->step_rows = r;
  }
  sim->step_order = 1;
  if (const char* v = std::getenv("MMX_STEP_ORDER")) sim->step_order = std::atoi(v) != 0;
  lanes = std::max(1, std::min(lanes, std::min(N, int(mmx_sim::kMaxLanes))));
  if (hipEventCreateWithFlags(&sim->ev_fork, hipEventDisableTiming) != hipSuccess) lanes = 1;
  for (int l = 1; l < lanes; l++)
    if (hipStreamCreateWithFlags(&sim->lane[l], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&sim->ev_join[l], hipEventDisableTiming) != hipSuccess) {
      if (sim->lane[l]) (void)hipStreamDestroy(sim->lane[l]);
      lanes = l;
      break;
    }
  sim->nlanes = lanes;
  sim->render_overlap = sim->rpose_alt != nullptr;
  if (const char* v = std::getenv("MMX_RENDER_OVERLAP")) sim->render_overlap = sim->render_overlap && std::atoi(v) != 0;
  if (sim->render_overlap && (hipStreamCreateWithFlags(&sim->rstream, hipStreamNonBlocking) != hipSuccess ||
                              hipEventCreateWithFlags(&sim->ev_step, hipEventDisableTiming) != hipSuccess ||
                              hipEventCreateWithFlags(&sim->ev_rend[0], hipEventDisableTiming) != hipSuccess ||
                              hipEventCreateWithFlags(&sim->ev_rend[1], hipEventDisableTiming) != hipSuccess))
    sim->render_overlap = 0;
  // the fixed overhead camera's background, once; the handle is published only when the sim is
  // complete (on a failure every allocation is released and *out stays null)
  int rc = S.bg_overhead ? hip_check(sim, mmx_launch_render_bg(&S, sim->stream), "mmx_create background") : 0;
  if (!rc) rc = hip_check(sim, hipDeviceSynchronize(), "mmx_create");
  if (rc) {
    mmx_destroy(sim);
    return rc;
  }
  *out = sim;
  return 0;
}

void mmx_destroy(mmx_sim* sim) {
  if (!sim) return;
  DeviceGuard guard(sim);
  (void)hipDeviceSynchronize();
  for (void* p : sim->allocs)
    if (p) (void)hipFree(p);
  for (int l = 1; l < sim->nlanes; l++) {
    (void)hipEventDestroy(sim->ev_join[l]);
    (void)hipStreamDestroy(sim->lane[l]);
  }
  if (sim->ev_fork) (void)hipEventDestroy(sim->ev_fork);
  for (hipEvent_t ev : {sim->ev_step, sim->ev_rend[0], sim->ev_rend[1]})
    if (ev) (void)hipEventDestroy(ev);
  if (sim->rstream) (void)hipStreamDestroy(sim->rstream);
  for (hipEvent_t ev : sim->ev_pool) (void)hipEventDestroy(ev);
  delete sim;
}

const char* mmx_last_error(const mmx_sim* sim) { return sim ? sim->err.c_str() : "null sim"; }

int mmx_reset(mmx_sim* sim, const uint64_t* seeds, const uint8_t* seed_given, const int32_t* task_override,
              const uint8_t* env_mask) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  MMXState& S = sim->S;
  const size_t n = static_cast<size_t>(S.N);
  if (seeds) {
    // re-seed selected envs: PCG64(SeedSequence(seed)); the 32-bit buffer is cleared
    std::vector<unsigned long long> rng(4 * n);
    if (hipStreamSynchronize(sim->stream) != hipSuccess) return fail(sim, MMX_EDEVICE, "mmx_reset sync");
    if (hipMemcpy(rng.data(), S.rng, rng.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
      return fail(sim, MMX_EDEVICE, "rng readback");
    std::vector<int> epi(EPI_N * n);
    if (hipMemcpy(epi.data(), S.epi, epi.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
      return fail(sim, MMX_EDEVICE, "epi readback");
    for (size_t i = 0; i < n; i++) {
      if (env_mask && !env_mask[i]) continue;
      if (seed_given && !seed_given[i]) continue;
      uint64_t st[4];
      pcg64_seed(seeds[i], st);
      for (int k = 0; k < 4; k++) rng[4 * i + k] = st[k];
      epi[EPI_N * i + EPI_RNG_HAS32] = 0;
    }
    if (hipMemcpy(S.rng, rng.data(), rng.size() * sizeof(unsigned long long), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(S.epi, epi.data(), epi.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
      return fail(sim, MMX_EDEVICE, "rng upload");
  }
  const unsigned char* dmask = nullptr;
  const int* dtask = nullptr;
  if (env_mask) {
    if (hipMemcpyAsync(sim->d_mask, env_mask, n, hipMemcpyHostToDevice, sim->stream) != hipSuccess)
      return fail(sim, MMX_EDEVICE, "mask upload");
    dmask = sim->d_mask;
  }
  if (task_override) {
    for (size_t i = 0; i < n; i++) {
      const int t = task_override[i];
      if (t >= 0 && ((t >> 4) > 2 || (t & 15) > 2)) return fail(sim, MMX_EINVAL, "task_override out of range");
    }
    if (hipMemcpyAsync(sim->d_task, task_override, n * sizeof(int), hipMemcpyHostToDevice, sim->stream) != hipSuccess)
      return fail(sim, MMX_EDEVICE, "task upload");
    dtask = sim->d_task;
  }
  int rc = hip_check(sim, mmx_launch_reset(&S, dmask, dtask, sim->stream), "mmx_reset");
  if (rc) return rc;
  rc = hip_check(sim, mmx_launch_render(&S, 0, S.N, sim->stream), "mmx_reset render");
  if (rc) return rc;
  rc = hip_check(sim, hipStreamSynchronize(sim->stream), "mmx_reset sync");
  return rc ? rc : check_fault(sim, "mmx_reset");
}

namespace {
static hipError_t launch_step(const mmx_sim* sim, const float* action, int adim, int expert, int base, int count, int nsteps,
                              hipStream_t st, const int* order = nullptr, const MMXState* S = nullptr) {
  if (!S) S = &sim->S;
  return sim->step_rows == 192 ? mmx_launch_step_l192(S, action, adim, expert, base, count, nsteps, st, order)
                               : mmx_launch_step(S, action, adim, expert, base, count, nsteps, st, order);
}
}  // namespace

int mmx_set_step_rows(mmx_sim* sim, int32_t rows) {
  if (!sim || (rows != 128 && rows != 192)) return MMX_EINVAL;
  sim->step_rows = rows;
  return MMX_OK;
}
int mmx_step_rows(const mmx_sim* sim) { return sim ? sim->step_rows : 0; }
int mmx_set_step_order(mmx_sim* sim, int32_t on) {
  if (!sim || (on != 0 && on != 1)) return MMX_EINVAL;
  sim->step_order = on;
  return MMX_OK;
}
int mmx_step_order(const mmx_sim* sim) { return sim ? sim->step_order : -1; }

int mmx_step(mmx_sim* sim, const float* action_dev, int32_t action_dim) {
  if (!sim || !action_dev) return MMX_EINVAL;
  DeviceGuard guard(sim);
  static const int kDim[5] = {4, 8, 10, 8, 10};
  if (action_dim < kDim[sim->S.action_mode]) return fail(sim, MMX_EINVAL, "action_dim too small for action_mode");
  // longest first by FSM phase (the expert's plan keeps it current; with policy actions it stays idle
  // and the order is index order up to ties)
  int* ord = sim->step_order ? sim->d_order : nullptr;
  hipError_t e = ord ? mmx_launch_order(&sim->S, 0, sim->S.N, ord, 1024, sim->stream) : hipSuccess;
  if (e == hipSuccess) e = launch_step(sim, action_dev, action_dim, 0, 0, sim->S.N, 1, sim->stream, ord);
  if (e == hipSuccess) e = mmx_launch_render(&sim->S, 0, sim->S.N, sim->stream);
  return hip_check(sim, e, "mmx_step");
}

int mmx_expert_plan(mmx_sim* sim, int32_t n_steps, float* action_dev_out) {
  if (!sim || n_steps < 0) return MMX_EINVAL;
  DeviceGuard guard(sim);
  return hip_check(sim, mmx_launch_expert(&sim->S, n_steps, action_dev_out, sim->stream), "mmx_expert_plan");
}


int mmx_kernel_timing(mmx_sim* sim, int32_t enable) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  if (enable) {  // start a new collection (the pool's events are reused)
    sim->ev_used = 0;
    sim->t_step.clear();
    sim->t_render.clear();
    // pre-size the pool, so no hipEventCreate runs between the launches of a timed window (2 events
    // per launch: a C5 window of 128 env steps on 4 lanes records 2048)
    while (sim->ev_pool.size() < kTimingPoolPresize) {
      hipEvent_t ev;
      if (hipEventCreate(&ev) != hipSuccess) break;
      sim->ev_pool.push_back(ev);
    }
  }
  sim->timing = enable != 0;
  return MMX_OK;
}

int mmx_kernel_times(mmx_sim* sim, float* step_ms, int32_t* step_launches, float* render_ms, int32_t* render_launches) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  auto sum = [&](const std::vector<std::pair<size_t, size_t>>& v, float* ms, int32_t* n) -> hipError_t {
    double tot = 0.0;
    for (const auto& pr : v) {
      hipError_t e = hipEventSynchronize(sim->ev_pool[pr.second]);
      float t = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&t, sim->ev_pool[pr.first], sim->ev_pool[pr.second]);
      if (e != hipSuccess) return e;
      tot += t;
    }
    if (ms) *ms = (float)tot;
    if (n) *n = (int32_t)v.size();
    return hipSuccess;
  };
  hipError_t e = sum(sim->t_step, step_ms, step_launches);
  if (e == hipSuccess) e = sum(sim->t_render, render_ms, render_launches);
  return hip_check(sim, e, "mmx_kernel_times");
}

// Launch plan of an n-step expert rollout without cameras.  A launch runs `len` consecutive env steps
// of its lane's envs, len = min(fuse, ceil(n / 4)); lane l of L starts with a launch of l * len / L
// steps (none for lane 0), then launches of len, then the remainder, so the lanes' launch boundaries
// are spread over the launch period instead of falling together.  Every launch ends with a drain (its
// slowest workgroups finish while its slots empty); the other lanes fill the slots it frees as long as
// they are not draining at the same time.  Measured on the driver's 20-step windows
// (tools/sweep_env.py, profiles/r06_sweep_driver_plans.json): equal 3-step launches, all lanes in step,
// 2.72 M env steps/s; the staggered 5-step plan 2.87 M (+5.4 %); staggered 3-, 4-, 6-, 7-, 10-step
// plans and 1-step final launches between them; 512-step windows +0.5 % (16-step launches offset by 4).
// With cameras every step is rendered: one step per launch, one lane.
static int rollout_len(const mmx_sim* sim, int n) {
  if (sim->S.image_size > 0) return 1;
  return std::max(1, std::min(sim->fuse, (n + 3) / 4));
}
// lanes of a rollout: with cameras one (every step ends in the render over all envs, and one launch
// orders all envs longest-first: C5 +2.0 % over 4 lanes)
static int rollout_lanes(const mmx_sim* sim) { return sim->S.image_size > 0 ? 1 : sim->nlanes; }
// Launch lengths of lane `lane` for an n-step rollout (above); env MMX_PLAN = "a,b,...[;c,d,...]" per
// lane (the last list repeats for the lanes after it) overrides it for experiments when its lengths sum
// to n.
static std::vector<int> rollout_plan(const mmx_sim* sim, int n, int lane) {
  std::vector<int> v;
  if (const char* e = std::getenv("MMX_PLAN")) {
    std::string all(e), mine;
    size_t pos = 0;
    for (int l = 0;; l++) {
      const size_t sc = all.find(';', pos);
      mine = all.substr(pos, sc == std::string::npos ? std::string::npos : sc - pos);
      if (l == lane || sc == std::string::npos) break;
      pos = sc + 1;
    }
    int sum = 0;
    for (size_t a = 0; a < mine.size();) {
      const int k = std::atoi(mine.c_str() + a);
      if (k <= 0) break;
      v.push_back(k);
      sum += k;
      const size_t c = mine.find(',', a);
      if (c == std::string::npos) break;
      a = c + 1;
    }
    if (sum == n) return v;
    v.clear();
  }
  if (n <= 0) return v;
  const int len = rollout_len(sim, n), L = rollout_lanes(sim);
  int rem = n;
  const int first = std::min(rem, lane * len / std::max(L, 1));
  if (first > 0) {
    v.push_back(first);
    rem -= first;
  }
  for (; rem > 0; rem -= std::min(rem, len)) v.push_back(std::min(rem, len));
  return v;
}
// the most launches any lane makes
static int rollout_launches(const mmx_sim* sim, int n) {
  size_t m = 0;
  for (int l = 0; l < rollout_lanes(sim); l++) m = std::max(m, rollout_plan(sim, n, l).size());
  return (int)m;
}
int mmx_rollout_launches(const mmx_sim* sim, int32_t n_env_steps) {
  return sim ? rollout_launches(sim, n_env_steps) : 0;
}
int mmx_rollout_expert(mmx_sim* sim, int32_t n_env_steps) {
  if (!sim || sim->S.action_mode != MMX_ACTION_ABS_POS) return MMX_EINVAL;
  DeviceGuard guard(sim);
  const int N = sim->S.N, L = n_env_steps > 1 ? rollout_lanes(sim) : 1;
  hipError_t e = hipSuccess;
  if (sim->render_overlap && sim->S.image_size > 0 && n_env_steps > 1) {
    // the render of step k on its own stream beside the step k + 1 on the caller's stream (a render
    // workgroup's 80 KB of LDS fits a CU the step launch's tail has half emptied: C5 +6.6 %, DESIGN
    // §8 f1); step k writes the pose buffer render k - 2 read, so it waits for that render only
    hipStream_t rs = sim->rstream;
    float* rp[2] = {sim->S.rpose, sim->rpose_alt};
    for (int k = 0; k < n_env_steps && e == hipSuccess; k++) {
      MMXState Sk = sim->S;
      Sk.rpose = rp[k & 1];
      if (k >= 2) e = hipStreamWaitEvent(sim->stream, sim->ev_rend[k & 1], 0);
      int* ord = sim->step_order ? sim->d_order : nullptr;
      if (e == hipSuccess && ord) e = mmx_launch_order(&Sk, 0, N, ord, 1024, sim->stream);
      if (e == hipSuccess)
        e = timed(sim, sim->stream, sim->t_step,
                  [&] { return launch_step(sim, sim->expert_action, 4, 1, 0, N, 1, sim->stream, ord, &Sk); });
      if (e == hipSuccess) e = hipEventRecord(sim->ev_step, sim->stream);
      if (e == hipSuccess) e = hipStreamWaitEvent(rs, sim->ev_step, 0);
      if (e == hipSuccess) e = timed(sim, rs, sim->t_render, [&] { return mmx_launch_render(&Sk, 0, N, rs); });
      if (e == hipSuccess) e = hipEventRecord(sim->ev_rend[k & 1], rs);
    }
    // the caller's stream sees the last render; S.rpose names the newest poses
    if (e == hipSuccess) e = hipStreamWaitEvent(sim->stream, sim->ev_rend[(n_env_steps - 1) & 1], 0);
    if (e == hipSuccess && ((n_env_steps - 1) & 1)) std::swap(sim->S.rpose, sim->rpose_alt);
    return hip_check(sim, e, "mmx_rollout_expert");
  }
  if (L > 1) {  // fork: every lane starts after the work already queued on the caller's stream
    e = hipEventRecord(sim->ev_fork, sim->stream);
    for (int l = 1; l < L && e == hipSuccess; l++) e = hipStreamWaitEvent(sim->lane[l], sim->ev_fork, 0);
  }
  // the step kernel plans with the FSM itself (expert=1); step k of range l only depends on step
  // k-1 of range l.  Without cameras a launch runs up to `fuse` consecutive steps of its envs
  // (mmx_rollout_steps_per_launch); with cameras every step is rendered, one step per launch.
  std::vector<int> plan[mmx_sim::kMaxLanes];
  size_t nl = 0;
  for (int l = 0; l < L; l++) {
    plan[l] = rollout_plan(sim, n_env_steps, l);
    nl = std::max(nl, plan[l].size());
  }
  // with cameras (L = 1): the step of all envs, then ONE render launch over all envs (the render's
  // 80 KB workgroups cannot share a CU with the step kernel's: a render per lane beside the other
  // lanes' steps ran as a trickle, C5 -2.8 %)
  for (size_t r = 0; r < nl && e == hipSuccess; r++) {
    for (int l = 0; l < L && e == hipSuccess; l++) {
      if (r >= plan[l].size()) continue;
      const int ns = plan[l][r];
      const int b0 = (int)((long)N * l / L), b1 = (int)((long)N * (l + 1) / L);
      hipStream_t st = l ? sim->lane[l] : sim->stream;
      int* ord = sim->step_order ? sim->d_order + b0 : nullptr;  // the lane's slice of the order buffer
      if (ord) e = mmx_launch_order(&sim->S, b0, b1 - b0, ord, L > 1 ? 64 : 1024, st);
      if (e == hipSuccess)
        e = timed(sim, st, sim->t_step,
                  [&] { return launch_step(sim, sim->expert_action, 4, 1, b0, b1 - b0, ns, st, ord); });
    }
    if (e == hipSuccess && sim->S.image_size > 0)
      e = timed(sim, sim->stream, sim->t_render, [&] { return mmx_launch_render(&sim->S, 0, N, sim->stream); });
  }
  if (L > 1)  // join: the caller's stream sees the whole rollout, as with a single launch chain
    for (int l = 1; l < L; l++) {
      hipError_t j = hipEventRecord(sim->ev_join[l], sim->lane[l]);
      if (j == hipSuccess) j = hipStreamWaitEvent(sim->stream, sim->ev_join[l], 0);
      if (e == hipSuccess) e = j;
    }
  return hip_check(sim, e, "mmx_rollout_expert");
}

int mmx_rollout_lanes(const mmx_sim* sim) { return sim ? rollout_lanes(sim) : 0; }
int mmx_rollout_render_overlap(const mmx_sim* sim) { return sim ? sim->render_overlap : 0; }
int mmx_rollout_render_launches(const mmx_sim* sim) {
  return sim && sim->S.image_size > 0 ? 1 : 0;
}

// the row-above match uses deflate distance 3 W + 1, which deflate caps at 32768: W <= 10922
static bool png_size_ok(int32_t width, int32_t height) {
  return width > 0 && height > 0 && height <= 1024 && width <= MMX_PNG_MAX_WIDTH;
}
int64_t mmx_png_bound(int32_t width, int32_t height) {
  return png_size_ok(width, height) ? mmx_png_bound_bytes(width, height) : -1;
}
int64_t mmx_png_scratch(int32_t width, int32_t height) {
  return png_size_ok(width, height) ? mmx_png_scratch_bytes(width, height) : -1;
}

int mmx_png_encode(mmx_sim* sim, const uint8_t* rgb_dev, int64_t img_stride, int32_t n, int32_t width, int32_t height,
                   uint8_t* out_dev, int64_t out_stride, int32_t* sizes_dev, void* scratch_dev) {
  if (!sim || n < 0 || (n > 0 && (!rgb_dev || !out_dev || !sizes_dev || !scratch_dev)) || !png_size_ok(width, height) ||
      img_stride < 3LL * width * height || out_stride < mmx_png_bound_bytes(width, height))
    return sim ? fail(sim, MMX_EINVAL, "mmx_png_encode: bad arguments") : MMX_EINVAL;
  DeviceGuard guard(sim);
  return hip_check(sim, mmx_launch_png(rgb_dev, img_stride, n, width, height, out_dev, out_stride, sizes_dev,
                                       static_cast<uint32_t*>(scratch_dev), sim->stream), "mmx_png_encode");
}

int mmx_png_pack(mmx_sim* sim, const uint8_t* out_dev, int64_t out_stride, const int32_t* sizes_dev,
                 const int64_t* offsets_dev, int32_t n, uint8_t* packed_dev) {
  if (!sim || n < 0 || (n > 0 && (!out_dev || !sizes_dev || !offsets_dev || !packed_dev)))
    return sim ? fail(sim, MMX_EINVAL, "mmx_png_pack: bad arguments") : MMX_EINVAL;
  DeviceGuard guard(sim);
  return hip_check(sim, mmx_launch_png_pack(out_dev, out_stride, sizes_dev, offsets_dev, n, packed_dev, sim->stream),
                   "mmx_png_pack");
}

int mmx_image_stats(mmx_sim* sim, const uint8_t* rgb_dev, int64_t img_stride, int32_t n, int32_t width, int32_t height,
                    int64_t* out_dev) {
  if (!sim || n < 0 || (n > 0 && (!rgb_dev || !out_dev)) || width <= 0 || height <= 0 || width > 4096 ||
      height > 4096 || img_stride < 3LL * width * height)
    return sim ? fail(sim, MMX_EINVAL, "mmx_image_stats: bad arguments") : MMX_EINVAL;
  DeviceGuard guard(sim);
  return hip_check(sim, mmx_launch_image_stats(rgb_dev, img_stride, n, (int64_t)width * height, out_dev, sim->stream),
                   "mmx_image_stats");
}

int64_t mmx_copy_ranges(int64_t n, const uint64_t* src, const uint64_t* dst, const int64_t* len) {
  if (n < 0 || (n > 0 && (!src || !dst || !len))) return -1;
  int64_t total = 0;
  for (int64_t k = 0; k < n; k++) {
    if (len[k] < 0) return -1;
    total += len[k];
  }
  for (int64_t k = 0; k < n; k++)
    if (len[k])
      std::memcpy(reinterpret_cast<void*>(static_cast<uintptr_t>(dst[k])),
                  reinterpret_cast<const void*>(static_cast<uintptr_t>(src[k])), (size_t)len[k]);
  return total;
}

int mmx_rollout_steps_per_launch(const mmx_sim* sim) {
  return sim ? (sim->S.image_size > 0 ? 1 : sim->fuse) : 0;
}

int mmx_physics_step(mmx_sim* sim, int32_t n, int32_t with_ik) {
  if (!sim || n < 0) return MMX_EINVAL;
  DeviceGuard guard(sim);
  return hip_check(sim, mmx_launch_physics(&sim->S, n, with_ik, sim->stream), "mmx_physics_step");
}

int mmx_expert_physics(mmx_sim* sim, int32_t n) {
  if (!sim || n < 0) return MMX_EINVAL;
  DeviceGuard guard(sim);
  hipError_t e = hipSuccess;
  for (int k = 0; k < n && e == hipSuccess; k += 256)  // bounded launches (a few ms each)
    e = mmx_launch_expert_physics(&sim->S, std::min(256, n - k), sim->stream);
  return hip_check(sim, e, "mmx_expert_physics");
}

int mmx_eval_reward(mmx_sim* sim, const float* obj, const float* ee, const float* ctrl7, const int32_t* pairs,
                    int32_t max_pairs) {
  if (!sim || !obj || !ee || !ctrl7 || max_pairs < 0 || (max_pairs > 0 && !pairs)) return MMX_EINVAL;
  DeviceGuard guard(sim);
  return hip_check(sim, mmx_launch_reward(&sim->S, obj, ee, ctrl7, pairs, max_pairs, sim->stream), "mmx_eval_reward");
}

int mmx_forward(mmx_sim* sim) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  hipError_t e = mmx_launch_forward(&sim->S, sim->stream);
  if (e == hipSuccess) e = mmx_launch_render(&sim->S, 0, sim->S.N, sim->stream);
  return hip_check(sim, e, "mmx_forward");
}

int mmx_get_buffers(mmx_sim* sim, mmx_buffers* b) {
  if (!sim || !b) return MMX_EINVAL;
  const MMXState& S = sim->S;
  b->num_envs = S.N;
  b->qpos = S.qpos;
  b->qvel = S.qvel;
  b->ctrl = S.ctrl;
  b->qacc_warmstart = S.qacc_ws;
  b->obs = S.obs;
  b->reward = S.reward;
  b->done = S.done;
  b->reward_components = S.reward_components;
  b->episode_i = S.epi;
  b->episode_f = S.epf;
  b->kin = S.kin;
  b->stats = S.stats;
  b->contacts = S.con;
  b->images = S.images;
  b->seg = S.seg;
  b->target = S.target;
  return MMX_OK;
}

int mmx_synchronize(mmx_sim* sim) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  const int rc = hip_check(sim, hipStreamSynchronize(sim->stream), "mmx_synchronize");
  return rc ? rc : check_fault(sim, "mmx_synchronize");
}

int mmx_get_state(mmx_sim* sim, float* qpos, float* qvel, float* ctrl, float* ws) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  const size_t n = static_cast<size_t>(sim->S.N);
  hipError_t e = hipStreamSynchronize(sim->stream);
  if (e == hipSuccess && qpos) e = hipMemcpy(qpos, sim->S.qpos, MMX_NQ_ * n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && qvel) e = hipMemcpy(qvel, sim->S.qvel, MMX_NV_ * n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && ctrl) e = hipMemcpy(ctrl, sim->S.ctrl, MMX_NU_ * n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && ws) e = hipMemcpy(ws, sim->S.qacc_ws, MMX_NV_ * n * 4, hipMemcpyDeviceToHost);
  return hip_check(sim, e, "mmx_get_state");
}

int mmx_set_state(mmx_sim* sim, const float* qpos, const float* qvel, const float* ctrl, const float* ws) {
  if (!sim) return MMX_EINVAL;
  DeviceGuard guard(sim);
  const size_t n = static_cast<size_t>(sim->S.N);
  hipError_t e = hipStreamSynchronize(sim->stream);
  if (e == hipSuccess && qpos) e = hipMemcpy(sim->S.qpos, qpos, MMX_NQ_ * n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && qvel) e = hipMemcpy(sim->S.qvel, qvel, MMX_NV_ * n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && ctrl) e = hipMemcpy(sim->S.ctrl, ctrl, MMX_NU_ * n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && ws) e = hipMemcpy(sim->S.qacc_ws, ws, MMX_NV_ * n * 4, hipMemcpyHostToDevice);
  return hip_check(sim, e, "mmx_set_state");
}

int mmx_queue_init(mmx_sim* sim, int32_t n_episodes, const uint64_t* seeds, const int32_t* tasks) {
  if (!sim || n_episodes < 0 || (n_episodes > 0 && !tasks)) return MMX_EINVAL;
  DeviceGuard guard(sim);
  const size_t E = static_cast<size_t>(n_episodes), n = static_cast<size_t>(sim->S.N);
  for (size_t e = 0; e < E; e++) {
    const int t = tasks[e];
    if (t >= 0 && ((t >> 4) > 2 || (t & 15) > 2)) return fail(sim, MMX_EINVAL, "queue task out of range");
  }
  if (hipStreamSynchronize(sim->stream) != hipSuccess) return fail(sim, MMX_EDEVICE, "mmx_queue_init sync");
  for (void* p : {static_cast<void*>(sim->q_slot), static_cast<void*>(sim->q_next), static_cast<void*>(sim->q_task),
                  static_cast<void*>(sim->q_rng)}) {
    if (!p) continue;
    sim->allocs.erase(std::remove(sim->allocs.begin(), sim->allocs.end(), p), sim->allocs.end());
    (void)hipFree(p);
  }
  sim->q_rng = nullptr;
  sim->q_n = -1;
  sim->q_slot = dalloc<int>(sim, n);
  sim->q_next = dalloc<int>(sim, 1);
  sim->q_task = dalloc<int>(sim, std::max<size_t>(E, 1));
  if (!sim->q_slot || !sim->q_next || !sim->q_task) return fail(sim, MMX_EDEVICE, "queue allocation");
  std::vector<int> slot(n, -1);
  hipError_t e = hipMemcpy(sim->q_slot, slot.data(), n * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess && E) e = hipMemcpy(sim->q_task, tasks, E * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess && seeds && E) {  // PCG64(SeedSequence(seed_e)) of every episode, once
    std::vector<unsigned long long> rng(4 * E);
    for (size_t k = 0; k < E; k++) {
      uint64_t st[4];
      pcg64_seed(seeds[k], st);
      for (int j = 0; j < 4; j++) rng[4 * k + j] = st[j];
    }
    sim->q_rng = dalloc<unsigned long long>(sim, 4 * E);
    if (!sim->q_rng) return fail(sim, MMX_EDEVICE, "queue allocation");
    e = hipMemcpy(sim->q_rng, rng.data(), rng.size() * sizeof(unsigned long long), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) return hip_check(sim, e, "mmx_queue_init upload");
  sim->q_n = n_episodes;
  return MMX_OK;
}

int mmx_queue_advance(mmx_sim* sim, int32_t* slot_ep_dev, int32_t* fin_ep_dev) {
  if (!sim) return MMX_EINVAL;
  if (sim->q_n < 0) return fail(sim, MMX_EINVAL, "mmx_queue_advance without mmx_queue_init");
  DeviceGuard guard(sim);
  MMXState& S = sim->S;
  hipError_t e = mmx_launch_queue(&S, sim->q_slot, sim->q_next, sim->q_n, sim->q_rng, sim->q_task, sim->d_mask,
                                  sim->d_task, slot_ep_dev, fin_ep_dev, sim->stream);
  if (e == hipSuccess) e = mmx_launch_reset(&S, sim->d_mask, sim->d_task, sim->stream);
  if (e == hipSuccess) e = mmx_launch_render_masked(&S, 0, S.N, sim->d_mask, sim->stream);
  return hip_check(sim, e, "mmx_queue_advance");
}

uint32_t mmx_episode_seed(uint64_t root, int32_t index) {
  return seedseq(seed_words(root), {static_cast<uint32_t>(index)}, 1)[0];
}

}  // extern "C"
