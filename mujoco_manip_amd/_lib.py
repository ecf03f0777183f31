"""ctypes binding of libmmx.so (include/mmx_api.h).

This is the reference-side binding a maintainer would add: the reference is Python, so the
binding to the C-ABI is ctypes.  Device buffers are exchanged as raw pointers; torch is used
only to own action tensors and to view sim-owned buffers (``__cuda_array_interface__``).
The product path fails loudly when the HIP library or the GPU is missing: there is no CPU
fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _build

NQ, NV, NU, NOBS = 30, 27, 8, 85
MAXCON, CON_F = 64, 13
PNG_MAX_WIDTH = 10922  # include/mmx_api.h MMX_PNG_MAX_WIDTH
MMX_ESAMPLING = -4  # include/mmx_api.h: spawn sampling exhausted (randomization.py:84-87 raises RuntimeError)
# env_error bits (mujoco_manip_amd/csrc/mmx_state.h)
ERR_CON_OVERFLOW, ERR_EFC_OVERFLOW, ERR_NAN, ERR_SAMPLING = 1, 2, 4, 8
EPI_N, EPF_N, KIN_N, STAT_N = 18, 28, 63, 19
EPI_FIELDS = ("obj", "bin", "step_count", "flags", "fsm_state", "fsm_task_index", "fsm_settle", "fsm_gripper_open",
              "fsm_has_target", "env_error", "ncon", "nefc", "episodes", "rng_has32", "successes", "placed", "error_resets",
              "fsm_phases")
EPI = {name: k for k, name in enumerate(EPI_FIELDS)}
STAT_FIELDS = ("sum_nefc", "sum_ncon", "sum_solver_iter", "substeps", "max_resid", "cyc_ik", "cyc_kinematics",
               "cyc_dynamics", "cyc_collision", "cyc_constraints", "cyc_solver", "cyc_integrate", "cyc_step_end",
               "cyc_aux0", "cyc_aux1", "cyc_aux2", "cyc_aux3", "exit_stall", "exit_cap")
ACTION_MODES = ("abs_pos", "ee_pos_quat_g", "ee_pos_rot6d_g", "ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel")
ACTION_DIMS = (4, 8, 10, 8, 10)
REWARD_TYPES = ("dense", "sparse", "staged")


class MMXConfig(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("device", C.c_int32), ("action_mode", C.c_int32), ("reward_type", C.c_int32),
        ("max_episode_steps", C.c_int32), ("randomize_objects", C.c_int32),
        ("spawn_x_range", C.c_double * 2), ("spawn_y_range", C.c_double * 2),
        ("n_tasks", C.c_int32), ("task_obj", C.c_int8 * 9), ("task_bin", C.c_int8 * 9),
        ("fixed_task_obj", C.c_int32), ("fixed_task_bin", C.c_int32), ("image_size", C.c_int32),
        ("autoreset", C.c_int32), ("solver_iterations", C.c_int32), ("solver_tolerance", C.c_float),
        ("stream", C.c_void_p),
    ]


class MMXBuffers(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("qpos", C.c_void_p), ("qvel", C.c_void_p), ("ctrl", C.c_void_p),
        ("qacc_warmstart", C.c_void_p), ("obs", C.c_void_p), ("reward", C.c_void_p), ("done", C.c_void_p),
        ("reward_components", C.c_void_p), ("episode_i", C.c_void_p), ("episode_f", C.c_void_p),
        ("kin", C.c_void_p), ("stats", C.c_void_p), ("contacts", C.c_void_p),
        ("images", C.c_void_p), ("seg", C.c_void_p), ("target", C.c_void_p),
    ]


EXPORTED = ("mmx_config_default", "mmx_create", "mmx_destroy", "mmx_last_error", "mmx_reset", "mmx_step",
            "mmx_expert_plan", "mmx_rollout_expert", "mmx_physics_step", "mmx_forward", "mmx_get_buffers",
            "mmx_synchronize", "mmx_get_state", "mmx_set_state", "mmx_episode_seed", "mmx_rollout_lanes",
            "mmx_rollout_steps_per_launch", "mmx_rollout_launches", "mmx_expert_physics", "mmx_eval_reward", "mmx_kernel_timing",
            "mmx_kernel_times", "mmx_png_bound", "mmx_png_scratch", "mmx_png_encode", "mmx_png_pack", "mmx_image_stats",
            "mmx_queue_init", "mmx_queue_advance", "mmx_set_step_rows", "mmx_step_rows", "mmx_copy_ranges", "mmx_rollout_render_launches",
            "mmx_set_step_order", "mmx_step_order", "mmx_rollout_render_overlap")

_lib = None


def load(build_if_missing: bool = True):
    """Load libmmx.so (built in-tree by _build.build)."""
    global _lib
    if _lib is not None:
        return _lib
    profile = os.environ.get("MMX_PROFILE", "0") not in ("", "0")
    # MMX_LIB_PATH: a prebuilt variant of the same sources (diagnostic probe builds, experiments)
    path = os.environ.get("MMX_LIB_PATH") or _build.lib_path(profile)
    if not os.path.exists(path):
        if not build_if_missing:
            raise RuntimeError(f"{os.path.basename(path)} missing at {path}; run __graft_entry__.build()")
        _build.build(profile=profile)
    L = C.CDLL(path)
    vp, u8p, i32p, u64p, fp = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.POINTER(C.c_float)
    L.mmx_config_default.argtypes = [C.POINTER(MMXConfig)]
    L.mmx_create.argtypes = [C.POINTER(MMXConfig), C.POINTER(vp)]
    L.mmx_destroy.argtypes = [vp]
    L.mmx_last_error.restype = C.c_char_p
    L.mmx_last_error.argtypes = [vp]
    L.mmx_reset.argtypes = [vp, u64p, u8p, i32p, u8p]
    L.mmx_step.argtypes = [vp, vp, C.c_int32]
    L.mmx_expert_plan.argtypes = [vp, C.c_int32, vp]
    L.mmx_rollout_expert.argtypes = [vp, C.c_int32]
    L.mmx_physics_step.argtypes = [vp, C.c_int32, C.c_int32]
    L.mmx_rollout_lanes.argtypes = [vp]
    L.mmx_rollout_lanes.restype = C.c_int
    L.mmx_rollout_render_launches.argtypes = [vp]
    L.mmx_rollout_render_launches.restype = C.c_int
    L.mmx_copy_ranges.argtypes = [C.c_int64, vp, vp, vp]
    L.mmx_copy_ranges.restype = C.c_int64
    L.mmx_set_step_rows.argtypes = [vp, C.c_int32]
    L.mmx_step_rows.argtypes = [vp]
    L.mmx_step_rows.restype = C.c_int
    L.mmx_set_step_order.argtypes = [vp, C.c_int32]
    L.mmx_rollout_render_overlap.argtypes = [vp]
    L.mmx_rollout_render_overlap.restype = C.c_int
    L.mmx_step_order.argtypes = [vp]
    L.mmx_step_order.restype = C.c_int
    L.mmx_rollout_steps_per_launch.argtypes = [vp]
    L.mmx_rollout_steps_per_launch.restype = C.c_int
    L.mmx_rollout_launches.argtypes = [vp, C.c_int32]
    L.mmx_rollout_launches.restype = C.c_int
    L.mmx_forward.argtypes = [vp]
    L.mmx_expert_physics.argtypes = [vp, C.c_int32]
    L.mmx_eval_reward.argtypes = [vp, vp, vp, vp, vp, C.c_int32]
    L.mmx_kernel_timing.argtypes = [vp, C.c_int32]
    L.mmx_png_bound.argtypes = [C.c_int32, C.c_int32]
    L.mmx_png_bound.restype = C.c_int64
    L.mmx_png_scratch.argtypes = [C.c_int32, C.c_int32]
    L.mmx_png_scratch.restype = C.c_int64
    L.mmx_png_encode.argtypes = [vp, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int64, vp, vp]
    L.mmx_png_pack.argtypes = [vp, vp, C.c_int64, vp, vp, C.c_int32, vp]
    L.mmx_image_stats.argtypes = [vp, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp]
    L.mmx_kernel_times.argtypes = [vp, fp, i32p, fp, i32p]
    L.mmx_get_buffers.argtypes = [vp, C.POINTER(MMXBuffers)]
    L.mmx_synchronize.argtypes = [vp]
    L.mmx_get_state.argtypes = [vp, fp, fp, fp, fp]
    L.mmx_set_state.argtypes = [vp, fp, fp, fp, fp]
    L.mmx_queue_init.argtypes = [vp, C.c_int32, u64p, i32p]
    L.mmx_queue_advance.argtypes = [vp, vp, vp]
    L.mmx_episode_seed.restype = C.c_uint32
    L.mmx_episode_seed.argtypes = [C.c_uint64, C.c_int32]
    for name in ("mmx_create", "mmx_reset", "mmx_step", "mmx_expert_plan", "mmx_rollout_expert", "mmx_physics_step",
                 "mmx_forward", "mmx_get_buffers", "mmx_synchronize", "mmx_get_state", "mmx_set_state",
                 "mmx_expert_physics", "mmx_eval_reward", "mmx_kernel_timing", "mmx_kernel_times", "mmx_png_encode",
                 "mmx_png_pack", "mmx_image_stats", "mmx_queue_init", "mmx_queue_advance", "mmx_set_step_rows", "mmx_set_step_order"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


def episode_seed(root: int, index: int) -> int:
    """SeedSequence(root).spawn(n)[index].generate_state(1)[0] (generate_dataset.py:263-268)."""
    return int(load().mmx_episode_seed(root, index))


class _DevArray:
    """Minimal __cuda_array_interface__ exporter for a sim-owned device buffer."""

    def __init__(self, ptr: int, shape, typestr: str, owner):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2, "strides": None}
        self._owner = owner


def _fptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


class Sim:
    """Owner of one mmx_sim (a batch of num_envs environments on one GPU)."""

    def __init__(self, num_envs: int, *, action_mode: str = "ee_pos_quat_g_rel", reward_type: str = "dense",
                 max_episode_steps: int = 500, randomize_objects: bool = False,
                 spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45), task_pool=None, fixed_task=None,
                 image_size: int = 224, autoreset: bool = False, solver_iterations: int = 30,
                 solver_tolerance: float = 1e-6, device: int = 0, stream: int | None = None):
        if action_mode not in ACTION_MODES:
            raise ValueError(f"action_mode must be one of {ACTION_MODES}, got '{action_mode}'")
        if reward_type not in REWARD_TYPES:
            raise ValueError(f"reward_type must be one of {REWARD_TYPES}, got '{reward_type}'")
        if not (0 <= int(image_size) <= 1024):
            raise ValueError(f"image_size must be in [0, 1024] (0 = no cameras), got {image_size}")
        if int(num_envs) <= 0:
            raise ValueError(f"num_envs must be positive, got {num_envs}")
        self.L = load()
        cfg = MMXConfig()
        self.L.mmx_config_default(C.byref(cfg))
        cfg.num_envs = int(num_envs)
        cfg.device = int(device)
        cfg.action_mode = ACTION_MODES.index(action_mode)
        cfg.reward_type = REWARD_TYPES.index(reward_type)
        cfg.max_episode_steps = int(max_episode_steps)
        cfg.randomize_objects = int(bool(randomize_objects))
        cfg.spawn_x_range[0], cfg.spawn_x_range[1] = spawn_x_range
        cfg.spawn_y_range[0], cfg.spawn_y_range[1] = spawn_y_range
        if task_pool is not None:
            cfg.n_tasks = len(task_pool)
            for k, (o, b) in enumerate(task_pool):
                cfg.task_obj[k], cfg.task_bin[k] = o, b
        if fixed_task is not None:
            cfg.fixed_task_obj, cfg.fixed_task_bin = fixed_task
        cfg.image_size = int(image_size)
        cfg.autoreset = int(bool(autoreset))
        cfg.solver_iterations = int(solver_iterations)
        cfg.solver_tolerance = float(solver_tolerance)
        cfg.stream = stream
        self.cfg = cfg
        self.num_envs = int(num_envs)
        self.action_dim = ACTION_DIMS[cfg.action_mode]
        ptr = C.c_void_p()
        rc = self.L.mmx_create(C.byref(cfg), C.byref(ptr))
        if rc != 0 or not ptr.value:
            raise RuntimeError(f"mmx_create failed ({rc}): no usable MI355X / HIP device?")
        self.ptr = ptr
        self.buffers = MMXBuffers()
        self._check(self.L.mmx_get_buffers(self.ptr, C.byref(self.buffers)), "mmx_get_buffers")

    def _check(self, rc, what):
        if rc == MMX_ESAMPLING:  # the reference's own exception and message (randomization.py:84-87)
            raise RuntimeError(self.L.mmx_last_error(self.ptr).decode())
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {self.L.mmx_last_error(self.ptr).decode()}")

    def close(self):
        if getattr(self, "ptr", None) is not None and self.ptr.value:
            self.L.mmx_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- C-ABI calls
    def reset(self, seeds=None, task_override=None, env_mask=None):
        N = self.num_envs
        u64p, u8p, i32p = C.POINTER(C.c_uint64), C.POINTER(C.c_uint8), C.POINTER(C.c_int32)
        s = g = t = m = None
        if seeds is not None:
            arr = np.zeros(N, np.uint64)
            given = np.zeros(N, np.uint8)
            for k, v in enumerate(seeds):
                if v is not None:
                    arr[k] = int(v)
                    given[k] = 1
            self._seed_arr, self._given_arr = arr, given
            s, g = arr.ctypes.data_as(u64p), given.ctypes.data_as(u8p)
        if task_override is not None:
            self._task_arr = np.ascontiguousarray(task_override, np.int32)
            t = self._task_arr.ctypes.data_as(i32p)
        if env_mask is not None:
            self._mask_arr = np.ascontiguousarray(env_mask, np.uint8)
            m = self._mask_arr.ctypes.data_as(u8p)
        self._check(self.L.mmx_reset(self.ptr, s, g, t, m), "mmx_reset")

    def queue_init(self, tasks, seeds=None):
        """Device-side episode queue (mmx_queue_init): tasks[e] = obj << 4 | bin of episode e and,
        optionally, its seed (PCG64(SeedSequence(seed)) at its reset)."""
        t = np.ascontiguousarray(tasks, np.int32)
        s = None if seeds is None else np.ascontiguousarray([int(v) for v in seeds], np.uint64)
        if s is not None and len(s) != len(t):
            raise ValueError("seeds and tasks must have one entry per episode")
        self._check(self.L.mmx_queue_init(self.ptr, len(t), None if s is None else s.ctypes.data_as(C.POINTER(C.c_uint64)),
                                          t.ctypes.data_as(C.POINTER(C.c_int32))), "mmx_queue_init")

    def queue_advance(self, slot_ep_ptr: int | None = None, fin_ep_ptr: int | None = None):
        """Hand the next episodes to the free / finished slots and reset them (mmx_queue_advance;
        asynchronous).  The pointers: device int32 [N] outputs (slot -> episode after the call,
        episode that ended in the slot at this call; -1 = none)."""
        self._check(self.L.mmx_queue_advance(self.ptr, C.c_void_p(slot_ep_ptr) if slot_ep_ptr else None,
                                             C.c_void_p(fin_ep_ptr) if fin_ep_ptr else None), "mmx_queue_advance")

    def step(self, action_ptr: int, action_dim: int):
        self._check(self.L.mmx_step(self.ptr, C.c_void_p(action_ptr), action_dim), "mmx_step")

    def expert_plan(self, n_steps: int, action_ptr: int | None):
        self._check(self.L.mmx_expert_plan(self.ptr, n_steps, C.c_void_p(action_ptr) if action_ptr else None),
                    "mmx_expert_plan")

    def rollout_expert(self, n_env_steps: int):
        self._check(self.L.mmx_rollout_expert(self.ptr, n_env_steps), "mmx_rollout_expert")

    def kernel_timing(self, enable: bool):
        """Start (True: a new collection) / stop bracketing every rollout launch with HIP events."""
        self._check(self.L.mmx_kernel_timing(self.ptr, int(bool(enable))), "mmx_kernel_timing")

    def kernel_times(self) -> dict:
        """Summed launch durations (ms) and launch counts since kernel_timing(True); waits for them."""
        sm, rm, sn, rn = C.c_float(), C.c_float(), C.c_int32(), C.c_int32()
        self._check(self.L.mmx_kernel_times(self.ptr, C.byref(sm), C.byref(sn), C.byref(rm), C.byref(rn)),
                    "mmx_kernel_times")
        return {"step_ms": sm.value, "step_launches": sn.value, "render_ms": rm.value, "render_launches": rn.value}

    def png_encode(self, images, max_batch: int = 4096):
        """PNG files of RGB8 images [n, H, W, 3] (a CUDA uint8 tensor, any row-contiguous layout)
        encoded on the device (mmx_png_encode), in batches of `max_batch`.  Returns (packed uint8
        CUDA tensor, int64 offsets [n + 1] on the host): file i is packed[offsets[i]:offsets[i + 1]].
        One host synchronisation per batch (the packed size)."""
        import torch

        n, H, W, c = images.shape
        assert c == 3 and images.dtype == torch.uint8 and images.is_cuda
        if n == 0:
            return torch.empty(0, dtype=torch.uint8, device=images.device), np.zeros(1, np.int64)
        bound, scr = int(self.L.mmx_png_bound(W, H)), int(self.L.mmx_png_scratch(W, H))
        if bound < 0:
            raise ValueError(f"unsupported image size {W} x {H}")
        # the encoder runs on the sim's stream: the buffers, the size scan and the read-back are
        # ordered on that stream too (and the caller's stream waits for the result), whatever
        # stream the caller is on
        cur = torch.cuda.current_stream(images.device)
        sst = (torch.cuda.ExternalStream(self.cfg.stream, device=images.device) if self.cfg.stream
               else torch.cuda.default_stream(images.device))
        sst.wait_stream(cur)
        with torch.cuda.stream(sst):
            imgs = images.contiguous()
            images.record_stream(sst)
            packed, offs = self._png_encode_on_stream(imgs, n, H, W, bound, scr, max_batch)
        cur.wait_stream(sst)
        packed.record_stream(cur)
        return packed, offs

    def _png_encode_on_stream(self, imgs, n, H, W, bound, scr, max_batch):
        import torch

        dev = imgs.device
        parts, offs = [], [0]
        for b0 in range(0, n, max_batch):
            m = min(max_batch, n - b0)
            out = torch.empty(m * bound, dtype=torch.uint8, device=dev)
            scratch = torch.empty(m * scr, dtype=torch.uint8, device=dev)
            sizes = torch.empty(m, dtype=torch.int32, device=dev)
            self._check(self.L.mmx_png_encode(self.ptr, C.c_void_p(imgs[b0].data_ptr()), H * W * 3, m, W, H,
                                              C.c_void_p(out.data_ptr()), bound, C.c_void_p(sizes.data_ptr()),
                                              C.c_void_p(scratch.data_ptr())), "mmx_png_encode")
            ends = torch.cumsum(sizes.to(torch.int64), 0)
            starts = ends - sizes.to(torch.int64)
            total = int(ends[-1].item())
            packed = torch.empty(total, dtype=torch.uint8, device=dev)
            self._check(self.L.mmx_png_pack(self.ptr, C.c_void_p(out.data_ptr()), bound, C.c_void_p(sizes.data_ptr()),
                                            C.c_void_p(starts.data_ptr()), m, C.c_void_p(packed.data_ptr())),
                        "mmx_png_pack")
            parts.append(packed)
            offs.extend((ends.cpu().numpy() + offs[-1]).tolist())
        packed = torch.cat(parts) if len(parts) > 1 else parts[0]
        return packed, np.asarray(offs, np.int64)

    def png_encode_device(self, images):
        """PNG files of RGB8 images [n, H, W, 3] (CUDA uint8, rows contiguous) encoded and packed on
        the device with NO host synchronisation: returns (packed, ends), both CUDA tensors on the
        caller's stream: file i is packed[ends[i - 1]:ends[i]] (ends int64 [n]); packed has room for
        n * mmx_png_bound bytes, of which the first ends[-1] are files.  The dataset loop copies
        the sizes and the packed bytes to the host asynchronously."""
        import torch

        n, H, W, c = images.shape
        assert c == 3 and images.dtype == torch.uint8 and images.is_cuda and n > 0
        assert images.stride(1) == W * 3 and images.stride(2) == 3 and images.stride(3) == 1, "rows must be contiguous"
        bound, scr = int(self.L.mmx_png_bound(W, H)), int(self.L.mmx_png_scratch(W, H))
        if bound < 0:
            raise ValueError(f"unsupported image size {W} x {H}")
        cur = torch.cuda.current_stream(images.device)
        sst = (torch.cuda.ExternalStream(self.cfg.stream, device=images.device) if self.cfg.stream
               else torch.cuda.default_stream(images.device))
        sst.wait_stream(cur)
        dev = images.device
        with torch.cuda.stream(sst):
            images.record_stream(sst)
            out = torch.empty(n * bound, dtype=torch.uint8, device=dev)
            scratch = torch.empty(n * scr, dtype=torch.uint8, device=dev)
            sizes = torch.empty(n, dtype=torch.int32, device=dev)
            self._check(self.L.mmx_png_encode(self.ptr, C.c_void_p(images.data_ptr()), images.stride(0), n, W, H,
                                              C.c_void_p(out.data_ptr()), bound, C.c_void_p(sizes.data_ptr()),
                                              C.c_void_p(scratch.data_ptr())), "mmx_png_encode")
            ends = torch.cumsum(sizes.to(torch.int64), 0)
            starts = ends - sizes.to(torch.int64)
            packed = torch.empty(n * bound, dtype=torch.uint8, device=dev)
            self._check(self.L.mmx_png_pack(self.ptr, C.c_void_p(out.data_ptr()), bound, C.c_void_p(sizes.data_ptr()),
                                            C.c_void_p(starts.data_ptr()), n, C.c_void_p(packed.data_ptr())),
                        "mmx_png_pack")
        cur.wait_stream(sst)
        packed.record_stream(cur)
        ends.record_stream(cur)
        return packed, ends

    def image_stats(self, images):
        """Per-image channel statistics of RGB8 images [n, H, W, 3] (CUDA uint8, rows contiguous, any
        stride between images) on the device, asynchronously on the caller's stream: int64 [n, 4, 3]
        = (min, max, sum, sum of squares) x (R, G, B) over every pixel (mmx_image_stats)."""
        import torch

        n, H, W, c = images.shape
        assert c == 3 and images.dtype == torch.uint8 and images.is_cuda
        assert images.stride(1) == W * 3 and images.stride(2) == 3 and images.stride(3) == 1, "rows must be contiguous"
        out = torch.empty((n, 4, 3), dtype=torch.int64, device=images.device)
        if n == 0:
            return out
        cur = torch.cuda.current_stream(images.device)
        sst = (torch.cuda.ExternalStream(self.cfg.stream, device=images.device) if self.cfg.stream
               else torch.cuda.default_stream(images.device))
        sst.wait_stream(cur)
        with torch.cuda.stream(sst):
            images.record_stream(sst)
            out.record_stream(sst)
            self._check(self.L.mmx_image_stats(self.ptr, C.c_void_p(images.data_ptr()), images.stride(0), n, W, H,
                                               C.c_void_p(out.data_ptr())), "mmx_image_stats")
        cur.wait_stream(sst)
        return out

    @property
    def rollout_lanes(self) -> int:
        return int(self.L.mmx_rollout_lanes(self.ptr))

    @property
    def rollout_render_launches(self) -> int:
        """Render launches per rollout step with cameras (1: one over all envs after every lane's step)."""
        return int(self.L.mmx_rollout_render_launches(self.ptr))

    @property
    def step_rows(self) -> int:
        """Constraint rows the env-step kernel keeps in LDS (128: twelve envs per CU; 192: four, each
        with a helper wave; chosen at create from the batch size)."""
        return int(self.L.mmx_step_rows(self.ptr))

    @step_rows.setter
    def step_rows(self, rows: int):
        self._check(self.L.mmx_set_step_rows(self.ptr, int(rows)), "mmx_set_step_rows")

    @property
    def rollout_render_overlap(self) -> bool:
        """Camera rollouts render step k beside the env-step launch of step k + 1 (timing only)."""
        return bool(self.L.mmx_rollout_render_overlap(self.ptr))

    @property
    def step_order(self) -> bool:
        """Env-step launches dispatch their envs longest first by FSM phase (True, the default) or in
        index order; results are bit-identical either way."""
        return bool(self.L.mmx_step_order(self.ptr))

    @step_order.setter
    def step_order(self, on: bool):
        self._check(self.L.mmx_set_step_order(self.ptr, 1 if on else 0), "mmx_set_step_order")

    @property
    def rollout_steps_per_launch(self) -> int:
        return int(self.L.mmx_rollout_steps_per_launch(self.ptr))

    def rollout_launches(self, n_env_steps: int) -> int:
        """Launches per rollout lane that rollout_expert(n_env_steps) makes."""
        return int(self.L.mmx_rollout_launches(self.ptr, int(n_env_steps)))

    def physics_step(self, n: int = 1, with_ik: bool = False):
        self._check(self.L.mmx_physics_step(self.ptr, n, int(with_ik)), "mmx_physics_step")

    def forward(self):
        self._check(self.L.mmx_forward(self.ptr), "mmx_forward")

    def expert_physics(self, n_physics_steps: int):
        """n x (PickAndPlaceTask.update() ; mj_step), main.py:65-91."""
        self._check(self.L.mmx_expert_physics(self.ptr, n_physics_steps), "mmx_expert_physics")

    def eval_reward(self, obj_ptr: int, ee_ptr: int, ctrl7_ptr: int, pairs_ptr: int | None, max_pairs: int):
        """Reward-layer harness (device pointers): _compute_reward at the given positions / contacts."""
        self._check(self.L.mmx_eval_reward(self.ptr, C.c_void_p(obj_ptr), C.c_void_p(ee_ptr), C.c_void_p(ctrl7_ptr),
                                           C.c_void_p(pairs_ptr) if pairs_ptr else None, max_pairs),
                    "mmx_eval_reward")

    def synchronize(self):
        self._check(self.L.mmx_synchronize(self.ptr), "mmx_synchronize")

    def get_state(self):
        N = self.num_envs
        qpos, qvel = np.zeros((N, NQ), np.float32), np.zeros((N, NV), np.float32)
        ctrl, ws = np.zeros((N, NU), np.float32), np.zeros((N, NV), np.float32)
        self._check(self.L.mmx_get_state(self.ptr, _fptr(qpos), _fptr(qvel), _fptr(ctrl), _fptr(ws)), "mmx_get_state")
        return qpos, qvel, ctrl, ws

    def set_state(self, qpos=None, qvel=None, ctrl=None, qacc_ws=None):
        arrs = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (qpos, qvel, ctrl, qacc_ws)]
        self._check(self.L.mmx_set_state(self.ptr, *[_fptr(a) for a in arrs]), "mmx_set_state")

    # ---- zero-copy torch views of sim-owned buffers (env-major [N][F])
    def image_views(self):
        """(rgb [N, 2, S, S, 3] uint8, seg [N, 2, S, S] uint8) or None when image_size == 0."""
        import torch

        S = int(self.cfg.image_size)
        if S <= 0 or not self.buffers.images:
            return None
        dev = f"cuda:{self.cfg.device}"
        rgb = torch.as_tensor(_DevArray(self.buffers.images, (self.num_envs, 2, S, S, 3), "|u1", self), device=dev)
        seg = torch.as_tensor(_DevArray(self.buffers.seg, (self.num_envs, 2, S, S), "|u1", self), device=dev)
        return rgb, seg

    def view(self, name: str, nfield: int, dtype: str = "<f4"):
        import torch

        ptr = getattr(self.buffers, name)
        shape = (self.num_envs, nfield) if nfield > 1 else (self.num_envs,)
        return torch.as_tensor(_DevArray(ptr, shape, dtype, self), device=f"cuda:{self.cfg.device}")
