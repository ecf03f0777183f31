"""Batched expert-demonstration dataset emission.

Mirrors `scripts/generate_dataset.py` of the reference (run_episode :83-198, main :201-333,
feature schema `mujoco_manip/features.py:10-106`), with the episodes run side by side on the
MI355X instead of one after another:

* every slot of a `PickPlaceVecEnv` runs one episode: `plan(ACTION_REPEAT)` on device, the frame
  is built from the PRE-step observation plus the FSM's commanded target in four SE(3)
  encodings, then `step(abs_pos action)`; the staged reward components of the step land in
  `next.reward` (reference :140-196);
* an episode ends when its FSM reaches DONE (terminated / truncated are ignored, as in the
  reference loop); the slot is then re-reset with the next episode's seed and task
  (episode e: task `task_list[e % len(task_list)]`, seed `SeedSequence(seed).spawn(E)[e]`
  when `randomize_objects`, reference :267-277);
* each step's frames are gathered on device and streamed to pinned host memory (device memory
  O(envs)); finished episodes go to a streaming writer in the LeRobot v3.0 on-disk layout
  (parquet data files, `meta/info.json`, `meta/tasks.parquet`, `meta/episodes/...parquet`,
  `meta/stats.json`) plus the reference's `metadata.json` (generation config + `episode_seeds`,
  :306-319), so host memory holds only the episodes in flight.

Camera images (observation.images.overhead / .wrist, features.py:11-20, 224 x 224 RGB) come from
the batched HIP renderer (mmx_render.hip): the PRE-step images of every active
slot are gathered on device each step, encoded to PNG files on the device (mmx_png.hip) and stored the way LeRobot stores
`dtype: image` features with use_videos=False (generate_dataset.py:250-260): a parquet struct
column {bytes: PNG, path} per frame, per-channel image statistics in meta/stats.json.
LeRobot itself is not importable here, so the on-disk layout follows LeRobot v3.0's documented
format without a round-trip check against the library ("format unpinned"); the frame VALUES are
pinned against the oracle running the reference loop (tests/test_dataset.py).
"""
from __future__ import annotations

import argparse
import functools
import json
import os
import time
from dataclasses import dataclass, field

import numpy as np

from .constants import ACTION_REPEAT, BINS, CONTROL_FPS, IMAGE_SIZE, OBJECTS, OBS_SLICES, TASK_SETS

# features.py:10-106 (IMAGE_SIZE = 224)
FEATURES = {
    "observation.images.overhead": {"dtype": "image", "shape": (224, 224, 3), "names": ["height", "width", "channels"]},
    "observation.images.wrist": {"dtype": "image", "shape": (224, 224, 3), "names": ["height", "width", "channels"]},
    "observation.state": {"dtype": "float32", "shape": (11,), "names": None},
    "observation.state.ee.pos_quat_g": {"dtype": "float32", "shape": (8,), "names": None},
    "observation.state.ee.pos_rot6d_g": {"dtype": "float32", "shape": (10,), "names": None},
    "observation.state.ee.pos_quat_g_rel": {"dtype": "float32", "shape": (8,), "names": None},
    "observation.state.ee.pos_rot6d_g_rel": {"dtype": "float32", "shape": (10,), "names": None},
    "action.ee.pos_quat_g": {"dtype": "float32", "shape": (8,), "names": None},
    "action.ee.pos_rot6d_g": {"dtype": "float32", "shape": (10,), "names": None},
    "action.ee.pos_quat_g_rel": {"dtype": "float32", "shape": (8,), "names": None},
    "action.ee.pos_rot6d_g_rel": {"dtype": "float32", "shape": (10,), "names": None},
    "observation.target_bin_onehot": {"dtype": "float32", "shape": (3,), "names": None},
    "observation.target_obj_onehot": {"dtype": "float32", "shape": (3,), "names": None},
    "observation.keypoints_overhead": {"dtype": "float32", "shape": (14,), "names": None},
    "observation.keypoints_wrist": {"dtype": "float32", "shape": (14,), "names": None},
    "observation.target_obj_keypoints_overhead": {"dtype": "float32", "shape": (2,), "names": None},
    "observation.target_bin_keypoints_overhead": {"dtype": "float32", "shape": (2,), "names": None},
    "observation.phase_description": {"dtype": "string", "shape": (1,), "names": None},
    "next.reward": {"dtype": "float32", "shape": (6,), "names": None},
}

# generate_dataset.py:26-38 (+ the flattened keypoints :158-168)
OBS_TO_FEATURE = {
    "state": "observation.state",
    "state.ee.pos_quat_g": "observation.state.ee.pos_quat_g",
    "state.ee.pos_rot6d_g": "observation.state.ee.pos_rot6d_g",
    "state.ee.pos_quat_g_rel": "observation.state.ee.pos_quat_g_rel",
    "state.ee.pos_rot6d_g_rel": "observation.state.ee.pos_rot6d_g_rel",
    "target_bin_onehot": "observation.target_bin_onehot",
    "target_obj_onehot": "observation.target_obj_onehot",
    "target_obj_keypoints_overhead": "observation.target_obj_keypoints_overhead",
    "target_bin_keypoints_overhead": "observation.target_bin_keypoints_overhead",
    "keypoints_overhead": "observation.keypoints_overhead",
    "keypoints_wrist": "observation.keypoints_wrist",
}
ACTION_KEYS = ("action.ee.pos_quat_g", "action.ee.pos_rot6d_g", "action.ee.pos_quat_g_rel", "action.ee.pos_rot6d_g_rel")
IMAGE_KEYS = ("observation.images.overhead", "observation.images.wrist")

# pick_and_place.py:12-49 (State order = device FSM codes 0..10) and :128-149
_STATE_PHASE = ["idle", "approaching", "grasping", "grasping", "lifting", "transporting", "transporting",
                "placing", "placing", "retreating", "done"]
FSM_DONE = 10

# controller.py TARGET_ORI: the FSM's commanded hand orientation
TARGET_ORI = np.array([[0.0, 1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, -1.0]])


def make_task_string(obj_name: str, bin_name: str) -> str:
    """generate_dataset.py:41-54."""
    return f"Pick {obj_name.replace('obj_', '')} object and place in {bin_name.replace('bin_', '')} bin"


_PHASE_LUT = {}


def _phase_lut(obj_name: str, bin_name: str) -> list:
    """phase_description of every device FSM code for one task (cached)."""
    key = (obj_name, bin_name)
    if key not in _PHASE_LUT:
        _PHASE_LUT[key] = [phase_description(k, obj_name, bin_name) for k in range(len(_STATE_PHASE))]
    return _PHASE_LUT[key]


@functools.lru_cache(maxsize=None)
def phase_description(state: int, obj_name: str, bin_name: str) -> str:
    """PickAndPlaceTask.phase_description (pick_and_place.py:128-149) for a device FSM code."""
    phase = _STATE_PHASE[int(state)]
    if phase in ("idle", "done"):
        return "idle"
    if phase == "retreating":
        return "retreating to neutral position"
    o, b = obj_name.replace("obj_", ""), bin_name.replace("bin_", "")
    return {"approaching": f"approaching the {o} cube", "grasping": f"grasping the {o} cube",
            "lifting": f"lifting the {o} cube", "transporting": f"transporting the {o} cube to the {b} bin",
            "placing": f"placing the {o} cube in the {b} bin"}[phase]


# ----------------------------------------------------------------------------- action encodings
def _quat_xyzw_t(R):
    """rotmat_to_quat_xyzw (pose_utils.py:48-82) on a batch [n, 3, 3], branch for branch."""
    import torch

    r00, r11, r22 = R[:, 0, 0], R[:, 1, 1], R[:, 2, 2]
    tr = r00 + r11 + r22
    one = torch.ones_like(tr)

    def safe_s(v):
        return 2.0 * torch.sqrt(torch.clamp(v, min=0.0) + 0.0) + (v <= 0).to(v.dtype) * 1.0  # never 0 in unused lanes

    s0 = safe_s(tr + 1.0)
    q0 = torch.stack([(R[:, 2, 1] - R[:, 1, 2]) / s0, (R[:, 0, 2] - R[:, 2, 0]) / s0, (R[:, 1, 0] - R[:, 0, 1]) / s0,
                      0.25 * s0], 1)
    s1 = safe_s(one + r00 - r11 - r22)
    q1 = torch.stack([0.25 * s1, (R[:, 0, 1] + R[:, 1, 0]) / s1, (R[:, 0, 2] + R[:, 2, 0]) / s1,
                      (R[:, 2, 1] - R[:, 1, 2]) / s1], 1)
    s2 = safe_s(one + r11 - r00 - r22)
    q2 = torch.stack([(R[:, 0, 1] + R[:, 1, 0]) / s2, 0.25 * s2, (R[:, 1, 2] + R[:, 2, 1]) / s2,
                      (R[:, 0, 2] - R[:, 2, 0]) / s2], 1)
    s3 = safe_s(one + r22 - r00 - r11)
    q3 = torch.stack([(R[:, 0, 2] + R[:, 2, 0]) / s3, (R[:, 1, 2] + R[:, 2, 1]) / s3, 0.25 * s3,
                      (R[:, 1, 0] - R[:, 0, 1]) / s3], 1)
    b0 = (tr > 0)[:, None]
    b1 = ((r00 > r11) & (r00 > r22))[:, None]
    b2 = (r11 > r22)[:, None]
    return torch.where(b0, q0, torch.where(b1, q1, torch.where(b2, q2, q3)))


_TARGET_ORI_DEV = {}


def encode_actions(target, gripper, T_init):
    """get_actions (generate_dataset.py:57-80) batched on device.

    target [n, 3], gripper [n], T_init [n, 4, 4] -> the four float32 encodings of the commanded
    SE(3) (absolute and relative to T_init), computed in float64 like the reference's numpy.
    """
    import torch

    dev = target.device
    n = target.shape[0]
    t = target.to(torch.float64)
    g = gripper.to(torch.float64)[:, None]
    Ti = T_init.to(torch.float64)
    key = str(dev)
    if key not in _TARGET_ORI_DEV:  # (a host -> device copy waits for the device: once per device)
        _TARGET_ORI_DEV[key] = torch.as_tensor(TARGET_ORI, dtype=torch.float64, device=dev)
    Rt = _TARGET_ORI_DEV[key].expand(n, 3, 3)
    # inv(T_init) @ T_target for a rigid transform: R' = Ri^T Rt, p' = Ri^T (t - pi)
    RiT = Ti[:, :3, :3].transpose(1, 2)
    Rr = RiT @ Rt
    pr = (RiT @ (t - Ti[:, :3, 3])[:, :, None])[:, :, 0]
    qa = _quat_xyzw_t(Rt)
    qr = _quat_xyzw_t(Rr)
    out = {
        "action.ee.pos_quat_g": torch.cat([t, qa, g], 1),
        "action.ee.pos_rot6d_g": torch.cat([t, Rt[:, :2, :].reshape(n, 6), g], 1),
        "action.ee.pos_quat_g_rel": torch.cat([pr, qr, g], 1),
        "action.ee.pos_rot6d_g_rel": torch.cat([pr, Rr[:, :2, :].reshape(n, 6), g], 1),
    }
    return {k: v.to(torch.float32) for k, v in out.items()}


# ----------------------------------------------------------------------------- batched collection
@dataclass
class Episode:
    index: int
    obj: str
    bin: str
    seed: int | None
    frames: dict = field(default_factory=dict)  # feature -> np.ndarray [T, ...] (strings, PNG bytes: list)
    length: int = 0
    image_stats: dict = field(default_factory=dict)  # image feature -> stats of a raw frame sample


class PngFrames:
    """An episode's PNG files back to back in one uint8 buffer (file i = data[offsets[i]:offsets[i+1]]).
    Reads as a sequence of `bytes` (len, indexing, iteration) wherever a list of PNG files is expected;
    the LeRobot writer hands the buffer to arrow as is (no Python object per frame)."""
    __slots__ = ("data", "offsets")

    def __init__(self, data: np.ndarray, offsets: np.ndarray):
        self.data, self.offsets = data, offsets

    def __len__(self):
        return len(self.offsets) - 1

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        return self.data[int(self.offsets[i]):int(self.offsets[i + 1])].tobytes()

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    @property
    def nbytes(self) -> int:
        return int(self.offsets[-1])


def _png_nbytes(frames) -> int:
    return frames.nbytes if isinstance(frames, PngFrames) else sum(map(len, frames))


def resolve_tasks(task=None, tasks="all"):
    """generate_dataset.py:205-216 (same ValueErrors)."""
    if task is not None:
        pair = tuple(task)
        if len(pair) != 2:
            raise ValueError(f"task must be [obj, bin], got {pair}")
        return [pair]
    if tasks in TASK_SETS:
        return TASK_SETS[tasks]
    raise ValueError(f"Unknown task set '{tasks}'. Choose from: {list(TASK_SETS.keys())}")


def resolve_features(features=None, reward_type="staged"):
    """generate_dataset.py:218-230: subset selection, unknown keys -> ValueError,
    next.reward only with the staged reward."""
    feats = dict(FEATURES)
    if features is not None:
        requested = list(features)
        unknown = [k for k in requested if k not in FEATURES]
        if unknown:
            raise ValueError(f"Unknown feature keys: {unknown}. Valid keys: {list(FEATURES.keys())}")
        feats = {k: FEATURES[k] for k in requested}
    if reward_type != "staged":
        feats.pop("next.reward", None)
    return feats


def png_encode(img: np.ndarray) -> bytes:
    """uint8 [H, W, 3] -> PNG bytes (what LeRobot embeds for an `image` feature)."""
    import io

    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(img)).save(buf, format="PNG", compress_level=1)
    return buf.getvalue()


def png_decode(data: bytes) -> np.ndarray:
    import io

    from PIL import Image

    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


def episode_seeds(seed: int, num_episodes: int) -> list[int]:
    """generate_dataset.py:263-268: SeedSequence(seed).spawn(E)[e].generate_state(1)[0]."""
    from . import _lib

    return [_lib.episode_seed(seed, e) for e in range(num_episodes)]


def rank_episodes(num_episodes: int, rank: int = 0, world_size: int = 1) -> list[int]:
    """Global episode indices a rank generates when the dataset is sharded over `world_size`
    processes (one per GPU): e = rank (mod world_size).  An episode keeps its global
    seed and task (generate_dataset.py:263-277), so the frames do not depend on the rank count."""
    if not (0 <= rank < world_size):
        raise ValueError(f"bad shard: rank {rank} of {world_size}")
    return list(range(rank, int(num_episodes), world_size))


def shard_dir(path: str, rank: int, world_size: int) -> str:
    """Where rank `rank` of `world_size` writes its LeRobot shard inside the dataset directory."""
    return os.path.join(path, f"shard-{rank:03d}-of-{world_size:03d}")


class _PinnedRing:
    """Pinned host staging for the per-step frame copies: device tensors are copied with
    non_blocking=True on a side stream that waits for the producing stream, an event marks
    completion, and at most `depth` copies are in flight (older ones are waited first)."""

    def __init__(self, dev, depth=4):
        import torch

        self.torch = torch
        self.stream = torch.cuda.Stream(device=dev)
        self.depth = depth
        self.pending = []  # (event, host dict, payload)

    def push(self, tensors: dict, payload):
        torch = self.torch
        self.stream.wait_stream(torch.cuda.current_stream(self.stream.device))
        host = {}
        with torch.cuda.stream(self.stream):
            for k, v in tensors.items():
                h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                h.copy_(v, non_blocking=True)
                v.record_stream(self.stream)
                host[k] = h
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.pending.append((ev, host, payload))

    def ready(self, block_over_depth=True):
        """Completed copies, oldest first (waits for the oldest ones beyond `depth`)."""
        out = []
        while self.pending and (self.pending[0][0].query() or (block_over_depth and len(self.pending) > self.depth)):
            ev, host, payload = self.pending.pop(0)
            ev.synchronize()
            out.append(({k: v.numpy() for k, v in host.items()}, payload))
        return out

    def drain(self):
        out = []
        while self.pending:
            ev, host, payload = self.pending.pop(0)
            ev.synchronize()
            out.append(({k: v.numpy() for k, v in host.items()}, payload))
        return out


def _raw_image_stats(frames_u8: list) -> dict:
    """Per-channel statistics of an image feature from raw uint8 frames [H, W, 3] (a sample),
    pixels scaled to [0, 1], shaped (3, 1, 1) as LeRobot keeps them; also the raw sums so episode
    statistics can be merged into the dataset's."""
    x = np.stack(frames_u8).reshape(-1, 3).astype(np.float64) / 255.0
    shape = lambda v: [[[float(a)]] for a in v]  # noqa: E731
    return {"min": shape(x.min(0)), "max": shape(x.max(0)), "mean": shape(x.mean(0)), "std": shape(x.std(0)),
            "_sum": x.sum(0).tolist(), "_sumsq": (x * x).sum(0).tolist(), "_n": int(len(x))}


# [min, max, sum, sum of squares] of the uint8 values -> the same of the values scaled to [0, 1]
_STAT_SCALE = (1.0 / 255.0, 1.0 / 255.0, 1.0 / 255.0, 1.0 / (255.0 * 255.0))
_STAT_SCALE_DEV = {}


def _frame_image_stats_device(sim, imgs):
    """Per-frame channel statistics of uint8 images [k, H, W, 3] by the HIP kernel mmx_image_stats
    (one pass over the frames, exact integers) -> float64 [k, 4, 3], the values of
    _frame_image_stats bit for bit (the same integers scaled by the same constants)."""
    import torch

    st = sim.image_stats(imgs).to(torch.float64)
    scale = _STAT_SCALE_DEV.get(st.device)
    if scale is None:  # cached per device: a host-to-device copy per step would wait for the queue
        scale = _STAT_SCALE_DEV[st.device] = torch.tensor(_STAT_SCALE, dtype=torch.float64, device=st.device)[None, :, None]
    return st * scale


def _frame_image_stats(imgs, chunk=None):
    """Torch form of _frame_image_stats_device (the reference for its test; the dataset loop uses
    the kernel): min, max, sum and sum of squares of the pixel values scaled to [0, 1] -> float64
    [k, 4, 3].  Min / max on the uint8 values, sums exact in integers (int32 values, int64 sums) and
    scaled at the end, in chunks of `chunk` images (default: 256 MB of int32 values)."""
    import torch

    k = imgs.shape[0]
    if chunk is None:
        chunk = max(1, (1 << 26) // max(1, imgs[0].numel()))
    x = imgs.reshape(k, -1, 3)
    out = torch.empty((k, 4, 3), dtype=torch.float64, device=imgs.device)
    out[:, 0] = x.amin(1).to(torch.float64) * (1.0 / 255.0)
    out[:, 1] = x.amax(1).to(torch.float64) * (1.0 / 255.0)
    for a in range(0, k, chunk):
        xi = x[a:a + chunk].to(torch.int32)
        out[a:a + chunk, 2] = xi.sum(1, dtype=torch.int64).to(torch.float64) * (1.0 / 255.0)
        out[a:a + chunk, 3] = (xi * xi).sum(1, dtype=torch.int64).to(torch.float64) * (1.0 / (255.0 * 255.0))
    return out


def _merge_image_stats(fs: np.ndarray, npx: int) -> dict:
    """Episode image statistics from its frames' [T, 4, 3] statistics (same layout as
    _raw_image_stats, over every pixel of every frame)."""
    mn, mx, sm, sq = fs[:, 0].min(0), fs[:, 1].max(0), fs[:, 2].sum(0), fs[:, 3].sum(0)
    n = npx * len(fs)
    mean = sm / n
    std = np.sqrt(np.maximum(sq / n - mean * mean, 0.0))
    v = np.stack([mn, mx, mean, std]).tolist()  # one conversion, then the (3, 1, 1) nesting
    return {"min": [[[a]] for a in v[0]], "max": [[[a]] for a in v[1]], "mean": [[[a]] for a in v[2]],
            "std": [[[a]] for a in v[3]], "_sum": sm.tolist(), "_sumsq": sq.tolist(), "_n": int(n)}


def collect_episodes(num_episodes: int, task_list, feature_keys, *, reward_type="staged", randomize_objects=False,
                     seed=0, spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45), num_envs=1024, device=0,
                     max_gym_steps=5000, on_step=None, sink=None, image_size=IMAGE_SIZE, episode_ids=None):
    """Run `num_episodes` reference run_episode loops (generate_dataset.py:83-198) side by side,
    or, with `episode_ids`, only those episodes of the `num_episodes`-episode job (a rank's shard,
    rank_episodes): each keeps its global index, seed and task.

    Streaming with no host synchronisation per step: the slot -> episode assignment runs on the
    device (mmx_queue_advance), each step's frames of every slot (plus the assignment) are copied
    to pinned host memory on a side stream, and the host splits them into their episodes a few
    steps later, as the copies complete.  Camera frames are
    encoded to PNG files on the device (mmx_png_encode; LeRobot embeds image features as PNG,
    generate_dataset.py:250-260) with their per-channel statistics, so only the compressed files
    cross PCIe and the host does no image work.  Device memory is O(envs): no frame stays on the
    device after its copy; the packed PNG buffers of the steps in flight (ring depth 4 + 1, room for
    n bounds each) dominate it: 13 GB at 128^2 and 32 GB at 224^2 for 8192 envs.  A finished episode (FSM DONE) is handed to `sink(episode)` in
    episode-index order, so the host holds only the episodes in flight; without a sink the episodes
    are returned as a list.  on_step(slots, episode_ids, env), when given, sees the env before each
    batched step (a diagnostic hook: it costs a host synchronisation per step).  Returns (episodes or
    None, seeds).
    """
    import torch

    from .vec_env import PickPlaceVecEnv

    seeds = episode_seeds(seed, int(num_episodes)) if randomize_objects else None
    ids = list(range(int(num_episodes))) if episode_ids is None else [int(g) for g in episode_ids]
    if any(not 0 <= g < int(num_episodes) for g in ids):
        raise ValueError(f"episode ids must lie in [0, {num_episodes})")
    E = len(ids)
    if E == 0:
        return ([] if sink is None else None), seeds
    N = max(1, min(int(num_envs), E))
    use_images = bool(set(feature_keys) & set(IMAGE_KEYS))
    env = PickPlaceVecEnv(N, tasks=[tuple(t) for t in task_list], action_mode="abs_pos", reward_type=reward_type,
                          randomize_objects=randomize_objects, spawn_x_range=tuple(spawn_x_range),
                          spawn_y_range=tuple(spawn_y_range), autoreset=False, device=device,
                          image_size=image_size if use_images else 0)
    dev = env.device
    need_actions = bool(set(feature_keys) & set(ACTION_KEYS))
    need_reward = "next.reward" in feature_keys and reward_type == "staged"
    obs_feats = [(k, f) for k, f in OBS_TO_FEATURE.items() if f in feature_keys]
    img_feats = [(cam, f) for cam, f in enumerate(IMAGE_KEYS) if f in feature_keys]
    npx = image_size * image_size

    # local position e <-> global episode ids[e]: slots and rows are indexed locally.  The slot ->
    # episode assignment runs on the device (mmx_queue_advance): a slot whose episode's FSM reached
    # DONE takes the next episode and is reset with its seed and task, in ascending slot order, with
    # no host synchronisation; the host learns the assignment from the per-step copies.
    eps = [Episode(g, *task_list[g % len(task_list)], seeds[g] if seeds else None) for g in ids]
    env.sim.queue_init([(OBJECTS.index(ep.obj) << 4) | BINS.index(ep.bin) for ep in eps],
                       [ep.seed for ep in eps] if seeds else None)
    out_eps = [] if sink is None else None
    emitted = 0
    done_eps = {}  # finished, awaiting in-order emission: episode -> True
    ep_slot = np.full(E, -1, np.int64)  # the slot an episode ran in

    # Host-side per-slot frame buffers: a slot's running episode gets one row per step, written for
    # all of the step's slots at once (one fancy-indexed store per feature); an episode's rows are
    # copied out when it finishes, before its slot's next episode writes there.  PNG files are cut
    # out of each step's packed buffer into the slot's list.
    bufs = {}  # host key -> [N, cap, ...]
    cap = [64]
    tpos = np.zeros(N, np.int64)  # rows of the slot's current episode so far
    buf_ep = np.full(N, -1, np.int64)  # the episode whose rows the slot holds
    # PNG files: every slot's running episode has one growing uint8 buffer per camera; each step's
    # files are appended to their slots' buffers straight out of the pinned copy of the step by one
    # C call per camera (mmx_copy_ranges: no Python object per frame, the GIL released for the copy),
    # and a finished episode hands its buffer over as PngFrames (no further copy)
    png_buf = {f: [None] * N for _, f in img_feats}  # camera -> slot -> buffer
    png_addr = {f: np.zeros(N, np.uint64) for _, f in img_feats}  # the buffers' addresses
    png_fill = {f: np.zeros(N, np.int64) for _, f in img_feats}  # bytes used
    png_cap = {f: np.zeros(N, np.int64) for _, f in img_feats}  # bytes allocated
    # first buffer size of an episode: 1.25 x the largest finished episode so far; before any has
    # finished, 160 frames of the first step's mean file size (grown by doubling when exceeded)
    png_guess = {f: 0 for _, f in img_feats}
    copy_ranges = env.sim.L.mmx_copy_ranges

    def png_alloc(f, s, cap, keep=0):
        buf = np.empty(int(cap), np.uint8)
        if keep:
            buf[:keep] = png_buf[f][s][:keep]
        png_buf[f][s] = buf
        png_addr[f][s] = buf.ctypes.data
        png_cap[f][s] = len(buf)

    def absorb(host, slots, ep_ids, png):
        if len(ep_ids) == 0:
            return
        ep_slot[ep_ids] = slots
        new = buf_ep[slots] != ep_ids
        if new.any():
            ns = slots[new]
            tpos[ns] = 0
            buf_ep[ns] = ep_ids[new]
            for f in png_buf:
                png_fill[f][ns] = 0
                for s in ns.tolist():
                    png_alloc(f, s, png_guess[f] or (1 << 16))
        for f, data in png.items():  # append the step's files to their episodes' buffers
            ends = host[f + "/ends"]
            if png_guess[f] == 0:
                png_guess[f] = 160 * max(1, int(ends[-1]) // max(1, len(ends)))
                for s in np.nonzero(png_cap[f][slots] < png_guess[f])[0].tolist():
                    if png_fill[f][slots[s]] == 0:
                        png_alloc(f, int(slots[s]), png_guess[f])
            starts = np.zeros_like(ends)
            starts[1:] = ends[:-1]
            lens = (ends - starts)[slots].astype(np.int64)
            need = png_fill[f][slots] + lens
            for k in np.nonzero(need > png_cap[f][slots])[0].tolist():  # (rare) grow
                s = int(slots[k])
                png_alloc(f, s, max(2 * int(need[k]), png_guess[f]), keep=int(png_fill[f][s]))
            src = (data.ctypes.data + starts[slots].astype(np.uint64)).astype(np.uint64)
            dst = png_addr[f][slots] + png_fill[f][slots].astype(np.uint64)
            if copy_ranges(len(slots), src.ctypes.data, dst.ctypes.data, lens.ctypes.data) != int(lens.sum()):
                raise RuntimeError("mmx_copy_ranges failed")
            png_fill[f][slots] = need
            host[f + "/plen"] = (ends - starts).astype(np.int64)
        t = tpos[slots]
        if int(t.max()) >= cap[0]:
            cap[0] *= 2
            for k, v in bufs.items():
                g = np.empty((N, cap[0]) + v.shape[2:], v.dtype)
                g[:, :v.shape[1]] = v
                bufs[k] = g
        flat = slots * cap[0] + t  # row (slot, t) of a [N, cap, ...] buffer as one flat index: numpy's
        for k, v in host.items():  # two-array fancy index is ~8x slower for the same scatter
            if k.endswith("/png") or k.endswith("/ends") or k.startswith("_q"):
                continue
            if k not in bufs:
                bufs[k] = np.empty((N, cap[0]) + v.shape[1:], v.dtype)
            b = bufs[k]
            b.reshape((N * cap[0],) + b.shape[2:])[flat] = v[slots]
        tpos[slots] = t + 1

    def finish(e):
        """Copy episode e's rows out of its slot's buffers (it has ended: no row of it is still in
        flight, and the slot's next episode has not written yet)."""
        ep = eps[e]
        s = int(ep_slot[e])
        L = int(tpos[s]) if s >= 0 and buf_ep[s] == e else 0
        ep.length = L
        ep.image_stats = {}
        for k in feature_keys:
            if k in IMAGE_KEYS:
                if L:
                    offs = np.zeros(L + 1, np.int64)
                    np.cumsum(bufs[k + "/plen"][s, :L], out=offs[1:])
                    if offs[-1] != png_fill[k][s]:
                        raise RuntimeError(f"episode {ep.index}: PNG bytes {png_fill[k][s]} != frames {offs[-1]}")
                    ep.frames[k] = PngFrames(png_buf[k][s][:int(offs[-1])], offs)
                    png_buf[k][s] = None
                    png_guess[k] = max(png_guess[k], int(offs[-1]) * 5 // 4)
                else:
                    ep.frames[k] = []
                ep.image_stats[k] = _merge_image_stats(bufs[k + "/stats"][s, :L], npx) if L else None
            elif k == "observation.phase_description":
                lut = _phase_lut(ep.obj, ep.bin)
                ep.frames[k] = [lut[v] for v in bufs["_fsm"][s, :L].tolist()] if L else []
            elif L and k in bufs:
                ep.frames[k] = bufs[k][s, :L].astype(np.float32)
        if L:
            buf_ep[s] = -1
        done_eps[e] = True

    def emit_ready():
        nonlocal emitted
        while emitted < E and emitted in done_eps:
            e = emitted
            del done_eps[e]
            if sink is not None:
                sink(eps[e])
                eps[e] = None  # the sink owns it now: host memory stays bounded by the episodes in flight
            else:
                out_eps.append(eps[e])
            emitted += 1

    import torch

    ring = _PinnedRing(dev)
    slot_dev = torch.empty(N, dtype=torch.int32, device=dev)
    fin_dev = torch.empty(N, dtype=torch.int32, device=dev)
    png_est = {}  # camera feature -> bytes copied per step: 1.25 x the largest packed size seen + 1 MB
    png_max = {}
    state = {"over": False, "started": False}

    def process(items):
        for host, payload in items:
            fin = host["_q_fin"]
            for e in fin[fin >= 0].tolist():  # ended before this step: every row of theirs is absorbed
                finish(e)
            slot = host["_q_slot"]
            act = np.nonzero(slot >= 0)[0]
            if len(act) == 0:
                state["over"] = state["over"] or state["started"]
                continue
            state["started"] = True
            png = {}
            for f, packed in payload.items():  # the step's packed PNG files (copied: a prefix)
                total = int(host[f + "/ends"][-1])
                data = host[f + "/png"]
                if total > len(data):  # more than the estimate: fetch the rest (rare)
                    data = np.concatenate([data, packed[len(data):total].cpu().numpy()])
                png_max[f] = max(png_max.get(f, 0), total)
                png_est[f] = (png_max[f] * 5) // 4 + (1 << 20)
                png[f] = data  # (absorb appends each slot's file to its episode's buffer)
            absorb(host, act, slot[act].astype(np.int64), png)

    step_no = 0
    while not state["over"]:
        # the host learns that the last episode ended from copies up to ring.depth steps behind the
        # device: allow that lag past the limit before calling the run unfinished
        if step_no >= max_gym_steps + ring.depth:
            process(ring.drain())
            if state["over"]:
                break
            still = [int(ids[e]) for e in range(E) if e >= emitted and e not in done_eps]
            raise RuntimeError(f"episodes did not finish within {max_gym_steps} gym steps: {len(still)} still "
                               f"open, e.g. {still[:16]}")
        env.sim.queue_advance(slot_dev.data_ptr(), fin_dev.data_ptr())  # resets the slots it assigns
        action = env.expert_plan(ACTION_REPEAT)  # fsm.plan(16) -> (target, gripper) for every slot
        frame = {"_q_slot": slot_dev.clone(), "_q_fin": fin_dev.clone()}
        obs_pre = env._obs.clone()  # PRE-step obs (from the reset or the previous step)
        for k, f in obs_feats:
            a, b, _ = OBS_SLICES[k]
            frame[f] = obs_pre[:, a:b]
        payload = {}
        for cam, f in img_feats:  # PRE-step images (rendered after the reset / previous step)
            imgs = env._images[:, cam]
            packed, ends = env.sim.png_encode_device(imgs)
            if f not in png_est:
                png_est[f] = packed.numel() // 4
            frame[f + "/png"] = packed[:min(png_est[f], packed.numel())]
            frame[f + "/ends"] = ends
            frame[f + "/stats"] = _frame_image_stats_device(env.sim, imgs)
            payload[f] = packed
        if need_actions:
            enc = encode_actions(action[:, :3], action[:, 3], env.initial_ee_se3)
            for k in ACTION_KEYS:
                if k in feature_keys:
                    frame[k] = enc[k]
        frame["_fsm"] = env._epi[:, 4].clone()
        if on_step is not None:  # diagnostic hook: reads the assignment back (a host sync per step)
            sl = slot_dev.cpu().numpy()
            act_slots = np.nonzero(sl >= 0)[0]
            on_step(act_slots, np.asarray(ids, np.int64)[sl[act_slots]], env)
        env.sim.step(action.data_ptr(), action.shape[1])
        if need_reward:
            frame["next.reward"] = env._rc.clone()
        ring.push(frame, payload)
        process(ring.ready())
        emit_ready()
        step_no += 1
    process(ring.drain())
    for e in range(E):  # episodes still open when the loop ended (none, unless max_gym_steps cut it)
        if e >= emitted and e not in done_eps:
            finish(e)
    emit_ready()
    torch.cuda.synchronize(dev)
    env.close()
    return out_eps, seeds


# ----------------------------------------------------------------------------- LeRobot v3.0 writer
class LeRobotWriter:
    """Streaming LeRobot v3.0 writer (use_videos=False: image features embedded as parquet structs
    {bytes: PNG, path}).  Episodes are added one at a time in episode-index order and appended to
    the open data file (pyarrow ParquetWriter), which rolls over at `data_files_size_in_mb`;
    statistics accumulate as running sums, so memory does not grow with the dataset.

    data/chunk-XXX/file-YYY.parquet  frames of consecutive episodes (features + timestamp,
                                     frame_index, episode_index, index, task_index)
    meta/info.json, meta/tasks.parquet, meta/episodes/chunk-000/file-000.parquet, meta/stats.json
    """

    def __init__(self, root: str, repo_id: str, features: dict, *, fps=CONTROL_FPS, robot_type="franka_panda",
                 chunks_size=1000, data_files_size_in_mb=100, threaded=False, queue_depth=64,
                 image_compression="SNAPPY", keep_image_sums=False, io_threads=None, batch_episodes=64,
                 batch_mb=64):
        import pyarrow as pa
        import pyarrow.compute  # noqa: F401  (imported here, not on the first episode)
        import pyarrow.parquet  # noqa: F401

        self.pa = pa
        self.root, self.repo_id, self.features, self.fps = root, repo_id, features, fps
        self.robot_type, self.chunks_size, self.data_files_size_in_mb = robot_type, chunks_size, data_files_size_in_mb
        os.makedirs(root, exist_ok=True)
        self.num_keys = [k for k, f in features.items() if f["dtype"] == "float32"]
        self.str_keys = [k for k, f in features.items() if f["dtype"] == "string"]
        self.img_keys = [k for k, f in features.items() if f["dtype"] == "image"]
        self.img_type = pa.struct([("bytes", pa.binary()), ("path", pa.string())])
        self.tasks, self.task_idx = [], {}
        self.ep_rows = []
        self.chunk, self.fileno, self.start = 0, 0, 0
        self.writer, self.cur_bytes = None, 0  # the open data file (its path) and its bytes so far
        self.limit = data_files_size_in_mb * 1024 * 1024
        # numeric features' running [min, max, sum, sumsq, count] over the concatenation of their
        # dims (num_keys order, _num_dims each): one set of vector ops per episode, split per feature
        # at close (elementwise, so bit-identical to per-feature accumulators)
        self._num_dims = [int(np.prod(features[k]["shape"])) for k in self.num_keys]
        self.num_acc = None
        self.img_acc = {}  # feature -> [min, max, sum, sumsq, pixels, frames]
        self.n_episodes = 0
        # seconds spent per part of the writer (diagnostics, tools/dataset_bench.py): episode
        # statistics + rows, arrow table building, waiting for a free I/O slot, parquet encode + write
        import threading as _threading

        self.timing = {"episode_stats_s": 0.0, "table_build_s": 0.0, "io_slot_wait_s": 0.0, "io_write_s": 0.0}
        self._timing_lock = _threading.Lock()
        # episodes are encoded in batches (one arrow table / parquet row group per run of episodes
        # that land in the same data file): the per-table arrow overhead is paid once per batch
        self.batch_episodes, self.batch_bytes = max(1, int(batch_episodes)), float(batch_mb) * 1024 * 1024
        self.pending, self.pending_bytes = [], 0
        self._frame_names = []  # "/frame_000000.png", ... (the image paths' per-frame suffixes)
        self.image_compression = image_compression
        # shards keep each episode's raw image sums in meta/episodes, so merge_shards rebuilds the
        # dataset statistics bit for bit
        self.keep_image_sums = keep_image_sums
        # threaded: episodes go through a bounded queue to one writer thread (the reference writes
        # with background threads too, generate_dataset.py:260); parquet encoding and the file write
        # release the GIL, so they overlap the collection loop.  Episode order is kept.
        # parquet encoding + file writes of consecutive data files run on `io_threads` single-thread
        # lanes (file f on lane f mod io_threads, so one file's row groups stay in episode order and
        # files are written side by side; the encoding releases the GIL); episodes, statistics and
        # meta rows stay in order on the collecting thread.  At most 64 tables are in flight.
        self.io_threads = (4 if threaded else 1) if io_threads is None else max(1, int(io_threads))
        self._lanes, self._files, self._futs, self._nfile = None, {}, [], 0
        if self.io_threads > 1:
            import threading
            from concurrent.futures import ThreadPoolExecutor

            self._lanes = [ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"lerobot-io{k}")
                           for k in range(self.io_threads)]
            self._inflight = threading.BoundedSemaphore(64)
        self._q, self._thread, self._err = None, None, None
        if threaded:
            import queue
            import threading

            self._q = queue.Queue(maxsize=queue_depth)
            self._thread = threading.Thread(target=self._drain, name="lerobot-writer", daemon=True)
            self._thread.start()

    def _drain(self):
        while True:
            ep = self._q.get()
            if ep is None:
                return
            if self._err is None:
                try:
                    self._add(ep)
                except BaseException as ex:  # re-raised on the caller's thread
                    self._err = ex

    def _raise_pending(self):
        if self._err is not None:
            err, self._err = self._err, None
            raise err

    def _task(self, ep):
        t = make_task_string(ep.obj, ep.bin)
        if t not in self.task_idx:
            self.task_idx[t] = len(self.tasks)
            self.tasks.append(t)
        return t

    def _table(self, eps, starts):
        """One arrow table holding the frames of consecutive episodes `eps` (dataset indices from
        `starts`)."""
        pa = self.pa
        lens = [ep.length for ep in eps]
        cols, fields = {}, []
        for k in self.num_keys:
            dim = int(np.prod(self.features[k]["shape"]))
            arr = np.concatenate([np.asarray(ep.frames[k], np.float32).reshape(ep.length, dim) for ep in eps])
            cols[k] = pa.FixedSizeListArray.from_arrays(pa.array(arr.ravel(), pa.float32()), dim)
            fields.append(pa.field(k, pa.list_(pa.float32(), dim)))
        for k in self.str_keys:
            cols[k] = pa.array([v for ep in eps for v in ep.frames[k]], pa.string())
            fields.append(pa.field(k, pa.string()))
        nmax = max(lens) if lens else 0
        if len(self._frame_names) < nmax:
            self._frame_names = [f"/frame_{i:06d}.png" for i in range(max(nmax, 2 * len(self._frame_names)))]
        fn = self._frame_names
        fi = np.concatenate([np.arange(L, dtype=np.int64) for L in lens])
        ei = np.repeat(np.arange(len(eps), dtype=np.int64), lens)
        names = pa.array(fn[:nmax], pa.string()).take(pa.array(fi))  # "/frame_000000.png", ... per frame
        for k in self.img_keys:  # LeRobot's embedded image layout (images/<key>/episode_<e>/frame_<i>.png)
            pre = pa.array([f"images/{k}/episode_{ep.index:06d}" for ep in eps], pa.string()).take(pa.array(ei))
            paths = pa.compute.binary_join_element_wise(pre, names, "")  # joined in arrow, not per frame in Python
            if all(isinstance(ep.frames[k], PngFrames) for ep in eps):
                # one chunk per episode straight over its PngFrames buffer (zero-copy)
                chunks, o = [], 0
                for ep in eps:
                    fr = ep.frames[k]
                    if fr.nbytes >= 1 << 31:
                        raise ValueError("an episode's PNG files exceed arrow's 32-bit binary offsets")
                    b = pa.Array.from_buffers(pa.binary(), len(fr), [None, pa.py_buffer(fr.offsets.astype(np.int32)),
                                                                     pa.py_buffer(fr.data)])
                    chunks.append(pa.StructArray.from_arrays([b, paths.slice(o, len(fr))], fields=list(self.img_type)))
                    o += len(fr)
                cols[k] = pa.chunked_array(chunks, type=self.img_type)
            else:
                cols[k] = pa.StructArray.from_arrays([pa.array([v for ep in eps for v in ep.frames[k]], pa.binary()),
                                                      paths], fields=list(self.img_type))
            fields.append(pa.field(k, self.img_type))
        extra = {"timestamp": pa.array((fi / self.fps).astype(np.float32)), "frame_index": pa.array(fi),
                 "episode_index": pa.array(np.repeat(np.array([ep.index for ep in eps], np.int64), lens)),
                 "index": pa.array(np.concatenate([st + np.arange(L, dtype=np.int64) for st, L in zip(starts, lens)])),
                 "task_index": pa.array(np.repeat(np.array([self.task_idx[make_task_string(ep.obj, ep.bin)] for ep in eps],
                                                           np.int64), lens))}
        for k, v in extra.items():
            cols[k] = v
            fields.append(pa.field(k, v.type))
        return pa.Table.from_arrays([cols[f.name] for f in fields], schema=pa.schema(fields))

    def _episode_bytes(self, ep):
        """An episode's size in the data file (the roll-over test): its column data."""
        n = 4 * ep.length * sum(self._num_dims)
        for k in self.str_keys:
            n += sum(map(len, ep.frames[k])) + 4 * ep.length
        for k in self.img_keys:
            n += _png_nbytes(ep.frames[k]) + 54 * ep.length
        return n + 36 * ep.length

    @staticmethod
    def _leaf_columns(schema):
        """Parquet leaf column paths ("a.list.element", "img.bytes", ...) of an arrow schema: read
        back from an empty file written with it."""
        import io

        import pyarrow.parquet as pq

        buf = io.BytesIO()
        pq.write_table(schema.empty_table(), buf)
        buf.seek(0)
        ps = pq.ParquetFile(buf).schema
        return [ps.column(i).path for i in range(len(ps))]

    def _io(self, fn, st):
        """Run fn(st) on the open file's I/O lane (st: that file's state), or inline without lanes."""
        if self._lanes is None:
            fn(st)
            return
        t0 = time.perf_counter()
        self._inflight.acquire()
        self.timing["io_slot_wait_s"] += time.perf_counter() - t0
        fut = self._lanes[st["lane"]].submit(fn, st)
        fut.add_done_callback(lambda _f: self._inflight.release())
        self._futs.append(fut)
        if len(self._futs) > 256:  # surface I/O errors early, keep the list short
            for f in [f for f in self._futs if f.done()]:
                f.result()
            self._futs = [f for f in self._futs if not f.done()]

    def _io_wait(self):
        for f in self._futs:
            f.result()
        self._futs = []

    def _close_file(self):
        if self.writer is not None:
            def close(st):
                if st.get("w") is not None:
                    st["w"].close()
                    st["w"] = None

            self._io(close, self.writer)
            self.writer = None
            self.fileno += 1
            if self.fileno >= self.chunks_size:
                self.chunk, self.fileno = self.chunk + 1, 0
            self.cur_bytes = 0

    def add_episode(self, ep):
        """Append one episode (in episode-index order); queued when the writer is threaded."""
        if self._q is not None:
            self._raise_pending()
            self._q.put(ep)
        else:
            self._add(ep)

    def _add(self, ep):
        t0 = time.perf_counter()
        self._task(ep)
        row = {"episode_index": ep.index, "tasks": [make_task_string(ep.obj, ep.bin)], "length": ep.length,
               "data/chunk_index": None, "data/file_index": None, "dataset_from_index": self.start,
               "dataset_to_index": self.start + ep.length, "meta/episodes/chunk_index": 0,
               "meta/episodes/file_index": 0}
        if self.num_keys:  # every numeric feature's statistics from one [length, sum of dims] array
            L = ep.length
            X = np.concatenate([np.asarray(ep.frames[k], np.float64).reshape(L, -1) for k in self.num_keys], axis=1)
            mn, mx, sm = X.min(0), X.max(0), X.sum(0)
            mean = sm / L
            d = X - mean
            std = np.sqrt((d * d).sum(0) / L)  # np.std's two-pass form
            sq = (X * X).sum(0)
            # one list conversion per statistic, then python slices per feature
            lmn, lmx, lmean, lstd = mn.tolist(), mx.tolist(), mean.tolist(), std.tolist()
            o = 0
            for k, n in zip(self.num_keys, self._num_dims):
                row[f"stats/{k}/min"], row[f"stats/{k}/max"] = lmn[o:o + n], lmx[o:o + n]
                row[f"stats/{k}/mean"], row[f"stats/{k}/std"] = lmean[o:o + n], lstd[o:o + n]
                row[f"stats/{k}/count"] = [int(L)]
                o += n
            acc = self.num_acc
            self.num_acc = [mn, mx, sm, sq, L] if acc is None else \
                [np.minimum(acc[0], mn), np.maximum(acc[1], mx), acc[2] + sm, acc[3] + sq, acc[4] + L]
        for k in self.img_keys:
            st = (getattr(ep, "image_stats", None) or {}).get(k)
            if st is None:  # episodes built elsewhere: decode a frame sample
                st = _raw_image_stats([png_decode(ep.frames[k][i])
                                       for i in np.linspace(0, ep.length - 1, min(ep.length, 8)).astype(int)])
            for name in ("min", "max", "mean", "std"):
                row[f"stats/{k}/{name}"] = st[name]
            row[f"stats/{k}/count"] = [int(ep.length)]
            if self.keep_image_sums:
                row[f"stats/{k}/_sum"], row[f"stats/{k}/_sumsq"] = list(st["_sum"]), list(st["_sumsq"])
                row[f"stats/{k}/_n"] = int(st["_n"])
            mn = np.array([c[0][0] for c in st["min"]])
            mx = np.array([c[0][0] for c in st["max"]])
            acc = self.img_acc.get(k)
            vals = [mn, mx, np.array(st["_sum"]), np.array(st["_sumsq"]), st["_n"], ep.length]
            self.img_acc[k] = vals if acc is None else [np.minimum(acc[0], mn), np.maximum(acc[1], mx), acc[2] + vals[2],
                                                        acc[3] + vals[3], acc[4] + vals[4], acc[5] + vals[5]]
        self.ep_rows.append(row)
        nb = self._episode_bytes(ep)
        self.timing["episode_stats_s"] += time.perf_counter() - t0
        self.pending.append((ep, row, self.start, nb))
        self.pending_bytes += nb
        self.start += ep.length
        self.n_episodes += 1
        if len(self.pending) >= self.batch_episodes or self.pending_bytes >= self.batch_bytes:
            self._flush()

    def _flush(self):
        """Write the pending episodes: each goes to the open data file unless its bytes would take
        the file past data_files_size_in_mb (then the file is closed and the next one opened); the
        episodes of one file are written as one table."""
        import pyarrow.parquet as pq

        pending, self.pending, self.pending_bytes = self.pending, [], 0
        run = []

        def emit():
            if not run:
                return
            t0 = time.perf_counter()
            tab = self._table([r[0] for r in run], [r[2] for r in run])
            self.timing["table_build_s"] += time.perf_counter() - t0
            if self.writer is None:
                d = os.path.join(self.root, "data", f"chunk-{self.chunk:03d}")
                os.makedirs(d, exist_ok=True)
                # PNG bytes are unique per frame: no dictionary attempt on them; their compression is
                # `image_compression` (SNAPPY, parquet's and LeRobot's default, still saves ~17 % on the
                # fixed-Huffman PNGs; NONE writes faster), the other columns keep dictionary + snappy
                plain = [c for c in tab.column_names if c not in self.img_keys]
                comp = {c: (self.image_compression if c.endswith(".bytes") and c[:-6] in self.img_keys else "SNAPPY")
                        for c in self._leaf_columns(tab.schema)}
                path = os.path.join(d, f"file-{self.fileno:03d}.parquet")
                self.writer = {"path": path, "lane": self._nfile % self.io_threads, "w": None,
                               "schema": tab.schema, "kw": dict(use_dictionary=plain, compression=comp)}
                self._nfile += 1

            def write(st, tab=tab):
                t1 = time.perf_counter()
                if st["w"] is None:
                    st["w"] = pq.ParquetWriter(st["path"], st["schema"], **st["kw"])
                st["w"].write_table(tab)
                with self._timing_lock:
                    self.timing["io_write_s"] += time.perf_counter() - t1

            self._io(write, self.writer)
            run.clear()

        for item in pending:
            ep, row, start, nb = item
            if self.cur_bytes > 0 and self.cur_bytes + nb > self.limit:
                emit()
                self._close_file()
            row["data/chunk_index"], row["data/file_index"] = self.chunk, self.fileno
            run.append(item)
            self.cur_bytes += nb
        emit()

    def close(self, extra_info=None):
        import pyarrow as pa
        import pyarrow.parquet as pq

        if self._q is not None:
            self._q.put(None)
            self._thread.join()
            self._q, self._thread = None, None
            self._raise_pending()
        self._flush()
        self._close_file()
        if self._lanes is not None:
            self._io_wait()
            for lane in self._lanes:
                lane.shutdown(wait=True)
            self._lanes = None
        meta = os.path.join(self.root, "meta")
        os.makedirs(os.path.join(meta, "episodes", "chunk-000"), exist_ok=True)
        rows = sorted(self.ep_rows, key=lambda r: r["episode_index"])
        pq.write_table(pa.Table.from_pylist(rows), os.path.join(meta, "episodes", "chunk-000", "file-000.parquet"))
        pq.write_table(pa.table({"task_index": pa.array(np.arange(len(self.tasks), dtype=np.int64)),
                                 "task": pa.array(self.tasks, pa.string())}), os.path.join(meta, "tasks.parquet"))
        stats = {}
        o = 0
        for k, nd in zip(self.num_keys, self._num_dims) if self.num_acc is not None else ():
            mn, mx, sm, sq, n = [a[o:o + nd] for a in self.num_acc[:4]] + [self.num_acc[4]]
            o += nd
            mean = sm / n
            stats[k] = {"min": mn.tolist(), "max": mx.tolist(), "mean": mean.tolist(),
                        "std": np.sqrt(np.maximum(sq / n - mean * mean, 0.0)).tolist(), "count": [int(n)]}
        shape = lambda v: [[[float(a)]] for a in v]  # noqa: E731
        for k, (mn, mx, sm, sq, npx, nfr) in self.img_acc.items():
            mean = sm / npx
            stats[k] = {"min": shape(mn), "max": shape(mx), "mean": shape(mean),
                        "std": shape(np.sqrt(np.maximum(sq / npx - mean * mean, 0.0))), "count": [int(nfr)]}
        with open(os.path.join(meta, "stats.json"), "w") as f:
            json.dump(stats, f, indent=1)
        feats = {k: {"dtype": v["dtype"], "shape": list(v["shape"]), "names": v["names"]}
                 for k, v in self.features.items()}
        for k, dt in (("timestamp", "float32"), ("frame_index", "int64"), ("episode_index", "int64"),
                      ("index", "int64"), ("task_index", "int64")):
            feats[k] = {"dtype": dt, "shape": [1], "names": None}
        info = {"codebase_version": "v3.0", "robot_type": self.robot_type, "total_episodes": self.n_episodes,
                "total_frames": int(self.start), "total_tasks": len(self.tasks), "chunks_size": self.chunks_size,
                "data_files_size_in_mb": self.data_files_size_in_mb, "video_files_size_in_mb": 500, "fps": self.fps,
                "splits": {"train": f"0:{self.n_episodes}"},
                "data_path": "data/chunk-{chunk_index:03d}/file-{file_index:03d}.parquet", "video_path": None,
                "features": feats}
        if extra_info:
            info.update(extra_info)
        with open(os.path.join(meta, "info.json"), "w") as f:
            json.dump(info, f, indent=4)
        return info


def write_lerobot_v3(root: str, repo_id: str, episodes, features: dict, *, fps=CONTROL_FPS,
                     robot_type="franka_panda", chunks_size=1000, data_files_size_in_mb=100, extra_info=None):
    """Write a list of episodes in the LeRobot v3.0 layout (LeRobotWriter, episodes in index order)."""
    w = LeRobotWriter(root, repo_id, features, fps=fps, robot_type=robot_type, chunks_size=chunks_size,
                      data_files_size_in_mb=data_files_size_in_mb)
    for ep in sorted(episodes, key=lambda e: e.index):
        w.add_episode(ep)
    return w.close(extra_info)


def read_lerobot_v3(root: str):
    """Load the frames written by write_lerobot_v3 -> (info, metadata or None, {episode: {feature: array}})."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    info = json.load(open(os.path.join(root, "meta", "info.json")))
    md_path = os.path.join(root, "metadata.json")
    metadata = json.load(open(md_path)) if os.path.exists(md_path) else None
    eps_tab = pq.read_table(os.path.join(root, "meta", "episodes", "chunk-000", "file-000.parquet")).to_pylist()
    out = {}
    files = {}
    for row in eps_tab:
        key = (row["data/chunk_index"], row["data/file_index"])
        if key not in files:
            p = info["data_path"].format(chunk_index=key[0], file_index=key[1])
            files[key] = pq.read_table(os.path.join(root, p))
        tab = files[key]
        epi = tab.column("episode_index").to_numpy()
        sel = np.where(epi == row["episode_index"])[0]
        fr = {}
        for name in tab.column_names:
            col = tab.column(name).take(sel).combine_chunks()
            if pa.types.is_fixed_size_list(col.type):
                fr[name] = np.asarray(col.flatten(), np.float32).reshape(len(sel), col.type.list_size)
            elif pa.types.is_struct(col.type):  # embedded image: {bytes: PNG, path}
                fr[name] = np.stack([png_decode(v["bytes"]) for v in col.to_pylist()]) if len(sel) else None
            elif pa.types.is_string(col.type):
                fr[name] = col.to_pylist()
            else:
                fr[name] = col.to_numpy()
        out[row["episode_index"]] = fr
    return info, metadata, out


# ----------------------------------------------------------------------------- entry point
def _features_at(feats: dict, image_size: int) -> dict:
    """The feature schema with the image features at the rendered size (features.py:11-20 states
    224 x 224; the renderer takes any size)."""
    return {k: (dict(v, shape=(image_size, image_size, 3)) if v["dtype"] == "image" else v) for k, v in feats.items()}


def generate(repo_id, num_episodes=100, root="./datasets", task=None, tasks="all", reward_type="staged",
             randomize_objects=False, seed=0, spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45),
             features=None, num_envs=1024, device=0, image_size=IMAGE_SIZE, rank=0, world_size=1):
    """generate_dataset.main (generate_dataset.py:201-333) with the episodes batched on the GPU and
    streamed to the LeRobot writer as they finish.

    Sharded (world_size > 1, one process per GPU): rank r generates the episodes
    e = r (mod world_size) with their global seeds and tasks and writes them as a LeRobot dataset
    of its own in `<root>/<repo_id>/shard-RRR-of-WWW` (local episode indices 0..n-1, the global
    ones in its metadata.json under "shard"); merge_shards then writes the dataset a single
    process would have written.  Returns (path written, info)."""
    if not repo_id:
        raise ValueError("repo_id is required (e.g. repo_id=user/pick-place)")
    task_list = resolve_tasks(task, tasks)
    feats = _features_at(resolve_features(features, reward_type), image_size)
    path = os.path.join(root, repo_id)
    ids = rank_episodes(num_episodes, rank, world_size)
    out = path if world_size == 1 else shard_dir(path, rank, world_size)
    writer = LeRobotWriter(out, repo_id, feats, threaded=True, keep_image_sums=world_size > 1)
    local = []

    def sink(ep):  # shard-local episode numbering (a LeRobot dataset counts from 0)
        local.append(ep.index)
        ep.index = len(local) - 1
        writer.add_episode(ep)

    _, seeds = collect_episodes(num_episodes, task_list, set(feats), reward_type=reward_type,
                                randomize_objects=randomize_objects, seed=seed, spawn_x_range=spawn_x_range,
                                spawn_y_range=spawn_y_range, num_envs=num_envs, device=device, sink=sink,
                                image_size=image_size, episode_ids=ids)
    cfg = {"repo_id": repo_id, "num_episodes": int(num_episodes), "root": root,
           "task": list(task) if task is not None else None, "tasks": tasks, "reward_type": reward_type,
           "randomize_objects": bool(randomize_objects), "seed": int(seed), "spawn_x_range": list(spawn_x_range),
           "spawn_y_range": list(spawn_y_range), "push_to_hub": False, "private": True,
           "features": list(features) if features is not None else None}
    if image_size != IMAGE_SIZE:
        cfg["image_size"] = int(image_size)
    if seeds is not None:
        cfg["episode_seeds"] = [int(s) for s in seeds]
    md = cfg if world_size == 1 else dict(cfg, shard={"rank": int(rank), "world_size": int(world_size),
                                                      "global_episode_index": local})
    info = writer.close(extra_info={"generation_config": md})
    with open(os.path.join(out, "metadata.json"), "w") as f:
        json.dump(md, f, indent=2)
    return out, info


def _shard_episodes(sdir: str, feats: dict, global_ids: list, seeds):
    """Episodes of one shard in its (global-index increasing) order, read file by file: Episode
    objects with their global index, PNG bytes as stored and the image statistics the writer kept."""
    import pyarrow.parquet as pq

    info = json.load(open(os.path.join(sdir, "meta", "info.json")))
    rows = pq.read_table(os.path.join(sdir, "meta", "episodes", "chunk-000", "file-000.parquet")).to_pylist()
    by_task = {make_task_string(o, b): (o, b) for o in OBJECTS for b in BINS}
    cur_key, tab, epi = None, None, None
    for row in sorted(rows, key=lambda r: r["episode_index"]):
        key = (row["data/chunk_index"], row["data/file_index"])
        if key != cur_key:
            cur_key = key
            tab = pq.read_table(os.path.join(sdir, info["data_path"].format(chunk_index=key[0], file_index=key[1])))
            epi = tab.column("episode_index").to_numpy()
        sel = np.where(epi == row["episode_index"])[0]
        g = int(global_ids[row["episode_index"]])
        obj, bin_ = by_task[row["tasks"][0]]
        ep = Episode(g, obj, bin_, int(seeds[g]) if seeds else None, length=int(row["length"]))
        part = tab.take(sel)
        for k, f in feats.items():
            col = part.column(k).combine_chunks()
            if f["dtype"] == "float32":
                ep.frames[k] = np.asarray(col.flatten(), np.float32).reshape(len(sel), -1)
            elif f["dtype"] == "string":
                ep.frames[k] = col.to_pylist()
            else:
                ep.frames[k] = col.field("bytes").to_pylist()
                ep.image_stats[k] = {n: row[f"stats/{k}/{n}"] for n in ("min", "max", "mean", "std", "_sum", "_sumsq",
                                                                        "_n")}
        yield ep


def merge_shards(path: str, remove_shards: bool = False):
    """Merge the LeRobot shards a sharded generate() wrote under `path` into the dataset one
    process would have written there (episodes in global order, global indices, the same
    statistics and metadata bit for bit).  Streams: one data file per shard is held at a time."""
    import heapq
    import shutil

    sdirs = sorted(d for d in (os.path.join(path, x) for x in os.listdir(path)) if os.path.basename(d).startswith("shard-"))
    if not sdirs:
        raise ValueError(f"no shards under {path}")
    mds = [json.load(open(os.path.join(d, "metadata.json"))) for d in sdirs]
    world = mds[0]["shard"]["world_size"]
    if len(sdirs) != world or sorted(m["shard"]["rank"] for m in mds) != list(range(world)):
        raise ValueError(f"expected {world} shards, found ranks {[m['shard']['rank'] for m in mds]}")
    cfg = {k: v for k, v in mds[0].items() if k != "shard"}
    feats = _features_at(resolve_features(cfg["features"], cfg["reward_type"]), cfg.get("image_size", IMAGE_SIZE))
    seeds = cfg.get("episode_seeds")
    writer = LeRobotWriter(path, cfg["repo_id"], feats, threaded=True)
    streams = [_shard_episodes(d, feats, m["shard"]["global_episode_index"], seeds) for d, m in zip(sdirs, mds)]
    n = 0
    for ep in heapq.merge(*streams, key=lambda e: e.index):
        if ep.index != n:
            raise ValueError(f"episode {n} missing from the shards (next is {ep.index})")
        writer.add_episode(ep)
        n += 1
    if n != cfg["num_episodes"]:
        raise ValueError(f"shards hold {n} of {cfg['num_episodes']} episodes")
    info = writer.close(extra_info={"generation_config": cfg})
    with open(os.path.join(path, "metadata.json"), "w") as f:
        json.dump(cfg, f, indent=2)
    if remove_shards:
        for d in sdirs:
            shutil.rmtree(d)
    return info


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate a LeRobot v3.0 dataset from batched expert FSM episodes")
    ap.add_argument("--repo-id", required=True)
    ap.add_argument("--num-episodes", type=int, default=100)
    ap.add_argument("--root", default="./datasets")
    ap.add_argument("--task", nargs=2, default=None, metavar=("OBJ", "BIN"))
    ap.add_argument("--tasks", default="all")
    ap.add_argument("--reward-type", default="staged")
    ap.add_argument("--randomize-objects", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--spawn-x-range", type=float, nargs=2, default=(-0.20, 0.20))
    ap.add_argument("--spawn-y-range", type=float, nargs=2, default=(0.30, 0.45))
    ap.add_argument("--features", nargs="*", default=None)
    ap.add_argument("--num-envs", type=int, default=1024, help="parallel envs per GPU")
    ap.add_argument("--image-size", type=int, default=IMAGE_SIZE)
    ap.add_argument("--no-merge", action="store_true", help="sharded run: keep the per-rank shards only")
    ap.add_argument("--dist-backend", default=None, help="sharded run: collective backend (default nccl = RCCL)")
    a = ap.parse_args(argv)
    # one process per GPU under torchrun (RANK / LOCAL_RANK / WORLD_SIZE): each rank writes its
    # shard, a gather of the per-rank summaries (the only collective) tells rank 0 they are done
    rank, local_rank, world = (int(os.environ.get(k, d)) for k, d in (("RANK", 0), ("LOCAL_RANK", 0), ("WORLD_SIZE", 1)))
    import time

    t0 = time.perf_counter()
    path, info = generate(a.repo_id, a.num_episodes, a.root, a.task, a.tasks, a.reward_type, a.randomize_objects,
                          a.seed, a.spawn_x_range, a.spawn_y_range, a.features, a.num_envs, device=local_rank,
                          image_size=a.image_size, rank=rank, world_size=world)
    summary = [float(info["total_episodes"]), float(info["total_frames"]), time.perf_counter() - t0]
    if world > 1:
        import torch
        import torch.distributed as dist

        backend = a.dist_backend or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend)
        dev = torch.device("cuda", local_rank) if backend == "nccl" else torch.device("cpu")
        mine = torch.tensor(summary, dtype=torch.float64, device=dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        dist.destroy_process_group()
        if rank != 0:
            return
        per_rank = [t.cpu().tolist() for t in every]
        print(json.dumps({"shards": [{"rank": r, "episodes": int(e), "frames": int(f), "seconds": round(s, 3)}
                                     for r, (e, f, s) in enumerate(per_rank)]}))
        if a.no_merge:
            return
        info = merge_shards(os.path.join(a.root, a.repo_id))
        path = os.path.join(a.root, a.repo_id)
    print(f"Dataset saved to {path}: {info['total_episodes']} episodes, {info['total_frames']} frames")


if __name__ == "__main__":
    main()
