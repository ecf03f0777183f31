"""PNG encoder A/B (experiment tooling): encode one deterministic image set with the library
MMX_LIB_PATH points at and print the SHA-256 of every packed file plus the encode time of 8192
rendered 128 x 128 frames (hipEvent-free: torch.cuda.synchronize around 20 repetitions)."""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_manip_amd import _lib
from mujoco_manip_amd.vec_env import PickPlaceVecEnv


def main():
    rng = np.random.default_rng(3)
    sim = _lib.Sim(1, action_mode="abs_pos", image_size=0)
    sets = [rng.integers(0, 256, (16, 128, 128, 3), dtype=np.uint8),
            np.repeat(rng.integers(0, 256, (4, 1, 224, 3), dtype=np.uint8), 224, axis=1),
            rng.integers(0, 4, (8, 57, 91, 3), dtype=np.uint8) * 60]
    env = PickPlaceVecEnv(8192, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=128, autoreset=True)
    env.reset(seed=[_lib.episode_seed(5, i) for i in range(8192)])
    for _ in range(30):
        env.step(env.expert_plan(16))
    frames = env._images[:, 0].contiguous()
    h = hashlib.sha256()
    for imgs in sets + [frames[:512].cpu().numpy(), env._images[:512, 1].contiguous().cpu().numpy()]:
        packed, offs = sim.png_encode(torch.as_tensor(imgs).cuda())
        h.update(packed.cpu().numpy().tobytes())
        h.update(np.asarray(offs, np.int64).tobytes())
    torch.cuda.synchronize()
    for _ in range(3):
        sim.png_encode_device(frames)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        packed, ends = sim.png_encode_device(frames)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 20 * 1e3
    print(json.dumps({"lib": _lib.load()._name, "sha256": h.hexdigest(), "encode_ms_8192x128": ms,
                      "mean_png_bytes": float(ends[-1].item()) / 8192}))


if __name__ == "__main__":
    sys.exit(main())
