"""Dump a few rendered frames (RGB + segment ids) as PNGs under gpurun_out/ (diagnostic)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from mujoco_manip_amd import _lib  # noqa: E402
from mujoco_manip_amd.vec_env import PickPlaceVecEnv  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 224
out = os.path.join(REPO, "gpurun_out", "render")
os.makedirs(out, exist_ok=True)
pal = np.array([[40, 60, 90], [60, 80, 100], [150, 120, 90], [180, 60, 60], [60, 160, 60], [60, 60, 180],
                [255, 0, 0], [0, 255, 0], [0, 0, 255], [230, 230, 230]], np.uint8)
env = PickPlaceVecEnv(2, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                      image_size=S)
env.reset(seed=[_lib.episode_seed(5, i) for i in range(2)])
for t in range(60):
    obs, *_ = env.step(env.expert_plan(16))
    if t in (0, 20, 40, 59):
        seg = env.segmentation.cpu().numpy()
        for ci, cam in enumerate(("overhead", "wrist")):
            img = obs["image_" + cam][0].cpu().numpy()
            Image.fromarray(np.concatenate([img, pal[seg[0, ci]]], 1)).save(os.path.join(out, f"{cam}_{t:03d}.png"))
print("wrote", sorted(os.listdir(out)))
