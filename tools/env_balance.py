"""Diagnostic: distribution of per-env shader cycles over a 16-step fused launch window (C3), from
the MMX_PROFILE=1 build's per-env phase clocks.  Shows how much a launch's slowest env exceeds the
mean (the launch-tail cost of lockstep launches)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MMX_PROFILE", "1")
from mujoco_manip_amd import _lib  # noqa: E402
from mujoco_manip_amd.vec_env import PickPlaceVecEnv  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                      autoreset=True, image_size=0)
env.reset(seed=[_lib.episode_seed(42, i) for i in range(N)])
env.rollout_expert(64)
out = {}
for w in range(4):
    env.clear_stats()
    env.rollout_expert(16)
    torch.cuda.synchronize()
    st = env.stats.double().cpu().numpy()
    cyc = st[:, 5:13].sum(1)  # phase cycles of the 16 steps, per env
    lane = cyc.reshape(4, -1)  # the 4 rollout lanes' env ranges
    out[f"window{w}"] = {"mean": cyc.mean(), "p50": np.percentile(cyc, 50), "p90": np.percentile(cyc, 90),
                         "p99": np.percentile(cyc, 99), "max": cyc.max(),
                         "lane_max_over_mean": (lane.max(1) / lane.mean(1)).tolist(),
                         "mean_nefc": float(st[:, 0].sum() / st[:, 3].sum())}
    env.rollout_expert(48)
print(json.dumps(out, indent=1))
