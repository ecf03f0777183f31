"""Render-only timing (experiment infrastructure): mmx_forward over C5-shaped states with and
without cameras; the difference is the render kernel's time for all envs and both cameras.

  python tools/render_time.py [--envs 8192] [--size 128] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_manip_amd import _lib  # noqa: E402
from mujoco_manip_amd.vec_env import PickPlaceVecEnv  # noqa: E402


def timed_forward(env, reps):
    env.sim.forward()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        env.sim.forward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    res = {"envs": a.envs, "image_size": a.size, "lib": os.environ.get("MMX_LIB_PATH", "libmmx.so"), "points": []}
    envs = {}
    for size in (a.size, 0):
        envs[size] = PickPlaceVecEnv(a.envs, tasks="all", action_mode="abs_pos", reward_type="staged",
                                     randomize_objects=True, autoreset=True, image_size=size)
        envs[size].reset(seed=[_lib.episode_seed(42, i) for i in range(a.envs)])
    for chunk in range(4):  # states spread over the episode (approach, grasp, transport, release)
        for e in envs.values():
            e.rollout_expert(20)
        q, v, c, w = envs[a.size].sim.get_state()
        envs[0].sim.set_state(q, v, c, w)
        ms_img = timed_forward(envs[a.size], a.reps)
        ms_0 = timed_forward(envs[0], a.reps)
        px = a.envs * 2 * a.size * a.size
        res["points"].append({"env_step": 20 * (chunk + 1), "forward_ms": ms_img, "forward_no_camera_ms": ms_0,
                              "render_ms": ms_img - ms_0, "gpix_per_s": px / (ms_img - ms_0) / 1e6})
    res["render_ms_mean"] = sum(p["render_ms"] for p in res["points"]) / len(res["points"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
