"""Per-stage wall-clock split of mmx_render_kernel (diagnostic): run with MMX_LIB_PATH pointing at
a build with -DMMR_CLOCK (tools/ab_build.py rclk:MMR_CLOCK).  C5 shape (8192 envs, 128^2, FSM
expert); prints wave 0's mean microseconds per workgroup per stage -> gpurun_out/render_clock.json."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_manip_amd import _lib  # noqa: E402
from mujoco_manip_amd.vec_env import PickPlaceVecEnv  # noqa: E402

STAGES = ["poses_camera_clear", "vertices", "triangle_setup_queues", "small_raster", "large_tiles_shading"]


def main():
    n = int(os.environ.get("RCLK_ENVS", "8192"))
    env = PickPlaceVecEnv(n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=128, autoreset=True)
    env.reset(seed=42)
    env.rollout_expert(8)
    torch.cuda.synchronize()
    L = _lib.load()
    buf = (C.c_ulonglong * 8)()
    L.mmx_render_clock.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    assert L.mmx_render_clock(buf, 1) == 0
    env.rollout_expert(16)
    torch.cuda.synchronize()
    assert L.mmx_render_clock(buf, 0) == 0
    wgs = max(buf[5], 1)
    us = {s: buf[k] / wgs / 100.0 for k, s in enumerate(STAGES)}  # 100 MHz ticks -> us
    res = {"workgroups": int(buf[5]), "small_triangles_per_workgroup": buf[6] / wgs,
           "small_bbox_px_per_workgroup": buf[7] / wgs, "us_per_workgroup": us, "total_us": sum(us.values()),
           "share": {s: v / sum(us.values()) for s, v in us.items()}}
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/render_clock.json", "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
