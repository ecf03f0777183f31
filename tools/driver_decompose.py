"""Decompose the driver configuration's window rates (bench.py --steps 20 --warmup 5: five 20-step
rollout calls after 5 warm-up steps) into the phase mix of each window and the per-call launch
overhead.  Diagnostic; run with MMX_PROFILE=1 (libmmx_prof.so, whose step
kernel adds per FSM state the shader cycles of each env step into a device table).

For every window W (and a long stationary window at the end):
  busy(W)   = sum over the window's env steps of the step's own cycles (all 16 substeps, prologue,
              epilogue: the workgroup's wall clock while it ran that step)
  T(W)      = wall time of the rollout call (host clock around rollout_expert + synchronize)
  fill(W)   = busy(W) / T(W): slot-cycles retired per second, i.e. resident slots x clock x the
              fraction of slot-time spent in env steps
The rate of a window is env_steps / T = fill / (busy / env_steps): the window's speed is its fill
(drain / launch overhead) times the inverse of its mean cycles per env step (phase mix).  Against
the stationary window: rate_W / rate_S = (fill_W / fill_S) x (cyc_S / cyc_W); the first factor is
the per-call overhead, the second the phase mix.  Writes gpurun_out/driver_decompose.json."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mujoco_manip_amd import _lib  # noqa: E402
from mujoco_manip_amd.vec_env import PickPlaceVecEnv  # noqa: E402

FSM = ["idle", "pre_grasp", "grasp", "close_gripper", "lift", "move_to_bin", "settle_at_bin", "lower_to_bin", "release",
       "retreat", "done"]


def main(N=4096, warm=5, steps=20, windows=5, long_steps=512):
    assert os.environ.get("MMX_PROFILE", "0") not in ("", "0"), "needs the profile build (MMX_PROFILE=1)"
    L = _lib.load()
    nf = L.mmx_fsm_profile_fields()
    buf = (C.c_double * (11 * nf))()
    L.mmx_fsm_profile.argtypes = [C.POINTER(C.c_double), C.c_int]
    P = 12  # phase fields before FSMP_STEP (tools/gpu_probe.py)
    SLOTS = torch.cuda.get_device_properties(0).multi_processor_count * 12  # twelve envs per CU (128-row build)
    env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          autoreset=True, image_size=0)
    env.reset(seed=[_lib.episode_seed(42, i) for i in range(N)])
    env.rollout_expert(warm)
    torch.cuda.synchronize()

    def window(n):
        L.mmx_fsm_profile(buf, 1)  # reset
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.rollout_expert(n)
        torch.cuda.synchronize()
        T = time.perf_counter() - t0
        L.mmx_fsm_profile(buf, 1)
        a = np.array(buf[:]).reshape(11, nf)
        cnt, cyc, rt = a[:, nf - 1], a[:, P], a[:, nf - 2]
        assert abs(cnt.sum() - N * n) < 0.5, (cnt.sum(), N * n)
        return {"env_steps": int(cnt.sum()), "seconds": T, "rate": cnt.sum() / T, "busy_cycles": float(cyc.sum()),
                "cycles_per_env_step": float(cyc.sum() / cnt.sum()), "fill_cycles_per_s": float(cyc.sum() / T),
                # absolute: the fraction of the window's slot-time (resident workgroup slots x wall time)
                # spent inside env steps, from the constant 100 MHz clock; and the shader clock
                "slot_occupancy": float(rt.sum() * 1e-8 / (T * SLOTS)),
                "shader_clock_ghz": float(cyc.sum() / max(rt.sum(), 1.0) * 0.1),
                "phase_env_steps": {FSM[s]: int(cnt[s]) for s in range(11) if cnt[s]},
                "phase_cycles_per_env_step": {FSM[s]: float(cyc[s] / cnt[s]) for s in range(11) if cnt[s]}}

    out = {"config": {"envs": N, "warmup": warm, "steps": steps, "windows": windows, "long_steps": long_steps,
                      "lanes": env.sim.rollout_lanes, "launches_per_lane": env.sim.rollout_launches(steps)},
           "windows": [window(steps) for _ in range(windows)]}
    env.rollout_expert(64)  # into the stationary mix (episodes desynchronised by autoresets)
    out["stationary"] = window(long_steps)
    S = out["stationary"]
    for w in out["windows"]:
        w["overhead_factor"] = w["fill_cycles_per_s"] / S["fill_cycles_per_s"]  # < 1: drain / launch gaps
        w["phase_mix_factor"] = S["cycles_per_env_step"] / w["cycles_per_env_step"]  # < 1: heavier phases
        w["rate_vs_stationary"] = w["rate"] / S["rate"]
    ws = out["windows"]
    med = sorted(ws, key=lambda w: w["rate"])[len(ws) // 2]
    out["summary"] = {"median_window_rate": med["rate"], "stationary_rate": S["rate"],
                      "median_overhead_factor": med["overhead_factor"], "median_phase_mix_factor": med["phase_mix_factor"],
                      "mean_overhead_factor": float(np.mean([w["overhead_factor"] for w in ws])),
                      "mean_phase_mix_factor": float(np.mean([w["phase_mix_factor"] for w in ws])),
                      "stationary_slot_occupancy": S["slot_occupancy"],
                      "mean_window_slot_occupancy": float(np.mean([w["slot_occupancy"] for w in ws]))}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "driver_decompose.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["summary"]))
    for w in ws:
        print(round(w["rate"]), round(w["overhead_factor"], 3), round(w["phase_mix_factor"], 3))


if __name__ == "__main__":
    main()
