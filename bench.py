#!/usr/bin/env python3
"""Benchmark: env steps/s (whole node) for the batched pick-and-place hot path on MI355X.

Workload (BASELINE.json configs[2], "C3"): 4096 parallel envs per GPU, tasks='all' (9 combos),
randomize_objects=True, env i seeded SeedSequence(42).spawn(N)[i].generate_state(1)[0]
(scripts/generate_dataset.py:263-268) using the GLOBAL env index (results independent of
sharding), FSM-expert abs_pos actions computed on device (pick_and_place.py plan(16)),
same-step autoreset.  One "step" = one PickPlaceGymEnv.step for every env: decode -> 16 x
(DLS IK + mj_step) -> mj_forward (position stage) -> staged reward -> 85-float obs.

Multi-GPU: one process per GPU (torchrun), weak scaling (4096 envs per rank), no data-path
collective; an all_reduce(MAX) of the elapsed time and an all_gather of per-rank stats for
logging only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SUBSTEPS = 16  # physics substeps per env step (all inside one mmx_env_step_kernel launch)


def algorithmic_bytes_per_env_step(nefc: float) -> float:
    """B = B_io + 16 (B_state + B_efc) bytes per env step, fp32 words, with
    B_io = 416, B_state = 2*4*(nq+nv+nv+nu) = 736, B_efc = 2*4*nefc*(nv+4) = 248 nefc."""
    return 416 + 16 * (2 * 4 * (30 + 27 + 27 + 8) + 2 * 4 * nefc * (27 + 4))


def min_hbm_bytes_per_env_step() -> float:
    """Bytes the fused kernel must move per env step: env record in+out (qpos, qvel, ctrl,
    warm start, IK cache, target, stats, episode ints/floats, rng) + obs/reward/flags out."""
    rec = 4 * (30 + 27 + 8 + 27 + 54 + 4 + 17 + 14 + 28) + 8 * 4 + 4
    return 2 * rec + 4 * (85 + 1 + 3 + 6)


def _cpu_worker(args) -> tuple:
    """One single-env C3 loop on the oracle for `seconds`; episodes worker, worker + P, ..."""
    worker, nworkers, seconds = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O
    from mujoco_manip_amd.constants import ALL_TASKS, BINS, OBJECTS

    steps = 0
    t0 = time.perf_counter()
    ep = worker
    while time.perf_counter() - t0 < seconds:
        e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                        tasks=[(OBJECTS.index(o), BINS.index(b)) for o, b in ALL_TASKS])
        e.reset(seed=O.episode_seed(42, ep))
        o, b = e.task()
        e.fsm_init([(o, b)])
        for _ in range(400):
            st = e.fsm_plan(16)
            if st == 10:
                break
            f = e.fsm_get()
            tgt = f["target"] if f["state"] != 0 else e.body(9)[0]
            e.step(np.array([*tgt, float(f["gripper_open"])], np.float32))
            steps += 1
            if time.perf_counter() - t0 > seconds:
                break
        ep += nworkers
    return steps, time.perf_counter() - t0, (ep - worker) // nworkers


def cpu_baseline(seconds: float = 12.0, workers: int | None = None) -> dict:
    """The oracle (fp64 C restatement; MuJoCo is absent on the box) on a bounded sample of the
    same workload: P independent single-env C3 loops, one per host core share,
    run before the process touches the GPU.  Throughput = sum over workers."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O

    O.build()
    if workers is None:
        workers = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(w, workers, seconds) for w in range(workers)])
    steps = sum(r[0] for r in res)
    rate = sum(r[0] / r[1] for r in res)
    eps = sum(r[2] for r in res)
    return {"value": rate, "unit": "env steps/s", "cores": workers, "kind": "port",
            "sample": f"{steps} env steps ({eps} FSM-expert episodes, C3 settings) in {seconds:.0f}s on each of "
                      f"{workers} worker processes (1 thread each); oracle/ fp64 C restatement, MuJoCo absent on "
                      f"the box; host cpu_count={os.cpu_count()}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # >= 500 timed env steps after >= 50 warm-up steps; multiples of the fused
    # launch length (16 env steps per launch) keep every timed dispatch the same size
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    # rehearsal of the N > 1 path on a 1-GPU box: ranks share device 0 and talk over gloo
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--share-device", action="store_true")
    # 0 = the C3 workload (no images); 128 = C5's two 128 x 128 RGB cameras per env step
    ap.add_argument("--image-size", type=int, default=0)
    # BASELINE.json configs: c3 (default, the metric's config), c2 (1024 envs, fixed task
    # (obj_red, bin_red), keyframe start, no randomisation), c5 (c3 settings + 2 x 128^2 RGB
    # cameras per env step, 8192 envs per GPU as in the 65536-env / 8-GPU config)
    ap.add_argument("--workload", default="c3", choices=("c2", "c3", "c5"))
    args = ap.parse_args()
    if args.workload == "c5":
        args.image_size = args.image_size or 128
        if args.envs_per_gpu == 4096:
            args.envs_per_gpu = 8192
    if args.workload == "c2" and args.envs_per_gpu == 4096:
        args.envs_per_gpu = 1024

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first: worker processes are forked before anything initialises the GPU
    cpu = None
    if not args.no_cpu_baseline and world == 1 and rank == 0:
        cpu = cpu_baseline(args.cpu_seconds)
    dist = None
    dev_index = 0 if args.share_device else local_rank
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(dev_index)
        dist.init_process_group(args.dist_backend)
    dev = torch.device(f"cuda:{dev_index}")
    torch.cuda.set_device(dev)
    # collectives run on device tensors over RCCL, on host tensors over gloo
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N = args.envs_per_gpu
    c2 = args.workload == "c2"
    env = PickPlaceVecEnv(N, task=("obj_red", "bin_red") if c2 else None, tasks="all", action_mode="abs_pos",
                          reward_type="staged", randomize_objects=not c2, image_size=args.image_size,
                          autoreset=True, device=dev_index)
    seeds = [_lib.episode_seed(42, rank * N + i) for i in range(N)]
    env.reset(seed=seeds)

    # warmup
    env.rollout_expert(args.warmup)
    torch.cuda.synchronize()
    env.clear_stats()
    # the sim launches on torch's current stream and forks its `lanes` concurrent env ranges from
    # it (each range: one mmx_env_step_kernel launch per env step on its own stream, joined back at
    # the end): events on that stream bracket the K env steps of every range, so kern_ms is the
    # per-step span over which the lanes' launches (N envs in total) ran side by side
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    env.rollout_expert(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # each lane runs ceil(K / spl) launches of up to spl env steps of its envs, back to back
    spl = env.sim.rollout_steps_per_launch
    launches = -(-args.steps // spl)
    kern_ms = ev0.elapsed_time(ev1) / launches  # per launch
    if dist:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    solver = env.solver_stats()
    env_steps = args.steps * N * world
    value = env_steps / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # spl env steps of the batch = `lanes` concurrent mmx_env_step_kernel dispatches of N / lanes
    # envs x spl steps each; they run side by side for the whole span, so a dispatch lasts ~kern_ms
    # (rocprof's per-dispatch average agrees) and the chip-level rate is lanes x one dispatch's
    # bytes / kern_ms
    lanes = env.sim.rollout_lanes
    envs_per_launch = N / lanes
    steps_per_launch = args.steps / launches
    bytes_per_launch = algorithmic_bytes_per_env_step(solver["mean_nefc"]) * envs_per_launch * steps_per_launch
    achieved = lanes * bytes_per_launch / (kern_ms * 1e-3) / 1e9
    min_bytes = min_hbm_bytes_per_env_step() * envs_per_launch * steps_per_launch

    stats_all = None
    if dist:
        loc = torch.tensor([solver["mean_nefc"], solver["mean_solver_iter"], value / world], device=cdev)
        gathered = [torch.zeros_like(loc) for _ in range(world)]
        dist.all_gather(gathered, loc)
        stats_all = [g.tolist() for g in gathered]

    if rank == 0:
        traffic = None
        tf = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(tf):
            try:
                traffic = json.load(open(tf)).get("bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": "env steps/sec (whole node) at 4096 parallel envs; 1/2/4/8 MI355X scaling",
            "value": value, "unit": "env steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (seeded randomized scenes, FSM-expert actions)",
            "config": {"workload": (f"C2: PickPlaceGymEnv.step x {N} envs/GPU, fixed task (obj_red, bin_red), "
                                    "keyframe start (no randomisation), staged reward, FSM expert abs_pos, autoreset"
                                    if c2 else
                                    f"C3: PickPlaceGymEnv.step x {N} envs/GPU, tasks=all, randomize_objects, "
                                    "seed=42 episode seeds, staged reward, FSM expert abs_pos, autoreset"
                                    if args.image_size == 0 else
                                    f"C5: C3 settings x {N} envs/GPU plus overhead + wrist RGB {args.image_size}x"
                                    f"{args.image_size} camera images rendered every env step"),
                       "envs_per_gpu": N, "global_envs": N * world, "substeps": 16, "image_size": args.image_size,
                       "parallelism": f"env-batch dp{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "mmx_env_step_kernel", "kernel_ms": kern_ms,
                         "concurrent_launches": lanes, "envs_per_launch": envs_per_launch,
                         "env_steps_per_launch": steps_per_launch,
                         "algorithmic_bytes_per_env_step": algorithmic_bytes_per_env_step(solver["mean_nefc"]),
                         "algorithmic_bytes_per_launch": bytes_per_launch, "mean_nefc": solver["mean_nefc"],
                         "traffic_note": "traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per dispatch "
                                         "(profiles/pmc_traffic.json), same dispatch size",
                         "min_hbm_bytes_per_launch": min_bytes,
                         "min_hbm_GBs": lanes * min_bytes / (kern_ms * 1e-3) / 1e9},
            "cpu_baseline": cpu,
            "solver": solver,
        }
        if stats_all:
            line["per_rank"] = stats_all
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
