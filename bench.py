#!/usr/bin/env python3
"""Benchmark: env steps/s (whole node) for the batched pick-and-place hot path on MI355X.

Workload (BASELINE.json configs[2], "C3"): 4096 parallel envs per GPU, tasks='all' (9 combos),
randomize_objects=True, env i seeded SeedSequence(42).spawn(N)[i].generate_state(1)[0]
(scripts/generate_dataset.py:263-268) using the GLOBAL env index (results independent of
sharding), FSM-expert abs_pos actions computed on device (pick_and_place.py plan(16)),
same-step autoreset.  One "step" = one PickPlaceGymEnv.step for every env: decode -> 16 x
(DLS IK + mj_step) -> mj_forward (position stage) -> staged reward -> 85-float obs.

Timing: W warm-up env steps, then `--repeats` windows of exactly K env steps,
each bracketed by a barrier + device synchronise on both sides and timed as the max over ranks;
the line reports the median window (all windows listed under "repeats").

Multi-GPU: one process per GPU, weak scaling (4096 envs per rank), no data-path collective.
Under torchrun the ranks come from the environment; `--gpus N` without torchrun starts the N
rank processes itself (before anything touches a GPU) and relays rank 0's line.  Collectives:
barrier, all_reduce(MAX) of the window time, all_reduce(SUM) of the episode counters, and after
each window (untimed) an all_gather_into_tensor of every env's 16-byte episode record to rank 0
(per-rank summaries in the line's `rank_envs`).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SUBSTEPS = 16  # physics substeps per env step (all inside one mmx_env_step_kernel launch)
METRIC = "env steps/sec (whole node) at 4096 parallel envs; 1/2/4/8 MI355X scaling"


def algorithmic_bytes_per_env_step(nefc: float) -> float:
    """B = B_io + 16 (B_state + B_efc) bytes per env step, fp32 words, with
    B_io = 416, B_state = 2*4*(nq+nv+nv+nu) = 736, B_efc = 2*4*nefc*(nv+4) = 248 nefc."""
    return 416 + 16 * (2 * 4 * (30 + 27 + 27 + 8) + 2 * 4 * nefc * (27 + 4))


def min_hbm_bytes_per_env_step() -> float:
    """Bytes the fused kernel must move per env step: env record in+out (qpos, qvel, ctrl,
    warm start, IK cache, target, stats, episode ints/floats, rng) + obs/reward/flags out."""
    rec = 4 * (30 + 27 + 8 + 27 + 63 + 4 + 19 + 18 + 28) + 8 * 4 + 4
    return 2 * rec + 4 * (85 + 1 + 3 + 6)


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_budget() -> tuple[int, dict]:
    """Host cores this process may use: the affinity mask, capped by the cgroup CPU quota and by
    OMP_NUM_THREADS when set (the GPU box grants each 1-GPU job a CPU share of the host)."""
    info = {"host_cpu_count": os.cpu_count(), "cpu_model": _cpu_model()}
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    info["affinity"] = n
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_quota_cpus"] = int(q) / int(p)
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        info["omp_num_threads"] = int(os.environ["OMP_NUM_THREADS"])
        n = min(n, max(1, int(os.environ["OMP_NUM_THREADS"])))
    return max(1, n), info


# MuJoCo's default Newton settings (tolerance 1e-8, 100 iterations): the CPU baseline
# solves to them, not to the parity tests' 1e-13 / 200
MUJOCO_SOLVER = (1e-8, 100)


def _expert_episode(e, seconds_left, t0):
    """One FSM-expert episode on an oracle env (generate_dataset.py:140-196): plan(16) -> abs_pos
    -> step until the FSM is done.  Returns (env steps, placed)."""
    o, b = e.task()
    e.fsm_init([(o, b)])
    steps = 0
    for _ in range(500):
        if e.fsm_plan(16) == 10:
            break
        f = e.fsm_get()
        e.step(np.array([*f["target"], float(f["gripper_open"])], np.float32))
        steps += 1
        if time.perf_counter() - t0 > seconds_left:
            break
    return steps


def _cpu_worker(args) -> tuple:
    """Single-env C3 loops on the oracle for `seconds`: episodes worker, worker + P, ..."""
    worker, nworkers, seconds = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O
    from mujoco_manip_amd.constants import ALL_TASKS, BINS, OBJECTS

    pool = [(OBJECTS.index(o), BINS.index(b)) for o, b in ALL_TASKS]
    steps, ep, solves, iters = 0, worker, 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=True, tasks=pool)
        e.set_solver(*MUJOCO_SOLVER)
        e.reset(seed=O.episode_seed(42, ep))
        steps += _expert_episode(e, seconds, t0)
        c, i = e.solver_stats()
        solves, iters = solves + c, iters + i
        ep += nworkers
    return steps, time.perf_counter() - t0, (ep - worker) // nworkers, solves, iters


def c1_single_thread(seconds: float = 5.0) -> dict:
    """C1: 1 env, task (obj_red, bin_red), staged reward, keyframe start, FSM
    expert (generate_dataset.py:140-196), timed single-threaded on the oracle."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O

    lengths, steps = [], 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", task=(0, 0))
        e.set_solver(*MUJOCO_SOLVER)
        e.reset(seed=len(lengths))
        n = _expert_episode(e, 1e9, t0)
        lengths.append(n)
        steps += n
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env steps/s", "cores": 1, "episodes": len(lengths),
            "episode_length": int(np.median(lengths)), "ms_per_env_step": 1000.0 * dt / max(steps, 1),
            "kind": "port", "sample": f"{len(lengths)} C1 FSM-expert episodes in {dt:.1f} s, one thread"}


def cpu_baseline(seconds: float = 30.0, workers: int | None = None) -> dict:
    """The oracle (fp64 C restatement; MuJoCo is absent on the box) on a bounded sample of the
    same workload: P independent single-env C3 loops for `seconds`, one per usable host core
    (BASELINE.md §4), run before the process touches the GPU.  Throughput = sum over workers."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O

    O.build()
    budget, info = cpu_budget()
    workers = workers or budget
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(w, workers, seconds) for w in range(workers)])
    steps = sum(r[0] for r in res)
    rate = sum(r[0] / r[1] for r in res)
    eps = sum(r[2] for r in res)
    solves, iters = sum(r[3] for r in res), sum(r[4] for r in res)
    out = {"value": rate, "unit": "env steps/s", "cores": workers, "kind": "port",
           "sample": f"{steps} env steps ({eps} FSM-expert C3 episodes) in {seconds:.0f} s on each of {workers} "
                     f"worker processes (1 thread each, one per usable core); engine: oracle/ fp64 C restatement "
                     f"(MuJoCo absent on the box) with MuJoCo's default Newton settings",
           "solver": {"tolerance": MUJOCO_SOLVER[0], "max_iterations": MUJOCO_SOLVER[1],
                      "mean_iterations": iters / max(solves, 1)}, **info}
    out["c1"] = c1_single_thread()
    return out


# ----------------------------------------------------------------------------- rank launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, cmd: list[str] | None = None, poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """`--gpus N` without torchrun: start N rank processes of this script (one GPU each, RCCL),
    before this process touches any GPU; rank 0 prints the line.  All ranks are polled: the first
    non-zero exit terminates the others (a dead rank would otherwise leave its peers blocked in a
    collective) and is returned; 0 once every rank exited cleanly.  `cmd` overrides the rank
    command (tests)."""
    port = str(_free_port())
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(cmd, env=env))
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = abs(bad[0]) or 1
                print(f"bench: a rank exited with {bad[0]}; stopping the other ranks", file=sys.stderr, flush=True)
                return rc
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.monotonic() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


# ----------------------------------------------------------------------------- PMC evidence
def pmc_evidence(workload: str, envs: int, lanes: int) -> dict | None:
    """Counter evidence recorded by tools/profile.sh for THIS configuration (same workload, envs
    per GPU and concurrent launches; the counters are per env step, which the launch length -- the
    record is loaded and stored once per launch, 2.5 KB of ~100 KB per env step -- barely moves);
    None when absent or different."""
    f = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(f):
        return None
    try:
        rec = json.load(open(f))
    except (OSError, ValueError):
        return None
    c = rec.get("config", {})
    if (c.get("workload"), c.get("envs_per_gpu"), c.get("lanes")) != (workload, envs, lanes):
        return None
    return rec


def binding_roof(pmc: dict | None, workload: str) -> dict | None:
    """What bounds the step kernel, from counter evidence of this configuration: the SQ pass of
    pmc_<workload>.json (VALU instructions and issue per wave, active lanes), the extended SQ pass
    (any-instruction issue per wave) and the VALU issue calibration (what a wave / SIMD can issue).
    HBM is not the roof: the constraint working set MuJoCo streams (SURVEY §8d's algorithmic bytes)
    stays in LDS here, so the HBM frac cannot pass ~0.2 by design."""
    if pmc is None or not pmc.get("valu"):
        return None
    v = pmc["valu"]
    out = {"valu_insts_per_env_step": v.get("valu_insts_per_env_step"),
           "valu_issue_per_wave": v.get("active_inst_valu_per_wave_cycle"),
           "waves_per_simd": v.get("waves_per_simd"),
           "valu_issue_per_simd": v.get("valu_issue_per_simd"),
           "active_lane_fraction": v.get("active_lane_fraction"),
           "lane_weighted_valu_issue_per_simd": (v["valu_issue_per_simd"] * v["active_lane_fraction"]
                                                 if v.get("valu_issue_per_simd") and v.get("active_lane_fraction") else None),
           "hbm_frac_note": "HBM frac <= ~0.2 by design while the efc working set stays in LDS (DESIGN §4)",
           "units": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (quad-cycles): instructions per quad-cycle"}
    cal_f = os.path.join(REPO, "profiles", "r05_valu_issue_calibration.json")
    # the newest round's extended SQ pass of this workload (tools/gpu.sh profile:<workload>)
    import glob

    ext = sorted(glob.glob(os.path.join(REPO, "profiles", f"r0*_{workload}_sq_extended.json")))
    ext_f = ext[-1] if ext else os.path.join(REPO, "profiles", f"r06_{workload}_sq_extended.json")
    try:
        # the calibration's measured issue (SQ units, 8 independent FMA chains per wave) at 1-4 waves per
        # SIMD, interpolated linearly to the kernel's resident waves per SIMD (2.75 at 11 envs per CU)
        cal = json.load(open(cal_f))
        rows = sorted((r["waves_per_simd"], r["sq_active_inst_valu_per_wave_quad_cycle"], r["sq_valu_per_simd_quad_cycle"])
                      for r in cal["scalar_v_fma_f32"] if r["chains"] == 8)
        w = float(v.get("waves_per_simd") or 2)
        ceil_w = float(np.interp(w, [r[0] for r in rows], [r[1] for r in rows]))  # per wave quad-cycle
        ceil_s = float(np.interp(w, [r[0] for r in rows], [r[2] for r in rows]))  # per SIMD quad-cycle
        out["valu_issue_ceiling_per_wave"] = ceil_w
        out["valu_issue_ceiling_per_simd"] = ceil_s
        out["valu_issue_frac_of_ceiling"] = v["active_inst_valu_per_wave_cycle"] / ceil_w
        out["valu_issue_simd_frac_of_ceiling"] = v["valu_issue_per_simd"] / ceil_s
        out["calibration"] = "profiles/r05_valu_issue_calibration.json (measured at 1-4 waves per SIMD, interpolated)"
    except (OSError, ValueError, KeyError, IndexError, TypeError, ZeroDivisionError):
        pass
    try:
        ext = json.load(open(ext_f))["per_wave_quad_cycle"]
        out["any_inst_issue_per_wave"] = ext["SQ_ACTIVE_INST_ANY"]
        out["salu_issue_per_wave"] = ext["SQ_INSTS_SALU"]
        out["extended_sq"] = os.path.relpath(ext_f, REPO)
    except (OSError, ValueError, KeyError):
        pass
    frac = out.get("valu_issue_frac_of_ceiling")
    out["bound"] = ("latency" if frac is not None and frac < 0.6 else "valu-issue")
    out["note"] = ("the calibration kernel's waves issue VALU at ~0.94 per quad-cycle alone and ~0.8 at 2.75 waves per "
                   "SIMD (2.2 per SIMD); the step kernel's waves issue VALU at the fraction above of that and any "
                   "instruction in ~56 % of their quad-cycles: latency / dependency-bound, so env steps/s follow "
                   "the resident envs per CU (profiles/r05_occupancy_probe.json) and the instructions on each "
                   "env's critical path, not the VALU rate")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # >= 500 timed env steps after >= 50 warm-up steps; multiples of the fused
    # launch length (16 env steps per launch) keep every timed dispatch the same size
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=30.0)
    # rehearsal of the N > 1 path on a 1-GPU box: ranks share device 0 and talk over gloo
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--share-device", action="store_true")
    ap.add_argument("--dist-timeout", type=float, default=300.0, help="seconds for rendezvous and each collective")
    # 0 = the C3 workload (no images); 128 = C5's two 128 x 128 RGB cameras per env step
    ap.add_argument("--image-size", type=int, default=0)
    # BASELINE.json configs: c3 (default, the metric's config), c2 (1024 envs, fixed task
    # (obj_red, bin_red), keyframe start, no randomisation), c5 (c3 settings + 2 x 128^2 RGB
    # cameras per env step, 8192 envs per GPU as in the 65536-env / 8-GPU config)
    ap.add_argument("--workload", default="c3", choices=("c2", "c3", "c5"))
    # env-step kernel layout (mmx_set_step_rows, bit-identical results): 0 = the library's choice from
    # the batch size (192 LDS rows with a helper wave per env up to four envs per CU, e.g. C2's 1024;
    # 128 rows, twelve per CU, above: DESIGN §2); 128 / 192 force one for A/B runs
    ap.add_argument("--step-rows", type=int, default=0, choices=(0, 128, 192))
    args = ap.parse_args()
    if args.workload == "c5":
        args.image_size = args.image_size or 128
        if args.envs_per_gpu == 4096:
            args.envs_per_gpu = 8192
    if args.workload == "c2" and args.envs_per_gpu == 4096:
        args.envs_per_gpu = 1024

    from mujoco_manip_amd.shard import dist_env, env_stats_record, gather_env_stats, shard_seeds, summarize_env_stats

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank, local_rank, world = dist_env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    # CPU baseline first (rank 0 at N = 1): worker processes fork before anything initialises the GPU
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args.cpu_seconds)
    dist = None
    dev_index = 0 if args.share_device else local_rank
    if world > 1 or "WORLD_SIZE" in os.environ:  # under torchrun: the process group even for 1 rank
        import torch.distributed as dist

        import datetime

        torch.cuda.set_device(dev_index)
        # bounded: a rank that never arrives ends the job instead of hanging it
        dist.init_process_group(args.dist_backend, timeout=datetime.timedelta(seconds=args.dist_timeout))
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
    if args.step_rows:
        env.sim.step_rows = args.step_rows
    env.reset(seed=shard_seeds(42, rank, world, N))
    env.rollout_expert(args.warmup)
    torch.cuda.synchronize()

    lanes = env.sim.rollout_lanes
    launches = env.sim.rollout_launches(args.steps)  # per lane (launch lengths within one of each other)
    # the sim launches on torch's current stream and forks its `lanes` concurrent env ranges from
    # it (each range: `launches` mmx_env_step_kernel launches of ~steps / launches env steps on its own stream, joined
    # back at the end): events on that stream bracket the K env steps of every range, so
    # kern_ms is the span over which one launch of each range (N envs in total) ran side by side
    stream = torch.cuda.current_stream(dev)
    cnt = [_lib.EPI[k] for k in ("episodes", "successes", "placed", "error_resets")]
    windows = []
    for _ in range(max(1, args.repeats)):
        env.clear_stats()
        epi0 = env._epi[:, cnt].sum(0).double()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        env.sim.kernel_timing(True)  # HIP event pair around every launch, on its own stream
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
        env.sim.kernel_timing(False)
        kt = env.sim.kernel_times()
        span_ms = ev0.elapsed_time(ev1) / launches  # the rollout's span per launch round
        # the step kernel's average launch duration (each launch: envs_per_launch envs x ~steps / launches steps)
        kern_ms = kt["step_ms"] / max(kt["step_launches"], 1)
        render_ms = kt["render_ms"] / kt["render_launches"] if kt["render_launches"] else None
        eps = (env._epi[:, cnt].sum(0).double() - epi0).tolist()
        errs_now = float((env.env_error != 0).sum().item())
        solver = env.solver_stats()
        if dist:
            t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            c = torch.tensor(eps + [errs_now], device=cdev, dtype=torch.float64)
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
            eps, errs_now = c[:4].tolist(), float(c[4].item())
            rk = torch.zeros(world, device=cdev, dtype=torch.float64)
            rk[rank] = kern_ms
            dist.all_reduce(rk, op=dist.ReduceOp.SUM)
            rank_kern_ms = rk.tolist()
        else:
            rank_kern_ms = [kern_ms]
        # SURVEY §8(e)'s logging collective, outside the timed region: every env's episode record
        # (return, length, counters, FSM phase; 16 B per env) gathered to rank 0
        rec = env_stats_record(env)
        gathered = gather_env_stats(rec if cdev.type == "cuda" else rec.cpu(), dist, world)
        env_summary = summarize_env_stats(gathered, world) if rank == 0 else None
        windows.append({"elapsed": elapsed, "kern_ms": kern_ms, "span_ms": span_ms, "render_ms": render_ms,
                        "launch_counts": [kt["step_launches"], kt["render_launches"]],
                        "rank_kernel_ms": rank_kern_ms, "solver": solver, "rank_envs": env_summary,
                        "episodes": {"completed": int(eps[0]), "successes": int(eps[1]), "placed": int(eps[2]),
                                     "error_resets": int(eps[3]), "envs_with_error_now": int(errs_now)}})
    isolated = None
    if args.image_size:
        # the render kernel on its own (no step kernels beside it): mmx_forward over the resident
        # states = the position stage (~0.04 ms for 8192 envs) + one render launch over all N envs
        env.sim.forward()
        torch.cuda.synchronize()
        reps = 10
        t1 = time.perf_counter()
        for _ in range(reps):
            env.sim.forward()
        torch.cuda.synchronize()
        fwd_ms = (time.perf_counter() - t1) / reps * 1e3
        isolated = {"forward_ms": fwd_ms, "envs": N,
                    "pixels_per_s": N * 2 * args.image_size ** 2 / (fwd_ms * 1e-3),
                    "note": "mmx_forward (position stage + render of all envs, both cameras) alone on the GPU"}
    values = [args.steps * N * world / w["elapsed"] for w in windows]
    med = windows[int(np.argsort(values)[len(values) // 2])]
    value = args.steps * N * world / med["elapsed"]
    solver, kern_ms = med["solver"], med["kern_ms"]
    # a launch round = `lanes` concurrent mmx_env_step_kernel dispatches of N / lanes envs x
    # steps / launches env steps each; they run side by side for the whole span, so a dispatch lasts ~kern_ms
    # (rocprof's per-dispatch average agrees) and the chip-level rate is lanes x one dispatch's
    # bytes / kern_ms.  nefc is the mean rows per substep counted on device in the same window.
    envs_per_launch = N / lanes
    # the lanes' launches differ in length (mmx_rollout_expert staggers them): the mean env steps per
    # launch from the window's launch count (every launch covers N / lanes envs)
    nlaunch = med["launch_counts"][0] or launches * lanes
    steps_per_launch = args.steps * lanes / nlaunch
    bpe = algorithmic_bytes_per_env_step(solver["mean_nefc"])
    bytes_per_launch = bpe * envs_per_launch * steps_per_launch
    achieved = lanes * bytes_per_launch / (kern_ms * 1e-3) / 1e9
    min_bytes = min_hbm_bytes_per_env_step() * envs_per_launch * steps_per_launch
    ep = med["episodes"]

    render = None
    if med["render_ms"]:
        # mmx_render_kernel: per env of a launch, 2 cameras x S^2 x (RGB + segment id) bytes written
        # and the 14 body poses read; one launch per rollout lane and env step, lanes side by side
        S = args.image_size
        # render launches per step: one over all envs after the step launch
        rl = max(1, env.sim.rollout_render_launches)
        r_envs = N / rl
        rbytes = r_envs * (2 * S * S * 4 + 14 * 12 * 4)
        r_achieved = rl * rbytes / (med["render_ms"] * 1e-3) / 1e9
        rpmc = pmc_evidence("render", N, lanes)
        # the default camera rollout renders step k on its own stream beside the step launch of step
        # k + 1 (mmx_rollout_render_overlap): kernel_ms is then the render launch's span on that
        # stream, shared with the step kernel; `isolated` is the render's own cost
        overlap = bool(env.sim.rollout_render_overlap)
        render = {"kernel": "mmx_render_kernel", "kernel_ms": med["render_ms"], "launches_per_step": rl,
                  "concurrent_with_step": overlap,
                  "envs_per_launch": r_envs, "image_size": S, "bytes_per_launch": rbytes,
                  "bound": None if rpmc is None else rpmc.get("valu", {}).get("bound"),
                  "hbm_achieved_GBs": r_achieved, "hbm_frac": r_achieved / HBM_PEAK_GBS,
                  "share_of_kernel_time": None if overlap else med["render_ms"] / (med["render_ms"] + kern_ms),
                  "pixels_per_s": rl * r_envs * 2 * S * S / (med["render_ms"] * 1e-3),
                  "valu": None if rpmc is None else rpmc.get("valu"), "isolated": isolated,
                  "note": "HBM is not the render kernel's roof (it writes 4 B per pixel); bound / valu: SQ counters "
                          "of tools/gpu.sh render_pmc for this configuration against the VALU issue calibration" +
                          ("; concurrent with the next step's launch: kernel_ms / pixels_per_s / hbm are "
                           "per span on the render stream, isolated.forward_ms is the render alone" if overlap else "")}
    if rank == 0:
        pmc = pmc_evidence(args.workload, N, lanes)
        traffic = None if pmc is None else pmc["hbm_bytes_per_env_step"] * envs_per_launch * steps_per_launch
        workload = (f"C2: PickPlaceGymEnv.step x {N} envs/GPU, fixed task (obj_red, bin_red), keyframe start (no "
                    "randomisation), staged reward, FSM expert abs_pos, autoreset" if c2 else
                    f"C3: PickPlaceGymEnv.step x {N} envs/GPU, tasks=all, randomize_objects, seed=42 episode seeds, "
                    "staged reward, FSM expert abs_pos, autoreset" if args.image_size == 0 else
                    f"C5: C3 settings x {N} envs/GPU plus overhead + wrist RGB {args.image_size}x{args.image_size} "
                    "camera images rendered every env step")
        line = {
            "metric": METRIC, "value": value, "unit": "env steps/s", "n_gpus": world,
            # distinct GPUs the ranks ran on: 1 for the --share-device rehearsal of the N-rank path
            "devices": 1 if args.share_device else world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * med["elapsed"] / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded randomized scenes, FSM-expert actions)",
            "config": {"workload": workload, "envs_per_gpu": N, "global_envs": N * world, "substeps": SUBSTEPS,
                       "step_kernel_lds_rows": env.sim.step_rows,
                       "image_size": args.image_size, "parallelism": f"env-batch dp{world}" + ("" if not args.share_device or world == 1
                                                                         else " (rehearsal: ranks share one GPU)")},
            "repeats": {"n": len(values), "values": values, "median_of": "value"},
            "physics_steps_per_s": SUBSTEPS * value,
            "episodes": {**ep, "placed_rate": ep["placed"] / max(ep["completed"], 1),
                         "note": "episodes that ended inside the median window (autoreset on FSM done / "
                                 "termination / truncation / divergence), summed over ranks; placed = target cube "
                                 "in the target bin at the episode's end; staged success needs the EE back at "
                                 "its start pose, which the expert's retreat target does not reach"},
            # the binding roof of the step kernel first (latency: VALU issue at ~0.38 of the calibrated
            # ceiling); the contract's HBM roofline object after it
            "bound": binding_roof(pmc, args.workload),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "mmx_env_step_kernel", "kernel_ms": kern_ms, "span_ms_per_launch_round": med["span_ms"],
                         "rank_kernel_ms": med["rank_kernel_ms"], "concurrent_launches": lanes,
                         "envs_per_launch": envs_per_launch, "env_steps_per_launch": steps_per_launch,
                         "algorithmic_bytes_per_env_step": bpe, "algorithmic_bytes_per_launch": bytes_per_launch,
                         "mean_nefc": solver["mean_nefc"],
                         "traffic_source": None if pmc is None else pmc.get("source"),
                         "min_hbm_bytes_per_launch": min_bytes,
                         "min_hbm_GBs": lanes * min_bytes / (kern_ms * 1e-3) / 1e9,
                         "binding": "no: the kernel keeps the efc working set in LDS, see `bound`"},
            "valu": None if pmc is None else pmc.get("valu"),
            "render": render,
            "cpu_baseline": cpu,
            "solver": solver,
            # per-rank summaries of the per-env episode records gathered to rank 0 after the median
            # window (all_gather_into_tensor over the default group: RCCL on N GPUs)
            "rank_envs": med["rank_envs"],
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
