"""Multi-process (world_size 2) checks of the env-batch sharding bench.py uses on N GPUs.

Envs shard embarrassingly: rank r owns global envs [r*n, (r+1)*n)
(mujoco_manip_amd.shard), each seeded from its GLOBAL index, so trajectories do not depend on the
number of ranks.  The only collectives are logging ones (all_gather / all_reduce(SUM) of
counters, all_reduce(MAX) of wall time).
  * CPU (gloo): each rank steps its shard with the oracle; the gathered result equals a
    single-process run.
  * GPU: two fresh rank processes share device 0 (gloo between them) and run the HIP rollout on
    their shards; the gathered per-env results are bit-equal to one process with all 2n envs.
"""
import subprocess
import sys
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_GLOBAL = 4
STEPS = 3


def shard_rollout(env_ids):
    import oracle_py as O

    out = []
    for g in env_ids:
        e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=True)
        e.reset(seed=O.episode_seed(42, g))
        o, b = e.task()
        e.fsm_init([(o, b)])
        for _ in range(STEPS):
            e.fsm_plan(16)
            f = e.fsm_get()
            e.step(np.array([*f["target"], float(f["gripper_open"])], np.float32))
        out.append(np.concatenate([e.get_state()[0], [o, b]]))
    return np.stack(out)


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mujoco_manip_amd.shard import shard_range

    local = torch.tensor(shard_rollout(shard_range(rank, world, N_GLOBAL // world)))
    gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((torch.cat(gathered).numpy(), float(t.item())))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_sharding_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, tmax = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert tmax == 2.0
    single = shard_rollout(range(N_GLOBAL))
    np.testing.assert_array_equal(gathered, single)


def _stats_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mujoco_manip_amd.shard import gather_env_stats, summarize_env_stats

    local = _synthetic_records(range(rank * 3, rank * 3 + 3))
    got = gather_env_stats(local, dist, world)
    if rank == 0:
        q.put((got.numpy(), summarize_env_stats(got, world)))
    dist.destroy_process_group()


def _synthetic_records(env_ids):
    """Per-env episode records as env_stats_record packs them, a function of the global env id."""
    rows = []
    for g in env_ids:
        ret = np.array([0.25 * g - 1.0], np.float32).view(np.int32)[0]
        rows.append([ret, 10 + g, g % 2, (g % 11) | ((g % 3) << 8) | ((g % 2) << 20)])
    return torch.tensor(rows, dtype=torch.int32)


def test_two_rank_env_stats_gather_matches_single_process():
    """SURVEY §8(e)'s logging collective: the per-env episode records (16 B per env) gathered to
    rank 0 over the default group equal one process's records, and the per-rank summaries follow."""
    from mujoco_manip_amd.shard import summarize_env_stats, unpack_env_stats

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, summ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    single = _synthetic_records(range(6))
    np.testing.assert_array_equal(got, single.numpy())
    u = unpack_env_stats(single)
    assert summ[1]["successes"] == int(u["successes"][3:].sum()) and summ[0]["envs"] == 3
    assert summ == summarize_env_stats(single, 2)
    assert abs(summ[0]["mean_return"] - np.mean([-1.0, -0.75, -0.5])) < 1e-7
    assert sum(summ[0]["fsm_phase_hist"]) == 3 and summ[1]["placed"] == sum(g % 3 for g in range(3, 6))


def test_shard_ranges_and_seeds():
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.shard import shard_range, shard_seeds

    assert list(shard_range(0, 2, 3)) == [0, 1, 2] and list(shard_range(1, 2, 3)) == [3, 4, 5]
    assert shard_seeds(42, 1, 4, 2) == [_lib.episode_seed(42, 2), _lib.episode_seed(42, 3)]
    all8 = sum((shard_seeds(42, r, 4, 2) for r in range(4)), [])
    assert all8 == [_lib.episode_seed(42, g) for g in range(8)]  # independent of the rank count
    with pytest.raises(ValueError):
        shard_range(2, 2, 3)


def test_bench_rejects_mismatched_world(monkeypatch):
    """bench.py --gpus N under a torchrun world of another size is an error, not a silent 1-GPU run."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_launcher_stops_peers_when_a_rank_dies():
    """bench.py's own rank launcher (--gpus N without torchrun): rank 1 exits with 3 at once while
    rank 0 would block (as in a collective waiting for the dead peer) for 120 s; the parent must
    terminate rank 0 and return the failing rank's code well within the block."""
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(120)\n")
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, cmd=[sys.executable, "-c", code], grace_s=5.0)
    assert rc == 3
    assert time.monotonic() - t0 < 30.0
    t0 = time.monotonic()
    assert bench.launch_ranks(2, cmd=[sys.executable, "-c", "pass"]) == 0
    assert time.monotonic() - t0 < 30.0


@pytest.mark.gpu
def test_two_rank_hip_rollout_matches_single_process(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    n, steps = 12, 48
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "ranks.npz")
    port = str(_free_port())
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "dist_rollout_worker.py"), str(n), str(steps), out],
                              env=dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port)) for r in range(2)]
    assert [p.wait(timeout=240) for p in procs] == [0, 0]
    ranks, stats = np.load(out)["rows"], np.load(out)["stats"]
    env = PickPlaceVecEnv(2 * n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=0, autoreset=True)
    env.reset(seed=[_lib.episode_seed(42, g) for g in range(2 * n)])
    env.rollout_expert(steps)
    torch.cuda.synchronize()
    q, v, _, _ = env.sim.get_state()
    epi = env.sim.view("episode_i", _lib.EPI_N, "<i4").cpu().numpy()
    np.testing.assert_array_equal(ranks, np.concatenate([q, v, epi.view(np.float32)], 1))
    from mujoco_manip_amd.shard import env_stats_record

    np.testing.assert_array_equal(stats, env_stats_record(env).cpu().numpy())  # §8(e) gather


@pytest.mark.gpu
def test_rccl_path_single_rank_torchrun():
    """bench.py under torchrun with one rank: the process group is RCCL (the `nccl` backend) and
    the line comes out of the RCCL branch (barriers, all_reduce of the window time and counters,
    all_gather_into_tensor of the per-env records on device tensors); the 8-GPU scaling runs use
    the same branch.  (Two ranks cannot share one GPU under RCCL, so the 1-GPU box tests N = 1.)"""
    import json

    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(repo, "bench.py"), "--gpus", "1", "--steps", "32", "--warmup", "8",
                        "--repeats", "2", "--no-cpu-baseline", "--dist-backend", "nccl"],
                       capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["rank_envs"][0]["envs"] == 4096 and sum(line["rank_envs"][0]["fsm_phase_hist"]) == 4096
