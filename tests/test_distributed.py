"""Multi-process (gloo, world_size 2) check of the env-batch sharding used by bench.py on N GPUs.

Envs shard embarrassingly: rank r owns global envs [r*n, (r+1)*n), each seeded
from its GLOBAL index, so trajectories do not depend on the number of ranks.  The only
collectives are logging ones (all_gather of per-env stats, all_reduce(MAX) of wall time).
Here each rank steps its shard with the CPU oracle and the gathered result must equal a
single-process run.
"""
import os
import socket

import numpy as np
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
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = N_GLOBAL // world
    local = torch.tensor(shard_rollout(range(rank * n, (rank + 1) * n)))
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
