"""Rank process of the multi-process GPU test (tests/test_distributed.py::test_two_rank_hip_rollout...):
one rank of a C3 rollout over the HIP path (bench.py's sharding), results gathered to rank 0 over
gloo and saved.  Run as: RANK=r WORLD_SIZE=R MASTER_ADDR=127.0.0.1 MASTER_PORT=p python
tests/dist_rollout_worker.py <envs_per_rank> <env_steps> <out.npz>."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    n, steps, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.shard import dist_env, env_stats_record, gather_env_stats, shard_seeds
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    rank, _, world = dist_env()
    dist.init_process_group("gloo")
    env = PickPlaceVecEnv(n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=0, autoreset=True, device=0)  # the ranks share the 1-GPU box's device
    env.reset(seed=shard_seeds(42, rank, world, n))
    env.rollout_expert(steps)
    torch.cuda.synchronize()
    q, v, _, _ = env.sim.get_state()
    epi = env.sim.view("episode_i", _lib.EPI_N, "<i4").cpu().numpy()
    local = torch.from_numpy(np.concatenate([q, v, epi.view(np.float32)], 1))
    gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    stats = gather_env_stats(env_stats_record(env).cpu(), dist, world)  # the bench's logging gather
    if rank == 0:
        np.savez(out, rows=torch.cat(gathered).numpy(), stats=stats.numpy())
    dist.destroy_process_group()
    env.close()


if __name__ == "__main__":
    main()
