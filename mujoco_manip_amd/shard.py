"""Env-batch sharding across ranks (one process per GPU), SURVEY §8e.

Environments are independent units: rank r of R owns global envs [r * n, (r + 1) * n) of a job
with n envs per rank, and every env is seeded from its GLOBAL index (episode seed
SeedSequence(root).spawn(R * n)[g].generate_state(1)[0], scripts/generate_dataset.py:263-268), so
the trajectory of global env g does not depend on R.  There is no data-path collective; ranks
only combine logging counters (sum) and wall time (max).
"""
from __future__ import annotations


def shard_range(rank: int, world: int, envs_per_rank: int) -> range:
    """Global env indices owned by `rank` (contiguous blocks of envs_per_rank)."""
    if not (0 <= rank < world) or envs_per_rank <= 0:
        raise ValueError(f"bad shard: rank {rank} of {world}, {envs_per_rank} envs per rank")
    return range(rank * envs_per_rank, (rank + 1) * envs_per_rank)


def shard_seeds(root: int, rank: int, world: int, envs_per_rank: int) -> list[int]:
    """Episode seeds of the envs `rank` owns, from their global indices."""
    from . import _lib

    return [_lib.episode_seed(root, g) for g in shard_range(rank, world, envs_per_rank)]


def dist_env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1 process when unset)."""
    import os

    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
