"""Env-batch sharding across ranks (one process per GPU), SURVEY §8e.

Environments are independent units: rank r of R owns global envs [r * n, (r + 1) * n) of a job
with n envs per rank, and every env is seeded from its GLOBAL index (episode seed
SeedSequence(root).spawn(R * n)[g].generate_state(1)[0], scripts/generate_dataset.py:263-268), so
the trajectory of global env g does not depend on R.  There is no data-path collective; ranks
only combine logging counters (sum) and wall time (max), and at log intervals gather every env's
episode record (return, length, counters, FSM phase: 16 B per env) to rank 0.
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


# per-env episode record gathered for logging: [return (f32 bits), length, successes, fsm_state |
# placed << 8 | error_resets << 20] as int32, 16 B per env
ENV_STAT_FIELDS = ("return", "length", "successes", "fsm_state", "placed", "error_resets")


def env_stats_record(env):
    """The env batch's per-env episode record (int32 [N, 4], on the env's device): the running
    episode's return and length (gym_env.py:562-577 bookkeeping), the sticky success counter, and
    the FSM phase (pick_and_place.py:12-49) with the placed / error-reset counters packed beside it."""
    import torch

    from . import _lib

    epi = env._epi
    ret = env._epf[:, 27].contiguous().view(torch.int32)  # EPF_EP_RETURN
    packed = epi[:, _lib.EPI["fsm_state"]] | (epi[:, _lib.EPI["placed"]].clamp(0, 4095) << 8) | \
        (epi[:, _lib.EPI["error_resets"]].clamp(0, 2047) << 20)
    return torch.stack([ret, epi[:, _lib.EPI["step_count"]], epi[:, _lib.EPI["successes"]], packed], 1).contiguous()


def unpack_env_stats(rec):
    """int32 [n, 4] records -> dict of numpy arrays (ENV_STAT_FIELDS)."""
    import numpy as np

    r = np.asarray(rec.cpu() if hasattr(rec, "cpu") else rec, np.int32)
    return {"return": r[:, 0].view(np.float32).copy(), "length": r[:, 1].copy(), "successes": r[:, 2].copy(),
            "fsm_state": r[:, 3] & 0xFF, "placed": (r[:, 3] >> 8) & 0xFFF, "error_resets": (r[:, 3] >> 20) & 0x7FF}


def gather_env_stats(rec, dist=None, world: int = 1):
    """All ranks' records in global env order ([world * n, 4]; every rank receives them): one
    all_gather_into_tensor over the default process group (RCCL with device tensors; gloo takes
    host tensors).  Logging only, outside any timed region."""
    import torch

    if dist is None:
        return rec
    out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    dist.all_gather_into_tensor(out, rec)
    return out


def summarize_env_stats(rec, world: int = 1) -> list[dict]:
    """Per-rank summaries of gathered records (rank r = rows [r n, (r + 1) n))."""
    import numpy as np

    u = unpack_env_stats(rec)
    n = len(u["length"]) // world
    out = []
    for r in range(world):
        sl = slice(r * n, (r + 1) * n)
        out.append({"rank": r, "envs": n, "mean_return": float(u["return"][sl].mean()),
                    "mean_length": float(u["length"][sl].mean()), "successes": int(u["successes"][sl].sum()),
                    "placed": int(u["placed"][sl].sum()), "error_resets": int(u["error_resets"][sl].sum()),
                    "fsm_phase_hist": np.bincount(u["fsm_state"][sl], minlength=11).tolist()})
    return out
