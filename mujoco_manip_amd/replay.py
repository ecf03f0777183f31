"""Batched replay / parity tool.

Mirrors `scripts/replay_actions.py` of the reference (main :14-161): read an episode's recorded
actions, restore the episode's object randomisation and task from `metadata.json`
(:74-100), build the env with the action mode named by the action key
(`action.ee.pos_quat_g` -> `ee_pos_quat_g`, :70-72), reset, step through the actions and report
per frame the decoded target, the EE position and their distance (:128-148).

MI355X-first difference: every requested episode is replayed at once, one env per episode, so a
whole dataset is checked in one batched pass; the viewer / slow-motion options of the reference
are out of scope (no UI). `replay()` returns the per-frame report as arrays; `main()` prints the
reference's table for one episode and a per-episode summary for all of them.
"""
from __future__ import annotations

import argparse
import os

import numpy as np

from .constants import BINS, OBJECTS, TASK_SETS
from .dataset import read_lerobot_v3

ACTION_MODES = ("ee_pos_quat_g", "ee_pos_rot6d_g", "ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel")


def decode_targets(mode: str, actions, T_init):
    """decode_action (gym_env.py:252-281) batched in torch: world target positions [n, 3].

    Absolute modes take the action's position; relative modes T_init @ T_rel, of which only the
    translation is used (R_init p_rel + p_init)."""
    import torch

    a = actions.to(torch.float64)
    if mode in ("ee_pos_quat_g", "ee_pos_rot6d_g", "abs_pos"):
        return a[:, :3]
    T = T_init.to(torch.float64)
    return (T[:, :3, :3] @ a[:, :3, None])[:, :, 0] + T[:, :3, 3]


def episode_setup(metadata, episode_index: int):
    """replay_actions.py:74-100: (seed or None, (obj, bin) or None, spawn_x, spawn_y).  A shard of a
    sharded generation (dataset.generate with world_size > 1) numbers its episodes locally: the
    global index its seed and task belong to is in metadata["shard"]."""
    spawn_x, spawn_y = (-0.20, 0.20), (0.30, 0.45)
    seed, task = None, None
    if metadata is not None and "shard" in metadata:
        episode_index = int(metadata["shard"]["global_episode_index"][episode_index])
    if metadata is not None:
        seeds = metadata.get("episode_seeds")
        if seeds and episode_index < len(seeds):
            seed = int(seeds[episode_index])
        if "spawn_x_range" in metadata:
            spawn_x = tuple(metadata["spawn_x_range"])
        if "spawn_y_range" in metadata:
            spawn_y = tuple(metadata["spawn_y_range"])
        mt, mts = metadata.get("task"), metadata.get("tasks", "all")
        if mt is not None:
            task_list = [tuple(mt)]
        elif mts in TASK_SETS:
            task_list = TASK_SETS[mts]
        else:
            task_list = TASK_SETS["all"]
        task = task_list[episode_index % len(task_list)]
    return seed, task, spawn_x, spawn_y


def replay(dataset_root: str, episodes=None, action_key: str = "action.ee.pos_quat_g", device: int = 0):
    """Replay the recorded actions of `episodes` (default: all) in one batch.

    Returns dict with per-episode lists: target [T, 3], ee [T, 3], err [T], obs_state [T, 11]
    (the post-step observation.state), plus the episodes' recorded frames for comparison."""
    import torch

    from .vec_env import PickPlaceVecEnv

    info, metadata, frames = read_lerobot_v3(dataset_root)
    ids = sorted(frames) if episodes is None else list(episodes)
    missing = [e for e in ids if e not in frames]
    if missing:
        raise ValueError(f"episodes {missing} not in the dataset")
    if action_key not in frames[ids[0]]:
        avail = [k for k in frames[ids[0]] if k.startswith("action.")]
        raise ValueError(f"'{action_key}' not found. Available: {avail}")
    mode = action_key.replace("action.", "").replace(".", "_")
    if mode not in ACTION_MODES:
        raise ValueError(f"action key {action_key} does not name an action mode")
    setups = [episode_setup(metadata, e) for e in ids]
    randomize = any(s[0] is not None for s in setups)
    sx, sy = setups[0][2], setups[0][3]
    n = len(ids)
    env = PickPlaceVecEnv(n, action_mode=mode, reward_type="staged", randomize_objects=randomize,
                          spawn_x_range=sx, spawn_y_range=sy, autoreset=False, image_size=0, device=device)
    task = None
    if all(s[1] is not None for s in setups):
        task = [s[1] for s in setups]
    env.reset(seed=[s[0] for s in setups] if randomize else None, options={"task": task} if task else None)
    T_init = env.initial_ee_se3
    lengths = np.array([len(frames[e][action_key]) for e in ids])
    T_max = int(lengths.max())
    dim = frames[ids[0]][action_key].shape[1]
    acts = np.zeros((T_max, n, dim), np.float32)
    for j, e in enumerate(ids):
        a = frames[e][action_key]
        acts[:len(a), j] = a
        acts[len(a):, j] = a[-1]  # finished episodes hold their last action (not reported)
    acts_d = torch.as_tensor(acts, device=env.device)
    tgt, ee, st = [], [], []
    for t in range(T_max):
        obs, *_ = env.step(acts_d[t])
        tgt.append(decode_targets(mode, acts_d[t], T_init))
        ee.append(obs["state"][:, :3].to(torch.float64))
        st.append(obs["state"])
    tgt = torch.stack(tgt).cpu().numpy()
    ee = torch.stack(ee).cpu().numpy()
    st = torch.stack(st).cpu().numpy()
    env.close()
    out = {"episodes": ids, "mode": mode, "target": [], "ee": [], "err": [], "obs_state": [], "frames": frames}
    for j, e in enumerate(ids):
        L = lengths[j]
        out["target"].append(tgt[:L, j])
        out["ee"].append(ee[:L, j])
        out["err"].append(np.linalg.norm(ee[:L, j] - tgt[:L, j], axis=1))
        out["obs_state"].append(st[:L, j])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="Replay dataset actions on the MI355X (batched over episodes)")
    ap.add_argument("--repo-id", required=True)
    ap.add_argument("--root", default="./datasets")
    ap.add_argument("--episode-index", type=int, nargs="*", default=[0],
                    help="episodes to replay (-1 = all); the first one is printed frame by frame")
    ap.add_argument("--action-key", default="action.ee.pos_quat_g")
    a = ap.parse_args(argv)
    root = os.path.join(a.root, a.repo_id)
    eps = None if a.episode_index == [-1] else a.episode_index
    r = replay(root, eps, a.action_key)
    e0 = r["episodes"][0]
    print(f"Loaded episode {e0}: {len(r['err'][0])} frames; action key {a.action_key} -> mode {r['mode']}")
    print(f"{'Frame':>6}  {'Action XYZ':>30}  {'EE XYZ':>30}  {'Error':>8}")
    print("-" * 82)
    for i, (t, p, d) in enumerate(zip(r["target"][0], r["ee"][0], r["err"][0])):
        print(f"{i:>6}  {t[0]:>9.4f} {t[1]:>9.4f} {t[2]:>9.4f}  {p[0]:>9.4f} {p[1]:>9.4f} {p[2]:>9.4f}  {d:>8.4f}")
    print("\nper-episode EE tracking error (m): episode, frames, mean, max")
    for e, err in zip(r["episodes"], r["err"]):
        print(f"{e:>6} {len(err):>6} {err.mean():>9.4f} {err.max():>9.4f}")


if __name__ == "__main__":
    main()
