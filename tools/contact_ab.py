"""Contact-list A/B of two builds on the same states (experiment infrastructure).

  MMX_LIB_PATH=build/libmmx_base.so python tools/contact_ab.py gen   # states + base contacts
  python tools/contact_ab.py cmp                                     # working-tree contacts, diff

`gen` rolls the C3 expert out and snapshots the state every 10 steps; each snapshot is re-set and
run through one substep (mj_step stores its contact list), and the list is saved.  `cmp` sets the same states in the other
build and reports per field how many contacts differ (bit for bit) and by how much.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mujoco_manip_amd import _lib  # noqa: E402

OUT = os.path.join(REPO, "gpurun_out", "contact_ab.npz")
N = 2048


def contacts(sim):
    torch.cuda.synchronize()
    c = sim.view("contacts", _lib.MAXCON * _lib.CON_F).cpu().numpy().reshape(N, _lib.MAXCON, _lib.CON_F)
    ncon = sim.view("episode_i", _lib.EPI_N, "<i4")[:, _lib.EPI["ncon"]].cpu().numpy()
    c[np.arange(_lib.MAXCON)[None, :] >= ncon[:, None]] = 0.0  # stale slots past the list
    return c


def main():
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          autoreset=True)
    env.reset(seed=[_lib.episode_seed(42, i) for i in range(N)])
    if sys.argv[1] == "gen":
        snaps = []
        for k in range(12):
            env.rollout_expert(10)
            torch.cuda.synchronize()
            snaps.append(env.sim.get_state())
        qs = np.stack([s[0] for s in snaps]); vs = np.stack([s[1] for s in snaps])
        cs = np.stack([s[2] for s in snaps]); ws = np.stack([s[3] for s in snaps])
    else:
        z = np.load(OUT)
        qs, vs, cs, ws = z["qpos"], z["qvel"], z["ctrl"], z["ws"]
    con = []
    for k in range(len(qs)):
        env.sim.set_state(qs[k], vs[k], cs[k], ws[k])
        env.sim.physics_step(1)  # stores the substep's contact list and ncon
        con.append(contacts(env.sim))
    con = np.stack(con)
    if sys.argv[1] == "gen":
        np.savez_compressed(OUT, qpos=qs, qvel=vs, ctrl=cs, ws=ws, con=con)
        print("saved", con.shape)
        return
    base = np.load(OUT)["con"]
    rep = {}
    names = ["dist", "px", "py", "pz", "nx", "ny", "nz", "mu0", "mu1", "mu2", "dim", "g1", "g2"]
    for f in range(_lib.CON_F):
        a, b = base[..., f], con[..., f]
        diff = a.view(np.uint32) != b.view(np.uint32)
        rep[names[f] if f < len(names) else str(f)] = {"n_diff": int(diff.sum()),
                                                       "max_abs": float(np.abs(a - b)[diff].max()) if diff.any() else 0.0}
    same_env = (base.view(np.uint32) == con.view(np.uint32)).all(axis=(2, 3))
    rep["envs_identical_frac"] = float(same_env.mean())
    bad = np.argwhere(~same_env)
    if len(bad):
        k, e = bad[0]
        rep["first_diff"] = {"snap": int(k), "env": int(e), "base": base[k, e, :8].tolist(), "new": con[k, e, :8].tolist()}
    print(json.dumps(rep, indent=1))
    json.dump(rep, open(os.path.join(REPO, "gpurun_out", "contact_ab.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
