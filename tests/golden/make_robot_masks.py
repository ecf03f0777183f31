"""Generates tests/golden/robot_masks.npz: robot silhouettes of the reference's FULL Panda visual
meshes (VERDICT r02 "next" #4), the fidelity pin of the batched renderer's per-body hull model.

Run in the build container, where the reference's model files are readable (data, read as text /
binary; nothing of the reference is imported or executed):

    python tests/golden/make_robot_masks.py

What it computes, per state and camera (overhead, wrist; 128 x 128, MuJoCo's pinhole model of
cameras.py:56-104 and env.py:52-65: fovy, square image, row 0 at the top, pixel centres at +0.5):
  * every visual mesh of panda.xml:123-246 (all `class="visual"` geoms, OBJ files of the
    reference's assets/ directory, file coordinates = body frame: the geoms carry no pos / quat),
    posed with the fp64 oracle's body poses and z-buffered by a point-sampling rasteriser
    (perspective-correct depth, both faces: a silhouette does not depend on winding);
  * every non-robot triangle of the render model (table, bins, cubes, floor grid: boxes and
    prisms, exact geometry) z-buffered the same way;
  * mask = pixels whose nearest surface is the robot.
States: eight points of oracle FSM episodes (keyframe task (red, red) and C3 seeds), spread over
approach, grasp, lift, transport and release.  The file holds qpos [K, 30] and the masks
[K, 2, S, S] (uint8 0/1); np.load needs no pickle.
"""
from __future__ import annotations

import json
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tools"))

S = 128
ROBOT = ["link0", "link1", "link2", "link3", "link4", "link5", "link6", "link7", "hand", "left_finger",
         "right_finger"]


def load_obj_tris(path):
    """OBJ vertices and faces (fan-triangulated, 1-based / negative indices, v/vt/vn forms)."""
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                idx = []
                for tok in line.split()[1:]:
                    i = int(tok.split("/")[0])
                    idx.append(i - 1 if i > 0 else len(verts) + i)
                for k in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[k], idx[k + 1]])
    return np.asarray(verts, float), np.asarray(faces, np.int64)


def robot_meshes():
    """{body name: (verts [n, 3], tris [m, 3])} of all visual geoms of each Panda body."""
    import compile_model as CM

    panda = ET.parse(CM.PANDA).getroot()
    meshfile = {}
    for m in panda.find("asset").findall("mesh"):
        fname = m.get("file")
        meshfile[m.get("name", os.path.splitext(fname)[0])] = os.path.join(CM.REF_DATA, "franka_emika_panda", "assets",
                                                                           fname)
    out = {}

    def walk(be):
        name = be.get("name")
        if name in ROBOT:
            vs, ts, base = [], [], 0
            for ge in be.findall("geom"):
                if ge.get("class") != "visual":
                    continue
                assert ge.get("pos") is None and ge.get("quat") is None
                v, t = load_obj_tris(meshfile[ge.get("mesh")])
                vs.append(v)
                ts.append(t + base)
                base += len(v)
            out[name] = (np.concatenate(vs), np.concatenate(ts))
        for c in be.findall("body"):
            walk(c)

    for be in panda.find("worldbody").findall("body"):
        walk(be)
    return out


def raster_depth(tri_w, cR, cp, fovy, S=S, near=1e-3, chunk=40000):
    """Nearest depth per pixel of world triangles [T, 3, 3] (inf where none covers the centre)."""
    f = (S / 2.0) / np.tan(np.radians(fovy) / 2.0)
    z = np.full(S * S, np.inf)
    c = (tri_w - cp) @ cR  # camera frame
    d = -c[..., 2]
    keep = (d > near).all(1)
    c, d = c[keep], d[keep]
    sx = S / 2.0 + f * c[..., 0] / d
    sy = S / 2.0 - f * c[..., 1] / d
    iz = 1.0 / d
    x0 = np.clip(np.ceil(sx.min(1) - 0.5), 0, S).astype(np.int64)
    x1 = np.clip(np.floor(sx.max(1) - 0.5), -1, S - 1).astype(np.int64)
    y0 = np.clip(np.ceil(sy.min(1) - 0.5), 0, S).astype(np.int64)
    y1 = np.clip(np.floor(sy.max(1) - 0.5), -1, S - 1).astype(np.int64)
    w = np.maximum(x1 - x0 + 1, 0)
    h = np.maximum(y1 - y0 + 1, 0)
    area = (sx[:, 1] - sx[:, 0]) * (sy[:, 2] - sy[:, 0]) - (sx[:, 2] - sx[:, 0]) * (sy[:, 1] - sy[:, 0])
    ok = (w * h > 0) & (np.abs(area) > 1e-12)
    idx = np.nonzero(ok)[0]
    n = w * h
    # candidate pixels in chunks of triangles (bounded memory)
    start = 0
    while start < len(idx):
        sel = idx[start:start + 1]
        tot = n[sel[0]]
        k = start + 1
        while k < len(idx) and tot + n[idx[k]] <= 4_000_000 and k - start < chunk:
            tot += n[idx[k]]
            k += 1
        sel = idx[start:k]
        start = k
        cnt = n[sel]
        t = np.repeat(sel, cnt)
        off = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
        px = x0[t] + off % w[t]
        py = y0[t] + off // w[t]
        X, Y = px + 0.5, py + 0.5
        ax, ay, bx, by, cx_, cy_ = sx[t, 0], sy[t, 0], sx[t, 1], sy[t, 1], sx[t, 2], sy[t, 2]
        w0 = (bx - X) * (cy_ - Y) - (cx_ - X) * (by - Y)
        w1 = (cx_ - X) * (ay - Y) - (ax - X) * (cy_ - Y)
        w2 = (ax - X) * (by - Y) - (bx - X) * (ay - Y)
        inside = ((w0 >= 0) & (w1 >= 0) & (w2 >= 0)) | ((w0 <= 0) & (w1 <= 0) & (w2 <= 0))
        a = w0 + w1 + w2
        izp = (w0 * iz[t, 0] + w1 * iz[t, 1] + w2 * iz[t, 2]) / np.where(a == 0, 1, a)
        m = inside & (izp > 0)
        np.minimum.at(z, (py * S + px)[m], 1.0 / izp[m])
    return z.reshape(S, S)


def body_pose_fn(e):
    def pose(b):
        p, R = e.body(b)
        return R, p
    return pose


def states():
    """(qpos, body-pose function) of 8 oracle FSM states."""
    import oracle_py as O
    from mujoco_manip_amd.constants import BINS, OBJECTS, TASK_SETS

    pool = [(OBJECTS.index(o), BINS.index(b)) for o, b in TASK_SETS["all"]]
    out = []
    for seed, picks in ((None, (8, 20, 34, 52)), (O.episode_seed(42, 3), (14, 28, 44, 66))):
        e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=seed is not None, tasks=pool,
                        task=(0, 0) if seed is None else None)
        e.reset(seed=seed if seed is not None else 0)
        o, b = e.task()
        e.fsm_init([(o, b)])
        for t in range(max(picks) + 1):
            if t in picks:
                out.append(e.get_state()[0].copy())
            if e.fsm_plan(16) == 10:
                break
            f = e.fsm_get()
            e.step(np.array([*f["target"], float(f["gripper_open"])], np.float32))
    return out


def masks_for(qpos, meshes, rm, bnames):
    import oracle_py as O
    import render_ref as RR

    e = O.OracleEnv()
    e.set_state(qpos=np.asarray(qpos, float))
    e.mj_forward()
    pose = body_pose_fn(e)
    robot_w = []
    for name, (v, t) in meshes.items():
        R, p = pose(bnames.index(name))
        robot_w.append((v @ R.T + p)[t])
    robot_w = np.concatenate(robot_w)
    seg = np.array([rm["materials"][k]["seg"] for k in rm["tri_mat"]])
    V = np.array(rm["verts"], float)
    vb = np.array(rm["vert_body"])
    Vw = np.empty_like(V)
    for b in np.unique(vb):
        R, p = pose(int(b))
        Vw[vb == b] = V[vb == b] @ np.asarray(R).T + p
    tris = np.array(rm["tris"])
    scene_w = Vw[tris[seg != 9]]
    out = []
    for cam in ("overhead", "wrist"):
        cR, cp = RR.camera_pose(cam, pose)
        fovy = [c for c in rm["cameras"] if c["name"] == cam][0]["fovy"]
        zr = raster_depth(robot_w, cR, cp, fovy)
        zs = raster_depth(scene_w, cR, cp, fovy)
        out.append((zr < zs).astype(np.uint8))
    return np.stack(out)


def main():
    import compile_model as CM

    meshes = robot_meshes()
    ntri = sum(len(t) for _, t in meshes.values())
    rm = json.load(open(os.path.join(REPO, "mujoco_manip_amd", "model", "render_model.json")))
    bnames = [b["name"] for b in CM.compile_model()["bodies"]]
    qs = states()
    masks = np.stack([masks_for(q, meshes, rm, bnames) for q in qs])
    np.savez_compressed(os.path.join(HERE, "robot_masks.npz"), qpos=np.stack(qs), masks=masks, size=np.int64(S),
                        visual_triangles=np.int64(ntri))
    print(f"{len(qs)} states, {ntri} visual triangles, robot pixels per image "
          f"{masks.reshape(len(qs), 2, -1).sum(-1).tolist()}")


if __name__ == "__main__":
    main()
