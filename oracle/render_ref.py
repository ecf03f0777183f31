"""CPU ray-cast checker for the batched camera renderer (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module; the product path never does.

The reference renders with MuJoCo's OpenGL renderer (`mujoco.Renderer`, cameras.py:9-53), which
is absent here, and pixels of a different rasterizer cannot match OpenGL's anyway.
What this checker pins is the geometry of the images at mask level: for every pixel it casts
the camera ray of MuJoCo's pinhole model (fovy, square image, row 0 at the top, pixel centres at
+0.5; cameras.py:56-104 for the intrinsics, env.py:52-65 for the wrist camera) against the same
triangle model (mujoco_manip_amd/model/render_model.json, built by tools/compile_render.py from
the reference's MJCF and meshes) posed with the fp64 oracle's body poses, and returns the
segment id of the nearest front face.  Möller-Trumbore intersection, vectorised over all
triangles per pixel row in numpy.
"""
from __future__ import annotations

import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_MODEL = None


def model():
    global _MODEL
    if _MODEL is None:
        with open(os.path.join(REPO, "mujoco_manip_amd", "model", "render_model.json")) as f:
            m = json.load(f)
        m["verts"] = np.array(m["verts"], float)
        m["vert_body"] = np.array(m["vert_body"], int)
        m["tris"] = np.array(m["tris"], int)
        m["tri_mat"] = np.array(m["tri_mat"], int)
        m["tri_seg"] = np.array([m["materials"][k]["seg"] for k in m["tri_mat"]], np.uint8)
        _MODEL = m
    return _MODEL


def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def camera_pose(name, body_pose):
    """World (R, p) of camera `name` given body_pose(bid) -> (R, p)."""
    cam = [c for c in model()["cameras"] if c["name"] == name][0]
    R = quat2mat(cam["quat"])
    p = np.array(cam["pos"], float)
    if cam["body"] != 0:
        bR, bp = body_pose(cam["body"])
        return bR @ R, bp + bR @ p
    return R, p


def render_seg(body_pose, cam_name: str, S: int):
    """Segment ids [S, S] (uint8) of camera `cam_name`; body_pose(bid) -> (R [3,3], p [3])."""
    m = model()
    V = np.empty_like(m["verts"])
    for b in np.unique(m["vert_body"]):
        R, p = body_pose(int(b))
        sel = m["vert_body"] == b
        V[sel] = m["verts"][sel] @ np.asarray(R).T + p
    cR, cp = camera_pose(cam_name, body_pose)
    fovy = [c for c in m["cameras"] if c["name"] == cam_name][0]["fovy"]
    f = (S / 2.0) / np.tan(np.radians(fovy) / 2.0)
    A, B, C = V[m["tris"][:, 0]], V[m["tris"][:, 1]], V[m["tris"][:, 2]]
    e1, e2 = B - A, C - A
    n = np.cross(e1, e2)
    seg = np.zeros((S, S), np.uint8)
    cols = (np.arange(S) + 0.5 - S / 2.0) / f
    for r in range(S):
        y = -(r + 0.5 - S / 2.0) / f
        d_cam = np.stack([cols, np.full(S, y), -np.ones(S)], 1)  # rays of this row, camera frame
        D = d_cam @ cR.T                                            # world directions [S, 3]
        # front faces only (outward normal against the ray), like the rasterizer's back-face cull
        pvec = np.cross(D[:, None, :], e2[None, :, :])              # [S, T, 3]
        det = np.einsum("tk,stk->st", e1, pvec)
        inv = 1.0 / np.where(np.abs(det) < 1e-18, np.inf, det)
        tvec = cp[None, :] - A                                      # [T, 3]
        u = np.einsum("tk,stk->st", tvec, pvec) * inv
        qvec = np.cross(tvec, e1)                                   # [T, 3]
        v = np.einsum("sk,tk->st", D, qvec) * inv
        t = np.einsum("tk,tk->t", e2, qvec)[None, :] * inv
        front = np.einsum("sk,tk->st", D, n) < 0
        hit = front & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 1e-6)
        t = np.where(hit, t, np.inf)
        k = np.argmin(t, axis=1)
        ok = np.isfinite(t[np.arange(S), k])
        seg[r] = np.where(ok, m["tri_seg"][k], 0)
    return seg
