"""Geometry for the collision known-answer tests (tests/test_collision_kat.py): test
infrastructure, independent of both implementations under test.

  * forward kinematics straight from the raw MJCF attributes (tests/golden/mjcf_raw.json, written
    by make_mjcf_fixture.py from panda.xml / pick_and_place_scene.xml, not by tools/compile_model.py);
  * the Panda's collision hulls from the raw STL / OBJ assets (tests/golden/collision_hulls.npz,
    make_collision_hulls.py);
  * exact penetration of two convex sets: the Minkowski difference A - B as a qhull hull; with the
    origin inside, the penetration depth is the distance from the origin to its nearest facet and
    the contact normal that facet's outward normal (translating B by depth * n separates the two).

MuJoCo's conventions restated here (documentation, "Computation / Collision detection"): a contact's
`dist` is the signed distance (negative = penetration), its frame's first row the normal from geom1
to geom2, geom1 the geom of the lower type (plane < cylinder < box < mesh), its position midway
between the two surfaces.
"""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

GT = {"plane": 0, "cylinder": 5, "box": 6, "mesh": 7}
ARM = ["joint1", "joint2", "joint3", "joint4", "joint5", "joint6", "joint7", "finger_joint1", "finger_joint2"]
CUBES = ["obj_red", "obj_green", "obj_blue"]
TABLE_TOP = 0.24


def quat2mat(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def mat2quat(R):
    w = np.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.copysign(np.sqrt(max(0.0, 1.0 + R[0, 0] - R[1, 1] - R[2, 2])) / 2, R[2, 1] - R[1, 2])
    y = np.copysign(np.sqrt(max(0.0, 1.0 - R[0, 0] + R[1, 1] - R[2, 2])) / 2, R[0, 2] - R[2, 0])
    z = np.copysign(np.sqrt(max(0.0, 1.0 - R[0, 0] - R[1, 1] + R[2, 2])) / 2, R[1, 0] - R[0, 1])
    q = np.array([w, x, y, z])
    return q / np.linalg.norm(q)


def axis_rot(axis, ang):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


class RawModel:
    """The scene as the MJCF states it: bodies, joints, collision geoms, hull vertices."""

    def __init__(self):
        raw = json.load(open(os.path.join(GOLDEN, "mjcf_raw.json")))
        self.bodies = raw["bodies"]
        self.key_qpos = np.array(raw["key_qpos"], float)
        hulls = np.load(os.path.join(GOLDEN, "collision_hulls.npz"))
        self.hulls = {str(n): hulls[str(n)] for n in hulls["meshes"]}
        # qpos addresses: the arm's 9 scalar joints, then one free joint (7) per cube
        self.qadr = {j: k for k, j in enumerate(ARM)}
        for k, c in enumerate(CUBES):
            self.qadr[c + "_jnt"] = 9 + 7 * k
        # geoms in MJCF order per body; world geoms (the floor) first
        self.geoms = [dict(body="world", type="plane", size=[2.0, 2.0, 0.01], pos=[0, 0, 0], name="floor")]
        for bname, b in self._body_order():
            for g in b["geoms"]:
                self.geoms.append(dict(g, body=bname))

    def _body_order(self):
        out, seen = [], {"world"}
        while len(out) < len(self.bodies):
            for n, b in self.bodies.items():
                if n not in seen and b["parent"] in seen:
                    out.append((n, b))
                    seen.add(n)
        return out

    def fk(self, qpos):
        """World pose (p, R) of every body at qpos (MuJoCo's joint conventions: hinge / slide about
        the body frame axis through the body origin, free joint = world position + quaternion)."""
        pose = {"world": (np.zeros(3), np.eye(3))}
        for n, b in self._body_order():
            pp, PR = pose[b["parent"]]
            p = pp + PR @ np.asarray(b["pos"], float)
            R = PR @ quat2mat(b["quat"])
            for j in b["joints"]:
                a = self.qadr[j["name"]]
                if j["type"] == "hinge":
                    R = R @ axis_rot(j["axis"], qpos[a])
                elif j["type"] == "slide":
                    p = p + R @ np.asarray(j["axis"], float) * qpos[a]
                elif j["type"] == "free":
                    p = np.asarray(qpos[a:a + 3], float)
                    R = quat2mat(qpos[a + 3:a + 7])
            pose[n] = (p, R)
        return pose

    def geom_points(self, g, pose):
        """A convex geom as a point set whose hull is the geom (boxes: 8 corners; hull meshes:
        their vertices), in world coordinates."""
        p, R = pose[g["body"]]
        if g["type"] == "box":
            h = np.asarray(g["size"], float)
            c = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * h
            return p + (R @ (np.asarray(g["pos"], float) + c).T).T
        if g["type"] == "mesh":
            return p + (R @ self.hulls[g["mesh"]].T).T
        raise ValueError(g["type"])

    def find(self, body, type_, k=0):
        """Index into self.geoms of the k-th geom of `type_` on `body`."""
        ids = [i for i, g in enumerate(self.geoms) if g["body"] == body and g["type"] == type_]
        return ids[k]


def penetration(A, B):
    """Exact penetration of hull(A) and hull(B) (point sets, world frame).

    Returns (depth, normal A->B, facets) with depth > 0 when they overlap: the origin's distance
    to the nearest facet of hull(A - B); `facets` = [(distance, normal, witness A, witness B)] of
    all facets sorted by distance, witnesses = the barycentric combination of the facet's A and B
    points at the origin's projection."""
    from scipy.spatial import ConvexHull

    A = np.asarray(A, float)
    B = np.asarray(B, float)
    ia, ib = np.meshgrid(np.arange(len(A)), np.arange(len(B)), indexing="ij")
    ia, ib = ia.ravel(), ib.ravel()
    M = A[ia] - B[ib]
    h = ConvexHull(M)
    dist = -h.equations[:, 3]  # outward unit normal n, n.x + off <= 0 inside: distance = -off
    order = np.argsort(dist)
    facets = []
    for f in order:
        n = h.equations[f, :3]
        tri = h.simplices[f]
        P = M[tri]
        x = n * dist[f]
        # barycentric coordinates of x in the facet triangle
        T = np.stack([P[1] - P[0], P[2] - P[0]], axis=1)
        lam12 = np.linalg.lstsq(T, x - P[0], rcond=None)[0]
        lam = np.r_[1 - lam12.sum(), lam12]
        wa = lam @ A[ia[tri]]
        wb = lam @ B[ib[tri]]
        facets.append((float(dist[f]), n.copy(), wa, wb, set(ia[tri].tolist()), set(ib[tri].tolist())))
    return facets[0][0], facets[0][1], facets


def feature_summary(facets, tol=1e-9):
    """The nearest facets (within tol of the minimum, same normal): the A and B point indices
    they span, so a single A index = a vertex-face contact whose witness is unique."""
    d0, n0 = facets[0][0], facets[0][1]
    ia, ib = set(), set()
    for d, n, _, _, sa, sb in facets:
        if d > d0 + tol:
            break
        if np.dot(n, n0) > 1 - 1e-9:
            ia |= sa
            ib |= sb
    return ia, ib


def normal_margin(facets, ang=1e-3):
    """Distance gap from the nearest facet to the nearest facet with a different normal: the
    EPA answer's normal is well defined when this is large against its tolerance."""
    d0, n0 = facets[0][0], facets[0][1]
    for d, n, *_ in facets[1:]:
        if np.dot(n, n0) < np.cos(ang):
            return d - d0
    return np.inf
