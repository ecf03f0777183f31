"""Generates tests/golden/collision_scenes.json: the INPUTS (arm configurations, cube poses) of the
mesh known-answer scenes in tests/test_collision_kat.py.  The answers are not stored: the test
derives them at run time from geometry alone (tests/collision_geometry.py: raw-MJCF kinematics,
hulls of the raw mesh assets, exact Minkowski-difference penetration).

    python tests/golden/make_collision_scenes.py

Needs only the committed fixtures (mjcf_raw.json, collision_hulls.npz), not the reference.
Two scene families, each with a single touching pair so the contact it must produce is known:

  * hull vs tabletop: a seeded random search over the arm's joint ranges; joint 2 is then bisected
    until the target hull's lowest point over the tabletop sits `depth` below its surface
    (z = 0.24); kept when no other robot geom touches the table (for the finger: at most its own
    pads, which sit inside the fingertip), the nearest facet of the
    Minkowski difference is the tabletop's top face (depth = that lowest point's depth, normal
    -z) and the next facet with another normal is >= 0.5 mm farther;
  * cube vs hull (arm at a fixed configuration above the table): the cube's face is pressed
    `depth` into the hull along a direction u where the hull's support vertex is unique
    (the next vertex >= depth + 0.5 mm behind it), the cube turned about u and shifted sideways
    so the vertex meets its face off-centre, or, where no such direction turns up, flat onto one
    of the hull's large facets (a face-face contact: depth and normal known, position not unique);
    kept when nothing else touches the cube (for the finger: at most its own pads).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from collision_geometry import ARM, RawModel, axis_rot, feature_summary, mat2quat, normal_margin, penetration  # noqa: E402

RANGES = [(-2.8973, 2.8973), (-1.7628, 1.7628), (-2.8973, 2.8973), (-3.0718, -0.0698), (-2.8973, 2.8973),
          (-0.0175, 3.7525), (-2.8973, 2.8973)]
ROBOT_BODIES = ("link2", "link3", "link4", "link5", "link6", "link7", "hand", "left_finger", "right_finger")
PARK = [[0.8, -0.6, 1.5], [-0.8, -0.6, 1.5], [0.0, -0.9, 1.5]]  # cubes out of everyone's reach


def parked_qpos(m, arm):
    q = m.key_qpos.copy()
    q[:9] = arm
    for k in range(3):
        q[9 + 7 * k: 12 + 7 * k] = PARK[k]
        q[12 + 7 * k: 16 + 7 * k] = [1, 0, 0, 0]
    return q


def over_table(P):
    return (P[:, 0] > -0.39) & (P[:, 0] < 0.39) & (P[:, 1] > 0.16) & (P[:, 1] < 0.74)


def table_scenes(m, depths, seed=1, tries=20000):
    robot = [i for i, g in enumerate(m.geoms) if g["body"] in ROBOT_BODIES]
    top = m.find("table", "box")
    rng = np.random.default_rng(seed)
    out, want = {}, {i for i in robot if m.geoms[i]["type"] == "mesh" and m.geoms[i]["body"] != "right_finger"}

    def low(q, g):
        P = m.geom_points(m.geoms[g], m.fk(q))
        P = P[over_table(P)]
        return P[:, 2].min() if len(P) else np.inf

    for trial in range(tries):
        if want <= set(out):
            break
        arm = np.r_[[rng.uniform(*r) for r in RANGES], [rng.uniform(0, 0.04)] * 2]
        q = parked_qpos(m, arm)
        L = sorted((low(q, g), g) for g in robot)
        tg = L[0][1]
        lenient = m.geoms[tg]["body"] == "left_finger"  # its pads sit inside the fingertip
        if not np.isfinite(L[1][0]) or (L[1][0] - L[0][0] < 0.005 and not lenient):
            continue
        if tg not in want or tg in out:
            continue
        depth = depths[len(out) % len(depths)]
        lo, hi = max(q[1] - 0.5, RANGES[1][0]), min(q[1] + 0.5, RANGES[1][1])

        def f(s):
            qq = q.copy()
            qq[1] = s
            return low(qq, tg) - (0.24 - depth)

        flo, fhi = f(lo), f(hi)
        if not (np.isfinite(flo) and np.isfinite(fhi)) or flo * fhi > 0:
            continue
        for _ in range(60):
            mid = 0.5 * (lo + hi)
            fm = f(mid)
            if fm * flo > 0:
                lo, flo = mid, fm
            else:
                hi = mid
        q[1] = 0.5 * (lo + hi)
        pose = m.fk(q)
        T = m.geom_points(m.geoms[top], pose)
        touching = [g for g in robot if g != tg and penetration(m.geom_points(m.geoms[g], pose), T)[0] > -1e-4]
        if touching and not (lenient and all(m.geoms[g]["type"] == "box" for g in touching) and len(touching) <= 4):
            continue
        d, n, fac = penetration(m.geom_points(m.geoms[tg], pose), T)
        if abs(d - depth) > 1e-9 or n[2] > -1 + 1e-12 or normal_margin(fac) < 5e-4:
            continue
        out[tg] = dict(kind="hull_table", geom=tg, body=m.geoms[tg]["body"], mesh=m.geoms[tg]["mesh"],
                       depth=depth, qpos=q.tolist(), trial=trial, also_touching=touching)
    return [out[k] for k in sorted(out)]


def cube_scenes(m, depths, seed=2):
    # the keyframe's arm (over the table, every link clear of it), gripper half open
    arm = np.r_[m.key_qpos[:7], 0.02, 0.02]
    rng = np.random.default_rng(seed)
    targets = [i for i, g in enumerate(m.geoms) if g["type"] == "mesh" and g["body"] in ROBOT_BODIES
               and g["body"] != "right_finger"]
    out = []
    for tg in targets:
        for trial in range(1500):
            facet = trial >= 400  # no unique support vertex found: press the cube onto a hull facet
            q = parked_qpos(m, arm)
            pose = m.fk(q)
            W = m.geom_points(m.geoms[tg], pose)
            if facet:
                from scipy.spatial import ConvexHull

                h = ConvexHull(W)
                area = np.array([np.linalg.norm(np.cross(W[t[1]] - W[t[0]], W[t[2]] - W[t[0]])) for t in h.simplices])
                big = np.argsort(-area)[: 8]
                u = h.equations[big[rng.integers(len(big))], :3]
            else:
                u = rng.normal(size=3)
                u /= np.linalg.norm(u)
            s = W @ u
            order = np.argsort(-s)
            depth = depths[len(out) % len(depths)]
            if not facet and s[order[0]] - s[order[1]] < depth + 5e-4:
                continue
            v = W[order[0]]
            # cube frame: z axis = -u (its -z face... its +z face looks at -u), turned about u
            z = -u
            x = np.cross(z, [0.3, 0.5, 0.8])
            x /= np.linalg.norm(x)
            x = axis_rot(z, rng.uniform(0, 2 * np.pi)) @ x
            R = np.stack([x, np.cross(z, x), z], axis=1)
            off = rng.uniform(-0.012, 0.012, size=2)
            c = v + u * (0.02 - depth) - R[:, 0] * off[0] - R[:, 1] * off[1]
            # the cube's +z face (normal -u... ) : centre + 0.02 z = c - 0.02 u: plane u.x = u.v - depth
            q[9:12] = c
            q[12:16] = mat2quat(R)
            pose = m.fk(q)
            C = m.geom_points(m.geoms[m.find("obj_red", "box")], pose)
            others = [g for g in range(len(m.geoms)) if g != tg and m.geoms[g]["type"] in ("box", "mesh")
                      and m.geoms[g]["body"] != "obj_red"]
            touching = [g for g in others if penetration(m.geom_points(m.geoms[g], pose), C)[0] > -1e-4]
            if touching and not all(m.geoms[g]["body"] == m.geoms[tg]["body"] for g in touching):
                continue  # (the finger's own pads may touch: they sit in the fingertip)
            if C[:, 2].min() < 0.25:
                continue
            d, n, fac = penetration(W, C)
            ia, _ = feature_summary(fac)
            if abs(d - depth) > 1e-9 or (len(ia) != 1 and not facet) or normal_margin(fac) < 5e-4:
                continue
            out.append(dict(kind="cube_hull", geom=tg, body=m.geoms[tg]["body"], mesh=m.geoms[tg]["mesh"],
                            depth=depth, qpos=q.tolist(), trial=trial, feature="vertex" if len(ia) == 1 else "facet",
                            also_touching=touching))
            break
    return out


def main():
    m = RawModel()
    scenes = table_scenes(m, [0.001, 0.0005, 0.002, 0.0015]) + cube_scenes(m, [0.001, 0.002, 0.0005, 0.0015])
    for s in scenes:
        print(s["kind"], s["body"], s["mesh"], s["depth"], "trial", s["trial"])
    json.dump(dict(_source="tests/golden/make_collision_scenes.py", scenes=scenes),
              open(os.path.join(HERE, "collision_scenes.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
