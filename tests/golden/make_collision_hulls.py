"""Generates tests/golden/collision_hulls.npz: the convex hulls MuJoCo collides the Panda's mesh
geoms with, computed straight from the reference's raw STL / OBJ assets (VERDICT r03 "next" #1).

Run in the build container, where the reference's model files are readable (binary / text data;
nothing of the reference is imported or executed):

    python tests/golden/make_collision_hulls.py [REFERENCE_ROOT]

Deliberately independent of tools/compile_model.py (its own STL / OBJ readers, its own hull call),
so the collision known-answer tests (tests/test_collision_kat.py) pin the compiled hull tables and
the narrowphase against geometry, not against the code that produced them.

MuJoCo collides a mesh geom through the convex hull of the mesh's vertices (qhull; the mesh's
frame = the file's coordinates, since every collision geom of panda.xml:134-223 carries no pos /
quat).  Sources: panda.xml:44-55 (collision mesh assets), :134-223 (the `class="collision"` geoms
and the bodies that own them).  The file holds, per mesh asset name, `<name>` = the hull's vertices
[n, 3] in the body frame (float64 of the float32 file values), and `meshes` = the names.
"""
from __future__ import annotations

import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np
from scipy.spatial import ConvexHull

HERE = os.path.dirname(os.path.abspath(__file__))


def read_stl(path):
    """Binary STL: 80-byte header, u32 count, 50-byte records (normal, 3 vertices, attribute)."""
    raw = open(path, "rb").read()
    n = struct.unpack_from("<I", raw, 80)[0]
    assert len(raw) == 84 + 50 * n, f"not a binary STL: {path}"
    rec = np.frombuffer(raw, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                        count=n, offset=84)
    return rec["v"].reshape(-1, 3).astype(np.float64)


def read_obj(path):
    out = []
    for line in open(path):
        t = line.split()
        if t and t[0] == "v":
            out.append([float(np.float32(x)) for x in t[1:4]])
    return np.asarray(out, np.float64)


def hull_vertices(pts):
    pts = np.unique(pts, axis=0)
    return pts[np.sort(ConvexHull(pts).vertices)]


def main(ref_root="/root/reference"):
    panda = os.path.join(ref_root, "mujoco_manip", "data", "franka_emika_panda")
    root = ET.parse(os.path.join(panda, "panda.xml")).getroot()
    meshdir = os.path.join(panda, root.find("compiler").get("meshdir", ""))
    files = {}
    for m in root.find("asset").iter("mesh"):
        f = m.get("file")
        files[m.get("name", os.path.splitext(f)[0])] = os.path.join(meshdir, f)
    used = []
    for g in root.iter("geom"):
        cls = g.get("class", "")
        if cls == "collision" and g.get("mesh") and g.get("mesh") not in used:
            used.append(g.get("mesh"))
    arrays = {}
    for name in used:
        path = files[name]
        pts = read_stl(path) if path.endswith(".stl") else read_obj(path)
        arrays[name] = hull_vertices(pts)
        print(f"{name}: {len(pts)} file vertices -> {len(arrays[name])} hull vertices")
    arrays["meshes"] = np.array(used)
    np.savez_compressed(os.path.join(HERE, "collision_hulls.npz"), **arrays)


if __name__ == "__main__":
    main(*sys.argv[1:])
