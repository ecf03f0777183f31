#!/usr/bin/env python3
"""Offline render-model compiler: scene + Panda visual meshes -> a triangle model.

Runs in the build container only (the MJCF and meshes live under the reference mount). Its
outputs are committed DATA:

  mujoco_manip_amd/csrc/mmx_render_gen.h       tables for the HIP rasterizer
  mujoco_manip_amd/model/render_model.json     the same model for the CPU ray-cast checker

Geometry (all vertices in their BODY frame, so the device only needs body poses):
  * floor plane (pick_and_place_scene.xml:40) as an 8 x 8 grid of quads, checker material
    `groundplane` (rgb1/rgb2, texrepeat 5 5, texuniform: 0.1 m squares);
  * every box geom of the table, bins and cubes (:43-125) as 12 triangles, the table legs
    (cylinders) as 16-gon prisms, each with its own material rgba;
  * the Panda's visual meshes (panda.xml:123-246, 134,888 triangles, far beyond what a batched
    per-env rasterizer should carry): all 57 visual parts decimated together under one budget of
    ROBOT_TRIS triangles by quadric-error edge collapse (tools/qem.py), each part in its own
    material, the hand and fingers' errors weighted by HAND_WEIGHT (the wrist camera's close-up).
Segment ids (the mask-level parity channel): 0 sky, 1 floor, 2 table, 3/4/5 bins red/green/blue,
6/7/8 cubes red/green/blue, 9 robot.
"""
from __future__ import annotations

import json
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np
from scipy.spatial import ConvexHull

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import compile_model as CM  # noqa: E402

MAX_HULL_VERTS = 96
# robot geometry (mean robot-mask IoU against the full 134,888-triangle
# visual meshes, tests/golden/robot_masks.npz, 8 states, 128 x 128, overhead / wrist):
#   one hull per body (r02)                                              0.89 / 0.75
#   convex pieces per link part + clustered hand / fingers, 2,033 tris   0.92 / 0.97  (r03-r05)
#   quadric-error collapse, one budget (tools/qem.py): 1,400 tris        0.951 / 0.969
#                                                     1,600              0.962 / 0.975
#                                                     1,800              0.973 / 0.977  <- kept
#                                                     2,000              0.976 / 0.975
#   hand / finger error weight at 1,800 tris: 30 -> 0.974 / 0.970, 100 -> 0.973 / 0.977 (kept);
#   at 2,000: 1 -> 0.979 / 0.792 (the fingers collapse), 300 -> 0.967 / 0.977
ROBOT_TRIS = 1800
HAND_WEIGHT = 100.0
# the r03-r05 reduction (robot_tris=0): convex pieces of ~7 cm per link part (<= 10 points), hand
# clustered at 20 mm, fingers at 6 mm
LINK_PIECE_SIZE = 0.07
LINK_PIECE_VERTS = 10
HAND_CELL = 0.02
FINGER_CELL = 0.006
FLOOR_GRID = 8
FLOOR_HALF = 2.0  # floor geom size 2 2 (pick_and_place_scene.xml:40)
CYL_SIDES = 12  # table legs (hidden under the top from both cameras)
SEG = {"floor": 1, "table": 2, "bin_red": 3, "bin_green": 4, "bin_blue": 5, "obj_red": 6, "obj_green": 7,
       "obj_blue": 8, "robot": 9}
ROBOT = ["link0", "link1", "link2", "link3", "link4", "link5", "link6", "link7", "hand", "left_finger",
         "right_finger"]


def rgba(s):
    return [float(x) for x in s.split()]


def box_mesh(half):
    hx, hy, hz = half
    v = np.array([[sx * hx, sy * hy, sz * hz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
    h = ConvexHull(v)
    return v, oriented_faces(v, h)


def cylinder_mesh(r, hh, n=CYL_SIDES):
    ang = 2 * np.pi * np.arange(n) / n
    ring = np.stack([r * np.cos(ang), r * np.sin(ang)], 1)
    v = np.concatenate([np.c_[ring, -hh * np.ones(n)], np.c_[ring, hh * np.ones(n)]])
    h = ConvexHull(v)
    return v, oriented_faces(v, h)


def oriented_faces(v, h):
    c = v.mean(0)
    out = []
    for s in h.simplices:
        a, b, cc = v[s]
        n = np.cross(b - a, cc - a)
        out.append([int(s[0]), int(s[1]), int(s[2])] if np.dot(n, a - c) > 0 else [int(s[0]), int(s[2]), int(s[1])])
    return out


def fps_subsample(p, k):
    """farthest-point sampling of k points (deterministic: start at the point farthest from the mean)."""
    if len(p) <= k:
        return p
    idx = [int(np.argmax(np.linalg.norm(p - p.mean(0), axis=1)))]
    d = np.linalg.norm(p - p[idx[0]], axis=1)
    for _ in range(k - 1):
        i = int(np.argmax(d))
        idx.append(i)
        d = np.minimum(d, np.linalg.norm(p - p[i], axis=1))
    return p[idx]


def hull_mesh(points, k=MAX_HULL_VERTS):
    h = ConvexHull(points)
    p = fps_subsample(points[h.vertices], k)
    h2 = ConvexHull(p)
    v = p[h2.vertices]
    remap = {int(j): i for i, j in enumerate(h2.vertices)}
    faces = [[remap[int(j)] for j in s] for s in h2.simplices]
    return v, oriented_faces(v, type("H", (), {"simplices": np.array(faces)})), float(h.volume)


def load_obj_tris(path):
    """OBJ vertices and fan-triangulated faces (v / v/vt / v/vt/vn forms, 1-based or negative)."""
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


def cluster_mesh(v, t, cell):
    """Vertex-clustering decimation: vertices merged per `cell`-sized grid cell (cell mean),
    triangles that collapse dropped; the surviving triangles keep the file's winding."""
    q = np.floor(v / cell).astype(np.int64)
    keys, inv = np.unique(q, axis=0, return_inverse=True)
    inv = inv.ravel()
    rep = np.zeros((len(keys), 3))
    cnt = np.zeros(len(keys))
    np.add.at(rep, inv, v)
    np.add.at(cnt, inv, 1)
    rep /= cnt[:, None]
    tt = inv[t]
    tt = tt[(tt[:, 0] != tt[:, 1]) & (tt[:, 1] != tt[:, 2]) & (tt[:, 0] != tt[:, 2])]
    tt = np.unique(tt, axis=0)
    used = np.unique(tt)
    remap = np.full(len(rep), -1)
    remap[used] = np.arange(len(used))
    return rep[used], remap[tt]


def convex_pieces(v, size, k):
    """A part's vertices split into ceil(extent / size) spatial clusters (k-means, fixed seed), each
    drawn as its convex hull (<= k points): concave links keep their silhouette far better than
    one hull per body at a fraction of the visual mesh's triangles."""
    from scipy.cluster.vq import kmeans2

    m = max(1, int(np.ceil(np.ptp(v, 0).max() / size)))
    groups = [v]
    if m > 1 and len(v) >= 8 * m:
        _, lab = kmeans2(v, m, minit="++", seed=0)
        groups = [v[lab == i] for i in range(m) if (lab == i).sum() >= 4]
    out = []
    for g in groups:
        try:
            hv, hf, _ = hull_mesh(g, k)
        except Exception:  # a degenerate (flat) cluster: covered by its neighbours
            continue
        out.append((hv, hf))
    return out


def geom_to_body(v, pos, quat):
    R = CM.quat2mat(quat)
    return v @ R.T + np.asarray(pos, float)


def build(robot_tris=ROBOT_TRIS, hand_weight=HAND_WEIGHT):
    model = CM.compile_model()
    bodies = model["bodies"]
    bnames = [b["name"] for b in bodies]
    scene = ET.parse(CM.SCENE).getroot()
    panda = ET.parse(CM.PANDA).getroot()
    mats = {}
    for m in list(scene.find("asset").iter("material")) + list(panda.find("asset").iter("material")):
        if m.get("rgba"):
            mats[m.get("name")] = rgba(m.get("rgba"))
    # checker floor colours (pick_and_place_scene.xml:19-22)
    tex = {t.get("name"): t for t in scene.find("asset").iter("texture")}["groundplane"]
    materials = [dict(name="groundplane", rgb=rgba(tex.get("rgb1")), rgb2=rgba(tex.get("rgb2")), checker=0.1,
                      seg=SEG["floor"])]
    mat_index = {}

    def material(name, seg):
        key = (name, seg)
        if key not in mat_index:
            mat_index[key] = len(materials)
            materials.append(dict(name=name, rgb=mats[name][:3], rgb2=mats[name][:3], checker=0.0, seg=seg))
        return mat_index[key]

    parts = []  # (body id, verts [k,3] body frame, faces, material index)
    # floor: grid over [-2, 2]^2 at z = 0 (body 0)
    g = np.linspace(-FLOOR_HALF, FLOOR_HALF, FLOOR_GRID + 1)
    fv = np.array([[x, y, 0.0] for y in g for x in g])
    ff = []
    for j in range(FLOOR_GRID):
        for i in range(FLOOR_GRID):
            a = j * (FLOOR_GRID + 1) + i
            b, c, d = a + 1, a + FLOOR_GRID + 1, a + FLOOR_GRID + 2
            ff += [[a, b, d], [a, d, c]]  # counter-clockwise seen from +z
    parts.append((0, fv, ff, 0))

    def scene_body(belem, bid):
        bname = belem.get("name")
        seg = SEG["table"] if bname == "table" else SEG[bname]
        for ge in belem.findall("geom"):
            t = ge.get("type")
            pos = CM.fl(ge.get("pos", "0 0 0"))
            size = CM.fl(ge.get("size"))
            if t == "box":
                v, f = box_mesh(size)
            elif t == "cylinder":
                v, f = cylinder_mesh(size[0], size[1])
            else:
                raise ValueError(t)
            parts.append((bid, geom_to_body(v, pos, [1, 0, 0, 0]), f, material(ge.get("material"), seg)))

    for be in scene.find("worldbody").findall("body"):
        scene_body(be, bnames.index(be.get("name")))

    # robot bodies: hull of the visual meshes (file coordinates = body frame; no geom pos/quat)
    meshfile = {}
    for m in panda.find("asset").findall("mesh"):
        fname = m.get("file")
        meshfile[m.get("name", os.path.splitext(fname)[0])] = os.path.join(CM.REF_DATA, "franka_emika_panda",
                                                                           "assets", fname)

    robot = []  # (body id, material, verts, faces) of every visual part

    def walk(be):
        name = be.get("name")
        if name in ROBOT:
            for ge in be.findall("geom"):
                if ge.get("class") != "visual":
                    continue
                assert ge.get("pos") is None and ge.get("quat") is None
                v, t = load_obj_tris(meshfile[ge.get("mesh")])
                robot.append((bnames.index(name), material(ge.get("material"), SEG["robot"]), v, t))
        for c in be.findall("body"):
            walk(c)

    for be in panda.find("worldbody").findall("body"):
        walk(be)
    if robot_tris:  # every visual part decimated under one triangle budget (tools/qem.py)
        import qem
        w = [hand_weight if bnames[b] in ("hand", "left_finger", "right_finger") else 1.0 for b, _, _, _ in robot]
        for (b, m, _, _), (dv, dt) in zip(robot, qem.decimate_many([(v, t) for _, _, v, t in robot], robot_tris, w)):
            parts.append((b, dv, dt.tolist(), m))
    else:
        for b, m, v, t in robot:
            if bnames[b].startswith("link"):  # arm links: convex pieces of each visual part
                for pv, pf in convex_pieces(v, LINK_PIECE_SIZE, LINK_PIECE_VERTS):
                    parts.append((b, pv, pf, m))
            else:  # hand and fingers (the wrist camera's close-up): clustered meshes
                cv, cf = cluster_mesh(v, t, HAND_CELL if bnames[b] == "hand" else FINGER_CELL)
                parts.append((b, cv, cf.tolist(), m))

    # flatten, vertices grouped by body
    verts, vbody, tris, tmat = [], [], [], []
    for bid, v, f, m in sorted(parts, key=lambda p: p[0]):
        base = len(verts)
        verts += [list(map(float, x)) for x in v]
        vbody += [bid] * len(v)
        tris += [[base + a, base + b, base + c] for a, b, c in f]
        tmat += [m] * len(f)
    return dict(verts=verts, vert_body=vbody, tris=tris, tri_mat=tmat, materials=materials,
                cameras=model["cameras"], body_names=bnames,
                static_body_pos={n: bodies[i]["pos"] for i, n in enumerate(bnames) if n in
                                 ("table", "bin_red", "bin_green", "bin_blue")})


def emit(rm, path):
    L = ["/* generated by tools/compile_render.py -- do not edit */\n#ifndef MMX_RENDER_GEN_H\n"
         "#define MMX_RENDER_GEN_H\n\n#ifndef MMR_QUAL\n#define MMR_QUAL static const\n#endif\n\n"]
    # the floor plane (body 0, material 0, checker) is not in the device tables: the renderer shades
    # it analytically behind everything (the CPU ray caster keeps its grid triangles)
    vkeep = np.array(rm["vert_body"]) != 0
    vmap = np.cumsum(vkeep) - 1
    tris = np.array(rm["tris"])
    tkeep = vkeep[tris].all(1)
    verts = [v for v, k in zip(rm["verts"], vkeep) if k]
    vbody = [b for b, k in zip(rm["vert_body"], vkeep) if k]
    dtris = vmap[tris[tkeep]].tolist()
    dmat = [m for m, k in zip(rm["tri_mat"], tkeep) if k]
    # the kernel packs each rasterised face's colour once (flat light x material): a checker
    # material among the device triangles would need per-pixel shading
    assert all(rm["materials"][m]["checker"] == 0.0 for m in set(dmat)), "checker material on a rasterised face"
    nv, nt, nm = len(verts), len(dtris), len(rm["materials"])
    L.append(f"#define MMR_NVERT {nv}\n#define MMR_NTRI {nt}\n#define MMR_NMAT {nm}\n")
    L.append(f"#define MMR_FLOOR_TRIS 0\n#define MMR_FLOOR_HALF {FLOOR_HALF!r}f\n#define MMR_FLOOR_MAT 0\n\n")
    L.append(CM.c_array("MMR_vert", "float", verts, "{:.9g}"))
    L.append(CM.c_array("MMR_vert_body", "unsigned char", vbody, "{}"))
    L.append(CM.c_array("MMR_tri", "unsigned short", dtris, "{}"))
    L.append(CM.c_array("MMR_tri_mat", "unsigned char", dmat, "{}"))
    L.append(CM.c_array("MMR_mat_rgb", "float", [m["rgb"] + m["rgb2"] for m in rm["materials"]], "{:.9g}"))
    L.append(CM.c_array("MMR_mat_checker", "float", [m["checker"] for m in rm["materials"]], "{:.9g}"))
    L.append(CM.c_array("MMR_mat_seg", "unsigned char", [m["seg"] for m in rm["materials"]], "{}"))
    L.append("\n#endif /* MMX_RENDER_GEN_H */\n")
    with open(path, "w") as f:
        f.write("".join(L).replace(CM.QUAL + " ", "MMR_QUAL "))


def main():
    rm = build()
    emit(rm, os.path.join(CM.REPO, "mujoco_manip_amd", "csrc", "mmx_render_gen.h"))
    with open(os.path.join(CM.REPO, "mujoco_manip_amd", "model", "render_model.json"), "w") as f:
        json.dump(rm, f, separators=(",", ":"))
    print(f"render model: {len(rm['verts'])} verts, {len(rm['tris'])} triangles, {len(rm['materials'])} materials")


if __name__ == "__main__":
    main()
