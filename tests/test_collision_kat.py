"""Collision known-answer scenes (VERDICT r03 "next" #1): the narrowphase pinned to geometry,
independently of both implementations under test.

The reference's contacts come from MuJoCo's collision pipeline inside mj_step (env.py:119-121;
MuJoCo 3.5.0, un-vendored, absent from this image) over the model's collision geoms
(panda.xml:134-240: link / hand / finger hull meshes and the 5 fingertip pad boxes per finger;
pick_and_place_scene.xml:40-124: floor plane, tabletop box, leg cylinders, bin boxes, cubes).
Every answer below is derived in this file from geometry alone:

  * box scenes (box-box face and edge contacts, plane-box corners): the contact polygon's corners,
    depths and normals in closed form;
  * the cylinder leg (convex path): the depth of a cube face pressed into its side;
  * hull scenes (GJK / EPA): hulls of the raw STL / OBJ assets (tests/golden/collision_hulls.npz,
    built by make_collision_hulls.py, not by tools/compile_model.py), posed by forward kinematics
    from the raw MJCF attributes (tests/collision_geometry.py), the exact penetration as the
    distance from the origin to the nearest facet of the Minkowski difference's hull; for the
    tabletop that is the closed form "depth of the hull's lowest vertex below z = 0.24", asserted
    too.  Scene inputs: tests/golden/collision_scenes.json (make_collision_scenes.py).

MuJoCo's contact conventions checked (documentation, Computation / Collision detection): dist < 0
is penetration; the frame's first row is the normal from geom1 to geom2; geom1 has the lower type
(plane < cylinder < box < mesh); the position lies midway between the surfaces; a convex (mesh or
cylinder) pair gives ONE contact (nativeccd, multiccd off).  The same scenes run on the
fp64 oracle (CPU) and on the HIP kernel (`-m gpu`, one scene per env, contacts of mmx_physics_step's
substep through the C-ABI).

What stays unpinned: which points MuJoCo's own box-box routine emits where the contact region is a
polygon (the corners here are the geometric answer, which the clip produces), and the position of a
face-face hull contact (not unique; depth and normal are checked).
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from collision_geometry import (CUBES, GOLDEN, GT, RawModel, axis_rot, feature_summary, mat2quat,
                                penetration)

H = 0.02  # cube half edge
PARK = [[0.8, -0.6, 1.5], [-0.8, -0.6, 1.5], [0.0, -0.9, 1.5]]
CPU_TOL = dict(depth=1e-9, normal=1e-9, pos=1e-9)
GPU_TOL_BOX = dict(depth=2e-6, normal=1e-5, pos=5e-6)     # fp32 geometry at 0.5 m: ~6e-8 per value
GPU_TOL_CONVEX = dict(depth=1e-5, normal=1e-4, pos=5e-5)  # plus EPA's termination (1e-6 relative)


@pytest.fixture(scope="module")
def raw():
    return RawModel()


def compiled_ids(m):
    """raw geom index -> the index in the compiled model's collision-geom list (what both
    implementations report as a contact's geom1 / geom2): the k-th collision geom of a given type
    on a given body."""
    cm = json.load(open(os.path.join(os.path.dirname(GOLDEN), "..", "mujoco_manip_amd", "model",
                                     "panda_pickplace.json")))
    bname = [b["name"] for b in cm["bodies"]]
    out = {}
    for i, g in enumerate(m.geoms):
        k = sum(1 for j in range(i) if m.geoms[j]["body"] == g["body"] and m.geoms[j]["type"] == g["type"])
        ids = [c for c in cm["col_geoms"] if bname[cm["geoms"][c]["body"]] == g["body"]
               and cm["geoms"][c]["type"] == g["type"]]
        out[i] = cm["col_geoms"].index(ids[k])
    return out


_IDS = {}


def col_id(m, g):
    if id(m) not in _IDS:
        _IDS[id(m)] = compiled_ids(m)
    return _IDS[id(m)][g]


def parked(m, arm=None):
    q = m.key_qpos.copy()
    if arm is not None:
        q[:9] = arm
    for k in range(3):
        q[9 + 7 * k: 12 + 7 * k] = PARK[k]
        q[12 + 7 * k: 16 + 7 * k] = [1, 0, 0, 0]
    return q


def put_cube(q, k, pos, R=np.eye(3)):
    q[9 + 7 * k: 12 + 7 * k] = pos
    q[12 + 7 * k: 16 + 7 * k] = mat2quat(R)


def ordered(m, ga, gb, n_ab):
    """MuJoCo's pair order: geom1 has the lower type; equal types keep the lower geom id first
    (both implementations do).  Returns (g1, g2, normal g1 -> g2) in raw indices."""
    ta, tb = GT[m.geoms[ga]["type"]], GT[m.geoms[gb]["type"]]
    first = (ta, col_id(m, ga)) < (tb, col_id(m, gb))
    return (ga, gb, np.asarray(n_ab, float)) if first else (gb, ga, -np.asarray(n_ab, float))


# --------------------------------------------------------------------------- scenes
def scene_cube_on_cube(m):
    """Green cube on the red one, shifted by half an edge in x and 5 mm in y, 1 mm deep: a face
    contact whose polygon is the overlap rectangle x in [x0, x0 + h], y in [y0 - h + 5 mm, y0 + h],
    4 corners at depth 1 mm, midway between the faces (z = top - 0.5 mm)."""
    q = parked(m)
    x0, y0, z0, d = 0.6, -0.2, 0.8, 0.001
    put_cube(q, 0, [x0, y0, z0])
    put_cube(q, 1, [x0 + H, y0 + 0.005, z0 + 2 * H - d])
    top = z0 + H
    pts = [[x, y, top - d / 2] for x in (x0, x0 + H) for y in (y0 - H + 0.005, y0 + H)]
    a, b = m.find("obj_red", "box"), m.find("obj_green", "box")
    return q, [dict(pair=ordered(m, a, b, [0, 0, 1]), depth=d, pts=pts)]


def scene_cube_on_cube_turned(m):
    """Green cube centred on the red one, turned 45 deg about z, 0.7 mm deep: the overlap of the
    two squares is a regular octagon (the turned square's edges |x| + |y| = h sqrt 2 cut the
    lower one's |x| = h, |y| = h at (sqrt 2 - 1) h): 8 contacts at its corners."""
    q = parked(m)
    x0, y0, z0, d = -0.6, -0.3, 0.9, 0.0007
    put_cube(q, 0, [x0, y0, z0])
    put_cube(q, 1, [x0, y0, z0 + 2 * H - d], axis_rot([0, 0, 1], np.pi / 4))
    s = (np.sqrt(2) - 1) * H
    pts = [[x0 + a, y0 + b, z0 + H - d / 2] for a, b in ((H, s), (H, -s), (-H, s), (-H, -s), (s, H), (-s, H),
                                                         (s, -H), (-s, -H))]
    return q, [dict(pair=ordered(m, m.find("obj_red", "box"), m.find("obj_green", "box"), [0, 0, 1]), depth=d,
                    pts=pts)]


def scene_cube_edge_on_edge(m):
    """Red cube turned 45 deg about x (top edge along x), green cube above it turned 45 deg about
    y (bottom edge along y), the edges crossing 0.9 mm deep: the edge-edge axis (z) is the
    separating-axis minimum, one contact at the midpoint of the edges' closest points."""
    q = parked(m)
    x0, y0, z0, d = 0.5, 0.9, 0.7, 0.0009
    r2 = H * np.sqrt(2)
    put_cube(q, 0, [x0, y0, z0], axis_rot([1, 0, 0], np.pi / 4))
    put_cube(q, 1, [x0, y0, z0 + 2 * r2 - d], axis_rot([0, 1, 0], np.pi / 4))
    return q, [dict(pair=ordered(m, m.find("obj_red", "box"), m.find("obj_green", "box"), [0, 0, 1]), depth=d,
                    pts=[[x0, y0, z0 + r2 - d / 2]])]


def scene_cube_edge_on_table(m):
    """A cube turned 45 deg about x, balanced on its lower edge on the tabletop 0.8 mm deep: two
    contacts at the edge's end corners, normal +z (table -> cube)."""
    q = parked(m)
    d = 0.0008
    c = np.array([0.1, 0.35, 0.24 + H * np.sqrt(2) - d])
    put_cube(q, 2, c, axis_rot([1, 0, 0], np.pi / 4))
    pts = [[c[0] + sx * H, c[1], 0.24 - d / 2] for sx in (-1, 1)]
    return q, [dict(pair=ordered(m, m.find("table", "box"), m.find("obj_blue", "box"), [0, 0, 1]), depth=d, pts=pts)]


def scene_cube_in_bin_corner(m):
    """The red cube in the red bin's front-left corner, pressed 0.4 mm into the front wall (y),
    0.7 mm into the left wall (x) and 1.1 mm into the bottom: three face contacts, 4 corners
    each (the cube's faces lie inside the walls' faces), at the three depths."""
    q = parked(m)
    dy, dx, dz = 0.0004, 0.0007, 0.0011
    # red bin at (-0.3, 0.55, 0.24): left wall inner face x = -0.358, front wall inner face
    # y = 0.492, bottom top face z = 0.242
    c = np.array([-0.358 + H - dx, 0.492 + H - dy, 0.242 + H - dz])
    put_cube(q, 0, c)
    cube = m.find("obj_red", "box")
    out = []
    for wall, ax, face, d in (("bin_red", 0, -0.358, dx), ("bin_red", 1, 0.492, dy), ("bin_red", 2, 0.242, dz)):
        k = {0: 3, 1: 1, 2: 0}[ax]  # left, front, bottom among the bin's boxes
        n = np.zeros(3)
        n[ax] = 1.0  # wall -> cube
        u, v = [i for i in range(3) if i != ax]
        pts = []
        for su in (-1, 1):
            for sv in (-1, 1):
                p = c.copy()
                p[ax] = face - d / 2
                p[u] += su * H
                p[v] += sv * H
                pts.append(p)
        out.append(dict(pair=ordered(m, m.find(wall, "box", k), cube, n), depth=d, pts=pts))
    return q, out


def scene_pad_clamp(m):
    """The left finger's large fingertip pad (panda.xml:20-22: half size (8.5, 4, 8.5) mm at
    (0, 5.5, 44.5) mm in the finger frame) pressed 0.6 mm into the green cube's side, the cube
    aligned with the finger frame: a face contact whose polygon is the pad's inner face (17 x 17
    mm, inside the cube's face), normal = the finger's +y, depth 0.6 mm."""
    arm = np.r_[m.key_qpos[:7], 0.03, 0.03]  # the keyframe's arm, gripper open 3 cm: clear of the table
    q = parked(m, arm)
    pose = m.fk(q)
    p, R = pose["left_finger"]
    d = 0.0006
    pad_c = np.array([0.0, 0.0055, 0.0445])
    pad_h = np.array([0.0085, 0.004, 0.0085])
    face_y = pad_c[1] + pad_h[1]  # inner face, finger frame
    c_local = np.array([0.003, face_y - d + H, pad_c[2] - 0.004])
    put_cube(q, 1, p + R @ c_local, R)
    pts = []
    for sx in (-1, 1):
        for sz in (-1, 1):
            loc = np.array([pad_c[0] + sx * pad_h[0], face_y - d / 2, pad_c[2] + sz * pad_h[2]])
            pts.append(p + R @ loc)
    pad = m.find("left_finger", "box", 0)
    return q, [dict(pair=ordered(m, pad, m.find("obj_green", "box"), R[:, 1]), depth=d, pts=pts,
                    others_ok={m.find("left_finger", "mesh")})]


def scene_cube_tilted_on_floor(m):
    """A cube on the floor plane (outside the table) turned so that exactly one corner points
    down, 1.5 mm deep: one plane-box contact at that corner, normal +z, midway."""
    q = parked(m)
    R = axis_rot([1, 0, 0], 0.4) @ axis_rot([0, 1, 0], 0.3)
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * H
    w = corners @ R.T
    low = np.argmin(w[:, 2])
    d = 0.0015
    c = np.array([0.75, -0.45, -w[low, 2] - d])
    put_cube(q, 0, c, R)
    zs = np.sort(w[:, 2])
    assert zs[1] - zs[0] > 2 * d  # a single corner below the plane
    return q, [dict(pair=ordered(m, 0, m.find("obj_red", "box"), [0, 0, 1]), depth=d, pts=[c + w[low] + [0, 0, d / 2]])]


def scene_cube_against_leg(m):
    """The blue cube (axis-aligned) under the table, its -x face pressed 0.9 mm into leg1's side
    (cylinder r = 25 mm at (0.35, 0.7), z in [0, 0.2]): one contact, depth 0.9 mm, normal +x
    (cylinder -> cube), midway at the cylinder's extreme point."""
    q = parked(m)
    d, r = 0.0009, 0.025
    axis_xy = np.array([0.35, 0.70])
    c = np.array([axis_xy[0] + r + H - d, axis_xy[1] + 0.004, 0.1])
    put_cube(q, 2, c)
    pts = [[axis_xy[0] + r - d / 2, axis_xy[1], None]]  # z anywhere on the cube face's span
    return q, [dict(pair=ordered(m, m.find("table", "cylinder", 0), m.find("obj_blue", "box"), [1, 0, 0]),
                    depth=d, pts=pts, convex=True)]


BOX_SCENES = [scene_cube_on_cube, scene_cube_on_cube_turned, scene_cube_edge_on_edge, scene_cube_edge_on_table, scene_cube_in_bin_corner, scene_pad_clamp,
              scene_cube_tilted_on_floor, scene_cube_against_leg]


def mesh_scenes(m):
    """Scenes of tests/golden/collision_scenes.json with their answers from geometry: exact
    penetration of the hull and the tabletop / cube, and (vertex-face features) the witness
    midpoint."""
    data = json.load(open(os.path.join(GOLDEN, "collision_scenes.json")))["scenes"]
    out = []
    for s in data:
        q = np.array(s["qpos"], float)
        out.append((s, q))
    return out


def mesh_answer(m, s, q):
    pose = m.fk(q)
    tg = s["geom"]
    other = m.find("table", "box") if s["kind"] == "hull_table" else m.find("obj_red", "box")
    W = m.geom_points(m.geoms[tg], pose)
    depth, n, fac = penetration(W, m.geom_points(m.geoms[other], pose))
    ia, _ = feature_summary(fac)
    pts = [0.5 * (fac[0][2] + fac[0][3])] if len(ia) == 1 else None
    if s["kind"] == "hull_table":
        # the closed form: the lowest hull vertex's depth below the tabletop, normal +z
        assert abs(depth - (0.24 - W[:, 2].min())) < 1e-9, (depth, W[:, 2].min())
        assert n[2] < -1 + 1e-12
    return dict(pair=ordered(m, tg, other, n), depth=depth, pts=pts, convex=True)


# --------------------------------------------------------------------------- checking
def check(m, ids, contacts, want, tol, label, others_allowed=()):
    """contacts: [(g1, g2, dist, pos[3], normal[3])] in compiled ids; want: the expected pair."""
    g1, g2, n = want["pair"]
    c1, c2 = ids[g1], ids[g2]
    mine = [c for c in contacts if (c[0], c[1]) == (c1, c2)]
    swapped = [c for c in contacts if (c[0], c[1]) == (c2, c1)]
    assert not swapped, f"{label}: pair reported in the wrong order (geom1 must have the lower type)"
    n = np.asarray(n, float) / np.linalg.norm(n)
    if want.get("convex"):
        assert len(mine) == 1, f"{label}: {len(mine)} contacts for a convex pair (MuJoCo: exactly one)"
    else:
        assert len(mine) == len(want["pts"]), f"{label}: {len(mine)} contacts, want {len(want['pts'])}"
    for c in mine:
        assert abs(-c[2] - want["depth"]) < tol["depth"], f"{label}: depth {-c[2]} want {want['depth']}"
        assert np.abs(np.asarray(c[4]) - n).max() < tol["normal"], f"{label}: normal {c[4]} want {n}"
    if want.get("pts") is not None:
        got = [np.asarray(c[3], float) for c in mine]
        for p in want["pts"]:
            mask = np.array([v is not None for v in p])
            pv = np.array([0.0 if v is None else v for v in p])
            dists = [np.abs((g - pv)[mask]).max() for g in got]
            assert min(dists) < tol["pos"], f"{label}: no contact at {p} (got {got})"


def oracle_contacts(q):
    import oracle_py as O

    e = O.OracleEnv()
    e.reset_keyframe()
    e.set_state(q, np.zeros(27), None, np.zeros(27))
    e.mj_forward()
    return [(int(c["geom"][0]), int(c["geom"][1]), c["dist"], c["pos"], c["frame"][0]) for c in e.contacts()]


def all_scenes(m):
    out = []
    for f in BOX_SCENES:
        q, wants = f(m)
        out.append((f.__name__, q, wants))
    for s, q in mesh_scenes(m):
        out.append((f"{s['kind']}:{s['mesh']}", q, None))
    return out


# --------------------------------------------------------------------------- CPU (fixtures, oracle)
def test_hull_fixture_matches_compiled_hulls(raw):
    """The compiled model's collision hulls (tools/compile_model.py -> the device and oracle
    tables) are the convex hulls of the raw assets: same vertex sets in the body frame."""
    cm = json.load(open(os.path.join(os.path.dirname(GOLDEN), "..", "mujoco_manip_amd", "model",
                                     "panda_pickplace.json")))
    from collision_geometry import quat2mat

    seen = set()
    for c in cm["col_geoms"]:
        g = cm["geoms"][c]
        if g["type"] != "mesh" or g["mesh"] in seen:
            continue
        seen.add(g["mesh"])
        mesh = next(x for x in cm["meshes"] if x["name"] == g["mesh"])
        V = np.asarray(mesh["verts"]) @ quat2mat(g["quat"]).T + np.asarray(g["pos"])
        F = raw.hulls[g["mesh"]]
        assert len(V) == len(F), (g["mesh"], len(V), len(F))
        dVF = np.sqrt(((V[:, None] - F[None]) ** 2).sum(-1))
        assert dVF.min(1).max() < 1e-7 and dVF.min(0).max() < 1e-7, g["mesh"]  # float32 file values
    assert seen == set(raw.hulls), (seen, set(raw.hulls))


def test_scene_inputs_are_what_they_claim(raw):
    """The scene fixtures' premises, from geometry: each mesh scene's hull touches only its
    partner (and, for the finger, its own pads), at the stated depth."""
    for s, q in mesh_scenes(raw):
        a = mesh_answer(raw, s, q)
        assert abs(a["depth"] - s["depth"]) < 1e-9, (s["mesh"], a["depth"], s["depth"])
    kinds = {(s["kind"], s["mesh"]) for s, _ in mesh_scenes(raw)}
    assert len([k for k in kinds if k[0] == "hull_table"]) >= 7
    assert len([k for k in kinds if k[0] == "cube_hull"]) >= 7
    assert ("hull_table", "finger_0") in kinds and ("hull_table", "hand_c") in kinds


@pytest.mark.parametrize("idx", range(len(BOX_SCENES)))
def test_oracle_box_scenes(raw, idx):
    ids = compiled_ids(raw)
    q, wants = BOX_SCENES[idx](raw)
    con = oracle_contacts(q)
    for w in wants:
        check(raw, ids, con, w, CPU_TOL if not w.get("convex") else dict(depth=2e-6, normal=1e-4, pos=2e-5),
              BOX_SCENES[idx].__name__)
    # nothing else touches in these scenes
    pairs = {(ids[w["pair"][0]], ids[w["pair"][1]]) for w in wants}
    extra = {(c[0], c[1]) for c in con} - pairs
    ok = {ids[g] for w in wants for g in w.get("others_ok", ())}
    extra = {p for p in extra if not (set(p) & ok)}
    assert not extra, extra


def test_oracle_mesh_scenes(raw):
    ids = compiled_ids(raw)
    for s, q in mesh_scenes(raw):
        want = mesh_answer(raw, s, q)
        # the oracle's EPA terminates at 1e-10 (absolute) on the support gap
        check(raw, ids, oracle_contacts(q), want, dict(depth=1e-8, normal=1e-6, pos=1e-6), f"{s['kind']}:{s['mesh']}")


# --------------------------------------------------------------------------- GPU (HIP kernel)
def gpu_contacts(qs):
    """Contacts of one substep of the kernel from each state (one env per state)."""
    import torch

    from mujoco_manip_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    n = len(qs)
    sim = _lib.Sim(n, action_mode="abs_pos", image_size=0)
    sim.reset()
    _, _, ctrl, _ = sim.get_state()
    Q = np.asarray(qs, np.float32)
    sim.set_state(Q, np.zeros((n, 27), np.float32), ctrl, np.zeros((n, 27), np.float32))
    sim.physics_step(1, with_ik=False)
    ncon = sim.view("episode_i", _lib.EPI_N, "<i4")[:, _lib.EPI["ncon"]].cpu().numpy()
    con = sim.view("contacts", _lib.MAXCON * _lib.CON_F).cpu().numpy().reshape(n, _lib.MAXCON, _lib.CON_F)
    sim.close()
    out = []
    for e in range(n):
        assert ncon[e] < _lib.MAXCON
        out.append([(int(c[11]), int(c[12]), float(c[0]), c[1:4].astype(float), c[4:7].astype(float))
                    for c in con[e, :ncon[e]]])
    return out, Q.astype(np.float64)


@pytest.mark.gpu
def test_gpu_box_scenes(raw):
    ids = compiled_ids(raw)
    scenes = [f(raw) for f in BOX_SCENES]
    got, _ = gpu_contacts([q for q, _ in scenes])
    for (q, wants), con, f in zip(scenes, got, BOX_SCENES):
        for w in wants:
            check(raw, ids, con, w, GPU_TOL_CONVEX if w.get("convex") else GPU_TOL_BOX, f.__name__)


@pytest.mark.gpu
def test_gpu_mesh_scenes(raw):
    """GJK / EPA on the kernel against the exact penetration of the raw-asset hulls, answers
    recomputed at the fp32-rounded states the kernel actually ran."""
    ids = compiled_ids(raw)
    scenes = mesh_scenes(raw)
    got, Q = gpu_contacts([q for _, q in scenes])
    for (s, _), con, q32 in zip(scenes, got, Q):
        check(raw, ids, con, mesh_answer(raw, s, q32), GPU_TOL_CONVEX, f"{s['kind']}:{s['mesh']}")
