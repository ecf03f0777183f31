#!/usr/bin/env python3
"""Offline model compiler: pick-and-place MJCF + collision meshes -> compiled constants.

Runs in the build container only (the MJCF and mesh files live under the reference
mount, which does not exist on the GPU box).  Its outputs are committed DATA:

  mujoco_manip_amd/model/panda_pickplace.json   canonical compiled model
  mujoco_manip_amd/csrc/mmx_model_gen.h          constants for the HIP kernels / C-ABI
  oracle/oracle_model_gen.h                      constants for the CPU oracle (fp64)

What it restates (MuJoCo 3.5.0 compiler semantics, from the MuJoCo documentation):
  * default-class resolution for the constructs the two files use
    (panda.xml:6-37 defaults, childclass on link0 panda.xml:120);
  * body tree order = depth-first document order, include first
    (pick_and_place_scene.xml:14 includes panda.xml before its own worldbody);
  * autolimits (panda.xml:2): a joint/actuator with a range is limited;
  * inertia: fullinertia/diaginertia (panda.xml:121-219); a body without <inertial>
    takes its inertia from its geoms (cubes, pick_and_place_scene.xml:107-125);
  * welding: a body without joints is welded to its parent (weldid), used for the
    collision filter (same weld / parent-weld, world exempt) and the contact
    exclude link0-link1 (panda.xml:284-286);
  * collision meshes are used through their convex hull (qhull, like MuJoCo);
  * body_invweight0 / dof_invweight0 computed at qpos0 as mj_setConst does
    (A = J M^-1 J^T at the body com, mean of translational / rotational diagonal).
"""
from __future__ import annotations

import json
import math
import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np
from scipy.spatial import ConvexHull

REF_DATA = "/root/reference/mujoco_manip/data"
SCENE = os.path.join(REF_DATA, "pick_and_place_scene.xml")
PANDA = os.path.join(REF_DATA, "franka_emika_panda", "panda.xml")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# MuJoCo default ("main" class) attribute values.
MAIN_DEFAULTS = {
    "joint": {"type": "hinge", "axis": "0 0 1", "pos": "0 0 0", "armature": "0", "damping": "0"},
    "geom": {
        "type": "sphere", "contype": "1", "conaffinity": "1", "condim": "3",
        "friction": "1 0.005 0.0001", "solref": "0.02 1", "solimp": "0.9 0.95 0.001 0.5 2",
        "margin": "0", "gap": "0", "pos": "0 0 0", "density": "1000",
    },
    "general": {"dyntype": "none", "gaintype": "fixed", "biastype": "none",
                "gainprm": "1 0 0", "biasprm": "0 0 0"},
    "material": {},
}

TIMESTEP = 0.002


def fl(s):
    return [float(x) for x in s.split()]


def quat_norm(q):
    q = np.asarray(q, float)
    return q / np.linalg.norm(q)


def quat2mat(q):
    w, x, y, z = quat_norm(q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
    ])


def xyaxes_to_quat(xy):
    x = np.array(xy[:3], float)
    x /= np.linalg.norm(x)
    y = np.array(xy[3:], float)
    y -= x * x.dot(y)
    y /= np.linalg.norm(y)
    z = np.cross(x, y)
    R = np.stack([x, y, z], axis=1)
    return mat2quat(R)


def mat2quat(R):
    tr = np.trace(R)
    if tr > 0:
        s = 2 * math.sqrt(tr + 1)
        return np.array([0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s])
    i = int(np.argmax(np.diag(R)))
    if i == 0:
        s = 2 * math.sqrt(1 + R[0, 0] - R[1, 1] - R[2, 2])
        return np.array([(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s])
    if i == 1:
        s = 2 * math.sqrt(1 + R[1, 1] - R[0, 0] - R[2, 2])
        return np.array([(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s])
    s = 2 * math.sqrt(1 + R[2, 2] - R[0, 0] - R[1, 1])
    return np.array([(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s])


# --------------------------------------------------------------------------- meshes
def load_stl(path):
    with open(path, "rb") as f:
        data = f.read()
    n = struct.unpack("<I", data[80:84])[0]
    if 84 + 50 * n == len(data):
        pts = []
        for i in range(n):
            off = 84 + 50 * i + 12
            pts.extend(struct.unpack("<9f", data[off:off + 36]))
        return np.array(pts, float).reshape(-1, 3)
    raise ValueError(f"ascii stl unsupported: {path}")


def load_obj(path):
    pts = []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                pts.append([float(x) for x in line.split()[1:4]])
    return np.array(pts, float)


def hull_of(points):
    pts = np.unique(np.round(points, 9), axis=0)
    h = ConvexHull(pts)
    verts = pts[h.vertices]
    remap = {int(v): i for i, v in enumerate(h.vertices)}
    faces = []
    for simplex, eq in zip(h.simplices, h.equations):
        tri = [remap[int(v)] for v in simplex]
        a, b, c = verts[tri]
        if np.dot(np.cross(b - a, c - a), eq[:3]) < 0:
            tri = [tri[0], tri[2], tri[1]]
        faces.append(tri)
    return verts, faces, float(h.volume)


# --------------------------------------------------------------------------- MJCF
class Defaults:
    def __init__(self):
        self.classes = {"main": {k: dict(v) for k, v in MAIN_DEFAULTS.items()}}

    def parse(self, elem, parent="main"):
        name = elem.get("class", "main")
        base = {k: dict(v) for k, v in self.classes[parent].items()} if name != parent else self.classes[parent]
        for child in elem:
            if child.tag == "default":
                continue
            base.setdefault(child.tag, {}).update(child.attrib)
        self.classes[name] = base
        for child in elem:
            if child.tag == "default":
                self.parse(child, name)

    def get(self, cls, tag, elem):
        d = dict(self.classes[cls].get(tag, {}))
        d.update(elem.attrib)
        return d


def compile_model():
    scene = ET.parse(SCENE).getroot()
    panda = ET.parse(PANDA).getroot()
    defaults = Defaults()
    for d in panda.findall("default"):
        for c in d:
            if c.tag == "default":
                defaults.parse(c, "main")
    meshes_decl = {}
    for m in panda.find("asset").findall("mesh"):
        fname = m.get("file")
        name = m.get("name", os.path.splitext(fname)[0])
        meshes_decl[name] = os.path.join(REF_DATA, "franka_emika_panda", "assets", fname)

    bodies, joints, geoms, cameras = [], [], [], []
    bodies.append(dict(name="world", parent=-1, pos=[0, 0, 0], quat=[1, 0, 0, 0], mass=0.0,
                       ipos=[0, 0, 0], inertia=np.zeros((3, 3)).tolist(), jnts=[], geoms=[]))

    def walk(belem, parent_id, cls):
        bcls = belem.get("childclass", cls)
        pos = fl(belem.get("pos", "0 0 0"))
        quat = quat_norm(fl(belem.get("quat", "1 0 0 0"))).tolist()
        bid = len(bodies)
        body = dict(name=belem.get("name"), parent=parent_id, pos=pos, quat=quat, jnts=[], geoms=[],
                    mass=None, ipos=[0, 0, 0], inertia=None)
        bodies.append(body)
        inert = belem.find("inertial")
        if inert is not None:
            body["mass"] = float(inert.get("mass"))
            body["ipos"] = fl(inert.get("pos", "0 0 0"))
            if inert.get("fullinertia"):
                ixx, iyy, izz, ixy, ixz, iyz = fl(inert.get("fullinertia"))
                I = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])
            else:
                I = np.diag(fl(inert.get("diaginertia")))
                if inert.get("quat"):
                    R = quat2mat(fl(inert.get("quat")))
                    I = R @ I @ R.T
            body["inertia"] = I.tolist()
        for child in belem:
            ccls = child.get("class", bcls)
            if child.tag in ("joint", "freejoint"):
                if child.tag == "freejoint":
                    a = {"type": "free", "name": child.get("name")}
                else:
                    a = defaults.get(ccls, "joint", child)
                j = dict(name=a.get("name"), type=a.get("type", "hinge"), body=bid,
                         axis=fl(a.get("axis", "0 0 1")), pos=fl(a.get("pos", "0 0 0")),
                         armature=float(a.get("armature", 0)), damping=float(a.get("damping", 0)),
                         range=fl(a["range"]) if "range" in a else [0.0, 0.0])
                j["limited"] = 1 if ("range" in a and j["type"] != "free") else 0
                if j["type"] != "free":
                    ax = np.array(j["axis"], float)
                    j["axis"] = (ax / np.linalg.norm(ax)).tolist()
                body["jnts"].append(len(joints))
                joints.append(j)
            elif child.tag == "geom":
                a = defaults.get(ccls, "geom", child)
                gtype = a.get("type", "sphere")
                if "mesh" in a and "type" not in child.attrib and gtype == "sphere":
                    gtype = "mesh"
                g = dict(name=a.get("name"), type=gtype, body=bid,
                         pos=fl(a.get("pos", "0 0 0")), quat=quat_norm(fl(a.get("quat", "1 0 0 0"))).tolist(),
                         size=fl(a.get("size", "0 0 0")), contype=int(a.get("contype", 1)),
                         conaffinity=int(a.get("conaffinity", 1)), condim=int(a.get("condim", 3)),
                         friction=fl(a.get("friction")), solref=fl(a.get("solref")), solimp=fl(a.get("solimp")),
                         margin=float(a.get("margin")), gap=float(a.get("gap")),
                         mass=float(a["mass"]) if "mass" in a else None,
                         density=float(a.get("density", 1000)), mesh=a.get("mesh"))
                body["geoms"].append(len(geoms))
                geoms.append(g)
            elif child.tag == "camera":
                q = quat_norm(fl(child.get("quat", "1 0 0 0")))
                if child.get("xyaxes"):
                    q = xyaxes_to_quat(fl(child.get("xyaxes")))
                cameras.append(dict(name=child.get("name"), body=bid, pos=fl(child.get("pos", "0 0 0")),
                                    quat=q.tolist(), fovy=float(child.get("fovy", 45))))
            elif child.tag == "body":
                walk(child, bid, bcls)

    world_geoms = []
    # include (panda) worldbody first, then the scene's own worldbody
    for wb in (panda.find("worldbody"), scene.find("worldbody")):
        for child in wb:
            if child.tag == "body":
                walk(child, 0, "main")
            elif child.tag == "geom":
                a = defaults.get("main", "geom", child)
                g = dict(name=a.get("name"), type=a.get("type"), body=0, pos=fl(a.get("pos", "0 0 0")),
                         quat=quat_norm(fl(a.get("quat", "1 0 0 0"))).tolist(), size=fl(a.get("size")),
                         contype=int(a["contype"]), conaffinity=int(a["conaffinity"]), condim=int(a["condim"]),
                         friction=fl(a["friction"]), solref=fl(a["solref"]), solimp=fl(a["solimp"]),
                         margin=float(a["margin"]), gap=float(a["gap"]), mass=None, density=1000.0, mesh=None)
                world_geoms.append(g)
            elif child.tag == "camera":
                q = xyaxes_to_quat(fl(child.get("xyaxes"))) if child.get("xyaxes") else quat_norm(fl(child.get("quat", "1 0 0 0")))
                cameras.append(dict(name=child.get("name"), body=0, pos=fl(child.get("pos", "0 0 0")),
                                    quat=q.tolist(), fovy=float(child.get("fovy", 45))))
    # world geoms come first in geom order (body 0)
    for g in geoms:
        pass
    ng_world = len(world_geoms)
    for b in bodies:
        b["geoms"] = [gi + ng_world for gi in b["geoms"]]
    geoms = world_geoms + geoms
    bodies[0]["geoms"] = list(range(ng_world))

    # wrist camera injected by env.py:52-65 via MjSpec (gym env only)
    hand_id = [b["name"] for b in bodies].index("hand")
    cameras.append(dict(name="wrist", body=hand_id, pos=[-0.07, 0.0, 0.055],
                        quat=quat_norm([-0.0616, -0.7044, 0.7044, 0.0616]).tolist(), fovy=128.0))

    # ------------------------------------------------------------- collision set
    mesh_list, mesh_index = [], {}
    col_geoms = [i for i, g in enumerate(geoms) if (g["contype"] or g["conaffinity"])]
    for gi in col_geoms:
        g = geoms[gi]
        if g["type"] == "mesh":
            name = g["mesh"]
            if name not in mesh_index:
                path = meshes_decl[name]
                pts = load_stl(path) if path.endswith(".stl") else load_obj(path)
                verts, faces, vol = hull_of(pts)
                mesh_index[name] = len(mesh_list)
                mesh_list.append(dict(name=name, verts=verts, faces=faces, volume=vol))

    # inertia from geoms for bodies without <inertial> (cubes; static bodies irrelevant)
    for b in bodies[1:]:
        if b["mass"] is None:
            m_tot, I_tot, c_acc = 0.0, np.zeros((3, 3)), np.zeros(3)
            parts = []
            for gi in b["geoms"]:
                g = geoms[gi]
                if not (g["contype"] or g["conaffinity"]) and g["type"] == "mesh":
                    continue
                if g["type"] == "box":
                    sx, sy, sz = [2 * s for s in g["size"][:3]]
                    m = g["mass"] if g["mass"] is not None else g["density"] * sx * sy * sz
                    Ig = m / 12.0 * np.diag([sy * sy + sz * sz, sx * sx + sz * sz, sx * sx + sy * sy])
                elif g["type"] == "cylinder":
                    r, h = g["size"][0], 2 * g["size"][1]
                    m = g["mass"] if g["mass"] is not None else g["density"] * math.pi * r * r * h
                    Ig = np.diag([m * (3 * r * r + h * h) / 12, m * (3 * r * r + h * h) / 12, m * r * r / 2])
                else:
                    continue
                R = quat2mat(g["quat"])
                parts.append((m, np.array(g["pos"]), R @ Ig @ R.T))
            for m, c, Ig in parts:
                m_tot += m
                c_acc += m * c
            com = c_acc / m_tot if m_tot > 0 else np.zeros(3)
            for m, c, Ig in parts:
                d = c - com
                I_tot += Ig + m * (d.dot(d) * np.eye(3) - np.outer(d, d))
            b["mass"] = m_tot
            b["ipos"] = com.tolist()
            b["inertia"] = I_tot.tolist()

    # weld ids (a body without joints is welded to its parent's weld)
    for bid, b in enumerate(bodies):
        if bid == 0:
            b["weld"] = 0
        else:
            b["weld"] = bid if b["jnts"] else bodies[b["parent"]]["weld"]
    for bid, b in enumerate(bodies):
        b["root"] = 0 if bid == 0 else (bid if b["parent"] == 0 else bodies[b["parent"]]["root"])

    # qpos / dof addressing
    qadr = dadr = 0
    for j in joints:
        j["qposadr"], j["dofadr"] = qadr, dadr
        nq, nd = {"free": (7, 6), "hinge": (1, 1), "slide": (1, 1)}[j["type"]]
        j["nq"], j["nv"] = nq, nd
        qadr += nq
        dadr += nd
    nq, nv = qadr, dadr

    # keyframe scene_start (pick_and_place_scene.xml:130-135)
    key = scene.find("keyframe").find("key")
    key_qpos = fl(key.get("qpos"))
    key_ctrl = fl(key.get("ctrl"))
    assert len(key_qpos) == nq

    # qpos0: hinge/slide 0, free = body pos + quat
    qpos0 = np.zeros(nq)
    for j in joints:
        if j["type"] == "free":
            b = bodies[j["body"]]
            qpos0[j["qposadr"]:j["qposadr"] + 3] = b["pos"]
            qpos0[j["qposadr"] + 3:j["qposadr"] + 7] = b["quat"]

    # actuators (panda.xml:264-278), defaults class panda
    actuators = []
    for a in panda.find("actuator"):
        d = defaults.get(a.get("class", "main"), "general", a)
        act = dict(name=d["name"], gain=fl(d["gainprm"])[0], bias=(fl(d["biasprm"]) + [0, 0, 0])[:3],
                   ctrlrange=fl(d["ctrlrange"]), forcerange=fl(d["forcerange"]),
                   ctrllimited=1 if "ctrlrange" in d else 0, forcelimited=1 if "forcerange" in d else 0)
        if "joint" in d:
            act["trn"] = "joint"
            act["target"] = [j["name"] for j in joints].index(d["joint"])
        else:
            act["trn"] = "tendon"
            act["target"] = 0
        actuators.append(act)

    # tendon split (panda.xml:253-258)
    ten = panda.find("tendon").find("fixed")
    tendon = dict(name=ten.get("name"),
                  joints=[[j["name"] for j in joints].index(x.get("joint")) for x in ten.findall("joint")],
                  coef=[float(x.get("coef")) for x in ten.findall("joint")])

    # equality (panda.xml:260-262)
    eq = panda.find("equality").find("joint")
    equality = dict(j1=[j["name"] for j in joints].index(eq.get("joint1")),
                    j2=[j["name"] for j in joints].index(eq.get("joint2")),
                    polycoef=[0, 1, 0, 0, 0], solref=fl(eq.get("solref")),
                    solimp=(fl(eq.get("solimp")) + [0.5, 2])[:5])

    excludes = []
    for ex in panda.find("contact").findall("exclude"):
        names = [b["name"] for b in bodies]
        excludes.append(sorted([names.index(ex.get("body1")), names.index(ex.get("body2"))]))

    # geom local frames: meshes are re-centred on their hull AABB centre (pure
    # re-parameterisation of the same geometry in the body frame)
    for gi in col_geoms:
        g = geoms[gi]
        if g["type"] == "mesh":
            mesh = mesh_list[mesh_index[g["mesh"]]]
            g["meshid"] = mesh_index[g["mesh"]]
        else:
            g["meshid"] = -1

    for m in mesh_list:
        v = m["verts"]
        c = 0.5 * (v.min(0) + v.max(0))
        m["center"] = c
        m["verts_local"] = v - c
    for gi in col_geoms:
        g = geoms[gi]
        if g["type"] == "mesh":
            m = mesh_list[g["meshid"]]
            R = quat2mat(g["quat"])
            g["pos"] = (np.array(g["pos"]) + R @ m["center"]).tolist()
            half = np.abs(m["verts_local"]).max(0)
            g["aabb"] = half.tolist()
            g["rbound"] = float(np.linalg.norm(m["verts_local"], axis=1).max())
        elif g["type"] == "box":
            g["aabb"] = g["size"][:3]
            g["rbound"] = float(np.linalg.norm(g["size"][:3]))
        elif g["type"] == "cylinder":
            r, h = g["size"][0], g["size"][1]
            g["aabb"] = [r, r, h]
            g["rbound"] = float(math.hypot(r, h))
        elif g["type"] == "plane":
            g["aabb"] = [1e6, 1e6, 0.0]
            g["rbound"] = 0.0  # infinite plane: never culled by sphere test
        else:
            raise ValueError(g["type"])

    # candidate geom pairs (MuJoCo's filter: contype/conaffinity, same weld,
    # parent weld unless world, explicit excludes)
    pairs = []
    for ai in range(len(col_geoms)):
        for bi in range(ai + 1, len(col_geoms)):
            g1, g2 = col_geoms[ai], col_geoms[bi]
            G1, G2 = geoms[g1], geoms[g2]
            if not ((G1["contype"] & G2["conaffinity"]) or (G2["contype"] & G1["conaffinity"])):
                continue
            b1, b2 = G1["body"], G2["body"]
            w1, w2 = bodies[b1]["weld"], bodies[b2]["weld"]
            if w1 == w2:
                continue
            wp1 = bodies[bodies[w1]["parent"]]["weld"] if w1 else 0
            wp2 = bodies[bodies[w2]["parent"]]["weld"] if w2 else 0
            if w1 != 0 and w2 != 0 and (w1 == wp2 or w2 == wp1):
                continue
            if sorted([b1, b2]) in excludes:
                continue
            if G1["type"] == "plane" and G2["type"] == "plane":
                continue
            pairs.append([g1, g2])

    model = dict(bodies=bodies, joints=joints, geoms=geoms, meshes=mesh_list, cameras=cameras,
                 actuators=actuators, tendon=tendon, equality=equality, excludes=excludes,
                 col_geoms=col_geoms, pairs=pairs, nq=nq, nv=nv, qpos0=qpos0.tolist(),
                 key_qpos=key_qpos, key_ctrl=key_ctrl,
                 opt=dict(timestep=TIMESTEP, gravity=[0, 0, -9.81], integrator="implicitfast",
                          impratio=1.0, o_solref=[0.02, 1.0]))
    invweights(model)
    return model


# --------------------------------------------------------------------------- invweight0
def kinematics_np(model, qpos):
    bodies, joints = model["bodies"], model["joints"]
    nb = len(bodies)
    xpos = np.zeros((nb, 3))
    xmat = np.zeros((nb, 3, 3))
    xmat[0] = np.eye(3)
    xanchor, xaxis = {}, {}
    for bid in range(1, nb):
        b = bodies[bid]
        p = b["parent"]
        pos = xpos[p] + xmat[p] @ np.array(b["pos"])
        R = xmat[p] @ quat2mat(b["quat"])
        for ji in b["jnts"]:
            j = joints[ji]
            qa = j["qposadr"]
            if j["type"] == "free":
                pos = np.array(qpos[qa:qa + 3])
                R = quat2mat(qpos[qa + 3:qa + 7])
                xanchor[ji] = pos.copy()
            elif j["type"] == "hinge":
                anchor = pos + R @ np.array(j["pos"])
                axis = R @ np.array(j["axis"])
                ang = qpos[qa] - model["qpos0"][qa]
                Rj = axis_angle(axis, ang)
                R = Rj @ R
                pos = anchor + Rj @ (pos - anchor)
                xanchor[ji], xaxis[ji] = anchor, axis
            elif j["type"] == "slide":
                axis = R @ np.array(j["axis"])
                xanchor[ji], xaxis[ji] = pos + R @ np.array(j["pos"]), axis
                pos = pos + axis * (qpos[qa] - model["qpos0"][qa])
        xpos[bid], xmat[bid] = pos, R
    xipos = np.array([xpos[i] + xmat[i] @ np.array(bodies[i]["ipos"]) for i in range(nb)])
    return xpos, xmat, xipos, xanchor, xaxis


def axis_angle(axis, ang):
    a = axis / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * K @ K


def body_jac(model, kin, bid, point):
    bodies, joints = model["bodies"], model["joints"]
    xpos, xmat, xipos, xanchor, xaxis = kin
    nv = model["nv"]
    jp, jr = np.zeros((3, nv)), np.zeros((3, nv))
    b = bid
    while b > 0:
        for ji in bodies[b]["jnts"]:
            j = joints[ji]
            da = j["dofadr"]
            if j["type"] == "free":
                jp[:, da:da + 3] = np.eye(3)
                for k in range(3):
                    ax = xmat[b][:, k]
                    jr[:, da + 3 + k] = ax
                    jp[:, da + 3 + k] = np.cross(ax, point - xanchor[ji])
            elif j["type"] == "hinge":
                jr[:, da] = xaxis[ji]
                jp[:, da] = np.cross(xaxis[ji], point - xanchor[ji])
            else:
                jp[:, da] = xaxis[ji]
        b = bodies[b]["parent"]
    return jp, jr


def mass_matrix_np(model, qpos):
    kin = kinematics_np(model, qpos)
    xpos, xmat, xipos = kin[:3]
    nv = model["nv"]
    M = np.zeros((nv, nv))
    for bid, b in enumerate(model["bodies"]):
        if bid == 0 or b["mass"] is None:
            continue
        jp, jr = body_jac(model, kin, bid, xipos[bid])
        Iw = xmat[bid] @ np.array(b["inertia"]) @ xmat[bid].T
        M += b["mass"] * jp.T @ jp + jr.T @ Iw @ jr
    for j in model["joints"]:
        for k in range(j["nv"]):
            M[j["dofadr"] + k, j["dofadr"] + k] += j["armature"]
    return M, kin


def invweights(model):
    M, kin = mass_matrix_np(model, np.array(model["qpos0"]))
    Minv = np.linalg.inv(M)
    binv = []
    for bid, b in enumerate(model["bodies"]):
        if bid == 0 or b["weld"] == 0:
            binv.append([0.0, 0.0])
            continue
        jp, jr = body_jac(model, kin, bid, kin[2][bid])
        J = np.vstack([jp, jr])
        A = J @ Minv @ J.T
        binv.append([max(1e-15, float(np.trace(A[:3, :3]) / 3)), max(1e-15, float(np.trace(A[3:, 3:]) / 3))])
    dinv = np.zeros(model["nv"])
    for j in model["joints"]:
        da = j["dofadr"]
        if j["type"] == "free":
            dinv[da:da + 3] = np.trace(Minv[da:da + 3, da:da + 3]) / 3
            dinv[da + 3:da + 6] = np.trace(Minv[da + 3:da + 6, da + 3:da + 6]) / 3
        else:
            dinv[da] = Minv[da, da]
    model["body_invweight0"] = binv
    model["dof_invweight0"] = dinv.tolist()
    # mj_setConst's m->stat.meaninertia: the mean diagonal of qM (armature included) at qpos0; the
    # Newton solver's convergence tests scale by 1 / (meaninertia * nv)
    model["meaninertia"] = float(np.trace(M) / model["nv"])


# --------------------------------------------------------------------------- emit
GEOM_TYPE = {"plane": 0, "cylinder": 5, "box": 6, "mesh": 7}
JNT_TYPE = {"free": 0, "slide": 2, "hinge": 3}


def to_jsonable(model):
    out = {}
    for k, v in model.items():
        out[k] = v
    out["meshes"] = [dict(name=m["name"], verts=m["verts_local"].tolist(), faces=m["faces"],
                          volume=m["volume"]) for m in model["meshes"]]
    return out


QUAL = "static const"


def c_array(name, ctype, values, fmt="{:.17g}"):
    flat = np.asarray(values).ravel().tolist()
    body = ", ".join(fmt.format(x) if ctype in ("double", "float") else str(int(x)) for x in flat)
    if ctype == "float":
        body = ", ".join((repr(float(np.float32(x))) + "f") for x in flat)
    return f"{QUAL} {ctype} {name}[{len(flat)}] = {{{body}}};\n"


def device_tables(model, P, R):
    """Extra tables for the device kernels: static geom world poses, body bounding
    spheres and the candidate pairs grouped by body pair (hierarchical broadphase)."""
    bodies, geoms = model["bodies"], model["geoms"]
    col = model["col_geoms"]
    cid = {g: i for i, g in enumerate(col)}
    kin = kinematics_np(model, np.array(model["key_qpos"]))
    xpos, xmat = kin[0], kin[1]
    L = []
    sx, sm = [], []
    for g in col:
        G = geoms[g]
        b = G["body"]
        p = xpos[b] + xmat[b] @ np.array(G["pos"])
        Rm = xmat[b] @ quat2mat(G["quat"])
        sx.append(p.tolist())
        sm.append(Rm.ravel().tolist())
    L.append(c_array(f"{P}geom_static_xpos", R, sx))
    L.append(c_array(f"{P}geom_static_xmat", R, sm))
    L.append(c_array(f"{P}geom_lmat", R, [quat2mat(geoms[g]["quat"]).ravel().tolist() for g in col]))
    L.append(c_array(f"{P}body_static", "int", [1 if b["weld"] == 0 else 0 for b in bodies]))
    # body bounding spheres (body frame for moving bodies, world frame for static ones)
    spheres = []
    for bid, b in enumerate(bodies):
        gl = [cid[g] for g in b["geoms"] if g in cid]
        if not gl or bid == 0:
            spheres.append([0, 0, 0, 0])
            continue
        cs = np.array([geoms[col[i]]["pos"] for i in gl])
        rs = np.array([geoms[col[i]]["rbound"] for i in gl])
        lo, hi = (cs - rs[:, None]).min(0), (cs + rs[:, None]).max(0)
        c = 0.5 * (lo + hi)
        r = float(max(np.linalg.norm(cs - c, axis=1) + rs))
        if b["weld"] == 0:
            c = xpos[bid] + xmat[bid] @ c
        spheres.append(c.tolist() + [r])
    L.append(c_array(f"{P}body_bsphere", R, spheres))
    # group pairs by body pair
    groups = {}
    for a, bb in model["pairs"]:
        key = (geoms[a]["body"], geoms[bb]["body"])
        groups.setdefault(key, []).append((cid[a], cid[bb]))
    bp, pl = [], []
    for (b1, b2), lst in groups.items():
        bp.append([b1, b2, len(pl), len(lst)])
        pl.extend(lst)
    L.append(f"#define {P}NBODYPAIR {len(bp)}\n")
    L.append(c_array(f"{P}bodypair", "int", bp))
    L.append(c_array(f"{P}bodypair_geoms", "int", pl))
    # the same pairs packed g1 | g2 << 8 with the lower geom type first (narrowphase dispatch order)
    L.append(c_array(f"{P}pair_packed", "int", [pack_pair(a, b, model) for a, b in pl]))
    return L


def pack_pair(a, b, model):
    col, geoms = model["col_geoms"], model["geoms"]
    ta, tb = GEOM_TYPE[geoms[col[a]]["type"]], GEOM_TYPE[geoms[col[b]]["type"]]
    if ta > tb:
        a, b = b, a
    return a | (b << 8)


def emit_header(model, path, real, prefix, guard):
    """Emit the compiled model as C arrays (geoms restricted to colliding ones)."""
    bodies, joints, geoms = model["bodies"], model["joints"], model["geoms"]
    col = model["col_geoms"]
    cid = {g: i for i, g in enumerate(col)}
    nb, nj, ng = len(bodies), len(joints), len(col)
    global QUAL
    QUAL = "MMX_MODEL_QUAL" if prefix == "MMX_" else "static const"
    L = [f"/* GENERATED by tools/compile_model.py from the reference MJCF\n"
         f" * (mujoco_manip/data/pick_and_place_scene.xml + franka_emika_panda/panda.xml).\n"
         f" * Data only; do not edit. */\n",
         f"#ifndef {guard}\n#define {guard}\n\n"]
    if prefix == "MMX_":
        L.append("#ifndef MMX_MODEL_QUAL\n#define MMX_MODEL_QUAL static const\n#endif\n\n")
    P = prefix
    L.append(f"#define {P}NBODY {nb}\n#define {P}NJNT {nj}\n#define {P}NQ {model['nq']}\n#define {P}NV {model['nv']}\n")
    L.append(f"#define {P}NGEOM {ng}\n#define {P}NMESH {len(model['meshes'])}\n#define {P}NPAIR {len(model['pairs'])}\n")
    L.append(f"#define {P}NU {len(model['actuators'])}\n#define {P}NCAM {len(model['cameras'])}\n\n")
    R = real
    L.append(c_array(f"{P}body_parent", "int", [b["parent"] for b in bodies]))
    L.append(c_array(f"{P}body_weld", "int", [b["weld"] for b in bodies]))
    L.append(c_array(f"{P}body_jnt", "int", [b["jnts"][0] if b["jnts"] else -1 for b in bodies]))
    L.append(c_array(f"{P}body_pos", R, [b["pos"] for b in bodies]))
    L.append(c_array(f"{P}body_quat", R, [b["quat"] for b in bodies]))
    L.append(c_array(f"{P}body_mass", R, [b["mass"] for b in bodies]))
    L.append(c_array(f"{P}body_ipos", R, [b["ipos"] for b in bodies]))
    L.append(c_array(f"{P}body_inertia", R, [b["inertia"] for b in bodies]))
    L.append(c_array(f"{P}body_invweight0", R, model["body_invweight0"]))
    L.append(c_array(f"{P}jnt_type", "int", [JNT_TYPE[j["type"]] for j in joints]))
    L.append(c_array(f"{P}jnt_body", "int", [j["body"] for j in joints]))
    L.append(c_array(f"{P}jnt_qposadr", "int", [j["qposadr"] for j in joints]))
    L.append(c_array(f"{P}jnt_dofadr", "int", [j["dofadr"] for j in joints]))
    L.append(c_array(f"{P}jnt_axis", R, [j["axis"] for j in joints]))
    L.append(c_array(f"{P}jnt_pos", R, [j["pos"] for j in joints]))
    L.append(c_array(f"{P}jnt_range", R, [j["range"] for j in joints]))
    L.append(c_array(f"{P}jnt_limited", "int", [j["limited"] for j in joints]))
    dof_arm = []
    dof_damp = []
    dof_body = []
    dof_jnt = []
    for ji, j in enumerate(joints):
        for k in range(j["nv"]):
            dof_arm.append(j["armature"])
            dof_damp.append(j["damping"])
            dof_body.append(j["body"])
            dof_jnt.append(ji)
    L.append(c_array(f"{P}dof_armature", R, dof_arm))
    L.append(c_array(f"{P}dof_damping", R, dof_damp))
    L.append(c_array(f"{P}dof_body", "int", dof_body))
    L.append(c_array(f"{P}dof_jnt", "int", dof_jnt))
    L.append(c_array(f"{P}dof_invweight0", R, model["dof_invweight0"]))
    L.append(c_array(f"{P}qpos0", R, model["qpos0"]))
    L.append(f"#define {P}MEANINERTIA {model['meaninertia']:.17g}\n")
    L.append(c_array(f"{P}key_qpos", R, model["key_qpos"]))
    L.append(c_array(f"{P}key_ctrl", R, model["key_ctrl"]))
    # geoms (colliding only, renumbered)
    L.append(c_array(f"{P}geom_type", "int", [GEOM_TYPE[geoms[g]["type"]] for g in col]))
    L.append(c_array(f"{P}geom_body", "int", [geoms[g]["body"] for g in col]))
    L.append(c_array(f"{P}geom_pos", R, [geoms[g]["pos"] for g in col]))
    L.append(c_array(f"{P}geom_quat", R, [geoms[g]["quat"] for g in col]))
    L.append(c_array(f"{P}geom_size", R, [(geoms[g]["size"] + [0, 0, 0])[:3] for g in col]))
    L.append(c_array(f"{P}geom_aabb", R, [geoms[g]["aabb"] for g in col]))
    L.append(c_array(f"{P}geom_rbound", R, [geoms[g]["rbound"] for g in col]))
    # the kernel stores a contact as 4 basis rows and forms the pyramid edges from the tangent rows
    # (mmx_kernels.hip edge_coef): a frictionless (condim 1) contact would get no edge at all
    bad = [geoms[g].get("name", g) for g in col if geoms[g]["condim"] not in (3, 4)]
    if bad:
        raise SystemExit(f"compile_model: condim must be 3 or 4 for every colliding geom (kernel contact rows), got {bad}")
    L.append(c_array(f"{P}geom_condim", "int", [geoms[g]["condim"] for g in col]))
    L.append(c_array(f"{P}geom_friction", R, [geoms[g]["friction"] for g in col]))
    L.append(c_array(f"{P}geom_solref", R, [geoms[g]["solref"] for g in col]))
    L.append(c_array(f"{P}geom_solimp", R, [geoms[g]["solimp"] for g in col]))
    L.append(c_array(f"{P}geom_mesh", "int", [geoms[g]["meshid"] for g in col]))
    # meshes: concatenated hull vertices
    vadr, vnum, verts = [], [], []
    for m in model["meshes"]:
        vadr.append(len(verts))
        vnum.append(len(m["verts_local"]))
        verts.extend(m["verts_local"].tolist())
    L.append(f"#define {P}NMESHVERT {len(verts)}\n")
    L.append(c_array(f"{P}mesh_vertadr", "int", vadr))
    L.append(c_array(f"{P}mesh_vertnum", "int", vnum))
    L.append(c_array(f"{P}mesh_vert", R, verts))
    # pairs in renumbered geom ids
    L.append(c_array(f"{P}pair_geom", "int", [[cid[a], cid[b]] for a, b in model["pairs"]]))
    # actuators
    acts = model["actuators"]
    L.append(c_array(f"{P}act_trn_joint", "int", [a["target"] if a["trn"] == "joint" else -1 for a in acts]))
    L.append(c_array(f"{P}act_gain", R, [a["gain"] for a in acts]))
    L.append(c_array(f"{P}act_bias", R, [a["bias"] for a in acts]))
    L.append(c_array(f"{P}act_ctrlrange", R, [a["ctrlrange"] for a in acts]))
    L.append(c_array(f"{P}act_forcerange", R, [a["forcerange"] for a in acts]))
    t = model["tendon"]
    L.append(c_array(f"{P}tendon_jnt", "int", t["joints"]))
    L.append(c_array(f"{P}tendon_coef", R, t["coef"]))
    e = model["equality"]
    L.append(c_array(f"{P}eq_jnt", "int", [e["j1"], e["j2"]]))
    L.append(c_array(f"{P}eq_solref", R, e["solref"]))
    L.append(c_array(f"{P}eq_solimp", R, e["solimp"]))
    cams = model["cameras"]
    L.append(c_array(f"{P}cam_body", "int", [c["body"] for c in cams]))
    L.append(c_array(f"{P}cam_pos", R, [c["pos"] for c in cams]))
    L.append(c_array(f"{P}cam_quat", R, [c["quat"] for c in cams]))
    L.append(c_array(f"{P}cam_fovy", R, [c["fovy"] for c in cams]))
    # named ids used by the task layer
    names = [b["name"] for b in bodies]
    for nm in ["hand", "obj_red", "obj_green", "obj_blue", "bin_red", "bin_green", "bin_blue", "table"]:
        L.append(f"#define {P}BODY_{nm.upper()} {names.index(nm)}\n")
    camn = [c["name"] for c in cams]
    L.append(f"#define {P}CAM_OVERHEAD {camn.index('overhead')}\n#define {P}CAM_WRIST {camn.index('wrist')}\n")
    # robot / obstacle classification for the staged collision penalty (gym_env.py:137-152)
    robot_names = {"link0", "link1", "link2", "link3", "link4", "link5", "link6", "link7", "hand",
                   "left_finger", "right_finger"}
    objs = {"obj_red", "obj_green", "obj_blue"}
    gclass = []
    for g in col:
        bn = names[geoms[g]["body"]]
        if bn in robot_names:
            gclass.append(1)
        elif bn != "world" and bn not in objs:
            gclass.append(2)
        else:
            gclass.append(0)
    L.append(c_array(f"{P}geom_class", "int", gclass))
    if prefix == "MMX_":
        L.extend(device_tables(model, P, R))
    L.append(f"\n#define {P}TIMESTEP {model['opt']['timestep']!r}\n#define {P}GRAVITY_Z (-9.81)\n")
    L.append(f"\n#endif /* {guard} */\n")
    with open(path, "w") as f:
        f.write("".join(L))


def main():
    model = compile_model()
    out_json = os.path.join(REPO, "mujoco_manip_amd", "model", "panda_pickplace.json")
    with open(out_json, "w") as f:
        json.dump(to_jsonable(model), f, separators=(",", ":"))
    emit_header(model, os.path.join(REPO, "mujoco_manip_amd", "csrc", "mmx_model_gen.h"), "float", "MMX_",
                "MMX_MODEL_GEN_H")
    emit_header(model, os.path.join(REPO, "oracle", "oracle_model_gen.h"), "double", "OM_", "ORACLE_MODEL_GEN_H")
    print(f"nbody={len(model['bodies'])} njnt={len(model['joints'])} nq={model['nq']} nv={model['nv']} "
          f"colgeoms={len(model['col_geoms'])} pairs={len(model['pairs'])} meshes={len(model['meshes'])} "
          f"hullverts={sum(len(m['verts']) for m in model['meshes'])}")
    print("body_invweight0", [(b['name'], w) for b, w in zip(model['bodies'], model['body_invweight0'])])
    print("dof_invweight0", model["dof_invweight0"])


if __name__ == "__main__":
    sys.exit(main())
