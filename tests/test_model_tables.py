"""Compiled model tables vs the MJCF.

The kernel (mmx_model_gen.h) and the oracle (oracle_model_gen.h) are generated from one compiled
model (tools/compile_model.py -> mujoco_manip_amd/model/panda_pickplace.json), so a compiler error
would pass every GPU-vs-oracle parity test.  These CPU tests check the compiled tables against
sources that do not go through the compiler:

* tests/golden/mjcf_raw.json: the reference MJCF read as plain XML by an independent script
  (tests/golden/make_mjcf_fixture.py) -- frames, inertials, joints with default classes,
  actuators, tendon, equality, keyframe, option, colliding primitive geoms;
* the oracle's CRBA mass matrix (or_physics.c crba) vs the compiler's Jacobian-sum mass matrix
  (compile_model.mass_matrix_np), a second algorithm for M, and invweight0 (mj_setConst,
  SURVEY A.4) recomputed from the oracle's M at qpos0;
* the two generated headers against each other and against the compiled JSON.
"""
from __future__ import annotations

import json
import os
import re
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

RAW = json.load(open(os.path.join(REPO, "tests", "golden", "mjcf_raw.json")))
MODEL = json.load(open(os.path.join(REPO, "mujoco_manip_amd", "model", "panda_pickplace.json")))
BODY = {b["name"]: (i, b) for i, b in enumerate(MODEL["bodies"])}
JOINT = {j["name"]: (i, j) for i, j in enumerate(MODEL["joints"])}


def _quat_close(a, b, tol=1e-9):
    a = np.asarray(a, float) / np.linalg.norm(a)
    b = np.asarray(b, float) / np.linalg.norm(b)
    return min(np.abs(a - b).max(), np.abs(a + b).max()) < tol


def test_body_tree_frames_and_inertials():
    assert set(RAW["bodies"]) <= set(BODY)
    for name, raw in RAW["bodies"].items():
        bid, b = BODY[name]
        parent = MODEL["bodies"][b["parent"]]["name"]
        assert parent == raw["parent"], name
        np.testing.assert_allclose(b["pos"], raw["pos"], atol=1e-12, err_msg=name)
        assert _quat_close(b["quat"], raw["quat"]), name
        if "mass" in raw:  # explicit <inertial>
            assert b["mass"] == pytest.approx(raw["mass"], rel=1e-12), name
            np.testing.assert_allclose(b["ipos"], raw["ipos"], atol=1e-12, err_msg=name)
            if "fullinertia" in raw:
                ixx, iyy, izz, ixy, ixz, iyz = raw["fullinertia"]
                I = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])
            else:
                I = np.diag(raw["diaginertia"])
            np.testing.assert_allclose(b["inertia"], I, rtol=1e-9, atol=1e-15, err_msg=name)
    # the cubes' inertia comes from their box geom (mass 0.05, half-size 0.02): m (b^2 + c^2) / 3
    for c in ("obj_red", "obj_green", "obj_blue"):
        g = RAW["bodies"][c]["geoms"][0]
        m, (hx, hy, hz) = g["mass"], g["size"]
        _, b = BODY[c]
        assert b["mass"] == pytest.approx(m)
        np.testing.assert_allclose(np.diag(b["inertia"]),
                                   [m * (hy * hy + hz * hz) / 3, m * (hx * hx + hz * hz) / 3,
                                    m * (hx * hx + hy * hy) / 3], rtol=1e-12)
        np.testing.assert_allclose(b["ipos"], 0.0, atol=1e-15)
    # static bodies are welded to the world; link0 has no joint, so it is welded too
    for name in ("table", "bin_red", "bin_green", "bin_blue", "link0"):
        assert MODEL["bodies"][BODY[name][0]]["weld"] == 0, name


def test_joints_with_default_classes():
    qadr = dadr = 0
    order = []
    for name, raw in RAW["bodies"].items():
        for j in raw["joints"]:
            order.append(j["name"])
            jid, cj = JOINT[j["name"]]
            assert MODEL["bodies"][cj["body"]]["name"] == name
            assert cj["type"] == j["type"], j["name"]
            if j["type"] == "free":
                assert (cj["nq"], cj["nv"], cj["limited"], cj["armature"], cj["damping"]) == (7, 6, 0, 0.0, 0.0)
                continue
            np.testing.assert_allclose(cj["axis"], j["axis"], atol=1e-12)
            np.testing.assert_allclose(cj["range"], j["range"], atol=1e-12)
            assert cj["limited"] == 1  # compiler autolimits="true" with a range
            assert (cj["armature"], cj["damping"]) == (j["armature"], j["damping"])
    assert len(order) == len(MODEL["joints"]) == 12
    # qpos / dof layout of SURVEY A.1: arm 0:7, fingers 7:9, cubes 9:16, 16:23, 23:30 (nv 27)
    for jid, j in enumerate(MODEL["joints"]):
        assert (j["qposadr"], j["dofadr"]) == (qadr, dadr), j["name"]
        qadr += j["nq"]
        dadr += j["nv"]
    assert (MODEL["nq"], MODEL["nv"]) == (qadr, dadr) == (30, 27)
    assert [MODEL["joints"][i]["name"] for i in range(9)] == [f"joint{k}" for k in range(1, 8)] + \
        ["finger_joint1", "finger_joint2"]


def test_actuators_tendon_equality_exclude():
    assert len(MODEL["actuators"]) == len(RAW["actuators"]) == 8
    for ca, ra in zip(MODEL["actuators"], RAW["actuators"]):
        assert ca["name"] == ra["name"]
        assert ra["biastype"] == "affine"
        assert ca["gain"] == pytest.approx(ra["gain"], rel=1e-12)
        np.testing.assert_allclose(ca["bias"], ra["bias"], rtol=1e-12)
        np.testing.assert_allclose(ca["ctrlrange"], ra["ctrlrange"], rtol=1e-12)
        np.testing.assert_allclose(ca["forcerange"], ra["forcerange"], rtol=1e-12)
        assert ca["ctrllimited"] == 1 and ca["forcelimited"] == 1
        if ra["joint"] is not None:
            assert ca["trn"] == "joint" and MODEL["joints"][ca["target"]]["name"] == ra["joint"]
        else:
            assert ca["trn"] == "tendon" and MODEL["tendon"]["name"] == ra["tendon"]
    ten = MODEL["tendon"]
    assert [[MODEL["joints"][j]["name"], c] for j, c in zip(ten["joints"], ten["coef"])] == RAW["tendon"]["joints"]
    eq = MODEL["equality"]
    assert (MODEL["joints"][eq["j1"]]["name"], MODEL["joints"][eq["j2"]]["name"]) == \
        (RAW["equality"]["joint1"], RAW["equality"]["joint2"])
    np.testing.assert_allclose(eq["solref"], RAW["equality"]["solref"])
    # unspecified solimp entries take MuJoCo's defaults (midpoint 0.5, power 2)
    np.testing.assert_allclose(eq["solimp"], RAW["equality"]["solimp"] + [0.5, 2.0])
    assert eq["polycoef"][:2] == [0, 1]
    assert [[MODEL["bodies"][a]["name"], MODEL["bodies"][b]["name"]] for a, b in MODEL["excludes"]] == RAW["exclude"]


def test_keyframe_option_and_qpos0():
    np.testing.assert_allclose(MODEL["key_qpos"], RAW["key_qpos"])
    np.testing.assert_allclose(MODEL["key_ctrl"], RAW["key_ctrl"])
    assert MODEL["opt"]["timestep"] == RAW["option"]["timestep"]
    np.testing.assert_allclose(MODEL["opt"]["gravity"], RAW["option"]["gravity"])
    assert MODEL["opt"]["integrator"] == RAW["option"]["integrator"] == "implicitfast"
    # qpos0: hinge/slide 0, free joints at the body's XML frame
    q0 = np.array(MODEL["qpos0"])
    np.testing.assert_allclose(q0[:9], 0.0)
    for k, c in enumerate(("obj_red", "obj_green", "obj_blue")):
        np.testing.assert_allclose(q0[9 + 7 * k:12 + 7 * k], RAW["bodies"][c]["pos"])
        np.testing.assert_allclose(q0[12 + 7 * k:16 + 7 * k], RAW["bodies"][c]["quat"])


def test_colliding_primitive_geoms():
    """Boxes / cylinders / plane: size, local position, condim, friction (pads, cubes, scene)."""
    by_body = {}
    for g in MODEL["geoms"]:
        if g["contype"] or g["conaffinity"]:
            by_body.setdefault(MODEL["bodies"][g["body"]]["name"], []).append(g)
    ncol = 0
    for name, raw in RAW["bodies"].items():
        comp = by_body.get(name, [])
        assert len(comp) == len(raw["geoms"]), name
        ncol += len(comp)
        for cg, rg in zip(comp, raw["geoms"]):
            assert cg["type"] == rg["type"], name
            assert cg["condim"] == rg["condim"], name
            np.testing.assert_allclose(cg["friction"], rg["friction"], err_msg=name)
            if rg["type"] != "mesh":  # meshes are re-centred by the compiler, like MuJoCo's
                n = len(rg["size"])
                np.testing.assert_allclose(cg["size"][:n], rg["size"], err_msg=name)
                np.testing.assert_allclose(cg["pos"], rg["pos"], atol=1e-12, err_msg=name)
    floor = [g for g in MODEL["geoms"] if g["name"] == "floor"][0]
    np.testing.assert_allclose(floor["size"], RAW["world_geoms"][0]["size"])
    assert ncol + 1 == len(MODEL["col_geoms"]) == 47  # 47 colliding geoms incl. the floor


def _oracle_env():
    from oracle import oracle_py

    oracle_py.build()
    return oracle_py.OracleEnv()


@pytest.mark.parametrize("which", ["qpos0", "keyframe", "random"])
def test_mass_matrix_crba_vs_jacobian_sum(which):
    """The oracle's CRBA qM equals the compiler's sum of J' m J + Jr' I Jr + armature."""
    import compile_model

    env = _oracle_env()
    q = np.array(MODEL["qpos0"] if which == "qpos0" else MODEL["key_qpos"], float)
    if which == "random":
        rng = np.random.default_rng(7)
        for j in MODEL["joints"][:9]:
            lo, hi = j["range"]
            q[j["qposadr"]] = rng.uniform(lo, hi)
        for k in range(3):
            quat = rng.normal(size=4)
            q[12 + 7 * k:16 + 7 * k] = quat / np.linalg.norm(quat)
    env.set_state(qpos=q, qvel=np.zeros(27))
    env.mj_forward()
    M_oracle = env.mass_matrix()
    M_comp, _ = compile_model.mass_matrix_np(MODEL, q)
    np.testing.assert_allclose(M_oracle, M_comp, rtol=1e-10, atol=1e-12)
    assert np.all(np.linalg.eigvalsh(M_oracle) > 0)


def test_invweight0_from_oracle_mass_matrix():
    """mj_setConst's dof/body invweight0 at qpos0 from the oracle's M."""
    import compile_model

    env = _oracle_env()
    q0 = np.array(MODEL["qpos0"], float)
    env.set_state(qpos=q0, qvel=np.zeros(27))
    env.mj_forward()
    Minv = np.linalg.inv(env.mass_matrix())
    dinv = []
    for j in MODEL["joints"]:
        da = j["dofadr"]
        if j["type"] == "free":
            dinv += [np.trace(Minv[da:da + 3, da:da + 3]) / 3] * 3
            dinv += [np.trace(Minv[da + 3:da + 6, da + 3:da + 6]) / 3] * 3
        else:
            dinv.append(Minv[da, da])
    np.testing.assert_allclose(MODEL["dof_invweight0"], dinv, rtol=1e-9)
    # free cube: 1/m translational, 1/I rotational (0.05 kg, I = 1.333e-5)
    np.testing.assert_allclose(MODEL["dof_invweight0"][9:15], [20.0] * 3 + [75000.0] * 3, rtol=1e-9)
    kin = compile_model.kinematics_np(MODEL, q0)
    for bid, b in enumerate(MODEL["bodies"]):
        if b["weld"] == 0:
            assert MODEL["body_invweight0"][bid] == [0.0, 0.0]
            continue
        p, _ = env.body(bid)
        # the oracle's body frame agrees with the compiler's kinematics at qpos0
        np.testing.assert_allclose(p, kin[0][bid], atol=1e-12)
        jp, jr = compile_model.body_jac(MODEL, kin, bid, kin[2][bid])
        J = np.vstack([jp, jr])
        A = J @ Minv @ J.T
        np.testing.assert_allclose(MODEL["body_invweight0"][bid],
                                   [np.trace(A[:3, :3]) / 3, np.trace(A[3:, 3:]) / 3], rtol=1e-9)


_ARR = re.compile(r"(?:MMX_MODEL_QUAL|static const)\s+(int|float|double)\s+(?:MMX_|OM_)(\w+)\[(\d+)\]\s*=\s*\{([^}]*)\}")


def _tables(path):
    out = {}
    for typ, name, n, body in _ARR.findall(open(path).read()):
        vals = [v.strip().rstrip("f") for v in body.split(",") if v.strip()]
        arr = np.array([float(v) for v in vals])
        assert arr.size == int(n), name
        out[name] = (typ, arr)
    return out


def test_kernel_and_oracle_headers_agree():
    kern = _tables(os.path.join(REPO, "mujoco_manip_amd", "csrc", "mmx_model_gen.h"))
    orac = _tables(os.path.join(REPO, "oracle", "oracle_model_gen.h"))
    common = set(kern) & set(orac)
    assert len(common) >= 50, sorted(common)
    for name in sorted(common):
        tk, ak = kern[name]
        to, ao = orac[name]
        assert ak.shape == ao.shape, name
        if tk == "int":
            np.testing.assert_array_equal(ak, ao, err_msg=name)
        else:  # fp32 copy of the oracle's fp64 table
            np.testing.assert_allclose(ak, ao.astype(np.float32), rtol=0, atol=0, err_msg=name)
    # and the oracle header carries the compiled JSON's values
    np.testing.assert_allclose(orac["body_mass"][1], [b["mass"] for b in MODEL["bodies"]], rtol=1e-15)
    np.testing.assert_allclose(orac["body_inertia"][1], np.ravel([b["inertia"] for b in MODEL["bodies"]]),
                               rtol=1e-15)
    np.testing.assert_allclose(orac["dof_invweight0"][1], MODEL["dof_invweight0"], rtol=1e-15)
    np.testing.assert_allclose(orac["body_invweight0"][1], np.ravel(MODEL["body_invweight0"]), rtol=1e-15)
    np.testing.assert_allclose(orac["jnt_range"][1], np.ravel([j["range"] for j in MODEL["joints"]]))
    np.testing.assert_allclose(orac["act_gain"][1], [a["gain"] for a in MODEL["actuators"]])
    np.testing.assert_allclose(orac["act_bias"][1], np.ravel([a["bias"] for a in MODEL["actuators"]]))
    np.testing.assert_allclose(orac["key_qpos"][1], MODEL["key_qpos"])

