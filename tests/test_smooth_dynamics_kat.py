"""Known answers for the smooth dynamics and the non-contact constraint rows (VERDICT r04 missing #1).

Until r04 the smooth part of mj_step (env.py:119-121) was checked only oracle-vs-kernel, i.e. the
same restatement twice: RNE bias, servo clamping, the tendon gripper, joint-limit and equality rows
and implicitfast's M - h qDeriv.  Here every answer is derived in this file, independently of both
implementations under test, from

  * the raw MJCF (tests/golden/mjcf_raw.json, read by make_mjcf_fixture.py, not by
    tools/compile_model.py): body frames and inertials, joints (axis, armature, damping, range),
    actuators (gain, affine bias, ctrlrange, forcerange), the `split` tendon and the finger equality
    (panda.xml:4,9,144,159,178,253-278), forward kinematics by tests/collision_geometry.RawModel;
  * the equations MuJoCo publishes (documentation, "Computation"):
      - M(q) = sum over bodies of m Jv' Jv + Jw' I_world Jw + diag(armature), Jacobians at the
        centres of mass from the joint axes (hinge: a x (c - anchor), a; slide: a, 0);
      - qfrc_bias = c(q, qd) + g(q): gravity g = dV/dq with V = sum m g z_com (checked against
        central differences of V), the velocity term from the identity
        c = Mdot qd - 1/2 d(qd' M qd)/dq (central differences of M), for a free body
        gravity m g and the gyroscopic w x (I w) in body coordinates;
      - actuator force = gain ctrl + b0 + b1 length + b2 velocity (ctrl clamped to ctrlrange, force
        to forcerange), the tendon's moment 0.5 / 0.5 on the fingers; passive -damping qd;
      - soft constraints: impedance d(pos) from solimp, aref = -b (J qd) - k d pos,
        b = 2 / (dmax tau), k = 1 / (dmax^2 tau^2 zeta^2) (tau >= 2 h), R = (1 - d) / d * diag
        with diag = dof_invweight0 (= (M^-1)_dd at qpos0, mj_setConst); the equality row is
        two-sided, a limit row acts while J a < aref (the primal cost 1/2 D (J a - aref)^2);
      - implicitfast: qacc = (M - h qDeriv)^-1 (qfrc_smooth + qfrc_constraint) with
        qDeriv = -damping - kv of every actuator whose force is not clamped (the tendon's kv through
        its moment: a 2 x 2 finger block), then qvel += h qacc, qpos += h qvel.

Each scene runs on the fp64 oracle (CPU: the smooth-force terms themselves and the state after one
substep) and on the HIP kernel (`-m gpu`: the state after one substep through mmx_physics_step).
Mutation checks show the tolerances discriminate: a sign error in the tendon bias, a missing qDeriv
entry, the velocity term left out, a limit row's R from the wrong diag or explicit Euler all move
the answer by far more than the kernel's tolerance.
"""
import json
import os

import numpy as np
import pytest

from collision_geometry import ARM, RawModel, quat2mat

HERE = os.path.dirname(os.path.abspath(__file__))
RAW = json.load(open(os.path.join(HERE, "golden", "mjcf_raw.json")))
H = RAW["option"]["timestep"]
GRAV = -RAW["option"]["gravity"][2]
NV = 27
ARM_BODIES = ["link1", "link2", "link3", "link4", "link5", "link6", "link7", "hand", "left_finger", "right_finger"]
CUBE_FAR = [(1.0, -1.0, 1.0), (1.2, -1.0, 1.0), (1.4, -1.0, 1.0)]  # far from everything: no contact
DEF_SOLREF, DEF_SOLIMP = (0.02, 1.0), (0.9, 0.95, 0.001, 0.5, 2.0)
KERNEL_TOL_QVEL = 1e-5  # fp32 kernel vs the fp64 answer after one substep (r05 measured <= 7.2e-7: profiles/archive/r05_parity_margins_smooth.json)
ORACLE_TOL_QVEL = 1e-8


class SmoothModel:
    """The arm's smooth dynamics straight from the raw MJCF (independent of compile_model / oracle)."""

    def __init__(self):
        self.rm = RawModel()
        self.joints = {}  # arm dof -> (body, joint)
        for bname, b in self.rm._body_order():
            for j in b["joints"]:
                if j["type"] in ("hinge", "slide"):
                    self.joints[ARM.index(j["name"])] = (bname, j)
        self.armature = np.array([self.joints[d][1]["armature"] for d in range(9)])
        self.damping = np.array([self.joints[d][1]["damping"] for d in range(9)])
        self.range = np.array([self.joints[d][1]["range"] for d in range(9)])
        self.inert = {}
        for n in ARM_BODIES:
            b = RAW["bodies"][n]
            if "fullinertia" in b:
                ixx, iyy, izz, ixy, ixz, iyz = b["fullinertia"]
                I = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])
            else:
                I = np.diag(b["diaginertia"])
            self.inert[n] = (b["mass"], np.asarray(b["ipos"], float), I)
        cg = RAW["bodies"]["obj_red"]["geoms"][0]
        self.cube_m, hs = cg["mass"], np.asarray(cg["size"], float)
        self.cube_I = self.cube_m / 3.0 * np.array([hs[1] ** 2 + hs[2] ** 2, hs[0] ** 2 + hs[2] ** 2, hs[0] ** 2 + hs[1] ** 2])
        self.acts = RAW["actuators"]
        self.ten = {ARM.index(j): c for j, c in RAW["tendon"]["joints"]}
        eq = RAW["equality"]
        self.eq = (ARM.index(eq["joint1"]), ARM.index(eq["joint2"]), tuple(eq["solref"]),
                   tuple(eq["solimp"]) + DEF_SOLIMP[len(eq["solimp"]):])
        q0 = np.zeros(30)
        for k, c in enumerate(("obj_red", "obj_green", "obj_blue")):
            q0[9 + 7 * k:12 + 7 * k] = RAW["bodies"][c]["pos"]
            q0[12 + 7 * k:16 + 7 * k] = RAW["bodies"][c]["quat"]
        # mj_setConst: dof_invweight0 of a hinge / slide dof = (M^-1)_dd at qpos0
        self.invweight0 = np.diag(np.linalg.inv(self.mass_arm(q0)))

    def _ancestors(self, n):
        out = []
        while n != "world":
            out.append(n)
            n = RAW["bodies"][n]["parent"]
        return out

    def jac(self, pose, body, point):
        """(Jv, Jw), 3 x 9 each: the arm dofs' velocity Jacobian at a world point of `body`."""
        Jv, Jw = np.zeros((3, 9)), np.zeros((3, 9))
        anc = self._ancestors(body)
        for d, (bname, j) in self.joints.items():
            if bname not in anc:
                continue
            p, R = pose[bname]
            a = R @ np.asarray(j["axis"], float)  # a rotation about the axis leaves it unchanged
            if j["type"] == "hinge":
                Jv[:, d] = np.cross(a, point - p)  # the joint sits at the body origin (no pos)
                Jw[:, d] = a
            else:
                Jv[:, d] = a
        return Jv, Jw

    def com_terms(self, q):
        pose = self.rm.fk(q)
        out = []
        for n in ARM_BODIES:
            m, ipos, I = self.inert[n]
            p, R = pose[n]
            c = p + R @ ipos
            Jv, Jw = self.jac(pose, n, c)
            out.append((m, c, R @ I @ R.T, Jv, Jw))
        return out

    def mass_arm(self, q):
        M = np.diag(self.armature).astype(float)
        for m, _, Iw, Jv, Jw in self.com_terms(q):
            M += m * Jv.T @ Jv + Jw.T @ Iw @ Jw
        return M

    def potential(self, q):
        return sum(m * GRAV * c[2] for m, c, *_ in self.com_terms(q))

    def gravity(self, q):
        return sum(m * GRAV * Jv[2] for m, _, _, Jv, _ in self.com_terms(q))

    def coriolis(self, q, qd, eps=1e-5):
        """c(q, qd) = Mdot qd - 1/2 d(qd' M qd)/dq by central differences of M."""
        qd9 = qd[:9]

        def shifted(dq):
            qq = q.copy()
            qq[:9] += dq
            return self.mass_arm(qq)

        mdot = (shifted(eps * qd9) - shifted(-eps * qd9)) / (2 * eps)
        grad = np.array([qd9 @ (shifted(eps * e) - shifted(-eps * e)) @ qd9 / (2 * eps) for e in np.eye(9)])
        return mdot @ qd9 - 0.5 * grad

    def mass_full(self, q):
        M = np.zeros((NV, NV))
        M[:9, :9] = self.mass_arm(q)
        for c in range(3):
            d = 9 + 6 * c
            M[d:d + 3, d:d + 3] = np.eye(3) * self.cube_m
            M[d + 3:d + 6, d + 3:d + 6] = np.diag(self.cube_I)
        return M

    def bias(self, q, qd, mutate=()):
        b = np.zeros(NV)
        b[:9] = self.gravity(q) + (0.0 if "no_coriolis" in mutate else self.coriolis(q, qd))
        for c in range(3):
            d = 9 + 6 * c
            w = qd[d + 3:d + 6]
            b[d + 2] = self.cube_m * GRAV
            b[d + 3:d + 6] = np.cross(w, self.cube_I * w)
        return b

    def actuation(self, q, qd, ctrl, mutate=()):
        """qfrc_actuator, the clamped forces and which actuators are inside their forcerange."""
        qf, forces, free = np.zeros(NV), [], []
        for a, act in enumerate(self.acts):
            c = np.clip(ctrl[a], *act["ctrlrange"])
            b0, b1, b2 = act["bias"]
            if act["joint"] is not None:
                d = ARM.index(act["joint"])
                length, vel, moment = q[d], qd[d], {d: 1.0}
            else:
                length = sum(cf * q[d] for d, cf in self.ten.items())
                vel = sum(cf * qd[d] for d, cf in self.ten.items())
                moment = dict(self.ten)
                if "tendon_bias_sign" in mutate:
                    b1 = -b1
            f = act["gain"] * c + b0 + b1 * length + b2 * vel
            lo, hi = act["forcerange"]
            free.append(lo < f < hi)
            f = min(max(f, lo), hi)
            forces.append(f)
            for d, m in moment.items():
                qf[d] += m * f
        return qf, np.array(forces), free

    @staticmethod
    def impedance(solimp, pos):
        dmin, dmax, width, mid, p = solimp
        x = abs(pos) / width
        if x >= 1.0:
            return dmax
        y = x ** p / mid ** (p - 1) if x <= mid else 1.0 - (1.0 - x) ** p / (1.0 - mid) ** (p - 1)
        return dmin + y * (dmax - dmin)

    def row(self, J, pos, vel, diag, solref, solimp):
        d = self.impedance(solimp, pos)
        dmax = solimp[1]
        tau, zeta = max(solref[0], 2 * H), solref[1]
        k, b = 1.0 / (dmax * dmax * tau * tau * zeta * zeta), 2.0 / (dmax * tau)
        return dict(J=J, aref=-b * vel - k * d * pos, D=1.0 / ((1.0 - d) / d * diag), pos=pos, R=(1.0 - d) / d * diag)

    def rows(self, q, qd, mutate=()):
        j1, j2, sref, simp = self.eq
        J = np.zeros(NV)
        J[j1], J[j2] = 1.0, -1.0
        eq = self.row(J, q[j1] - q[j2], J @ qd, self.invweight0[j1] + self.invweight0[j2], sref, simp)
        lim = []
        for d in range(9):
            lo, hi = self.range[d]
            for sg, dist in ((1.0, q[d] - lo), (-1.0, hi - q[d])):
                if dist < 0:
                    J = np.zeros(NV)
                    J[d] = sg
                    diag = self.invweight0[d] * (2.0 if "limit_diag" in mutate else 1.0)
                    lim.append(self.row(J, dist, J @ qd, diag, DEF_SOLREF, DEF_SOLIMP))
        return eq, lim

    def answer(self, q, qd, ctrl, mutate=()):
        """The state after one mj_step (implicitfast) and the intermediate terms, fp64."""
        M = self.mass_full(q)
        bias = self.bias(q, qd, mutate)
        act, forces, free = self.actuation(q, qd, ctrl, mutate)
        passive = np.zeros(NV)
        passive[:9] = -self.damping * qd[:9]
        smooth = passive - bias + act
        a0 = np.linalg.solve(M, smooth)
        eq, lim = self.rows(q, qd, mutate)
        best = None
        for mask in range(1 << len(lim)):  # the active set of the one-sided limit rows
            act_rows = [eq] + [r for i, r in enumerate(lim) if (mask >> i) & 1]
            A, rhs = M.copy(), M @ a0
            for r in act_rows:
                A += r["D"] * np.outer(r["J"], r["J"])
                rhs += r["D"] * r["aref"] * r["J"]
            a = np.linalg.solve(A, rhs)
            if all(((r["J"] @ a < r["aref"]) == bool((mask >> i) & 1)) for i, r in enumerate(lim)):
                best = (a, act_rows)
                break
        assert best is not None, "no consistent active set"
        a, act_rows = best
        qfrc_con = sum(r["D"] * (r["aref"] - r["J"] @ a) * r["J"] for r in act_rows)
        MD = M.copy()
        if "explicit" not in mutate:
            MD[:9, :9] += H * np.diag(self.damping)
            for k, act_ in enumerate(self.acts):
                if not free[k]:
                    continue
                kv = -act_["bias"][2]
                if act_["joint"] is not None:
                    d = ARM.index(act_["joint"])
                    MD[d, d] += H * kv
                else:
                    t = np.zeros(NV)
                    for d, cf in self.ten.items():
                        t[d] = cf
                    blk = np.outer(t, t)
                    if "tendon_offdiag" in mutate:
                        blk = np.diag(np.diag(blk))
                    MD += H * kv * blk
        qacc = np.linalg.solve(MD, smooth + qfrc_con)
        qvel = qd + H * qacc
        qpos = q.copy()
        qpos[:9] += H * qvel[:9]
        return dict(qvel=qvel, qpos=qpos, qacc=qacc, bias=bias, actuator=act, passive=passive, act_force=forces,
                    free=free, qacc_smooth=a0, constraint=qfrc_con, rows=[eq] + lim, qacc_con=a)


_MODEL = None


def model():
    global _MODEL
    if _MODEL is None:
        _MODEL = SmoothModel()
    return _MODEL


def _qpos(arm9):
    q = np.array(RAW["key_qpos"], float)
    q[:9] = arm9
    for k, p in enumerate(CUBE_FAR):
        q[9 + 7 * k:12 + 7 * k] = p
        q[12 + 7 * k:16 + 7 * k] = (1.0, 0.0, 0.0, 0.0)
    return q


KEY = np.array(RAW["key_qpos"][:9], float)


def scenes():
    """name -> (qpos, qvel, ctrl): arm poses near the keyframe (clear of the table), cubes far away."""
    rng = np.random.default_rng(5)
    out = {}
    # gravity only: at rest, servos holding their position (zero force), gripper open at rest length
    q = _qpos(KEY + np.r_[0.2, -0.25, 0.3, 0.2, -0.4, 0.3, 0.5, 0.0, 0.0])
    out["gravity"] = (q, np.zeros(NV), np.r_[q[:7], 255.0])
    # velocity term: every arm joint moving, servos inside their force range, fingers apart
    q = _qpos(KEY + np.r_[-0.15, 0.1, -0.2, 0.25, 0.3, -0.2, -0.4, -0.01, -0.015])
    qd = np.zeros(NV)
    qd[:7] = rng.uniform(-1.5, 1.5, 7)
    qd[7:9] = (0.05, -0.03)
    # kp (ctrl - q) - kv qd stays inside +-87 / +-12: ctrl leads q by (kv / kp) qd (= 0.1 qd) + a little
    ctrl = np.r_[q[:7] + 0.1 * qd[:7] + rng.uniform(-0.003, 0.003, 7), 120.0]
    out["coriolis"] = (q, qd, ctrl)
    # saturation: servos 1, 2 (+-87) and 5, 6 (+-12) pushed past their force range, gripper tendon
    # force beyond +-100 (finger velocity), so their kv leaves qDeriv
    q = _qpos(KEY + np.r_[0.1, 0.05, -0.1, 0.1, 0.2, 0.1, -0.2, -0.005, -0.002])
    qd = np.zeros(NV)
    qd[:7] = (0.3, -0.2, 0.1, 0.4, -0.5, 0.2, 0.6)
    qd[7:9] = (-11.0, -13.0)
    ctrl = np.r_[q[:7] + np.r_[0.5, -0.4, 0.0, 0.01, 0.5, -0.5, 0.002], 0.0]
    out["saturation"] = (q, qd, ctrl)
    # joint limits: joint 4 past its upper limit (-0.0698) and moving further out fast enough that
    # its limit row acts although the (saturated) servo pulls back; both fingers past their upper
    # limit (0.04), opening further
    q = _qpos(np.r_[KEY[:3], -0.05, KEY[4:7], 0.043, 0.043])
    qd = np.zeros(NV)
    qd[3], qd[7], qd[8] = 3.0, 0.2, 0.2
    out["limits"] = (q, qd, np.r_[q[:7], 255.0])
    return out


def _oracle(q, qd, ctrl):
    import oracle_py as O

    e = O.OracleEnv()
    e.set_state(q, qd, ctrl, np.zeros(NV))
    e.mj_forward()
    return e


# --------------------------------------------------------------------------- the answers themselves
def test_answer_generator_self_checks():
    """The independent model agrees with itself: gravity = central differences of the potential;
    M is symmetric positive definite; the velocity term is quadratic in qd and does no work
    (qd' (Mdot qd - 2 c) = 0 is the skew identity's consequence qd' (Mdot - 2 C) qd = 0)."""
    sm = model()
    for name, (q, qd, _) in scenes().items():
        g = sm.gravity(q)
        fd = np.array([(sm.potential(q + 1e-6 * np.r_[e, np.zeros(21)]) - sm.potential(q - 1e-6 * np.r_[e, np.zeros(21)]))
                       / 2e-6 for e in np.eye(9)])
        np.testing.assert_allclose(g, fd, rtol=1e-7, atol=1e-8, err_msg=name)
        M = sm.mass_arm(q)
        np.testing.assert_allclose(M, M.T, atol=1e-14)
        assert np.linalg.eigvalsh(M).min() > 0
        c = sm.coriolis(q, qd)
        np.testing.assert_allclose(sm.coriolis(q, 2 * qd), 4 * c, rtol=1e-6, atol=1e-9)
        eps = 1e-5
        mdot = (sm.mass_arm(q + np.r_[eps * qd[:9], np.zeros(21)]) - sm.mass_arm(q - np.r_[eps * qd[:9], np.zeros(21)])) / (2 * eps)
        assert abs(qd[:9] @ (mdot @ qd[:9] - 2 * c)) < 1e-7 * (1 + abs(qd[:9] @ mdot @ qd[:9]))


def test_scenes_exercise_every_term():
    sm = model()
    sc = scenes()
    a = sm.answer(*sc["saturation"])
    assert not a["free"][0] and not a["free"][1] and not a["free"][4] and not a["free"][5]  # +-87, +-12
    assert not a["free"][7] and abs(a["act_force"][7]) == 100.0  # the tendon actuator at its forcerange
    assert all(sm.answer(*sc["coriolis"])["free"])
    al = sm.answer(*sc["limits"])
    lim = al["rows"][1:]
    assert len(lim) == 3 and {int(np.flatnonzero(r["J"])[0]) for r in lim} == {3, 7, 8}
    assert all(r["J"] @ al["qacc_con"] < r["aref"] for r in lim)  # both limit rows act
    assert np.abs(sm.answer(*sc["coriolis"])["bias"][:9] - sm.gravity(sc["coriolis"][0])).max() > 0.05


def test_mutations_exceed_the_kernel_tolerance():
    """Each modelling error the oracle and the kernel could share moves qvel after one substep by at
    least 20x the GPU tolerance, so the GPU test below can see it."""
    sm = model()
    sc = scenes()
    for scene, mut in (("coriolis", "no_coriolis"), ("coriolis", "tendon_bias_sign"), ("coriolis", "tendon_offdiag"),
                       ("coriolis", "explicit"), ("limits", "limit_diag"), ("saturation", "explicit")):
        base = sm.answer(*sc[scene])["qvel"]
        bad = sm.answer(*sc[scene], mutate=(mut,))["qvel"]
        assert np.abs(bad - base).max() > 20 * KERNEL_TOL_QVEL, (scene, mut, np.abs(bad - base).max())


# --------------------------------------------------------------------------- oracle (CPU, fp64)
@pytest.mark.parametrize("name", ["gravity", "coriolis", "saturation", "limits"])
def test_oracle_smooth_terms_and_step(name):
    """The oracle's RNE bias, actuator / passive forces, qacc_smooth, constraint rows and the state
    after one implicitfast substep against the independent answer."""
    sm = model()
    q, qd, ctrl = scenes()[name]
    want = sm.answer(q, qd, ctrl)
    e = _oracle(q, qd, ctrl)
    assert e.contacts() == [], "scene must be contact-free"
    got = e.smooth()
    np.testing.assert_allclose(got["bias"], want["bias"], rtol=1e-7, atol=1e-8)
    np.testing.assert_allclose(got["actuator"], want["actuator"], rtol=1e-12, atol=1e-10)
    np.testing.assert_allclose(got["act_force"], want["act_force"], rtol=1e-12, atol=1e-10)
    np.testing.assert_allclose(got["passive"], want["passive"], atol=1e-14)
    np.testing.assert_allclose(got["qacc_smooth"], want["qacc_smooth"], rtol=1e-7, atol=1e-7)
    np.testing.assert_allclose(e.mass_matrix(), sm.mass_full(q), rtol=1e-10, atol=1e-12)
    efc = e.efc()
    assert len(efc["type"]) == len(want["rows"])
    for r, typ, pos, R, aref in zip(want["rows"], efc["type"], efc["pos"], efc["R"], efc["aref"]):
        assert typ == (0 if r is want["rows"][0] else 1)
        assert abs(pos - r["pos"]) < 1e-14 and abs(R - r["R"]) < 1e-9 * r["R"] and abs(aref - r["aref"]) < 1e-8 * (1 + abs(r["aref"]))
    np.testing.assert_allclose(got["constraint"], want["constraint"], rtol=1e-6, atol=1e-7)
    e.mj_step()
    gq, gv, _, _ = e.get_state()
    np.testing.assert_allclose(gv, want["qvel"], atol=ORACLE_TOL_QVEL)
    np.testing.assert_allclose(gq[:9], want["qpos"][:9], atol=1e-10)


# --------------------------------------------------------------------------- HIP kernel (GPU, fp32)
@pytest.mark.gpu
def test_gpu_smooth_step_known_answers(margin):
    """The same scenes through mmx_physics_step (one substep, no IK, ctrl as given) on the kernel."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import _lib

    sm = model()
    sc = scenes()
    names = list(sc)
    n = len(names)
    qpos = np.stack([sc[k][0] for k in names]).astype(np.float32)
    qvel = np.stack([sc[k][1] for k in names]).astype(np.float32)
    ctrl = np.stack([sc[k][2] for k in names]).astype(np.float32)
    sim = _lib.Sim(n, action_mode="abs_pos", image_size=0)
    sim.set_state(qpos, qvel, ctrl, np.zeros((n, NV), np.float32))
    sim.physics_step(1, with_ik=False)
    gq, gv, _, _ = sim.get_state()
    epi = sim.view("episode_i", _lib.EPI_N, "<i4").cpu().numpy()
    sim.close()
    assert (epi[:, _lib.EPI["ncon"]] == 0).all() and (epi[:, _lib.EPI["env_error"]] == 0).all()
    worst = 0.0
    for k, name in enumerate(names):
        # the answer from the fp32 inputs the kernel actually saw
        want = sm.answer(qpos[k].astype(float), qvel[k].astype(float), ctrl[k].astype(float))
        dv = float(np.abs(gv[k] - want["qvel"]).max())
        dq = float(np.abs(gq[k, :9] - want["qpos"][:9]).max())
        margin(f"{name}_max_abs_dqvel", dv, KERNEL_TOL_QVEL)
        margin(f"{name}_max_abs_dqpos", dq, 1e-6)
        worst = max(worst, dv)
        assert dv < KERNEL_TOL_QVEL, (name, dv, np.abs(gv[k] - want["qvel"]))
        assert dq < 1e-6, (name, dq)
