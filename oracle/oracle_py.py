"""ORACLE ctypes binding — test infrastructure only.

Loads oracle/liboracle.so (the fp64 CPU restatement of the reference hot path, see
oracle/oracle.h).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module; the product (mujoco_manip_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

NQ, NV, NU = 30, 27, 8
ACTION_MODES = ("abs_pos", "ee_pos_quat_g", "ee_pos_rot6d_g", "ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel")
REWARD_TYPES = ("dense", "sparse", "staged")

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        fp = C.POINTER(C.c_float)
        ip = C.POINTER(C.c_int)
        L.or_create.restype = C.c_void_p
        L.or_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp, dp, C.c_int]
        L.or_destroy.argtypes = [C.c_void_p]
        L.or_set_task_pool.argtypes = [C.c_void_p, C.c_int, ip, ip]
        L.or_set_fixed_task.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.or_reset.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_int, C.c_int, fp]
        L.or_reset.restype = C.c_int
        L.or_step.restype = C.c_double
        L.or_step.argtypes = [C.c_void_p, fp, fp, ip, ip, ip, fp]
        for name in ("or_reset_keyframe", "or_mj_step", "or_mj_forward", "or_fsm_actuate"):
            getattr(L, name).argtypes = [C.c_void_p]
        L.or_ik_compute.argtypes = [C.c_void_p, dp, dp]
        L.or_ik_reached.restype = C.c_int
        L.or_ik_reached.argtypes = [C.c_void_p, dp]
        L.or_set_arm_ctrl.argtypes = [C.c_void_p, dp]
        L.or_set_gripper.argtypes = [C.c_void_p, C.c_int]
        L.or_fsm_init.argtypes = [C.c_void_p, C.c_int, ip, ip]
        L.or_fsm_plan.restype = C.c_int
        L.or_fsm_plan.argtypes = [C.c_void_p, C.c_int]
        L.or_fsm_get.argtypes = [C.c_void_p, ip, ip, ip, dp, ip]
        L.or_get_state.argtypes = [C.c_void_p, dp, dp, dp, dp]
        L.or_set_state.argtypes = [C.c_void_p, dp, dp, dp, dp]
        L.or_get_body.argtypes = [C.c_void_p, C.c_int, dp, dp]
        L.or_ncon.restype = C.c_int
        L.or_ncon.argtypes = [C.c_void_p]
        L.or_nefc.restype = C.c_int
        L.or_nefc.argtypes = [C.c_void_p]
        L.or_get_contact.argtypes = [C.c_void_p, C.c_int, ip, dp, dp, dp]
        L.or_get_efc_force.argtypes = [C.c_void_p, dp]
        L.or_solver_residual.restype = C.c_double
        L.or_solver_residual.argtypes = [C.c_void_p]
        L.or_get_qacc.argtypes = [C.c_void_p, dp]
        L.or_set_solver.argtypes = [C.c_void_p, C.c_double, C.c_int]
        L.or_set_solver_mj.argtypes = [C.c_void_p, C.c_double]
        L.or_solver_stats.argtypes = [C.c_void_p, C.POINTER(C.c_long), C.POINTER(C.c_long)]
        L.or_get_efc.restype = C.c_int
        L.or_get_efc.argtypes = [C.c_void_p, ip, dp, dp, dp]
        L.or_get_mass_matrix.argtypes = [C.c_void_p, dp]
        L.or_get_smooth.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp]
        L.or_get_obs.argtypes = [C.c_void_p, fp]
        L.or_get_initial_ee.argtypes = [C.c_void_p, dp]
        L.or_step_count.restype = C.c_int
        L.or_step_count.argtypes = [C.c_void_p]
        L.or_get_task.argtypes = [C.c_void_p, ip, ip]
        L.or_get_hwm.argtypes = [C.c_void_p, dp]
        L.or_orientation_error.argtypes = [dp, dp, dp]
        L.or_ik_math.argtypes = [dp, dp, dp, dp, dp, dp, dp]
        L.or_rotmat_to_quat_xyzw.argtypes = [dp, dp]
        L.or_quat_xyzw_to_rotmat.argtypes = [dp, dp]
        L.or_rotmat_from_6d.argtypes = [dp, dp]
        L.or_decode_action.argtypes = [C.c_int, fp, dp, dp, dp]
        L.or_seedseq_state.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_uint32), C.c_int,
                                       C.POINTER(C.c_uint32), C.c_int]
        L.or_pcg64_seed.argtypes = [C.c_void_p, C.c_uint64]
        L.or_pcg64_next64.restype = C.c_uint64
        L.or_pcg64_next64.argtypes = [C.c_void_p]
        L.or_pcg64_double.restype = C.c_double
        L.or_pcg64_double.argtypes = [C.c_void_p]
        L.or_pcg64_integers.restype = C.c_int64
        L.or_pcg64_integers.argtypes = [C.c_void_p, C.c_int64]
        L.or_episode_seed.restype = C.c_uint32
        L.or_episode_seed.argtypes = [C.c_uint64, C.c_int]
        L.or_sample_positions.restype = C.c_int
        L.or_sample_positions.argtypes = [C.c_void_p, dp, dp, C.c_double, dp]
        L.or_debug_set_xpos.argtypes = [C.c_void_p, C.c_int, dp]
        L.or_debug_set_contacts.argtypes = [C.c_void_p, C.c_int, ip]
        L.or_debug_set_episode.argtypes = [C.c_void_p, C.c_int, C.c_int, dp]
        L.or_debug_reward.restype = C.c_double
        L.or_debug_reward.argtypes = [C.c_void_p, ip]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class PCG64:
    """numpy-compatible Generator(PCG64(SeedSequence(seed))) restatement."""

    def __init__(self, seed: int):
        self._buf = C.create_string_buffer(48)
        lib().or_pcg64_seed(self._buf, seed)

    def next64(self) -> int:
        return lib().or_pcg64_next64(self._buf)

    def random(self) -> float:
        return lib().or_pcg64_double(self._buf)

    def integers(self, high: int) -> int:
        return lib().or_pcg64_integers(self._buf, high)

    def sample_positions(self, xr=(-0.2, 0.2), yr=(0.3, 0.45), min_sep=0.08):
        out = np.zeros(6)
        n = lib().or_sample_positions(self._buf, _d(np.array(xr, float)), _d(np.array(yr, float)), min_sep, _d(out))
        return out.reshape(3, 2), n


def seedseq_state(entropy, spawn_key=(), n_out=4):
    ent = np.array(entropy, dtype=np.uint32)
    sk = np.array(spawn_key, dtype=np.uint32) if len(spawn_key) else np.zeros(1, np.uint32)
    out = np.zeros(n_out, dtype=np.uint32)
    u32 = C.POINTER(C.c_uint32)
    lib().or_seedseq_state(ent.ctypes.data_as(u32), len(ent), sk.ctypes.data_as(u32), len(spawn_key),
                           out.ctypes.data_as(u32), n_out)
    return out


def episode_seed(root: int, index: int) -> int:
    return int(lib().or_episode_seed(root, index))


class OracleEnv:
    """Single-env fp64 oracle with the reference gym semantics."""

    def __init__(self, action_mode="abs_pos", reward_type="dense", max_episode_steps=500, randomize_objects=False,
                 spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45), image_size=224, tasks=None, task=None):
        L = lib()
        self._sx = np.array(spawn_x_range, float)
        self._sy = np.array(spawn_y_range, float)
        self.ptr = L.or_create(ACTION_MODES.index(action_mode), REWARD_TYPES.index(reward_type),
                               max_episode_steps, int(bool(randomize_objects)), _d(self._sx), _d(self._sy),
                               image_size)
        if tasks is not None:
            o = np.array([t[0] for t in tasks], np.int32)
            b = np.array([t[1] for t in tasks], np.int32)
            L.or_set_task_pool(self.ptr, len(tasks), _i(o), _i(b))
        if task is not None:
            L.or_set_fixed_task(self.ptr, task[0], task[1])

    def __del__(self):
        try:
            lib().or_destroy(self.ptr)
        except Exception:
            pass

    # gym level
    def reset(self, seed=None, task=None):
        obs = np.zeros(85, np.float32)
        to, tb = task if task is not None else (-1, -1)
        if lib().or_reset(self.ptr, int(seed is not None), int(seed or 0), to, tb, _f(obs)) < 0:
            # randomization.py:84-87
            raise RuntimeError("Failed to sample 3 positions with min_separation=0.08 in 1000 attempts")
        return obs

    def step(self, action):
        a = np.zeros(10, np.float32)
        act = np.asarray(action, np.float32)
        a[:len(act)] = act
        obs = np.zeros(85, np.float32)
        t, tr, s = (C.c_int(), C.c_int(), C.c_int())
        rc = np.zeros(6, np.float32)
        r = lib().or_step(self.ptr, _f(a), _f(obs), C.byref(t), C.byref(tr), C.byref(s), _f(rc))
        return obs, r, bool(t.value), bool(tr.value), {"success": bool(s.value), "reward_components": rc}

    # physics level
    def reset_keyframe(self):
        lib().or_reset_keyframe(self.ptr)

    def mj_step(self):
        lib().or_mj_step(self.ptr)

    def mj_forward(self):
        lib().or_mj_forward(self.ptr)

    def ik(self, target):
        q = np.zeros(7)
        lib().or_ik_compute(self.ptr, _d(np.asarray(target, float)), _d(q))
        return q

    def reached(self, target):
        return bool(lib().or_ik_reached(self.ptr, _d(np.asarray(target, float))))

    def set_arm_ctrl(self, q):
        lib().or_set_arm_ctrl(self.ptr, _d(np.asarray(q, float)))

    def set_gripper(self, open_):
        lib().or_set_gripper(self.ptr, int(open_))

    def fsm_init(self, tasks):
        o = np.array([t[0] for t in tasks], np.int32)
        b = np.array([t[1] for t in tasks], np.int32)
        lib().or_fsm_init(self.ptr, len(tasks), _i(o), _i(b))

    def fsm_plan(self, n=1):
        return lib().or_fsm_plan(self.ptr, n)

    def fsm_actuate(self):
        lib().or_fsm_actuate(self.ptr)

    def fsm_get(self):
        s, ti, st, go = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        tgt = np.zeros(3)
        lib().or_fsm_get(self.ptr, C.byref(s), C.byref(ti), C.byref(st), _d(tgt), C.byref(go))
        return dict(state=s.value, task_index=ti.value, settle=st.value, target=tgt, gripper_open=go.value)

    def get_state(self):
        qpos, qvel, ctrl, ws = np.zeros(NQ), np.zeros(NV), np.zeros(NU), np.zeros(NV)
        lib().or_get_state(self.ptr, _d(qpos), _d(qvel), _d(ctrl), _d(ws))
        return qpos, qvel, ctrl, ws

    def set_state(self, qpos=None, qvel=None, ctrl=None, qacc_ws=None):
        cur = self.get_state()
        vals = [np.ascontiguousarray(v if v is not None else c, dtype=float)
                for v, c in zip((qpos, qvel, ctrl, qacc_ws), cur)]
        lib().or_set_state(self.ptr, *[_d(v) for v in vals])

    def body(self, bid):
        p, R = np.zeros(3), np.zeros(9)
        lib().or_get_body(self.ptr, bid, _d(p), _d(R))
        return p, R.reshape(3, 3)

    def contacts(self):
        out = []
        for i in range(lib().or_ncon(self.ptr)):
            g = np.zeros(2, np.int32)
            dist = C.c_double()
            pos, frame = np.zeros(3), np.zeros(9)
            lib().or_get_contact(self.ptr, i, _i(g), C.byref(dist), _d(pos), _d(frame))
            out.append(dict(geom=tuple(g), dist=dist.value, pos=pos, frame=frame.reshape(3, 3)))
        return out

    def nefc(self):
        return lib().or_nefc(self.ptr)

    def efc_force(self):
        f = np.zeros(max(1, self.nefc()))
        lib().or_get_efc_force(self.ptr, _d(f))
        return f[:self.nefc()]

    def solver_residual(self):
        return lib().or_solver_residual(self.ptr)

    def set_solver(self, tol=1e-13, maxiter=200):
        """Newton tolerance / iteration cap (defaults: the parity tests' 1e-13 / 200; MuJoCo's own
        defaults are 1e-8 / 100)."""
        lib().or_set_solver(self.ptr, float(tol), int(maxiter))

    def set_solver_mj(self, mj_tol=1e-8):
        """MuJoCo's convergence tests at opt.tolerance (improvement / scaled gradient after each
        iteration); 0 turns them off (the parity tests' default)."""
        lib().or_set_solver_mj(self.ptr, float(mj_tol))

    def solver_stats(self):
        """(solves, Newton iterations) since creation."""
        c, i = C.c_long(), C.c_long()
        lib().or_solver_stats(self.ptr, C.byref(c), C.byref(i))
        return c.value, i.value

    def efc(self):
        """Constraint rows of the last solve: dict of type (0 equality, 1 limit, 2 contact edge),
        pos, R, aref arrays."""
        n = 640
        t, pos, R, aref = np.zeros(n, np.int32), np.zeros(n), np.zeros(n), np.zeros(n)
        m = lib().or_get_efc(self.ptr, _i(t), _d(pos), _d(R), _d(aref))
        return dict(type=t[:m], pos=pos[:m], R=R[:m], aref=aref[:m])

    def qacc(self):
        q = np.zeros(NV)
        lib().or_get_qacc(self.ptr, _d(q))
        return q

    def mass_matrix(self):
        """qM of the last forward (CRBA + armature), dense NV x NV."""
        M = np.zeros(NV * NV)
        lib().or_get_mass_matrix(self.ptr, _d(M))
        return M.reshape(NV, NV)

    def smooth(self):
        """Smooth-force terms of the last forward: qfrc_bias, qfrc_actuator, qfrc_passive,
        qacc_smooth, qfrc_constraint (NV each) and the clamped actuator forces (NU)."""
        out = [np.zeros(NV) for _ in range(5)] + [np.zeros(NU)]
        lib().or_get_smooth(self.ptr, *[_d(a) for a in out])
        return dict(zip(("bias", "actuator", "passive", "qacc_smooth", "constraint", "act_force"), out))

    def obs(self):
        o = np.zeros(85, np.float32)
        lib().or_get_obs(self.ptr, _f(o))
        return o

    def initial_ee(self):
        T = np.zeros(16)
        lib().or_get_initial_ee(self.ptr, _d(T))
        return T.reshape(4, 4)

    def task(self):
        o, b = C.c_int(), C.c_int()
        lib().or_get_task(self.ptr, C.byref(o), C.byref(b))
        return o.value, b.value

    def hwm(self):
        h = np.zeros(5)
        lib().or_get_hwm(self.ptr, _d(h))
        return h

    # test hooks
    def debug_set_xpos(self, body, p):
        lib().or_debug_set_xpos(self.ptr, body, _d(np.ascontiguousarray(p, float)))

    def debug_set_contacts(self, pairs):
        arr = np.array(pairs if len(pairs) else [[0, 0]], np.int32).ravel()
        lib().or_debug_set_contacts(self.ptr, len(pairs), _i(arr))

    def debug_set_episode(self, obj, bin_, T_init):
        lib().or_debug_set_episode(self.ptr, obj, bin_, _d(np.ascontiguousarray(T_init, float)))

    def debug_reward(self):
        s = C.c_int()
        r = lib().or_debug_reward(self.ptr, C.byref(s))
        return r, bool(s.value)

    @property
    def step_count(self):
        return lib().or_step_count(self.ptr)


# pure-math helpers
def orientation_error(Rc, Rt):
    out = np.zeros(3)
    lib().or_orientation_error(_d(np.ascontiguousarray(Rc, float)), _d(np.ascontiguousarray(Rt, float)), _d(out))
    return out


def ik_math(J, ee_pos, ee_xmat, q, target, jnt_range):
    out = np.zeros(7)
    args = [np.ascontiguousarray(x, float) for x in (J, ee_pos, ee_xmat, q, target, jnt_range)]
    lib().or_ik_math(*[_d(a) for a in args], _d(out))
    return out


def rotmat_to_quat_xyzw(R):
    q = np.zeros(4)
    lib().or_rotmat_to_quat_xyzw(_d(np.ascontiguousarray(R, float)), _d(q))
    return q


def quat_xyzw_to_rotmat(q):
    R = np.zeros(9)
    lib().or_quat_xyzw_to_rotmat(_d(np.ascontiguousarray(q, float)), _d(R))
    return R.reshape(3, 3)


def rotmat_from_6d(d6):
    R = np.zeros(9)
    lib().or_rotmat_from_6d(_d(np.ascontiguousarray(d6, float)), _d(R))
    return R.reshape(3, 3)


def decode_action(mode, action, T_init):
    a = np.zeros(10, np.float32)
    act = np.asarray(action, np.float32)
    a[:len(act)] = act
    tgt, g = np.zeros(3), C.c_double()
    lib().or_decode_action(ACTION_MODES.index(mode), _f(a), _d(np.ascontiguousarray(T_init, float)), _d(tgt),
                           C.byref(g))
    return tgt, g.value
