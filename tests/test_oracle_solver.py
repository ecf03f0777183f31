"""The Newton exit test against MuJoCo's own (CPU, oracle only).

MuJoCo's mj_solNewton stops after an iteration whose cost improvement or gradient norm, both scaled
by 1 / (meaninertia * nv) (mj_setConst's stat.meaninertia: the mean diagonal of qM at qpos0), falls
below opt.tolerance (1e-8 by default; the two quantities are what mjSolverStat records per
iteration as `improvement` / `gradient`).  The HIP solver and the oracle's parity mode use a relative
gradient test, |g| / (1 + |qfrc_smooth|) < tol (1e-6 on the GPU: fp32 cannot resolve MuJoCo's
scaled gradient of 1e-8).  These tests show that the iteration counts and trajectories of the two
tests agree on C3 expert episodes, i.e. the kernel's iteration count is MuJoCo's and not
inflated by its exit test.
"""
import os
import sys

import numpy as np

import oracle_py as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _episode(ep, tol, maxiter, mj_tol, steps=60):
    from mujoco_manip_amd.constants import ALL_TASKS, BINS, OBJECTS

    pool = [(OBJECTS.index(o), BINS.index(b)) for o, b in ALL_TASKS]
    e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=True, tasks=pool)
    e.set_solver(tol, maxiter)
    e.set_solver_mj(mj_tol)
    e.reset(seed=O.episode_seed(42, ep))
    o, b = e.task()
    e.fsm_init([(o, b)])
    for _ in range(steps):  # through the grasp and the lift (the phases with 2-3 iterations)
        if e.fsm_plan(16) == 10:
            break
        f = e.fsm_get()
        e.step(np.array([*f["target"], float(f["gripper_open"])], np.float32))
    calls, iters = e.solver_stats()
    return iters / calls, e.get_state()[0].copy()


def test_meaninertia_matches_model():
    import json

    m = json.load(open(os.path.join(REPO, "mujoco_manip_amd", "model", "panda_pickplace.json")))
    assert abs(m["meaninertia"] - 0.19166375415014703) < 1e-12  # trace(qM(qpos0)) / nv, armature included
    assert m["meaninertia"] > 0


def test_mujoco_exit_test_same_iterations_and_trajectory():
    for ep in (0, 1):
        it_rel, q_rel = _episode(ep, 1e-6, 30, 0.0)        # the GPU's relative test (at fp32's floor)
        it_mj, q_mj = _episode(ep, 0.0, 100, 1e-8)         # MuJoCo's tests only, its defaults
        it_conv, q_conv = _episode(ep, 1e-13, 200, 0.0)    # fully converged (the parity tests' oracle)
        assert 1.0 <= it_mj <= 3.0
        assert abs(it_rel - it_mj) / it_mj < 0.03, (it_rel, it_mj)
        np.testing.assert_allclose(q_mj, q_conv, atol=1e-6)
        np.testing.assert_allclose(q_rel, q_conv, atol=1e-4)
