"""GPU parity and behavioural tests (MI355X only), all through the C-ABI library libmmx.so.

Parity tiers (tolerances stated per test):
  L0  reset / RNG / observation codecs vs the fp64 oracle: fp32 rounding only;
  L1  physics (IK + CRBA/RNE + contacts + Newton + implicitfast) one substep and one env step
      (16 substeps) from states sampled along an oracle expert episode, incl. grasps;
  L2  multi-step env parity with expert actions, all 5 action modes;
  L3  the reference's own behavioural thresholds (tests/test_controller.py, test_gym_env.py,
      test_pick_and_place.py) run on the GPU batch.
The oracle is the checker only; every value under test comes out of the HIP kernels.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _require_gpu()
    from mujoco_manip_amd import _lib

    _lib.load(build_if_missing=False)  # the native library must be the one under test


TARGET_ORI = np.array([[0, 1, 0], [1, 0, 0], [0, 0, -1.0]])


def oracle_states(n=40):
    import oracle_py as O

    e = O.OracleEnv()
    e.reset_keyframe()
    e.fsm_init([(0, 0)])
    states = []
    for _ in range(200):
        st = e.fsm_plan(16)
        e.fsm_actuate()
        for _ in range(16):
            e.mj_step()
        states.append(e.get_state())
        if st == 10:
            break
    idx = np.linspace(0, len(states) - 1, n).astype(int)
    return [states[i] for i in idx]


def _physics_parity(nsub, sts=None, nefc_out=None):
    import oracle_py as O
    from mujoco_manip_amd import _lib

    sts = oracle_states() if sts is None else sts
    qpos, qvel, ctrl, ws = [np.stack([s[k] for s in sts]).astype(np.float32) for k in range(4)]
    sim = _lib.Sim(len(sts))
    sim.set_state(qpos, qvel, ctrl, ws)
    sim.physics_step(nsub)
    gq, gv, _, _ = sim.get_state()
    if nefc_out is not None:  # constraint rows of the run (summed over its substeps), per env
        nefc_out.append(sim.view("stats", _lib.STAT_N)[:, 0].cpu().numpy().copy())
    err_q, err_v = [], []
    for k in range(len(sts)):
        e = O.OracleEnv()
        e.set_state(*(a[k].astype(float) for a in (qpos, qvel, ctrl, ws)))
        for _ in range(nsub):
            e.mj_step()
        rq, rv, _, _ = e.get_state()
        err_q.append(np.abs(gq[k] - rq).max())
        err_v.append(np.abs(gv[k] - rv).max())
    errs = sim.view("episode_i", _lib.EPI_N, "<i4")[:, 9].cpu().numpy()
    assert (errs == 0).all(), "contact/row capacity overflow or NaN"
    return np.array(err_q), np.array(err_v)


def test_physics_parity_one_substep(margin):  # L1: fp32 GPU vs fp64 oracle, contacts incl. grasps
    dq, dv = _physics_parity(1)
    margin("max_abs_dqpos", float(dq.max()), 1e-5)
    margin("max_abs_dqvel", float(dv.max()), 5e-3)
    assert dq.max() < 1e-5, dq.max()
    assert dv.max() < 5e-3, dv.max()


def test_step_layout_api():
    """mmx_set_step_rows / mmx_step_rows: by default 192 rows (four envs per CU, each with a helper
    wave) while the batch fits four per CU, 128 (twelve per CU) above, with or without cameras; either
    on request, anything else rejected."""
    from mujoco_manip_amd import _lib

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    a = _lib.Sim(8, action_mode="abs_pos", image_size=0)
    b = _lib.Sim(8, action_mode="abs_pos", image_size=32)
    c = _lib.Sim(4 * cus + 1, action_mode="abs_pos", image_size=0)
    try:
        assert a.step_rows == 192 and b.step_rows == 192 and c.step_rows == 128
        a.step_rows = 128
        assert a.step_rows == 128
        with pytest.raises(RuntimeError):
            a.step_rows = 100
        assert a.step_rows == 128
    finally:
        a.close()
        b.close()
        c.close()


def test_step_order_bit_identical(margin, monkeypatch):
    """mmx_set_step_order: the longest-first dispatch order (default) changes only which workgroup the
    hardware starts first, so 512 C3 envs (enough to spread over several FSM phases and the four
    cost classes) end an expert rollout bit-identical to index order, through fused launches on two
    rollout lanes (the single-wave sort) and through one mmx_step launch of all envs (the 1,024-lane
    sort)."""
    monkeypatch.setenv("MMX_STREAMS", "2")
    import oracle_py as O
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    n = 512
    seeds = [O.episode_seed(11, i) for i in range(n)]
    outs = []
    for on in (True, False):
        env = PickPlaceVecEnv(n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                              autoreset=True, image_size=0)
        assert env.sim.step_order is True and env.sim.rollout_lanes == 2  # the default order
        env.sim.step_order = on
        assert env.sim.step_order is on
        with pytest.raises(RuntimeError):
            env.sim._check(env.sim.L.mmx_set_step_order(env.sim.ptr, 2), "mmx_set_step_order")
        env.reset(seed=seeds)
        env.rollout_expert(96)  # fused launches on the rollout lanes
        act = torch.zeros(n, 4, device="cuda")
        env.sim.expert_plan(1, act.data_ptr())
        env.sim.step(act.data_ptr(), 4)  # one mmx_step launch of all envs
        torch.cuda.synchronize()
        q, v, _, _ = env.sim.get_state()
        fsm = env.sim.view("episode_i", _lib_epi_n(), "<i4").cpu().numpy()
        outs.append((np.concatenate([q, v], 1), fsm))
        env.close()
    phases = np.unique(outs[0][1][:, _lib.EPI["fsm_state"]])
    margin("fsm_phases_in_batch", int(len(phases)))
    assert len(phases) >= 3, phases  # the order had more than one class to sort
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


def test_step_layouts_agree(margin):
    """The two env-step kernel layouts (128 LDS rows + HBM overflow at twelve envs per CU; 192 LDS rows
    at four, each env with a helper wave running its IK, dynamics and GJK / EPA pairs beside the env
    wave's kinematics, broadphase and box pairs) are a performance choice only: 1024 C3 envs in lockstep
    through their approach and grasp
    phases, where the contact piles put rows past 128 into the overflow block of the first layout
    only, end every one of 60 env steps bit-identical (the Hessian pass assigns each row group to the
    same MFMA accumulator whichever address space holds it)."""
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    import oracle_py as O

    envs = []
    for rows in (128, 192):
        e = PickPlaceVecEnv(1024, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                            autoreset=False, image_size=0)
        e.sim.step_rows = rows
        e.reset(seed=[O.episode_seed(42, i) for i in range(1024)])
        envs.append(e)
    dmax, first_diff, deep = 0.0, -1, 0.0
    for t in range(60):
        before = envs[0].stats[:, 0].clone()
        for e in envs:
            e.step(e.expert_plan(16))
        deep = max(deep, float(((envs[0].stats[:, 0] - before) / 16).max()))
        d = max(float((envs[0].qpos - envs[1].qpos).abs().max()), float((envs[0].qvel - envs[1].qvel).abs().max()))
        if d > 0 and first_diff < 0:
            first_diff = t
        dmax = max(dmax, d)
    fsm_diff = int((envs[0].fsm_state != envs[1].fsm_state).sum())
    for e in envs:
        e.close()
    print(f"max |dqpos|, |dqvel| over 60 steps {dmax:.2e} (first differing step {first_diff}); FSM phases "
          f"differing: {fsm_diff}; largest mean rows per substep {deep:.0f}")
    margin("max_abs_dstate_60_steps", dmax, 0.0)
    # (stats count MuJoCo's rows: 6 pyramid edges per contact where the kernel stores 4 basis rows,
    # so > 200 MuJoCo rows is > ~135 stored ones)
    assert deep > 200, "no env step used the overflow rows of the 128-row layout"
    assert dmax == 0.0 and fsm_diff == 0, (dmax, first_diff, fsm_diff)


def test_physics_parity_one_env_step(margin):  # L1: 16 substeps; SURVEY bound qpos <= 1e-4
    dq, dv = _physics_parity(16)
    margin("max_abs_dqpos", float(dq.max()), 1e-4)
    margin("max_abs_dqvel", float(dv.max()), 2e-2)
    assert dq.max() < 1e-4, dq.max()
    assert dv.max() < 2e-2, dv.max()


def _pile_states(n_want=6, min_mean_nefc=215.0):
    """States (qpos, qvel, ctrl, warm start) just before C3 env steps whose substeps averaged more
    than `min_mean_nefc` constraint rows: piles of contacts whose rows past MMX_LDSEFC (128 since r05;
    192 before) live in the env's HBM overflow block instead of LDS."""
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    import oracle_py as O

    env = PickPlaceVecEnv(1024, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          autoreset=True, image_size=0)
    env.reset(seed=[O.episode_seed(42, i) for i in range(1024)])
    found = []
    for _ in range(400):
        snap = env.sim.get_state()
        before = env.stats[:, 0].clone()
        env.step(env.expert_plan(16))
        mean = ((env.stats[:, 0] - before) / 16).cpu().numpy()
        for k in np.where(mean > min_mean_nefc)[0]:
            found.append(tuple(a[k].astype(float) for a in snap))
        if len(found) >= n_want:
            break
    env.close()
    return found[:n_want]


def test_physics_parity_hbm_overflow_rows(margin):  # L1 on contact piles: rows 128..303 live in HBM
    sts = _pile_states()
    assert len(sts) >= 4, f"only {len(sts)} pile states in 400 C3 steps"
    rows1, rows16 = [], []
    dq, dv = _physics_parity(1, sts, rows1)
    print(f"pile states: rows of the first substep {rows1[0].astype(int).tolist()}, errors qpos {dq.max():.2e} "
          f"qvel {dv.max():.2e}")
    assert (rows1[0] > 192).any(), f"no substep used the overflow rows deeply: {rows1[0]}"
    margin("substep1_max_abs_dqpos", float(dq.max()), 1e-5)
    margin("substep1_max_abs_dqvel", float(dv.max()), 5e-3)
    assert dq.max() < 1e-5, dq.max()
    assert dv.max() < 5e-3, dv.max()
    dq, dv = _physics_parity(16, sts, rows16)
    margin("substep16_max_abs_dqpos", float(dq.max()), 1e-4)
    margin("substep16_max_abs_dqvel", float(dv.max()), 2e-2)
    assert dq.max() < 1e-4, dq.max()
    assert dv.max() < 2e-2, dv.max()


def _flat(obs, n):  # the 85 numeric observation values (camera images excluded)
    return torch.cat([obs[k].reshape(n, -1) for k in obs if not k.startswith("image_")], 1).cpu().numpy()


def test_reset_parity_randomized_seeds(margin):  # L0: PCG64 stream, spawn, task draw, obs codecs
    import oracle_py as O
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N = 16
    seeds = [O.episode_seed(42, i) for i in range(N)]
    env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True)
    obs, _ = env.reset(seed=seeds)
    refs = [O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=True) for _ in range(N)]
    robs = np.stack([r.reset(seed=s) for r, s in zip(refs, seeds)])
    margin("max_abs_dobs", float(np.abs(_flat(obs, N) - robs).max()), 2e-6)
    np.testing.assert_allclose(_flat(obs, N), robs, atol=2e-6)
    assert [tuple(r.task()) for r in refs] == [(o, b) for o, b in env._epi[:, :2].cpu().numpy().tolist()]
    ref_q = np.stack([r.get_state()[0] for r in refs])
    np.testing.assert_array_equal(env.qpos.cpu().numpy()[:, 9:30], ref_q[:, 9:30].astype(np.float32))


@pytest.mark.parametrize("mode", ["abs_pos", "ee_pos_quat_g", "ee_pos_rot6d_g", "ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel"])
def test_env_step_parity_action_modes(mode, margin):  # L2: decode + 16 x (IK + mj_step) + forward + obs
    import oracle_py as O
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N = 4
    rng = np.random.default_rng(7)
    env = PickPlaceVecEnv(N, task=("obj_red", "bin_red"), action_mode=mode, reward_type="dense")
    env.reset(seed=0)
    refs = [O.OracleEnv(action_mode=mode, reward_type="dense", task=(0, 0)) for _ in range(N)]
    for k, r in enumerate(refs):
        r.reset(seed=k)
    dim = env.action_dim
    dmax, rmax = 0.0, 0.0
    for t in range(6):
        a = np.zeros((N, dim), np.float32)
        a[:, :3] = rng.uniform(-0.05, 0.05, (N, 3)) + ([0.0, 0.45, 0.42] if "rel" not in mode else 0.0)
        if dim >= 8:
            a[:, 3:7] = [0, 0, 0, 1] if "quat" in mode else [1, 0, 0, 0]
        if dim == 10:
            a[:, 3:9] = [1, 0, 0, 0, 1, 0]
        a[:, -1] = float(t % 2)
        obs, rew, term, trunc, info = env.step(torch.tensor(a, device="cuda"))
        got = _flat(obs, N)
        for k, r in enumerate(refs):
            ro, rr, rt, rtr, ri = r.step(a[k])
            dmax = max(dmax, float(np.abs(got[k, :11] - ro[:11]).max()))
            rmax = max(rmax, abs(float(rew[k]) - rr))
            margin("max_abs_dstate", dmax, 1e-4)
            margin("max_abs_dreward", rmax, 1e-3)
            np.testing.assert_allclose(got[k, :11], ro[:11], atol=1e-4)
            assert abs(float(rew[k]) - rr) < 1e-3


def test_expert_rollout_parity_and_completion(margin):  # L2 + L3 (test_pick_and_place.py:274-289)
    import oracle_py as O
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N = 18
    seeds = [O.episode_seed(7, i) for i in range(N)]
    env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True)
    env.reset(seed=seeds)
    done_at = np.full(N, -1)
    placed = np.zeros(N, bool)
    first_err = []
    refs = [O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=True) for _ in range(2)]
    for r, s in zip(refs, seeds[:2]):
        r.reset(seed=s)
    for t in range(200):
        act = env.expert_plan(16)
        obs, rew, term, trunc, info = env.step(act)
        if t < 5:  # early steps: trajectories still comparable to the oracle
            a = act.cpu().numpy()
            for k, r in enumerate(refs):
                ro = r.step(a[k])[0]
                first_err.append(np.abs(obs["state"][k].cpu().numpy() - ro[:11]).max())
        placed |= ((env.episode_flags & 8) != 0).cpu().numpy()
        fsm = env.fsm_state.cpu().numpy()
        done_at[(done_at < 0) & (fsm == 10)] = t
        if (done_at >= 0).all():
            break
    margin("first5_max_abs_dstate", float(max(first_err)), 1e-4)
    margin("episode_length_max", int(done_at.max()), 2000)
    assert max(first_err) < 1e-4
    assert (done_at >= 0).all(), f"FSM unfinished: {np.where(done_at < 0)[0]}"
    assert done_at.max() < 2000  # reference KAT: <= 2000 gym steps
    assert placed.all()
    assert (env.env_error.cpu().numpy() == 0).all()


def test_fsm_golden_traces_on_device(golden):  # pick_and_place.py:167-277, golden traces (single task)
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.constants import BINS, OBJECTS

    names = ["IDLE", "PRE_GRASP", "GRASP", "CLOSE_GRIPPER", "LIFT", "MOVE_TO_BIN", "SETTLE_AT_BIN",
             "LOWER_TO_BIN", "RELEASE", "RETREAT", "DONE"]
    traces = [tr for tr in golden["fsm"] if len(tr["tasks"]) == 1]  # the gym FSM runs one task per episode
    assert traces
    for tr in traces:
        o, b = tr["tasks"][0]
        sim = _lib.Sim(1, action_mode="abs_pos", reward_type="staged",
                       fixed_task=(OBJECTS.index(o), BINS.index(b)))
        sim.reset()
        kin = sim.view("kin", _lib.KIN_N)
        qpos = sim.view("qpos", _lib.NQ)
        epi = sim.view("episode_i", _lib.EPI_N, "<i4")
        epf = sim.view("episode_f", _lib.EPF_N)
        act = torch.zeros(1, 4, device="cuda")
        for k, st in enumerate(tr["trace"]):
            kin[0, 0:3] = torch.tensor(st["ee"], dtype=torch.float32)
            for j, nm in enumerate(OBJECTS):
                qpos[0, 9 + 7 * j:12 + 7 * j] = torch.tensor(st["objs"][nm], dtype=torch.float32)
            sim.expert_plan(tr["n_steps"], act.data_ptr())
            torch.cuda.synchronize()
            e = epi[0].cpu().numpy()
            assert names[e[4]] == st["state"], f"step {k}"
            assert e[6] == st["settle"], f"step {k}"
            assert float(e[7]) == st["gripper"], f"step {k}"
            if st["target"] is not None:
                np.testing.assert_allclose(epf[0, 21:24].cpu().numpy(), st["target"], atol=2e-6, err_msg=f"step {k}")
                np.testing.assert_allclose(act[0, :3].cpu().numpy(), st["target"], atol=2e-6, err_msg=f"step {k}")
            assert act[0, 3].item() == st["gripper"]
        sim.close()


def test_ik_convergence_kat():  # tests/test_controller.py:84-139 on the GPU batch
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    targets = np.array([[0.0, 0.4, 0.4], [-0.15, 0.45, 0.36], [-0.3, 0.55, 0.45]], np.float32)
    env = PickPlaceVecEnv(3, task=("obj_red", "bin_red"), action_mode="abs_pos")
    env.reset(seed=0)
    a = torch.tensor(np.concatenate([targets, np.ones((3, 1), np.float32)], 1), device="cuda")
    for _ in range(13):  # 208 x (IK + mj_step) >= the reference's 200
        obs, *_ = env.step(a)
    ee = obs["state"][:, :3].cpu().numpy()
    assert (np.linalg.norm(ee - targets, axis=1) < 0.03).all()
    q = obs["state.ee.pos_quat_g"][:, 3:7].cpu().numpy()
    for k in range(3):
        x, y, z, w = q[k]
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        np.testing.assert_allclose(R, TARGET_ORI, atol=0.1)


def test_gym_kats_relative_and_absolute():  # tests/test_gym_env.py:258-339, 622-687
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(2, task=("obj_red", "bin_red"), action_mode="ee_pos_quat_g_rel", max_episode_steps=50)
    env.reset(seed=0)
    T0 = env.initial_ee_se3.cpu().numpy()
    ident = torch.tensor([[0, 0, 0, 0, 0, 0, 1, 1]] * 2, dtype=torch.float32, device="cuda")
    for _ in range(5):
        obs, *_ = env.step(ident)
    assert (np.linalg.norm(obs["state"][:, :3].cpu().numpy() - T0[:, :3, 3], axis=1) < 0.05).all()
    move = torch.tensor([[0.1, 0, 0, 0, 0, 0, 1, 1]] * 2, dtype=torch.float32, device="cuda")
    for _ in range(20):
        obs, *_ = env.step(move)
    want = (T0 @ np.array([0.1, 0, 0, 1.0]))[:, :3]
    assert (np.linalg.norm(obs["state"][:, :3].cpu().numpy() - want, axis=1) < 0.05).all()
    env = PickPlaceVecEnv(1, task=("obj_red", "bin_red"), action_mode="abs_pos")
    env.reset(seed=0)
    a = torch.tensor([[0.0, 0.4, 0.45, 1.0]], device="cuda")
    for _ in range(20):
        obs, *_ = env.step(a)
    assert np.linalg.norm(obs["state"][0, :3].cpu().numpy() - [0.0, 0.4, 0.45]) < 0.05


def test_staged_collision_penalty():  # gym_env.py:428-430 ; tests/test_gym_env.py:868-876
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(1, task=("obj_red", "bin_red"), action_mode="abs_pos", reward_type="staged")
    env.reset(seed=0)
    a = torch.tensor([[0.25, 0.35, 0.05, 1.0]], device="cuda")  # drive the hand into the tabletop
    hit = False
    for _ in range(60):
        obs, rew, term, trunc, info = env.step(a)
        if float(rew[0]) == -1.0:
            hit = True
            assert bool(term[0]) and not bool(info["success"][0])
            break
    assert hit


def test_determinism_and_shard_independence():
    import oracle_py as O
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    seeds = [O.episode_seed(42, i) for i in range(8)]
    outs = []
    for ss in (seeds, seeds, seeds[4:]):
        env = PickPlaceVecEnv(len(ss), tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True)
        env.reset(seed=ss)
        for _ in range(8):
            obs, *_ = env.step(env.expert_plan(16))
        outs.append(_flat(obs, len(ss)))
    np.testing.assert_array_equal(outs[0], outs[1])  # bit-identical reruns
    np.testing.assert_array_equal(outs[0][4:], outs[2])  # result independent of batch composition


def test_rollout_lanes_bit_identical(monkeypatch):
    """Concurrent env ranges on separate streams (mmx_rollout_lanes) change nothing but timing
    (rollouts without cameras: with cameras a rollout runs on one lane)."""
    import oracle_py as O
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    seeds = [O.episode_seed(3, i) for i in range(10)]
    outs = []
    for lanes in ("1", "3"):  # 3 lanes over 10 envs: ragged ranges 3/3/4
        monkeypatch.setenv("MMX_STREAMS", lanes)
        env = PickPlaceVecEnv(10, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                              autoreset=True, image_size=0)
        assert env.sim.rollout_lanes == int(lanes)
        env.reset(seed=seeds)
        env.rollout_expert(40)
        torch.cuda.synchronize()
        q, v, _, _ = env.sim.get_state()
        outs.append(np.concatenate([q, v, env.sim.view("episode_i", _lib_epi_n(), "<i4").cpu().numpy()], 1))
    np.testing.assert_array_equal(outs[0], outs[1])


def _plan_launches(n, fuse, lanes):
    """mmx_rollout_expert's plan (mmx_api.cpp rollout_plan): len = min(fuse, ceil(n / 4)); lane l starts
    with l * len / lanes steps, then launches of len, then the remainder; the most launches of a lane."""
    ln = max(1, min(fuse, -(-n // 4)))
    out = 0
    for l in range(lanes):
        first = min(n, l * ln // lanes)
        out = max(out, (1 if first else 0) + -(-(n - first) // ln))
    return out


def test_fused_rollout_bit_identical(monkeypatch):
    """Several env steps per launch (mmx_rollout_steps_per_launch, mmx_rollout_launches) change
    nothing but timing: state, episode records, observations, rewards, flags and solver stats match
    one launch per step bit for bit, incl. autoresets inside a fused launch and launches of unequal
    length (43 steps at a cap of 7 on one lane: 7 x 6 + 1; at a cap of 32 on three staggered lanes:
    11,11,11,10 / 3,11,11,11,7 / 7,11,11,11,3)."""
    import oracle_py as O
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    seeds = [O.episode_seed(5, i) for i in range(12)]
    outs = []
    for lanes, fuse in (("1", "1"), ("1", "7"), ("3", "32")):
        monkeypatch.setenv("MMX_STREAMS", lanes)
        monkeypatch.setenv("MMX_FUSE", fuse)
        env = PickPlaceVecEnv(12, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                              autoreset=True, image_size=0, max_episode_steps=25)
        assert env.sim.rollout_steps_per_launch == int(fuse)
        assert env.sim.rollout_launches(43) == _plan_launches(43, int(fuse), int(lanes))
        assert env.sim.rollout_launches(512) == _plan_launches(512, int(fuse), int(lanes))
        env.reset(seed=seeds)
        env.rollout_expert(43)
        torch.cuda.synchronize()
        q, v, _, _ = env.sim.get_state()
        s = env.sim
        outs.append(np.concatenate([q, v, s.view("episode_i", _lib.EPI_N, "<i4").cpu().numpy().view(np.float32),
                                    s.view("obs", _lib.NOBS).cpu().numpy(), s.view("reward", 1).cpu().numpy()[:, None],
                                    s.view("done", 3, "<i4").cpu().numpy().view(np.float32),
                                    env.stats[:, :4].cpu().numpy()], 1))
        env.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[0], outs[2])


def _lib_epi_n():
    from mujoco_manip_amd import _lib

    return _lib.EPI_N


def test_autoreset_and_truncation():
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(4, tasks="all", action_mode="abs_pos", max_episode_steps=3, autoreset=True,
                          randomize_objects=True)
    env.reset(seed=1)
    a = torch.tensor([[0.0, 0.45, 0.45, 1.0]] * 4, device="cuda")
    for t in range(3):
        obs, rew, term, trunc, info = env.step(a)
    assert bool(trunc.all())
    assert (env.step_count.cpu().numpy() == 0).all()  # reset inside the same step
    assert (env._epi[:, 12].cpu().numpy() == 2).all()  # second episode running


def test_abi_rejects_bad_action_dim():
    from mujoco_manip_amd import _lib

    sim = _lib.Sim(2, action_mode="ee_pos_rot6d_g")
    a = torch.zeros(2, 4, device="cuda")
    with pytest.raises(RuntimeError):
        sim.step(a.data_ptr(), 4)


SAMPLING_MSG = "Failed to sample 3 positions with min_separation=0.08 in 1000 attempts"


def test_sampling_exhaustion_raises_like_reference():  # randomization.py:78-87 ; gym_env.py:496-501
    import oracle_py as O
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.gym_env import PickPlaceGymEnv
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    xr, yr = (0.0, 0.01), (0.30, 0.31)  # three cubes 8 cm apart cannot fit: every draw is rejected
    env = PickPlaceVecEnv(4, tasks="all", action_mode="abs_pos", randomize_objects=True, spawn_x_range=xr,
                          spawn_y_range=yr)
    with pytest.raises(RuntimeError, match="^" + SAMPLING_MSG + "$"):
        env.reset(seed=[0, 3, 42, 7])
    err = env.env_error.cpu().numpy()
    assert ((err & _lib.ERR_SAMPLING) != 0).all()
    key = O.OracleEnv()
    key.reset_keyframe()
    q = env.qpos.cpu().numpy()
    np.testing.assert_array_equal(q[:, 9:30], np.tile(key.get_state()[0][9:30].astype(np.float32), (4, 1)))
    env.synchronize()  # the fault was reported once and cleared
    # the oracle raises for the same seeds and ranges
    o = O.OracleEnv(randomize_objects=True, spawn_x_range=xr, spawn_y_range=yr)
    with pytest.raises(RuntimeError, match=SAMPLING_MSG):
        o.reset(seed=3)
    # a feasible range in the same process resets cleanly (the fault word is per sim)
    ok = PickPlaceVecEnv(2, tasks="all", action_mode="abs_pos", randomize_objects=True)
    ok.reset(seed=1)
    assert (ok.env_error.cpu().numpy() == 0).all()
    # the single-env facade raises the same exception
    g = PickPlaceGymEnv(action_mode="abs_pos", randomize_objects=True, spawn_x_range=xr, spawn_y_range=yr, image_size=0)
    with pytest.raises(RuntimeError, match=SAMPLING_MSG):
        g.reset(seed=5)


def test_sampling_exhaustion_on_autoreset_reported_at_sync():
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(2, tasks="all", action_mode="abs_pos", randomize_objects=True, spawn_x_range=(0.0, 0.01),
                          spawn_y_range=(0.30, 0.31), max_episode_steps=1, autoreset=True)
    with pytest.raises(RuntimeError, match=SAMPLING_MSG):
        env.reset(seed=1)
    a = torch.tensor([[0.0, 0.45, 0.45, 1.0]] * 2, device="cuda")
    env.step(a)  # truncated after one step: the autoreset's sampling is exhausted again
    with pytest.raises(RuntimeError, match=SAMPLING_MSG):
        env.synchronize()
    assert ((env.env_error.cpu().numpy() & _lib.ERR_SAMPLING) != 0).all()
    assert np.isfinite(env.qpos.cpu().numpy()).all()
