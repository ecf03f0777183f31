"""The single-env Gymnasium façade (mujoco_manip_amd.gym_env.PickPlaceGymEnv) against the
reference's own tests (/root/reference/tests/test_gym_env.py), re-targeted at the façade.

CPU part: the action / observation spaces (test_gym_env.py:90-142) built by the same functions
the façade uses.  GPU part: the reference's behavioural KATs through the façade (every step runs
the HIP kernels): reset / step API and dtypes, relative-pose decode, cross-mode parity (:395),
truncation (:428-442), dense and sparse reward (:450-468), task selection incl. the pool
coverage (:476-517), render (:525-531), absolute SE(3) targets (:622-687), target keypoints
(:695-780), multiple resets (:788-813) and the staged reward (:821-885).
"""
import numpy as np
import pytest

from mujoco_manip_amd import gym_env as G
from mujoco_manip_amd.pose_utils import pos_rotmat_to_se3, rotmat_to_6d, se3_to_pos_quat_g, se3_to_pos_rot6d_g

TARGET_ORI = np.array([[0, 1, 0], [1, 0, 0], [0, 0, -1.0]])  # controller.py:12-18
OBS_KEYS = {"image_overhead", "image_wrist", "state", "state.ee.pos_quat_g", "state.ee.pos_rot6d_g",
            "state.ee.pos_quat_g_rel", "state.ee.pos_rot6d_g_rel", "target_bin_onehot", "target_obj_onehot",
            "keypoints_overhead", "keypoints_wrist", "target_obj_keypoints_overhead", "target_bin_keypoints_overhead"}


# ----------------------------------------------------------------------------- spaces (CPU)
@pytest.mark.parametrize("mode,dim", [("ee_pos_quat_g_rel", 8), ("ee_pos_rot6d_g_rel", 10), ("ee_pos_quat_g", 8),
                                      ("ee_pos_rot6d_g", 10), ("abs_pos", 4)])
def test_action_space_shape_and_bounds(mode, dim):  # test_gym_env.py:95-124
    sp = G.make_action_space(mode)
    assert sp.shape == (dim,) and sp.dtype == np.float32
    if mode == "abs_pos":
        np.testing.assert_array_equal(sp.low, np.array([-0.5, 0.0, 0.24, 0.0], np.float32))
        np.testing.assert_array_equal(sp.high, np.array([0.5, 0.8, 0.60, 1.0], np.float32))
    else:
        assert sp.low[dim - 1] == 0.0 and sp.high[dim - 1] == 1.0
        assert np.all(sp.low[:dim - 1] == -np.inf) and np.all(sp.high[:dim - 1] == np.inf)
    for _ in range(20):
        assert sp.contains(sp.sample())


def test_observation_space_keys_and_shapes():  # test_gym_env.py:126-142, gym_env.py:172-208
    sp = G.make_observation_space(224)
    assert set(sp.spaces.keys()) == OBS_KEYS
    assert sp["image_overhead"].shape == (224, 224, 3) and sp["image_overhead"].dtype == np.uint8
    assert sp["keypoints_wrist"].shape == (7, 2) and sp["state"].shape == (11,)


def test_invalid_action_mode_raises():  # test_gym_env.py:91-93 (raised before any device work)
    with pytest.raises(ValueError, match="action_mode must be one of"):
        G.PickPlaceGymEnv(action_mode="invalid")


# ----------------------------------------------------------------------------- façade on the GPU
torch = pytest.importorskip("torch")


def _env(**kw):
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    args = dict(task=("obj_red", "bin_red"), max_episode_steps=50)
    args.update(kw)
    return G.PickPlaceGymEnv(**args)


@pytest.fixture(params=["ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel"])
def env(request):
    e = _env(action_mode=request.param)
    yield e
    e.close()


@pytest.mark.gpu
def test_reset_and_step_api(env):  # test_gym_env.py:150-220
    obs, info = env.reset()
    assert isinstance(obs, dict) and isinstance(info, dict) and set(obs) == OBS_KEYS
    assert obs["image_overhead"].shape == (224, 224, 3) and obs["image_overhead"].dtype == np.uint8
    assert obs["state"].shape == (11,) and obs["state"].dtype == np.float32
    obs, r, term, trunc, info = env.step(env.action_space.sample())
    assert isinstance(r, float) and isinstance(term, bool) and isinstance(trunc, bool) and "success" in info
    assert env.step_count == 1


@pytest.mark.gpu
def test_gripper_command_and_state(env):  # test_gym_env.py:360-384
    env.reset()
    n = env.action_space.shape[0]
    a = np.zeros(n, np.float32)
    if env.action_mode == "ee_pos_quat_g_rel":
        a[6] = 1.0
    else:
        a[3:9] = rotmat_to_6d(np.eye(3))
    a[-1] = 1.0
    obs_open, *_ = env.step(a)
    assert env.robot.gripper_ctrl == 255.0
    a[-1] = 0.0
    obs_close, *_ = env.step(a)
    assert env.robot.gripper_ctrl == 0.0
    assert obs_open["state"][3] > obs_close["state"][3]


@pytest.mark.gpu
def test_same_relative_pose_same_ee_position():  # test_gym_env.py:392-420
    e8, e10 = _env(action_mode="ee_pos_quat_g_rel"), _env(action_mode="ee_pos_rot6d_g_rel")
    obs8, _ = e8.reset(seed=0)
    obs10, _ = e10.reset(seed=0)
    np.testing.assert_allclose(obs8["state"][:3], obs10["state"][:3], atol=1e-5)
    T_rel = pos_rotmat_to_se3(np.array([0.05, -0.03, 0.02]), np.eye(3))
    a8, a10 = se3_to_pos_quat_g(T_rel, gripper=1.0), se3_to_pos_rot6d_g(T_rel, gripper=1.0)
    for _ in range(15):
        obs8, *_ = e8.step(a8)
        obs10, *_ = e10.step(a10)
    np.testing.assert_allclose(obs8["state"][:3], obs10["state"][:3], atol=0.01)
    e8.close()
    e10.close()


@pytest.mark.gpu
def test_truncation(env):  # test_gym_env.py:428-442
    env.reset()
    _, _, _, truncated, _ = env.step(env.action_space.sample())
    assert not truncated
    env.reset()
    terminated = truncated = False
    for _ in range(env._max_episode_steps):
        _, _, terminated, truncated, _ = env.step(env.action_space.sample())
        if terminated:
            break
    if not terminated:
        assert truncated


@pytest.mark.gpu
def test_dense_and_sparse_reward():  # test_gym_env.py:450-468
    e = _env(action_mode="ee_pos_quat_g_rel")
    e.reset()
    _, r, *_ = e.step(e.action_space.sample())
    assert isinstance(r, float)
    e.close()
    e = _env(action_mode="ee_pos_quat_g_rel", reward_type="sparse", max_episode_steps=10)
    e.reset()
    _, r, *_ = e.step(e.action_space.sample())
    assert r in (0.0, 1.0)
    e.close()


@pytest.mark.gpu
def test_task_selection():  # test_gym_env.py:476-517
    e = _env(action_mode="ee_pos_quat_g_rel", task=("obj_blue", "bin_green"), max_episode_steps=10)
    obs, _ = e.reset()
    np.testing.assert_array_equal(obs["target_bin_onehot"], [0, 1, 0])
    np.testing.assert_array_equal(obs["target_obj_onehot"], [0, 0, 1])
    e.close()
    e = _env(action_mode="ee_pos_quat_g_rel", task=None, tasks="all", max_episode_steps=10)
    seen = set()
    for _ in range(30):  # reset() without a seed continues the env's stream
        obs, _ = e.reset()
        seen.add(int(np.argmax(obs["target_bin_onehot"])))
    assert len(seen) == 3, seen
    e.close()
    custom = [("obj_red", "bin_blue"), ("obj_green", "bin_red")]
    e = _env(action_mode="ee_pos_rot6d_g_rel", task=None, tasks=custom, max_episode_steps=10)
    for _ in range(10):
        e.reset()
        assert (e.obj_name, e.bin_name) in custom
    e.close()


@pytest.mark.gpu
def test_render_returns_image(env):  # test_gym_env.py:525-531
    env.reset()
    img = env.render()
    assert img is not None and img.shape == (224, 224, 3) and img.dtype == np.uint8


@pytest.mark.gpu
def test_relative_pose_decode(env):  # test_gym_env.py:539-585
    env.reset()
    initial = env.robot.ee_pos.copy()
    if env.action_mode == "ee_pos_quat_g_rel":
        ident = np.array([0, 0, 0, 0, 0, 0, 1, 1.0], np.float32)
    else:
        ident = np.array([0, 0, 0, *rotmat_to_6d(np.eye(3)), 0.5], np.float32)
    world, g = env.decode_action(ident)
    np.testing.assert_allclose(world, initial, atol=1e-6)
    T_init_inv = np.linalg.inv(env.initial_ee_se3)
    target = np.array([-0.1, 0.5, 0.40])
    T_rel = T_init_inv @ pos_rotmat_to_se3(target, TARGET_ORI)
    enc = se3_to_pos_quat_g if env.action_mode == "ee_pos_quat_g_rel" else se3_to_pos_rot6d_g
    world, _ = env.decode_action(enc(T_rel, gripper=1.0))
    np.testing.assert_allclose(world, target, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["ee_pos_quat_g", "ee_pos_rot6d_g"])
def test_absolute_se3_targets(mode):  # test_gym_env.py:622-687
    e = _env(action_mode=mode)
    enc = se3_to_pos_quat_g if mode == "ee_pos_quat_g" else se3_to_pos_rot6d_g
    obs, _ = e.reset()
    initial = obs["state"][:3].copy()
    a = enc(e.initial_ee_se3.copy(), gripper=1.0)
    for _ in range(5):
        obs, *_ = e.step(a)
    assert np.linalg.norm(obs["state"][:3] - initial) < 0.05
    e.reset()
    target = np.array([0.0, 0.4, 0.45])
    a = enc(pos_rotmat_to_se3(target, TARGET_ORI), gripper=1.0)
    for _ in range(20):
        obs, *_ = e.step(a)
    assert np.linalg.norm(obs["state"][:3] - target) < 0.05
    e.close()


@pytest.mark.gpu
def test_abs_pos_passthrough():  # test_gym_env.py:587-592
    e = _env(action_mode="abs_pos")
    e.reset()
    a = np.array([0.1, 0.4, 0.35, 0.8], np.float32)
    world, g = e.decode_action(a)
    np.testing.assert_array_equal(world, a[:3])
    assert g == pytest.approx(0.8)
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["target_obj_keypoints_overhead", "target_bin_keypoints_overhead"])
def test_target_keypoints(env, key):  # test_gym_env.py:695-780
    obs, _ = env.reset()
    kp = obs[key]
    assert kp.shape == (2,) and kp.dtype == np.float32 and np.all((kp >= 0.0) & (kp <= 1.0))
    kp0 = kp.copy()
    for _ in range(3):
        obs, *_ = env.step(env.action_space.sample())
    np.testing.assert_array_equal(obs[key], kp0)
    e1 = _env(action_mode="ee_pos_quat_g_rel", task=("obj_red", "bin_red"), max_episode_steps=10)
    e2 = _env(action_mode="ee_pos_quat_g_rel", task=("obj_blue", "bin_green"), max_episode_steps=10)
    o1, _ = e1.reset()
    o2, _ = e2.reset()
    assert not np.allclose(o1[key], o2[key])
    e1.close()
    e2.close()


@pytest.mark.gpu
def test_multiple_resets(env):  # test_gym_env.py:788-813
    env.reset()
    T1 = env.initial_ee_se3.copy()
    env.step(env.action_space.sample())
    env.step(env.action_space.sample())
    assert env.step_count == 2
    env.reset()
    assert env.step_count == 0
    np.testing.assert_allclose(env.initial_ee_se3, T1, atol=1e-6)
    for _ in range(3):
        env.reset()
        for _ in range(5):
            _, _, term, trunc, _ = env.step(env.action_space.sample())
            if term or trunc:
                break


@pytest.fixture
def staged_env():
    e = _env(action_mode="abs_pos", reward_type="staged", max_episode_steps=500)
    yield e
    e.close()


@pytest.mark.gpu
def test_staged_reward_monotonic_on_approach(staged_env):  # test_gym_env.py:840-852
    staged_env.reset()
    obj = staged_env.pick_place_env.get_body_pos(staged_env.obj_name)
    prev = -1.0
    for _ in range(15):
        _, r, term, _, _ = staged_env.step(np.array([obj[0], obj[1], 0.44, 1.0], np.float32))
        if term and r < 0:
            break
        assert r >= prev, (r, prev)
        prev = r


@pytest.mark.gpu
def test_staged_reward_range_and_collision(staged_env):  # test_gym_env.py:868-885
    staged_env.reset()
    for _ in range(10):
        _, r, term, _, _ = staged_env.step(staged_env.action_space.sample())
        if term and r < 0:
            break
        assert 0.0 <= r <= 1.0
    staged_env.reset()
    for _ in range(30):  # the arm driven into the table (the reference asserts only on termination)
        _, r, term, _, _ = staged_env.step(np.array([0.0, 0.4, 0.10, 1.0], np.float32))
        if term:
            assert r == -1.0
            break
