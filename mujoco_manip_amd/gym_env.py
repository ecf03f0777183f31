"""PickPlaceGymEnv — single-env façade with the reference interface (mujoco_manip/gym_env.py:39-602).

A drop-in for ``mujoco_manip.gym_env.PickPlaceGymEnv``: the same constructor signature and
defaults (``render_mode="rgb_array"``, ``image_size=224``), the same ``action_space`` /
``observation_space`` (gym_env.py:154-208), ``reset`` / ``step`` returning numpy observations (camera
images from the HIP renderer), float rewards and bool flags, ``decode_action``, ``render`` and the
properties ``action_mode``, ``pick_place_env``, ``robot``, ``controller``, ``step_count``,
``obj_name``, ``bin_name`` and ``initial_ee_se3`` (gym_env.py:210-243, 472-475).  Internally it is a
PickPlaceVecEnv with num_envs=1 on the MI355X; ``pick_place_env`` / ``robot`` / ``controller`` are
read-only views of the device state (the MuJoCo model/data objects they wrap in the reference do
not exist here).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, spaces
from .constants import ACTION_REPEAT, BINS, IMAGE_SIZE, KEYPOINT_BODIES, MAX_EPISODE_STEPS, OBJECTS
from .pose_utils import se3_from_pos_quat_g, se3_from_pos_rot6d_g
from .vec_env import PickPlaceVecEnv

ACTION_MODES = ("abs_pos", "ee_pos_quat_g", "ee_pos_rot6d_g", "ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel")
# static body positions (bodies welded to the world: pick_and_place_scene.xml:47-103)
_STATIC_BODY_POS = {"bin_red": (-0.3, 0.55, 0.24), "bin_green": (0.0, 0.65, 0.24), "bin_blue": (0.3, 0.55, 0.24),
                    "table": (0.0, 0.45, 0.0), "world": (0.0, 0.0, 0.0), "link0": (0.0, 0.0, 0.0)}

try:  # keep the reference's registration id when gymnasium is available (mujoco_manip/__init__.py:3-6)
    import gymnasium as _gym

    _Base = _gym.Env
except Exception:  # gymnasium absent in this image
    _gym = None
    _Base = object


class _RobotView:
    """PandaRobot (robot.py:7-79) read side over the device state."""

    NUM_ARM_JOINTS = 7
    GRIPPER_OPEN = 255.0
    GRIPPER_CLOSED = 0.0
    EE_BODY_NAME = "hand"

    def __init__(self, vec: PickPlaceVecEnv):
        self._vec = vec

    @property
    def ee_pos(self) -> np.ndarray:  # data.xpos[hand] after the step's mj_forward
        return self._vec.sim.view("kin", _lib.KIN_N)[0, 0:3].double().cpu().numpy()

    @property
    def ee_xmat(self) -> np.ndarray:
        return self._vec.sim.view("kin", _lib.KIN_N)[0, 3:12].double().cpu().numpy().reshape(3, 3)

    @property
    def arm_qpos(self) -> np.ndarray:
        return self._vec.qpos[0, :7].double().cpu().numpy()

    @property
    def gripper_ctrl(self) -> float:
        return float(self._vec.ctrl[0, 7].item())


class _SceneView:
    """PickPlaceEnv.get_body_pos / get_body_xmat (env.py:134-177) for the bodies the task reads."""

    def __init__(self, vec: PickPlaceVecEnv):
        self._vec = vec

    def get_body_pos(self, name: str) -> np.ndarray:
        if name in OBJECTS:
            k = OBJECTS.index(name)
            return self._vec.qpos[0, 9 + 7 * k:12 + 7 * k].double().cpu().numpy()
        if name == "hand":
            return _RobotView(self._vec).ee_pos
        if name in _STATIC_BODY_POS:
            return np.array(_STATIC_BODY_POS[name], dtype=np.float64)
        raise ValueError(f"Body '{name}' not found")

    def get_body_xmat(self, name: str) -> np.ndarray:
        if name in OBJECTS:
            k = OBJECTS.index(name)
            w, x, y, z = self._vec.qpos[0, 12 + 7 * k:16 + 7 * k].double().cpu().numpy()
            n = w * w + x * x + y * y + z * z
            w, x, y, z = np.array([w, x, y, z]) / np.sqrt(n)
            return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                             [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                             [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        if name == "hand":
            return _RobotView(self._vec).ee_xmat
        if name in _STATIC_BODY_POS:
            return np.eye(3)
        raise ValueError(f"Body '{name}' not found")


class _ControllerView:
    """IKController (controller.py:46-145): gains and ``reached``; ``compute`` runs on the device
    inside every physics substep of ``step``."""

    pos_tolerance = 0.02  # controller.py:60

    def __init__(self, vec: PickPlaceVecEnv):
        self._robot = _RobotView(vec)

    def reached(self, target_pos) -> bool:
        return bool(np.linalg.norm(self._robot.ee_pos - np.asarray(target_pos, float)) < self.pos_tolerance)


def make_action_space(action_mode: str):
    """gym_env.py:154-170."""
    if action_mode == "abs_pos":
        return spaces.Box(low=np.array([-0.5, 0.0, 0.24, 0.0], dtype=np.float32),
                          high=np.array([0.5, 0.8, 0.60, 1.0], dtype=np.float32))
    n = 8 if action_mode in ("ee_pos_quat_g", "ee_pos_quat_g_rel") else 10
    low = np.full(n, -np.inf, dtype=np.float32)
    high = np.full(n, np.inf, dtype=np.float32)
    low[n - 1], high[n - 1] = 0.0, 1.0  # gripper
    return spaces.Box(low=low, high=high)


def make_observation_space(image_size: int):
    """gym_env.py:172-208."""
    S, K, inf = image_size, len(KEYPOINT_BODIES), np.inf
    return spaces.Dict({
        "image_overhead": spaces.Box(0, 255, (S, S, 3), dtype=np.uint8),
        "image_wrist": spaces.Box(0, 255, (S, S, 3), dtype=np.uint8),
        "state": spaces.Box(-inf, inf, (11,), dtype=np.float32),
        "state.ee.pos_quat_g": spaces.Box(-inf, inf, (8,), dtype=np.float32),
        "state.ee.pos_rot6d_g": spaces.Box(-inf, inf, (10,), dtype=np.float32),
        "state.ee.pos_quat_g_rel": spaces.Box(-inf, inf, (8,), dtype=np.float32),
        "state.ee.pos_rot6d_g_rel": spaces.Box(-inf, inf, (10,), dtype=np.float32),
        "target_bin_onehot": spaces.Box(0.0, 1.0, (3,), dtype=np.float32),
        "target_obj_onehot": spaces.Box(0.0, 1.0, (3,), dtype=np.float32),
        "keypoints_overhead": spaces.Box(0.0, 1.0, (K, 2), dtype=np.float32),
        "keypoints_wrist": spaces.Box(0.0, 1.0, (K, 2), dtype=np.float32),
        "target_obj_keypoints_overhead": spaces.Box(0.0, 1.0, (2,), dtype=np.float32),
        "target_bin_keypoints_overhead": spaces.Box(0.0, 1.0, (2,), dtype=np.float32),
    })


class PickPlaceGymEnv(_Base):
    metadata = {"render_modes": ["rgb_array", "human"], "render_fps": 30}

    def __init__(self, xml_path: str | None = None, task: tuple[str, str] | None = None, tasks="all",
                 action_mode: str = "ee_pos_quat_g_rel", reward_type: str = "dense", image_size: int = IMAGE_SIZE,
                 render_mode: str = "rgb_array", max_episode_steps: int = MAX_EPISODE_STEPS,
                 randomize_objects: bool = False, spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45),
                 device: int = 0):
        if action_mode not in ACTION_MODES:
            raise ValueError(f"action_mode must be one of {ACTION_MODES}, got '{action_mode}'")
        # xml_path is accepted for signature compatibility: the model is compiled offline
        # (tools/compile_model.py) from the reference scene into mujoco_manip_amd/model/.
        self._xml_path = xml_path
        self._vec = PickPlaceVecEnv(1, task=task, tasks=tasks, action_mode=action_mode, reward_type=reward_type,
                                    image_size=image_size, render_mode=render_mode,
                                    max_episode_steps=max_episode_steps, randomize_objects=randomize_objects,
                                    spawn_x_range=spawn_x_range, spawn_y_range=spawn_y_range, device=device)
        self._action_mode = action_mode
        self._reward_type = reward_type
        self._image_size = image_size
        self._max_episode_steps = max_episode_steps
        self.render_mode = render_mode
        self._scene, self._robot, self._controller = _SceneView(self._vec), _RobotView(self._vec), \
            _ControllerView(self._vec)

        self.action_space = make_action_space(action_mode)
        self.observation_space = make_observation_space(image_size)

    # ------------------------------------------------------------------ properties (gym_env.py:210-243)
    @property
    def action_mode(self) -> str:
        return self._action_mode

    @property
    def pick_place_env(self) -> _SceneView:
        return self._scene

    @property
    def robot(self) -> _RobotView:
        return self._robot

    @property
    def controller(self) -> _ControllerView:
        return self._controller

    @property
    def step_count(self) -> int:
        return int(self._vec.step_count[0].item())

    @property
    def obj_name(self) -> str:
        return self._vec.tasks[0][0]

    @property
    def bin_name(self) -> str:
        return self._vec.tasks[0][1]

    @property
    def initial_ee_se3(self) -> np.ndarray:
        return self._vec.initial_ee_se3[0].double().cpu().numpy()

    @property
    def vec_env(self) -> PickPlaceVecEnv:
        return self._vec

    # ------------------------------------------------------------------ gym API
    def decode_action(self, action: np.ndarray) -> tuple[np.ndarray, float]:
        """gym_env.py:252-281 (host-side mirror; the device applies the same decode)."""
        a = np.asarray(action, dtype=np.float32)
        m = self._action_mode
        if m == "abs_pos":
            return a[:3], a[3]
        if m == "ee_pos_quat_g":
            return se3_from_pos_quat_g(a)[:3, 3], a[7]
        if m == "ee_pos_rot6d_g":
            return se3_from_pos_rot6d_g(a)[:3, 3], a[9]
        T_rel = se3_from_pos_quat_g(a) if m == "ee_pos_quat_g_rel" else se3_from_pos_rot6d_g(a)
        g = a[7] if m == "ee_pos_quat_g_rel" else a[9]
        return (self.initial_ee_se3 @ T_rel)[:3, 3], g

    def reset(self, *, seed: int | None = None, options: dict | None = None):
        """gym_env.py:477-534: seed=None continues the env's PCG64 stream (gymnasium semantics)."""
        obs, info = self._vec.reset(seed=None if seed is None else [seed], options=options)
        return {k: v[0].cpu().numpy() for k, v in obs.items()}, {}

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, dtype=np.float32)[None, :], device=self._vec.device)
        obs, r, term, trunc, info = self._vec.step(a)
        out_info = {"success": bool(info["success"][0].item())}
        if "reward_components" in info:
            out_info["reward_components"] = info["reward_components"][0].cpu().numpy()
        return ({k: v[0].cpu().numpy() for k, v in obs.items()}, float(r[0].item()), bool(term[0].item()),
                bool(trunc[0].item()), out_info)

    def expert_action(self, n_steps: int = ACTION_REPEAT) -> np.ndarray:
        """PickAndPlaceTask.plan(n_steps) + abs_pos action (generate_dataset.py:142-148)."""
        return self._vec.expert_plan(n_steps)[0].cpu().numpy()

    def render(self):
        """gym_env.py:583-596: 'rgb_array' returns the overhead RGB image of the current state
        (rendered on the GPU at image_size); 'human' (interactive viewer) is out of scope."""
        if self.render_mode == "rgb_array":
            if self._vec._images is None:
                raise ValueError("render_mode='rgb_array' needs image_size > 0")
            return self._vec._images[0, 0].cpu().numpy()
        if self.render_mode == "human":
            raise NotImplementedError("the interactive MuJoCo viewer is out of scope (no display on the GPU box)")
        return None

    def close(self):
        self._vec.close()


__all__ = ["PickPlaceGymEnv", "ACTION_MODES", "BINS", "OBJECTS"]

if _gym is not None:
    try:
        from gymnasium.envs.registration import register

        register(id="mujoco_manip_amd/PickPlace-v0", entry_point="mujoco_manip_amd.gym_env:PickPlaceGymEnv")
    except Exception:
        pass
