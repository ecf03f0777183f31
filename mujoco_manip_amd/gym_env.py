"""PickPlaceGymEnv — single-env façade with the reference signature (gym_env.py:62-75).

A drop-in for mujoco_manip.gym_env.PickPlaceGymEnv on the numeric path: reset/step return
numpy observations (same keys; camera images from the HIP renderer when image_size > 0), float rewards and bool flags.
Internally it is a PickPlaceVecEnv with num_envs=1 running on the MI355X.
"""
from __future__ import annotations

import numpy as np
import torch

from .constants import ACTION_REPEAT, IMAGE_SIZE, MAX_EPISODE_STEPS
from .pose_utils import se3_from_pos_quat_g, se3_from_pos_rot6d_g
from .vec_env import PickPlaceVecEnv

ACTION_MODES = ("abs_pos", "ee_pos_quat_g", "ee_pos_rot6d_g", "ee_pos_quat_g_rel", "ee_pos_rot6d_g_rel")

try:  # keep the reference's registration id when gymnasium is available (mujoco_manip/__init__.py:3-6)
    import gymnasium as _gym

    _Base = _gym.Env
except Exception:  # gymnasium absent in this image
    _gym = None
    _Base = object


class PickPlaceGymEnv(_Base):
    metadata = {"render_modes": ["rgb_array", "human"], "render_fps": 30}

    def __init__(self, xml_path: str | None = None, task: tuple[str, str] | None = None, tasks="all",
                 action_mode: str = "ee_pos_quat_g_rel", reward_type: str = "dense", image_size: int = IMAGE_SIZE,
                 render_mode: str | None = None, max_episode_steps: int = MAX_EPISODE_STEPS,
                 randomize_objects: bool = False, spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45),
                 device: int = 0):
        if action_mode not in ACTION_MODES:
            raise ValueError(f"action_mode must be one of {ACTION_MODES}, got '{action_mode}'")
        # xml_path is accepted for signature compatibility: the model is compiled offline
        # (tools/compile_model.py) from the reference scene into mujoco_manip_amd/model/.
        self._vec = PickPlaceVecEnv(1, task=task, tasks=tasks, action_mode=action_mode, reward_type=reward_type,
                                    image_size=image_size, render_mode=render_mode,
                                    max_episode_steps=max_episode_steps, randomize_objects=randomize_objects,
                                    spawn_x_range=spawn_x_range, spawn_y_range=spawn_y_range, device=device)
        self._action_mode = action_mode
        self._reward_type = reward_type
        self.render_mode = render_mode
        self._seed_next = None

    @property
    def action_mode(self) -> str:
        return self._action_mode

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


if _gym is not None:
    try:
        from gymnasium.envs.registration import register

        register(id="mujoco_manip_amd/PickPlace-v0", entry_point="mujoco_manip_amd.gym_env:PickPlaceGymEnv")
    except Exception:
        pass
