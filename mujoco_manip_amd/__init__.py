"""mujoco_manip_amd — MI355X-native batched pick-and-place simulator.

Drop-in for the hot path of Jack-Tattershall/mujoco-manip: PickPlaceGymEnv.step
(mujoco_manip/gym_env.py:536-581) = decode -> 16 x (DLS IK + mj_step) -> mj_forward ->
reward -> obs, plus reset/randomization and the FSM expert, executed for thousands of
environments in lockstep by HIP kernels (libmmx.so, C-ABI in include/mmx_api.h).
"""
from .constants import ACTION_REPEAT, ALL_TASKS, BINS, OBJECTS, TASK_SETS  # noqa: F401

__all__ = ["PickPlaceVecEnv", "PickPlaceGymEnv", "build_library", "episode_seed"]


def build_library(force: bool = False) -> str:
    from . import _build

    return _build.build(force=force)


def episode_seed(root: int, index: int) -> int:
    from . import _lib

    return _lib.episode_seed(root, index)


def __getattr__(name):
    if name == "PickPlaceVecEnv":
        from .vec_env import PickPlaceVecEnv

        return PickPlaceVecEnv
    if name == "PickPlaceGymEnv":
        from .gym_env import PickPlaceGymEnv

        return PickPlaceGymEnv
    raise AttributeError(name)
