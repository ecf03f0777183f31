"""PickPlaceVecEnv — batched torch façade over the C-ABI (one MI355X, num_envs lanes).

Mirrors PickPlaceGymEnv (mujoco_manip/gym_env.py:39-602) with a leading env dimension:
same constructor keywords, same 5 action modes, same numeric observation keys and reward
types.  Differences, all documented in DESIGN.md:
  * observations are torch tensors on the GPU ([N, ...]); with image_size > 0 the
    `image_overhead` / `image_wrist` keys are uint8 [N, S, S, 3] from the batched HIP rasteriser
    (mmx_render.hip: the Panda's visual parts reduced to convex pieces and clustered meshes per
    part, flat-lit with the scene's lights, no shadows or specular), image_size = 0
    skips them;
  * reset(seed=s) seeds env i with s + i (gymnasium vector convention); a list gives one
    seed per env;
  * with autoreset=True an env that terminated/truncated (or whose FSM expert finished: reported
    as truncated) is reset inside the same step (the returned obs is the first obs of the new
    episode).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .constants import ACTION_REPEAT, BINS, IMAGE_SIZE, MAX_EPISODE_STEPS, OBJECTS, OBS_SLICES, TASK_SETS, task_index


class PickPlaceVecEnv:
    metadata = {"render_modes": [], "render_fps": 30}

    def __init__(self, num_envs: int = 1, task: tuple[str, str] | None = None, tasks="all",
                 action_mode: str = "ee_pos_quat_g_rel", reward_type: str = "dense", image_size: int = IMAGE_SIZE,
                 render_mode: str | None = None, max_episode_steps: int = MAX_EPISODE_STEPS,
                 randomize_objects: bool = False, spawn_x_range=(-0.20, 0.20), spawn_y_range=(0.30, 0.45),
                 autoreset: bool = False, device: int = 0, solver_iterations: int = 30,
                 solver_tolerance: float = 1e-6):
        if not torch.cuda.is_available():
            raise RuntimeError("PickPlaceVecEnv needs an MI355X GPU (HIP); no CPU fallback exists")
        pool = TASK_SETS[tasks] if isinstance(tasks, str) else list(tasks)
        self.num_envs = int(num_envs)
        self.device = torch.device(f"cuda:{device}")
        self.render_mode = render_mode
        self._action_mode = action_mode
        self._reward_type = reward_type
        self._task_pool = pool
        self._fixed_task = task
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
        self.sim = _lib.Sim(self.num_envs, action_mode=action_mode, reward_type=reward_type,
                            max_episode_steps=max_episode_steps, randomize_objects=randomize_objects,
                            spawn_x_range=spawn_x_range, spawn_y_range=spawn_y_range,
                            task_pool=[task_index(t) for t in pool],
                            fixed_task=None if task is None else task_index(task), image_size=image_size,
                            autoreset=autoreset, solver_iterations=solver_iterations,
                            solver_tolerance=solver_tolerance, device=device, stream=stream)
        s = self.sim
        self.action_dim = s.action_dim
        self._obs = s.view("obs", _lib.NOBS)
        self._reward = s.view("reward", 1)
        self._done = s.view("done", 3, "<i4")
        self._rc = s.view("reward_components", 6)
        self._epi = s.view("episode_i", _lib.EPI_N, "<i4")
        self._epf = s.view("episode_f", _lib.EPF_N)
        self.qpos = s.view("qpos", _lib.NQ)
        self.qvel = s.view("qvel", _lib.NV)
        self.ctrl = s.view("ctrl", _lib.NU)
        self.stats = s.view("stats", _lib.STAT_N)
        self._expert_action = torch.zeros(self.num_envs, 4, device=self.device, dtype=torch.float32)
        iv = s.image_views()
        self._images, self._seg = iv if iv is not None else (None, None)

    # ------------------------------------------------------------------ gym API
    def _obs_dict(self):
        flat = self._obs
        out = {}
        for k, (a, b, shape) in OBS_SLICES.items():
            out[k] = flat[:, a:b].reshape(self.num_envs, *shape).clone()
        if self._images is not None:  # gym_env.py:325-326
            out["image_overhead"] = self._images[:, 0].clone()
            out["image_wrist"] = self._images[:, 1].clone()
        return out

    @property
    def segmentation(self) -> torch.Tensor | None:
        """Segment ids [N, 2, S, S] of the last rendered images (overhead, wrist), or None."""
        return None if self._seg is None else self._seg.clone()

    def reset(self, *, seed=None, options: dict | None = None):
        """PickPlaceGymEnv.reset (gym_env.py:477-534), batched."""
        N = self.num_envs
        seeds = None
        if seed is not None:
            seeds = [int(seed) + k for k in range(N)] if np.isscalar(seed) else list(seed)
        task = None
        if options and "task" in options:
            t = options["task"]
            if isinstance(t, tuple) and isinstance(t[0], str):
                o, b = task_index(t)
                task = np.full(N, (o << 4) | b, np.int32)
            else:
                task = np.array([(task_index(x)[0] << 4) | task_index(x)[1] for x in t], np.int32)
        self.sim.reset(seeds=seeds, task_override=task)
        return self._obs_dict(), {}

    def synchronize(self):
        """Wait for the env's queued launches.  Raises the reference's RuntimeError (randomization.py:84-87)
        when an autoreset since the last reset / synchronize exhausted its spawn sampling (that env's
        env_error carries bit 8 and its cubes stay at the keyframe, as where the reference raises)."""
        self.sim.synchronize()

    def step(self, actions: torch.Tensor):
        """PickPlaceGymEnv.step (gym_env.py:536-581), batched: actions [N, action_dim] fp32 on the GPU."""
        a = torch.as_tensor(actions, dtype=torch.float32, device=self.device)
        if a.dim() != 2 or a.shape[0] != self.num_envs or a.shape[1] < self.action_dim:
            raise ValueError(f"actions must be [{self.num_envs}, {self.action_dim}], got {tuple(a.shape)}")
        a = a.contiguous()
        self.sim.step(a.data_ptr(), a.shape[1])
        obs = self._obs_dict()
        reward = self._reward.clone()
        terminated = self._done[:, 0].bool().clone()
        truncated = self._done[:, 1].bool().clone()
        info = {"success": self._done[:, 2].bool().clone()}
        if self._reward_type == "staged":
            info["reward_components"] = self._rc.clone()
        self._last_action = a
        return obs, reward, terminated, truncated, info

    # ------------------------------------------------------------------ expert + helpers
    def expert_plan(self, n_steps: int = ACTION_REPEAT) -> torch.Tensor:
        """PickAndPlaceTask.plan(n_steps) for all envs -> abs_pos actions [N, 4]."""
        self.sim.expert_plan(n_steps, self._expert_action.data_ptr())
        return self._expert_action.clone()

    def rollout_expert(self, n_env_steps: int):
        """Device-resident FSM rollout (generate_dataset.py:140-196), no host round trips."""
        self.sim.rollout_expert(n_env_steps)

    @property
    def step_count(self) -> torch.Tensor:
        return self._epi[:, 2].clone()

    @property
    def tasks(self) -> list[tuple[str, str]]:
        ob = self._epi[:, 0].cpu().numpy()
        bn = self._epi[:, 1].cpu().numpy()
        return [(OBJECTS[o], BINS[b]) for o, b in zip(ob, bn)]

    @property
    def fsm_state(self) -> torch.Tensor:
        return self._epi[:, 4].clone()

    @property
    def episode_flags(self) -> torch.Tensor:
        """staged-reward sticky flags: 1 grasped, 2 lifted, 4 above target, 8 placed"""
        return self._epi[:, 3].clone()

    @property
    def env_error(self) -> torch.Tensor:
        return self._epi[:, 9].clone()

    @property
    def initial_ee_se3(self) -> torch.Tensor:
        T = torch.zeros(self.num_envs, 4, 4, device=self.device)
        f = self._epf
        T[:, :3, :3] = f[:, 0:9].reshape(-1, 3, 3)
        T[:, :3, 3] = f[:, 9:12]
        T[:, 3, 3] = 1.0
        return T

    def solver_stats(self) -> dict:
        s = self.stats.double().sum(dim=0).cpu().numpy()
        sub = max(s[3], 1.0)
        ks, kc = _lib.STAT_FIELDS.index("exit_stall"), _lib.STAT_FIELDS.index("exit_cap")
        out = {"mean_nefc": s[0] / sub, "mean_ncon": s[1] / sub, "mean_solver_iter": s[2] / sub,
               "max_resid": float(self.stats[:, 4].max().item()), "substeps": int(s[3]),
               # substeps whose Newton solve ended above the tolerance, by cause
               "exit_above_tol": {"no_progress": int(s[ks]), "iteration_cap": int(s[kc]),
                                  "fraction": float((s[ks] + s[kc]) / sub)}}
        # per-phase shader-clock cycles per substep per env (s_memtime ticks = shader cycles)
        for k, name in enumerate(_lib.STAT_FIELDS[5:17], start=5):
            out[name + "_per_substep"] = s[k] / sub
        return out

    def clear_stats(self):
        self.stats.zero_()

    def close(self):
        self.sim.close()
