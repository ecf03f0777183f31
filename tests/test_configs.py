"""BASELINE.json configs C2 and C4 on the HIP path against the oracle (VERDICT r02 "next" #1).

  * C2 (configs[1]): keyframe start, fixed task (obj_red, bin_red), randomize_objects=False, the
    plan(16) expert (generate_dataset.py:140-196): to FSM done against the oracle's run_episode at
    the SURVEY §8d L2 bar, and under the bench's gym autoreset (episodes end at the staged
    reward's termination) against the oracle's gym episode.
  * C4 (configs[3]): shards r = 0 and r = 7 of the real 8 x 4096 layout, each a full 4096-env
    batch seeded by global index (shard_seeds(42, r, 8, 4096)); every env runs its first episode to
    FSM done.  Properties over the whole shard (every cube placed, no error), and 16 sampled envs
    per shard against the oracle's run_episode by global index.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

BIN_POS = np.array([(-0.3, 0.55, 0.24), (0.0, 0.65, 0.24), (0.3, 0.55, 0.24)])


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import _lib

    _lib.load(build_if_missing=False)


def _placed(cube, b):
    return bool(np.hypot(*(cube[:2] - BIN_POS[b][:2])) < 0.05 and cube[2] < BIN_POS[b][2] + 0.06)


def oracle_episode(seed, fixed_task=None, randomize=True):
    """scripts/generate_dataset.py:140-196 on the oracle: plan(16) -> abs_pos step until the FSM
    is done.  Returns (task, env steps, success seen, final cube, placed)."""
    import oracle_py as O
    from mujoco_manip_amd.constants import BINS, OBJECTS, TASK_SETS

    pool = [(OBJECTS.index(o), BINS.index(b)) for o, b in TASK_SETS["all"]]
    e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=randomize, tasks=pool,
                    task=fixed_task)
    e.reset(seed=seed)
    o, b = e.task()
    e.fsm_init([(o, b)])
    n, succ = 0, False
    for _ in range(500):
        if e.fsm_plan(16) == 10:
            break
        f = e.fsm_get()
        _, _, _, _, info = e.step(np.array([*f["target"], float(f["gripper_open"])], np.float32))
        succ |= info["success"]
        n += 1
    cube = e.get_state()[0][9 + 7 * o: 12 + 7 * o].copy()
    return (o, b), n, succ, cube, _placed(cube, b)


def run_episodes(env, n_episodes, max_steps=600):
    """Host-driven expert loop (expert_plan(16) -> step) recording, per env and episode, the length,
    the success flag and the target cube when the FSM reports DONE (before the step that autoresets
    it, as run_episode breaks there)."""
    N = env.num_envs
    length = np.full((N, n_episodes), -1)
    final = np.zeros((N, n_episodes, 3), np.float32)
    succ = np.zeros((N, n_episodes), bool)
    task = np.zeros((N, n_episodes, 2), int)
    ep = np.zeros(N, int)
    t0 = np.zeros(N, int)
    for t in range(max_steps):
        act = env.expert_plan(16)
        fsm = env.fsm_state.cpu().numpy()
        epi = env._epi[:, :2].cpu().numpy()
        q = env.qpos.cpu().numpy()
        ended = (fsm == 10) & (ep < n_episodes)
        for k in np.where(ended)[0]:
            o = epi[k, 0]
            final[k, ep[k]] = q[k, 9 + 7 * o: 12 + 7 * o]
            length[k, ep[k]] = t - t0[k]
            task[k, ep[k]] = epi[k]
            ep[k] += 1
            t0[k] = t + 1
        if (ep >= n_episodes).all():
            break
        _, _, _, trunc, info = env.step(act)
        s = info["success"].cpu().numpy()
        live = (ep < n_episodes) & ~ended  # the DONE step itself belongs to no recorded episode
        succ[live, ep[live]] |= s[live]
    return length, succ, final, task


def _c2_env(n, autoreset):
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(n, task=("obj_red", "bin_red"), tasks="all", action_mode="abs_pos", reward_type="staged",
                          randomize_objects=False, image_size=0, autoreset=autoreset)
    env.reset(seed=list(range(n)))
    return env


def test_c2_fixed_task_keyframe_expert_matches_oracle():
    """C2 to FSM done (run_episode semantics: terminated / truncated ignored,
    generate_dataset.py:140-196) on 16 lockstep envs: each equals the oracle's run_episode of the
    keyframe (obj_red, bin_red) task at the L2 bar, and the 16 envs are bit-identical."""
    N = 16
    env = _c2_env(N, autoreset=False)
    length, succ, final, task = run_episodes(env, 1)
    length, succ, final, task = length[:, 0], succ[:, 0], final[:, 0], task[:, 0]
    assert (length >= 0).all(), length
    assert (env.env_error.cpu().numpy() == 0).all() and (task == 0).all()
    (o, b), n, rs, rcube, rplaced = oracle_episode(0, fixed_task=(0, 0), randomize=False)
    assert (o, b) == (0, 0) and rplaced
    for k in range(N):
        d = float(np.linalg.norm(final[k] - rcube))
        assert abs(int(length[k]) - n) <= 2 and d <= 0.01, (k, int(length[k]), n, d)
        assert bool(succ[k]) == rs and _placed(final[k], 0) == rplaced, k
    assert (length == length[0]).all() and (final == final[0]).all()
    print(f"C2 run_episode length {int(length[0])} (oracle {n}), cube error {np.linalg.norm(final[0] - rcube):.2e}")
    env.close()


def oracle_gym_episode(fixed_task=(0, 0)):
    """One C2 episode under gym autoreset semantics (the bench's C2): plan(16) -> step until the
    step reports terminated / truncated or the FSM is done.  Returns (env steps including the
    ending one, ended by termination, cube placed at the end)."""
    import oracle_py as O

    e = O.OracleEnv(action_mode="abs_pos", reward_type="staged", randomize_objects=False, task=fixed_task)
    e.reset(seed=0)
    o, b = e.task()
    e.fsm_init([(o, b)])
    for t in range(500):
        if e.fsm_plan(16) == 10:
            return t, False, _placed(e.get_state()[0][9 + 7 * o: 12 + 7 * o], b)
        f = e.fsm_get()
        _, _, term, trunc, _ = e.step(np.array([*f["target"], float(f["gripper_open"])], np.float32))
        if term or trunc:
            return t + 1, term, _placed(e.get_state()[0][9 + 7 * o: 12 + 7 * o], b)
    raise AssertionError("oracle C2 episode did not end")


def test_c2_autoreset_episodes_match_oracle():
    """C2 as the bench runs it (gym autoreset): the keyframe episode ends with the staged reward's
    robot x obstacle termination during RETREAT (gym_env.py:428-430, reward -1), the cube already
    in the bin; 16 envs x 3 episodes end at the oracle's ending step (+-2), are all counted as
    placed by the sticky counter, and every episode repeats the first bit for bit."""
    from mujoco_manip_amd import _lib

    n_ref, term_ref, placed_ref = oracle_gym_episode()
    assert term_ref and placed_ref
    N, E = 16, 3
    env = _c2_env(N, autoreset=True)
    ends = [[] for _ in range(N)]
    t0 = np.zeros(N, int)
    for t in range(E * (n_ref + 10)):
        _, r, term, trunc, _ = env.step(env.expert_plan(16))
        d = (term | trunc).cpu().numpy()
        for k in np.where(d)[0]:
            ends[k].append((t + 1 - t0[k], bool(term[k])))
            t0[k] = t + 1
        if min(len(x) for x in ends) >= E:
            break
    epi = env._epi.cpu().numpy()
    for k in range(N):
        assert len(ends[k]) >= E, (k, ends[k])
        for length, by_term in ends[k][:E]:
            assert abs(length - n_ref) <= 2 and by_term == term_ref, (k, ends[k], n_ref)
        assert ends[k][:E] == ends[0][:E]
    assert (epi[:, _lib.EPI["placed"]] == epi[:, _lib.EPI["episodes"]] - 1).all()
    assert (epi[:, _lib.EPI["error_resets"]] == 0).all()
    print(f"C2 autoreset episode length {ends[0][0][0]} (oracle {n_ref}), ended by termination")
    env.close()


@pytest.mark.parametrize("rank", [0, 7])
def test_c4_shard_matches_oracle(rank):
    """C4 shard `rank` of 8 x 4096 (global-index seeds): all 4096 first episodes finish with the
    cube placed and no error; 16 envs spread over the shard match the oracle's run_episode of
    their global index (task equal, length +-2, success / placement equal, cube within 1 cm)."""
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.shard import shard_range, shard_seeds
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N, R = 4096, 8
    seeds = shard_seeds(42, rank, R, N)
    env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=0, autoreset=False)
    env.reset(seed=seeds)
    length, succ, final, task = run_episodes(env, 1, max_steps=500)
    length, succ, final, task = length[:, 0], succ[:, 0], final[:, 0], task[:, 0]
    assert (length >= 0).all(), np.where(length < 0)
    assert (env.env_error.cpu().numpy() == 0).all()
    assert int(env._epi[:, _lib.EPI["error_resets"]].sum().item()) == 0
    placed = np.array([_placed(final[k], task[k, 1]) for k in range(N)])
    assert placed.all(), np.where(~placed)
    glob = list(shard_range(rank, R, N))
    bad = []
    for k in np.linspace(0, N - 1, 16).astype(int):
        tk, n, rs, rcube, rplaced = oracle_episode(_lib.episode_seed(42, glob[k]))
        d = float(np.linalg.norm(final[k] - rcube))
        if tuple(task[k]) != tk or abs(int(length[k]) - n) > 2 or d > 0.01 or bool(succ[k]) != rs or \
                placed[k] != rplaced:
            bad.append((int(k), glob[k], tk, tuple(task[k]), int(length[k]), n, round(d, 4)))
    print(f"C4 shard {rank}: episode lengths {np.percentile(length, [0, 50, 100]).tolist()}, all placed")
    assert not bad, bad
    env.close()


def test_fsm_done_autoreset_reports_truncated():
    """host-action steps after the FSM reached DONE without success or termination:
    the autoreset that follows is reported as truncated (never a reset without a done flag)."""
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(4, tasks="all", action_mode="abs_pos", reward_type="dense", randomize_objects=True,
                          image_size=0, autoreset=True)
    env.reset(seed=[1, 2, 3, 4])
    env._epi[1, _lib.EPI["fsm_state"]] = 10  # as if mmx_expert_plan had reached DONE
    a = torch.tensor([[0.0, 0.45, 0.45, 1.0]] * 4, device="cuda")
    _, _, term, trunc, _ = env.step(a)
    assert term.cpu().numpy().tolist() == [False] * 4
    assert trunc.cpu().numpy().tolist() == [False, True, False, False]
    epi = env._epi.cpu().numpy()
    assert epi[:, _lib.EPI["step_count"]].tolist() == [1, 0, 1, 1]
    assert epi[:, _lib.EPI["fsm_state"]].tolist() == [0, 0, 0, 0]
    env.close()
