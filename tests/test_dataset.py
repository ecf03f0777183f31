"""Dataset emission and replay (f4).

CPU: the batched action encodings against the golden-pinned oracle codecs, the LeRobot v3.0
writer round trip, the reference's configuration errors, phase strings.
GPU: batched episodes vs the oracle running the reference's run_episode loop
(generate_dataset.py:83-198) on the same seeds and tasks; replay of the written dataset
reproduces the generation trajectory (replay_actions.py:128-148).

LeRobot is not importable here, so the on-disk layout is checked against its documented v3.0
structure only (format unpinned); frame values are pinned against the oracle.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from mujoco_manip_amd import dataset as D  # noqa: E402
from mujoco_manip_amd.constants import BINS, OBJECTS, OBS_SLICES, TASK_SETS  # noqa: E402

NUMERIC = [k for k, f in D.FEATURES.items() if f["dtype"] == "float32"]


def test_image_features_roundtrip(tmp_path):
    """generate_dataset.py:250-260 (use_videos=False): image frames embedded as parquet structs
    {bytes: PNG, path}, decoded back bit-exactly; per-channel image stats in meta/stats.json."""
    rng = np.random.default_rng(5)
    small = {k: dict(v, shape=(16, 16, 3)) for k, v in D.FEATURES.items() if k in D.IMAGE_KEYS}
    feats = {**small, "observation.state": D.FEATURES["observation.state"]}
    eps = _synthetic_episodes(rng, feats, n_eps=2)
    root = str(tmp_path / "img")
    info = D.write_lerobot_v3(root, "u/img", eps, feats)
    assert info["features"]["observation.images.wrist"]["dtype"] == "image"
    _, _, frames = D.read_lerobot_v3(root)
    for ep in eps:
        for k in D.IMAGE_KEYS:
            want = np.stack([D.png_decode(b) for b in ep.frames[k]])
            np.testing.assert_array_equal(frames[ep.index][k], want)
    st = json.load(open(os.path.join(root, "meta", "stats.json")))
    assert np.array(st["observation.images.overhead"]["mean"]).shape == (3, 1, 1)


def _rigid(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = rng.uniform(-0.5, 0.5, 3)
    return T


def _ref_actions(target, g, T_init):
    """get_actions (generate_dataset.py:57-80) with the oracle's golden-pinned codecs."""
    import oracle_py as O

    Tt = np.eye(4)
    Tt[:3, :3] = D.TARGET_ORI
    Tt[:3, 3] = target
    Tr = np.linalg.inv(T_init) @ Tt
    enc = lambda T: (np.array([*T[:3, 3], *O.rotmat_to_quat_xyzw(T[:3, :3]), g], np.float32),  # noqa: E731
                     np.array([*T[:3, 3], *T[:2, :3].ravel(), g], np.float32))
    (qa, ra), (qr, rr) = enc(Tt), enc(Tr)
    return {"action.ee.pos_quat_g": qa, "action.ee.pos_rot6d_g": ra, "action.ee.pos_quat_g_rel": qr,
            "action.ee.pos_rot6d_g_rel": rr}


def test_encode_actions_matches_oracle_codecs():
    rng = np.random.default_rng(0)
    n = 64
    T = np.stack([_rigid(rng) for _ in range(n)])
    tgt = rng.uniform(-0.6, 0.6, (n, 3)).astype(np.float32)
    g = (rng.random(n) > 0.5).astype(np.float32)
    enc = D.encode_actions(torch.tensor(tgt), torch.tensor(g), torch.tensor(T))
    for i in range(n):
        ref = _ref_actions(tgt[i].astype(float), float(g[i]), T[i])
        for k in D.ACTION_KEYS:
            np.testing.assert_allclose(enc[k][i].numpy(), ref[k], atol=2e-6, err_msg=k)


def test_quat_branches_cover_all_cases():
    import oracle_py as O

    # trace > 0, and each of the three diagonal-dominant branches of pose_utils.py:57-82
    Rs = [np.eye(3), np.diag([1.0, -1.0, -1.0]), np.diag([-1.0, 1.0, -1.0]), np.diag([-1.0, -1.0, 1.0]),
          D.TARGET_ORI]
    q = D._quat_xyzw_t(torch.tensor(np.stack(Rs))).numpy()
    for R, qq in zip(Rs, q):
        np.testing.assert_allclose(qq, O.rotmat_to_quat_xyzw(R), atol=1e-12)


def test_phase_descriptions():
    # pick_and_place.py:128-149 through the State -> Phase map :38-49
    want = ["idle", "approaching the red cube", "grasping the red cube", "grasping the red cube",
            "lifting the red cube", "transporting the red cube to the blue bin",
            "transporting the red cube to the blue bin", "placing the red cube in the blue bin",
            "placing the red cube in the blue bin", "retreating to neutral position", "idle"]
    assert [D.phase_description(s, "obj_red", "bin_blue") for s in range(11)] == want
    assert D.make_task_string("obj_green", "bin_red") == "Pick green object and place in red bin"


def test_configuration_errors():
    with pytest.raises(ValueError, match="repo_id"):
        D.generate("")
    with pytest.raises(ValueError, match="Unknown task set"):
        D.resolve_tasks(None, "nope")
    with pytest.raises(ValueError, match="task must be"):
        D.resolve_tasks(["obj_red"], "all")
    with pytest.raises(ValueError, match="Unknown feature keys"):
        D.resolve_features(["observation.bogus"])
    assert set(D.IMAGE_KEYS) <= set(D.resolve_features(None))  # the default includes both cameras
    f = D.resolve_features(["observation.state", "next.reward"], reward_type="dense")
    assert list(f) == ["observation.state"]  # next.reward only for staged (generate_dataset.py:228-229)
    assert D.resolve_tasks(None, "cross") == TASK_SETS["cross"]


def _synthetic_episodes(rng, feats, n_eps=3):
    eps = []
    for e in range(n_eps):
        L = int(rng.integers(3, 9))
        ep = D.Episode(e, OBJECTS[e % 3], BINS[(e + 1) % 3], None, length=L)
        for k, f in feats.items():
            if f["dtype"] == "string":
                ep.frames[k] = [f"phase {e}.{t}" for t in range(L)]
            elif f["dtype"] == "image":
                ep.frames[k] = [D.png_encode(rng.integers(0, 256, f["shape"], dtype=np.uint8)) for _ in range(L)]
            else:
                ep.frames[k] = rng.normal(size=(L, *f["shape"])).astype(np.float32)
        eps.append(ep)
    return eps


def test_lerobot_v3_writer_roundtrip(tmp_path):
    import pyarrow.parquet as pq

    rng = np.random.default_rng(1)
    feats = {k: v for k, v in D.FEATURES.items() if k not in D.IMAGE_KEYS}
    eps = _synthetic_episodes(rng, feats)
    root = str(tmp_path / "user" / "ds")
    info = D.write_lerobot_v3(root, "user/ds", eps, feats)
    assert info["codebase_version"] == "v3.0" and info["fps"] == 30 and info["robot_type"] == "franka_panda"
    assert info["total_episodes"] == 3 and info["total_frames"] == sum(e.length for e in eps)
    for k in ("timestamp", "frame_index", "episode_index", "index", "task_index"):
        assert k in info["features"]
    disk_info, _, frames = D.read_lerobot_v3(root)
    assert disk_info == json.load(open(os.path.join(root, "meta", "info.json")))
    start = 0
    for ep in eps:
        fr = frames[ep.index]
        for k in NUMERIC:
            np.testing.assert_array_equal(fr[k], ep.frames[k].reshape(ep.length, -1))
        assert fr["observation.phase_description"] == ep.frames["observation.phase_description"]
        np.testing.assert_array_equal(fr["frame_index"], np.arange(ep.length))
        np.testing.assert_array_equal(fr["index"], start + np.arange(ep.length))
        np.testing.assert_allclose(fr["timestamp"], np.arange(ep.length) / 30.0, rtol=1e-6)
        start += ep.length
    tasks = pq.read_table(os.path.join(root, "meta", "tasks.parquet")).to_pylist()
    assert [t["task"] for t in tasks] == [D.make_task_string(e.obj, e.bin) for e in eps]
    meta = pq.read_table(os.path.join(root, "meta", "episodes", "chunk-000", "file-000.parquet")).to_pylist()
    assert [m["length"] for m in meta] == [e.length for e in eps]
    assert meta[1]["dataset_from_index"] == eps[0].length
    stats = json.load(open(os.path.join(root, "meta", "stats.json")))
    allx = np.concatenate([e.frames["observation.state"] for e in eps])
    np.testing.assert_allclose(stats["observation.state"]["mean"], allx.mean(0), rtol=1e-5, atol=1e-6)
    assert stats["observation.state"]["count"] == [len(allx)]


def test_writer_splits_data_files(tmp_path):
    rng = np.random.default_rng(2)
    feats = {"observation.state": D.FEATURES["observation.state"]}
    eps = _synthetic_episodes(rng, feats, n_eps=4)
    root = str(tmp_path / "ds")
    D.write_lerobot_v3(root, "ds", eps, feats, data_files_size_in_mb=1e-6)  # one episode per file
    files = sorted(os.listdir(os.path.join(root, "data", "chunk-000")))
    assert files == [f"file-{i:03d}.parquet" for i in range(4)]
    _, _, frames = D.read_lerobot_v3(root)
    for ep in eps:
        np.testing.assert_array_equal(frames[ep.index]["observation.state"], ep.frames["observation.state"])


def test_threaded_writer_matches_inline_and_keeps_png_uncompressed(tmp_path):
    """The background-thread writer (generate()'s) writes the same dataset as the inline one; PNG
    bytes take no dictionary encoding and the requested compression (here NONE), numeric columns
    keep snappy."""
    import pyarrow.parquet as pq

    rng = np.random.default_rng(3)
    feats = {k: v for k, v in D.FEATURES.items() if k in ("observation.state", "action.joint_pos")}
    feats.update({k: dict(D.FEATURES[k], shape=(8, 8, 3)) for k in D.IMAGE_KEYS})
    eps = _synthetic_episodes(rng, feats, n_eps=5)
    out = {}
    for mode in (False, True):
        root = str(tmp_path / f"ds{int(mode)}")
        w = D.LeRobotWriter(root, "u/ds", feats, threaded=mode, image_compression="NONE" if mode else "SNAPPY")
        for ep in eps:
            w.add_episode(ep)
        info = w.close()
        out[mode] = (info, D.read_lerobot_v3(root)[2], root)
    assert out[False][0] == out[True][0]
    for ep in eps:
        a, b = out[False][1][ep.index], out[True][1][ep.index]
        assert set(a) == set(b)
        for k in a:
            if isinstance(a[k], np.ndarray):
                np.testing.assert_array_equal(a[k], b[k])
            else:
                assert a[k] == b[k]
        for k in D.IMAGE_KEYS:  # (read back decoded)
            np.testing.assert_array_equal(np.stack(list(b[k])), np.stack([D.png_decode(x) for x in ep.frames[k]]))
    md = pq.ParquetFile(os.path.join(out[True][2], "data", "chunk-000", "file-000.parquet")).metadata
    comp = {md.row_group(0).column(i).path_in_schema: md.row_group(0).column(i).compression
            for i in range(md.num_columns)}
    enc = {md.row_group(0).column(i).path_in_schema: md.row_group(0).column(i).encodings
           for i in range(md.num_columns)}
    for k in D.IMAGE_KEYS:
        assert comp[f"{k}.bytes"] == "UNCOMPRESSED"
        assert not any("DICTIONARY" in e for e in enc[f"{k}.bytes"])
    assert comp["observation.state.list.element"] == "SNAPPY"


def _as_png_frames(frames):
    lens = np.array([len(b) for b in frames], np.int64)
    offs = np.zeros(len(frames) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    return D.PngFrames(np.frombuffer(b"".join(frames), np.uint8).copy(), offs)


def test_png_frames_sequence_and_writer(tmp_path):
    """PngFrames (an episode's PNG files in one buffer, as collect_episodes builds them with
    mmx_copy_ranges) reads like the list of files, and the writer's zero-copy per-episode chunks
    give the same dataset (frames, meta/stats.json, info, episode metadata) as list frames."""
    import pyarrow.parquet as pq

    rng = np.random.default_rng(5)
    feats = {k: v for k, v in D.FEATURES.items() if k in ("observation.state", "action.joint_pos")}
    feats.update({k: dict(D.FEATURES[k], shape=(8, 8, 3)) for k in D.IMAGE_KEYS})
    eps = _synthetic_episodes(rng, feats, n_eps=6)
    pf = _as_png_frames(eps[0].frames[D.IMAGE_KEYS[0]])
    want = eps[0].frames[D.IMAGE_KEYS[0]]
    assert len(pf) == len(want) and list(pf) == want and pf[-1] == want[-1] and pf[1:3] == want[1:3]
    assert pf.nbytes == sum(map(len, want)) == D._png_nbytes(want)
    with pytest.raises(IndexError):
        pf[len(want)]
    out = {}
    for mode in ("list", "buffer"):
        root = str(tmp_path / mode)
        w = D.LeRobotWriter(root, "u/ds", feats, threaded=False, batch_episodes=4)
        for ep in eps:
            if mode == "buffer":
                ep = D.Episode(ep.index, ep.obj, ep.bin, ep.seed, length=ep.length,
                               frames={k: (_as_png_frames(v) if k in D.IMAGE_KEYS else v) for k, v in ep.frames.items()})
            w.add_episode(ep)
        info = w.close()
        out[mode] = (info, D.read_lerobot_v3(root)[2], root)
    assert out["list"][0] == out["buffer"][0]
    for ep in eps:
        a, b = out["list"][1][ep.index], out["buffer"][1][ep.index]
        for k in a:
            if isinstance(a[k], np.ndarray):
                np.testing.assert_array_equal(a[k], b[k])
            else:
                assert a[k] == b[k], k
    for name in ("stats.json", "info.json"):
        assert open(os.path.join(out["list"][2], "meta", name)).read() == \
            open(os.path.join(out["buffer"][2], "meta", name)).read()
    meta = [pq.read_table(os.path.join(out[m][2], "meta", "episodes", "chunk-000", "file-000.parquet")).to_pylist()
            for m in ("list", "buffer")]
    assert meta[0] == meta[1]


def test_copy_ranges_host_helper():
    """mmx_copy_ranges (host code of the C-ABI library, no GPU): n byte ranges src[k] -> dst[k]."""
    from mujoco_manip_amd import _lib

    L = _lib.load(build_if_missing=False)
    a = np.frombuffer(b"0123456789abcdefghij", np.uint8).copy()
    out = np.zeros(12, np.uint8)
    src = np.array([a.ctypes.data + 10, a.ctypes.data, a.ctypes.data + 5, a.ctypes.data], np.uint64)
    dst = np.array([out.ctypes.data + 9, out.ctypes.data, out.ctypes.data + 2, out.ctypes.data + 2], np.uint64)
    ln = np.array([3, 2, 0, 4], np.int64)
    assert L.mmx_copy_ranges(4, src.ctypes.data, dst.ctypes.data, ln.ctypes.data) == 9
    assert out.tobytes() == b"010123\x00\x00\x00abc"
    bad = np.array([2, -1], np.int64)
    before = out.copy()
    assert L.mmx_copy_ranges(2, src.ctypes.data, dst.ctypes.data, bad.ctypes.data) == -1
    np.testing.assert_array_equal(out, before)  # nothing copied on bad arguments
    assert L.mmx_copy_ranges(0, None, None, None) == 0


def test_threaded_writer_reports_errors(tmp_path):
    rng = np.random.default_rng(4)
    feats = {"observation.state": D.FEATURES["observation.state"]}
    eps = _synthetic_episodes(rng, feats, n_eps=2)
    bad = D.Episode(2, "not_an_object", BINS[0], None, length=eps[0].length, frames=dict(eps[0].frames))
    bad.frames["observation.state"] = np.zeros((1, 3), np.float32)  # wrong shape: fails in the thread
    w = D.LeRobotWriter(str(tmp_path / "ds"), "ds", feats, threaded=True)
    for ep in eps + [bad]:
        w.add_episode(ep)
    with pytest.raises(Exception):
        w.close()


# ----------------------------------------------------------------------------------------- GPU
def _oracle_episode(seed, task, feats, reward_type="staged", randomize=True):
    """The reference run_episode loop (generate_dataset.py:83-198) on the fp64 oracle."""
    import oracle_py as O

    o, b = OBJECTS.index(task[0]), BINS.index(task[1])
    e = O.OracleEnv(action_mode="abs_pos", reward_type=reward_type, randomize_objects=randomize)
    obs = e.reset(seed=seed, task=(o, b))
    e.fsm_init([(o, b)])
    T_init = e.initial_ee()
    frames = {k: [] for k in feats}
    for _ in range(3000):
        if e.fsm_get()["state"] == D.FSM_DONE:
            break
        e.fsm_plan(16)
        f = e.fsm_get()
        g = 1.0 if f["gripper_open"] else 0.0
        for ok, fk in D.OBS_TO_FEATURE.items():
            if fk in feats:
                a, bb, _ = OBS_SLICES[ok]
                frames[fk].append(obs[a:bb].copy())
        acts = _ref_actions(f["target"], g, T_init)
        for k in D.ACTION_KEYS:
            if k in feats:
                frames[k].append(acts[k])
        if "observation.phase_description" in feats:
            frames["observation.phase_description"].append(D.phase_description(f["state"], *task))
        obs, r, term, trunc, info = e.step(np.array([*f["target"], g], np.float32))
        if "next.reward" in feats:
            frames["next.reward"].append(info["reward_components"])
    return frames


@pytest.mark.gpu
def test_batched_episodes_match_oracle_run_episode():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    feats = D.resolve_features([k for k in D.FEATURES if k not in D.IMAGE_KEYS])
    task_list = TASK_SETS["all"]
    eps, seeds = D.collect_episodes(3, task_list, set(feats), randomize_objects=True, seed=0, num_envs=2)
    assert seeds == D.episode_seeds(0, 3)
    for ep in eps:
        assert (ep.obj, ep.bin) == task_list[ep.index]
        ref = _oracle_episode(seeds[ep.index], (ep.obj, ep.bin), feats)
        L = len(ref["observation.state"])
        assert abs(ep.length - L) <= 3, (ep.index, ep.length, L)  # behavioural over an episode
        for k in feats:
            if k == "observation.phase_description":
                assert ep.frames[k][:5] == ref[k][:5]
                assert ep.frames[k][-1] == ref[k][-1]
            else:  # early frames: trajectories still comparable (fp32 vs fp64); the wrist camera sits
                # ~0.1 m from the cubes, so its normalised keypoints magnify EE pose error ~10x
                tol = 1e-3 if k == "observation.keypoints_wrist" else 1e-4
                np.testing.assert_allclose(ep.frames[k][:5], np.array(ref[k][:5]), atol=tol, err_msg=k)


@pytest.mark.gpu
def test_device_episode_queue():
    """mmx_queue_advance, the dataset loop's slot reassignment on the device: episodes go to the
    free / FSM-DONE slots in ascending slot order, each exactly once, the ended episode is reported
    per slot, and an assigned slot's state is bit for bit PickPlaceGymEnv.reset with that episode's
    seed and task (generate_dataset.py:263-277)."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N, E = 3, 7
    seeds = D.episode_seeds(5, E)
    tl = TASK_SETS["all"]
    codes = [(OBJECTS.index(tl[e % len(tl)][0]) << 4) | BINS.index(tl[e % len(tl)][1]) for e in range(E)]
    env = PickPlaceVecEnv(N, action_mode="abs_pos", randomize_objects=True, image_size=0)
    env.sim.queue_init(codes, seeds)
    slot = torch.empty(N, dtype=torch.int32, device=env.device)
    fin = torch.empty_like(slot)

    def reset_state(e):
        ref = PickPlaceVecEnv(1, action_mode="abs_pos", randomize_objects=True, image_size=0)
        ref.sim.reset(seeds=[seeds[e]], task_override=np.array([codes[e]], np.int32))
        q, v, _, _ = ref.sim.get_state()
        o = ref._obs.cpu().numpy()[0]
        ref.close()
        return q[0], v[0], o

    def check_slot(s, e):
        q, v, _, _ = env.sim.get_state()
        rq, rv, ro = reset_state(e)
        assert (q[s] == rq).all() and (v[s] == rv).all(), (s, e)
        assert (env._obs.cpu().numpy()[s] == ro).all(), (s, e)

    env.sim.queue_advance(slot.data_ptr(), fin.data_ptr())
    assert slot.tolist() == [0, 1, 2] and fin.tolist() == [-1, -1, -1]
    for s in range(N):
        check_slot(s, s)
    ended, nxt, checked = [], N, 0
    for _ in range(1500):
        a = env.expert_plan(16)
        env.sim.step(a.data_ptr(), a.shape[1])
        prev = slot.tolist()
        env.sim.queue_advance(slot.data_ptr(), fin.data_ptr())
        sl, fl = slot.tolist(), fin.tolist()
        for s in range(N):
            if fl[s] >= 0:  # the slot's episode ended: it takes the next one (ascending slot order)
                assert fl[s] == prev[s]
                ended.append(fl[s])
                assert sl[s] == (nxt if nxt < E else -1)
                if nxt < E and checked < 2:
                    check_slot(s, nxt)
                    checked += 1
                nxt += 1
            else:
                assert sl[s] == prev[s]
        if all(x < 0 for x in sl):
            break
    assert sorted(ended) == list(range(E)) and checked == 2
    env.close()


@pytest.mark.gpu
def test_generate_then_replay_reproduces_trajectory(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import replay as R

    keys = ["observation.state", "action.ee.pos_quat_g", "action.ee.pos_rot6d_g_rel", "next.reward"]
    path, info = D.generate("user/pp", num_episodes=4, root=str(tmp_path), tasks="match", randomize_objects=True,
                            seed=3, features=keys, num_envs=4)
    md = json.load(open(os.path.join(path, "metadata.json")))
    assert md["episode_seeds"] == D.episode_seeds(3, 4)
    r = R.replay(path, None, "action.ee.pos_quat_g")
    for j, e in enumerate(r["episodes"]):
        rec = r["frames"][e]["observation.state"]
        # abs pose actions decode to the generation's abs_pos targets: the same trajectory, bit for bit
        np.testing.assert_array_equal(r["obs_state"][j][:-1], rec[1:])
        assert r["err"][j][-1] < 0.02  # the episode ends once the EE reached the retreat target
    r6 = R.replay(path, [1, 2], "action.ee.pos_rot6d_g_rel")  # relative 6D: T_init @ T_rel
    for j, e in enumerate(r6["episodes"]):
        rec = r6["frames"][e]["observation.state"]
        np.testing.assert_allclose(r6["obs_state"][j][:20], rec[1:21], atol=1e-4)


def oracle_replay(path, episode_index, action_key):
    """scripts/replay_actions.py:58-148 on the oracle: the episode's seed / task from
    metadata.json, a fresh env in the key's action mode, one step per recorded action, and per
    frame the decoded target, the EE position (robot.ee_pos after the step) and their distance."""
    import oracle_py as O

    from mujoco_manip_amd import replay as R

    _, md, frames = D.read_lerobot_v3(path)
    seed, task, sx, sy = R.episode_setup(md, episode_index)
    mode = action_key.replace("action.", "").replace(".", "_")
    e = O.OracleEnv(action_mode=mode, reward_type="staged", randomize_objects=seed is not None,
                    spawn_x_range=sx, spawn_y_range=sy)
    e.reset(seed=seed, task=None if task is None else (OBJECTS.index(task[0]), BINS.index(task[1])))
    T_init = e.initial_ee()
    tgt, ee = [], []
    for a in frames[episode_index][action_key]:
        obs, *_ = e.step(a)
        tgt.append(O.decode_action(mode, a, T_init)[0])
        ee.append(obs[:3].astype(float))
    tgt, ee = np.array(tgt), np.array(ee)
    return tgt, ee, np.linalg.norm(ee - tgt, axis=1)


@pytest.mark.gpu
def test_replay_report_matches_oracle(tmp_path):
    """f4 against the oracle: a generated dataset's absolute-quaternion and
    relative-6D actions replayed through the HIP path (replay.replay, all episodes in one batch)
    and through the oracle (the reference's replay loop, replay_actions.py:128-148) give the same
    per-frame report: decoded targets within 1e-5 m, EE positions within 5 mm (the
    cube contacts of a whole episode are chaotic), errors within 5 mm per frame and 1 mm on the
    episode mean."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import replay as R

    keys = ["observation.state", "action.ee.pos_quat_g", "action.ee.pos_rot6d_g_rel"]
    path, _ = D.generate("user/rp", num_episodes=4, root=str(tmp_path), tasks="match", randomize_objects=True,
                         seed=11, features=keys, num_envs=4)
    for key in ("action.ee.pos_quat_g", "action.ee.pos_rot6d_g_rel"):
        r = R.replay(path, None, key)
        for j, ep in enumerate(r["episodes"]):
            tgt, ee, err = oracle_replay(path, ep, key)
            assert len(err) == len(r["err"][j])
            np.testing.assert_allclose(r["target"][j], tgt, atol=1e-5, err_msg=f"{key} ep {ep}")
            np.testing.assert_allclose(r["ee"][j], ee, atol=5e-3, err_msg=f"{key} ep {ep}")
            assert np.abs(r["err"][j] - err).max() < 5e-3, (key, ep)
            assert abs(r["err"][j].mean() - err.mean()) < 1e-3, (key, ep, r["err"][j].mean(), err.mean())


@pytest.mark.gpu
def test_image_frames_match_renderer_and_raycast(tmp_path):
    """f2 with cameras (generate_dataset.py:26-28, 250-260): the written PNG frames decode to
    exactly what the batched renderer draws for the recorded pre-step state, and that state's
    segment masks agree with the CPU ray caster (oracle/render_ref.py) at 224 x 224."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import render_ref as RR

    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    feats = D.resolve_features(["observation.images.overhead", "observation.images.wrist", "observation.state"])
    seen, states = {}, {}

    def hook(slots, ep_ids, env):
        q = env.qpos.cpu().numpy()
        for s, e in zip(slots, ep_ids):
            t = seen.get(int(e), 0)
            seen[int(e)] = t + 1
            if t in (0, 12, 40):
                states[(int(e), t)] = q[s].copy()

    eps, _ = D.collect_episodes(2, TASK_SETS["all"], set(feats), randomize_objects=True, seed=4, num_envs=2,
                                on_step=hook)
    root = str(tmp_path / "cams")
    D.write_lerobot_v3(root, "u/cams", eps, feats)
    _, _, frames = D.read_lerobot_v3(root)
    keys = sorted(states)
    env = PickPlaceVecEnv(len(keys), action_mode="abs_pos", image_size=224)
    env.reset(seed=0)
    q, v, c, w = env.sim.get_state()
    for j, k in enumerate(keys):
        q[j] = states[k]
    env.sim.set_state(q, v, c, w)
    env.sim.forward()
    torch.cuda.synchronize()
    rgb = env._images.cpu().numpy()
    seg = env.segmentation.cpu().numpy()
    for j, (e, t) in enumerate(keys):
        for cam, key in enumerate(D.IMAGE_KEYS):
            img = frames[e][key][t]
            assert img.shape == (224, 224, 3) and img.dtype == np.uint8
            assert (img == rgb[j, cam]).all(-1).mean() > 0.995, (e, t, key)
    from test_render import _oracle_pose_fn

    j, (e, t) = 1, keys[1]
    for cam, name in enumerate(("overhead", "wrist")):
        ref = RR.render_seg(_oracle_pose_fn(states[(e, t)]), name, 224)
        assert (seg[j, cam] == ref).mean() > 0.98, (name, (seg[j, cam] == ref).mean())


# ----------------------------------------------------------------------------- sharded generation
def test_rank_episodes_partition():
    """generate_dataset.py:263-277 per rank: the ranks' episode sets partition the job, each
    episode keeps its global index (hence seed and task) whatever the rank count."""
    for E, W in ((10, 1), (10, 3), (7, 8), (65536, 8)):
        parts = [D.rank_episodes(E, r, W) for r in range(W)]
        assert sorted(sum(parts, [])) == list(range(E))
        assert all(all(e % W == r for e in p) for r, p in enumerate(parts))
    with pytest.raises(ValueError):
        D.rank_episodes(4, 2, 2)


def _write_shards(tmp_path, eps, feats, world, cfg):
    path = str(tmp_path / "sharded")
    for r in range(world):
        mine = [e for e in eps if e.index % world == r]
        out = D.shard_dir(path, r, world)
        w = D.LeRobotWriter(out, "u/ds", feats, keep_image_sums=True)
        for j, ep in enumerate(mine):
            w.add_episode(D.Episode(j, ep.obj, ep.bin, ep.seed, dict(ep.frames), ep.length))
        md = dict(cfg, shard={"rank": r, "world_size": world, "global_episode_index": [e.index for e in mine]})
        w.close(extra_info={"generation_config": md})
        json.dump(md, open(os.path.join(out, "metadata.json"), "w"))
    return path


def test_merge_shards_equals_single_writer(tmp_path):
    """Shards written rank by rank (local episode numbering, global indices in metadata.json) merge
    into exactly the dataset one writer produces from all episodes in global order: frames, PNG
    bytes, meta/episodes, stats and info."""
    import pyarrow.parquet as pq

    rng = np.random.default_rng(11)
    feats = {k: v for k, v in D.FEATURES.items() if k not in D.IMAGE_KEYS}
    feats.update({k: dict(D.FEATURES[k], shape=(8, 8, 3)) for k in D.IMAGE_KEYS})
    eps = _synthetic_episodes(rng, feats, n_eps=7)
    for ep in eps:
        ep.obj, ep.bin = TASK_SETS["all"][ep.index % 9]
    cfg = {"repo_id": "u/ds", "num_episodes": 7, "features": None, "reward_type": "staged", "image_size": 8,
           "tasks": "all", "task": None}
    single = str(tmp_path / "single")
    w = D.LeRobotWriter(single, "u/ds", feats)
    for ep in eps:
        w.add_episode(ep)
    info1 = w.close(extra_info={"generation_config": cfg})
    path = _write_shards(tmp_path, eps, feats, 3, cfg)
    info2 = D.merge_shards(path, remove_shards=True)
    assert info1 == info2
    assert not [d for d in os.listdir(path) if d.startswith("shard-")]
    for rel in ("meta/stats.json", "meta/info.json"):
        assert json.load(open(os.path.join(single, rel))) == json.load(open(os.path.join(path, rel)))
    for rel in ("meta/episodes/chunk-000/file-000.parquet", "meta/tasks.parquet", "data/chunk-000/file-000.parquet"):
        assert pq.read_table(os.path.join(single, rel)).equals(pq.read_table(os.path.join(path, rel))), rel
    assert json.load(open(os.path.join(path, "metadata.json"))) == cfg


def test_merge_shards_rejects_missing_rank(tmp_path):
    rng = np.random.default_rng(12)
    feats = {"observation.state": D.FEATURES["observation.state"]}
    eps = _synthetic_episodes(rng, feats, n_eps=4)
    cfg = {"repo_id": "u/ds", "num_episodes": 4, "features": ["observation.state"], "reward_type": "staged",
           "tasks": "all", "task": None}
    path = _write_shards(tmp_path, eps, feats, 2, cfg)
    import shutil

    shutil.rmtree(D.shard_dir(path, 1, 2))
    with pytest.raises(ValueError, match="expected 2 shards"):
        D.merge_shards(path)


@pytest.mark.gpu
def test_sharded_generation_matches_single_process(tmp_path):
    """VERDICT r03 "next" #3: two rank processes (the dataset CLI under a torchrun-style
    environment, sharing the 1-GPU box's device, gloo for their gather) each write the shard of
    episodes e = rank (mod 2) with the global seeds and tasks; merged by global index, the dataset
    equals one process's bit for bit (numeric frames, PNG frames, statistics, metadata)."""
    import subprocess
    import sys

    import pyarrow.parquet as pq

    from tests_util_port import free_port

    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    args = ["--num-episodes", "5", "--randomize-objects", "--seed", "7", "--num-envs", "2", "--image-size", "32"]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = str(free_port())
    procs = [subprocess.Popen([sys.executable, "-m", "mujoco_manip_amd.dataset", "--repo-id", "u/sh",
                               "--root", str(tmp_path / "sh"), "--dist-backend", "gloo", *args], cwd=repo,
                              env=dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert [p.returncode for p in procs] == [0, 0], outs
    shards = json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][0])["shards"]
    assert [s["episodes"] for s in shards] == [3, 2]
    single, _ = D.generate("u/one", num_episodes=5, root=str(tmp_path / "one"), randomize_objects=True, seed=7,
                           num_envs=3, image_size=32)
    merged = str(tmp_path / "sh" / "u" / "sh")
    for rel in ("meta/stats.json",):
        assert json.load(open(os.path.join(single, rel))) == json.load(open(os.path.join(merged, rel)))
    i1, i2 = (json.load(open(os.path.join(p, "meta/info.json"))) for p in (single, merged))
    for k in ("generation_config",):
        i1[k].pop("repo_id"), i2[k].pop("repo_id"), i1[k].pop("root"), i2[k].pop("root")
    assert i1 == i2
    for rel in ("meta/episodes/chunk-000/file-000.parquet", "data/chunk-000/file-000.parquet"):
        assert pq.read_table(os.path.join(single, rel)).equals(pq.read_table(os.path.join(merged, rel))), rel
    # a shard replays on its own: its local episode 1 is global episode 2 (rank 0: 0, 2, 4)
    md = json.load(open(os.path.join(D.shard_dir(merged, 0, 2), "metadata.json")))
    from mujoco_manip_amd import replay as R

    assert R.episode_setup(md, 1)[0] == D.episode_seeds(7, 5)[2]


def test_frame_image_stats_exact():
    """Per-frame image statistics from integer sums (no float64 copy of the frames):
    equal to the float64 definition over every pixel."""
    rng = np.random.default_rng(13)
    imgs = rng.integers(0, 256, (5, 17, 23, 3), dtype=np.uint8)
    got = D._frame_image_stats(torch.as_tensor(imgs), chunk=2).numpy()
    x = imgs.reshape(5, -1, 3).astype(np.float64) / 255.0
    want = np.stack([x.min(1), x.max(1), x.sum(1), (x * x).sum(1)], 1)
    np.testing.assert_allclose(got, want, rtol=1e-13, atol=0)


def test_writer_io_lanes_match_single_thread(tmp_path):
    """Data files written side by side on I/O lanes (file f on lane f mod k) hold exactly what the
    single-thread writer writes: same files, same rows, same meta and statistics."""
    import pyarrow.parquet as pq

    rng = np.random.default_rng(14)
    feats = {k: v for k, v in D.FEATURES.items() if k in ("observation.state", "observation.phase_description")}
    feats.update({k: dict(D.FEATURES[k], shape=(8, 8, 3)) for k in D.IMAGE_KEYS})
    eps = _synthetic_episodes(rng, feats, n_eps=9)
    out = {}
    for k in (1, 3):
        root = str(tmp_path / f"io{k}")
        w = D.LeRobotWriter(root, "u/ds", feats, threaded=True, io_threads=k, data_files_size_in_mb=2e-3)
        for ep in eps:
            w.add_episode(ep)
        out[k] = (w.close(), root)
    assert out[1][0] == out[3][0]
    files = sorted(os.listdir(os.path.join(out[1][1], "data", "chunk-000")))
    assert len(files) >= 3 and files == sorted(os.listdir(os.path.join(out[3][1], "data", "chunk-000")))
    for rel in [os.path.join("data", "chunk-000", f) for f in files] + ["meta/episodes/chunk-000/file-000.parquet"]:
        assert pq.read_table(os.path.join(out[1][1], rel)).equals(pq.read_table(os.path.join(out[3][1], rel))), rel
    assert json.load(open(os.path.join(out[1][1], "meta/stats.json"))) == json.load(open(os.path.join(out[3][1], "meta/stats.json")))
