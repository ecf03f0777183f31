"""Camera renderer: mask-level parity of the batched HIP rasterizer.

Pixel parity with MuJoCo's OpenGL renderer is not attainable (and MuJoCo is absent), so the
images are pinned at the level SURVEY §8 f1 names: segment masks against the CPU ray caster
oracle/render_ref.py on the same states (body poses from the fp64 oracle), the analytic pinhole
projection of the cubes, and a keypoint overlay with the reference's own keypoint projection
(cameras.py:56-104).  That projection divides by the camera-frame z, which is negative in front
of a MuJoCo camera, so its (u, v) is the image point mirrored through the centre: the overlay
checks the rendered mask at (1 - u, 1 - v).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

SEG_CUBE = {0: 6, 1: 7, 2: 8}


def _oracle_pose_fn(qpos):
    import oracle_py as O

    e = O.OracleEnv()
    e.set_state(qpos=np.asarray(qpos, float))
    e.mj_forward()
    cache = {}

    def pose(b):
        if b not in cache:
            p, R = e.body(b)
            cache[b] = (R, p)
        return cache[b]

    return pose


def _keyframe_qpos():
    import json
    import os

    m = json.load(open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "mujoco_manip_amd", "model",
                                    "panda_pickplace.json")))
    return np.array(m["key_qpos"], float)


def test_raycast_checker_against_analytic_projection():
    """Pin the checker: each cube's centre pixel (true pinhole image point) is that cube."""
    import render_ref as RR

    q = _keyframe_qpos()
    q[0] = -1.5708  # arm turned away from the table: no cube occluded
    pose = _oracle_pose_fn(q)
    S = 64
    seg = RR.render_seg(pose, "overhead", S)
    cR, cp = RR.camera_pose("overhead", pose)
    f = (S / 2) / np.tan(np.radians(45.0) / 2)
    for k in range(3):
        c = cR.T @ (q[9 + 7 * k:12 + 7 * k] - cp)
        col = S / 2 + f * c[0] / -c[2]
        row = S / 2 - f * c[1] / -c[2]
        assert seg[int(row), int(col)] == SEG_CUBE[k]
    assert (seg == 2).sum() > 0.1 * S * S  # the table fills a good part of the overhead view
    assert (seg == 1).sum() > 0            # floor around it
    wrist = RR.render_seg(_oracle_pose_fn(_keyframe_qpos()), "wrist", S)  # looking at the table
    assert {2, 6, 7, 8} <= set(np.unique(wrist).tolist())


def _gpu_states(n=3, steps=40, size=64):
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=size)
    env.reset(seed=[_lib.episode_seed(11, i) for i in range(n)])
    for _ in range(steps):
        obs, *_ = env.step(env.expert_plan(16))
    torch.cuda.synchronize()
    return env, obs


@pytest.mark.gpu
@pytest.mark.parametrize("size", [64, 84])
def test_render_masks_match_raycast(size):
    """Segment masks vs the ray caster; 84 is not a multiple of 16 (the reference accepts any
    image size: the raster grid rounds up, the pixels outside the image are not written)."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import render_ref as RR

    env, obs = _gpu_states(n=3, steps=40, size=size)
    seg = env.segmentation.cpu().numpy()
    assert seg.shape == (3, 2, size, size) and obs["image_wrist"].shape == (3, size, size, 3)
    qpos = env.qpos.cpu().numpy()
    for i in range(3):
        pose = _oracle_pose_fn(qpos[i])
        for ci, cam in enumerate(("overhead", "wrist")):
            ref = RR.render_seg(pose, cam, size)
            agree = (seg[i, ci] == ref).mean()
            assert agree > 0.98, (i, cam, agree)  # silhouette edges may differ by a pixel
            for sid in np.unique(ref):
                a, b = seg[i, ci] == sid, ref == sid
                if b.sum() >= 30:  # objects large enough for an IoU to mean something
                    iou = (a & b).sum() / (a | b).sum()
                    assert iou > 0.85, (i, cam, int(sid), iou)


@pytest.mark.gpu
def test_render_keypoint_overlay_and_colours():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import render_ref as RR

    S = 128
    env, obs = _gpu_states(n=2, steps=3, size=S)  # cubes still on the table, arm above them
    seg = env.segmentation.cpu().numpy()
    rgb = obs["image_overhead"].cpu().numpy()
    assert rgb.shape == (2, S, S, 3) and rgb.dtype == np.uint8
    kp = obs["keypoints_overhead"].cpu().numpy()  # reference projection (cameras.py:56-104)
    qpos = env.qpos.cpu().numpy()
    checked = 0
    for i in range(2):
        ref = RR.render_seg(_oracle_pose_fn(qpos[i]), "overhead", S)
        for k in range(3):
            u, v = kp[i, k]
            col, row = int((1.0 - u) * S), int((1.0 - v) * S)
            if ref[row, col] != SEG_CUBE[k]:
                continue  # occluded by the arm in this state
            assert seg[i, 0, row, col] == SEG_CUBE[k]
            checked += 1
            r, g, b = rgb[i, row, col].astype(int)
            assert [r, g, b][k] == max(r, g, b) and [r, g, b][k] > 100  # red / green / blue cube
        floor = rgb[i][seg[i, 0] == 1]
        assert len(np.unique(floor, axis=0)) >= 2  # checker squares
    assert checked >= 2
    # a re-render of the same state (mj_forward's lane-serial kinematics instead of the step's
    # wave-parallel one: same poses up to fp32 rounding) reproduces the image
    env.sim.forward()
    torch.cuda.synchronize()
    assert (env._images[:, 0].cpu().numpy() == rgb).all(-1).mean() > 0.995


# --------------------------------------------------------------------------- fidelity vs full meshes
def _fixture():
    import os

    return np.load(os.path.join(os.path.dirname(__file__), "golden", "robot_masks.npz"))


def _iou(a, b):
    return float((a & b).sum()) / max(float((a | b).sum()), 1.0)


# robot-mask IoU against the full 134,888-triangle visual meshes (tests/golden/make_robot_masks.py):
# one convex hull per body (the r02 model) reached 0.89 (overhead) / 0.75 (wrist) on these states,
# the r03-r05 convex pieces 0.92 / 0.97, the quadric-error model (tools/compile_render.py) 0.973 / 0.977
IOU_MIN = {"overhead": 0.97, "wrist": 0.97}
IOU_GPU_SLACK = 0.02  # the HIP rasteriser's edge rules against make_robot_masks.raster_depth: gate 0.95


def test_render_model_robot_silhouettes_match_full_meshes():
    """The render model's robot (convex pieces per link part, clustered hand / fingers; front
    faces only, as the rasterizer culls) against the full visual meshes, same poses and z-buffer
    rules (make_robot_masks.raster_depth): mean robot-mask IoU per camera above IOU_MIN."""
    import json
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_robot_masks as MR
    import render_ref as RR

    d = _fixture()
    rm = json.load(open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "mujoco_manip_amd", "model",
                                     "render_model.json")))
    seg = np.array([rm["materials"][k]["seg"] for k in rm["tri_mat"]])
    V, vb, tris = np.array(rm["verts"], float), np.array(rm["vert_body"]), np.array(rm["tris"])
    ious = {"overhead": [], "wrist": []}
    for k, q in enumerate(d["qpos"]):
        pose = _oracle_pose_fn(q)
        Vw = np.empty_like(V)
        for b in np.unique(vb):
            R, p = pose(int(b))
            Vw[vb == b] = V[vb == b] @ np.asarray(R).T + p
        for c, cam in enumerate(("overhead", "wrist")):
            cR, cp = RR.camera_pose(cam, pose)
            fovy = [x for x in rm["cameras"] if x["name"] == cam][0]["fovy"]
            rw = Vw[tris[seg == 9]]
            cam_pts = (rw - cp) @ cR
            front = np.einsum("ij,ij->i", np.cross(cam_pts[:, 1] - cam_pts[:, 0], cam_pts[:, 2] - cam_pts[:, 0]),
                              cam_pts[:, 0]) < 0
            zr = MR.raster_depth(rw[front], cR, cp, fovy)
            zs = MR.raster_depth(Vw[tris[seg != 9]], cR, cp, fovy)
            ious[cam].append(_iou(zr < zs, d["masks"][k, c].astype(bool)))
    print({c: [round(x, 3) for x in v] for c, v in ious.items()})
    for cam, v in ious.items():
        assert np.mean(v) >= IOU_MIN[cam], (cam, v)


@pytest.mark.gpu
def test_gpu_robot_silhouettes_match_full_meshes():
    """The HIP renderer's robot segment (id 9) at 128 x 128 for the fixture's states against the
    full visual meshes: mean IoU per camera above IOU_MIN less IOU_GPU_SLACK (edge rules differ)."""
    from mujoco_manip_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    d = _fixture()
    n = len(d["qpos"])
    sim = _lib.Sim(n, action_mode="abs_pos", image_size=int(d["size"]))
    sim.reset()
    q, v, c, w = sim.get_state()
    q[:] = d["qpos"].astype(np.float32)
    sim.set_state(q, v, c, w)
    sim.forward()
    torch.cuda.synchronize()
    seg = sim.image_views()[1].cpu().numpy()
    sim.close()
    for ci, cam in enumerate(("overhead", "wrist")):
        ious = [_iou(seg[k, ci] == 9, d["masks"][k, ci].astype(bool)) for k in range(n)]
        print(cam, [round(x, 3) for x in ious])
        assert np.mean(ious) >= IOU_MIN[cam] - IOU_GPU_SLACK, (cam, ious)


@pytest.mark.gpu
def test_c5_full_batch_properties():
    """C5 at full size (VERDICT r03 "next" #5): 8192 envs x both 128 x 128 cameras, 16 fused
    expert env steps through the launch shape the bench uses (one longest-first step launch and one
    render launch over all envs per step): no env error, every segment id a valid material class, no
    constant camera image, and 4 envs spread over the batch against the CPU ray caster."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import render_ref as RR

    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N, S = 8192, 128
    env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=S, autoreset=True)
    env.reset(seed=[_lib.episode_seed(42, i) for i in range(N)])
    assert env.sim.rollout_lanes == 1  # camera rollouts: one step launch over all envs, then the render
    env.rollout_expert(16)
    torch.cuda.synchronize()
    assert int((env.env_error != 0).sum().item()) == 0
    seg = env.segmentation
    assert seg.shape == (N, 2, S, S)
    assert int(seg.max().item()) <= 9
    rgb, _ = env.sim.image_views()
    flat = rgb.reshape(N, 2, -1)
    assert bool((flat.amax(-1) > flat.amin(-1)).all()), "a constant camera image"
    qpos = env.qpos.cpu().numpy()
    for i in (5, 2048 + 700, 4096 + 1500, N - 1):
        pose = _oracle_pose_fn(qpos[i])
        for ci, cam in enumerate(("overhead", "wrist")):
            ref = RR.render_seg(pose, cam, S)
            agree = (seg[i, ci].cpu().numpy() == ref).mean()
            assert agree > 0.98, (i, cam, agree)
    env.close()


@pytest.mark.gpu
def test_render_overlap_bit_identical(monkeypatch):
    """MMX_RENDER_OVERLAP=1: the render of step k runs on its own stream beside step k + 1 with the
    body poses double-buffered; images, segment ids and states after an odd number of camera steps
    (the pose buffers swap roles) equal the serial rollout's bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    N, S = 2048, 64
    outs = []
    for ov in ("0", "1"):
        monkeypatch.setenv("MMX_RENDER_OVERLAP", ov)
        env = PickPlaceVecEnv(N, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                              image_size=S, autoreset=True)
        env.reset(seed=[_lib.episode_seed(5, i) for i in range(N)])
        env.rollout_expert(7)
        torch.cuda.synchronize()
        rgb, _ = env.sim.image_views()
        q, v, _, _ = env.sim.get_state()
        outs.append((rgb.cpu().numpy().copy(), env.segmentation.cpu().numpy().copy(), q.copy(), v.copy()))
        env.rollout_expert(2)  # a second call starts from the swapped buffers
        torch.cuda.synchronize()
        rgb, _ = env.sim.image_views()
        outs[-1] = outs[-1] + (rgb.cpu().numpy().copy(),)
        env.close()
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_render_after_divergence_without_autoreset():
    """with autoreset off (the dataset loop's setting) a diverged env's NaN / Inf poses
    reach the renderer.  The step must flag the env (env_error NaN bit), the render must complete
    without a fault, and every other env's images must equal a run without the injected state bit
    for bit (the renderer's NaN culling is an integer test, independent of the fp-math flags)."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    outs = []
    for inject in (False, True):
        env = PickPlaceVecEnv(4, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                              image_size=64, autoreset=False)
        env.reset(seed=[_lib.episode_seed(13, i) for i in range(4)])
        if inject:
            q, v, c, w = env.sim.get_state()
            v[1, 3] = np.nan
            v[2, 0] = np.inf
            env.sim.set_state(q, v, c, w)
        for _ in range(2):
            obs, *_ = env.step(env.expert_plan(16))
        torch.cuda.synchronize()
        outs.append((obs["image_overhead"].cpu().numpy(), obs["image_wrist"].cpu().numpy(),
                     env.segmentation.cpu().numpy(), env.env_error.cpu().numpy()))
        env.close()
    (o0, w0, s0, e0), (o1, w1, s1, e1) = outs
    assert (e0 == 0).all()
    assert e1[1] != 0 and e1[2] != 0 and e1[0] == 0 and e1[3] == 0, e1
    for k in (0, 3):
        np.testing.assert_array_equal(o1[k], o0[k])
        np.testing.assert_array_equal(w1[k], w0[k])
        np.testing.assert_array_equal(s1[k], s0[k])
    assert s1.max() <= 9  # valid segment ids everywhere, the diverged envs' images included
