"""C-ABI boundary checks that need no GPU: libmmx.so loads, exports every symbol declared in
include/mmx_api.h, and its host-side seeding matches numpy (scripts/generate_dataset.py:263-268)."""
import os
import re

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(headers=("mmx_api.h", "mmx_tuning.h")):
    src = "".join(open(os.path.join(REPO, "include", h)).read() for h in headers)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void|const char\*|uint32_t)\s+(mmx_\w+)\s*\(", src, re.M)))


def test_reference_boundary_header_has_no_tuning_entry_points():
    """include/mmx_api.h holds the reference boundary only; the launch-shape / layout / timing calls a
    reference-side binding never needs live in include/mmx_tuning.h."""
    api, tuning = declared_functions(("mmx_api.h",)), declared_functions(("mmx_tuning.h",))
    assert not set(api) & set(tuning)
    assert {"mmx_set_step_rows", "mmx_kernel_timing", "mmx_rollout_lanes"} <= set(tuning)
    assert {"mmx_create", "mmx_reset", "mmx_step", "mmx_rollout_expert"} <= set(api)


def test_library_exports_every_declared_symbol():
    from mujoco_manip_amd import _lib

    L = _lib.load()
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(L, n), f"libmmx.so does not export {n}"
    assert set(names) == set(_lib.EXPORTED)


def test_episode_seed_matches_numpy():
    from mujoco_manip_amd import _lib

    ss = np.random.SeedSequence(42)
    ref = [int(c.generate_state(1)[0]) for c in ss.spawn(64)]
    assert [_lib.episode_seed(42, i) for i in range(64)] == ref
    ss = np.random.SeedSequence(2**40 + 3)
    assert [_lib.episode_seed(2**40 + 3, i) for i in range(8)] == [int(c.generate_state(1)[0]) for c in ss.spawn(8)]


def test_create_fails_cleanly_without_gpu_or_with_bad_args():
    import ctypes as C

    from mujoco_manip_amd import _lib

    L = _lib.load()
    cfg = _lib.MMXConfig()
    L.mmx_config_default(C.byref(cfg))
    assert cfg.max_episode_steps == 500 and cfg.n_tasks == 9 and cfg.image_size == 224
    cfg.action_mode = 7  # invalid -> MMX_EINVAL, never aborts (ValueError in the reference)
    ptr = C.c_void_p()
    assert L.mmx_create(C.byref(cfg), C.byref(ptr)) == -1
    assert not ptr.value


def test_state_layout_constants_match_header():
    src = open(os.path.join(REPO, "mujoco_manip_amd", "csrc", "mmx_state.h")).read()
    from mujoco_manip_amd import _lib

    assert f"#define MMX_MAXCON {_lib.MAXCON}" in src
    assert f"KIN_N = {_lib.KIN_N}" in src
    # the episode_i enum: names up to EPI_N, in order (comments stripped)
    body = re.search(r"enum \{\s*(EPI_OBJ.*?)EPI_N\s*\}", src, re.S).group(1)
    body = re.sub(r"//[^\n]*", "", body)
    names = [t.strip() for t in body.replace("\n", " ").split(",") if t.strip()]
    assert len(names) == _lib.EPI_N == len(_lib.EPI_FIELDS)
    assert [n.split("=")[0].strip() for n in names][-4:] == ["EPI_NSUCCESS", "EPI_NPLACED", "EPI_NERROR", "EPI_PHASES"]

    def enum_count(first, last):
        """Value of `last` in the C enum that starts with `first` (explicit values honoured)."""
        body = re.search(rf"enum \{{\s*({first}.*?){last}\s*\}}", src, re.S).group(1)
        body = re.sub(r"//[^\n]*", "", body)
        v = -1
        for t in [t.strip() for t in body.replace("\n", " ").split(",") if t.strip()]:
            v = int(t.split("=")[1]) if "=" in t else v + 1
        return v + 1

    assert enum_count("CON_DIST", "CON_F") == _lib.CON_F  # contact record width (r02 binding said 12)
    assert enum_count("STAT_NEFC", "STAT_N") == _lib.STAT_N == len(_lib.STAT_FIELDS)
    hdr = open(os.path.join(REPO, "include", "mmx_api.h")).read()
    assert f"[N][{_lib.MAXCON}][{_lib.CON_F}]" in hdr and f"[N][{_lib.STAT_N}]" in hdr
    assert f"#define MMX_PNG_MAX_WIDTH {_lib.PNG_MAX_WIDTH}" in hdr and 3 * _lib.PNG_MAX_WIDTH + 1 <= 32768


def test_obs_layout_covers_reference_keys():
    from mujoco_manip_amd.constants import OBS_SLICES

    # gym_env.py:172-208 observation keys minus the two camera images
    keys = {"state", "state.ee.pos_quat_g", "state.ee.pos_rot6d_g", "state.ee.pos_quat_g_rel",
            "state.ee.pos_rot6d_g_rel", "target_bin_onehot", "target_obj_onehot", "keypoints_overhead",
            "keypoints_wrist", "target_obj_keypoints_overhead", "target_bin_keypoints_overhead"}
    assert set(OBS_SLICES) == keys
    end = 0
    for k, (a, b, shape) in OBS_SLICES.items():
        assert a == end and int(np.prod(shape)) == b - a
        end = b
    assert end == 85
