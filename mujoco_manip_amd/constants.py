"""Task constants (mirror of mujoco_manip/constants.py:3-37)."""

OBJECTS = ["obj_red", "obj_green", "obj_blue"]
BINS = ["bin_red", "bin_green", "bin_blue"]

MATCH_TASKS = [("obj_red", "bin_red"), ("obj_green", "bin_green"), ("obj_blue", "bin_blue")]
CROSS_TASKS = [(o, b) for o in OBJECTS for b in BINS if o.split("_")[1] != b.split("_")[1]]
ALL_TASKS = [(o, b) for o in OBJECTS for b in BINS]
TASK_SETS = {"all": ALL_TASKS, "match": MATCH_TASKS, "cross": CROSS_TASKS}

IMAGE_SIZE = 224
CONTROL_FPS = 30
PHYSICS_DT = 0.002
ACTION_REPEAT = 16
MAX_EPISODE_STEPS = 500

KEYPOINT_BODIES = ["obj_red", "obj_green", "obj_blue", "bin_red", "bin_green", "bin_blue", "hand"]

# numeric observation layout of the device obs buffer (gym_env.py:325-339 order, images excluded)
OBS_SLICES = {
    "state": (0, 11, (11,)),
    "state.ee.pos_quat_g": (11, 19, (8,)),
    "state.ee.pos_rot6d_g": (19, 29, (10,)),
    "state.ee.pos_quat_g_rel": (29, 37, (8,)),
    "state.ee.pos_rot6d_g_rel": (37, 47, (10,)),
    "target_bin_onehot": (47, 50, (3,)),
    "target_obj_onehot": (50, 53, (3,)),
    "keypoints_overhead": (53, 67, (7, 2)),
    "keypoints_wrist": (67, 81, (7, 2)),
    "target_obj_keypoints_overhead": (81, 83, (2,)),
    "target_bin_keypoints_overhead": (83, 85, (2,)),
}


def task_index(task):
    """(obj_name, bin_name) -> (obj_idx, bin_idx)."""
    o, b = task
    return OBJECTS.index(o), BINS.index(b)
