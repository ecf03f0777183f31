"""Collision candidate tests with test-only builds (_build.TEST_VARIANTS), each run in a child process
because the binding loads one library per process.  The test builds recompile the 128-row kernel only
(their 192-row kernel is the product's), so the children pin the 128-row layout (MMX_STEP_ROWS).

* Contact-overflow KAT: more sphere-test survivors than the candidate list holds must reach
  env_error as ERR_CON_OVERFLOW, whichever substep of the env step overflowed (the flag is sticky from
  the record load to the step's fold).  The product list holds 320 of the 780 pairs, which no C3 state
  comes near, so the path is forced with libmmx_col4.so (a 4-entry list); the product library shows no
  overflow over a C3 rollout.
* The persistent broadphase list against the full prune (libmmx_nolist.so: a 1-entry list, so every
  pass runs the full prune): bit-identical states and contacts through the release / retreat phases."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/oracle")
import oracle_py as O
from mujoco_manip_amd import _lib
from mujoco_manip_amd.vec_env import PickPlaceVecEnv
env = PickPlaceVecEnv(64, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                      image_size=0)
env.reset(seed=[O.episode_seed(42, i) for i in range(64)])
hit = np.zeros(64, bool)
for t in range(12):
    env.step(env.expert_plan(16))
    hit |= (env.env_error.cpu().numpy() & _lib.ERR_CON_OVERFLOW) != 0
print("OVERFLOW_ENVS", int(hit.sum()), "NAN_ENVS", int(((env.env_error.cpu().numpy() & _lib.ERR_NAN) != 0).sum()))
"""


def test_candidate_list_overflow_reaches_env_error():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    lib = os.path.join(REPO, "mujoco_manip_amd", "libmmx_col4.so")
    assert os.path.exists(lib), "test build missing: run __graft_entry__.build()"
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=dict(os.environ, MMX_LIB_PATH=lib, MMX_STEP_ROWS="128"),
                       capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("OVERFLOW_ENVS")][0].split()
    print(" ".join(line))
    assert int(line[1]) > 0  # envs whose sphere test kept more than 4 pairs (3 cubes on the table + the gripper)


def test_product_c3_rollout_has_no_contact_overflow():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import oracle_py as O
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    n = 1024
    env = PickPlaceVecEnv(n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=0)
    env.reset(seed=[O.episode_seed(42, i) for i in range(n)])
    seen = np.zeros(n, np.int32)
    for t in range(60):  # approach, grasps, transport: the contact piles
        env.step(env.expert_plan(16))
        seen |= env.env_error.cpu().numpy()
    assert not (seen & (_lib.ERR_CON_OVERFLOW | _lib.ERR_EFC_OVERFLOW)).any()


CHILD_DIGEST = r"""
import sys, hashlib
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/oracle")
import torch
import oracle_py as O
from mujoco_manip_amd import _lib
from mujoco_manip_amd.vec_env import PickPlaceVecEnv
n = 512
env = PickPlaceVecEnv(n, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                      autoreset=True, image_size=0)
env.reset(seed=[O.episode_seed(42, i) for i in range(n)])
out, phases = [], set()
for k in range(9):
    env.rollout_expert(10)
    torch.cuda.synchronize()
    phases |= set(env.fsm_state.cpu().numpy().tolist())
    h = hashlib.sha256()
    for t in (env.qpos, env.qvel, env.sim.view("contacts", _lib.MAXCON * _lib.CON_F)):
        h.update(t.cpu().numpy().tobytes())
    out.append(h.hexdigest()[:16])
print("DIGESTS", " ".join(out))
print("PHASES", " ".join(str(p) for p in sorted(phases)))
"""


def test_broadphase_list_equals_full_prune():
    """the persistent broadphase list (the pairs within 8 cm of contact when it was
    built, kept while the bodies' displacement bound stays under half of that) gives the same
    candidates, in the same order, as the full 780-pair prune.  512 C3 envs for 90 env steps (approach,
    grasp, transport, release, retreat): the product library (a 256-entry list) and the test build
    libmmx_nolist.so (a 1-entry list: the full prune in every collision pass) end every 10-step block
    with bit-identical states and last-substep contact lists."""
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    res = []
    for lib in ("libmmx.so", "libmmx_nolist.so"):
        path = os.path.join(REPO, "mujoco_manip_amd", lib)
        assert os.path.exists(path), "test build missing: run __graft_entry__.build()"
        r = subprocess.run([sys.executable, "-c", CHILD_DIGEST, REPO], env=dict(os.environ, MMX_LIB_PATH=path, MMX_STEP_ROWS="128"),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines() if ln.startswith(("DIGESTS", "PHASES"))}
        res.append(lines)
    print(res[0]["PHASES"], res[0]["DIGESTS"][:3])
    assert {"8", "9"} <= set(res[0]["PHASES"])  # release and retreat were reached
    assert res[0]["DIGESTS"] == res[1]["DIGESTS"]
