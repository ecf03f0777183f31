"""Build experiment variants of libmmx.so for A/B runs (tools/ab.sh): each argument is
`name:DEFINE[,DEFINE...]` (sources of the working tree) or `name@REV` (the csrc/ + include/ of a git
revision, exported to a temp dir).  Output: build/libmmx_<name>.so.  Experiment infrastructure."""
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mujoco_manip_amd import _build  # noqa: E402


def one(spec):
    """name:D1,D2 | name@REV[:D1,...]; a define PROF makes a phase-clock (profile) build."""
    out = os.path.join(REPO, "build", f"libmmx_{spec.split(':')[0].split('@')[0]}.so")
    defs = [d for d in (spec.split(":", 1)[1].split(",") if ":" in spec else []) if d]
    prof = "PROF" in defs
    defs = [d for d in defs if d != "PROF"]
    if "@" in spec:
        name, rev = spec.split(":")[0].split("@")
        tmp = tempfile.mkdtemp(prefix=f"mmx_{name}_")
        subprocess.check_call(f"git -C {REPO} archive {rev} mujoco_manip_amd/csrc include | tar -x -C {tmp}", shell=True)
        saved = _build.CSRC
        _build.CSRC = os.path.join(tmp, "mujoco_manip_amd", "csrc")
        try:
            return _build.build_variant(out, defs, profile=prof)
        finally:
            _build.CSRC = saved
    return _build.build_variant(out, defs, profile=prof)


if __name__ == "__main__":
    with ThreadPoolExecutor(max_workers=3) as ex:
        print(list(ex.map(one, sys.argv[1:])))
