"""Build the diagnostic probe variants build/libmmx_prof<P>.so (MMX_PROBE=P) on the CPU host;
tools/probe_sets.sh runs them on the GPU box.  Test / diagnostic infrastructure."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mujoco_manip_amd import _build  # noqa: E402

sets = [int(a) for a in sys.argv[1:]] or [1, 2, 3]
with ThreadPoolExecutor(max_workers=3) as ex:
    list(ex.map(lambda p: _build.build_variant(os.path.join(REPO, "build", f"libmmx_prof{p}.so"), [f"MMX_PROBE={p}"]),
                sets))
print("built", sets)
