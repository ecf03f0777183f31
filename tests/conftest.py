import json
import os
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

# Parity margins: tests that assert a tolerance also record what they measured,
# so the distance of every green test to its bound is kept.  Written at session end to
# $MMX_MARGINS_OUT (default gpurun_out/parity_margins.json) when any test recorded a value.
_MARGINS: dict = {}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU oracle episode")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(REPO, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture
def margin(request):
    """margin(key, measured, bound=None, **extra): record a measured parity value of this test."""
    name = request.node.name

    def rec(key, measured, bound=None, **extra):
        v = measured.tolist() if hasattr(measured, "tolist") else measured
        entry = {"measured": v}
        if bound is not None:
            entry["bound"] = bound
            if isinstance(v, (int, float)) and bound:
                entry["fraction_of_bound"] = round(float(v) / float(bound), 4)
        entry.update({k: (x.tolist() if hasattr(x, "tolist") else x) for k, x in extra.items()})
        _MARGINS.setdefault(name, {})[key] = entry

    return rec


def pytest_sessionfinish(session, exitstatus):
    if not _MARGINS:
        return
    out = os.environ.get("MMX_MARGINS_OUT", os.path.join(REPO, "gpurun_out", "parity_margins.json"))
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    doc = {"library": os.environ.get("MMX_LIB_PATH", "mujoco_manip_amd/libmmx.so"),
           "time": time.strftime("%Y-%m-%dT%H:%M:%S"), "exitstatus": int(exitstatus), "tests": _MARGINS}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
