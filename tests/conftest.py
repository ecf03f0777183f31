import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU oracle episode")


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(REPO, "tests", "golden", "golden.json")) as f:
        return json.load(f)
