"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r1 missing #7).

`make -C oracle sanitize` builds oracle/or_selftest.c with the oracle sources and
-fsanitize=address,undefined -fno-sanitize-recover=all (host code only; GPU sanitizers are not
available on the MI355X pool).  The driver runs expert episodes under all reward types with
autoreset stream continuation, all 5 action modes, the per-physics-step expert loop and mj_step
from interpenetrating cube piles; any sanitizer finding aborts it.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_asan_ubsan_selftest():
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ORACLE, "_san", "or_selftest"), "2"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "oracle selftest ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
