"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host code only).

oracle/selftest.c drives every model, both dtypes and arithmetic modes, pCN and
RW sweeps with boxes, schedules, sums and the regularizer, init_phi and
len_burn_in on small ragged shapes; the binary is built with
-fsanitize=address,undefined (oracle/Makefile `asan`).  A sanitizer report
or a non-zero exit fails the test.
"""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

ORACLE = os.path.join(REPO, "oracle")


def test_oracle_clean_under_asan_ubsan():
    if shutil.which(os.environ.get("CC", "gcc")) is None:
        pytest.skip("no C compiler")
    b = subprocess.run(["make", "-C", ORACLE, "-s", "asan"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in (b.stderr + b.stdout) and "cannot find" in (b.stderr + b.stdout):
        pytest.skip("sanitizer runtime not available")
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(ORACLE, "_build", "orc_selftest_asan")], capture_output=True, text=True,
                       env=env, timeout=600)
    report = r.stderr[-4000:]
    assert r.returncode == 0, report
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, report
    assert "oracle selftest ok" in r.stdout
