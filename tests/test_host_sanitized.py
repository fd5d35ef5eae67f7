"""libipmc_host.so's source under AddressSanitizer + UBSan and ThreadSanitizer.

libipmc_host.so is on the product path (config 1's draws without a GPU, the
posterior mean's ordered sum inside bench.py's timed region), so its C++ runs
under the sanitizers SURVEY §5 asks for -- host code only.
ip_mcmc_amd/csrc/ipmc_host_selftest.cpp drives every entry point of
include/ipmc_host.h: threaded ipmc_host_pcn_draws on element counts no thread
count divides, the Cholesky prior, f32 and f64, ids and steps at the range
limits; ipmc_host_ordered_sum with row_stride > k, div != 1 and no rows; every
error return.  It checks each result (threaded == one thread == the
ipmc_rng.hpp element functions; the ordered sum == a plain row-order loop).
A sanitizer report or a non-zero exit fails the test.
"""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

CSRC = os.path.join(REPO, "ip_mcmc_amd", "csrc")
BUILD = os.path.join(REPO, "build", "host_san")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_library_clean_under_sanitizers(kind):
    if shutil.which("g++") is None:
        pytest.skip("no C++ compiler")
    b = subprocess.run(["make", "-C", CSRC, "-s", f"host-{kind}"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in (b.stderr + b.stdout) and "cannot find" in (b.stderr + b.stdout):
        pytest.skip("sanitizer runtime not available")
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(BUILD, f"host_selftest_{kind}")], capture_output=True, text=True, env=env,
                       timeout=600)
    report = r.stderr[-4000:]
    assert r.returncode == 0, report
    for marker in ("runtime error", "AddressSanitizer", "ThreadSanitizer", "LeakSanitizer"):
        assert marker not in r.stderr, report
    assert "host selftest ok" in r.stdout
