"""The C-ABI from a non-Python caller: examples/c_api/l96_pcn (host C++,
hipMalloc'ed buffers, ipmc_init_phi + ipmc_pcn_sweep) gives the CPU oracle's
bits on the same inputs."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

BIN = os.path.join(REPO, "examples", "c_api", "l96_pcn")


def _inputs(n):
    D = 40
    x0 = np.full(D, 8.0)
    x0[0] += 0.01
    y = 8.0 + (np.arange(D) % 5) / 8.0
    c = np.arange(n)[:, None]
    k = np.arange(D)[None, :]
    u0 = ((7 * c + 13 * k) % 17 - 8) / 64.0
    return x0, y, u0


def test_c_example_is_built_and_links_libipmc():
    """build() compiles the example; it finds libipmc.so through its rpath."""
    assert os.access(BIN, os.X_OK), "run __graft_entry__.build()"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    line = [l for l in out.splitlines() if "libipmc.so" in l]
    assert line and "not found" not in line[0] and "ip_mcmc_amd/lib/libipmc.so" in line[0], out


@pytest.mark.gpu
def test_c_caller_matches_the_oracle(orc, tmp_path):
    from ip_mcmc_amd import Lorenz96Operator

    n, steps = 2048, 4
    dump = tmp_path / "out.bin"
    r = subprocess.run([BIN, str(n), str(steps), "--dump", str(dump)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = dump.read_bytes()
    u = np.frombuffer(raw, dtype=np.float64, count=n * 40).reshape(n, 40)
    phi = np.frombuffer(raw, dtype=np.float64, count=n, offset=n * 40 * 8)
    acc = np.frombuffer(raw, dtype=np.int64, count=n, offset=n * 41 * 8)

    x0, y, u0 = _inputs(n)
    op = Lorenz96Operator(40, 8.0, x0=x0, dt=0.005, n_steps=200)
    idx = np.arange(0, n, 97)  # a sample of chains (the oracle is one CPU thread per chain)
    U = np.ascontiguousarray(u0[idx])
    P = orc.potential(op, U, y, np.full(40, 10.0))
    A = np.zeros(len(idx), dtype=np.int64)
    for j, i in enumerate(idx):
        Ui, Pi, Ai = U[j:j + 1].copy(), P[j:j + 1].copy(), A[j:j + 1].copy()
        orc.pcn_sweep(op, Ui, Pi, y, np.full(40, 10.0), np.ones(40), 0.2, 7, 0, steps, accepts=Ai,
                      chain_offset=int(i))
        assert np.array_equal(Ui[0], u[i]) and Pi[0] == phi[i] and Ai[0] == acc[i], i
    assert acc.sum() > 0  # some proposals were accepted
