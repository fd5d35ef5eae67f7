"""Parity at BASELINE's full sizes (configs 2, 4 and 5), through the C-ABI / torch ops.

The oracle cannot re-run whole ensembles of this size in seconds, so each test
runs the full ensemble on the device once and checks (a) sampled chains
against the oracle bit for bit (forward map, Φ, sweep) and (b) the
size-independent sharding property: the ensemble split into the per-GPU
shards of an 8-GPU run (chain_offset = r·C/8) gives the same bits as one launch.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from test_gpu_parity import _np, _sweep_device, _sweep_oracle, _t  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return torch.device("cuda", 0)


def _device_phi(op, U0, y, ginv, dtype, dev):
    from ip_mcmc_amd import torch_ops

    return torch_ops.potential(op, _t(U0, dtype, dev), _t(y, dtype, dev), _t(ginv, dtype, dev)).cpu().numpy()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_cfg5_gpu_share_full_length(dev, orc, dtype):
    """Config 5 per-GPU share: Lorenz-96 d=256, 10 000 RK4 steps, 131 072 chains
    (2^20 / 8), as the last rank's shard (global chain ids 7·2^17 ...)."""
    from ip_mcmc_amd import Lorenz96Operator, torch_ops

    op = Lorenz96Operator(256, 8.0, dt=0.005, n_steps=10000)
    C_, off = 131072, 7 * 131072
    rng = np.random.default_rng(55)
    U0 = (0.05 * rng.normal(size=(C_, 256))).astype(_np(dtype)).astype(np.float64)
    y = orc.forward(op, U0[:1])[0] + 0.1 * rng.normal(size=256)
    ginv, sq = np.full(256, 10.0), np.ones(256)
    idx = np.array([0, 1, 4097, 65536, C_ - 1])
    g = torch_ops.forward(op, _t(U0, dtype, dev)).cpu().numpy()
    assert np.array_equal(g[idx], orc.forward(op, U0[idx], _np(dtype)))
    phi0 = _device_phi(op, U0, y, ginv, dtype, dev).astype(np.float64)
    assert np.array_equal(phi0[idx], orc.potential(op, U0[idx], y, ginv, _np(dtype)).astype(np.float64))
    d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.002, 41, 0, 1, dtype, dev, chain_offset=off)
    for i in idx:
        o = _sweep_oracle(orc, op, U0[i:i + 1], phi0[i:i + 1], y, ginv, sq, 0.002, 41, 0, 1, dtype,
                          chain_offset=off + int(i))
        assert np.array_equal(d["u"][i], o["u"][0]) and d["acc"][i] == o["acc"][0], (dtype, i)
        assert d["phi"][i] == o["phi"][0], (dtype, i)
    assert np.all(np.isfinite(d["phi"]))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_cfg4_full_ensemble_and_shards(dev, orc, dtype):
    """Config 4: viscous Burgers (nu = 1e-3) N=256, fixed dt 1e-3 x 1000, beta
    0.15, all 16 384 chains in one launch == the eight 2 048-chain shards of an
    8-GPU run; sampled chains == the oracle."""
    from ip_mcmc_amd import BurgersOperator

    op = BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=1000, nu=1e-3)
    C_, P = 16384, 8
    rng = np.random.default_rng(44)
    U0 = (0.25 * rng.normal(size=(C_, 3))).astype(_np(dtype)).astype(np.float64)
    # truth (δ1, δ2, σ0) = (0.025, -0.025, -0.02) of burgers_beta.py, as a perturbation of the prior mean
    y = orc.forward(op, [[0.025 - 1.5, -0.025 - 0.25, -0.02 + 0.5]])[0] + 0.05 * rng.normal(size=op.q)
    ginv, sq = np.full(op.q, 1 / 0.05), np.full(3, 0.25)
    phi0 = _device_phi(op, U0, y, ginv, dtype, dev).astype(np.float64)
    n = 3
    full = _sweep_device(op, U0, phi0, y, ginv, sq, 0.15, 23, 0, n, dtype, dev)
    assert full["acc"].sum() > 0
    S = C_ // P
    for r in range(P):
        sl = slice(r * S, (r + 1) * S)
        sh = _sweep_device(op, U0[sl], phi0[sl], y, ginv, sq, 0.15, 23, 0, n, dtype, dev, chain_offset=r * S)
        for key in ("u", "phi", "acc", "calls"):
            assert np.array_equal(sh[key], full[key][sl]), (r, key)
    idx = np.sort(rng.choice(C_, 12, replace=False))
    for i in idx:
        o = _sweep_oracle(orc, op, U0[i:i + 1], phi0[i:i + 1], y, ginv, sq, 0.15, 23, 0, n, dtype,
                          chain_offset=int(i))
        assert np.array_equal(full["u"][i], o["u"][0]) and full["acc"][i] == o["acc"][0], (dtype, i)
        assert full["phi"][i] == o["phi"][0], (dtype, i)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_headline_samples_overlapped_copy(dev, dtype, monkeypatch):
    """MCMCSampler.run at the headline size (65 536 chains, d=40, 2 000 RK4
    steps, 20 samples = 420 MB of f64 samples): the samples go to the host in
    blocks while later blocks sweep (rectangular D2H at the real pitch).  The
    result equals the run with one copy at the end, and its last sample is the
    chains' final state."""
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, Lorenz96Operator,
                             MCMCSampler, PhiloxRNG, pCNAccepter)
    from ip_mcmc_amd import sampler as S

    d, C_ = 40, 65536
    op = Lorenz96Operator(d, 8.0, dt=0.005, n_steps=2000)
    rng = np.random.default_rng(8)
    y = op(np.zeros(d)) + 0.1 * rng.normal(size=d)
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(d), 0.01 * np.eye(d)))
    prior = GaussianDistribution(np.zeros(d), np.eye(d))
    u0 = 0.05 * rng.normal(size=(C_, d))

    def run():
        s = MCMCSampler(ConstSteppCNProposer(0.2, prior), pCNAccepter(pot), PhiloxRNG(4), dtype=dtype)
        out = s.run(u0, n_samples=20, burn_in=1, sample_interval=1)
        return out, s.state.u

    assert C_ * 20 * d * 8 >= S.OVERLAP_COPY_MIN_BYTES  # the default path overlaps
    a, ua = run()
    monkeypatch.setattr(S, "OVERLAP_COPY_MIN_BYTES", 1 << 62)
    b, _ = run()
    assert a.shape == (C_, 20, d) and a.dtype == np.float64
    assert np.array_equal(a, b)
    assert np.array_equal(a[:, -1, :], np.asarray(ua, dtype=np.float64))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_cfg2_full_shape(dev, orc, dtype):
    """Config 2 as SURVEY §8(d) defines it (tools/config_bench.cfg2_problem):
    Lorenz-63, 500 RK4 steps of 0.01 from the spun-up state, prior
    N(0, diag(1, 1, 0.1)), y = the truth's long-run moment means, Γ = 0.5²·diag(var
    of the moments), beta 0.2, 4 096 chains.  One launch of 128 pCN steps with
    the automatic plan -- ipmc_plan_sweep reports the speculative sweep of
    width 16 -- and every chain's state, Φ, accept and call counts equal the
    oracle's sequential chain."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import ctypes as C

    import config_bench as CB
    from ip_mcmc_amd import _abi
    from ip_mcmc_amd._lib import call

    op, y, ginv, sq, beta = CB.cfg2_problem()
    C_, n = 4096, 128
    rng = np.random.default_rng(22)
    U0 = (sq * rng.normal(size=(C_, 3))).astype(_np(dtype)).astype(np.float64)  # prior draws
    phi0 = _device_phi(op, U0, y, ginv, dtype, dev).astype(np.float64)
    assert np.array_equal(phi0, orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64))
    m, _ = op.model(dtype, dev)
    sw = _abi.IpmcSweep()
    sw.dtype, sw.n_chains, sw.n_steps, sw.spec_width = (_abi.F64 if dtype == torch.float64 else _abi.F32), C_, n, 0
    plan = _abi.IpmcPlan()
    call("ipmc_plan_sweep", C.byref(m), C.byref(sw), C.byref(plan))
    assert plan.spec_width == 16
    d = _sweep_device(op, U0, phi0, y, ginv, sq, beta, 2, 0, n, dtype, dev, spec=0)
    o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, beta, 2, 0, n, dtype)
    for key in ("u", "phi", "acc", "calls"):
        assert np.array_equal(d[key], o[key]), key
    rate = o["acc"].sum() / (C_ * n)
    assert 0.01 < rate < 0.99, rate


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_strong_scaled_8gpu_shard_both_plans(dev, orc, dtype):
    """The 8-GPU shard of the headline (8 192 chains of d=40, the last rank's
    global ids) under both automatic plans: a short launch runs sequentially on
    8 interleaved lanes, a >= 256-step launch speculates on 4 lanes x 2 slots
    (ipmc_plan_sweep); every chain equals the oracle's sequential chain.  The
    forward map is shortened to 20 RK4 steps so the oracle checks all chains
    in seconds; the bench problem's burn-in from u = 0 (y from the forcing
    field F = 8 + 0.5 sin) makes acceptances frequent early on."""
    import ctypes as C

    from ip_mcmc_amd import Lorenz96Operator, _abi
    from ip_mcmc_amd._lib import call

    op = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=20)
    C_, off = 8192, 7 * 8192
    k = np.arange(40)
    y = orc.forward(op, (0.5 * np.sin(2 * np.pi * k / 40))[None, :])[0] + 0.1 * np.random.default_rng(3).normal(size=40)
    ginv, sq = np.full(40, 10.0), np.ones(40)
    U0 = np.zeros((C_, 40))
    phi0 = _device_phi(op, U0, y, ginv, dtype, dev).astype(np.float64)
    m, _ = op.model(dtype, dev)
    for n, want in ((16, (8, 1, 1)), (256, (4, 1, 2))):
        sw = _abi.IpmcSweep()
        sw.dtype, sw.n_chains, sw.n_steps, sw.spec_width = (_abi.F64 if dtype == torch.float64 else _abi.F32), C_, n, 0
        plan = _abi.IpmcPlan()
        call("ipmc_plan_sweep", C.byref(m), C.byref(sw), C.byref(plan))
        assert (plan.lanes_per_chain, plan.chains_per_lane, plan.spec_width) == want
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.2, 2, 0, n, dtype, dev, spec=0, chain_offset=off)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.2, 2, 0, n, dtype, chain_offset=off)
        for key in ("u", "phi", "acc"):
            assert np.array_equal(d[key], o[key]), (n, key)
        assert 0 < o["acc"].sum() < C_ * n


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_cfg2_long_launch_equals_short_launches(dev, orc, dtype):
    """Config 2 at the sampler's launch length (sampler.STEPS_PER_LAUNCH =
    16 384 for this ensemble): one 4 096-step launch -- each chain settles its
    steps in its own number of speculative rounds while the launch waits for
    the slowest -- equals 32 launches of 128 steps for all 4 096 chains (state,
    Φ, accept and call counts), and 8 chains equal the oracle's sequential
    chain over the 4 096 steps."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import config_bench as CB
    from ip_mcmc_amd.sampler import _steps_per_launch

    op, y, ginv, sq, beta = CB.cfg2_problem()
    m, _ = op.model(dtype, dev)
    assert _steps_per_launch(m, 4096) == 16384
    C_, n, short = 4096, 4096, 128
    rng = np.random.default_rng(23)
    U0 = (sq * rng.normal(size=(C_, 3))).astype(_np(dtype)).astype(np.float64)
    phi0 = _device_phi(op, U0, y, ginv, dtype, dev).astype(np.float64)
    a = _sweep_device(op, U0, phi0, y, ginv, sq, beta, 4, 0, n, dtype, dev, spec=0)
    b = dict(u=U0, phi=phi0, acc=np.zeros(C_, dtype=np.int64), calls=np.zeros(C_, dtype=np.int64))
    for st in range(0, n, short):
        r = _sweep_device(op, b["u"], b["phi"], y, ginv, sq, beta, 4, st, short, dtype, dev, spec=0)
        b = dict(u=r["u"].astype(np.float64), phi=r["phi"].astype(np.float64), acc=b["acc"] + r["acc"],
                 calls=b["calls"] + r["calls"])
    for key in ("u", "phi", "acc", "calls"):
        assert np.array_equal(np.asarray(a[key], dtype=np.float64), np.asarray(b[key], dtype=np.float64)), key
    idx = np.array([0, 1, 777, 2048, 3000, 4000, 4094, 4095])
    for i in idx:
        o = _sweep_oracle(orc, op, U0[i:i + 1], phi0[i:i + 1], y, ginv, sq, beta, 4, 0, n, dtype, chain_offset=int(i))
        for key in ("u", "phi", "acc", "calls"):
            assert np.array_equal(a[key][i], o[key][0]), (i, key)
    rate = a["acc"].sum() / (C_ * n)
    assert 0.5 < rate < 0.99, rate
