"""HIP kernels (libipmc.so, called through the C-ABI) vs the CPU oracle.

Bar: bit-exact.  Every draw, every forward map, every Φ, every accept decision
and every state must equal the oracle's on the same inputs, in fp32 and fp64
and in both arithmetic modes.  The oracle itself is pinned to
the reference in test_oracle_golden.py.
"""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return torch.device("cuda", 0)


def _t(a, dtype, dev):
    return torch.as_tensor(np.asarray(a, dtype=np.float64)).to(dtype).to(dev).contiguous()


def _np(dtype):
    return np.float32 if dtype == torch.float32 else np.float64


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


# ------------------------------------------------------------------- RNG
def test_normals_bit_exact(dev, orc):
    from ip_mcmc_amd import device as D

    for step in (0, 1, 12345, (1 << 33) + 7):
        z = D.normals(99, 5, 3000, step, 7, torch.float64, dev).cpu().numpy()
        assert np.array_equal(z, orc.normals(99, 5, 3000, step, 7))
        z32 = D.normals(99, 5, 300, step, 7, torch.float32, dev).cpu().numpy()
        assert np.array_equal(z32, orc.normals(99, 5, 300, step, 7).astype(np.float32))


def test_uniforms_bit_exact(dev, orc):
    from ip_mcmc_amd import device as D

    for seed in (0, 1, 2**63 + 5):
        r = D.uniforms(seed, 3, 50_000, 77, dev).cpu().numpy()
        assert np.array_equal(r, orc.uniforms(seed, 3, 50_000, 77))


# ---------------------------------------------------------- forward maps
def _ops():
    from ip_mcmc_amd import LinearOperator, Lorenz63Operator, Lorenz96Operator

    rng = np.random.default_rng(3)
    ops = []
    for arith in ("fma", "reference"):
        ops.append(("lin", LinearOperator(rng.normal(size=(3, 5)), rng.normal(size=5), arith=arith)))
        ops.append(("l63", Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=300, arith=arith)))
        for K in (8, 40):
            ops.append((f"l96_{K}", Lorenz96Operator(K, 8.0, dt=0.005, n_steps=200, arith=arith)))
    return ops


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_forward_and_potential_bit_exact(dev, orc, dtype):
    rng = np.random.default_rng(11)
    for name, op in _ops():
        U = 0.3 * rng.normal(size=(257, op.k))
        g = op.forward_device(_t(U, dtype, dev)).cpu().numpy()
        go = orc.forward(op, U, _np(dtype))
        assert np.array_equal(g, go), (name, op.arith, np.abs(g - go).max())
        y = go[0] + 0.1 * rng.normal(size=op.q)
        ginv = 1.0 / (0.1 + rng.random(op.q))
        from ip_mcmc_amd import EvolutionPotential, GaussianDistribution

        pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(op.q), np.diag(1 / ginv**2)))
        phi = pot.phi_device(_t(U, dtype, dev)).cpu().numpy()
        phio = orc.potential(op, U, y, pot.device_terms()[1], _np(dtype))
        assert np.array_equal(phi, phio), (name, op.arith)


# ----------------------------------------------------------------- sweep
def _sweep_device(op, U0, phi0, y, ginv, sq, beta, seed, step0, n_steps, dtype, dev, lanes=0, box=None,
                  sched=None, chain_offset=0, want_sums=False, cpl=0, proposal="pcn", reg_scale=None, spec=1,
                  chol=None):
    """One ipmc_pcn_sweep launch.  spec=1 (default) runs the sequential kernels;
    spec=0 lets the library choose a speculation width, >1 forces one."""
    from ip_mcmc_amd import _abi
    from ip_mcmc_amd._lib import call

    rs_t = None if reg_scale is None else _t(reg_scale, dtype, dev)

    U = _t(U0, dtype, dev)
    phi = _t(phi0, dtype, dev)
    acc = torch.zeros(U.shape[0], dtype=torch.int64, device=dev)
    calls = torch.zeros(U.shape[0], dtype=torch.int64, device=dev)
    yt, gt, st = _t(y, dtype, dev), _t(ginv, dtype, dev), _t(sq, dtype, dev)
    m, _ = op.model(dtype, dev)
    s = _abi.IpmcSweep()
    s.dtype = _abi.F64 if dtype == torch.float64 else _abi.F32
    s.lanes_per_chain = lanes
    s.chains_per_lane = cpl
    s.spec_width = spec
    s.n_chains, s.chain_offset = U.shape[0], chain_offset
    s.u, s.phi, s.accepts, s.calls = U.data_ptr(), phi.data_ptr(), acc.data_ptr(), calls.data_ptr()
    s.y, s.gamma_inv, s.prior_sqrt = yt.data_ptr(), gt.data_ptr(), st.data_ptr()
    keep = []
    if chol is not None:  # non-diagonal prior: the factor replaces prior_sqrt
        ct = _t(chol, dtype, dev)
        keep.append(ct)
        s.prior_chol, s.prior_sqrt = ct.data_ptr(), None
    if box is not None:
        bt = [None if b is None else _t(b, dtype, dev) for b in box]
        keep += bt
        s.box_lo, s.box_hi, s.box_off = [None if b is None else b.data_ptr() for b in bt]
    if sched is not None:
        sc = torch.as_tensor(sched).to(dev)
        keep.append(sc)
        s.beta_schedule = sc.data_ptr()
    s.beta, s.contraction = beta, (float(np.sqrt(1 - beta**2)) if proposal == "pcn" else 1.0)
    s.proposal = _abi.PROPOSAL_RW if proposal == "rw" else _abi.PROPOSAL_PCN
    s.reg_scale = None if rs_t is None else rs_t.data_ptr()
    s.seed, s.step0, s.n_steps = seed, step0, n_steps
    samp = torch.zeros_like(U)
    s.sample_out, s.sample_stride = samp.data_ptr(), U.shape[1]
    sums = None
    if want_sums:
        sums = (torch.zeros(U.shape, dtype=torch.float64, device=dev),
                torch.zeros(U.shape, dtype=torch.float64, device=dev))
        s.sum_u, s.sum_u2 = sums[0].data_ptr(), sums[1].data_ptr()
    call("ipmc_pcn_sweep", C.byref(m), C.byref(s), _stream(dev))
    torch.cuda.synchronize(dev)
    out = dict(u=U.cpu().numpy(), phi=phi.cpu().numpy(), acc=acc.cpu().numpy(), calls=calls.cpu().numpy(),
               samp=samp.cpu().numpy())
    if sums:
        out["sum_u"], out["sum_u2"] = sums[0].cpu().numpy(), sums[1].cpu().numpy()
    return out


def _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, beta, seed, step0, n_steps, dtype, box=None, sched=None,
                  chain_offset=0, want_sums=False, proposal="pcn", reg_scale=None, chol=None):
    npd = _np(dtype)
    U = np.ascontiguousarray(U0.astype(npd))
    phi = np.ascontiguousarray(phi0.astype(npd))
    acc = np.zeros(U.shape[0], dtype=np.int64)
    calls = np.zeros(U.shape[0], dtype=np.int64)
    sums = (np.zeros(U.shape), np.zeros(U.shape)) if want_sums else None
    orc.pcn_sweep(op, U, phi, y, ginv, sq, beta, seed, step0, n_steps, accepts=acc, calls=calls,
                  chain_offset=chain_offset, box=box or (None, None, None), beta_schedule=sched, sums=sums,
                  n_threads=8, proposal=proposal, reg_scale=reg_scale, prior_chol=chol)
    out = dict(u=U, phi=phi, acc=acc, calls=calls)
    if want_sums:
        out["sum_u"], out["sum_u2"] = sums
    return out


def _problem(op, n_chains, dtype, orc, seed=0):
    rng = np.random.default_rng(seed)
    U0 = 0.2 * rng.normal(size=(n_chains, op.k))
    g = orc.forward(op, 0.1 * rng.normal(size=(1, op.k)))[0]
    y = g + 0.05 * rng.normal(size=op.q)
    ginv = np.full(op.q, 1 / 0.05)
    sq = 0.5 + rng.random(op.k)
    phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
    return U0.astype(_np(dtype)).astype(np.float64), phi0, y, ginv, sq


def _assert_same(a, b, what):
    for key in ("u", "phi", "acc", "calls"):
        assert np.array_equal(a[key], b[key]), (what, key)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_sweep_small_models_bit_exact(dev, orc, dtype):
    for name, op in _ops():
        if not name.startswith(("lin", "l63")):
            continue
        U0, phi0, y, ginv, sq = _problem(op, 300, dtype, orc)
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 1234, 10, 25, dtype, dev)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 1234, 10, 25, dtype)
        _assert_same(d, o, (name, op.arith))
        assert np.array_equal(d["samp"], o["u"])
        assert 0 < o["acc"].sum() < 300 * 25


@pytest.mark.parametrize("dtype,cpl", [(torch.float64, 1), (torch.float32, 1), (torch.float32, 2)])
@pytest.mark.parametrize("K,lanes", [(8, 1), (8, 2), (8, 4), (40, 1), (40, 2), (40, 4), (40, 8), (32, 16), (64, 16),
                                     (6, 2), (10, 2), (60, 4), (80, 16)])
def test_sweep_l96_bit_exact_every_layout(dev, orc, dtype, cpl, K, lanes):
    """Every (lanes per chain, chains per lane) layout gives the oracle's bits;
    131 chains so the packed fp32 layout has a phantom partner in its last pair."""
    from ip_mcmc_amd import Lorenz96Operator

    from ip_mcmc_amd._lib import UnsupportedOnDevice

    if (dtype == torch.float64 or cpl == 2) and K // lanes > 20:
        # no 8-byte-storage kernel holds more than 20 components per lane: the
        # library refuses the layout by name (ipmc_last_error) instead of
        # running another one
        op = Lorenz96Operator(K, 8.0, dt=0.005, n_steps=60)
        U0, phi0, y, ginv, sq = _problem(op, 131, dtype, orc, seed=K)
        with pytest.raises(UnsupportedOnDevice, match=f"dim={K} lanes_per_chain={lanes}"):
            _sweep_device(op, U0, phi0, y, ginv, sq, 0.25, 77, 5, 6, dtype, dev, lanes=lanes, cpl=cpl)
        return
    for arith in ("fma", "reference"):
        op = Lorenz96Operator(K, 8.0, dt=0.005, n_steps=60, arith=arith)
        U0, phi0, y, ginv, sq = _problem(op, 131, dtype, orc, seed=K)
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.25, 77, 5, 6, dtype, dev, lanes=lanes, cpl=cpl,
                          want_sums=True)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.25, 77, 5, 6, dtype, want_sums=True)
        _assert_same(d, o, (K, lanes, cpl, arith))
        assert np.array_equal(d["samp"], o["u"])
        assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["sum_u2"], o["sum_u2"])


@pytest.mark.parametrize("dtype,cpl", [(torch.float64, 1), (torch.float32, 1), (torch.float32, 2)])
@pytest.mark.parametrize("K", [16, 40, 80])
def test_sweep_l96_interleaved_8_lanes_box_rw_schedule(dev, orc, dtype, cpl, K):
    """8 lanes per chain run two chains interleaved per 16-lane row
    (group_vlane): the box's group vote, the RW regularizer's and the misfit's
    LDS-staged in-order sums and the halos all follow the interleaved lanes.
    131 chains: the last row's odd lanes (and a packed pair's partner) are
    phantoms."""
    from ip_mcmc_amd import Lorenz96Operator

    if (dtype == torch.float64 or cpl == 2) and K // 8 > 20:
        pytest.skip("no 8-byte-storage instantiation with more than 20 components per lane")
    n = 9
    sched = np.stack([np.linspace(0.05, 0.4, n), np.sqrt(1 - np.linspace(0.05, 0.4, n) ** 2)], axis=1)
    op = Lorenz96Operator(K, 8.0, dt=0.005, n_steps=40)
    U0, phi0, y, ginv, sq = _problem(op, 131, dtype, orc, seed=K + 1)
    box = (np.full(K, -0.6), np.full(K, 0.7), np.linspace(-0.05, 0.05, K))
    rs = np.linspace(0.5, 2.0, K)
    phr = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs).astype(np.float64)
    for kw, ph in ((dict(box=box, sched=sched), phi0), (dict(proposal="rw", reg_scale=rs, box=box), phr)):
        o = _sweep_oracle(orc, op, U0, ph, y, ginv, sq, 0.2, 13, 3, n, dtype, **kw)
        assert 0 < o["acc"].sum() < 131 * n
        d = _sweep_device(op, U0, ph, y, ginv, sq, 0.2, 13, 3, n, dtype, dev, lanes=8, cpl=cpl, spec=1, **kw)
        _assert_same(d, o, (K, str(dtype), cpl, sorted(kw)))


@pytest.mark.parametrize("dtype,cpl", [(torch.float64, 1), (torch.float32, 2)])
@pytest.mark.parametrize("lanes", [4, 8])
def test_sweep_l96_rk_steps_not_a_multiple_of_the_unroll(dev, orc, dtype, cpl, lanes):
    """Up to 10 components per lane the RK4 loop runs 4 steps per iteration
    and the remaining 1-3 after it (l96_forward, round 6): forward maps of 1,
    2, 3, 5, 7 and 41 RK4 steps (d=40 on 4 and 8 lanes: 10 and 5 components),
    both arithmetics, sweeps with sums -- the oracle's bits."""
    from ip_mcmc_amd import Lorenz96Operator

    for n_rk in (1, 2, 3, 5, 7, 41):
        for arith in ("fma", "reference"):
            op = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=n_rk, arith=arith)
            U0, phi0, y, ginv, sq = _problem(op, 131, dtype, orc, seed=n_rk)
            d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.25, 31, 2, 5, dtype, dev, lanes=lanes, cpl=cpl,
                              want_sums=True)
            o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.25, 31, 2, 5, dtype, want_sums=True)
            _assert_same(d, o, (n_rk, arith, lanes, str(dtype)))
            assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["sum_u2"], o["sum_u2"])
            # G and Φ alone (the eval kernels, auto layout for 16 384 chains: 4 lanes, 10 components)
            U = 0.3 * np.random.default_rng(n_rk).normal(size=(16384, 40))
            g = op.forward_device(_t(U, dtype, dev)).cpu().numpy()
            assert np.array_equal(g, orc.forward(op, U, _np(dtype))), (n_rk, arith)


def test_sweep_l96_d256_subset_bit_exact(dev, orc):
    """Config 5 shape at reduced length (d=256, 500 RK4 steps, 4096 chains), auto layouts."""
    from ip_mcmc_amd import Lorenz96Operator

    op = Lorenz96Operator(256, 8.0, dt=0.005, n_steps=500)
    idx = [0, 1, 2, 777, 2048, 4095]
    for dtype in (torch.float32, torch.float64):
        U0, phi0, y, ginv, sq = _problem(op, 4096, dtype, orc, seed=2)
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.05, 8, 0, 2, dtype, dev)
        for i in idx:
            o = _sweep_oracle(orc, op, U0[i:i + 1], phi0[i:i + 1], y, ginv, sq, 0.05, 8, 0, 2, dtype,
                              chain_offset=i)
            assert np.array_equal(d["u"][i], o["u"][0]) and d["acc"][i] == o["acc"][0], (dtype, i)


def test_sweep_box_schedule_sums_offset(dev, orc):
    """ConstrainAccepter box, VarStep beta schedule, running sums, chain offset."""
    from ip_mcmc_amd import Lorenz96Operator

    dtype = torch.float64
    op = Lorenz96Operator(8, 8.0, dt=0.01, n_steps=40)
    U0, phi0, y, ginv, sq = _problem(op, 200, dtype, orc, seed=5)
    box = (np.full(8, -0.6), np.full(8, 0.6), np.zeros(8))
    n = 12
    sched = np.stack([np.linspace(0.1, 0.5, n), np.sqrt(1 - np.linspace(0.1, 0.5, n) ** 2)], axis=1)
    d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 9, 100, n, dtype, dev, lanes=2, box=box, sched=sched,
                      chain_offset=1000, want_sums=True)
    o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 9, 100, n, dtype, box=box, sched=sched,
                      chain_offset=1000, want_sums=True)
    _assert_same(d, o, "box")
    assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["sum_u2"], o["sum_u2"])
    assert (o["calls"] < n).any(), "box never rejected: test is vacuous"


def test_sweep_split_launches_and_shards_identical(dev, orc):
    """One launch of n steps == two launches; chains [0,C) == shards [0,a) + [a,C)."""
    from ip_mcmc_amd import Lorenz96Operator

    dtype = torch.float32
    op = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=50)
    U0, phi0, y, ginv, sq = _problem(op, 256, dtype, orc, seed=8)
    full = _sweep_device(op, U0, phi0, y, ginv, sq, 0.2, 3, 0, 8, dtype, dev)
    a = _sweep_device(op, U0, phi0, y, ginv, sq, 0.2, 3, 0, 5, dtype, dev)
    b = _sweep_device(op, a["u"], a["phi"], y, ginv, sq, 0.2, 3, 5, 3, dtype, dev)
    assert np.array_equal(full["u"], b["u"]) and np.array_equal(full["acc"], a["acc"] + b["acc"])
    s1 = _sweep_device(op, U0[:100], phi0[:100], y, ginv, sq, 0.2, 3, 0, 8, dtype, dev, chain_offset=0)
    s2 = _sweep_device(op, U0[100:], phi0[100:], y, ginv, sq, 0.2, 3, 0, 8, dtype, dev, chain_offset=100)
    assert np.array_equal(full["u"], np.concatenate([s1["u"], s2["u"]]))


def test_headline_shape_subset_bit_exact(dev, orc):
    """Config 3 shape (d=40, 2000 RK4 steps, 65 536 chains, fp32 and fp64): one
    pCN step of the whole ensemble on the device; 48 chains re-run on the oracle."""
    from ip_mcmc_amd import Lorenz96Operator

    op = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=2000)
    C_ = 65536
    rng = np.random.default_rng(21)
    idx = np.sort(rng.choice(C_, 48, replace=False))
    from ip_mcmc_amd import _abi
    from ip_mcmc_amd._lib import call

    for dtype in (torch.float32, torch.float64):
        # Φ(u0) of the whole ensemble on the device (the oracle would need minutes
        # for 65 536 chains x 2000 RK4 steps); the sampled chains' Φ is checked below
        rng0 = np.random.default_rng(21)
        U0 = (0.2 * rng0.normal(size=(C_, 40))).astype(_np(dtype)).astype(np.float64)
        y = orc.forward(op, 0.1 * rng0.normal(size=(1, 40)))[0] + 0.05 * rng0.normal(size=40)
        ginv = np.full(40, 1 / 0.05)
        m, _ = op.model(dtype, dev)
        Ut, yt, gt = _t(U0, dtype, dev), _t(y, dtype, dev), _t(ginv, dtype, dev)
        pt = torch.empty(C_, dtype=dtype, device=dev)
        call("ipmc_potential", C.byref(m), _abi.F64 if dtype == torch.float64 else _abi.F32, C_, Ut.data_ptr(),
             yt.data_ptr(), gt.data_ptr(), pt.data_ptr(), _stream(dev))
        phi0 = pt.cpu().numpy().astype(np.float64)
        po = orc.potential(op, U0[idx], y, ginv, _np(dtype)).astype(np.float64)
        assert np.array_equal(phi0[idx], po), dtype
        d = _sweep_device(op, U0, phi0, y, ginv, np.ones(40), 0.2, 5, 0, 1, dtype, dev)
        for i in idx:
            o = _sweep_oracle(orc, op, U0[i:i + 1], phi0[i:i + 1], y, ginv, np.ones(40), 0.2, 5, 0, 1, dtype,
                              chain_offset=int(i))
            assert np.array_equal(d["u"][i], o["u"][0]) and d["acc"][i] == o["acc"][0], (dtype, i)
        assert np.all(np.isfinite(d["phi"]))


# ------------------------------------------------------------- sampler API
def test_sampler_linear_gaussian_posterior(dev):
    """Config 1 problem (stuart_examples.py-style linear G) through MCMCSampler:
    the posterior mean over 4096 chains matches the analytic Gaussian posterior
    (results.org:59-62) within 4 Monte-Carlo standard errors."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             LinearOperator, MCMCSampler, pCNAccepter)

    g = np.array([3.0, 1.0, 4.0, 1.0])
    gamma, y = 0.5, np.array([np.dot(g, [2.0, 7.0, 1.0, 8.0]) + 0.3])
    prior = GaussianDistribution(np.zeros(4), np.eye(4))
    pot = EvolutionPotential(LinearOperator(g), y, GaussianDistribution(0, gamma**2))
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(ConstSteppCNProposer(0.5, prior), acc, 7)
    C_ = 4096
    samples = s.run(np.zeros((C_, 4)), n_samples=50, burn_in=200, sample_interval=10)
    assert samples.shape == (C_, 50, 4)
    S0g = g
    denom = gamma**2 + g @ g
    m = S0g * y[0] / denom
    cov = np.eye(4) - np.outer(S0g, S0g) / denom
    est = samples[:, -1, :].mean(axis=0)
    se = np.sqrt(np.diag(cov) / C_)
    assert np.all(np.abs(est - m) < 4 * se + 1e-3), (est, m)
    r = acc.ratio()
    assert r.shape == (C_,) and 0.02 < r.mean() < 0.95
    assert int(acc.calls[0]) == max(0, 200 - 10) + 50 * 10


def test_sampler_single_chain_matches_reference_fixture(dev, golden):
    """The drop-in path: one chain, reference API, reference fixture (linear,
    injected draws) reproduced by MCMCSampler on the GPU."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             LinearOperator, MCMCSampler, PhiloxRNG, pCNAccepter)

    gamma, beta, seed, n_samples, burn_in, interval = golden["lin_meta"]
    pot = EvolutionPotential(LinearOperator(golden["lin_g"], arith="reference"), golden["lin_y"],
                             GaussianDistribution(0, gamma**2))
    for chain in range(4):
        acc = CountedAccepter(pCNAccepter(pot))
        s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc,
                        PhiloxRNG(int(seed)), chain_offset=chain)
        out = s.run(np.zeros(4), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
        assert out.shape == (int(n_samples), 4)
        assert np.array_equal(out, golden["lin_samples"][chain])
        assert acc.accepts == int(golden["lin_counts"][chain, 1])
        assert acc.calls == int(golden["lin_counts"][chain, 0])


def test_sampler_constrained_chain_matches_reference_fixture(dev, golden):
    """ConstrainAccepter(CountedAccepter(pCNAccepter), BoxConstraint) through the
    drop-in API reproduces the reference's constrained chains (accepter.py:39-55):
    samples, accepts and the inner accepter's calls."""
    from ip_mcmc_amd import (BoxConstraint, ConstrainAccepter, ConstSteppCNProposer, CountedAccepter,
                             EvolutionPotential, GaussianDistribution, LinearOperator, MCMCSampler, PhiloxRNG,
                             pCNAccepter)

    gamma, beta, seed, n_samples, burn_in, interval = golden["con_meta"]
    pot = EvolutionPotential(LinearOperator(golden["con_g"], arith="reference"), golden["con_y"],
                             GaussianDistribution(0, gamma**2))
    for chain in range(3):
        inner = CountedAccepter(pCNAccepter(pot))
        acc = ConstrainAccepter(inner, BoxConstraint(lower=golden["con_lo"], upper=golden["con_hi"]))
        s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc,
                        PhiloxRNG(int(seed)), chain_offset=chain)
        out = s.run(np.zeros(4), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
        assert np.array_equal(out, golden["con_samples"][chain])
        assert inner.calls == int(golden["con_counts"][chain, 0])
        assert inner.accepts == int(golden["con_counts"][chain, 1])


def test_sampler_l96_chain_matches_reference_fixture(dev, golden):
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, Lorenz96Operator,
                             MCMCSampler, PhiloxRNG, pCNAccepter)

    K, n, dt, gamma, beta, seed, n_samples, burn_in, interval = golden["l96c_meta"]
    K = int(K)
    op = Lorenz96Operator(K, 8.0, x0=golden["l96c_x0"], dt=dt, n_steps=int(n), arith="reference")
    pot = EvolutionPotential(op, golden["l96c_y"], GaussianDistribution(np.zeros(K), gamma**2 * np.eye(K)))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(K), np.eye(K))), pCNAccepter(pot),
                    PhiloxRNG(int(seed)))
    out = s.run(np.zeros((3, K)), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
    assert np.array_equal(out, golden["l96c_samples"])


def test_sampler_runs_host_callables_on_the_host_path(dev):
    """A Python G is no longer refused: it takes the host-side step
    (hostloop.py) with the GPU's draws."""
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, MCMCSampler,
                             pCNAccepter)

    pot = EvolutionPotential(lambda u: u, np.zeros(2), GaussianDistribution(np.zeros(2), np.eye(2)))
    s = MCMCSampler(ConstSteppCNProposer(0.5, GaussianDistribution(np.zeros(2), np.eye(2))), pCNAccepter(pot), 1)
    out = s.run(np.zeros(2), 2, 0, 1)
    assert out.shape == (2, 2) and s.last_path == "host"


# ---------------------------------------------------------------- Burgers
def _burgers_ops():
    from ip_mcmc_amd import BurgersOperator

    out = []
    for arith in ("fma", "reference"):
        for N in (32, 128, 200, 256):
            out.append(BurgersOperator(N=N, dt_mode="cfl", arith=arith))
        out.append(BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=1000, arith=arith))
        out.append(BurgersOperator(N=128, dt_mode="fixed", dt=2e-3, n_steps=400, nu=1e-3, arith=arith))
        out.append(BurgersOperator(N=64, dt_mode="cfl", cfl=0.4, nu=5e-4, arith=arith))
    return out


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_burgers_forward_potential_bit_exact(dev, orc, dtype):
    rng = np.random.default_rng(4)
    for op in _burgers_ops():
        U = 0.25 * rng.normal(size=(96, 3))
        U[0] = 0.0
        U[1] = [3.0, 0.0, 0.0]  # fast left state: violates the fixed-dt CFL guard
        # the jump inside the first / last cell: an IC ghost unlike its neighbour cell
        U[2] = [0.0, 0.0, -1.0 - op.theta0[2]]
        U[3] = [0.0, 0.0, 1.0 - op.theta0[2]]
        g = op.forward_device(_t(U, dtype, dev)).cpu().numpy()
        go = orc.forward(op, U, _np(dtype))
        assert np.array_equal(g, go, equal_nan=True), (op.N, op.dt_mode, op.arith, np.nanmax(np.abs(g - go)))
        y = np.nan_to_num(go[0]) + 0.05 * rng.normal(size=op.q)
        ginv = np.full(op.q, 20.0)
        from ip_mcmc_amd import EvolutionPotential, GaussianDistribution

        pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(op.q), np.diag(1 / ginv**2)))
        phi = pot.phi_device(_t(U, dtype, dev)).cpu().numpy()
        phio = orc.potential(op, U, y, ginv, _np(dtype))
        assert np.array_equal(phi, phio), (op.N, op.dt_mode, op.arith)
    fixed = _burgers_ops()[4]
    gi = orc.forward(fixed, [[3.0, 0.0, 0.0]])
    assert np.all(np.isnan(gi)), "CFL guard never tripped: test is vacuous"


@pytest.mark.parametrize("N", [32, 128, 256])
def test_burgers_device_matches_reference_fixture(dev, golden, N):
    """RusanovFVM.integrate + Measurer of the reference, on the GPU, fp64 REFERENCE arith: bit-exact."""
    from ip_mcmc_amd import BurgersOperator

    op = BurgersOperator(prior_mean=(0.0, 0.0, 0.0), N=N, T=1.0, dt_mode="cfl", arith="reference")
    g = op.forward_device(_t(golden[f"bur{N}_theta"], torch.float64, dev)).cpu().numpy()
    assert np.array_equal(g, golden[f"bur{N}_G"])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_burgers_sweep_bit_exact(dev, orc, dtype):
    """Config 4 shape (N=256, fixed dt 1e-3 x 1000, beta 0.15) and the CFL scheme with the
    is_valid_IC box constraint (burgers_wasserstein_chain.py:47-55)."""
    from ip_mcmc_amd import BurgersOperator

    for op in (BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=1000),
               BurgersOperator(N=128, dt_mode="cfl", arith="reference")):
        rng = np.random.default_rng(12)
        U0 = 0.25 * rng.normal(size=(64, 3))
        truth = orc.forward(op, [[0.025 - 1.5, -0.025 - 0.25, -0.02 + 0.5]])[0]
        y = truth + 0.05 * rng.normal(size=op.q)
        ginv = np.full(op.q, 1 / 0.05)
        sq = np.full(3, 0.25)
        phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
        U0 = U0.astype(_np(dtype)).astype(np.float64)
        box = (np.array([-np.inf, -np.inf, -1.0]), np.array([np.inf, np.inf, 1.0]), op.theta0)
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.15, 31, 0, 6, dtype, dev, box=box)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.15, 31, 0, 6, dtype, box=box)
        _assert_same(d, o, (op.N, op.dt_mode))
        assert o["acc"].sum() > 0


# ------------------------------------------------- random walk (§8(f) #1)
def test_rw_sweeps_bit_exact(dev, orc):
    """RW proposal + StandardRWAccepter regularizer, const and scheduled step
    sizes, on every kernel family (small, Lorenz-96 incl. packed fp32, Burgers)."""
    from ip_mcmc_amd import BurgersOperator, LinearOperator, Lorenz63Operator, Lorenz96Operator

    rng = np.random.default_rng(17)
    ops = [LinearOperator(rng.normal(size=(2, 4))), Lorenz63Operator(x0=(1.0, 2.0, 20.0), n_steps=200),
           Lorenz96Operator(40, 8.0, dt=0.005, n_steps=50), BurgersOperator(N=64, dt_mode="cfl")]
    for op in ops:
        for dtype, cpl in ((torch.float64, 0), (torch.float32, 1), (torch.float32, 2)):
            if cpl and not isinstance(op, Lorenz96Operator):
                continue
            U0, phi0, y, ginv, sq = _problem(op, 70, dtype, orc, seed=3)
            rs = 0.5 + rng.random(op.k)
            phi0 = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs).astype(np.float64)
            n = 5
            sched = np.stack([np.linspace(0.05, 0.2, n), np.ones(n)], axis=1)
            for sc in (None, sched):
                d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.1, 4, 3, n, dtype, dev, sched=sc, cpl=cpl,
                                  proposal="rw", reg_scale=rs)
                o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.1, 4, 3, n, dtype, sched=sc, proposal="rw",
                                  reg_scale=rs)
                _assert_same(d, o, (type(op).__name__, dtype, cpl, sc is None))


def test_init_phi_with_regularizer_bit_exact(dev, orc):
    from ip_mcmc_amd import Lorenz96Operator, _abi
    from ip_mcmc_amd._lib import call

    op = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=40)
    for dtype in (torch.float64, torch.float32):
        U0, phi0, y, ginv, sq = _problem(op, 90, dtype, orc, seed=6)
        rs = np.linspace(0.5, 2.0, 40)
        want = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs)
        U, yt, gt, rt = _t(U0, dtype, dev), _t(y, dtype, dev), _t(ginv, dtype, dev), _t(rs, dtype, dev)
        phi = torch.empty(90, dtype=dtype, device=dev)
        m, _ = op.model(dtype, dev)
        s = _abi.IpmcSweep()
        s.dtype = _abi.F64 if dtype == torch.float64 else _abi.F32
        s.n_chains, s.u, s.phi = 90, U.data_ptr(), phi.data_ptr()
        s.y, s.gamma_inv, s.reg_scale = yt.data_ptr(), gt.data_ptr(), rt.data_ptr()
        call("ipmc_init_phi", C.byref(m), C.byref(s), _stream(dev))
        torch.cuda.synchronize(dev)
        assert np.array_equal(phi.cpu().numpy(), want)


@pytest.mark.parametrize("kind", ["const", "var"])
def test_sampler_rw_matches_reference_fixture(dev, golden, kind):
    """Reference RW sampler (ConstStep/VarStepStandardRWProposer + CountedAccepter(StandardRWAccepter))
    with injected draws, reproduced through MCMCSampler on the GPU."""
    from ip_mcmc_amd import (ConstStepStandardRWProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             LinearOperator, MCMCSampler, PhiloxRNG, PWLinear, StandardRWAccepter,
                             VarStepStandardRWProposer)

    meta = golden["rw_meta"]
    gamma, seed, n_samples, burn_in, interval = meta[0], int(meta[1]), int(meta[2]), int(meta[3]), int(meta[4])
    prior = GaussianDistribution(np.zeros(4), np.diag(golden["rw_prior_var"]))
    pot = EvolutionPotential(LinearOperator(golden["rw_g"], arith="reference"), golden["rw_y"],
                             GaussianDistribution(0, gamma**2))
    for chain in range(3):
        prop = (ConstStepStandardRWProposer(meta[5], prior) if kind == "const"
                else VarStepStandardRWProposer(PWLinear(meta[6], meta[7], int(meta[8])), prior))
        acc = CountedAccepter(StandardRWAccepter(pot, prior))
        s = MCMCSampler(prop, acc, PhiloxRNG(seed), chain_offset=chain)
        out = s.run(np.zeros(4), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
        assert np.array_equal(out, golden[f"rw_{kind}_samples"][chain])
        assert acc.accepts == int(golden[f"rw_{kind}_counts"][chain, 1])


@pytest.mark.parametrize("kind", ["pcn", "rw"])
def test_sampler_burgers_chain_matches_reference_fixture(dev, golden, kind):
    """The reference's Burgers study (burgers_beta.py:25-128, N=32, CFL Rusanov =
    RusanovFVM.integrate) through its own sampler with injected draws, reproduced
    by MCMCSampler on the GPU: the stack of 3 chains in one launch per block and
    each chain alone, pCN and the study's RW composition
    ConstrainAccepter(CountedAccepter(StandardRWAccepter), is_valid_IC) with
    VarStepStandardRWProposer(PWLinear)."""
    from ip_mcmc_amd import (BoxConstraint, BurgersOperator, ConstrainAccepter, ConstSteppCNProposer,
                             CountedAccepter, EvolutionPotential, GaussianDistribution, MCMCSampler, PhiloxRNG,
                             PWLinear, StandardRWAccepter, VarStepStandardRWProposer, pCNAccepter)

    meta = golden["bch_meta"]
    N, gamma, sigma_p, beta, seed = int(meta[0]), meta[1], meta[2], meta[3], int(meta[4])
    n_samples, burn_in, interval = int(meta[5]), int(meta[6]), int(meta[7])
    pm = golden["bch_prior_mean"]
    op = BurgersOperator(prior_mean=pm, N=N, T=1.0, dt_mode="cfl", arith="reference")
    pot = EvolutionPotential(op, golden["bch_y"], GaussianDistribution(np.zeros(5), gamma**2 * np.eye(5)))
    prior = GaussianDistribution(np.zeros(3), sigma_p**2 * np.eye(3))
    want = golden[f"bch_{kind}_samples"]
    counts = golden[f"bch_{kind}_counts"]

    def sampler(chain_offset):
        if kind == "pcn":
            inner = CountedAccepter(pCNAccepter(pot))
            return MCMCSampler(ConstSteppCNProposer(beta, prior), inner, PhiloxRNG(seed),
                               chain_offset=chain_offset), inner
        inner = CountedAccepter(StandardRWAccepter(pot, prior))
        box = BoxConstraint(lower=[-np.inf, -np.inf, -1.0], upper=[np.inf, np.inf, 1.0], offset=pm)
        prop = VarStepStandardRWProposer(PWLinear(meta[8], meta[9], int(meta[10])), prior)
        return MCMCSampler(prop, ConstrainAccepter(inner, box), PhiloxRNG(seed + 1), chain_offset=chain_offset), inner

    s, inner = sampler(0)
    out = s.run(np.zeros((3, 3)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    assert np.array_equal(out, want)
    assert np.array_equal(np.asarray(inner.accepts), counts[:, 1])
    assert np.array_equal(np.asarray(inner.calls), counts[:, 0])
    for chain in range(3):
        s, inner = sampler(chain)
        out = s.run(np.zeros(3), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
        assert np.array_equal(out, want[chain])
        assert inner.accepts == int(counts[chain, 1]) and inner.calls == int(counts[chain, 0])


# ------------------------------------------- two-scale Lorenz-96 (§8(f) #4)
def _ts_ops():
    from ip_mcmc_amd import TwoScaleLorenz96Operator as TS

    rng = np.random.default_rng(21)
    out = []
    for arith in ("fma", "reference"):
        for K, J, mom in ((6, 4, "reference"), (6, 4, "mean"), (4, 8, "mean"), (36, 10, "mean"), (3, 1, "reference"),
                          (5, 16, "reference"), (40, 2, "mean"), (64, 1, "mean")):
            x0 = rng.normal(0, 1, size=K * (1 + J))
            out.append(TS(K=K, J=J, x0=x0, dt=0.004, n_steps=40, moments=mom, arith=arith))
    return out


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_l96ts_forward_potential_bit_exact(dev, orc, dtype):
    from ip_mcmc_amd import EvolutionPotential, GaussianDistribution

    rng = np.random.default_rng(8)
    for op in _ts_ops():
        U = 0.3 * rng.normal(size=(67, 3))
        g = op.forward_device(_t(U, dtype, dev)).cpu().numpy()
        go = orc.forward(op, U, _np(dtype))
        assert np.array_equal(g, go), (op.K, op.J, op.moments, op.arith, np.abs(g - go).max())
        y = go[0] + 0.1 * rng.normal(size=op.q)
        ginv = 1.0 / (0.1 + rng.random(op.q))
        pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(op.q), np.diag(1 / ginv**2)))
        phi = pot.phi_device(_t(U, dtype, dev)).cpu().numpy()
        assert np.array_equal(phi, orc.potential(op, U, y, pot.device_terms()[1], _np(dtype))), (op.K, op.J)


def test_l96ts_device_matches_reference_fixture(dev, golden):
    from ip_mcmc_amd import TwoScaleLorenz96Operator as TS

    for K, J in ((6, 4), (4, 8), (3, 1)):
        n, dt, c = golden[f"ts_G{K}_{J}_meta"]
        op = TS(K=K, J=J, c=c, x0=golden[f"ts_G{K}_{J}_x0"], dt=dt, n_steps=int(n), arith="reference")
        g = op.forward_device(_t(golden[f"ts_G{K}_{J}_u"], torch.float64, dev)).cpu().numpy()
        assert np.array_equal(g, golden[f"ts_G{K}_{J}_G"]), (K, J)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_l96ts_sweeps_bit_exact(dev, orc, dtype):
    """pCN and RW (+ regularizer, schedule, box) sweeps of the two-scale model."""
    ops = _ts_ops()
    for op in (ops[0], ops[3], ops[12], ops[15]):
        U0, phi0, y, ginv, sq = _problem(op, 77, dtype, orc, seed=op.K)
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 9, 2, 5, dtype, dev, want_sums=True)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 9, 2, 5, dtype, want_sums=True)
        _assert_same(d, o, (op.K, op.J, op.arith))
        assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["samp"], o["u"])
        box = (np.array([-np.inf, 7.8, -np.inf]), None, op.theta0)
        d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 9, 2, 5, dtype, dev, box=box)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 9, 2, 5, dtype, box=box)
        _assert_same(d, o, (op.K, op.J, "box"))
        assert o["calls"].sum() < 77 * 5, "box never rejected: vacuous"
        rs = np.array([0.5, 1.0, 2.0])
        phr = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs).astype(np.float64)
        sched = np.stack([np.linspace(0.05, 0.2, 4), np.ones(4)], axis=1)
        d = _sweep_device(op, U0, phr, y, ginv, sq, 0.1, 5, 0, 4, dtype, dev, sched=sched, proposal="rw",
                          reg_scale=rs)
        o = _sweep_oracle(orc, op, U0, phr, y, ginv, sq, 0.1, 5, 0, 4, dtype, sched=sched, proposal="rw",
                          reg_scale=rs)
        _assert_same(d, o, (op.K, op.J, "rw"))


def test_sampler_l96ts_chain_matches_reference_fixture(dev, golden):
    """Reference sampler on the two-scale problem (injected draws) reproduced by MCMCSampler on the GPU."""
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, MCMCSampler, PhiloxRNG,
                             TwoScaleLorenz96Operator, pCNAccepter)

    K, J, n, dt, c, gamma, beta, seed, n_samples, burn_in, interval = golden["tsc_meta"]
    op = TwoScaleLorenz96Operator(K=int(K), J=int(J), c=c, x0=golden["tsc_x0"], dt=dt, n_steps=int(n),
                                  arith="reference")
    q = op.q
    pot = EvolutionPotential(op, golden["tsc_y"], GaussianDistribution(np.zeros(q), gamma**2 * np.eye(q)))
    prior = GaussianDistribution(np.zeros(3), np.diag([10.0, 1.0, 10.0]))
    s = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(int(seed)))
    out = s.run(np.zeros((2, 3)), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
    assert np.array_equal(out, golden["tsc_samples"])


def test_f32_and_f64_posterior_means_agree(dev):
    """SURVEY §8(d) cfg 5 check on a mixing problem: the f32 and f64 kernels
    give posterior means that agree within 4 standard errors (per-chain
    agreement is impossible under chaos; the statistics must agree)."""
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, Lorenz96Operator,
                             MCMCSampler, PhiloxRNG, pCNAccepter)

    K = 8
    op = Lorenz96Operator(K, 8.0, dt=0.01, n_steps=100)
    ut = 0.5 * np.sin(2 * np.pi * np.arange(K) / K)
    y = op(ut) + 0.1 * np.random.default_rng(0).normal(size=K)
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(K), 0.01 * np.eye(K)))
    prior = GaussianDistribution(np.zeros(K), np.eye(K))
    C = 16384
    means, ses = [], []
    for dtype in (np.float32, np.float64):
        s = MCMCSampler(ConstSteppCNProposer(0.2, prior), pCNAccepter(pot), PhiloxRNG(11), dtype=dtype)
        last = s.run(np.zeros((C, K)), n_samples=1, burn_in=600, sample_interval=1, keep="last")
        last = np.asarray(last, dtype=np.float64).reshape(C, K)
        means.append(last.mean(axis=0))
        ses.append(last.std(axis=0) / np.sqrt(C))
    z = np.abs(means[0] - means[1]) / np.sqrt(ses[0] ** 2 + ses[1] ** 2)
    assert np.all(z < 4), z


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_burgers_every_layout_bit_exact(dev, orc, dtype):
    """Both cells-per-lane layouts (8 and 4; in fp32 FMA arith 4 and 2 cell
    pairs per lane) of the Burgers kernel give the oracle's bits, inviscid and
    viscous."""
    from ip_mcmc_amd import BurgersOperator

    for N, lanes_list in ((128, (16, 32)), (256, (32, 64))):
        for arith in ("fma", "reference"):
            for nu in (0.0, 1e-3):
                op = BurgersOperator(N=N, dt_mode="cfl", arith=arith, nu=nu)
                U0, phi0, y, ginv, sq = _problem(op, 40, dtype, orc, seed=N)
                o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.15, 3, 0, 3, dtype)
                for lanes in lanes_list:
                    d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.15, 3, 0, 3, dtype, dev, lanes=lanes)
                    _assert_same(d, o, (N, arith, nu, lanes))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_small_speculative_sweeps_bit_exact(dev, orc, dtype):
    """small_spec_kernel (S lanes = the first S nodes of the speculation tree
    for the chain's recent acceptance rate: the reject chain, the accept chain
    or a branching tree between them) equals the sequential chain bit for bit,
    for every width, with schedules, box constraint, sums and the RW
    regularizer, at low, intermediate and high acceptance."""
    from ip_mcmc_amd import LinearOperator, Lorenz63Operator

    rng = np.random.default_rng(23)
    # linear G: A, y, 1/γ staged in LDS (q (k + 2) <= 1024: the first three) or read
    # from global memory (the last, q = 300)
    ops = [LinearOperator(rng.normal(size=(3, 5)), rng.normal(size=5), arith="reference"),
           LinearOperator(rng.normal(size=(4, 3)), rng.normal(size=3)),
           LinearOperator(0.1 * rng.normal(size=(100, 8)), rng.normal(size=8)),
           LinearOperator(0.05 * rng.normal(size=(300, 6)), rng.normal(size=6)),
           Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=200),
           Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=200, arith="reference")]
    n = 37
    sched = np.stack([np.linspace(0.05, 0.4, n), np.sqrt(1 - np.linspace(0.05, 0.4, n) ** 2)], axis=1)
    high = 0
    for op, broad in [(o, b) for o in ops for b in (False, True)]:
        U0, phi0, y, ginv, sq = _problem(op, 45, dtype, orc, seed=2)
        if broad:  # a broad posterior: 76-92 % of the steps accepted, the kernel speculates along the accept path
            ginv = ginv * (0.001 if isinstance(op, Lorenz63Operator) else 0.03)
            phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
        box = (np.full(op.k, -1.5), None, None)
        box2 = (np.full(op.k, -1.2), np.full(op.k, 1.4), np.full(op.k, 0.1))
        for kw in (dict(), dict(box=box), dict(box=box2), dict(sched=sched), dict(want_sums=True)):
            o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 71, 4, n, dtype, **kw)
            assert 0 < o["acc"].sum() < 45 * n
            high += o["acc"].sum() > 0.6 * 45 * n
            for w in (1, 0, 2, 8, 64):
                d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 71, 4, n, dtype, dev, spec=w, **kw)
                _assert_same(d, o, (type(op).__name__, op.arith, w, list(kw)))
                assert np.array_equal(d["samp"], o["u"])
                if "want_sums" in kw:
                    assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["sum_u2"], o["sum_u2"])
        rs = 0.5 + rng.random(op.k)
        phr = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs).astype(np.float64)
        o = _sweep_oracle(orc, op, U0, phr, y, ginv, sq, 0.2, 9, 0, n, dtype, proposal="rw", reg_scale=rs)
        for w in (4, 32):
            d = _sweep_device(op, U0, phr, y, ginv, sq, 0.2, 9, 0, n, dtype, dev, spec=w, proposal="rw",
                              reg_scale=rs)
            _assert_same(d, o, (type(op).__name__, "rw", w))
    assert high >= 10, high  # the accept-chain trees ran


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_l96_speculative_sweeps_bit_exact(dev, orc, dtype):
    """l96_spec_kernel (spec_width slots of lanes_per_chain lanes per chain) equals the
    sequential chain bit for bit, for every (lanes, width) pair, with schedules,
    box constraint, sums, the RW regularizer and both arithmetic modes."""
    from ip_mcmc_amd import Lorenz96Operator

    n = 23
    sched = np.stack([np.linspace(0.05, 0.4, n), np.sqrt(1 - np.linspace(0.05, 0.4, n) ** 2)], axis=1)
    for (K, lanes_list, arith), scale in [(c, sc) for c in ((8, (1, 2, 4), "fma"), (40, (2, 4, 8), "fma"),
                                                            (32, (4, 16), "reference")) for sc in (0.05, 1.0)]:
        op = Lorenz96Operator(K, 8.0, dt=0.005, n_steps=40, arith=arith)
        U0, phi0, y, ginv, sq = _problem(op, 21, dtype, orc, seed=K)
        # 0.05: a broad posterior, ~99 % accepted (the accept path); 1.0: 9-31 %
        # accepted, acceptances inside the reject path's rounds
        ginv = ginv * scale
        phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
        box = (np.full(K, -0.6), None, None)
        for kw in (dict(), dict(box=box, sched=sched), dict(want_sums=True)):
            o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 5, 2**32 - 7, n, dtype, **kw)
            assert 0 < o["acc"].sum() < 21 * n, o["acc"].sum()
            for lanes in lanes_list:
                for w in (0, 2, 64 // lanes, 256 // lanes):  # 256 // lanes: slots over the 4 waves of a block
                    d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 5, 2**32 - 7, n, dtype, dev, lanes=lanes,
                                      cpl=1, spec=w, **kw)
                    _assert_same(d, o, (K, arith, lanes, w, list(kw)))
                    assert np.array_equal(d["samp"], o["u"])
                    if "want_sums" in kw:
                        assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["sum_u2"], o["sum_u2"])
        rs = np.linspace(0.5, 2.0, K)
        phr = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs).astype(np.float64)
        o = _sweep_oracle(orc, op, U0, phr, y, ginv, sq, 0.1, 9, 0, n, dtype, proposal="rw", reg_scale=rs)
        for w in (4, 256 // lanes_list[-1]):
            d = _sweep_device(op, U0, phr, y, ginv, sq, 0.1, 9, 0, n, dtype, dev, lanes=lanes_list[-1], cpl=1,
                              spec=w, proposal="rw", reg_scale=rs)
            _assert_same(d, o, (K, "rw", w))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ts_and_burgers_speculative_sweeps_bit_exact(dev, orc, dtype):
    """Speculative slots in the two-scale (S·K lanes per chain) and Burgers
    (S·GS lanes) sweeps equal the sequential chain bit for bit, at 10-45 %
    acceptance (branching trees) and 80-97 % (the accept chain), with sums --
    the Burgers cases with two chains per wave caught the recorded-state bug
    spec_replay avoids (ipmc_sweep_common.hpp)."""
    from ip_mcmc_amd import BurgersOperator, TwoScaleLorenz96Operator

    n = 17
    sched = np.stack([np.linspace(0.05, 0.3, n), np.sqrt(1 - np.linspace(0.05, 0.3, n) ** 2)], axis=1)
    rng = np.random.default_rng(31)
    cases = []
    for K, J, arith in ((6, 4, "fma"), (3, 1, "reference"), (11, 2, "fma")):
        op = TwoScaleLorenz96Operator(K=K, J=J, x0=rng.normal(size=K * (1 + J)), dt=0.004, n_steps=25, arith=arith)
        cases.append((op, (0, 2, 64 // K)))
    for N, arith in ((128, "reference"), (256, "fma")):
        op = BurgersOperator(N=N, dt_mode="cfl", T=0.2, arith=arith)
        # the last width spans a whole block (256 lanes: 16 slots of 16 lanes, 8 of 32)
        cases.append((op, (0, 2, 4, 16) if N == 128 else (0, 2, 8)))
    high = 0
    for (op, widths), scale in [(c, sc) for c in cases for sc in (0.2, 3.0)]:
        U0, phi0, y, ginv, sq = _problem(op, 19, dtype, orc, seed=3)
        # 3.0: 10-45 % of the steps accepted (branching speculation trees); 0.2:
        # broad enough that 80-97 % are (the accept chain)
        ginv = ginv * scale
        phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
        for kw in (dict(), dict(box=(np.full(3, -0.3), None, None), sched=sched), dict(want_sums=True)):
            o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 8, 2**32 - 3, n, dtype, **kw)
            assert 0 < o["acc"].sum() < 19 * n, (type(op).__name__, o["acc"].sum())
            high += isinstance(op, TwoScaleLorenz96Operator) and o["acc"].sum() > 0.6 * 19 * n
            for w in widths:
                d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 8, 2**32 - 3, n, dtype, dev, spec=w, **kw)
                _assert_same(d, o, (type(op).__name__, op.arith, w, list(kw)))
                assert np.array_equal(d["samp"], o["u"])
                if "want_sums" in kw:
                    assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["sum_u2"], o["sum_u2"])
        rs = np.array([0.5, 1.0, 2.0])
        phr = orc.init_phi(op, U0.astype(_np(dtype)), y, ginv, reg_scale=rs).astype(np.float64)
        o = _sweep_oracle(orc, op, U0, phr, y, ginv, sq, 0.1, 9, 0, n, dtype, proposal="rw", reg_scale=rs)
        d = _sweep_device(op, U0, phr, y, ginv, sq, 0.1, 9, 0, n, dtype, dev, spec=widths[-1], proposal="rw",
                          reg_scale=rs)
        _assert_same(d, o, (type(op).__name__, "rw"))
    assert high >= 3, high  # the two-scale accept-chain rounds ran


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_speculative_recorded_states_short_launches(dev, orc, dtype):
    """Running sums of speculative sweeps at launch lengths 1, 2, 3 and 5 (a
    round cut short by the launch's end, trees of every shape at 10-97 %
    acceptance), every kernel family, with several chains per wave: the
    recorded states are the ones the walk settled (spec_replay) -- the case
    that caught cross-lane reads inside the walk (Burgers, two chains per
    wave).  In-launch samples: tests/test_gpu_run.py."""
    from ip_mcmc_amd import BurgersOperator, Lorenz63Operator, Lorenz96Operator, TwoScaleLorenz96Operator

    rng = np.random.default_rng(12)
    cases = [(BurgersOperator(N=128, dt_mode="cfl", T=0.2), (2, 4, 16)),
             (TwoScaleLorenz96Operator(K=6, J=4, x0=rng.normal(size=30), dt=0.004, n_steps=25), (2, 4, 8)),
             (Lorenz96Operator(8, 8.0, dt=0.005, n_steps=40), (2, 8, 0)),
             (Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=100), (2, 8, 64))]
    for op, widths in cases:
        for scale in (0.2, 3.0):
            U0, phi0, y, ginv, sq = _problem(op, 19, dtype, orc, seed=3)
            ginv = ginv * scale
            phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
            for n in (1, 2, 3, 5):
                o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 8, 2**32 - 3, n, dtype, want_sums=True)
                for w in widths:
                    d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 8, 2**32 - 3, n, dtype, dev, spec=w,
                                      want_sums=True)
                    what = (type(op).__name__, scale, n, w)
                    _assert_same(d, o, what)
                    assert np.array_equal(d["sum_u"], o["sum_u"]), what
                    assert np.array_equal(d["sum_u2"], o["sum_u2"]), what


# ------------------------------------------------ non-diagonal priors (L·ξ)
def _dense_chol(k, seed):
    """A random SPD prior covariance's lower Cholesky factor (correlated components)."""
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(k, k)) / np.sqrt(k)
    C = 0.3 * np.eye(k) + A @ A.T
    return np.linalg.cholesky(C)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_dense_prior_every_kernel_family_bit_exact(dev, orc, dtype):
    """prior_chol (w = L·ξ, include/ipmc.h) in every sweep kernel family vs the
    oracle: Lorenz-96 (DPP / LDS layouts, packed fp32 pairs, speculation in a
    wave and over a block), Lorenz-63 and linear (one lane per chain and
    speculative slots; linear k = 12 beyond the speculative kernel's k <= 8),
    Burgers and two-scale Lorenz-96 (k = 3); pCN and RW, with a box."""
    from ip_mcmc_amd import (BurgersOperator, LinearOperator, Lorenz63Operator, Lorenz96Operator,
                             TwoScaleLorenz96Operator)

    rng = np.random.default_rng(4)
    cases = [
        (Lorenz96Operator(40, 8.0, dt=0.005, n_steps=40), dict(lanes=4), 131, 5),
        (Lorenz96Operator(40, 8.0, dt=0.005, n_steps=40, arith="reference"), dict(lanes=8), 131, 5),
        (Lorenz96Operator(8, 8.0, dt=0.005, n_steps=40), dict(lanes=2, cpl=2 if dtype == torch.float32 else 0), 131,
         5),
        (Lorenz96Operator(40, 8.0, dt=0.005, n_steps=40), dict(spec=0), 3, 40),  # auto: block-wide slots
        (Lorenz96Operator(16, 8.0, dt=0.005, n_steps=40), dict(spec=8, lanes=4), 17, 30),
        (Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=100), dict(), 200, 12),
        (Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=100), dict(spec=0), 50, 40),
        (LinearOperator(rng.normal(size=(3, 12)), rng.normal(size=12)), dict(), 200, 12),
        (LinearOperator(rng.normal(size=(2, 7)), rng.normal(size=7)), dict(spec=16), 40, 40),
        (BurgersOperator(N=64, dt_mode="fixed", dt=2e-3, n_steps=150), dict(), 70, 4),
        (TwoScaleLorenz96Operator(K=6, J=4, x0=rng.normal(size=30), dt=0.004, n_steps=40), dict(), 70, 6),
    ]
    for i, (op, kw, n, steps) in enumerate(cases):
        U0, phi0, y, ginv, sq = _problem(op, n, dtype, orc, seed=i)
        L = 0.4 * _dense_chol(op.k, i)
        for proposal in ("pcn", "rw"):
            box = None
            if i == 5:  # a box on one component of Lorenz-63
                box = (np.array([-np.inf, -0.6, -np.inf]), np.array([np.inf, 0.6, np.inf]), None)
            d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 500 + i, 3, steps, dtype, dev, chol=L,
                              proposal=proposal, box=box, **kw)
            o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 500 + i, 3, steps, dtype, chol=L,
                              proposal=proposal, box=box)
            _assert_same(d, o, (type(op).__name__, kw, proposal))
            assert np.array_equal(d["samp"], o["u"])
            assert o["acc"].sum() > 0, (type(op).__name__, proposal)


def test_dense_prior_diagonal_factor_equals_diagonal_path(dev, orc):
    """A diagonal L through prior_chol gives the bits of prior_sqrt (0 + p = p)."""
    from ip_mcmc_amd import Lorenz96Operator

    op = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=40)
    U0, phi0, y, ginv, sq = _problem(op, 64, torch.float64, orc, seed=9)
    a = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 42, 0, 6, torch.float64, dev)
    b = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 42, 0, 6, torch.float64, dev, chol=np.diag(sq))
    _assert_same(a, b, "diag")


@pytest.mark.parametrize("case", ["linear", "l96"])
def test_sampler_dense_prior_matches_reference_fixture(dev, golden, case):
    """MCMCSampler with a non-diagonal prior GaussianDistribution reproduces the
    reference sampler's chains (proposer.py:59-82, injected L·ξ draws)."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             LinearOperator, Lorenz96Operator, MCMCSampler, PhiloxRNG, pCNAccepter)

    if case == "linear":
        gamma, beta, seed, n_samples, burn_in, interval = golden["dpl_meta"]
        op = LinearOperator(golden["dpl_g"], arith="reference")
        y, cov, key = golden["dpl_y"], golden["dpl_cov"], "dpl"
    else:
        K, n, dt, gamma, beta, seed, n_samples, burn_in, interval = golden["dp96_meta"]
        op = Lorenz96Operator(int(K), 8.0, x0=golden["l96c_x0"], dt=dt, n_steps=int(n), arith="reference")
        y, cov, key = golden["l96c_y"], golden["dp96_cov"], "dp96"
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(op.q), gamma**2 * np.eye(op.q)))
    prior = GaussianDistribution(np.zeros(op.k), cov)
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(ConstSteppCNProposer(beta, prior), acc, PhiloxRNG(int(seed)))
    out = s.run(np.zeros((3, op.k)), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
    assert np.array_equal(out, golden[f"{key}_samples"])
    assert np.array_equal(np.asarray(acc.accepts), golden[f"{key}_accepts"])
