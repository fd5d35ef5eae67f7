"""The host-side step (ip_mcmc_amd/hostloop.py) on the reference's own fixtures.

On this CPU-only machine the draws come from the product's host library
libipmc_host.so (the kernels' ipmc_rng.hpp compiled by g++; checked against
the oracle's Philox restatement here and against ipmc_pcn_draws on the GPU by
tests/test_gpu_hostloop.py), so every test below runs the product path end to
end: the composition parsing, the draws, the proposal arithmetic, Python
forward maps and predicates, the accept rule and the counters.  The fixtures are the reference sampler's chains with the same
draws injected (tests/golden/make_golden.py): config 1's closure
G(u) = np.dot(g, u) (stuart_examples.py:69-70), a constraint predicate
(accepter.py:39-55), a non-diagonal prior, and the reference Burgers study's
own is_valid_IC + VarStepStandardRWProposer(PWLinear) + StandardRWAccepter.
"""
import numpy as np
import pytest

from ip_mcmc_amd import (ConstrainAccepter, ConstSteppCNProposer, CountedAccepter, EvolutionPotential,
                         GaussianDistribution, MCMCSampler, PhiloxRNG, ProbabilisticAccepter, ProposerBase,
                         StandardRWAccepter, VarStepStandardRWProposer, PWLinear, pCNAccepter, pCNProposer)
from ip_mcmc_amd import hostloop


def _oracle_w(orc):
    """The oracle's restatement of ipmc_pcn_draws (the checker of the host library)."""
    def draws(seed, off, C_, step0, n, k, T, sq, chol, device=None):
        w = np.empty((n, C_, k), dtype=T)
        lr = np.empty((n, C_))
        for s in range(n):
            xi = orc.normals(seed, off, C_, step0 + s, k).astype(T)
            if chol is None:
                w[s] = np.asarray(sq, dtype=np.float64).astype(T)[None, :] * xi
            else:
                L = np.asarray(chol, dtype=np.float64).astype(T)
                acc = np.zeros((C_, k), dtype=T)
                for j in range(k):
                    a = np.zeros(C_, dtype=T)
                    for i in range(j + 1):
                        a = a + xi[:, i] * L[j, i]
                    acc[:, j] = a
                w[s] = acc
            lr[s] = orc.det_log(orc.uniforms(seed, off, C_, step0 + s))
        return w, lr

    return draws


@pytest.fixture
def odraws(monkeypatch):
    """The product's draws on a machine without a GPU: libipmc_host.so."""
    monkeypatch.setattr(hostloop, "DRAW_SOURCE", "auto")
    assert hostloop.draw_source() == "host"


@pytest.mark.parametrize("T", [np.float64, np.float32])
def test_host_library_draws_equal_the_oracle(orc, T):
    """ipmc_host_pcn_draws (diagonal and Cholesky priors, f32/f64) and the raw
    normals / uniforms equal the oracle's restatement bit for bit."""
    rng = np.random.default_rng(2)
    k = 7
    A = rng.normal(size=(k, k))
    L = np.linalg.cholesky(A @ A.T + k * np.eye(k))
    sq = rng.uniform(0.5, 2.0, size=k)
    for prior_sqrt, chol in ((sq, None), (None, L)):
        for seed, off, C_, step0, n in ((42, 0, 5, 0, 3), (2**64 - 3, 2**32 - 6, 6, 2**40 + 7, 2)):
            w, lr = hostloop.host_draws(seed, off, C_, step0, n, k, T, prior_sqrt, chol)
            wo, lro = _oracle_w(orc)(seed, off, C_, step0, n, k, T, prior_sqrt, chol)
            assert w.dtype == T and np.array_equal(w, wo) and np.array_equal(lr, lro)
    xi, r = hostloop.host_raw_draws(9, 3, 4, 100, 2, 5)
    assert np.array_equal(xi[1], orc.normals(9, 3, 4, 101, 5)) and np.array_equal(r[1], orc.uniforms(9, 3, 4, 101))


def test_host_library_threads_and_errors():
    """A block large enough to be split over threads equals the one-thread
    draws; out-of-range chain ids and steps are rejected like the device's."""
    from ip_mcmc_amd import IpmcError, _hostlib

    a = _hostlib.pcn_draws(5, 0, 4096, 0, 8, 40, np.float64, np.ones(40), None, n_threads=8)
    b = _hostlib.pcn_draws(5, 0, 4096, 0, 8, 40, np.float64, np.ones(40), None, n_threads=1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    with pytest.raises(IpmcError, match="2\\^32"):
        _hostlib.pcn_draws(5, 2**32 - 1, 2, 0, 1, 3, np.float64, np.ones(3), None)
    with pytest.raises(IpmcError, match="2\\^63"):
        _hostlib.pcn_draws(5, 0, 1, 2**63 - 1, 2, 3, np.float64, np.ones(3), None)
    with pytest.raises(IpmcError, match="both NULL"):
        _hostlib.pcn_draws(5, 0, 1, 0, 1, 3, np.float64, None, None)
    u = _hostlib.extra_uniforms(5, 7, 11, 3)
    assert u[0] == _hostlib.uniforms(5, 7, 1, 11)[0] and len(set(u)) == 3


def _lin(golden):
    gamma, beta, seed, n_samples, burn_in, interval = golden["lin_meta"]
    g = golden["lin_g"]

    def G(u):  # stuart_examples.py:69-70, the reference's closure
        return np.dot(g, u)

    return G, gamma, beta, int(seed), int(n_samples), int(burn_in), int(interval)


def test_python_G_single_chains_match_reference_fixture(odraws, golden):
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    for chain in range(4):
        acc = CountedAccepter(pCNAccepter(pot))
        s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc,
                        PhiloxRNG(seed), chain_offset=chain)
        out = s.run(np.zeros(4), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
        assert s.last_path == "host"
        assert out.shape == (n_samples, 4)
        np.testing.assert_array_equal(out, golden["lin_samples"][chain])
        assert acc.accepts == int(golden["lin_counts"][chain, 1])
        assert acc.calls == int(golden["lin_counts"][chain, 0])


def test_python_G_many_chains_match_reference_fixture(odraws, golden):
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(pCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc, PhiloxRNG(seed))
    out = s.run(np.zeros((4, 4)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    np.testing.assert_array_equal(out, golden["lin_samples"])
    assert np.array_equal(acc.accepts, golden["lin_counts"][:, 1])
    assert np.array_equal(acc.calls, golden["lin_counts"][:, 0])
    # the Philox position carries over like one Generator (code.org:12-13)
    assert s.rng.step == max(0, burn_in - interval) + n_samples * interval


def test_user_proposer_and_accepter_match_reference_fixture(odraws, golden):
    """The generic tier: a caller's own ProposerBase / ProbabilisticAccepter
    subclasses (the reference's classes, restated) get the same draws through
    rng.multivariate_normal / rng.random."""
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)

    class MyPCN(ProposerBase):  # proposer.py:59-82
        def __init__(self, beta, prior):
            self.beta, self.prior = beta, prior

        def __call__(self, u, rng):
            w = rng.multivariate_normal(mean=np.zeros(4), cov=self.prior.covariance)
            return np.sqrt(1 - self.beta**2) * u + self.beta * w

    noise = GaussianDistribution(0, gamma**2)

    class MyAccepter(ProbabilisticAccepter):  # accepter.py:109-122
        def accept_probability(self, u, v):
            phi = lambda x: -noise.logpdf(golden["lin_y"] - G(x))
            return np.exp(phi(u) - phi(v))

    acc = CountedAccepter(MyAccepter())
    s = MCMCSampler(MyPCN(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc, PhiloxRNG(seed))
    out = s.run(np.zeros((4, 4)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    assert s.last_path == "host-generic"
    np.testing.assert_array_equal(out, golden["lin_samples"])
    assert np.array_equal(acc.accepts, golden["lin_counts"][:, 1])


def test_constraint_predicate_matches_reference_fixture(odraws, golden):
    gamma, beta, seed, n_samples, burn_in, interval = golden["con_meta"]
    g, lo, hi = golden["con_g"], golden["con_lo"], golden["con_hi"]
    pot = EvolutionPotential(lambda u: np.dot(g, u), golden["con_y"], GaussianDistribution(0, gamma**2))
    inner = CountedAccepter(pCNAccepter(pot))
    acc = ConstrainAccepter(inner, lambda v: bool(np.all(lo < v) and np.all(v < hi)))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc,
                    PhiloxRNG(int(seed)))
    out = s.run(np.zeros((3, 4)), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
    np.testing.assert_array_equal(out, golden["con_samples"])
    assert np.array_equal(inner.calls, golden["con_counts"][:, 0])
    assert np.array_equal(inner.accepts, golden["con_counts"][:, 1])
    assert np.array_equal(s.state.calls, golden["con_counts"][:, 0])


def test_dense_prior_with_python_G_matches_reference_fixture(odraws, golden):
    gamma, beta, seed, n_samples, burn_in, interval = golden["dpl_meta"]
    g = golden["dpl_g"]
    k = g.shape[-1]
    pot = EvolutionPotential(lambda u: np.atleast_1d(np.dot(g, u)), golden["dpl_y"],
                             GaussianDistribution(np.zeros(len(golden["dpl_y"])),
                                                  gamma**2 * np.eye(len(golden["dpl_y"]))))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(k), golden["dpl_cov"])),
                    CountedAccepter(pCNAccepter(pot)), PhiloxRNG(int(seed)))
    out = s.run(np.zeros((3, k)), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
    np.testing.assert_array_equal(out, golden["dpl_samples"])
    assert np.array_equal(s.accepter.accepts, golden["dpl_accepts"])


def test_burgers_study_rw_with_is_valid_IC_matches_reference_fixture(orc, odraws, golden):
    """burgers_beta.py's RW study: VarStepStandardRWProposer(PWLinear) +
    StandardRWAccepter inside ConstrainAccepter(is_valid_IC) -- the predicate a
    Python function as the reference writes it (burgers_wasserstein_chain.py:47-55),
    G a Python function (here the oracle's CFL Rusanov + Measurer; on the GPU
    the device operator)."""
    from ip_mcmc_amd import BurgersOperator

    meta = golden["bch_meta"]
    N, gamma, sigma_p, beta, seed = int(meta[0]), meta[1], meta[2], meta[3], int(meta[4])
    n_samples, burn_in, interval = int(meta[5]), int(meta[6]), int(meta[7])
    d_s, d_e, l = meta[8], meta[9], meta[10]
    pm = golden["bch_prior_mean"]
    op = BurgersOperator(prior_mean=pm, N=N, T=1.0, dt_mode="cfl", arith="reference")

    def G(u):
        return orc.forward(op, np.asarray(u)[None, :])[0]

    def is_valid_IC(u):  # burgers_wasserstein_chain.py:47-55, on the perturbation's prior-mean shift
        return -1 < (pm + u)[2] < 1

    prior = GaussianDistribution(np.zeros(3), sigma_p**2 * np.eye(3))
    pot = EvolutionPotential(G, golden["bch_y"], GaussianDistribution(np.zeros(5), gamma**2 * np.eye(5)))
    inner = CountedAccepter(StandardRWAccepter(pot, prior))
    acc = ConstrainAccepter(inner, is_valid_IC)
    s = MCMCSampler(VarStepStandardRWProposer(PWLinear(d_s, d_e, l), prior), acc, PhiloxRNG(seed + 1))
    out = s.run(np.zeros((3, 3)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    np.testing.assert_array_equal(out, golden["bch_rw_samples"])
    assert np.array_equal(inner.calls, golden["bch_rw_counts"][:, 0])
    assert np.array_equal(inner.accepts, golden["bch_rw_counts"][:, 1])


def test_dense_noise_follows_the_reference_accept_rule(odraws, orc):
    """A non-diagonal noise covariance (no device form): the host loop's chains
    equal a direct restatement of the reference step (sampler.py:35-41 with
    pCNAccepter on -noise.logpdf, accepter.py:62) under the same draws."""
    rng = np.random.default_rng(3)
    A = rng.normal(size=(3, 2))
    Gam = np.array([[0.3, 0.1, 0.0], [0.1, 0.2, 0.05], [0.0, 0.05, 0.25]])
    noise = GaussianDistribution(np.zeros(3), Gam)
    y = A @ np.array([0.5, -1.0]) + rng.multivariate_normal(np.zeros(3), Gam)
    G = lambda u: A @ u
    beta, seed, C_, n = 0.4, 77, 5, 60
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(2), np.eye(2))),
                    CountedAccepter(pCNAccepter(EvolutionPotential(G, y, noise))), PhiloxRNG(seed))
    out = s.run(np.zeros((C_, 2)), n_samples=n, burn_in=1, sample_interval=1)
    # the reference step, one chain at a time
    ref = np.zeros((C_, n, 2))
    for c in range(C_):
        u = np.zeros(2)
        for t in range(n):
            xi = orc.normals(seed, c, 1, t, 2)[0]
            v = np.sqrt(1 - beta**2) * u + beta * xi
            r = orc.uniforms(seed, c, 1, t)[0]
            phi = lambda x: -noise.logpdf(y - G(x))
            if np.exp(phi(u) - phi(v)) > r:
                u = v
            ref[c, t] = u
    np.testing.assert_array_equal(out, ref)
    assert 0 < np.sum(s.accepter.accepts) < C_ * n


def test_moments_last_and_interval_zero(odraws, golden):
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    prior = GaussianDistribution(np.zeros(4), np.eye(4))
    s = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed))
    smp = s.run(np.zeros((4, 4)), n_samples=6, burn_in=3, sample_interval=1)
    s2 = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed))
    mom = s2.run(np.zeros((4, 4)), n_samples=6, burn_in=3, sample_interval=1, keep="moments")
    np.testing.assert_array_equal(mom["sum_u"], smp.sum(axis=1))
    assert mom["n"] == 6
    s3 = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed))
    last = s3.run(np.zeros((4, 4)), n_samples=6, burn_in=3, sample_interval=1, keep="last")
    np.testing.assert_array_equal(last, smp[:, -1])
    s4 = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed))
    z = s4.run(np.zeros(4), n_samples=3, burn_in=5, sample_interval=0)
    assert z.shape == (3, 4) and np.array_equal(z[0], z[2]) and s4.rng.step == 5


def test_resume_continues_exactly(odraws, golden):
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    prior = GaussianDistribution(np.zeros(4), np.eye(4))
    full = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed)).run(
        np.zeros((4, 4)), n_samples=10, burn_in=1, sample_interval=3)
    s = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed))
    a = s.run(np.zeros((4, 4)), n_samples=4, burn_in=1, sample_interval=3)
    st = s.checkpoint()
    s2 = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(0))
    b = s2.run(st, n_samples=6, burn_in=0, sample_interval=3)
    np.testing.assert_array_equal(np.concatenate([a, b], axis=1), full)


def test_python_potential_value_is_the_reference_formula(golden):
    """EvolutionPotential.__call__ with a Python G: −noise.logpdf(y − G(u))
    (potential.py:53-54) = the reference's values in the fixture."""
    G, gamma, *_ = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    vals = np.array([pot(u) for u in golden["lin_phi_u"]])
    np.testing.assert_allclose(vals, golden["lin_phi"], rtol=1e-14, atol=1e-13)


def test_sample_file_streams_the_same_samples(odraws, golden, tmp_path):
    """run(sample_file=...) on the host path writes an np.load-able .npy equal
    to the in-memory samples."""
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    prior = GaussianDistribution(np.zeros(4), np.eye(4))
    mem = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed)).run(
        np.zeros((4, 4)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    f = str(tmp_path / "chains.npy")
    out = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed)).run(
        np.zeros((4, 4)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval, sample_file=f)
    np.testing.assert_array_equal(np.asarray(out), mem)
    np.testing.assert_array_equal(np.load(f), golden["lin_samples"])
    one = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed)).run(
        np.zeros(4), n_samples=n_samples, burn_in=burn_in, sample_interval=interval, sample_file=f)
    np.testing.assert_array_equal(np.asarray(one), golden["lin_samples"][0])


def test_float32_chains_round_like_the_kernels(odraws, orc):
    """f32 chains on the host path: v, Φ and the accept comparison in float32
    (the kernels' dtype rules), equal to the oracle's f32 sweep for the same
    linear G evaluated in float32 by the caller."""
    from ip_mcmc_amd import LinearOperator

    rng = np.random.default_rng(6)
    A = rng.normal(size=(3, 4)).astype(np.float32).astype(np.float64)
    op = LinearOperator(A, arith="reference")
    y = A @ np.array([0.3, -0.2, 0.5, 0.1]) + 0.1 * rng.normal(size=3)
    ginv = np.full(3, 10.0)
    U0 = (0.2 * rng.normal(size=(5, 4))).astype(np.float32)

    def G32(u):  # G in float32, in the kernels' order: acc = 0; acc = acc + A_ij (θ0_j + u_j)
        u32 = np.asarray(u, dtype=np.float32)
        A32 = A.astype(np.float32)
        acc = np.zeros(3, dtype=np.float32)
        for j in range(4):
            acc = acc + A32[:, j] * (np.float32(0) + u32[j])
        return acc.astype(np.float64)

    noise = GaussianDistribution(np.zeros(3), 0.01 * np.eye(3))
    s = MCMCSampler(ConstSteppCNProposer(0.3, GaussianDistribution(np.zeros(4), np.eye(4))),
                    CountedAccepter(pCNAccepter(EvolutionPotential(G32, y, noise))), PhiloxRNG(8), dtype=np.float32)
    last = s.run(U0.astype(np.float64), n_samples=1, burn_in=30, sample_interval=30, keep="last")
    Uo = U0.copy()
    phio = orc.potential(op, Uo, y, ginv, np.float32)
    acco = np.zeros(5, dtype=np.int64)
    orc.pcn_sweep(op, Uo, phio, y, ginv, np.ones(4), 0.3, 8, 0, 30, accepts=acco)
    np.testing.assert_array_equal(last, Uo.astype(np.float64))
    np.testing.assert_array_equal(s.state.phi, phio)
    assert np.array_equal(s.accepter.accepts, acco) and acco.sum() > 0


def test_verbose_prints_per_sample_and_shape_errors(odraws, golden, capsys):
    """verbose=True prints sampler.py:24's 'Sampling i/n' and the acceptance
    ratio (:30-31); a forward map returning the wrong number of values raises."""
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))),
                    CountedAccepter(pCNAccepter(pot)), PhiloxRNG(seed), verbose=True)
    s.run(np.zeros(4), n_samples=3, burn_in=5, sample_interval=2)
    out = capsys.readouterr().out.splitlines()
    assert out[:3] == ["Sampling 1/3", "Sampling 2/3", "Sampling 3/3"] and out[3].startswith("Acceptance ratio")
    bad = EvolutionPotential(lambda u: np.array([1.0, 2.0]), golden["lin_y"], GaussianDistribution(0, gamma**2))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), pCNAccepter(bad),
                    PhiloxRNG(seed))
    with pytest.raises(ValueError, match="forward map returned"):
        s.run(np.zeros(4), n_samples=2, burn_in=0, sample_interval=1)


@pytest.mark.parametrize("keep", ["samples", "moments", "last"])
def test_single_chain_float_loop_equals_array_loop(orc, odraws, golden, monkeypatch, keep):
    """One f64 chain runs the host step on Python floats; it equals the array
    loop bit for bit -- RW with the prior regularizer, a predicate, two counted
    layers and each recording mode (the pCN case is pinned to the fixture by
    test_python_G_single_chains_match_reference_fixture)."""
    meta = golden["bch_meta"]
    gamma, sigma_p, seed = meta[1], meta[2], int(meta[4])
    d_s, d_e, l = meta[8], meta[9], meta[10]
    A = np.random.default_rng(5).normal(size=(5, 3))
    prior = GaussianDistribution(np.zeros(3), np.diag([sigma_p**2, 0.5 * sigma_p**2, 2 * sigma_p**2]))
    pot = EvolutionPotential(lambda u: A @ u, A @ np.array([0.1, -0.2, 0.3]) + 0.05,
                             GaussianDistribution(np.zeros(5), gamma**2 * np.eye(5)))
    runs = []
    for fast in (True, False):
        monkeypatch.setattr(hostloop, "SINGLE_CHAIN_FLOATS", fast)
        inner = CountedAccepter(StandardRWAccepter(pot, prior))
        outer = CountedAccepter(ConstrainAccepter(inner, lambda u: abs(u[2]) < 0.4))
        s = MCMCSampler(VarStepStandardRWProposer(PWLinear(d_s, d_e, l), prior), outer, PhiloxRNG(seed),
                        chain_offset=3)
        out = s.run(np.zeros(3), n_samples=40, burn_in=17, sample_interval=3, keep=keep)
        runs.append((out, inner.calls, inner.accepts, outer.calls, outer.accepts, s.state.u, s.state.phi))
    for a, b in zip(*runs):
        if isinstance(a, dict):
            assert a.keys() == b.keys() and all(np.array_equal(a[key], b[key]) for key in a)
        else:
            assert np.array_equal(np.asarray(a), np.asarray(b))
    assert 0 < runs[0][2] < runs[0][1] < runs[0][3]


# ------------------------------------------------ generic tier
class _MyPCN(ProposerBase):
    """proposer.py:59-82 restated as a caller's own class; `parts` splits the
    draw into several multivariate_normal calls (a product prior that samples
    its components one by one, distribution.py:57-59)."""

    def __init__(self, beta, k, parts=(None,)):
        self.beta, self.k, self.parts = beta, k, parts

    def __call__(self, u, rng):
        if self.parts == (None,):
            w = rng.multivariate_normal(mean=np.zeros(self.k), cov=np.eye(self.k))
        else:
            w = np.concatenate([rng.multivariate_normal(mean=np.zeros(p), cov=np.eye(p)) for p in self.parts])
        return np.sqrt(1 - self.beta**2) * u + self.beta * w


def test_generic_tier_product_prior_draws_continue_the_stream(odraws, golden):
    """Two multivariate_normal calls in one step get ξ[0:2] and ξ[2:4] (a
    cursor), so a product prior equals the one-draw proposer: the lin_*
    fixture again, and no two draws of a step are the same numbers."""
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    s = MCMCSampler(_MyPCN(beta, 4, parts=(2, 2)), CountedAccepter(pCNAccepter(pot)), PhiloxRNG(seed))
    out = s.run(np.zeros((4, 4)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    assert s.last_path == "host-generic"
    np.testing.assert_array_equal(out, golden["lin_samples"])


def test_generic_tier_rng_cursor_and_unsupported_methods():
    from ip_mcmc_amd import _hostlib

    rng = hostloop.StepRNG(5)
    xi = _hostlib.normals(5, 7, 1, 11, 3)[0]
    rng.set(xi, _hostlib.uniforms(5, 7, 1, 11)[0], gid=7, step=11)
    a = rng.standard_normal(2)
    b = rng.normal(1.0, 2.0)  # the third component
    c = rng.standard_normal(3)  # components 3..5 from the host library
    full = _hostlib.normals(5, 7, 1, 11, 6)[0]
    np.testing.assert_array_equal(a, full[:2])
    assert b == 1.0 + 2.0 * full[2]
    np.testing.assert_array_equal(c, full[3:6])
    u0, u1, u2 = rng.random(), rng.random(), rng.uniform(2.0, 4.0)
    ex = _hostlib.extra_uniforms(5, 7, 11, 3)
    assert (u0, u1, u2) == (ex[0], ex[1], 2.0 + 2.0 * ex[2]) and u0 != u1
    with pytest.raises(AttributeError, match="supports multivariate_normal"):
        rng.gamma(2.0)


def test_generic_tier_counts_decisions_without_a_counted_accepter(odraws, golden):
    G, gamma, beta, seed, n_samples, burn_in, interval = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    s = MCMCSampler(_MyPCN(beta, 4), pCNAccepter(pot), PhiloxRNG(seed))
    s.run(np.zeros((4, 4)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
    assert np.array_equal(s.state.accepts, golden["lin_counts"][:, 1])
    assert s.state.accept_kind == "generic"


class _MyVarPCN(ProposerBase):
    """A stateful caller proposer (VarSteppCNProposer's pattern, proposer.py:
    105-115: i incremented before use)."""

    def __init__(self, k):
        self.k, self.i = k, 0

    def __call__(self, u, rng):
        self.i += 1
        beta = 0.5 / (1 + 0.1 * self.i)
        w = rng.multivariate_normal(mean=np.zeros(self.k), cov=np.eye(self.k))
        return np.sqrt(1 - beta**2) * u + beta * w


def test_generic_tier_stateful_proposer_advances_once_per_step(odraws, golden):
    """Several chains at once give each chain the schedule one chain would
    see: the multi-chain run equals the chains run one at a time."""
    G, gamma, _, seed, _, _, _ = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    many = MCMCSampler(_MyVarPCN(4), pCNAccepter(pot), PhiloxRNG(seed))
    out = many.run(np.zeros((3, 4)), n_samples=5, burn_in=4, sample_interval=3)
    assert many.proposer.i == 1 + 5 * 3
    for c in range(3):
        one = MCMCSampler(_MyVarPCN(4), pCNAccepter(pot), PhiloxRNG(seed), chain_offset=c)
        np.testing.assert_array_equal(one.run(np.zeros(4), n_samples=5, burn_in=4, sample_interval=3), out[c])


def test_generic_checkpoint_resumes_on_the_structured_tier_with_a_fresh_phi(odraws, golden):
    """A generic run caches no Φ (NaN); resuming its state on a structured
    sampler recomputes Φ(u) and continues exactly like a structured run from
    the same states and Philox position."""
    G, gamma, beta, seed, *_ = _lin(golden)
    pot = EvolutionPotential(G, golden["lin_y"], GaussianDistribution(0, gamma**2))
    prior = GaussianDistribution(np.zeros(4), np.eye(4))
    g = MCMCSampler(_MyPCN(beta, 4), pCNAccepter(pot), PhiloxRNG(seed))
    g.run(np.zeros((4, 4)), n_samples=3, burn_in=1, sample_interval=4)
    st = g.checkpoint()
    assert np.all(np.isnan(st.phi))
    s = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(0))
    a = s.run(st, n_samples=5, burn_in=0, sample_interval=2)
    assert np.all(np.isfinite(s.state.phi))
    ref = MCMCSampler(ConstSteppCNProposer(beta, prior), pCNAccepter(pot), PhiloxRNG(seed))
    ref.rng.step = st.step
    b = ref.run(st.u.copy(), n_samples=5, burn_in=0, sample_interval=2)
    np.testing.assert_array_equal(a, b)
