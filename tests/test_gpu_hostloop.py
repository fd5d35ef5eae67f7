"""The host-side step on the GPU: ipmc_pcn_draws against the oracle, the
reference fixtures through Python forward maps and predicates with the
device's draws, and bit-for-bit agreement with the fused kernels when the
Python G is a device operator in REFERENCE arith."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from test_hostloop_cpu import _oracle_w  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("dense", [False, True])
def test_pcn_draws_match_oracle(dev, orc, dtype, dense):
    from ip_mcmc_amd.hostloop import device_draws

    k, C_, n, off, step0, seed = 7, 37, 5, 1000, 123456789, 0xBEEF
    rng = np.random.default_rng(2)
    if dense:
        A = rng.normal(size=(k, k))
        L, sq = np.linalg.cholesky(A @ A.T + k * np.eye(k)), None
    else:
        L, sq = None, rng.uniform(0.5, 2, size=k)
    w, lr = device_draws(seed, off, C_, step0, n, k, dtype, sq, L, dev)
    wo, lro = _oracle_w(orc)(seed, off, C_, step0, n, k, dtype, sq, L)
    assert w.dtype == dtype and w.shape == (n, C_, k)
    assert np.array_equal(w, wo)
    assert np.array_equal(lr, lro)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("dense", [False, True])
def test_host_library_draws_equal_device_draws(dev, dtype, dense):
    """libipmc_host.so (g++, the CPU) and ipmc_pcn_draws / ipmc_normal /
    ipmc_uniform (hipcc, the GPU) compile one source (csrc/ipmc_rng.hpp) and
    give the same bits -- over a large block (threaded on the host), extreme
    seeds, chain ids near 2^32 and steps near 2^63."""
    from ip_mcmc_amd import _hostlib, device as D
    from ip_mcmc_amd.hostloop import device_draws, host_draws

    rng = np.random.default_rng(4)
    k = 40 if not dense else 9
    if dense:
        A = rng.normal(size=(k, k))
        L, sq = np.linalg.cholesky(A @ A.T + k * np.eye(k)), None
    else:
        L, sq = None, rng.uniform(0.5, 2, size=k)
    for seed, off, C_, step0, n in ((0xBEEF, 0, 4096, 0, 16), (2**64 - 1, 2**32 - 300, 300, 2**63 - 4, 4)):
        w, lr = device_draws(seed, off, C_, step0, n, k, dtype, sq, L, dev)
        wh, lrh = host_draws(seed, off, C_, step0, n, k, dtype, sq, L)
        assert np.array_equal(w, wh) and np.array_equal(lr, lrh)
    # the raw normals and uniforms, including steps from 2^63 on (host-side draws)
    for step in (7, 2**63 + 3):
        z = D.normals(11, 5, 64, step, 13, torch.float64, dev).cpu().numpy()
        assert np.array_equal(z, _hostlib.normals(11, 5, 64, step, 13))
        u = D.uniforms(11, 5, 64, step, dev).cpu().numpy()
        assert np.array_equal(u, _hostlib.uniforms(11, 5, 64, step))


def test_python_G_matches_reference_fixture_with_device_draws(dev, golden):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             MCMCSampler, PhiloxRNG, pCNAccepter)

    gamma, beta, seed, n_samples, burn_in, interval = golden["lin_meta"]
    g = golden["lin_g"]
    pot = EvolutionPotential(lambda u: np.dot(g, u), golden["lin_y"], GaussianDistribution(0, gamma**2))
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(4), np.eye(4))), acc,
                    PhiloxRNG(int(seed)))
    out = s.run(np.zeros((4, 4)), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
    assert s.last_path == "host"
    np.testing.assert_array_equal(out, golden["lin_samples"])
    assert np.array_equal(acc.accepts, golden["lin_counts"][:, 1])


def _l96_problem(dtype):
    from ip_mcmc_amd import EvolutionPotential, GaussianDistribution, Lorenz96Operator

    K = 8
    op = Lorenz96Operator(K, 8.0, dt=0.01, n_steps=100, arith="reference")
    rng = np.random.default_rng(9)
    y = op(0.3 * rng.normal(size=K)) + 0.1 * rng.normal(size=K)
    noise = GaussianDistribution(np.zeros(K), 0.1**2 * np.eye(K))
    return op, y, noise, K


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_host_loop_equals_fused_kernel_in_reference_arith(dev, dtype):
    """G = lambda u: op(u) for a REFERENCE-arith device operator takes the
    host step (one ipmc_forward per chain and step); its samples, accept
    counts and state equal the fused sweep's bit for bit."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             MCMCSampler, PhiloxRNG, pCNAccepter)

    op, y, noise, K = _l96_problem(dtype)
    prior = GaussianDistribution(np.zeros(K), np.eye(K))
    u0 = 0.1 * np.random.default_rng(4).normal(size=(6, K))
    runs = {}
    for name, G in (("device", op), ("host", lambda u: op(u, dtype=dtype))):
        acc = CountedAccepter(pCNAccepter(EvolutionPotential(G, y, noise)))
        s = MCMCSampler(ConstSteppCNProposer(0.3, prior), acc, PhiloxRNG(31), dtype=dtype, chain_offset=5)
        out = s.run(u0, n_samples=5, burn_in=4, sample_interval=3)
        assert s.last_path == name
        runs[name] = (out, np.asarray(acc.accepts), s.state.u, s.state.phi)
    for a, b in zip(runs["device"], runs["host"]):
        assert np.array_equal(a, b)
    assert runs["host"][1].sum() > 0


def test_host_predicate_equals_device_box(dev, golden):
    """The reference Burgers RW study with is_valid_IC as a Python predicate
    and G a device operator (batched ipmc_forward per step) equals the fused
    kernel with the equivalent BoxConstraint, and both equal the reference
    fixture."""
    from ip_mcmc_amd import (BoxConstraint, BurgersOperator, ConstrainAccepter, CountedAccepter,
                             EvolutionPotential, GaussianDistribution, MCMCSampler, PhiloxRNG, PWLinear,
                             StandardRWAccepter, VarStepStandardRWProposer)

    meta = golden["bch_meta"]
    N, gamma, sigma_p, seed = int(meta[0]), meta[1], meta[2], int(meta[4])
    n_samples, burn_in, interval = int(meta[5]), int(meta[6]), int(meta[7])
    d_s, d_e, l = meta[8], meta[9], meta[10]
    pm = golden["bch_prior_mean"]
    op = BurgersOperator(prior_mean=pm, N=N, T=1.0, dt_mode="cfl", arith="reference")
    prior = GaussianDistribution(np.zeros(3), sigma_p**2 * np.eye(3))
    noise = GaussianDistribution(np.zeros(5), gamma**2 * np.eye(5))
    outs = {}
    for name, constraint in (("host", lambda u: -1 < (pm + u)[2] < 1),
                             ("device", BoxConstraint([-np.inf, -np.inf, -1.0], [np.inf, np.inf, 1.0], pm))):
        inner = CountedAccepter(StandardRWAccepter(EvolutionPotential(op, golden["bch_y"], noise), prior))
        s = MCMCSampler(VarStepStandardRWProposer(PWLinear(d_s, d_e, l), prior), ConstrainAccepter(inner, constraint),
                        PhiloxRNG(seed + 1))
        outs[name] = s.run(np.zeros((3, 3)), n_samples=n_samples, burn_in=burn_in, sample_interval=interval)
        assert s.last_path == name
        assert np.array_equal(inner.calls, golden["bch_rw_counts"][:, 0])
    np.testing.assert_array_equal(outs["host"], golden["bch_rw_samples"])
    np.testing.assert_array_equal(outs["device"], golden["bch_rw_samples"])


def test_dense_noise_with_device_G(dev, orc):
    """A non-diagonal noise covariance over a device forward map: G evaluated
    by the kernels for all chains at once, Φ = ½‖L⁻¹(y − G)‖² on the host; the
    chains follow the reference accept rule exp(Φu − Φv) > r (accepter.py:62)
    under the same draws."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             LinearOperator, MCMCSampler, PhiloxRNG, pCNAccepter)

    rng = np.random.default_rng(3)
    A = rng.normal(size=(3, 2))
    Gam = np.array([[0.3, 0.1, 0.0], [0.1, 0.2, 0.05], [0.0, 0.05, 0.25]])
    noise = GaussianDistribution(np.zeros(3), Gam)
    y = A @ np.array([0.5, -1.0]) + rng.multivariate_normal(np.zeros(3), Gam)
    op = LinearOperator(A, arith="reference")
    beta, seed, C_, n = 0.4, 77, 64, 40
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(2), np.eye(2))),
                    CountedAccepter(pCNAccepter(EvolutionPotential(op, y, noise))), PhiloxRNG(seed))
    out = s.run(np.zeros((C_, 2)), n_samples=n, burn_in=1, sample_interval=1)
    assert s.last_path == "host"
    ref = np.zeros((C_, n, 2))
    for c in range(C_):
        u = np.zeros(2)
        for t in range(n):
            v = np.sqrt(1 - beta**2) * u + beta * orc.normals(seed, c, 1, t, 2)[0]
            phi = lambda x: -noise.logpdf(y - A @ x)
            if np.exp(phi(u) - phi(v)) > orc.uniforms(seed, c, 1, t)[0]:
                u = v
            ref[c, t] = u
    np.testing.assert_array_equal(out, ref)


def test_stuart_example_21_composition_unchanged(dev):
    """report/scripts/stuart_examples.py:58-109 as written: pCNProposer(beta=0.25),
    CountedAccepter(pCNAccepter), the closure G(u) = np.dot(g, u), scalar noise,
    one numpy Generator for the data and the sampler; n_samples reduced from
    5 000 to 400 for the test (examples/stuart_reference.py runs all 5 000).
    The samples' mean matches the exact posterior (results.org:59-62) within
    4 standard errors of 400 samples 200 steps apart."""
    from ip_mcmc_amd import (CountedAccepter, EvolutionPotential, GaussianDistribution, MCMCSampler,
                             pCNAccepter, pCNProposer)

    n = 1
    g = np.array([int(x) for x in str(np.pi) if x != "."])[:n]
    u = np.array([int(x) for x in str(np.e) if x != "."])[:n]

    def G(u):
        return np.dot(g, u)

    prior = GaussianDistribution(mean=np.zeros_like(u), covariance=np.identity(n))
    gamma = 0.5
    noise = GaussianDistribution(mean=0, covariance=gamma**2)
    rng = np.random.default_rng(1)
    data = G(u) + noise.sample(rng)  # SyntheticModel.observe
    potential = EvolutionPotential(G, data, noise)
    accepter = CountedAccepter(pCNAccepter(potential=potential))
    sampler = MCMCSampler(pCNProposer(beta=0.25, prior=prior), accepter, rng)
    samples = sampler.run(u_0=np.zeros_like(u), n_samples=400)
    assert samples.shape == (400, 1) and sampler.last_path == "host"
    assert accepter.calls == 1000 - 200 + 400 * 200
    denom = gamma**2 + float(g @ g)
    m, v = float(g[0]) * float(np.ravel(data)[0]) / denom, 1 - float(g @ g) / denom
    assert abs(samples.mean() - m) < 4 * np.sqrt(v / 400)
    assert 0.2 < accepter.ratio() < 0.9


def test_dense_prior_draws_have_the_prior_covariance(dev):
    """Dense priors are pinned to the reference only distributionally (the
    reference samples N(0, C) by numpy's SVD path, the build by L·ξ;
    tests/golden/make_golden.py:make_dense_prior): over 262 144 chains the
    sample covariance of ipmc_pcn_draws' w equals C entrywise within 5
    standard errors, se_ij = sqrt((C_ii C_jj + C_ij²) / n), and the mean is 0
    within 5 se."""
    from ip_mcmc_amd.hostloop import device_draws

    k, n = 6, 262144
    idx = np.arange(k)
    C = 0.7 ** np.abs(idx[:, None] - idx[None, :]) * np.sqrt(np.outer(1 + idx, 1 + idx))
    L = np.linalg.cholesky(C)
    w, _ = device_draws(99, 0, n, 5, 1, k, np.float64, None, L, dev)
    w = w[0]
    mean = w.mean(axis=0)
    assert np.all(np.abs(mean) < 5 * np.sqrt(np.diag(C) / n)), mean
    S = np.cov(w, rowvar=False)
    se = np.sqrt((np.outer(np.diag(C), np.diag(C)) + C**2) / n)
    z = np.abs(S - C) / se
    assert z.max() < 5, z.max()
