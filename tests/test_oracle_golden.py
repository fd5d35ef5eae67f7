"""The CPU oracle (oracle/liboracle.so) pinned against the reference.

Fixtures: tests/golden/reference_golden.npz, made by tests/golden/make_golden.py
from the reference itself (ochsnerd/ip_mcmc in /root/reference).
"""
import numpy as np
import pytest

from ip_mcmc_amd.forward import BurgersOperator, LinearOperator, Lorenz96Operator, TwoScaleLorenz96Operator


# ----------------------------------------------------------------- RNG
def test_philox_random123_kats(orc):
    # Random123 known-answer vectors for philox4x32-10
    assert list(orc.philox([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(orc.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(orc.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_det_log_accuracy(orc):
    x = np.exp(np.random.default_rng(0).uniform(-37.0, 0.0, 200_000))
    x = np.concatenate([x, [1.0, 2.0**-53, 0.5, np.nextafter(1.0, 0.0)]])
    err = np.abs(orc.det_log(x) - np.log(x))
    assert err.max() < 4e-15
    assert orc.det_log(np.array([0.0]))[0] == -np.inf


def test_det_sincos_accuracy(orc):
    t = np.concatenate([np.random.default_rng(1).random(200_000), [0.0, 0.125, 0.25, 0.5, 0.75, 1 - 2.0**-53]])
    s, c = orc.sincos_2pi(t)
    assert np.abs(s - np.sin(2 * np.pi * t)).max() < 2e-15
    assert np.abs(c - np.cos(2 * np.pi * t)).max() < 2e-15
    assert np.all(s * s + c * c <= 1 + 4e-16)


def test_normals_and_uniforms_distribution(orc):
    z = orc.normals(7, 0, 100_000, 3, 4).ravel()
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1) < 0.01
    assert abs((z**4).mean() - 3) < 0.05
    r = orc.uniforms(7, 0, 100_000, 3)
    assert r.min() >= 0 and r.max() < 1 and abs(r.mean() - 0.5) < 0.005
    # counter-based: a chain's draw depends on its global id only
    a = orc.normals(7, 10, 5, 3, 4)
    b = orc.normals(7, 0, 20, 3, 4)[10:15]
    assert np.array_equal(a, b)


# ------------------------------------------------------------ Lorenz-96
def test_l96_rhs_reference_order_bit_exact(orc, golden):
    """REFERENCE arith reproduces Lorenz96.__call__ (lorenz.py:77-81) bit for bit."""
    for pre in ("l96_rhs", "l96_rhs4"):
        X, F, R = golden[pre + "_x"], golden[pre + "_F"], golden[pre + "_out"]
        got = np.stack([orc.l96_rhs(X[i], F[i], "reference") for i in range(len(X))])
        assert np.array_equal(got, R)


def test_l96_rhs_fma_close(orc, golden):
    X, F, R = golden["l96_rhs_x"], golden["l96_rhs_F"], golden["l96_rhs_out"]
    got = np.stack([orc.l96_rhs(X[i], F[i], "fma") for i in range(len(X))])
    np.testing.assert_allclose(got, R, rtol=0, atol=1e-13 * np.abs(X).max() ** 2)


@pytest.mark.parametrize("name,K,F", [("forcing", 3, 2.0), ("slow_nonlinearity", 4, 0.0)])
def test_l96_reference_kats(orc, golden, name, K, F):
    """lorenz.py:114-171 known answers (slow part; the build's L96 is single scale)."""
    x = golden[f"l96_kat_{name}_in"][:K]
    want = golden[f"l96_kat_{name}_out"][:K]
    assert np.array_equal(orc.l96_rhs(x, F, "reference"), want)


@pytest.mark.parametrize("K", [40, 8])
def test_l96_forward_reference_bit_exact(orc, golden, K):
    """G(u) (RK4 time average) with the reference RHS object vs the oracle, fp64."""
    n, dt = golden[f"l96_G{K}_meta"]
    op = Lorenz96Operator(K, 8.0, x0=golden[f"l96_G{K}_x0"], dt=dt, n_steps=int(n), arith="reference")
    got = orc.forward(op, golden[f"l96_G{K}_u"])
    assert np.array_equal(got, golden[f"l96_G{K}_G"])
    op_f = Lorenz96Operator(K, 8.0, x0=golden[f"l96_G{K}_x0"], dt=dt, n_steps=int(n), arith="fma")
    np.testing.assert_allclose(orc.forward(op_f, golden[f"l96_G{K}_u"]), golden[f"l96_G{K}_G"], rtol=1e-9)


def _replay(orc, op, meta_samples, y, gamma, beta, seed, n_samples, burn_in, interval, n_chains, prior_sqrt):
    U = np.zeros((n_chains, op.k))
    ginv = np.full(op.q, 1.0 / gamma)
    phi = orc.potential(op, U, y, ginv)
    acc = np.zeros(n_chains, dtype=np.int64)
    step = 0
    nb = max(0, burn_in - interval)
    orc.pcn_sweep(op, U, phi, y, ginv, prior_sqrt, beta, seed, step, nb, accepts=acc)
    step += nb
    samples = np.zeros((n_chains, n_samples, op.k))
    for i in range(n_samples):
        orc.pcn_sweep(op, U, phi, y, ginv, prior_sqrt, beta, seed, step, interval, accepts=acc)
        step += interval
        samples[:, i] = U
    return samples, acc


def test_linear_chain_matches_reference_sampler(orc, golden):
    """Config 1 through the reference MCMCSampler (injected draws) vs the oracle."""
    gamma, beta, seed, n_samples, burn_in, interval = golden["lin_meta"]
    op = LinearOperator(golden["lin_g"], arith="reference")
    samples, acc = _replay(orc, op, None, golden["lin_y"], gamma, beta, int(seed), int(n_samples), int(burn_in),
                           int(interval), 4, np.ones(4))
    assert np.array_equal(acc, golden["lin_decisions"].sum(axis=1))
    assert np.array_equal(acc, golden["lin_counts"][:, 1])
    np.testing.assert_array_equal(samples, golden["lin_samples"])


def _rw_schedule(kind, meta, i0, n):
    """Step sizes of the reference's RW proposers for proposals i0+1 .. i0+n."""
    delta_c, d_s, d_e, l = meta[5], meta[6], meta[7], meta[8]
    if kind == "const":
        return None, float(np.sqrt(2 * delta_c))
    slope = (d_s - d_e) / l
    d = [d_e if i > l else d_s - slope * i for i in range(i0 + 1, i0 + n + 1)]
    sched = np.stack([np.sqrt(2) * np.sqrt(np.array(d)), np.ones(n)], axis=1)
    return sched, 0.0


@pytest.mark.parametrize("kind", ["const", "var"])
def test_rw_chain_matches_reference_sampler(orc, golden, kind):
    """ConstStep/VarStepStandardRWProposer + StandardRWAccepter (accepter.py:86-106,
    incl. its sqrt-covariance regularizer, Q6) through the reference sampler vs the oracle."""
    meta = golden["rw_meta"]
    gamma, seed, n_samples, burn_in, interval = meta[0], int(meta[1]), int(meta[2]), int(meta[3]), int(meta[4])
    op = LinearOperator(golden["rw_g"], arith="reference")
    sq = np.sqrt(golden["rw_prior_var"])
    y, ginv = golden["rw_y"], np.array([1 / gamma])
    U = np.zeros((3, 4))
    phi = orc.init_phi(op, U, y, ginv, reg_scale=sq)
    acc = np.zeros(3, dtype=np.int64)
    step = 0
    samples = np.zeros((3, n_samples, 4))
    blocks = [max(0, burn_in - interval)] + [interval] * n_samples
    for b, n in enumerate(blocks):
        sched, beta = _rw_schedule(kind, meta, step, n)
        orc.pcn_sweep(op, U, phi, y, ginv, sq, beta, seed, step, n, accepts=acc, beta_schedule=sched,
                      proposal="rw", reg_scale=sq)
        step += n
        if b > 0:
            samples[:, b - 1] = U
    assert np.array_equal(acc, golden[f"rw_{kind}_counts"][:, 1])
    np.testing.assert_array_equal(samples, golden[f"rw_{kind}_samples"])


def test_rw_accept_potential_matches_reference(orc, golden):
    """I(u) = Φ(u) + ½‖C^{1/2}u‖² (accepter.py:104-106) vs StandardRWAccepter._I, up to Φ's constant."""
    gamma = golden["rw_meta"][0]
    op = LinearOperator(golden["rw_g"], arith="reference")
    U = np.ascontiguousarray(golden["rw_I_u"])
    got = orc.init_phi(op, U, golden["rw_y"], [1 / gamma], reg_scale=np.sqrt(golden["rw_prior_var"]))
    const = 0.5 * (np.log(2 * np.pi) + np.log(gamma**2))
    np.testing.assert_allclose(got + const, golden["rw_I"], rtol=1e-13, atol=1e-12)


def test_linear_potential_matches_reference_up_to_constant(orc, golden):
    gamma = golden["lin_meta"][0]
    op = LinearOperator(golden["lin_g"], arith="reference")
    phi = orc.potential(op, golden["lin_phi_u"], golden["lin_y"], [1 / gamma])
    const = 0.5 * (np.log(2 * np.pi) + np.log(gamma**2))
    np.testing.assert_allclose(phi + const, golden["lin_phi"], rtol=1e-13, atol=1e-12)


def test_l96_chain_matches_reference_sampler(orc, golden):
    K, n, dt, gamma, beta, seed, n_samples, burn_in, interval = golden["l96c_meta"]
    K = int(K)
    op = Lorenz96Operator(K, 8.0, x0=golden["l96c_x0"], dt=dt, n_steps=int(n), arith="reference")
    samples, acc = _replay(orc, op, None, golden["l96c_y"], gamma, beta, int(seed), int(n_samples), int(burn_in),
                           int(interval), 3, np.ones(K))
    assert np.array_equal(acc, golden["l96c_decisions"].sum(axis=1))
    np.testing.assert_array_equal(samples, golden["l96c_samples"])


# ------------------------------------------------- two-scale Lorenz-96
TS_RHS_CASES = [(6, 4), (5, 8), (4, 10), (3, 1), (7, 16), (2, 2)]


@pytest.mark.parametrize("K,J", TS_RHS_CASES)
def test_l96ts_rhs_reference_order_bit_exact(orc, golden, K, J):
    """Two-scale Lorenz96.__call__ (lorenz.py:44-101) reproduced bit for bit (REFERENCE arith)."""
    X, P, R = golden[f"ts_rhs_{K}_{J}_x"], golden[f"ts_rhs_{K}_{J}_p"], golden[f"ts_rhs_{K}_{J}_out"]
    got = np.stack([orc.l96ts_rhs(X[i], K, J, P[i]) for i in range(len(X))])
    assert np.array_equal(got, R)
    fm = np.stack([orc.l96ts_rhs(X[i], K, J, P[i], "fma") for i in range(len(X))])
    np.testing.assert_allclose(fm, R, rtol=1e-12, atol=1e-12 * np.abs(R).max())


@pytest.mark.parametrize("name,K,J,p", [
    ("forcing", 3, 1, (2, 1, 1, 1)),
    ("slow_nonlinearity", 4, 1, (0, 0, 0, 0)),
    ("fast_nonlinearity", 1, 4, (0, 0, 1, 2)),
    ("step", 2, 2, (1, 1, 1, 1)),
])
def test_l96ts_reference_kats(orc, golden, name, K, J, p):
    """All four test_Lorenz96 known answers (lorenz.py:114-171), two-scale RHS."""
    x = golden[f"l96_kat_{name}_in"]
    assert np.array_equal(orc.l96ts_rhs(x, K, J, p), golden[f"l96_kat_{name}_out"])


@pytest.mark.parametrize("K,J", [(6, 4), (4, 8), (3, 1)])
def test_l96ts_forward_reference_bit_exact(orc, golden, K, J):
    """G = time-averaged reference moment_function (lorenz_mcmc.py:17-40) of the
    RK4 trajectory of the reference RHS object, vs the oracle, fp64."""
    n, dt, c = golden[f"ts_G{K}_{J}_meta"]
    kw = dict(K=K, J=J, c=c, x0=golden[f"ts_G{K}_{J}_x0"], dt=dt, n_steps=int(n))
    got = orc.forward(TwoScaleLorenz96Operator(**kw, arith="reference"), golden[f"ts_G{K}_{J}_u"])
    assert np.array_equal(got, golden[f"ts_G{K}_{J}_G"])
    fm = orc.forward(TwoScaleLorenz96Operator(**kw, arith="fma"), golden[f"ts_G{K}_{J}_u"])
    np.testing.assert_allclose(fm, golden[f"ts_G{K}_{J}_G"], rtol=1e-9, atol=1e-10)


def test_l96ts_moment_function_matches_reference(golden):
    """The oracle's moment definition (reference mode: Ybar_k = Y_{k,0}, Q8) vs
    moment_function itself on a random trajectory."""
    Y, f = golden["ts_mom_y"], golden["ts_mom_f"]
    K, J = 6, 4
    X, Yb = Y[:K], Y[K::J][:K]
    assert np.array_equal(np.concatenate([X, Yb, X * X, X * Yb, Yb * Yb]), f)


def test_l96ts_chain_matches_reference_sampler(orc, golden):
    K, J, n, dt, c, gamma, beta, seed, n_samples, burn_in, interval = golden["tsc_meta"]
    op = TwoScaleLorenz96Operator(K=int(K), J=int(J), c=c, x0=golden["tsc_x0"], dt=dt, n_steps=int(n),
                                  arith="reference")
    samples, acc = _replay(orc, op, None, golden["tsc_y"], gamma, beta, int(seed), int(n_samples), int(burn_in),
                           int(interval), 2, np.sqrt([10.0, 1.0, 10.0]))
    assert np.array_equal(acc, golden["tsc_decisions"].sum(axis=1))
    np.testing.assert_array_equal(samples, golden["tsc_samples"])


# ---------------------------------------------------------------- Burgers
def test_rusanov_kats(orc, golden):
    """rusanov.py:144-164 known answers, evaluated by the reference."""
    for (a, b), want in zip(golden["rus_kat_flux_in"], golden["rus_kat_flux_out"]):
        assert orc.rusanov_flux(a, b) == want
    r = orc.rusanov_rate(golden["rus_kat_rate_in"], golden["rus_kat_rate_dx"][0])
    assert np.array_equal(r[1:-1], golden["rus_kat_rate_out"])
    np.testing.assert_allclose(r[1:-1], [-10, 32.5, -37.5])
    r = orc.rusanov_rate(golden["rus_rate_w"], golden["rus_rate_dx"][0])
    assert np.array_equal(r[1:-1], golden["rus_rate_out"])


def test_rusanov_kats_fma_arith(orc, golden):
    """The fp64 kernels' FMA-arith flux (the F2 = 4F scale, rus_rate_f2) on the
    same known answers: exact on these small integers, the rates within a few
    ulps of the reference's."""
    for (a, b), want in zip(golden["rus_kat_flux_in"], golden["rus_kat_flux_out"]):
        assert orc.rusanov_flux(a, b, "fma") == want
    r = orc.rusanov_rate(golden["rus_kat_rate_in"], golden["rus_kat_rate_dx"][0], "fma")
    np.testing.assert_allclose(r[1:-1], golden["rus_kat_rate_out"], rtol=1e-14)
    r = orc.rusanov_rate(golden["rus_rate_w"], golden["rus_rate_dx"][0], "fma")
    np.testing.assert_allclose(r[1:-1], golden["rus_rate_out"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("N", [32, 128, 256])
def test_burgers_forward_reference_bit_exact(orc, golden, N):
    """FVMObservationOperator = Measurer(RusanovFVM.integrate(IC)) of the reference vs the oracle, fp64, CFL dt."""
    op = BurgersOperator(prior_mean=(0.0, 0.0, 0.0), N=N, T=1.0, dt_mode="cfl", arith="reference")
    np.testing.assert_array_equal(op.x, golden[f"bur{N}_x"])
    assert op.dx == golden[f"bur{N}_dx"][0]
    np.testing.assert_array_equal(np.stack([op.win_lo, op.win_hi]), golden[f"bur{N}_win"])
    G = orc.forward(op, golden[f"bur{N}_theta"])
    np.testing.assert_array_equal(G, golden[f"bur{N}_G"])
    op_f = BurgersOperator(prior_mean=(0.0, 0.0, 0.0), N=N, T=1.0, dt_mode="cfl", arith="fma")
    np.testing.assert_allclose(orc.forward(op_f, golden[f"bur{N}_theta"]), golden[f"bur{N}_G"], rtol=1e-9,
                               atol=1e-12)


# ------------------------------------------------------ burn-in (§8(f) #2)
def test_burn_in_oracle_matches_reference(orc, golden):
    """len_burn_in (burgers/utilities.py:134-167), run by make_golden.py on the
    reference's own function, vs the C restatement: identical indices."""
    for i in range(int(golden["bi_count"])):
        assert orc.burn_in(golden[f"bi_x_{i}"]) == int(golden[f"bi_out_{i}"]), i
    assert np.array_equal(orc.burn_in(golden["bi_batch_x"]), golden["bi_batch_out"])
    assert len(set(golden["bi_batch_out"].tolist())) > 5, "fixture exercises too few outcomes"


def test_constrained_chain_matches_reference_sampler(orc, golden):
    """ConstrainAccepter(CountedAccepter(pCNAccepter)) through the reference sampler
    (accepter.py:39-55): box-rejected proposals neither call the inner accepter nor
    draw its uniform; the oracle's box reproduces samples, accepts and calls."""
    gamma, beta, seed, n_samples, burn_in, interval = golden["con_meta"]
    op = LinearOperator(golden["con_g"], arith="reference")
    n_chains, y = 3, golden["con_y"]
    U = np.zeros((n_chains, 4))
    ginv = np.full(1, 1.0 / gamma)
    phi = orc.potential(op, U, y, ginv)
    acc = np.zeros(n_chains, dtype=np.int64)
    calls = np.zeros(n_chains, dtype=np.int64)
    box = (golden["con_lo"], golden["con_hi"], None)
    step = 0
    nb = max(0, int(burn_in) - int(interval))
    orc.pcn_sweep(op, U, phi, y, ginv, np.ones(4), beta, int(seed), step, nb, accepts=acc, calls=calls, box=box)
    step += nb
    samples = np.zeros((n_chains, int(n_samples), 4))
    for i in range(int(n_samples)):
        orc.pcn_sweep(op, U, phi, y, ginv, np.ones(4), beta, int(seed), step, int(interval), accepts=acc,
                      calls=calls, box=box)
        step += int(interval)
        samples[:, i] = U
    np.testing.assert_array_equal(samples, golden["con_samples"])
    assert np.array_equal(calls, golden["con_counts"][:, 0])
    assert np.array_equal(acc, golden["con_counts"][:, 1])


def _bch_blocks(meta):
    burn_in, interval, n_samples = int(meta[6]), int(meta[7]), int(meta[5])
    return [max(0, burn_in - interval)] + [interval] * n_samples


@pytest.mark.parametrize("kind", ["pcn", "rw"])
def test_burgers_chain_matches_reference_sampler(orc, golden, kind):
    """The reference's Burgers study (burgers_beta.py:25-128, N=32) through its own
    sampler with injected draws: pCN, and VarStepStandardRWProposer(PWLinear) +
    StandardRWAccepter inside ConstrainAccepter(is_valid_IC) -- the oracle's
    CFL Rusanov chains reproduce samples, accepts and calls bit for bit."""
    meta = golden["bch_meta"]
    N, gamma, sigma_p, beta, seed = int(meta[0]), meta[1], meta[2], meta[3], int(meta[4])
    op = BurgersOperator(prior_mean=golden["bch_prior_mean"], N=N, T=1.0, dt_mode="cfl", arith="reference")
    y, ginv, sq = golden["bch_y"], np.full(5, 1 / gamma), np.full(3, sigma_p)
    U = np.zeros((3, 3))
    acc = np.zeros(3, dtype=np.int64)
    calls = np.zeros(3, dtype=np.int64)
    samples = np.zeros((3, int(meta[5]), 3))
    step = 0
    if kind == "pcn":
        phi = orc.potential(op, U, y, ginv)
        for b, n in enumerate(_bch_blocks(meta)):
            orc.pcn_sweep(op, U, phi, y, ginv, sq, beta, seed, step, n, accepts=acc, calls=calls)
            step += n
            if b > 0:
                samples[:, b - 1] = U
    else:
        phi = orc.init_phi(op, U, y, ginv, reg_scale=sq)
        d_s, d_e, l = meta[8], meta[9], meta[10]
        box = (np.array([-np.inf, -np.inf, -1.0]), np.array([np.inf, np.inf, 1.0]), golden["bch_prior_mean"])
        for b, n in enumerate(_bch_blocks(meta)):
            d = [d_e if i > l else d_s - (d_s - d_e) / l * i for i in range(step + 1, step + n + 1)]
            sched = np.stack([np.sqrt(2) * np.sqrt(np.array(d)), np.ones(n)], axis=1)
            orc.pcn_sweep(op, U, phi, y, ginv, sq, 0.0, seed + 1, step, n, accepts=acc, calls=calls, box=box,
                          beta_schedule=sched, proposal="rw", reg_scale=sq)
            step += n
            if b > 0:
                samples[:, b - 1] = U
    np.testing.assert_array_equal(samples, golden[f"bch_{kind}_samples"])
    assert np.array_equal(calls, golden[f"bch_{kind}_counts"][:, 0])
    assert np.array_equal(acc, golden[f"bch_{kind}_counts"][:, 1])


@pytest.mark.parametrize("case", ["linear", "l96"])
def test_dense_prior_chain_matches_reference_sampler(orc, golden, case):
    """A non-diagonal prior covariance (proposer.py:59-82, w ~ N(0, C) from
    GaussianDistribution.sample) through the reference sampler with injected
    L·ξ draws: the oracle's prior_chol proposal reproduces samples and accepts."""
    if case == "linear":
        gamma, beta, seed, n_samples, burn_in, interval = golden["dpl_meta"]
        op = LinearOperator(golden["dpl_g"], arith="reference")
        y, cov, key = golden["dpl_y"], golden["dpl_cov"], "dpl"
    else:
        K, n, dt, gamma, beta, seed, n_samples, burn_in, interval = golden["dp96_meta"]
        op = Lorenz96Operator(int(K), 8.0, x0=golden["l96c_x0"], dt=dt, n_steps=int(n), arith="reference")
        y, cov, key = golden["l96c_y"], golden["dp96_cov"], "dp96"
    k = op.k
    L = np.linalg.cholesky(cov)
    U = np.zeros((3, k))
    ginv = np.full(op.q, 1.0 / gamma)
    phi = orc.potential(op, U, y, ginv)
    acc = np.zeros(3, dtype=np.int64)
    step = 0
    samples = np.zeros((3, int(n_samples), k))
    for b, nb in enumerate([max(0, int(burn_in) - int(interval))] + [int(interval)] * int(n_samples)):
        orc.pcn_sweep(op, U, phi, y, ginv, None, beta, int(seed), step, nb, accepts=acc, prior_chol=L)
        step += nb
        if b > 0:
            samples[:, b - 1] = U
    np.testing.assert_array_equal(samples, golden[f"{key}_samples"])
    assert np.array_equal(acc, golden[f"{key}_accepts"])


def _burgers_textbook(op, u):
    """Viscous Burgers by the textbook form in numpy float64: SSPRK2 with
    L(w) = -(F_{i+1/2} - F_{i-1/2})/dx + nu (w_{i+1} - 2 w_i + w_{i-1})/dx^2,
    Rusanov F, outflow ghosts (rusanov.py:62-100), fixed dt, then the
    Measurer windows (utilities.py:82-109)."""
    left, right, jump = 1.0 + op.theta0[0] + u[0], op.theta0[1] + u[1], op.theta0[2] + u[2]
    w = np.where(op.x < jump, left, right).astype(np.float64)
    dx, nu, dt = op.dx, op.nu, op.dt

    def rate(w):
        a, b = w[:-1], w[1:]
        F = 0.25 * (a * a + b * b) - 0.5 * np.maximum(np.abs(a), np.abs(b)) * (b - a)
        r = np.zeros_like(w)
        r[1:-1] = -(F[1:] - F[:-1]) / dx + nu * (w[2:] - 2.0 * w[1:-1] + w[:-2]) / dx**2
        return r

    for _ in range(op.n_steps):
        ws = w + dt * rate(w)
        ws[0], ws[-1] = ws[1], ws[-2]
        ws = ws + dt * rate(ws)
        w = 0.5 * (w + ws)
        w[0], w[-1] = w[1], w[-2]
    v = w[1:-1]
    return np.array([op.meas_scale * np.trapz(v[lo:hi], dx=op.meas_dx) for lo, hi in zip(op.win_lo, op.win_hi)])


@pytest.mark.parametrize("arith", ["fma", "reference"])
def test_viscous_burgers_is_the_central_difference_scheme(orc, arith):
    """The viscous extension (no reference exists): FMA arith folds nu/dx^2 into
    the Rusanov flux's wave-speed term, REFERENCE arith adds the central
    difference; both are the textbook scheme to rounding (1e-10 relative)."""
    from ip_mcmc_amd import BurgersOperator

    op = BurgersOperator(N=64, dt_mode="fixed", dt=2e-3, n_steps=300, nu=2e-3, arith=arith)
    for u in ([0.0, 0.0, 0.0], [0.05, -0.1, 0.2], [-0.2, 0.1, -0.3]):
        u = np.asarray(u)
        g = orc.forward(op, u[None, :])[0]
        want = _burgers_textbook(op, u)
        assert np.allclose(g, want, rtol=1e-10, atol=1e-12), (arith, u, g, want)
    inv = BurgersOperator(N=64, dt_mode="fixed", dt=2e-3, n_steps=300, nu=0.0, arith=arith)
    assert not np.allclose(orc.forward(inv, u[None, :])[0], want, rtol=1e-6)  # the viscous term matters here


def _l63_textbook(theta, x0, dt, n):
    """Classical RK4 Lorenz-63 in numpy float64, G = time averages of
    (x, y, z, x^2, y^2, z^2) over the n post-step states."""
    sg, rh, bb = theta

    def f(s):
        return np.array([sg * (s[1] - s[0]), s[0] * (rh - s[2]) - s[1], s[0] * s[1] - bb * s[2]])

    x = np.asarray(x0, dtype=np.float64).copy()
    ob = np.zeros(6)
    for _ in range(n):
        k1 = f(x)
        k2 = f(x + 0.5 * dt * k1)
        k3 = f(x + 0.5 * dt * k2)
        k4 = f(x + dt * k3)
        x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        ob += np.concatenate([x, x * x])
    return ob / n


@pytest.mark.parametrize("arith", ["fma", "reference"])
def test_lorenz63_oracle_is_textbook_rk4(orc, arith):
    """Lorenz-63 has no reference implementation: the oracle's G
    (both arithmetic modes) is classical RK4 to rounding over a horizon short
    enough that the chaos does not amplify it (1e-11 relative)."""
    from ip_mcmc_amd import Lorenz63Operator

    op = Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=150, arith=arith)
    for u in ([0.0, 0.0, 0.0], [0.5, -1.0, 0.1], [-1.0, 2.0, -0.2]):
        u = np.asarray(u)
        g = orc.forward(op, u[None, :])[0]
        want = _l63_textbook(op.theta0 + u, op.x0, op.dt, op.n_steps)
        assert np.allclose(g, want, rtol=1e-11, atol=1e-11), (arith, u, g - want)


@pytest.mark.parametrize("every", [1, 3, 7])
def test_oracle_in_launch_samples_equal_per_sample_sweeps(orc, every):
    """ipmc_sweep.sample_every (ABI 9): one sweep of n steps recording u after
    every `every` steps equals n/every sweeps of `every` steps each recording
    its final state (sampler.py:23-28), for the state, Φ and the counters."""
    from ip_mcmc_amd import Lorenz96Operator

    op = Lorenz96Operator(8, 8.0, dt=0.01, n_steps=30)
    rng = np.random.default_rng(4)
    y, ginv = op.x0 + 0.3 * rng.normal(size=8), np.full(8, 4.0)
    U0 = 0.2 * rng.normal(size=(5, 8))
    phi0 = orc.potential(op, U0, y, ginv)
    n = 21
    U1, P1, A1 = U0.copy(), phi0.copy(), np.zeros(5, dtype=np.int64)
    S1 = np.zeros((5, n // every, 8))
    orc.pcn_sweep(op, U1, P1, y, ginv, np.ones(8), 0.4, 9, 100, n, accepts=A1, samples=S1, sample_every=every)
    U2, P2, A2 = U0.copy(), phi0.copy(), np.zeros(5, dtype=np.int64)
    S2 = np.zeros((5, n // every, 8))
    for b in range(n // every):
        one = np.zeros((5, 1, 8))
        orc.pcn_sweep(op, U2, P2, y, ginv, np.ones(8), 0.4, 9, 100 + b * every, every, accepts=A2, samples=one)
        S2[:, b] = one[:, 0]
    rest = n - (n // every) * every
    if rest:
        orc.pcn_sweep(op, U2, P2, y, ginv, np.ones(8), 0.4, 9, 100 + n - rest, rest, accepts=A2)
    assert np.array_equal(S1, S2) and np.array_equal(U1, U2) and np.array_equal(P1, P2) and np.array_equal(A1, A2)
    assert A1.sum() > 0


def test_oracle_in_launch_samples_edge_cases(orc):
    """sample_every larger than the launch writes nothing; a launch that ends
    between samples leaves the rest of the buffer untouched."""
    from ip_mcmc_amd import LinearOperator

    op = LinearOperator(np.array([[1.0, 2.0, 0.5]]))
    U = np.zeros((3, 3))
    P = orc.potential(op, U, np.array([1.0]), np.array([2.0]))
    S = np.full((3, 4, 3), 7.0)
    orc.pcn_sweep(op, U, P, [1.0], [2.0], np.ones(3), 0.5, 1, 0, 5, samples=S, sample_every=9)
    assert np.all(S == 7.0)
    U2 = np.zeros((3, 3))
    P2 = orc.potential(op, U2, np.array([1.0]), np.array([2.0]))
    orc.pcn_sweep(op, U2, P2, [1.0], [2.0], np.ones(3), 0.5, 1, 0, 7, samples=S, sample_every=3)
    assert not np.all(S[:, :2] == 7.0) and np.all(S[:, 2:] == 7.0)  # samples after steps 3 and 6 only
    with pytest.raises(AssertionError):  # the C oracle rejects a negative sample_every
        orc.pcn_sweep(op, U2, P2, [1.0], [2.0], np.ones(3), 0.5, 1, 0, 7, samples=S, sample_every=-1)
