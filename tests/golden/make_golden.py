"""Generate the golden fixtures in tests/golden/ by running the REFERENCE.

Run in the build container only (needs /root/reference, which the GPU box
does not have):   python tests/golden/make_golden.py

Nothing of the reference is copied: this script imports its modules from
/root/reference, calls them, and stores inputs and outputs as .npz data.

Shims (all are name/compat fixes on the reference's own code):
  * ``ip_mcmc.pCNProposer`` is aliased to ``ConstSteppCNProposer`` so that
    report/scripts/lorenz.py (which imports the stale name) imports.
  * burgers/rusanov.py is imported directly; RusanovFVM.integrate uses the
    removed ``np.float`` (rusanov.py:32), so the harness sets the initial
    state itself and then drives the reference's own ``_cfl`` / ``_step``
    exactly as integrate does (rusanov.py:34-45).
  * burgers/utilities.py is NOT imported (it imports helpers.py, which needs
    the absent POT package); its Measurer formula (utilities.py:100-109,
    10 * np.trapz(values[l:r], dx)) is evaluated with numpy's own trapz.
The reference's RNG seam (test_utilities.py:11-26: a np.random.Generator
subclass) injects the build's counter-based draws into the reference sampler.
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "ip_mcmc"))
sys.path.insert(0, os.path.join(REF, "report", "scripts"))
sys.path.insert(0, os.path.join(REF, "report", "scripts", "burgers"))

import numpy as np  # noqa: E402

import matplotlib  # noqa: E402

matplotlib.use("Agg")

import ip_mcmc  # noqa: E402
from ip_mcmc import (  # noqa: E402
    ConstrainAccepter,
    ConstStepStandardRWProposer,
    ConstSteppCNProposer,
    StandardRWAccepter,
    VarStepStandardRWProposer,
    CountedAccepter,
    EvolutionPotential,
    GaussianDistribution,
    MCMCSampler,
    pCNAccepter,
)

ip_mcmc.pCNProposer = ConstSteppCNProposer  # stale name in lorenz.py:8
import lorenz  # noqa: E402  report/scripts/lorenz.py
import lorenz_mcmc  # noqa: E402  report/scripts/lorenz_mcmc.py (moment_function)
import rusanov  # noqa: E402  report/scripts/burgers/rusanov.py

from oracle import oracle as O  # noqa: E402  (draws only: Philox stream)


# --------------------------------------------------------------- injection
class CounterRNG(np.random.Generator):
    """The reference's MockRNG seam (test_utilities.py:11-26) fed with the
    build's counter-based draws: multivariate_normal returns sqrt(C)·ξ(step)
    and random() returns r(step) for one chain.  Each multivariate_normal call
    starts a new step (the proposal precedes the accept draw, sampler.py:36-38)."""

    def __init__(self, seed, chain, step0=0):
        super().__init__(np.random.PCG64())
        self.s = seed
        self.chain = chain
        self.step = step0 - 1
        self.uniform_steps = []

    def multivariate_normal(self, mean=None, cov=None):
        self.step += 1
        k = len(mean)
        xi = O.normals(self.s, self.chain, 1, self.step, k)[0]
        cov = np.asarray(cov)
        if np.all(cov == np.diag(np.diag(cov))):
            return np.sqrt(np.diag(cov)) * xi + mean
        # a non-diagonal covariance: L·ξ with L = cholesky(C), summed in the
        # device's order (include/ipmc.h prior_chol: ascending i from +0)
        L = np.linalg.cholesky(cov)
        w = np.zeros(k)
        for j in range(k):
            acc = 0.0
            for i in range(j + 1):
                acc = acc + float(xi[i]) * float(L[j, i])
            w[j] = acc
        return w + mean

    def random(self):
        self.uniform_steps.append(self.step)
        return float(O.uniforms(self.s, self.chain, 1, self.step)[0])


class RecordingAccepter:
    """Wraps the reference accepter and records the decision of every step."""

    def __init__(self, inner):
        self.inner = inner
        self.decisions = []

    def __call__(self, u, v, rng):
        a = self.inner(u, v, rng)
        self.decisions.append(bool(a))
        return a


def run_reference_chain(G, y, noise_cov_diag, prior_var_diag, beta, u0, seed, chain, n_samples, burn_in, interval,
                        box=None, proposer=None, rw_accept=False, prior_cov=None):
    cov = np.diag(prior_var_diag) if prior_cov is None else np.asarray(prior_cov)
    prior = GaussianDistribution(mean=np.zeros(len(u0)), covariance=cov)
    noise = GaussianDistribution(mean=np.zeros(len(y)), covariance=np.diag(noise_cov_diag))
    pot = EvolutionPotential(G, y, noise)
    prop = ConstSteppCNProposer(beta, prior) if proposer is None else proposer(prior)
    inner = CountedAccepter(StandardRWAccepter(pot, prior) if rw_accept else pCNAccepter(pot))
    rec = RecordingAccepter(inner)
    acc = rec if box is None else ConstrainAccepter(rec, box)
    rng = CounterRNG(seed, chain)
    sampler = MCMCSampler(prop, acc, rng)
    import contextlib
    import io

    with contextlib.redirect_stdout(io.StringIO()):
        samples = sampler.run(np.asarray(u0, dtype=float), n_samples=n_samples, burn_in=burn_in,
                              sample_interval=interval)
    return samples, rec.decisions, rng.step + 1, inner.calls, inner.accepts


# ------------------------------------------------------------ Lorenz-96
def l96_ref_rhs(K, F):
    """The reference RHS object: Lorenz96(K, J=0, F, h, c, b) (lorenz.py:13-111)."""
    f = lorenz.Lorenz96(K, 0, F, 0.0, 0.0, 0.0)
    return lambda x: f(0.0, x)


def rk4_time_average(f, x0, dt, n):
    """Classical RK4 + time average in the build's contract order (DESIGN.md §4,
    REFERENCE arith), with the reference's RHS object as f."""
    x = np.array(x0, dtype=np.float64)
    h, h2, h6 = dt, dt * 0.5, dt / 6.0
    ob = np.zeros_like(x)
    for _ in range(n):
        k1 = f(x)
        k2 = f(x + h2 * k1)
        k3 = f(x + h2 * k2)
        k4 = f(x + h * k3)
        x = x + h6 * (((k1 + 2.0 * k2) + 2.0 * k3) + k4)
        ob = ob + x
    return ob / float(n)


def make_l96(out):
    rng = np.random.default_rng(1234)
    # RHS vectors: K=40 single scale, per-component forcing
    X = rng.normal(0, 4, size=(64, 40))
    F = 8.0 + rng.normal(0, 1, size=(64, 40))
    R = np.stack([l96_ref_rhs(40, F[i])(X[i]) for i in range(64)])
    # small-K cases incl. the edge K=4
    X4 = rng.normal(0, 3, size=(16, 4))
    F4 = rng.normal(8, 1, size=(16, 4))
    R4 = np.stack([l96_ref_rhs(4, F4[i])(X4[i]) for i in range(16)])
    # test_Lorenz96 known answers (lorenz.py:114-171), evaluated by the reference
    kat = {
        "forcing": (lorenz.Lorenz96(3, 1, 2, 1, 1, 1), [0, 0, 0, 0, 0, 0]),
        "slow_nonlinearity": (lorenz.Lorenz96(4, 1, 0, 0, 0, 0), [1, 2, 3, 4, 0, 0, 0, 0]),
        "fast_nonlinearity": (lorenz.Lorenz96(1, 4, 0, 0, 1, 2), [0, 1, 2, 3, 4]),
        "step": (lorenz.Lorenz96(2, 2, 1, 1, 1, 1), [2, 3, 4, 5, 6, 7]),
    }
    for name, (obj, x) in kat.items():
        out[f"l96_kat_{name}_in"] = np.asarray(x, dtype=float)
        out[f"l96_kat_{name}_out"] = obj(1, np.asarray(x, dtype=float))
    out["l96_rhs_x"], out["l96_rhs_F"], out["l96_rhs_out"] = X, F, R
    out["l96_rhs4_x"], out["l96_rhs4_F"], out["l96_rhs4_out"] = X4, F4, R4

    # Time-averaged RK4 forward map G with the reference RHS (K=40 and K=8)
    for K, n, dt in ((40, 200, 0.005), (8, 300, 0.01)):
        fm = np.full(K, 8.0)
        x0 = 8.0 + rng.normal(0, 1, size=K)
        U = rng.normal(0, 1, size=(6, K))
        G = np.stack([rk4_time_average(l96_ref_rhs(K, fm + U[i]), x0, dt, n) for i in range(6)])
        out[f"l96_G{K}_x0"], out[f"l96_G{K}_u"], out[f"l96_G{K}_G"] = x0, U, G
        out[f"l96_G{K}_meta"] = np.array([n, dt])


def make_l96_chain(out):
    """pCN chains on Lorenz-96 K=8 through the reference sampler."""
    K, n, dt = 8, 100, 0.01
    rng = np.random.default_rng(99)
    fm = np.full(K, 8.0)
    x0 = 8.0 + rng.normal(0, 1, size=K)
    utrue = 0.5 * rng.normal(size=K)
    y = rk4_time_average(l96_ref_rhs(K, fm + utrue), x0, dt, n) + 0.05 * rng.normal(size=K)
    gamma = 0.1
    seed = 0x1234ABCD
    chains = []
    for chain in range(3):
        def G(u):
            return rk4_time_average(l96_ref_rhs(K, fm + u), x0, dt, n)

        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, np.full(K, gamma**2), np.ones(K), 0.3, np.zeros(K), seed, chain, n_samples=6, burn_in=20,
            interval=10)
        chains.append((s, dec))
    out["l96c_x0"], out["l96c_y"] = x0, y
    out["l96c_meta"] = np.array([K, n, dt, gamma, 0.3, seed, 6, 20, 10], dtype=np.float64)
    out["l96c_samples"] = np.stack([c[0] for c in chains])
    out["l96c_decisions"] = np.stack([np.array(c[1]) for c in chains])


# ------------------------------------------------- two-scale Lorenz-96
def l96ts_G(K, J, theta, c, x0, dt, n):
    """Two-scale G: RK4 (contract order, as rk4_time_average) with the
    reference RHS object Lorenz96(K, J, F, h, c, b), the post-step states fed
    to the reference moment_function (lorenz_mcmc.py:17-40), and its columns
    time-averaged in step order (the build's accumulation contract)."""
    F, h, b = theta
    obj = lorenz.Lorenz96(K, J, F, h, c, b)
    x = np.array(x0, dtype=np.float64)
    hh, h2, h6 = dt, dt * 0.5, dt / 6.0
    traj = np.empty((x.size, n))
    for t in range(n):
        k1 = obj(0.0, x)
        k2 = obj(0.0, x + h2 * k1)
        k3 = obj(0.0, x + h2 * k2)
        k4 = obj(0.0, x + hh * k3)
        x = x + h6 * (((k1 + 2.0 * k2) + 2.0 * k3) + k4)
        traj[:, t] = x
    f = lorenz_mcmc.moment_function(traj, K, J)
    ob = np.zeros(5 * K)
    for t in range(n):
        ob = ob + f[:, t]
    return ob / float(n)


def make_l96ts(out):
    rng = np.random.default_rng(4321)
    # RHS of the reference object on random states, (K, J) incl. J = 1 and 16
    for K, J in ((6, 4), (5, 8), (4, 10), (3, 1), (7, 16), (2, 2)):
        n = 8
        X = rng.normal(0, 3, size=(n, K * (1 + J)))
        P = np.stack([rng.normal(10, 2, size=n), rng.normal(5, 2, size=n), rng.uniform(0.5, 10, size=n),
                      rng.normal(8, 2, size=n)], axis=1)  # F, h, c, b
        R = np.stack([lorenz.Lorenz96(K, J, *P[i])(0.0, X[i]) for i in range(n)])
        out[f"ts_rhs_{K}_{J}_x"], out[f"ts_rhs_{K}_{J}_p"], out[f"ts_rhs_{K}_{J}_out"] = X, P, R
    # moment_function on a random trajectory (reference, incl. its Ybar = Y_{k,0})
    Y = rng.normal(0, 2, size=(6 * 5, 11))
    out["ts_mom_y"], out["ts_mom_f"] = Y, lorenz_mcmc.moment_function(Y, 6, 4)
    # G: K=6 J=4 (the thesis's problem), K=4 J=8, K=3 J=1
    for K, J, n, dt in ((6, 4, 60, 0.005), (4, 8, 40, 0.004), (3, 1, 50, 0.01)):
        x0 = rng.normal(0, 1, size=K * (1 + J))
        th0 = np.array([12.0, 8.0, 9.0])
        U = rng.normal(0, 0.5, size=(4, 3))
        G = np.stack([l96ts_G(K, J, th0 + U[i], 1.0, x0, dt, n) for i in range(4)])
        out[f"ts_G{K}_{J}_x0"], out[f"ts_G{K}_{J}_u"], out[f"ts_G{K}_{J}_G"] = x0, U, G
        out[f"ts_G{K}_{J}_meta"] = np.array([n, dt, 1.0])
    # pCN chains through the reference sampler, K=4 J=4
    K, J, n, dt, c = 4, 4, 30, 0.005, 1.0
    x0 = rng.normal(0, 1, size=K * (1 + J))
    th0 = np.array([12.0, 8.0, 9.0])
    y = l96ts_G(K, J, th0 + np.array([-1.0, 1.0, 0.5]), c, x0, dt, n) + 0.05 * rng.normal(size=5 * K)
    gamma, beta, seed = 0.2, 0.4, 0x5EED2
    chains = []
    for chain in range(2):
        def G(u):
            return l96ts_G(K, J, th0 + u, c, x0, dt, n)

        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, np.full(5 * K, gamma**2), np.array([10.0, 1.0, 10.0]), beta, np.zeros(3), seed, chain,
            n_samples=4, burn_in=6, interval=3)
        chains.append((s, dec))
    out["tsc_x0"], out["tsc_y"] = x0, y
    out["tsc_meta"] = np.array([K, J, n, dt, c, gamma, beta, seed, 4, 6, 3], dtype=np.float64)
    out["tsc_samples"] = np.stack([ch[0] for ch in chains])
    out["tsc_decisions"] = np.stack([np.array(ch[1]) for ch in chains])


# -------------------------------------------------------- linear Gaussian
def make_linear(out):
    """Config 1: G(u)=<g,u>, g=[3,1,4,1], u*=[2,7,1,8], γ=0.5,
    prior N(0, I4), β=0.5, through the reference sampler with injected draws."""
    g = np.array([3.0, 1.0, 4.0, 1.0])
    ustar = np.array([2.0, 7.0, 1.0, 8.0])
    gamma = 0.5
    rng = np.random.default_rng(1)
    y = np.array([np.dot(g, ustar) + gamma * rng.normal()])
    seed = 20240501

    def G(u):
        return np.dot(g, u)  # stuart_examples.py:69-70

    res = []
    for chain in range(4):
        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, np.array([gamma**2]), np.ones(4), 0.5, np.zeros(4), seed, chain, n_samples=40, burn_in=100,
            interval=20)
        res.append((s, dec, calls, accepts))
    out["lin_g"], out["lin_y"] = g, y
    out["lin_meta"] = np.array([gamma, 0.5, seed, 40, 100, 20], dtype=np.float64)
    out["lin_samples"] = np.stack([r[0] for r in res])
    out["lin_decisions"] = np.stack([np.array(r[1]) for r in res])
    out["lin_counts"] = np.array([[r[2], r[3]] for r in res])
    # EvolutionPotential values (potential.py:53-54) on random points: pins Φ up to its constant
    U = np.random.default_rng(5).normal(size=(20, 4)) * 2
    noise = GaussianDistribution(mean=np.zeros(1), covariance=np.array([[gamma**2]]))
    pot = EvolutionPotential(G, y, noise)
    out["lin_phi_u"] = U
    out["lin_phi"] = np.array([pot(u) for u in U])


def make_constrained(out):
    """ConstrainAccepter (accepter.py:39-55) around CountedAccepter(pCNAccepter)
    through the reference sampler: a proposal the constraint rejects never
    reaches the inner accepter (no call counted, no uniform drawn).  The
    constraint is a strict box on two components, like is_valid_IC
    (burgers_wasserstein_chain.py:47-55)."""
    g = np.array([3.0, 1.0, 4.0, 1.0])
    gamma = 0.5
    y = np.array([np.dot(g, [2.0, 7.0, 1.0, 8.0]) + 0.1])
    lo = np.array([-0.6, -np.inf, -1.0, -np.inf])
    hi = np.array([0.6, np.inf, 1.0, np.inf])
    seed = 4242

    def is_valid(v):
        return bool(np.all(lo < v) and np.all(v < hi))

    def G(u):
        return np.dot(g, u)

    res = []
    for chain in range(3):
        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, np.array([gamma**2]), np.ones(4), 0.5, np.zeros(4), seed, chain, n_samples=30, burn_in=60,
            interval=10, box=is_valid)
        res.append((s, calls, accepts))
    out["con_g"], out["con_y"], out["con_lo"], out["con_hi"] = g, y, lo, hi
    out["con_meta"] = np.array([gamma, 0.5, seed, 30, 60, 10], dtype=np.float64)
    out["con_samples"] = np.stack([r[0] for r in res])
    out["con_counts"] = np.array([[r[1], r[2]] for r in res])


def pw_linear(d_s, d_e, l):
    """The harness's step schedule, the formula of burgers_beta.py:131-147's PWLinear
    (that script cannot be imported here: it pulls in helpers.py, which needs POT)."""
    slope = (d_s - d_e) / l
    return lambda i: d_e if i > l else d_s - slope * i


def make_rw(out):
    """Random-walk chains (proposer.py:14-56 + accepter.py:86-106, the §8(f) #1
    composition of burgers_beta.py:104-128) through the reference sampler."""
    g = np.array([3.0, 1.0, 4.0, 1.0])
    gamma = 0.5
    y = np.array([np.dot(g, [2.0, 7.0, 1.0, 8.0]) + 0.2])
    prior_var = np.array([0.5, 2.0, 1.0, 1.5])
    seed = 777

    def G(u):
        return np.dot(g, u)

    cases = {
        "const": lambda prior: ConstStepStandardRWProposer(0.05, prior),
        "var": lambda prior: VarStepStandardRWProposer(pw_linear(0.1, 0.001, 60), prior),
    }
    for name, mk in cases.items():
        res = []
        for chain in range(3):
            s, dec, steps, calls, accepts = run_reference_chain(
                G, y, np.array([gamma**2]), prior_var, None, np.zeros(4), seed, chain, n_samples=20, burn_in=60,
                interval=10, proposer=mk, rw_accept=True)
            res.append((s, calls, accepts))
        out[f"rw_{name}_samples"] = np.stack([r[0] for r in res])
        out[f"rw_{name}_counts"] = np.array([[r[1], r[2]] for r in res])
    out["rw_g"], out["rw_y"], out["rw_prior_var"] = g, y, prior_var
    out["rw_meta"] = np.array([gamma, seed, 20, 60, 10, 0.05, 0.1, 0.001, 60], dtype=np.float64)
    # StandardRWAccepter._I values (accepter.py:104-106) on random points
    prior = GaussianDistribution(np.zeros(4), np.diag(prior_var))
    acc = StandardRWAccepter(EvolutionPotential(G, y, GaussianDistribution(0, gamma**2)), prior)
    U = np.random.default_rng(8).normal(size=(12, 4))
    out["rw_I_u"] = U
    out["rw_I"] = np.array([acc._I(u) for u in U])


# ---------------------------------------------------------------- Burgers
def burgers_flux(w):
    return 0.5 * w * w  # utilities.py:114-115 (BurgersEquation.flux)


def burgers_flux_prime(w):
    return w


def ref_integrate(N, domain, theta, T):
    """RusanovFVM.integrate (rusanov.py:31-60) of the reference, driven
    step by step (its np.float line replaced by the same values computed here)."""
    r = rusanov.RusanovFVM(burgers_flux, burgers_flux_prime, domain, N)
    left, right, jump = 1 + theta[0], theta[1], theta[2]  # PerturbedRiemannIC, utilities.py:55-62
    r.u[:] = np.array([left if x_ < jump else right for x_ in r.x], dtype=float)
    t = 0
    steps = 0
    while t < T:  # rusanov.py:40-45
        dt = r._cfl()
        t += dt
        r._step(dt)
        steps += 1
    return np.copy(r.u[1:-1]), t, steps, r.x, r.dx


def make_burgers(out):
    r = rusanov.RusanovFVM(burgers_flux, burgers_flux_prime, (0, 1), 10)
    out["rus_kat_flux_in"] = np.array([[1, 1], [0, 1], [0, -1], [4, 5]], dtype=float)
    out["rus_kat_flux_out"] = np.array([r._flux(a, b) for a, b in out["rus_kat_flux_in"]])
    r3 = rusanov.RusanovFVM(burgers_flux, burgers_flux_prime, (0, 0.3), 3)
    u = np.array([1, 1, -1, 2, 2], dtype=float)
    r3._rate_of_change(u, 0.1)
    out["rus_kat_rate_in"] = u
    out["rus_kat_rate_dx"] = np.array([r3.dx])
    out["rus_kat_rate_out"] = r3.dudt[1:-1].copy()
    rng = np.random.default_rng(7)
    wr = rng.normal(1, 1, size=66)
    rr = rusanov.RusanovFVM(burgers_flux, burgers_flux_prime, (-1, 1), 64)
    rr._rate_of_change(wr, 0.01)
    out["rus_rate_w"], out["rus_rate_dx"], out["rus_rate_out"] = wr, np.array([rr.dx]), rr.dudt[1:-1].copy()

    prior_mean = np.array([1.5, 0.25, -0.5])  # burgers_beta.py:64-67
    points = np.array([-0.5, -0.25, 0.25, 0.5, 0.75])
    interval = 0.1
    for N in (32, 128, 256):
        thetas = prior_mean + 0.25 * rng.normal(size=(4, 3))
        thetas[0] = prior_mean
        finals, ts, steps, meas = [], [], [], []
        for th in thetas:
            w, t, n, x, dx = ref_integrate(N, (-1, 1), th, 1.0)
            xv = x[1:-1]
            lo = np.searchsorted(xv, points - interval / 2, side="left")
            hi = np.searchsorted(xv, points + interval / 2, side="left")
            mdx = xv[1] - xv[0]
            m = np.array([10 * np.trapz(w[a:b], dx=mdx) for a, b in zip(lo, hi)])  # utilities.py:100-109
            finals.append(w)
            ts.append(t)
            steps.append(n)
            meas.append(m)
        out[f"bur{N}_theta"] = thetas
        out[f"bur{N}_final"] = np.stack(finals)
        out[f"bur{N}_t"] = np.array(ts)
        out[f"bur{N}_steps"] = np.array(steps)
        out[f"bur{N}_G"] = np.stack(meas)
        out[f"bur{N}_x"], out[f"bur{N}_dx"] = x, np.array([dx])
        out[f"bur{N}_win"] = np.stack([lo, hi])


def make_burgers_chain(out):
    """Burgers chains through the reference sampler (burgers_beta.py:25-128's
    study at N=32): G = Measurer(RusanovFVM.integrate(PerturbedRiemannIC(
    prior_mean + u))), data = G at the ground truth (burgers_beta.py:116,
    no noise added), noise γ = 0.05, prior N(0, 0.25²).  Two compositions:
    pCN (β = 0.15, burgers.org:222-231) and the study's own RW path,
    VarStepStandardRWProposer(PWLinear) + CountedAccepter(StandardRWAccepter)
    inside ConstrainAccepter(is_valid_IC) (burgers_wasserstein_chain.py:47-55)."""
    N = 32
    prior_mean = np.array([1.5, 0.25, -0.5])  # burgers_beta.py:64-67
    truth = np.array([0.025, -0.025, -0.02])  # burgers_beta.py:31-35
    points = np.array([-0.5, -0.25, 0.25, 0.5, 0.75])
    interval, gamma, sigma_p = 0.1, 0.05, 0.25

    def measure(theta):
        w, t, n, x, dx = ref_integrate(N, (-1, 1), theta, 1.0)
        xv = x[1:-1]
        lo = np.searchsorted(xv, points - interval / 2, side="left")
        hi = np.searchsorted(xv, points + interval / 2, side="left")
        return np.array([10 * np.trapz(w[a:b], dx=xv[1] - xv[0]) for a, b in zip(lo, hi)])  # utilities.py:100-109

    def G(u):  # FVMObservationOperator (utilities.py:17-41): evaluated at prior_mean + u
        return measure(prior_mean + u)

    y = measure(truth)

    def is_valid_IC(u):  # burgers_wasserstein_chain.py:47-55
        s = u[2] + prior_mean[2]
        return bool(-1 < s < 1)

    seed = 2024
    noise = np.full(5, gamma**2)
    prior_var = np.full(3, sigma_p**2)
    res = []
    for chain in range(3):
        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, noise, prior_var, 0.15, np.zeros(3), seed, chain, n_samples=5, burn_in=10, interval=4)
        res.append((s, calls, accepts))
    out["bch_pcn_samples"] = np.stack([r[0] for r in res])
    out["bch_pcn_counts"] = np.array([[r[1], r[2]] for r in res])
    res = []
    for chain in range(3):
        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, noise, prior_var, None, np.zeros(3), seed + 1, chain, n_samples=5, burn_in=10, interval=4,
            box=is_valid_IC, proposer=lambda prior: VarStepStandardRWProposer(pw_linear(0.1, 0.01, 10), prior),
            rw_accept=True)
        res.append((s, calls, accepts))
    out["bch_rw_samples"] = np.stack([r[0] for r in res])
    out["bch_rw_counts"] = np.array([[r[1], r[2]] for r in res])
    out["bch_y"], out["bch_prior_mean"] = y, prior_mean
    # N, gamma, sigma_p, beta, seed, n_samples, burn_in, interval, PWLinear (d_s, d_e, l)
    out["bch_meta"] = np.array([N, gamma, sigma_p, 0.15, seed, 5, 10, 4, 0.1, 0.01, 10], dtype=np.float64)


def make_dense_prior(out):
    """pCN with a NON-diagonal prior covariance through the reference sampler
    (proposer.py:59-82: w ~ N(0, C) drawn by GaussianDistribution.sample,
    distribution.py:114-118), the draws injected as L·ξ: the linear problem of
    config 1 with an AR(1) prior, and the Lorenz-96 K=8 chain problem with a
    periodic squared-exponential prior on the forcing field.

    Parity scope: the reference draws w ~ N(0, C) through numpy's SVD-based
    multivariate_normal; this harness substitutes L·ξ (L = cholesky(C), the
    build's own draw, summed in the device's order).  These fixtures therefore
    pin the reference's proposal arithmetic, accept rule and bookkeeping for a
    non-diagonal prior, but NOT its sampling path: for the draws themselves
    parity with the reference is distributional only ("parity unpinned" bit
    for bit; tests/test_gpu_hostloop.py checks the device's L·ξ covariance
    against C within Monte-Carlo error)."""
    g = np.array([3.0, 1.0, 4.0, 1.0])
    gamma = 0.5
    y = np.array([np.dot(g, [2.0, 7.0, 1.0, 8.0]) + 0.3])
    idx = np.arange(4)
    cov = 0.8 ** np.abs(idx[:, None] - idx[None, :])
    seed = 5150

    def G(u):
        return np.dot(g, u)

    res = []
    for chain in range(3):
        s, dec, steps, calls, accepts = run_reference_chain(
            G, y, np.array([gamma**2]), None, 0.5, np.zeros(4), seed, chain, n_samples=30, burn_in=60, interval=10,
            prior_cov=cov)
        res.append((s, accepts))
    out["dpl_cov"], out["dpl_g"], out["dpl_y"] = cov, g, y
    out["dpl_meta"] = np.array([gamma, 0.5, seed, 30, 60, 10], dtype=np.float64)
    out["dpl_samples"] = np.stack([r[0] for r in res])
    out["dpl_accepts"] = np.array([r[1] for r in res])

    K, n, dt = 8, 100, 0.01
    x0, y96 = out["l96c_x0"], out["l96c_y"]
    d = np.abs(np.arange(K)[:, None] - np.arange(K)[None, :])
    d = np.minimum(d, K - d)
    cov96 = np.exp(-0.5 * (d / 1.2) ** 2) + 0.05 * np.eye(K)
    fm = np.full(K, 8.0)
    seed96 = 0x5EED
    res = []
    for chain in range(3):
        def G96(u):
            return rk4_time_average(l96_ref_rhs(K, fm + u), x0, dt, n)

        s, dec, steps, calls, accepts = run_reference_chain(
            G96, y96, np.full(K, 0.1**2), None, 0.3, np.zeros(K), seed96, chain, n_samples=6, burn_in=20, interval=10,
            prior_cov=cov96)
        res.append((s, accepts))
    out["dp96_cov"] = cov96
    out["dp96_meta"] = np.array([K, n, dt, 0.1, 0.3, seed96, 6, 20, 10], dtype=np.float64)
    out["dp96_samples"] = np.stack([r[0] for r in res])
    out["dp96_accepts"] = np.array([r[1] for r in res])


# ----------------------------------------------- distributions & schedule
def make_misc(out):
    g = GaussianDistribution(mean=np.array([1.0, -2.0, 0.5]), covariance=np.diag([0.5, 2.0, 1.5]))
    X = np.random.default_rng(3).normal(size=(10, 3)) * 2
    out["gauss_x"] = X
    out["gauss_logpdf"] = np.array([g.logpdf(x) for x in X])
    gf = GaussianDistribution(mean=np.array([0.0, 1.0]), covariance=np.array([[2.0, 0.5], [0.5, 1.0]]))
    out["gaussfull_x"] = X[:, :2]
    out["gaussfull_logpdf"] = np.array([gf.logpdf(x) for x in X[:, :2]])
    # step-count arithmetic of MCMCSampler.run (sampler.py:18-26)
    from ip_mcmc.test_utilities import MockProposer, MockRNG
    from ip_mcmc import AnalyticAccepter
    import contextlib
    import io

    rows = []
    for b, n, s in ((100, 10, 20), (0, 5, 3), (50, 4, 50), (10, 3, 20), (1000, 2, 200)):
        a = CountedAccepter(AnalyticAccepter(lambda x: x))
        smp = MCMCSampler(MockProposer(), a, MockRNG(0.1))
        with contextlib.redirect_stdout(io.StringIO()):
            smp.run(np.array([1.0]), n_samples=n, burn_in=b, sample_interval=s)
        rows.append([b, n, s, a.calls])
    out["schedule"] = np.array(rows)
    # MCMCSampler.autocorr (sampler.py:43-54) on random-walk series and a constant one
    xs = np.random.default_rng(11).normal(size=(6, 120)).cumsum(axis=1)
    xs[5] = 3.0
    out["ac_x"] = xs
    out["ac_ref"] = np.stack([MCMCSampler.autocorr(x) for x in xs])


def _reference_functions(path, names, namespace):
    """Execute the named top-level function definitions of a reference script
    (helpers.py / burgers/utilities.py import the absent POT package at module
    level, so the module itself cannot be imported; the functions used here
    need only numpy and MCMCSampler)."""
    import ast

    tree = ast.parse(open(path).read(), filename=path)
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert sorted(n.name for n in body) == sorted(names)
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), namespace)
    return namespace


def _synthetic_chain(rng, n_vars, n):
    """An MCMC-like trace: exponential relaxation from a far start onto a
    stationary AR(1) around a mean (burn-in, then correlated noise)."""
    mean = rng.uniform(0.2, 2, size=n_vars) * rng.choice([-1, 1], size=n_vars)
    start = mean + rng.uniform(-3, 3, size=n_vars)
    tau = rng.uniform(5, n / 3)
    sig = 10 ** rng.uniform(-2.5, 0.3)
    phi = rng.uniform(0.5, 0.995)
    x = np.empty((n_vars, n))
    e = np.zeros(n_vars)
    for t in range(n):
        e = phi * e + sig * rng.normal(size=n_vars)
        x[:, t] = mean + (start - mean) * np.exp(-t / tau) + e
    return x


def make_burn_in(out):
    """len_burn_in / uncorrelated_sample_spacing / clean_samples
    (burgers/utilities.py:134-195) on synthetic traces."""
    ns = {"np": np, "MCMCSampler": MCMCSampler}
    _reference_functions(os.path.join(REF, "report", "scripts", "helpers.py"), ["autocorrelation"], ns)
    _reference_functions(os.path.join(REF, "report", "scripts", "burgers", "utilities.py"),
                         ["len_burn_in", "uncorrelated_sample_spacing", "clean_samples"], ns)
    rng = np.random.default_rng(77)
    sizes = [50, 51, 100, 153, 400, 1000, 1500, 3000]
    i = 0
    for n in sizes:
        for n_vars in (1, 3):
            x = np.ascontiguousarray(_synthetic_chain(rng, n_vars, n))
            out[f"bi_x_{i}"] = x
            out[f"bi_out_{i}"] = np.array(ns["len_burn_in"](x))
            i += 1
    # a chain whose moving average keeps changing (tiny mean) and a flat one
    x = np.ascontiguousarray(np.stack([np.linspace(0, 1, 700), 1e-3 * rng.normal(size=700)]))
    out[f"bi_x_{i}"], out[f"bi_out_{i}"] = x, np.array(ns["len_burn_in"](x))
    i += 1
    x = np.ones((2, 300))
    out[f"bi_x_{i}"], out[f"bi_out_{i}"] = x, np.array(ns["len_burn_in"](x))
    out["bi_count"] = np.array(i + 1)
    # batch: 40 chains of 3 variables x 1200 samples
    B = np.stack([_synthetic_chain(rng, 3, 1200) for _ in range(40)])
    out["bi_batch_x"] = B
    out["bi_batch_out"] = np.array([ns["len_burn_in"](np.ascontiguousarray(b)) for b in B])
    # decorrelation spacing and the cleaned samples
    for j, n in enumerate((400, 2000, 5000)):
        x = np.ascontiguousarray(_synthetic_chain(rng, 3, n))
        out[f"us_x_{j}"] = x
        out[f"us_out_{j}"] = np.array(ns["uncorrelated_sample_spacing"](x))
        out[f"cs_out_{j}"] = ns["clean_samples"](x)


def main():
    path = os.path.join(HERE, "reference_golden.npz")
    if sys.argv[1:]:
        # regenerate only the named groups, keeping the other arrays of the file
        z = np.load(path, allow_pickle=False)
        out = {k: z[k] for k in z.files}
        for name in sys.argv[1:]:
            globals()[f"make_{name}"](out)
        np.savez_compressed(path, **out)
        print(f"updated {path} ({', '.join(sys.argv[1:])}): {len(out)} arrays, {os.path.getsize(path)} bytes")
        return
    out = {}
    make_l96(out)
    make_l96_chain(out)
    make_l96ts(out)
    make_linear(out)
    make_constrained(out)
    make_rw(out)
    make_burgers(out)
    make_misc(out)
    make_burn_in(out)
    make_burgers_chain(out)
    make_dense_prior(out)
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
