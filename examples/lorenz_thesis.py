"""The reference's two-scale Lorenz-96 experiment (report/scripts/lorenz_mcmc.py:81-170)
on the GPU, with many chains instead of one.

Same problem: K=6 slow and J=4 fast variables per slow one, true theta =
(F, h, c, b) = (10, 10, 1, 10); data = time averages of the moment function
[X, Ȳ, X², XȲ, Ȳ²] over a long truth run, noise Γ = r²·diag(their variances)
with r = 0.5; prior N((12, 8, 9), diag(10, 1, 10)) on (F, h, b); pCN β = 0.5,
u_0 = (-1.9, 1.9, 0.9), 2 000 samples after a burn-in of 100, sample interval 1;
G integrates T = 20 from the truth run's end state.  Differences (DESIGN.md
§3): classical RK4 (dt 0.005) instead of solve_ivp's RK45, a stateless G, and
the truth run is a host RK4 run of T = 100 instead of T = 500.

  python examples/lorenz_thesis.py [chains]

Prints one JSON line: posterior means and standard deviations of (F, h, b)
over all chains and samples, the accept rate, the integrated autocorrelation
of F (the reference's windowed average, helpers.autocorrelation), wall time.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, TwoScaleLorenz96Operator, pCNAccepter)
from ip_mcmc_amd.diagnostics import autocorrelation  # noqa: E402


def moment_function(traj, K, J):
    """lorenz_mcmc.py:17-40 on a (K(1+J), T) trajectory: rows [X, Ȳ, X², XȲ, Ȳ²],
    Ȳ_k = Y_{k,0} as the reference computes it."""
    X = traj[:K]
    Yb = traj[K::J][:K]
    return np.concatenate([X, Yb, X * X, X * Yb, Yb * Yb])


def truth_run(K, J, theta, dt, n, seed=1):
    F, h, c, b = theta
    x = np.random.default_rng(seed).random((J + 1) * K)  # lorenz_mcmc.py:76-79
    rhs = TwoScaleLorenz96Operator.rhs
    traj = np.empty((x.size, n))
    for t in range(n):
        k1 = rhs(x, K, J, F, h, c, b)
        k2 = rhs(x + 0.5 * dt * k1, K, J, F, h, c, b)
        k3 = rhs(x + 0.5 * dt * k2, K, J, F, h, c, b)
        k4 = rhs(x + dt * k3, K, J, F, h, c, b)
        x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        traj[:, t] = x
    return traj


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    K, J, dt = 6, 4, 0.005
    theta = np.array([10.0, 10.0, 1.0, 10.0])  # F, h, c, b
    r = 0.5
    traj = truth_run(K, J, theta, dt, 20000)  # T = 100
    mf = moment_function(traj[:, 2000:], K, J)  # drop the first T = 10 as transient
    y, var = mf.mean(axis=1), mf.var(axis=1)
    noise = GaussianDistribution(np.zeros_like(var), r**2 * np.diag(var))
    prior_means = np.array([12.0, 8.0, 9.0])
    prior = GaussianDistribution(np.zeros(3), np.diag([10.0, 1.0, 10.0]))
    G = TwoScaleLorenz96Operator(K, J, prior_means=prior_means, c=theta[2], x0=traj[:, -1], dt=dt,
                                 n_steps=int(round(20 / dt)))
    acc = CountedAccepter(pCNAccepter(EvolutionPotential(G, y, noise)))
    sampler = MCMCSampler(ConstSteppCNProposer(0.5, prior), acc, np.random.default_rng(1))
    u0 = np.tile([-1.9, 1.9, 0.9], (chains, 1))
    t0 = time.perf_counter()
    samples = sampler.run(u0, n_samples=2000, burn_in=100, sample_interval=1)  # (C, 2000, 3)
    wall = time.perf_counter() - t0
    post = samples + prior_means
    ac = autocorrelation(post[0].T, 100)  # the reference's windowed average, chain 0
    rec = {
        "problem": "two-scale Lorenz-96 K=6 J=4, lorenz_mcmc.py settings",
        "chains": chains,
        "pcn_steps_per_chain": 2000 + 99,
        "posterior_mean_F_h_b": post.reshape(-1, 3).mean(axis=0).tolist(),
        "posterior_std_F_h_b": post.reshape(-1, 3).std(axis=0).tolist(),
        "truth_F_h_b": [theta[0], theta[1], theta[3]],
        "accept_rate": float(np.mean(acc.ratio())),
        "autocorr_F_lag10_chain0": float(ac[0, 10]),
        "wall_s": wall,
        "pcn_steps_per_s": chains * 2099 / wall,
    }
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
