"""fp32 vs fp64 tolerance sweep (BASELINE config 5: Lorenz-96 d=256).

  python tools/precision_sweep.py [chains] [n_samples]

For Lorenz-96 d=256 with 10 000 RK4 steps per G (config 5) and shorter
integrations, runs the same chains (same Philox draws, same u_0) through
MCMCSampler in float64 and float32 (keep='moments') and reports, per
integration length n:
  * the accept rate in each precision;
  * the fraction of chains whose accept COUNT is identical in both (per-chain
    agreement: rounding differences are amplified by the chaotic forward map);
  * the posterior means' agreement in Monte-Carlo standard errors:
    z_i = |m32_i - m64_i| / sqrt(se32_i^2 + se64_i^2) over the d parameters
    (se = between-chain standard deviation of the chain means / sqrt(C)),
    reported as max and median.  z well below ~4 = statistically identical.
One JSON line per n.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, Lorenz96Operator, MCMCSampler, pCNAccepter)


def run(n_rk, dtype, chains, n_samples, beta, gamma, d=256):
    G = Lorenz96Operator(d, 8.0, dt=0.005, n_steps=n_rk)
    k = np.arange(d)
    y = G(0.5 * np.sin(2 * np.pi * k / d)) + gamma * np.random.default_rng(3).normal(size=d)
    pot = EvolutionPotential(G, y, GaussianDistribution(np.zeros(d), gamma**2 * np.eye(d)))
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(d), np.eye(d))), acc, 11, dtype=dtype)
    u0 = 0.05 * np.random.default_rng(5).normal(size=(chains, d))
    t = time.perf_counter()
    mom = s.run(u0, n_samples=n_samples, burn_in=20, sample_interval=1, keep="moments")
    el = time.perf_counter() - t
    means = mom["sum_u"] / mom["n"]  # per-chain time averages (C, d)
    return means, np.asarray(acc.accepts), el


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    n_samples = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    for n_rk, beta, gamma in ((50, 0.05, 0.1), (200, 0.05, 0.1), (1000, 0.02, 0.1), (10000, 0.01, 0.1)):
        m64, a64, t64 = run(n_rk, np.float64, chains, n_samples, beta, gamma)
        m32, a32, t32 = run(n_rk, np.float32, chains, n_samples, beta, gamma)
        se64 = m64.std(axis=0, ddof=1) / np.sqrt(chains)
        se32 = m32.std(axis=0, ddof=1) / np.sqrt(chains)
        den = np.sqrt(se64**2 + se32**2)
        z = np.abs(m32.mean(axis=0) - m64.mean(axis=0)) / np.where(den > 0, den, np.inf)
        steps = n_samples + 20 - 1  # burn-in max(0, 20 - 1) + n_samples * 1
        rec = {
            "d": 256, "rk4_steps": n_rk, "beta": beta, "chains": chains, "pcn_steps": steps,
            "accept_rate_f64": float(a64.sum()) / (chains * steps),
            "accept_rate_f32": float(a32.sum()) / (chains * steps),
            "chains_same_accept_count": float(np.mean(a64 == a32)),
            "z_max": float(np.max(z)) if np.isfinite(z).any() else None,
            "z_median": float(np.median(z[np.isfinite(z)])) if np.isfinite(z).any() else None,
            "mean_abs_diff_max": float(np.max(np.abs(m32.mean(axis=0) - m64.mean(axis=0)))),
            "seconds_f64": t64, "seconds_f32": t32,
        }
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
