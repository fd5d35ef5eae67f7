"""The reference's linear-Gaussian examples (report/scripts/stuart_examples.py:58-163,
Stuart 2010 examples 2.1 and 2.2) on the GPU, with many chains instead of one.

Same problems: G(u) = <g, u> with g the first n digits of pi (example 2.1,
n = 1, u_true = 2, scalar noise variance 0.5^2) and G(u) = g u with q = 2
observations of a scalar u (example 2.2 with its cubic coefficient beta = 0,
u_true = 0.5, noise 0.5^2 I); prior N(0, I); pCN with beta = 0.25
(build_evolution_pCN_sampler, stuart_examples.py:50-55); the data drawn from
np.random.default_rng(1) as the reference does (SyntheticModel.observe);
n_samples = 5 000 with the sampler's default burn-in 1 000 and interval 200.
The reference plots a histogram of the one chain; here every chain's samples
are pooled and compared with the exact Gaussian posterior
(results.org:59-62): mean Σ0 Gᵀ(γ²I + GΣ0Gᵀ)⁻¹ y, covariance
Σ0 − Σ0Gᵀ(γ²I + GΣ0Gᵀ)⁻¹GΣ0.

  python examples/stuart_examples.py [chains]

Prints one JSON line per example: posterior mean and variance of the pooled
samples, the exact values, the deviation of the mean in Monte-Carlo standard
errors (per-chain means, so autocorrelation is accounted for), accept rate and
wall time.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, LinearOperator, MCMCSampler, pCNAccepter)


def digits(x, n):
    return np.array([int(c) for c in str(x) if c != "."])[:n]


def exact_posterior(A, y, gamma, prior_cov):
    S = gamma**2 * np.eye(A.shape[0]) + A @ prior_cov @ A.T
    gain = prior_cov @ A.T @ np.linalg.inv(S)
    return gain @ y, prior_cov - gain @ A @ prior_cov


def run_example(name, A, u_true, gamma, noise, chains, n_samples=5000, beta=0.25):
    k = A.shape[1]
    prior = GaussianDistribution(mean=np.zeros(k), covariance=np.identity(k))
    rng = np.random.default_rng(1)
    G = LinearOperator(A)
    y = np.atleast_1d(A @ u_true + noise.sample(rng))  # SyntheticModel.observe (stuart_examples.py:34-41)
    potential = EvolutionPotential(G, y, noise)
    accepter = CountedAccepter(pCNAccepter(potential=potential))
    sampler = MCMCSampler(ConstSteppCNProposer(beta=beta, prior=prior), accepter, rng)
    t0 = time.perf_counter()
    samples = sampler.run(np.zeros((chains, k)), n_samples)  # (chains, n_samples, k)
    wall = time.perf_counter() - t0
    mean, cov = exact_posterior(A, y, gamma, np.identity(k))
    per_chain = samples.mean(axis=1)  # (chains, k)
    mcse = per_chain.std(axis=0, ddof=1) / np.sqrt(chains)
    pooled = samples.reshape(-1, k)
    return {
        "example": name,
        "chains": chains,
        "n_samples": n_samples,
        "y": y.tolist(),
        "posterior_mean": pooled.mean(axis=0).tolist(),
        "exact_mean": mean.tolist(),
        "mean_error_in_mcse": ((pooled.mean(axis=0) - mean) / mcse).tolist(),
        "posterior_var": pooled.var(axis=0).tolist(),
        "exact_var": np.diag(cov).tolist(),
        "accept_rate": float(np.mean(accepter.ratio())),
        "pcn_steps_per_s": chains * (1000 + n_samples * 200) / wall,
        "wall_s": wall,
    }


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    gamma = 0.5
    # example 2.1: n = 1, G(u) = <g, u>, scalar noise (stuart_examples.py:58-109)
    g1 = digits(np.pi, 1).astype(float)
    print(json.dumps(run_example("2.1", g1.reshape(1, 1), digits(np.e, 1).astype(float), gamma,
                                 GaussianDistribution(mean=0, covariance=gamma**2), chains)), flush=True)
    # example 2.2: q = 2 observations of scalar u, G(u) = g u (stuart_examples.py:112-163, beta = 0)
    g2 = digits(np.pi, 2).astype(float)
    print(json.dumps(run_example("2.2", g2.reshape(2, 1), np.array([0.5]), gamma,
                                 GaussianDistribution(mean=np.zeros(2), covariance=np.identity(2) * gamma**2),
                                 chains)), flush=True)


if __name__ == "__main__":
    main()
