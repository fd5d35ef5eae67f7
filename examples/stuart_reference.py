"""The reference's Stuart 2010 examples composed exactly as its script does
(report/scripts/stuart_examples.py:50-163): a closure G, pCNProposer(beta=0.25),
CountedAccepter(pCNAccepter(EvolutionPotential(G, data, noise))), one numpy
Generator for the data and the sampler, one chain, n_samples = 5 000 with the
default burn-in 1 000 and interval 200 -- BASELINE config 1's "1 chain on the
NumPy path".  The Python G runs in MCMCSampler's host-side step
(ip_mcmc_amd/hostloop.py); the draws come from the GPU when there is one and
from libipmc_host.so (the kernels' draw arithmetic compiled for the CPU, the
same bits) when there is none.  Instead of the
reference's histogram this prints the sample mean and variance next to the
exact posterior (results.org:59-62) and the wall time.

  python examples/stuart_reference.py [n_samples]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (CountedAccepter, EvolutionPotential, GaussianDistribution, MCMCSampler,  # noqa: E402
                         pCNAccepter, pCNProposer)


def build_evolution_pCN_sampler(observation_operator, data, noise, prior, rng):
    """stuart_examples.py:50-55."""
    potential = EvolutionPotential(observation_operator, data, noise)
    proposer = pCNProposer(beta=0.25, prior=prior)
    accepter = CountedAccepter(pCNAccepter(potential=potential))
    return MCMCSampler(proposer, accepter, rng), accepter


def exact(Gmat, y, gamma, k):
    S = gamma**2 * np.eye(Gmat.shape[0]) + Gmat @ Gmat.T
    gain = Gmat.T @ np.linalg.inv(S)
    return gain @ y, np.eye(k) - gain @ Gmat


def example(name, G, Gmat, u, noise, gamma, n_samples):
    prior = GaussianDistribution(mean=np.zeros_like(u, dtype=float), covariance=np.identity(len(u)))
    rng = np.random.default_rng(1)
    data = G(u) + noise.sample(rng)  # SyntheticModel.observe (stuart_examples.py:34-41)
    sampler, accepter = build_evolution_pCN_sampler(G, data, noise, prior, rng)
    t0 = time.perf_counter()
    samples = sampler.run(u_0=np.zeros_like(u, dtype=float), n_samples=n_samples)
    wall = time.perf_counter() - t0
    m, c = exact(Gmat, np.atleast_1d(data), gamma, len(u))
    steps = max(0, 1000 - 200) + n_samples * 200
    return {"example": name, "path": sampler.last_path, "n_samples": n_samples, "pcn_steps": steps,
            "wall_s": wall, "pcn_steps_per_s": steps / wall, "accept_ratio": float(accepter.ratio()),
            "sample_mean": samples.mean(axis=0).tolist(), "exact_mean": m.tolist(),
            "sample_var": samples.var(axis=0).tolist(), "exact_var": np.diag(c).tolist()}


def main():
    n_samples = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    gamma = 0.5
    # example 2.1 (stuart_examples.py:58-109)
    g = np.array([int(x) for x in str(np.pi) if x != "."])[:1]
    u = np.array([int(x) for x in str(np.e) if x != "."])[:1]
    print(json.dumps(example("2.1", lambda v: np.dot(g, v), g.reshape(1, 1).astype(float), u,
                             GaussianDistribution(mean=0, covariance=gamma**2), gamma, n_samples)), flush=True)
    # example 2.2 (stuart_examples.py:112-163), its cubic coefficient beta = 0
    g2 = np.array([int(x) for x in str(np.pi) if x != "."])[:2]
    b = 0

    def G2(v):
        return g2 * (v + b * np.array([v[0] ** 3]))

    print(json.dumps(example("2.2", G2, g2.reshape(2, 1).astype(float), np.array([0.5]),
                             GaussianDistribution(mean=np.zeros(2), covariance=np.identity(2) * gamma**2), gamma,
                             n_samples)), flush=True)


if __name__ == "__main__":
    main()
