"""The reference's Burgers random-walk study (report/scripts/burgers/burgers_beta.py:25-200)
on the GPU, with many chains instead of one.

Same problem: Burgers' equation on (-1, 1) with N = 128 cells to T = 1 by the
reference's Rusanov scheme (CFL time stepping, rusanov.py), perturbed Riemann
initial condition (δ1, δ2, σ0) with truth (0.025, -0.025, -0.02), five
windowed measurements at (-0.5, -0.25, 0.25, 0.5, 0.75), noise-free data
(burgers_beta.py:118), noise std 0.05, prior N((1.5, 0.25, -0.5), 0.25² I);
VarStepStandardRWProposer with PWLinear(0.1, 0.001, 250) and
StandardRWAccepter, u_0 = 0, 5 000 steps recorded every step
(run(u_0, 5000, 0, 1)), burn-in 250 and thinning 20 when summarising
(burgers_beta.py:171-174).

  python examples/burgers_beta.py [chains]

Also runs the pCN chain the report prefers (burgers.org:222-234, β = 0.15,
burn-in 500, interval 25).  Prints one JSON line per study: posterior means /
standard deviations of (δ1, δ2, σ0) over all chains, the fraction of chains
that end within 0.05 of the truth (and their posterior mean), the accept
rate, the median burn-in len_burn_in finds (device kernel,
utilities.py:134-167) and wall time.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (BurgersOperator, ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, PWLinear, StandardRWAccepter, VarStepStandardRWProposer,
                         pCNAccepter)
from ip_mcmc_amd.diagnostics import burn_in_lengths  # noqa: E402


def summarise(name, full, prior_mean, truth, burn_in, interval, acc, wall, chains):
    post = full[:, burn_in::interval, :] + prior_mean
    last = full[:, -1, :] + prior_mean
    near = np.max(np.abs(last - truth), axis=1) < 0.05  # chain ended within 0.05 of the truth
    bi = burn_in_lengths(full, layout="time_vars")
    return {
        "study": name,
        "chains": chains,
        "steps_per_chain": full.shape[1],
        "posterior_mean_d1_d2_s0": post.reshape(-1, 3).mean(axis=0).tolist(),
        "posterior_std_d1_d2_s0": post.reshape(-1, 3).std(axis=0).tolist(),
        "truth_d1_d2_s0": truth.tolist(),
        "fraction_of_chains_ending_near_truth": float(near.mean()),
        "posterior_mean_of_those_chains": (post[near].reshape(-1, 3).mean(axis=0).tolist() if near.any() else None),
        "accept_rate": float(np.mean(acc.ratio())),
        "burn_in_median": float(np.median(bi)),
        "wall_s": wall,
        "steps_per_s": chains * full.shape[1] / wall,
    }


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    prior_mean = np.array([1.5, 0.25, -0.5])
    truth = np.array([0.025, -0.025, -0.02])
    G = BurgersOperator(prior_mean=prior_mean, N=128, T=1.0, dt_mode="cfl")
    y = G(truth - prior_mean)  # noise-free data, as the reference (burgers_beta.py:118)
    noise = GaussianDistribution(np.zeros(5), 0.05**2 * np.eye(5))
    prior = GaussianDistribution(prior_mean, 0.25**2 * np.eye(3))
    pot = EvolutionPotential(G, y, noise)
    u0 = np.zeros((chains, 3))

    # 1. burgers_beta.py main(): RW, PWLinear(0.1, 0.001, 250), StandardRWAccepter,
    #    run(u_0, 5000, 0, 1), burn-in 250 and interval 20 when summarising
    acc = CountedAccepter(StandardRWAccepter(pot, prior))
    s = MCMCSampler(VarStepStandardRWProposer(PWLinear(0.1, 0.001, 250), prior), acc, np.random.default_rng(2))
    t0 = time.perf_counter()
    full = s.run(u0, n_samples=5000, burn_in=0, sample_interval=1)  # (C, 5000, 3)
    wall = time.perf_counter() - t0
    print(json.dumps(summarise("RW + PWLinear(0.1, 0.001, 250) (burgers_beta.py)", full, prior_mean, truth, 250, 20,
                               acc, wall, chains)))

    # 2. the pCN chain of burgers.org:222-234 / 280: beta 0.15, burn-in 500, interval 25
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(ConstSteppCNProposer(0.15, GaussianDistribution(np.zeros(3), 0.25**2 * np.eye(3))), acc,
                    np.random.default_rng(2))
    t0 = time.perf_counter()
    full = s.run(u0, n_samples=5000, burn_in=0, sample_interval=1)
    wall = time.perf_counter() - t0
    print(json.dumps(summarise("pCN beta 0.15 (burgers.org:222-234)", full, prior_mean, truth, 500, 25, acc, wall,
                               chains)))


if __name__ == "__main__":
    main()
