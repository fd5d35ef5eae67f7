"""The reference's Burgers pCN study (burgers.org:222-234: N=128, CFL stepping
to T=1, β=0.15, the burgers_beta.py posterior; ~12 % acceptance) with small
ensembles: sequential vs speculation in a wave (2 slots of 32 lanes) vs
speculation over a block (8 slots, auto).  500 pCN steps per chain.

  python tools/probes/burgers_small.py
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ip_mcmc_amd import (BurgersOperator, ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, pCNAccepter)


def main():
    prior_mean = np.array([1.5, 0.25, -0.5])
    G = BurgersOperator(prior_mean=prior_mean, N=128, T=1.0, dt_mode="cfl")
    y = G(np.array([0.025, -0.025, -0.02]) - prior_mean)
    pot = EvolutionPotential(G, y, GaussianDistribution(np.zeros(5), 0.05**2 * np.eye(5)))
    for n in (1, 16, 64, 256):
        for mode, spec in (("sequential", 1), ("wave", 2), ("auto", 0)):
            acc = CountedAccepter(pCNAccepter(pot))
            s = MCMCSampler(ConstSteppCNProposer(0.15, GaussianDistribution(np.zeros(3), 0.25**2 * np.eye(3))), acc,
                            2, spec_width=spec)
            u0 = np.zeros((n, 3))
            s.run(u0, n_samples=1, burn_in=0, sample_interval=20)  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.run(u0, n_samples=1, burn_in=0, sample_interval=500)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            print(json.dumps({"chains": n, "mode": mode, "spec_width": spec, "pcn_steps_per_s": n * 500 / wall,
                              "accept_rate": float(np.mean(acc.ratio()))}), flush=True)


if __name__ == "__main__":
    main()
