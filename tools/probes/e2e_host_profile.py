"""Host-side profile of one MCMCSampler.run on the headline problem (after a
same-size warm-up): where the wall time outside the GPU sweeps goes.

  python tools/probes/e2e_host_profile.py [chains] [n_samples] [interval] [samples|moments]
"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench as B  # noqa: E402
from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, PhiloxRNG, pCNAccepter)


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    interval = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    keep = sys.argv[4] if len(sys.argv) > 4 else "samples"
    op, y = B.problem()
    d = B.D
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(d), B.GAMMA**2 * np.eye(d)))
    prior = GaussianDistribution(np.zeros(d), np.eye(d))
    s = MCMCSampler(ConstSteppCNProposer(B.BETA, prior), CountedAccepter(pCNAccepter(pot)), PhiloxRNG(2))
    s.run(np.zeros((chains, d)), n_samples=n, burn_in=interval, sample_interval=interval, keep=keep)
    u0 = np.full((chains, d), 0.0)  # written, i.e. resident (np.zeros maps its pages on first touch, inside run())
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    s.run(u0, n_samples=n, burn_in=interval, sample_interval=interval, keep=keep)
    pr.disable()
    print(f"wall {time.perf_counter() - t0:.4f} s; timing {s.last_run_timing}")
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
