"""Config 1 end to end through the drop-in API (the reference's own use: one
chain, linear G, 5 000 samples every 200 steps after a burn-in of 1 000,
stuart_examples.py:62-89 / sampler.py:12 defaults).  Prints wall time, launches
and the device time of the sweeps (HIP events around the run on the torch
stream) so launch overhead shows as the difference.

  python tools/probes/cfg1_e2e.py [chains]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, LinearOperator, MCMCSampler, PhiloxRNG, pCNAccepter)


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    g = np.array([3.0, 1.0, 4.0, 1.0])
    y = np.array([g @ np.array([2.0, 7.0, 1.0, 8.0])])
    pot = EvolutionPotential(LinearOperator(g), y, GaussianDistribution(0, 0.5**2))
    for spec in (1, 0):
        acc = CountedAccepter(pCNAccepter(pot))
        s = MCMCSampler(ConstSteppCNProposer(0.5, GaussianDistribution(np.zeros(4), np.eye(4))), acc, PhiloxRNG(1),
                        spec_width=spec)
        u0 = np.zeros(4) if chains == 1 else np.zeros((chains, 4))
        s.run(u0, n_samples=10, burn_in=200, sample_interval=200)  # warm-up
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        out = s.run(u0, n_samples=5000, burn_in=1000, sample_interval=200)
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        steps = chains * (800 + 5000 * 200)
        print(json.dumps({"chains": chains, "spec_width": spec, "wall_s": wall, "stream_s": e0.elapsed_time(e1) / 1e3,
                          "pcn_steps_per_s": steps / wall, "samples_shape": list(out.shape),
                          "accept_rate": float(np.mean(acc.ratio()))}), flush=True)


if __name__ == "__main__":
    main()
