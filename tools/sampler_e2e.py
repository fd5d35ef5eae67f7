"""End-to-end throughput of the drop-in API on the headline problem.

  python tools/sampler_e2e.py [chains] [n_samples] [sample_interval]

MCMCSampler.run (ConstSteppCNProposer + CountedAccepter(pCNAccepter(
EvolutionPotential(Lorenz96Operator)))) from host u_0 to host samples, timed
around the whole call: H2D of u_0, the fused sweeps, the D2H of the
(C, n_samples, k) samples.  Reported next to the in-kernel time
(sampler.last_run_seconds) so the host-transfer share is visible.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, PhiloxRNG, pCNAccepter)


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    n_samples = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    interval = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    op, y = B.problem()
    d = B.D
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(d), B.GAMMA**2 * np.eye(d)))
    prior = GaussianDistribution(np.zeros(d), np.eye(d))
    for dtype in (np.float64, np.float32):
        for keep in ("samples", "moments"):
            acc = CountedAccepter(pCNAccepter(pot))
            s = MCMCSampler(ConstSteppCNProposer(B.BETA, prior), acc, PhiloxRNG(2), dtype=dtype)
            # warm-up of the same size: the page-locked result buffer of a run is
            # recycled by torch's host allocator once the caller drops it
            s.run(np.zeros((chains, d)), n_samples=n_samples, burn_in=interval, sample_interval=interval, keep=keep)
            u0 = np.full((chains, d), 0.0)  # written, i.e. resident (np.zeros maps its pages on first touch, inside run())
            t0 = time.perf_counter()
            out = s.run(u0, n_samples=n_samples, burn_in=interval, sample_interval=interval, keep=keep)
            wall = time.perf_counter() - t0
            steps = n_samples * interval  # burn_in == interval: no extra burn-in steps (sampler.py:18)
            rec = {
                "dtype": np.dtype(dtype).name,
                "keep": keep,
                "chains": chains,
                "pcn_steps_per_chain": steps,
                "wall_s": wall,
                "kernel_region_s": s.last_run_seconds,
                "pcn_steps_per_s_end_to_end": chains * steps / wall,
                "pcn_steps_per_s_device": chains * steps / s.last_run_seconds,
                "output_bytes": int(out.nbytes) if keep == "samples" else int(out["sum_u"].nbytes * 2),
                "accept_ratio_mean": float(np.mean(acc.ratio())),
            }
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
