"""BASELINE config 2 through the drop-in API: Lorenz-63 parameter inference,
500 RK4 steps per forward map, pCN beta = 0.2, 4 096 chains on one MI355X.

The composition is the reference's (lorenz_mcmc.py:87-130 pattern):
MCMCSampler(ConstSteppCNProposer(0.2, prior), CountedAccepter(pCNAccepter(
EvolutionPotential(G, y, noise)))), with G the time averages of (x, y, z, x²,
y², z²) over the trajectory from the spun-up state for theta = (10, 28, 8/3) + u,
y = the truth's long-run moment means and noise Γ = 0.5²·diag(var of the
instantaneous moments) (tools/config_bench.cfg2_problem).  The
sampler runs the speculative sweep (16 slots per chain along the accept path)
in launches of up to sampler.STEPS_PER_LAUNCH steps.

  python examples/lorenz63_config2.py [chains] [steps]

Prints one JSON line per run: posterior mean / std of u over chains and steps
(keep="moments"), the accept rate, and end-to-end pCN steps/s of run().
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import config_bench as CB  # noqa: E402
from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, PhiloxRNG, pCNAccepter)


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    op, y, ginv, sq, beta = CB.cfg2_problem()
    noise = GaussianDistribution(np.zeros(6), np.diag(1.0 / ginv**2))
    prior = GaussianDistribution(np.zeros(3), np.diag(sq**2))
    rng = np.random.default_rng(7)
    u0 = sq * rng.normal(size=(chains, 3))  # prior draws
    for dtype in (np.float64, np.float32):
        acc = CountedAccepter(pCNAccepter(EvolutionPotential(op, y, noise)))
        s = MCMCSampler(ConstSteppCNProposer(beta, prior), acc, PhiloxRNG(3), dtype=dtype)
        s.run(u0, n_samples=4096, burn_in=1, sample_interval=1, keep="moments")  # warm-up (clock ramp, plans)
        acc = CountedAccepter(pCNAccepter(EvolutionPotential(op, y, noise)))
        s = MCMCSampler(ConstSteppCNProposer(beta, prior), acc, PhiloxRNG(3), dtype=dtype)
        t0 = time.perf_counter()
        m = s.run(u0, n_samples=steps, burn_in=1, sample_interval=1, keep="moments")
        wall = time.perf_counter() - t0
        n = m["n"] if "n" in m else steps
        mean = m["sum_u"] / n
        var = m["sum_u2"] / n - mean**2
        print(json.dumps({
            "config": "BASELINE config 2 (Lorenz-63, 500 RK4, pCN beta 0.2) through MCMCSampler.run",
            "dtype": np.dtype(dtype).name,
            "chains": chains,
            "pcn_steps_per_chain": steps,
            "posterior_mean_sigma_rho_b_offset": mean.mean(axis=0).tolist(),
            "posterior_std_sigma_rho_b_offset": np.sqrt(np.maximum(var.mean(axis=0), 0.0)).tolist(),
            "accept_rate": float(np.mean(acc.ratio())),
            "wall_s": wall,
            "pcn_steps_per_s_end_to_end": chains * steps / wall,
            "timing": s.last_run_timing,
        }), flush=True)


if __name__ == "__main__":
    main()
