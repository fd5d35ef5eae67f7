"""Burgers small-ensemble speculation on the reference's studies (examples/burgers_beta.py),
the sweep alone: run(keep="last") over 5 000 steps, no sample copies.  CFL
stepping (the reference's) and a fixed step, to separate the speculation
trees from the forward map's proposal-dependent cost.

  python tools/probes/burgers_spec_probe.py [chains] [spec_width]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ip_mcmc_amd import (BurgersOperator, ConstSteppCNProposer, CountedAccepter, EvolutionPotential,  # noqa: E402
                         GaussianDistribution, MCMCSampler, PWLinear, StandardRWAccepter, VarStepStandardRWProposer,
                         pCNAccepter)


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    spec = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    only = sys.argv[3] if len(sys.argv) > 3 else ""  # e.g. "pcn-cfl"
    prior_mean = np.array([1.5, 0.25, -0.5])
    truth = np.array([0.025, -0.025, -0.02])
    for dt_mode in ("cfl", "fixed"):
        kw = dict(dt=2.5e-3, n_steps=400) if dt_mode == "fixed" else {}
        G = BurgersOperator(prior_mean=prior_mean, N=128, T=1.0, dt_mode=dt_mode, **kw)
        y = G(truth - prior_mean)
        noise = GaussianDistribution(np.zeros(5), 0.05**2 * np.eye(5))
        prior = GaussianDistribution(prior_mean, 0.25**2 * np.eye(3))
        pot = EvolutionPotential(G, y, noise)
        for study in ("rw", "pcn"):
            if only and only != f"{study}-{dt_mode}":
                continue
            if study == "rw":
                acc = CountedAccepter(StandardRWAccepter(pot, prior))
                prop = VarStepStandardRWProposer(PWLinear(0.1, 0.001, 250), prior)
            else:
                acc = CountedAccepter(pCNAccepter(pot))
                prop = ConstSteppCNProposer(0.15, GaussianDistribution(np.zeros(3), 0.25**2 * np.eye(3)))
            s = MCMCSampler(prop, acc, np.random.default_rng(2), spec_width=spec)
            u0 = np.zeros((chains, 3))
            s.run(u0, n_samples=1, burn_in=0, sample_interval=50, keep="last")  # warm-up
            torch.cuda.synchronize()
            s = MCMCSampler(prop, acc, np.random.default_rng(2), spec_width=spec)
            t0 = time.perf_counter()
            s.run(u0, n_samples=1, burn_in=0, sample_interval=5000, keep="last")
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            print(json.dumps({"study": study, "dt_mode": dt_mode, "chains": chains, "spec_width": spec,
                              "accept_rate": float(np.mean(acc.ratio())), "wall_s": wall,
                              "steps_per_s": chains * 5000 / wall,
                              "lib": os.environ.get("IPMC_LIB_PATH", "product")}), flush=True)


if __name__ == "__main__":
    main()
