"""BASELINE config 5 over the GPUs of one node through the drop-in API.

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/sharded_config5.py [chains] [steps]
  python examples/sharded_config5.py 16384 4          # one GPU, a smaller ensemble

Lorenz-96 d=256, 10 000 RK4 steps per forward map, 2^20 chains by default,
fp32 and fp64: every rank builds the same sampler with its own chain_offset
(shard.run_sharded), runs its block of global chain ids, and the posterior
mean -- the per-chain time averages averaged over the chains in global order
by fixed-order block sums -- is identical for any number of GPUs.
Prints one JSON line per precision (rank 0): pCN steps/s over the node, the
accept rate and the fp32-fp64 difference of the posterior means.
"""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution,  # noqa: E402
                         Lorenz96Operator, MCMCSampler, PhiloxRNG, pCNAccepter)
from ip_mcmc_amd.shard import run_sharded  # noqa: E402

D, N_RK = 256, 10000


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    G = Lorenz96Operator(D, 8.0, dt=0.005, n_steps=N_RK)
    k = np.arange(D)
    y = G(0.5 * np.sin(2 * np.pi * k / D)) + 0.1 * np.random.default_rng(3).normal(size=D)
    noise = GaussianDistribution(np.zeros(D), 0.01 * np.eye(D))
    prior = GaussianDistribution(np.zeros(D), np.eye(D))
    # this rank's own rows of the node's u_0 only (run_sharded(n_total=)): no
    # rank allocates the 2^20 x 256 ensemble
    u0 = lambda lo, hi: np.zeros((hi - lo, D))  # noqa: E731
    means = {}
    for dtype in (np.float64, np.float32):
        def make(chain_offset=0):
            return MCMCSampler(ConstSteppCNProposer(0.2, prior), pCNAccepter(EvolutionPotential(G, y, noise)),
                               PhiloxRNG(7), dtype=dtype, chain_offset=chain_offset)

        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        res = run_sharded(make, u0, n_samples=1, burn_in=0, sample_interval=steps, keep="moments", gather="mean",
                          n_total=chains)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        means[dtype] = res["mean"]
        if res["rank"] == 0:
            print(json.dumps({"config": 5, "dtype": np.dtype(dtype).name, "gpus": world, "chains": chains,
                              "pcn_steps": steps, "wall_s": wall, "pcn_steps_per_s": chains * steps / wall,
                              "accept_rate": float(res["accepts"].sum()) / (chains * steps)}), flush=True)
    if int(os.environ.get("RANK", "0")) == 0:
        d = means[np.float32] - means[np.float64]
        print(json.dumps({"posterior_mean_max_abs_diff_f32_f64": float(np.max(np.abs(d)))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
