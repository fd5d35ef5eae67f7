"""Multi-process sharding through the product path on the GPU.

Two ranks (gloo for the gather; both on cuda:0 of the one-GPU box) each run
their block of global chain ids through MCMCSampler -> libipmc with
chain_offset = their first id, and all-gather samples, accept counts and the
ordered posterior mean (shard.gather_chains / ordered_mean).  The gathered
result must equal one process running every chain, bit for bit: the draws are
keyed by global chain id.  (bench.py's N-GPU path is the same decomposition
over RCCL.)
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

pytestmark = pytest.mark.gpu

C_TOTAL, K = 1001, 40


def _u0():
    return 0.1 * np.random.default_rng(9).normal(size=(C_TOTAL, K))


def _run(a, b):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             Lorenz96Operator, MCMCSampler, pCNAccepter)

    G = Lorenz96Operator(K, 8.0, dt=0.005, n_steps=150)
    y = G(np.zeros(K)) + 0.1 * np.random.default_rng(3).normal(size=K)
    pot = EvolutionPotential(G, y, GaussianDistribution(np.zeros(K), 0.01 * np.eye(K)))
    acc = CountedAccepter(pCNAccepter(pot))
    s = MCMCSampler(ConstSteppCNProposer(0.1, GaussianDistribution(np.zeros(K), np.eye(K))), acc, 7,
                    chain_offset=a)
    samples = s.run(_u0()[a:b], n_samples=3, burn_in=8, sample_interval=4)
    return samples, np.asarray(acc.accepts, dtype=np.int64)


def _worker(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import chain_range, gather_chains, ordered_mean

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = chain_range(C_TOTAL, rank, world)
    samples, accepts = _run(a, b)
    sg = gather_chains(torch.from_numpy(samples.reshape(b - a, -1)), C_TOTAL)
    ag = gather_chains(torch.from_numpy(accepts).view(-1, 1), C_TOTAL)
    mean = ordered_mean(sg)
    if rank == 0:
        np.savez(out_path, S=sg.numpy(), acc=ag.numpy().ravel(), mean=mean)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gpu_run_equals_one_process(tmp_path):
    from ip_mcmc_amd.shard import ordered_mean

    out = str(tmp_path / "g.npz")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    got = np.load(out)
    samples, accepts = _run(0, C_TOTAL)
    assert accepts.sum() > 0
    assert np.array_equal(got["S"], samples.reshape(C_TOTAL, -1))
    assert np.array_equal(got["acc"], accepts)
    assert np.array_equal(got["mean"], ordered_mean(torch.from_numpy(samples.reshape(C_TOTAL, -1))))
