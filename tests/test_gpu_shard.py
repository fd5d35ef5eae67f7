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


def test_device_ordered_sum_equals_the_host_library():
    """ipmc_ordered_sum (the device's chain-ordered column sums) == the host
    library's ipmc_host_ordered_sum bit for bit: mixed magnitudes, a row stride
    wider than k, div != 1, a running acc, no rows."""
    from ip_mcmc_amd import _hostlib
    from ip_mcmc_amd import device as D

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(4)
    for n, k, stride, div in ((65536, 40, 40, 1.0), (3001, 257, 300, 7.0), (5, 3, 3, 0.5), (0, 4, 4, 2.0),
                              (1, 1, 1, 1.0)):
        a = rng.normal(size=(n, stride)) * np.exp(rng.normal(scale=6, size=(n, 1)))
        acc0 = rng.normal(size=k)
        want = acc0.copy()
        if n:
            _hostlib.call("ipmc_host_ordered_sum", a.ctypes.data, n, k, stride, float(div), want.ctypes.data)
        rows = torch.as_tensor(a, device=dev)[:, :k]
        acc = torch.as_tensor(acc0, device=dev).clone()
        D.ordered_sum(rows, acc, div)
        assert np.array_equal(acc.cpu().numpy(), want), (n, k, stride, div)


def _mean_worker(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = run_sharded(_make_sampler, _u0(), n_samples=1, burn_in=0, sample_interval=6, keep="moments", gather="mean")
    s = res["sampler"]
    assert s.last_path == "device" and s.last_device_sums is None
    if rank == 1:
        np.savez(out_path, mean=res["mean"], phi=res["phi"], acc=res["accepts"])
    dist.barrier()
    dist.destroy_process_group()


def _make_sampler(chain_offset=0):
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, Lorenz96Operator,
                             MCMCSampler, pCNAccepter)

    G = Lorenz96Operator(K, 8.0, dt=0.005, n_steps=150)
    y = G(np.zeros(K)) + 0.1 * np.random.default_rng(3).normal(size=K)
    pot = EvolutionPotential(G, y, GaussianDistribution(np.zeros(K), 0.01 * np.eye(K)))
    return MCMCSampler(ConstSteppCNProposer(0.1, GaussianDistribution(np.zeros(K), np.eye(K))), pCNAccepter(pot), 7,
                       chain_offset=chain_offset)


def test_device_block_sums_equal_the_host_library():
    """ipmc_block_sums (the posterior mean's per-block sums, blocks in parallel)
    == ipmc_host_ordered_sum from zero on each block, bit for bit: whole and
    ragged last blocks, a row stride wider than k, div != 1, one row, no rows;
    and shard.ordered_sum_sharded on device rows == shard.block_sum on the host."""
    from ip_mcmc_amd import device as D
    from ip_mcmc_amd.shard import _seq_sum, block_sum, ordered_sum_sharded

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    for n, k, stride, block, div in ((65536, 40, 40, 1024, 1.0), (5003, 257, 300, 1024, 7.0), (100, 3, 5, 16, 0.5),
                                     (1, 1, 1, 1024, 1.0), (0, 4, 4, 8, 2.0), (4096, 40, 40, 1, 1.0)):
        a = rng.normal(size=(n, stride)) * np.exp(rng.normal(scale=6, size=(n, 1)))
        want = np.stack([_seq_sum(a[b : b + block, :k], np.zeros(k), div) for b in range(0, n, block)]) \
            if n else np.zeros((0, k))
        got = D.block_sums(torch.as_tensor(a, device=dev)[:, :k], block, div).cpu().numpy()
        assert got.shape == want.shape and np.array_equal(got, want), (n, k, stride, block, div)
        if n:
            rows = torch.as_tensor(np.ascontiguousarray(a[:, :k]), device=dev)
            assert np.array_equal(ordered_sum_sharded(rows, div=div, block=block),
                                  block_sum(a[:, :k], div=div, block=block)), (n, k, block)


def test_run_sharded_mean_on_the_device_equals_the_host_mean(tmp_path):
    """gather='mean' sums the sweeps' device sums (ipmc_block_sums on each
    rank, one all_gather): one process and two ranks (gloo, both on cuda:0)
    give the host block_sum mean of the per-chain sums bit for bit."""
    from ip_mcmc_amd.shard import block_sum, run_sharded

    one = run_sharded(_make_sampler, _u0(), n_samples=1, burn_in=0, sample_interval=6, keep="moments", gather="mean")
    host = block_sum(one["sum_u"]) / (float(one["n"]) * C_TOTAL)  # the host library's additions
    assert np.array_equal(one["mean"], host)
    out = str(tmp_path / "m.npz")
    mp.start_processes(_mean_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    got = np.load(out)
    assert np.array_equal(got["mean"], one["mean"])
    assert np.array_equal(got["phi"], one["phi"]) and np.array_equal(got["acc"], one["accepts"])


def _osum_rows(n):
    rng = np.random.default_rng(n)
    return rng.normal(size=(n, 7)) * np.exp(rng.normal(scale=6, size=(n, 1)))


def _osum_worker(rank, world, port, out_path, n_total, div):
    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import chain_range, ordered_sum_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = chain_range(n_total, rank, world)
    rows = torch.as_tensor(_osum_rows(n_total)[lo:hi], device=torch.device("cuda", 0))
    got = ordered_sum_sharded(rows, div=div)
    if rank == world - 1:
        np.save(out_path, got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,div", [(2, 5003, 1.0), (3, 4100, 3.0)])
def test_sharded_block_sums_on_the_device_equal_block_sum(tmp_path, world, n_total, div):
    """Device rows over ranks (gloo, all on cuda:0): each rank's whole blocks
    by ipmc_block_sums, the blocks it shares with a neighbour as raw rows, one
    all_gather -- block_sum over all rows on the host, bit for bit."""
    from ip_mcmc_amd.shard import block_sum

    out = str(tmp_path / "o.npy")
    mp.start_processes(_osum_worker, args=(world, _free_port(), out, n_total, div), nprocs=world,
                       start_method="spawn")
    assert np.array_equal(np.load(out), block_sum(_osum_rows(n_total), div=div))


def test_results_on_the_device_equal_the_host_results():
    """results='device': a run that starts (u_0 a device tensor) and ends in
    HBM gives the host run's sums, states, Φ and counters bit for bit; the
    checkpoint's states stay on the device and a resumed run from it equals
    one resumed from the host state; run_sharded's gather='mean' keeps the
    rank's rows on the device and forms the same mean."""
    from ip_mcmc_amd.shard import run_sharded

    dev = torch.device("cuda", 0)
    u0 = _u0()
    a, b = _make_sampler(), _make_sampler()
    rh = a.run(u0, n_samples=2, burn_in=0, sample_interval=3, keep="moments")
    rd = b.run(torch.as_tensor(u0, device=dev), n_samples=2, burn_in=0, sample_interval=3, keep="moments",
               results="device")
    assert rd["sum_u"].is_cuda and b.state.u_device is not None
    assert np.array_equal(rd["sum_u"].cpu().numpy(), rh["sum_u"])
    assert np.array_equal(rd["sum_u2"].cpu().numpy(), rh["sum_u2"])
    assert np.array_equal(b.state.phi, a.state.phi) and np.array_equal(b.state.accepts, a.state.accepts)
    assert np.array_equal(b.state.u, a.state.u)  # copied to the host on first access
    la = a.run(a.checkpoint(), n_samples=1, burn_in=0, sample_interval=2, keep="last")
    lb = b.run(b.checkpoint(), n_samples=1, burn_in=0, sample_interval=2, keep="last", results="device")
    assert lb.is_cuda and np.array_equal(lb.cpu().numpy(), la)
    with pytest.raises(ValueError):
        b.run(u0, n_samples=1, burn_in=0, sample_interval=1, keep="samples", results="device")
    one = run_sharded(_make_sampler, u0, n_samples=1, burn_in=0, sample_interval=6, keep="moments", gather="mean")
    dd = run_sharded(_make_sampler, torch.as_tensor(u0, device=dev), n_samples=1, burn_in=0, sample_interval=6,
                     keep="moments", gather="mean", results="device")
    assert dd["u"].is_cuda and dd["sum_u"].is_cuda
    for key in ("mean", "phi", "accepts"):
        assert np.array_equal(dd[key], one[key]), key
    assert np.array_equal(dd["u"].cpu().numpy(), one["u"]) and np.array_equal(dd["sum_u"].cpu().numpy(),
                                                                               one["sum_u"])
    # the returned state is a copy, not the checkpoint's own tensor
    ck = dd["sampler"].checkpoint().u_device
    before = ck.clone()
    dd["u"].add_(1.0)
    assert torch.equal(ck, before) and dd["u"].dtype == torch.float64


def _rccl_worker(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    import bench
    from ip_mcmc_amd.shard import run_sharded

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    assert dist.get_backend() == "nccl"
    # every collective of the product path, over RCCL on the device
    ga = run_sharded(_make_sampler, _u0(), n_samples=1, burn_in=0, sample_interval=6, keep="moments", gather="all")
    gm = run_sharded(_make_sampler, torch.as_tensor(_u0(), device=dev), n_samples=1, burn_in=0, sample_interval=6,
                     keep="moments", gather="mean", results="device")
    mx = bench.max_over_ranks(2.5, world, dev)
    dist.barrier()
    np.savez(out_path, u=ga["u"], phi=ga["phi"], acc=ga["accepts"], sum_u=ga["sum_u"], mean_all=ga["mean"],
             mean=gm["mean"], phi_m=gm["phi"], acc_m=gm["accepts"], mx=mx)
    dist.destroy_process_group()


def test_rccl_collectives_of_the_product_path(tmp_path):
    """The RCCL branches on hardware: a one-rank "nccl" process group (RCCL
    refuses two ranks on one GPU, profiles/r5/rccl_probe.json) runs every
    collective run_sharded and bench.py issue -- the packed all_gather
    (gather='all'), the counts / block-sum all_gathers (gather='mean', device
    rows), the MAX all_reduce of the wall time -- on device tensors.  The
    results equal the process-group-free run bit for bit."""
    from ip_mcmc_amd.shard import run_sharded

    out = str(tmp_path / "rccl_world1.npz")
    mp.start_processes(_rccl_worker, args=(1, _free_port(), out), nprocs=1, start_method="spawn")
    got = np.load(out)
    one = run_sharded(_make_sampler, _u0(), n_samples=1, burn_in=0, sample_interval=6, keep="moments", gather="all")
    for key, want in (("u", one["u"]), ("phi", one["phi"]), ("acc", one["accepts"]), ("sum_u", one["sum_u"]),
                      ("mean_all", one["mean"]), ("mean", one["mean"]), ("phi_m", one["phi"]),
                      ("acc_m", one["accepts"])):
        assert np.array_equal(got[key], want), key
    assert float(got["mx"]) == 2.5


def _mean_worker_n(rank, world, port, out_path, n_total):
    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import chain_range, run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = chain_range(n_total, rank, world)
    u0 = torch.as_tensor(0.1 * np.random.default_rng(9).normal(size=(n_total, K))[lo:hi], device="cuda:0")
    res = run_sharded(_make_sampler, u0, n_samples=1, burn_in=0, sample_interval=4, keep="moments", gather="mean",
                      results="device", n_total=n_total)
    assert res["sampler"].pre_sync_result is None  # consumed
    if rank == 1:
        np.savez(out_path, mean=res["mean"], phi=res["phi"], acc=res["accepts"])
    dist.barrier()
    dist.destroy_process_group()


def test_run_sharded_mean_with_whole_and_shared_blocks_two_ranks(tmp_path):
    """5 003 chains over two ranks (gloo, both on cuda:0), rank-local u_0 on the
    device: each rank's whole blocks of 1 024 chains summed on the device and
    its shared rows copied to the host before the run's one synchronisation
    (MCMCSampler.pre_sync) -- the mean, Φ and accept counts equal one
    process's bit for bit."""
    from ip_mcmc_amd.shard import block_sum, run_sharded

    n_total = 5003
    u0 = 0.1 * np.random.default_rng(9).normal(size=(n_total, K))
    one = run_sharded(_make_sampler, u0, n_samples=1, burn_in=0, sample_interval=4, keep="moments", gather="all")
    assert np.array_equal(one["mean"], block_sum(one["sum_u"]) / (4.0 * n_total))
    out = str(tmp_path / "m2.npz")
    mp.start_processes(_mean_worker_n, args=(2, _free_port(), out, n_total), nprocs=2, start_method="spawn")
    got = np.load(out)
    assert np.array_equal(got["mean"], one["mean"])
    assert np.array_equal(got["phi"], one["phi"]) and np.array_equal(got["acc"], one["accepts"])
