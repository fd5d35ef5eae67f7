"""Multi-process chain sharding on CPU (gloo, world_size 2, 3 and 8).

Each rank owns a contiguous block of global chain ids (shard.chain_range),
advances it with the CPU oracle (the per-rank compute stand-in: on the GPU box
the same ranks call libipmc), and the blocks are all-gathered in rank order
(shard.gather_chains).  The gathered states, accept counts and the ordered
posterior mean must equal one single-process run bit for bit: the RNG is keyed
by global chain id, so sharding changes nothing.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

C_TOTAL, K, STEPS = 37, 8, 5


def _problem():
    from ip_mcmc_amd.forward import Lorenz96Operator

    op = Lorenz96Operator(K, 8.0, dt=0.01, n_steps=30)
    rng = np.random.default_rng(0)
    U0 = 0.2 * rng.normal(size=(C_TOTAL, K))
    y = 8.0 + 0.3 * rng.normal(size=K)
    return op, U0, y, np.full(K, 10.0), np.ones(K)


def _run_block(start, stop):
    import sys

    sys.path.insert(0, REPO)
    from oracle import oracle as O

    op, U0, y, ginv, sq = _problem()
    U = np.ascontiguousarray(U0[start:stop])
    phi = O.potential(op, U, y, ginv)
    acc = np.zeros(stop - start, dtype=np.int64)
    O.pcn_sweep(op, U, phi, y, ginv, sq, 0.3, 11, 0, STEPS, accepts=acc, chain_offset=start)
    return U, phi, acc


def _worker(rank, world, port, out_path):
    import sys

    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import chain_range, gather_chains, ordered_mean

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = chain_range(C_TOTAL, rank, world)
    U, phi, acc = _run_block(a, b)
    Ug = gather_chains(torch.from_numpy(U), C_TOTAL)
    accg = gather_chains(torch.from_numpy(acc).view(-1, 1), C_TOTAL)
    mean = ordered_mean(Ug)
    if rank == 0:
        np.savez(out_path, U=Ug.numpy(), acc=accg.numpy().ravel(), mean=mean)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_chain_range_partitions():
    from ip_mcmc_amd.shard import chain_range

    for n in (1, 7, 37, 65536):
        for w in (1, 2, 3, 8):
            blocks = [chain_range(n, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_run_equals_single_process(tmp_path, world):
    from ip_mcmc_amd.shard import ordered_mean

    out = str(tmp_path / "g.npz")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, start_method="spawn")
    got = np.load(out)
    U, phi, acc = _run_block(0, C_TOTAL)
    assert np.array_equal(got["U"], U)
    assert np.array_equal(got["acc"], acc)
    assert np.array_equal(got["mean"], ordered_mean(torch.from_numpy(U)))


def _blocked_loop(a, div=1.0, block=None):
    """block_sum's additions as a plain loop: each block's rows from zero, then
    the block sums in order."""
    from ip_mcmc_amd.shard import MEAN_BLOCK

    block = block or MEAN_BLOCK
    tot = np.zeros(a.shape[1])
    for b0 in range(0, a.shape[0], block):
        s = np.zeros(a.shape[1])
        for row in a[b0 : b0 + block]:
            s = s + row / div
        tot = tot + s
    return tot


def test_block_sum_is_the_blocked_sequential_loop():
    """shard.block_sum / ordered_mean (ipmc_host_ordered_sum per block, then
    over the block sums) is the loop of the same additions, bit for bit, at
    10^5 rows with mixed magnitudes; with div the rows are divided first; up to
    one block it is the plain running sum."""
    from ip_mcmc_amd.shard import MEAN_BLOCK, _seq_sum, block_sum, ordered_mean

    rng = np.random.default_rng(0)
    a = rng.normal(size=(100_000, 7)) * np.exp(rng.normal(scale=8, size=(100_000, 1)))
    assert np.array_equal(ordered_mean(torch.from_numpy(a)), _blocked_loop(a) / a.shape[0])
    assert np.array_equal(ordered_mean(a[:5]), np.cumsum(a[:5], axis=0)[-1] / 5)
    assert np.array_equal(block_sum(a[:MEAN_BLOCK]), _seq_sum(a[:MEAN_BLOCK], np.zeros(7)))
    assert np.array_equal(ordered_mean(a[:3000], div=37.0), _blocked_loop(a[:3000], 37.0) / 3000)
    assert np.array_equal(block_sum(a[:1000], block=16), _blocked_loop(a[:1000], block=16))
    assert np.array_equal(block_sum(np.zeros((0, 3))), np.zeros(3))
    # _seq_sum continues a running sum from any row (the shared blocks' rows)
    part = _seq_sum(a[:1234], np.zeros(7))
    assert np.array_equal(_seq_sum(a[1234:], part), _seq_sum(a, np.zeros(7)))


def test_split_partitions_a_range_at_block_boundaries():
    """shard._split: head + whole blocks + tail cover [lo, hi) in order; the
    whole blocks are exactly the blocks inside the range; head and tail each
    lie in one block that the range does not cover whole."""
    from ip_mcmc_amd.shard import _split

    for block in (1, 3, 16):
        for lo in range(0, 40):
            for hi in range(lo, 60):
                head, (b0, b1), tail = _split(lo, hi, block)
                rows = []
                if head is not None:
                    assert head[0] // block == (head[1] - 1) // block and head[1] - head[0] < block
                    rows += list(range(*head))
                rows += list(range(b0 * block, b1 * block))
                if tail is not None:
                    assert tail[0] // block == (tail[1] - 1) // block and tail[1] - tail[0] < block
                    rows += list(range(*tail))
                assert rows == list(range(lo, hi)), (lo, hi, block)
                inside = [b for b in range(0, 60 // block + 2) if lo <= b * block and (b + 1) * block <= hi]
                assert list(range(b0, b1)) == inside, (lo, hi, block)


def _osum_rows(n):
    rng = np.random.default_rng(n)
    return rng.normal(size=(n, 5)) * np.exp(rng.normal(scale=6, size=(n, 1)))


def _osum_worker(rank, world, port, out_path, n_total, block, div):
    import sys

    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import chain_range, ordered_sum_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = chain_range(n_total, rank, world)
    rows = _osum_rows(n_total)[lo:hi]
    got = ordered_sum_sharded(rows, div=div, block=block)
    # the rank's whole-block sums and shared rows formed ahead (run_sharded's
    # pre_sync path, here on host rows): the same bits
    from ip_mcmc_amd.shard import _rank_parts

    assert np.array_equal(ordered_sum_sharded(rows, div=div, block=block, parts=_rank_parts(rows, lo, block, div)),
                          got)
    # bench.py's max over ranks of the wall time (gloo: on the host)
    import bench

    assert bench.max_over_ranks(float(rank), world, "cpu") == float(world - 1)
    if rank == world - 1:
        np.save(out_path, got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,block,div", [(3, 5003, 1024, 1.0), (8, 203, 16, 37.0), (8, 100, 64, 1.0)])
def test_ordered_sum_sharded_equals_block_sum(tmp_path, world, n_total, block, div):
    """The sharded sum (whole blocks summed on their rank, shared blocks' rows
    and the block sums in one all_gather, gloo) == block_sum over all rows, bit
    for bit: ranks spanning several blocks, blocks spanning several ranks, a
    ragged last block, div != 1."""
    from ip_mcmc_amd.shard import block_sum

    out = str(tmp_path / "o.npy")
    mp.start_processes(_osum_worker, args=(world, _free_port(), out, n_total, block, div), nprocs=world,
                       start_method="spawn")
    assert np.array_equal(np.load(out), block_sum(_osum_rows(n_total), div=div, block=block))


# ---------------------------------------------- shard.run_sharded (product)
def _lin_sampler_factory():
    """A host-tier composition (a Python closure G, the reference's config-1
    form) that runs on CPU ranks: the host step draws from libipmc_host.so."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             MCMCSampler, PhiloxRNG, pCNAccepter)

    g = np.array([3.0, 1.0, 4.0, 1.0])
    y = np.dot(g, [2.0, 7.0, 1.0, 8.0]) + 0.5 * 0.3

    def make(chain_offset=0):
        pot = EvolutionPotential(lambda u: np.dot(g, u), y, GaussianDistribution(0, 0.25))
        return MCMCSampler(ConstSteppCNProposer(0.5, GaussianDistribution(np.zeros(4), np.eye(4))),
                           CountedAccepter(pCNAccepter(pot)), PhiloxRNG(21), chain_offset=chain_offset)

    return make


def _sharded_worker(rank, world, port, out_path, keep, gather="all", n_total=C_TOTAL, u0_form="full"):
    import sys

    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import chain_range, run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = 0.1 * np.random.default_rng(1).normal(size=(n_total, 4))
    kw = {}
    if u0_form == "full":  # the node's ensemble on every rank
        u0 = full
    elif u0_form == "local":  # only this rank's block of rows
        a, b = chain_range(n_total, rank, world)
        u0, kw = full[a:b].copy(), {"n_total": n_total}
        del full
    else:  # a callable building this rank's rows
        u0, kw = (lambda lo, hi: 0.1 * np.random.default_rng(1).normal(size=(n_total, 4))[lo:hi]), {"n_total": n_total}
    res = run_sharded(_lin_sampler_factory(), u0, n_samples=6, burn_in=9, sample_interval=4, keep=keep,
                      gather=gather, **kw)
    assert res["world"] == world and res["sampler"].last_path == "host"
    if rank == 1:  # every rank holds the gathered result
        body = {k: v for k, v in res.items() if isinstance(v, np.ndarray)}
        np.savez(out_path, **body)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("keep", ["moments", "samples"])
def test_run_sharded_equals_one_process(tmp_path, keep):
    """run_sharded over gloo, world 3, = one process's run(): states, Φ, accept
    counts, sums or samples and the ordered posterior mean, bit for bit."""
    from ip_mcmc_amd.shard import run_sharded

    out = str(tmp_path / "s.npz")
    mp.start_processes(_sharded_worker, args=(3, _free_port(), out, keep), nprocs=3, start_method="spawn")
    got = np.load(out)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(C_TOTAL, 4))
    one = run_sharded(_lin_sampler_factory(), u0, n_samples=6, burn_in=9, sample_interval=4, keep=keep)
    assert one["world"] == 1
    keys = ["u", "phi", "accepts"] + (["sum_u", "sum_u2", "mean"] if keep == "moments" else ["samples"])
    for key in keys:
        assert np.array_equal(got[key], one[key]), key
    assert one["accepts"].sum() > 0
    if keep == "moments":
        want = _lin_sampler_factory()(0).run(u0, n_samples=6, burn_in=9, sample_interval=4, keep="moments")
        np.testing.assert_array_equal(one["sum_u"], want["sum_u"])


def test_run_sharded_mean_by_block_sums(tmp_path):
    """gather='mean': no per-chain sums leave their rank, yet the posterior
    mean (fixed-order block sums) and the gathered Φ / accept counts
    equal the one-process run's bit for bit (gloo, world 3)."""
    from ip_mcmc_amd.shard import run_sharded

    out = str(tmp_path / "m.npz")
    mp.start_processes(_sharded_worker, args=(3, _free_port(), out, "moments", "mean"), nprocs=3,
                       start_method="spawn")
    got = np.load(out)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(C_TOTAL, 4))
    one = run_sharded(_lin_sampler_factory(), u0, n_samples=6, burn_in=9, sample_interval=4, keep="moments")
    for key in ("mean", "phi", "accepts"):
        assert np.array_equal(got[key], one[key]), key
    assert got["sum_u"].shape[0] == 12  # rank 1's own block of chain_range(37, 1, 3)


@pytest.mark.parametrize("n_total", [1003, 5])
@pytest.mark.parametrize("gather", ["all", "mean"])
def test_run_sharded_world_8_uneven(tmp_path, gather, n_total):
    """An 8-rank rehearsal of the node (gloo): 1 003 chains (ranks of 126 and
    125) and 5 chains (three ranks with none).  The gathered Φ and accept
    counts and the posterior mean equal one process's bit for bit in both
    gather modes; gather='all' also the states and sums."""
    from ip_mcmc_amd.shard import chain_range, run_sharded

    out = str(tmp_path / "w8.npz")
    mp.start_processes(_sharded_worker, args=(8, _free_port(), out, "moments", gather, n_total), nprocs=8,
                       start_method="spawn")
    got = np.load(out)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(n_total, 4))
    one = run_sharded(_lin_sampler_factory(), u0, n_samples=6, burn_in=9, sample_interval=4, keep="moments")
    keys = ("mean", "phi", "accepts") + (("u", "sum_u", "sum_u2") if gather == "all" else ())
    for key in keys:
        assert np.array_equal(got[key], one[key]), key
    if gather == "mean":  # rank 1's own rows only
        a, b = chain_range(n_total, 1, 8)
        assert np.array_equal(got["sum_u"], one["sum_u"][a:b])
    assert one["accepts"].sum() > 0


@pytest.mark.parametrize("u0_form", ["local", "callable"])
def test_run_sharded_world_8_rank_local_u0(tmp_path, u0_form):
    """u_0 given per rank -- each rank's own block with n_total, or a callable
    u_0(lo, hi) -- instead of the node's ensemble on every rank (VERDICT r5:
    no rank allocates the others' rows): the same bits as one process, 8 ranks
    of 126/125 chains, both gather modes' results."""
    from ip_mcmc_amd.shard import chain_range, run_sharded

    n_total = 1003
    out = str(tmp_path / "w8l.npz")
    mp.start_processes(_sharded_worker, args=(8, _free_port(), out, "moments", "mean", n_total, u0_form), nprocs=8,
                       start_method="spawn")
    got = np.load(out)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(n_total, 4))
    one = run_sharded(_lin_sampler_factory(), u0, n_samples=6, burn_in=9, sample_interval=4, keep="moments")
    for key in ("mean", "phi", "accepts"):
        assert np.array_equal(got[key], one[key]), key
    a, b = chain_range(n_total, 1, 8)
    assert np.array_equal(got["sum_u"], one["sum_u"][a:b]) and np.array_equal(got["u"], one["u"][a:b])


def test_local_start_forms():
    """shard.local_start: the full ensemble, a rank's block with n_total, a
    callable; a block of the wrong size is refused."""
    from ip_mcmc_amd.shard import local_start

    full = np.arange(20.0).reshape(10, 2)
    blk, n = local_start(full, None, 1, 3)  # chain_range(10, 1, 3) = [4, 7)
    assert n == 10 and np.array_equal(blk, full[4:7])
    blk, n = local_start(full[4:7], 10, 1, 3)
    assert n == 10 and np.array_equal(blk, full[4:7])
    blk, n = local_start(lambda lo, hi: full[lo:hi], 10, 2, 3)
    assert n == 10 and np.array_equal(blk, full[7:10])
    with pytest.raises(ValueError, match="neither"):
        local_start(full[4:6], 10, 1, 3)
    with pytest.raises(ValueError, match="needs n_total"):
        local_start(lambda lo, hi: full[lo:hi], None, 0, 3)
    with pytest.raises(ValueError, match="must return"):
        local_start(lambda lo, hi: full[:1], 10, 0, 3)


def _sharded_file_worker(rank, world, port, prefix):
    import sys

    sys.path.insert(0, REPO)
    from ip_mcmc_amd.shard import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(C_TOTAL, 4))
    res = run_sharded(_lin_sampler_factory(), u0, n_samples=6, burn_in=9, sample_interval=4, keep="samples",
                      sample_file=prefix)
    assert "samples" not in res and res["u"].shape == (C_TOTAL, 4)
    dist.barrier()
    dist.destroy_process_group()


def test_run_sharded_streams_each_ranks_samples_to_its_own_file(tmp_path):
    """keep='samples' with sample_file: rank r streams its block of chains to
    <prefix>.rank<r>.npy; the files concatenated in rank order are the
    one-process samples."""
    from ip_mcmc_amd.shard import chain_range

    prefix = str(tmp_path / "chains")
    mp.start_processes(_sharded_file_worker, args=(3, _free_port(), prefix), nprocs=3, start_method="spawn")
    parts = [np.load(f"{prefix}.rank{r}.npy") for r in range(3)]
    assert [p.shape[0] for p in parts] == [b - a for a, b in (chain_range(C_TOTAL, r, 3) for r in range(3))]
    u0 = 0.1 * np.random.default_rng(1).normal(size=(C_TOTAL, 4))
    one = _lin_sampler_factory()(0).run(u0, n_samples=6, burn_in=9, sample_interval=4)
    np.testing.assert_array_equal(np.concatenate(parts, axis=0), one)
