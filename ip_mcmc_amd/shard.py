"""Chain sharding across the GPUs of a node (one process per GPU).

Chains are independent (no exchange during sampling), so rank r of P owns a
contiguous block of global chain ids and passes its first id as
``chain_offset``: the counter-based draws are keyed by the GLOBAL chain id,
so every chain's trajectory is bitwise identical for any P.  The only
collective is the final gather of per-chain results to every rank
(``torch.distributed.all_gather_into_tensor``; backend "nccl" = RCCL over
xGMI on MI355X, "gloo" on CPU) and a reduction in fixed global chain order
(fixed blocks of chains summed in parallel -- on the device when the sums
are, ipmc_block_sums -- then the block sums in order; ipmc_host_ordered_sum
gives the host the same bits), so posterior means are also bitwise
independent of P.
"""
import os

import numpy as np
import torch
import torch.distributed as dist


def chain_range(n_total, rank, world):
    """Contiguous balanced block [start, stop) of global chain ids for `rank`."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_chains(local, n_total, group=None):
    """All-gather per-chain rows (first dim = the rank's chains, in rank
    order) into the full [n_total, ...] tensor on every rank."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    per = max(chain_range(n_total, r, world)[1] - chain_range(n_total, r, world)[0] for r in range(world))
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((per * world,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad.contiguous(), group=group)
    parts = []
    for r in range(world):
        a, b = chain_range(n_total, r, world)
        parts.append(out[r * per : r * per + (b - a)])
    return torch.cat(parts, dim=0)


# Chains per block of the posterior-mean sum.  Fixed, so the order of the
# additions -- and the bits of the mean -- does not depend on how the chains
# are sharded; the blocks are summed in parallel.
MEAN_BLOCK = 1024


def ordered_mean(x, div=1.0, block=MEAN_BLOCK):
    """Mean over the chain axis (dim 0) in a fixed order (block_sum), on the
    host in float64: identical for every sharding of the same chains."""
    a = x.detach().double().cpu().numpy() if hasattr(x, "detach") else np.asarray(x, dtype=np.float64)
    return block_sum(a, div, block) / a.shape[0]


def block_sum(a, div=1.0, block=MEAN_BLOCK):
    """The posterior mean's sum over the chain axis in its fixed order: the rows
    of each block of `block` consecutive chains added from zero in row order
    (S_b = ((0 + x_bB/div) + x_bB+1/div) + ...), then the block sums in block
    order ((0 + S_0) + S_1) + ... .  One block (<= `block` chains) is the plain
    sequential sum.  ordered_sum_sharded forms the same additions over the
    ranks' rows (device: ipmc_block_sums), so the bits do not depend on the
    number of ranks."""
    a = np.asarray(a, dtype=np.float64)
    k = int(np.prod(a.shape[1:], dtype=np.int64))
    rows = a.reshape(a.shape[0], k)
    return _seq_sum(_host_block_sums(rows, div, block), np.zeros(k)).reshape(a.shape[1:])


def _host_block_sums(rows, div, block):
    """[ceil(n / block), k]: each block's rows from zero in row order
    (ipmc_host_ordered_sum; ipmc_block_sums is the device twin)."""
    nb = -(-rows.shape[0] // block)
    out = np.empty((nb, rows.shape[1]), dtype=np.float64)
    for b in range(nb):
        out[b] = _seq_sum(rows[b * block : (b + 1) * block], np.zeros(rows.shape[1]), div)
    return out


def _seq_sum(a, acc, div=1.0):
    """acc + a[0]/div + a[1]/div + ... strictly in row order (in place)."""
    from . import _hostlib

    a = np.asarray(a, dtype=np.float64)
    acc = np.ascontiguousarray(acc, dtype=np.float64).reshape(-1).copy()
    if a.shape[0]:
        _hostlib.ordered_sum(a.reshape(a.shape[0], -1), acc, div)
    return acc.reshape(a.shape[1:])


def _split(lo, hi, block):
    """[lo, hi) against the blocks of `block` rows: (head, (b0, b1), tail) --
    the whole blocks b0..b1-1 and the rows (start, stop) before and after them
    that share a block with other ranks (None where there are none)."""
    fb, lb = -(-lo // block), hi // block
    if fb > lb:  # inside one block, no boundary in between
        return ((lo, hi) if hi > lo else None), (0, 0), None
    head = (lo, fb * block) if lo < fb * block else None
    tail = (lb * block, hi) if lb * block < hi else None
    return head, (fb, lb), tail


def _rank_parts(rows, lo, block, div=1.0):
    """A rank's contribution to the posterior mean's block sums, for its rows
    [lo, lo + n) of the global chain order: (F, shared) -- F the sums of its
    whole blocks (device rows: ipmc_block_sums, queued on the current stream),
    shared the rows of the at most two blocks it shares with other ranks."""
    n, k = int(rows.shape[0]), int(rows.shape[1])
    head, (b0, b1), tail = _split(lo, lo + n, block)
    on_dev = isinstance(rows, torch.Tensor) and rows.is_cuda
    if b1 > b0:
        f0, f1 = b0 * block - lo, b1 * block - lo
        if on_dev:
            from . import device as D

            F = D.block_sums(rows[f0:f1], block, div)
        else:
            F = _host_block_sums(rows[f0:f1], div, block)
    else:
        F = torch.zeros((0, k), dtype=torch.float64, device=rows.device) if on_dev else np.zeros((0, k))
    return F, [rows[seg[0] - lo : seg[1] - lo] for seg in (head, tail) if seg is not None]


def _to_host_async(t):
    """A device tensor's page-locked host copy, queued on the current stream
    (valid once the stream is synchronised)."""
    h = torch.empty(tuple(t.shape), dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    return h


def ordered_sum_sharded(local, group=None, div=1.0, block=MEAN_BLOCK, parts=None):
    """block_sum over the chains of all ranks in global (rank) order, each rank
    holding its own rows: a rank sums its whole blocks (on the device when
    `local` is a CUDA tensor: ipmc_block_sums, one launch) and contributes those
    sums plus the raw rows of the (at most two) blocks it shares with other
    ranks to one all_gather; every rank then finishes the same additions on the
    host (the shared blocks' rows in rank order, then the block sums in block
    order).  Bit-identical to block_sum over the gathered rows, without
    gathering them (config 5's per-chain sums are 4 GB), and no rank waits on
    another's sum: one all_gather of ~k / block of the data instead of P - 1
    sequential hops.  parts: this rank's (F, shared) already formed and on
    the host (_rank_parts at the rank's global offset; run_sharded queues them
    before the run's synchronisation)."""
    rank, world = world_info(group)
    on_dev = isinstance(local, torch.Tensor) and local.is_cuda
    shape = tuple(local.shape[1:])
    k = int(np.prod(shape, dtype=np.int64))
    if on_dev:
        rows = local.reshape(local.shape[0], k)
    else:
        a = local.detach().cpu().numpy() if isinstance(local, torch.Tensor) else local
        rows = np.asarray(a, dtype=np.float64).reshape(len(a), k)
    n_local = int(rows.shape[0])
    comm = _dist_on()
    if comm:  # (a one-rank process group too: the collectives run, over RCCL on the GPU)
        dev = _comm_device(group)
        counts = torch.empty(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(counts, torch.tensor([n_local], dtype=torch.int64, device=dev), group=group)
        counts = counts.cpu().tolist()
    else:
        counts = [n_local]
    los = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    lo = int(los[rank])
    if parts is None:  # this rank's whole blocks in one call, its shared rows
        F, shared = _rank_parts(rows, lo, block, div)
        F = F.cpu().numpy() if on_dev else F
        shared = [p.cpu().numpy() if on_dev else p for p in shared]
    else:
        F, shared = parts
    mine = np.concatenate([F.reshape(-1)] + [p.reshape(-1) for p in shared]) if (len(F) or shared) else np.zeros(0)

    def size(r):  # every rank's contribution, known from the counts alone
        h, (c0, c1), t = _split(int(los[r]), int(los[r + 1]), block)
        return ((c1 - c0) + sum(seg[1] - seg[0] for seg in (h, t) if seg is not None)) * k

    if comm:
        per = max(max(size(r) for r in range(world)), 1)
        buf = torch.zeros(per, dtype=torch.float64, device=dev)
        buf[: mine.size] = torch.from_numpy(mine).to(dev)
        allb = torch.empty(per * world, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allb, buf, group=group)
        allb = allb.cpu().numpy().reshape(world, per)
        parts = [allb[r] for r in range(world)]
    else:
        parts = [mine]
    n_total = int(los[-1])
    sums = np.zeros((-(-n_total // block), k), dtype=np.float64)
    pieces = {}
    for r in range(world):
        h, (c0, c1), t = _split(int(los[r]), int(los[r + 1]), block)
        sums[c0:c1] = parts[r][: (c1 - c0) * k].reshape(c1 - c0, k)
        off = (c1 - c0) * k
        for seg in (h, t):  # head rows, then tail rows: global row order
            if seg is not None:
                m = (seg[1] - seg[0]) * k
                pieces.setdefault(seg[0] // block, []).append(parts[r][off : off + m].reshape(seg[1] - seg[0], k))
                off += m
    for b, pc in pieces.items():  # a block over several ranks: its rows in rank order, from zero
        sums[b] = _seq_sum(np.concatenate(pc), np.zeros(k), div)
    return _seq_sum(sums, np.zeros(k)).reshape(shape)


def _dist_on():
    """A process group is initialised: the gathers run as collectives (RCCL
    with backend "nccl") even for a one-rank group."""
    return dist.is_available() and dist.is_initialized()


def world_info(group=None):
    """(rank, world size) of this process: the initialised process group, else
    RANK / WORLD_SIZE from the environment (torchrun), else (0, 1)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def _comm_device(group):
    """Where a collective's tensors live: the rank's GPU for RCCL ("nccl"),
    host memory for gloo."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def local_start(u_0, n_total, rank, world):
    """This rank's block of starting states, rows chain_range(C_total, rank,
    world), and C_total.  u_0 is one of
      * the full ensemble (C_total, k) (n_total None or C_total): its rows
        [lo, hi) are read (a memory-mapped .npy reads only those);
      * a callable u_0(lo, hi) -> (hi - lo, k) (n_total required): the rank
        builds only its own rows;
      * this rank's own block (hi - lo, k) with n_total = C_total given: no
        rank holds another's rows (per-rank memory stays
        C_total / P whatever the node's ensemble)."""
    if callable(u_0) and not isinstance(u_0, (np.ndarray, torch.Tensor)):
        if n_total is None:
            raise ValueError("a callable u_0(lo, hi) needs n_total (the node's chain count)")
        lo, hi = chain_range(int(n_total), rank, world)
        block = u_0(lo, hi)
        if len(np.shape(block)) != 2 or np.shape(block)[0] != hi - lo:
            raise ValueError(f"u_0({lo}, {hi}) must return ({hi - lo}, k) rows, got shape {np.shape(block)}")
        return block, int(n_total)
    if len(np.shape(u_0)) != 2:
        raise ValueError("run_sharded needs u_0 of shape (chains, k)")
    rows = int(np.shape(u_0)[0])
    n_total = rows if n_total is None else int(n_total)
    lo, hi = chain_range(n_total, rank, world)
    if rows == n_total:  # the full ensemble: this rank's rows of it
        return u_0[lo:hi], n_total
    if rows != hi - lo:
        raise ValueError(f"u_0 has {rows} rows: neither the {n_total} chains of the node nor rank {rank}'s "
                         f"{hi - lo} (chain_range({n_total}, {rank}, {world}))")
    return u_0, n_total


def run_sharded(make_sampler, u_0, n_samples, burn_in=1000, sample_interval=200, keep="moments", group=None,
                sample_file=None, gather="all", results="host", n_total=None):
    """MCMCSampler.run over the chains of every rank of a node, one process per GPU.

    make_sampler(chain_offset=...) builds this rank's sampler (the same
    proposer / accepter / potential / rng seed on every rank; the sampler's
    chain_offset must be the one passed).  u_0 gives the starting states:
    the full ensemble (C_total, k) on every rank (an array, e.g. a
    memory-mapped .npy; each rank reads only its block of rows), or -- with
    n_total=C_total -- only this rank's block (hi - lo, k) or a callable
    u_0(lo, hi) returning it (local_start), so that no rank allocates the
    node's ensemble.  Rank r runs the
    chains chain_range(C_total, r, P) -- global ids, so every chain's
    trajectory is the one-process run's bit for bit -- and the per-chain
    results of all ranks are gathered by one all_gather_into_tensor (RCCL over
    xGMI with backend "nccl", gloo on CPU) into global chain order.

    Returns a dict on every rank:
      "u", "phi", "accepts"   the final chain states (C_total, k), Φ, accept counts
      keep="moments": "sum_u", "sum_u2" (C_total, k) and "n", plus "mean"
                     (the posterior-mean estimate: the per-chain sums added
                     over the chains in a fixed order, block_sum, over
                     n x C_total -- bit-identical for any number of ranks)
      keep="samples": "samples" (C_total, n_samples, k); with sample_file each
                     rank streams its own block to f"{sample_file}.rank{r}.npy"
                     and nothing is gathered but the state
      keep="last":   "last" (C_total, k)
      "rank", "world", "chain_range", "local" (this rank's own run() result),
      "sampler" (this rank's sampler, state included), "run_seconds" (this
      rank's run()), "gather_seconds".
    gather="mean" (keep="moments" only) gathers just Φ and the accept counts
    and forms "mean" by ordered_sum_sharded (block sums), for ensembles
    whose per-chain arrays are too large to copy to every rank (config 5:
    2^20 chains x 256); "u", "sum_u", "sum_u2" are then this rank's rows only.
    results="device" (with gather="mean"): the rank's per-chain results stay
    in HBM ("u", "sum_u", "sum_u2" are this rank's device tensors; u_0 may be
    a device tensor) -- a job that starts and ends in HBM, no PCIe on the data
    path; "mean", "phi" and "accepts" are host arrays as before.
    With one rank (no process group) it is a plain run()."""
    import time

    rank, world = world_info(group)
    if world > 1 and not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("run_sharded with WORLD_SIZE > 1 needs an initialised process group "
                           "(torch.distributed.init_process_group('nccl') on the GPUs, 'gloo' on CPU)")
    if gather not in ("all", "mean"):
        raise ValueError("gather must be 'all' or 'mean'")
    if gather == "mean" and keep != "moments":
        raise ValueError("gather='mean' needs keep='moments'")
    if results == "device" and gather != "mean":
        raise ValueError("results='device' needs gather='mean' (the per-chain rows stay on their rank)")
    local_u0, n_total = local_start(u_0, n_total, rank, world)
    lo, hi = chain_range(n_total, rank, world)
    sampler = make_sampler(chain_offset=lo)
    if sampler.chain_offset != lo:
        raise ValueError(f"make_sampler must build the sampler with chain_offset={lo}, got {sampler.chain_offset}")
    # gather="mean": the posterior mean's block sums run on the device sums the
    # sweeps left (MCMCSampler.last_device_sums) when the run was a device run,
    # queued before the run's one synchronisation (pre_sync), their host copies
    # page-locked
    sampler.keep_device_sums = gather == "mean"
    if gather == "mean":
        def _queue_block_sums(sums):
            F, shared = _rank_parts(sums[0], lo, MEAN_BLOCK)
            return [_to_host_async(F)] + [_to_host_async(p) for p in shared]

        sampler.pre_sync = _queue_block_sums
    if not isinstance(local_u0, torch.Tensor):
        local_u0 = np.asarray(local_u0, dtype=np.float64)
    sf = None if sample_file is None else f"{sample_file}.rank{rank}.npy"
    t0 = time.perf_counter()
    res = sampler.run(local_u0, n_samples, burn_in=burn_in, sample_interval=sample_interval, keep=keep,
                      sample_file=sf, results=results)
    run_s = time.perf_counter() - t0
    st = sampler.state
    k = local_u0.shape[1]
    u_rows = st.u_device if st.u_device is not None else np.asarray(st.u, dtype=np.float64).reshape(hi - lo, k)
    cols = [u_rows,
            np.asarray(st.phi, dtype=np.float64).reshape(hi - lo, 1),
            np.asarray(st.accepts, dtype=np.float64).reshape(hi - lo, 1)]  # counts < 2^53: exact
    if gather == "mean":
        t1 = time.perf_counter()
        if _dist_on():
            small = np.concatenate(cols[1:], axis=1)
            small = gather_chains(torch.from_numpy(np.ascontiguousarray(small)).to(_comm_device(group)), n_total,
                                  group).cpu().numpy()
            phi_all, acc_all = small[:, 0], small[:, 1].astype(np.int64)
        else:  # one rank: this process's arrays are the result
            phi_all, acc_all = cols[1][:, 0], np.asarray(st.accepts, dtype=np.int64)
        n = max(1, res["n"])
        dsum = getattr(sampler, "last_device_sums", None)
        rows = dsum[0] if dsum is not None else res["sum_u"].reshape(hi - lo, k)
        pre = sampler.pre_sync_result if dsum is not None else None
        parts = None if pre is None else (pre[0].numpy(), [p.numpy() for p in pre[1:]])
        mean = ordered_sum_sharded(rows, group, parts=parts) / (float(n) * n_total)
        sampler.last_device_sums = sampler.pre_sync = sampler.pre_sync_result = None
        # a device state is the checkpoint's own tensor (in the run's dtype):
        # hand out an f64 copy, as the host path and MCMCSampler.run(keep='last') do
        u_out = cols[0].to(torch.float64, copy=True) if isinstance(cols[0], torch.Tensor) else cols[0]
        return {"u": u_out, "phi": phi_all, "accepts": acc_all, "sum_u": res["sum_u"],
                "sum_u2": res["sum_u2"], "n": res["n"], "mean": mean, "rank": rank, "world": world,
                "chain_range": (lo, hi), "local": res, "sampler": sampler, "run_seconds": run_s,
                "gather_seconds": time.perf_counter() - t1}
    t1 = time.perf_counter()
    out = {"rank": rank, "world": world, "chain_range": (lo, hi), "local": res, "sampler": sampler,
           "run_seconds": run_s}
    if not _dist_on():  # no process group, one rank: this process's arrays are the result
        out.update(u=cols[0], phi=cols[1][:, 0], accepts=np.asarray(st.accepts, dtype=np.int64))
        if keep == "moments":
            out.update(sum_u=res["sum_u"].reshape(hi - lo, k), sum_u2=res["sum_u2"].reshape(hi - lo, k), n=res["n"])
        elif keep == "samples" and sf is None:
            out["samples"] = np.asarray(res, dtype=np.float64).reshape(hi - lo, -1, k)
        elif keep == "last":
            out["last"] = np.asarray(res, dtype=np.float64).reshape(hi - lo, k)
    else:
        if keep == "moments":
            cols += [res["sum_u"].reshape(hi - lo, k), res["sum_u2"].reshape(hi - lo, k)]
        elif keep == "samples" and sf is None:
            cols.append(np.asarray(res, dtype=np.float64).reshape(hi - lo, -1))
        elif keep == "last":
            cols.append(np.asarray(res, dtype=np.float64).reshape(hi - lo, k))
        packed = np.concatenate(cols, axis=1) if hi > lo else np.zeros((0, sum(c.shape[1] for c in cols)))
        full = gather_chains(torch.from_numpy(np.ascontiguousarray(packed)).to(_comm_device(group)), n_total,
                             group).cpu().numpy()
        out.update(u=full[:, :k], phi=full[:, k], accepts=full[:, k + 1].astype(np.int64))
        rest = full[:, k + 2:]
        if keep == "moments":
            out.update(sum_u=rest[:, :k], sum_u2=rest[:, k:2 * k], n=res["n"])
        elif keep == "samples" and sf is None:
            out["samples"] = rest.reshape(n_total, -1, k)
        elif keep == "last":
            out["last"] = rest
    if keep == "moments":
        # Σ over chains (block_sum's fixed order) of the per-chain sums, / (steps × chains) once
        S = block_sum(np.asarray(out["sum_u"]))
        out["mean"] = S / (float(max(1, res["n"])) * n_total)
    out["gather_seconds"] = time.perf_counter() - t1
    return out
