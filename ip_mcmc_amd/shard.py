"""Chain sharding across the GPUs of a node (one process per GPU).

Chains are independent (no exchange during sampling), so rank r of P owns a
contiguous block of global chain ids and passes its first id as
``chain_offset``: the counter-based draws are keyed by the GLOBAL chain id,
so every chain's trajectory is bitwise identical for any P.  The only
collective is the final gather of per-chain results to every rank
(``torch.distributed.all_gather_into_tensor``; backend "nccl" = RCCL over
xGMI on MI355X, "gloo" on CPU), followed by a host reduction in fixed global
chain order, so posterior means are also bitwise independent of P.
"""
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


def ordered_mean(x, block=1 << 16):
    """Mean over the chain axis (dim 0) in fixed sequential chain order, on the
    host in float64: identical for every sharding of the same chains.  The
    running sum ((0 + row_0) + row_1) + ... is np.cumsum along the chain axis
    (a strictly sequential accumulate), taken in blocks of rows so that the
    2^20-chain case needs no full-size temporary."""
    import numpy as np

    a = x.detach().double().cpu().numpy() if hasattr(x, "detach") else np.asarray(x, dtype=np.float64)
    acc = np.zeros(a.shape[1:], dtype=np.float64)
    for i in range(0, a.shape[0], block):
        blk = a[i : i + block].copy()
        blk[0] = acc + blk[0]
        acc = np.cumsum(blk, axis=0)[-1]
    return acc / a.shape[0]
