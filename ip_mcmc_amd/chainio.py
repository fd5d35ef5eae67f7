"""On-disk chains and exact resume.

The reference memoises whole chains as ``.npy`` (helpers.py:23-38,
``load_or_compute``) and callers transpose them to (k, n) (burgers_beta.py:170).
Here:

  * ``load_or_compute(path, function, args)`` — same contract (np.load if the
    file exists, otherwise compute, np.save and return).
  * ``NpySampleSink(path, shape)`` — a np.load-compatible ``.npy`` file (via
    ``np.lib.format.open_memmap``) that ``MCMCSampler.run(..., sample_file=)``
    fills block by block as samples leave the GPU, so an ensemble whose
    samples exceed host memory still streams to disk.
  * ``ChainState`` / ``save_state`` / ``load_state`` — the sampler's full
    state (u, cached Φ or I, accept/call counters, Philox seed and global step,
    the variable-step proposer's counter).  Because every draw is a function of
    (seed, global chain id, global step), ``run(state, ...)`` continues a chain
    bit for bit as if it had never stopped.
"""
import os

import numpy as np


def load_or_compute(path, function, args):
    """helpers.py:23-38: load ``path`` (.npy) if present, else compute and save."""
    p = path if path.endswith(".npy") else path + ".npy"
    if os.path.exists(p):
        return np.load(p, allow_pickle=False)
    res = function(*args)
    np.save(p, res)
    return res


class NpySampleSink:
    """A .npy file of float64 samples, (n_samples, k) for one chain (the
    reference's layout) or (C, n_samples, k) for C chains."""

    def __init__(self, path, shape):
        self.path = path if path.endswith(".npy") else path + ".npy"
        self.shape = tuple(int(s) for s in shape)
        self.mm = np.lib.format.open_memmap(self.path, mode="w+", dtype=np.float64, shape=self.shape)

    def write(self, i0, block):
        """block: (C, b, k) samples i0 .. i0+b-1 (or (b, k) for one chain)."""
        block = np.asarray(block, dtype=np.float64)
        if len(self.shape) == 2:
            self.mm[i0 : i0 + block.shape[-2]] = block.reshape(-1, self.shape[1])
        else:
            self.mm[:, i0 : i0 + block.shape[1]] = block

    def close(self):
        self.mm.flush()
        return np.load(self.path, mmap_mode="r", allow_pickle=False)


class ChainState:
    """Everything needed to continue a run exactly (host numpy arrays).  A run
    with results='device' leaves the chain states in HBM: ``u`` is then copied
    to the host on first access, and ``u_device`` is the device tensor (what a
    resumed run starts from, without a round trip)."""

    def __init__(self, u, phi, accepts, calls, seed, step, proposer_i, dtype, chain_offset=None, accept_kind=None):
        if hasattr(u, "is_cuda") and u.is_cuda:
            self.u_device, self._u = u, None
        else:
            self.u_device, self._u = None, np.asarray(u)
        self.phi = np.asarray(phi)
        self.accepts = np.asarray(accepts)
        self.calls = None if calls is None else np.asarray(calls)
        self.seed = int(seed)
        self.step = int(step)
        self.proposer_i = int(proposer_i)
        self.dtype = str(dtype)
        # global id of chain 0 (the Philox streams) and the cached potential's
        # kind ('pcn': Φ, 'rw_reg': Φ + StandardRWAccepter's regularizer);
        # None for states written before they were recorded
        self.chain_offset = None if chain_offset is None else int(chain_offset)
        self.accept_kind = None if accept_kind is None else str(accept_kind)

    @property
    def u(self):
        if self._u is None:
            self._u = self.u_device.detach().cpu().numpy()
        return self._u

    @u.setter
    def u(self, value):
        self.u_device, self._u = None, np.asarray(value)

    @property
    def n_chains(self):
        return (self.u_device if self._u is None else self._u).shape[0]


def save_state(path, state):
    p = path if path.endswith(".npz") else path + ".npz"
    np.savez(
        p,
        u=state.u,
        phi=state.phi,
        accepts=state.accepts,
        calls=np.zeros(0, dtype=np.int64) if state.calls is None else state.calls,
        has_calls=np.array(state.calls is not None),
        seed=np.array(state.seed, dtype=np.uint64),
        step=np.array(state.step, dtype=np.int64),
        proposer_i=np.array(state.proposer_i, dtype=np.int64),
        dtype=np.array(state.dtype),
        chain_offset=np.array(-1 if state.chain_offset is None else state.chain_offset, dtype=np.int64),
        accept_kind=np.array("" if state.accept_kind is None else state.accept_kind),
    )
    return p


def load_state(path):
    p = path if path.endswith(".npz") else path + ".npz"
    z = np.load(p, allow_pickle=False)
    off = int(z["chain_offset"]) if "chain_offset" in z.files else -1
    kind = str(z["accept_kind"]) if "accept_kind" in z.files else ""
    return ChainState(
        z["u"], z["phi"], z["accepts"], z["calls"] if bool(z["has_calls"]) else None, int(z["seed"]),
        int(z["step"]), int(z["proposer_i"]), str(z["dtype"]), chain_offset=None if off < 0 else off,
        accept_kind=kind or None,
    )
