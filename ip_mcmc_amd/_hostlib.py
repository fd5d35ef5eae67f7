"""Loader for ``ip_mcmc_amd/lib/libipmc_host.so`` (include/ipmc_host.h).

The pCN path's counter-based draws on the host CPU, compiled by g++ from the
kernels' own ``csrc/ipmc_rng.hpp`` (bit-identical to libipmc.so's
``ipmc_pcn_draws`` / ``ipmc_normal`` / ``ipmc_uniform``).  It needs no GPU: the
host step's randomness on a machine without one (BASELINE config 1).  Like
``_lib``, a missing library raises; there is no Python fallback.
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from ._lib import IpmcError

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libipmc_host.so")
ABI_VERSION = 1

_P = C.c_void_p
SIGNATURES = {
    "ipmc_host_abi_version": (C.c_int, []),
    "ipmc_host_last_error": (C.c_char_p, []),
    "ipmc_host_pcn_draws": (C.c_int, [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, C.c_int64, C.c_int32, C.c_int32,
                                      _P, _P, _P, _P, C.c_int32]),
    "ipmc_host_normal": (C.c_int, [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, C.c_int32, C.c_int32, _P]),
    "ipmc_host_uniform": (C.c_int, [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, _P]),
    "ipmc_host_step_uniforms": (C.c_int, [C.c_uint64, C.c_int64, C.c_uint64, C.c_int32, _P]),
    "ipmc_host_ordered_sum": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_int64, C.c_double, _P]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libipmc_host.so not found at {LIB_PATH}; build it first: "
                               "make -C ip_mcmc_amd/csrc host (g++ only, no ROCm needed)")
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
        v = h.ipmc_host_abi_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"libipmc_host ABI version {v} != {ABI_VERSION}")
        _lib = h
    return _lib


def call(name, *args):
    h = lib()
    rc = getattr(h, name)(*args)
    if rc != _abi.OK:
        raise IpmcError(name, rc, h.ipmc_host_last_error().decode(errors="replace"))
    return rc


def _ptr(a):
    return None if a is None else a.ctypes.data


def pcn_draws(seed, chain_offset, n_chains, step0, n_steps, k, np_dtype, prior_sqrt, prior_chol, n_threads=0):
    """(w [n_steps, C, k] in np_dtype, log r [n_steps, C] float64): the host
    twin of ipmc_pcn_draws."""
    T = np.dtype(np_dtype)
    sq = None if prior_sqrt is None else np.ascontiguousarray(prior_sqrt, dtype=np.float64).astype(T)
    ch = None if prior_chol is None else np.ascontiguousarray(prior_chol, dtype=np.float64).astype(T)
    w = np.empty((n_steps, n_chains, k), dtype=T)
    lr = np.empty((n_steps, n_chains), dtype=np.float64)
    call("ipmc_host_pcn_draws", seed, chain_offset, n_chains, step0, n_steps, k,
         _abi.F64 if T == np.float64 else _abi.F32, _ptr(sq), _ptr(ch), _ptr(w), _ptr(lr), int(n_threads))
    return w, lr


def normals(seed, chain_offset, n_chains, step, k, np_dtype=np.float64):
    """ξ [n_chains, k] of (seed, chain_offset + c, step): the host twin of ipmc_normal."""
    T = np.dtype(np_dtype)
    out = np.empty((n_chains, k), dtype=T)
    call("ipmc_host_normal", seed, chain_offset, n_chains, step, k, _abi.F64 if T == np.float64 else _abi.F32,
         _ptr(out))
    return out


def uniforms(seed, chain_offset, n_chains, step):
    """r [n_chains] in [0, 1): the host twin of ipmc_uniform."""
    out = np.empty(n_chains, dtype=np.float64)
    call("ipmc_host_uniform", seed, chain_offset, n_chains, step, _ptr(out))
    return out


def extra_uniforms(seed, chain, step, n):
    """The first n uniforms of one (chain, step): [0] is the accept uniform,
    [i] comes from Philox slot 0xFFFFFFFF - i."""
    out = np.empty(n, dtype=np.float64)
    call("ipmc_host_step_uniforms", seed, chain, step, n, _ptr(out))
    return out


def ordered_sum(rows, acc, div=1.0):
    """acc (k,) + rows[0]/div + rows[1]/div + ... strictly in row order, in place
    (rows: (n, k) float64, C-contiguous rows)."""
    a = np.ascontiguousarray(rows, dtype=np.float64).reshape(len(rows), -1) if len(rows) else None
    if a is None:
        return acc
    assert acc.dtype == np.float64 and acc.flags.c_contiguous and acc.shape[0] == a.shape[1]
    call("ipmc_host_ordered_sum", _ptr(a), a.shape[0], a.shape[1], a.shape[1], float(div), _ptr(acc))
    return acc
