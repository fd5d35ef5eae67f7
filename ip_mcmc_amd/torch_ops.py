"""``torch.ops.ipmc`` — the TORCH_LIBRARY front end of libipmc.

The ops take tensors instead of raw pointers and run the same HIP kernels as
the C-ABI (``csrc/ipmc_torch.cpp`` validates the tensors and calls
``ipmc_pcn_sweep`` / ``ipmc_potential`` / ``ipmc_forward``); they are
registered for device tensors only, so a CPU tensor raises rather than falling
back.  ``model`` is the ``ipmc_model`` an ObservationOperator builds
(``op.model(dtype, device)``), passed by address; the default stream is torch's
current stream on the tensors' device.

    from ip_mcmc_amd import torch_ops
    torch_ops.pcn_sweep(op, u, phi, accepts, y, gamma_inv, prior_sqrt, beta=0.2, seed=1, step0=0, n_steps=10)
"""
import ctypes as C
import math
import os

import torch

from ._lib import lib as _ipmc_lib

TORCH_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libipmc_torch.so")
_loaded = False


def load():
    """Load libipmc_torch.so (registers torch.ops.ipmc); raises if it is missing."""
    global _loaded
    if not _loaded:
        if not os.path.exists(TORCH_LIB_PATH):
            raise RuntimeError(f"{TORCH_LIB_PATH} not found; build it with __graft_entry__.build()")
        _ipmc_lib()  # libipmc.so first (the ABI version check lives there)
        torch.ops.load_library(TORCH_LIB_PATH)
        from . import _abi

        v = int(torch.ops.ipmc.abi_version())
        if v != _abi.ABI_VERSION:
            raise RuntimeError(f"libipmc_torch.so was built against ABI {v}, the package is ABI {_abi.ABI_VERSION}: "
                               "rebuild it with __graft_entry__.build()")
        _loaded = True
    return torch.ops.ipmc


def _model_address(op, dtype, device):
    """Address of op's ipmc_model for (dtype, device); the operator caches it
    with its device arrays for its own lifetime."""
    m, _ = op.model(dtype, device)
    return C.addressof(m)


def _stream(t, stream):
    return torch.cuda.current_stream(t.device).cuda_stream if stream is None else int(stream)


def _require_device(u):
    """The ops have no CPU kernel: a host tensor raises here, before any
    model arrays are built for it (torch's dispatcher raises the same for
    the raw ops)."""
    if u.device.type != "cuda":
        raise NotImplementedError(f"torch.ops.ipmc runs on ROCm device tensors only, got a {u.device.type} tensor")


def pcn_sweep(op, u, phi, accepts, y, gamma_inv, prior_sqrt, beta, seed, step0, n_steps, chain_offset=0,
              proposal="pcn", sum_u=None, sum_u2=None, stream=None):
    """n_steps pCN (or RW) steps of every chain of u [C, k], in place; see include/ipmc.h ipmc_pcn_sweep."""
    ops = load()
    _require_device(u)
    contraction = math.sqrt(1.0 - beta * beta) if proposal == "pcn" else 1.0
    ops.pcn_sweep(u, phi, accepts, y, gamma_inv, prior_sqrt, _model_address(op, u.dtype, u.device),
                  float(beta), contraction, int(seed), int(chain_offset), int(step0), int(n_steps),
                  _stream(u, stream), 1 if proposal == "rw" else 0, sum_u, sum_u2)


def potential(op, u, y, gamma_inv, stream=None):
    """Φ(u) for u [n, k] (device tensor) -> phi [n]."""
    ops = load()
    _require_device(u)
    phi = torch.empty(u.shape[0], dtype=u.dtype, device=u.device)
    ops.potential(u, y, gamma_inv, phi, _model_address(op, u.dtype, u.device), _stream(u, stream))
    return phi


def forward(op, u, stream=None):
    """G(u) for u [n, k] (device tensor) -> g [n, q]."""
    ops = load()
    _require_device(u)
    g = torch.empty((u.shape[0], op.q), dtype=u.dtype, device=u.device)
    ops.forward(u, g, _model_address(op, u.dtype, u.device), _stream(u, stream))
    return g
