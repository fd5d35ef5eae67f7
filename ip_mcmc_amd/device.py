"""Device plumbing: torch tensors for HBM buffers, the current HIP stream, and
thin wrappers over the libipmc entry points that are not the sweep itself.

PyTorch is used only for memory, streams and torch.distributed; all compute is
libipmc's HIP kernels.
"""
import numpy as np
import torch

from . import _abi
from ._lib import call

F32 = torch.float32
F64 = torch.float64


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("ip_mcmc_amd needs a ROCm GPU (torch.cuda.is_available() is False)")


def resolve_device(device=None):
    require_gpu()
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"device must be a cuda (ROCm) device, got {d}")
    if d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def torch_dtype(dtype):
    if dtype in (None, np.float64, "float64", "f64", torch.float64, float):
        return F64
    if dtype in (np.float32, "float32", "f32", torch.float32):
        return F32
    raise ValueError(f"unsupported dtype {dtype!r} (float32 or float64)")


def abi_dtype(tdtype):
    return _abi.F64 if tdtype == F64 else _abi.F32


def stream_handle(device):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def to_device(x, dtype, device):
    """numpy / list / tensor -> contiguous tensor of `dtype` on `device`."""
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.asarray(x, dtype=np.float64), dtype=dtype).to(device).contiguous()


# small read-only problem constants (y, 1/γ, sqrt diag C, ...) by content: a
# run() re-uses the device copy of the same values instead of a synchronous
# host-to-device copy each (three of them were ~0.1 ms of an 8 192-chain
# run's set-up, during which the GPU waits)
_CONST_MAX_BYTES = 1 << 16
_CONST_CACHE = {}


def const_to_device(x, dtype, device):
    """to_device for a small array the kernels only read: the device copy is
    shared by every call with the same values, dtype and device.  Callers
    must not write to the result.  Arrays above 64 KiB are copied as usual."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if a.nbytes > _CONST_MAX_BYTES:
        return to_device(a, dtype, device)
    key = (a.shape, a.tobytes(), str(dtype), str(device))
    t = _CONST_CACHE.get(key)
    if t is None:
        if len(_CONST_CACHE) >= 256:
            _CONST_CACHE.clear()
        t = _CONST_CACHE[key] = to_device(a, dtype, device)
    return t


def rect_copy_available():
    """The block-wise sample copy goes through libipmc (ipmc_copy_rows_d2h),
    which runs on the HIP runtime the caller's streams belong to: always
    available once the library loads."""
    return True


def copy_rows_d2h(dst, dst_pitch, src, src_pitch, width, rows, stream):
    """Asynchronous rectangular copy device -> (page-locked) host on `stream`:
    `rows` rows of `width` bytes, row r from src + r*src_pitch to
    dst + r*dst_pitch (ipmc_copy_rows_d2h = hipMemcpy2DAsync inside libipmc)."""
    if rows <= 0 or width <= 0:
        return
    call("ipmc_copy_rows_d2h", dst, dst_pitch, src, src_pitch, width, rows, stream)


def ordered_sum(rows, acc, div=1.0):
    """DEPRECATED (ABI 13; not on the product path: the posterior mean is
    block_sums + the block sums in order, shard.ordered_sum_sharded).
    acc (device f64 [k], in place) + rows[0]/div + rows[1]/div + ... strictly
    in row order on the device (ipmc_ordered_sum, the current stream): the bits
    of the host library's ipmc_host_ordered_sum.  rows: device f64 [n, k] with
    unit column stride."""
    if rows.dtype != torch.float64 or acc.dtype != torch.float64 or rows.dim() != 2:
        raise ValueError("ordered_sum needs f64 rows [n, k] and an f64 acc")
    if acc.shape != (rows.shape[1],) or not acc.is_contiguous() or acc.device != rows.device:
        raise ValueError("ordered_sum: acc must be a contiguous [k] tensor on the rows' device")
    if rows.shape[0] == 0 or rows.shape[1] == 0:
        return acc
    if rows.stride(1) != 1:
        raise ValueError("ordered_sum needs rows with contiguous columns")
    call("ipmc_ordered_sum", rows.data_ptr(), rows.shape[0], rows.shape[1], rows.stride(0), float(div),
         acc.data_ptr(), stream_handle(rows.device))
    return acc


def block_sums(rows, block, div=1.0):
    """out[b] = rows[bB]/div + rows[bB+1]/div + ... from zero in row order over
    each block of B = `block` consecutive rows (the last one possibly shorter),
    on the device (ipmc_block_sums, the current stream): the bits of the host
    library's ipmc_host_ordered_sum on each block.  rows: device f64 [n, k] with
    unit column stride; returns a new device f64 [ceil(n / B), k]."""
    if rows.dtype != torch.float64 or rows.dim() != 2:
        raise ValueError("block_sums needs f64 rows [n, k]")
    if block <= 0:
        raise ValueError("block_sums: block must be positive")
    n, k = rows.shape
    out = torch.empty(((n + block - 1) // block, k), dtype=torch.float64, device=rows.device)
    if n == 0 or k == 0:
        return out
    if rows.stride(1) != 1:
        raise ValueError("block_sums needs rows with contiguous columns")
    call("ipmc_block_sums", rows.data_ptr(), n, k, rows.stride(0), int(block), float(div), out.data_ptr(),
         stream_handle(rows.device))
    return out


def normals(seed, chain_offset, n_chains, step, k, dtype=None, device=None):
    device = resolve_device(device)
    td = torch_dtype(dtype)
    out = torch.empty((n_chains, k), dtype=td, device=device)
    call("ipmc_normal", seed, chain_offset, n_chains, step, k, abi_dtype(td), ptr(out), stream_handle(device))
    return out


def uniforms(seed, chain_offset, n_chains, step, device=None):
    device = resolve_device(device)
    out = torch.empty((n_chains,), dtype=F64, device=device)
    call("ipmc_uniform", seed, chain_offset, n_chains, step, ptr(out), stream_handle(device))
    return out
