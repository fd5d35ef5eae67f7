"""Chain diagnostics on the device.

  autocorr(x, max_lag)            batched MCMCSampler.autocorr (sampler.py:43-54)
  autocorrelation(samples, tau)   helpers.autocorrelation (report/scripts/helpers.py:41-54)
  chain_autocorr(samples, lag)    per chain and component, for run()'s (C, n_samples, k) output

All three call libipmc's ``ipmc_autocorr`` kernel (one workgroup per series,
the series staged in LDS); results agree with the reference's np.correlate
formula to rounding (the summation order differs).
"""
import numpy as np
import torch

from . import device as dev
from ._lib import call


def _series_tensor(x, device=None):
    if isinstance(x, torch.Tensor) and x.is_cuda:
        return x
    return torch.as_tensor(np.asarray(x, dtype=np.float64)).to(dev.resolve_device(device))


def autocorr(x, max_lag=None, device=None):
    """Normalised autocorrelation of every series along the last axis of x
    (numpy or device tensor, shape (..., n)); returns (..., max_lag) float64,
    numpy for numpy input.  max_lag defaults to n (the reference returns all n lags)."""
    numpy_in = not (isinstance(x, torch.Tensor) and x.is_cuda)
    t = _series_tensor(x, device)
    if t.dtype not in (torch.float32, torch.float64):
        t = t.double()
    shape = tuple(t.shape)
    n = shape[-1]
    lag = n if max_lag is None else int(max_lag)
    flat = t.reshape(-1, n).contiguous()
    out = torch.empty((flat.shape[0], lag), dtype=torch.float64, device=flat.device)
    call("ipmc_autocorr", flat.data_ptr(), dev.abi_dtype(flat.dtype), flat.shape[0], n, n, 1, lag, out.data_ptr(),
         dev.stream_handle(flat.device))
    out = out.reshape(shape[:-1] + (lag,))
    return out.cpu().numpy() if numpy_in else out


def autocorrelation(samples, tau_max, device=None):
    """helpers.autocorrelation (helpers.py:41-54): samples (n_vars, N) -> (n_vars, tau_max),
    the autocorrelation averaged over the N // tau_max consecutive windows of tau_max samples."""
    a = np.asarray(samples, dtype=np.float64)
    avg_over = int(len(a[0, :]) / tau_max)
    assert avg_over > 0, "Not enough samples to compute autocorrelationwith specified length"
    windows = a[:, : avg_over * tau_max].reshape(a.shape[0], avg_over, tau_max)
    ac_w = autocorr(windows, tau_max, device)  # (n_vars, avg_over, tau_max)
    ac = np.zeros((a.shape[0], tau_max))
    for i in range(avg_over):  # the reference's accumulation order
        ac += ac_w[:, i, :]
    return ac / avg_over


def chain_autocorr(samples, max_lag=None, device=None):
    """(C, n_samples, k) samples from MCMCSampler.run -> (C, k, max_lag) autocorrelations."""
    t = _series_tensor(samples, device)
    if t.dim() == 2:
        t = t.unsqueeze(0)
    return autocorr(t.transpose(1, 2).contiguous(), max_lag, device) if isinstance(samples, torch.Tensor) else (
        autocorr(t.transpose(1, 2).contiguous(), max_lag, device).cpu().numpy())
