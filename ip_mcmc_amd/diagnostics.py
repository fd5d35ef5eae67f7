"""Chain diagnostics on the device.

  autocorr(x, max_lag)            batched MCMCSampler.autocorr (sampler.py:43-54)
  autocorrelation(samples, tau)   helpers.autocorrelation (report/scripts/helpers.py:41-54)
  chain_autocorr(samples, lag)    per chain and component, for run()'s (C, n_samples, k) output
  burn_in_lengths(chains)         batched len_burn_in (burgers/utilities.py:134-167), ipmc_burn_in kernel
  len_burn_in / uncorrelated_sample_spacing / clean_samples   utilities.py:134-195, reference signatures

The autocorrelations call libipmc's ``ipmc_autocorr`` kernel (one workgroup
per series, the series staged in LDS); results agree with the reference's
np.correlate formula to rounding (the summation order differs).  Burn-in
detection calls ``ipmc_burn_in``, which keeps np.cumsum's and np.mean's
summation orders, so its moving averages and decisions equal the
reference's bit for bit.
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


# ------------------------------------------------------------------ burn-in
def burn_in_lengths(chains, avg_window=50, accepted_change=0.03, layout="vars_time", device=None):
    """len_burn_in (burgers/utilities.py:134-167) for a batch of chains on the device.

    chains: (C, n_vars, n) with layout='vars_time' (the reference's x, one per
    chain), or run()'s (C, n_samples, k) output with layout='time_vars'.
    Returns int64 (C,) (numpy for numpy input)."""
    numpy_in = not (isinstance(chains, torch.Tensor) and chains.is_cuda)
    t = _series_tensor(chains, device)
    if t.dtype not in (torch.float32, torch.float64):
        t = t.double()
    if t.dim() == 2:
        t = t.unsqueeze(0)
    t = t.contiguous()
    C, a, b = t.shape
    if layout == "vars_time":
        n_vars, n, s_var, s_t = a, b, b, 1
    elif layout == "time_vars":
        n, n_vars, s_var, s_t = a, b, 1, b
    else:
        raise ValueError("layout must be 'vars_time' or 'time_vars'")
    if n < avg_window:
        raise ValueError(f"len_burn_in needs at least avg_window={avg_window} samples, got {n}")
    words = (n + 31) // 32
    flags = torch.empty(max(1, C * words), dtype=torch.int32, device=t.device)
    out = torch.empty(C, dtype=torch.int64, device=t.device)
    call("ipmc_burn_in", t.data_ptr(), dev.abi_dtype(t.dtype), C, n_vars, n, a * b, s_var, s_t, int(avg_window),
         float(accepted_change), flags.data_ptr(), out.data_ptr(), dev.stream_handle(t.device))
    return out.cpu().numpy() if numpy_in else out


def len_burn_in(x, device=None):
    """Reference signature (utilities.py:134): x (n_vars, n) -> burn-in index (int)."""
    return int(burn_in_lengths(np.asarray(x, dtype=np.float64)[None], device=device)[0])


def uncorrelated_sample_spacing(x, device=None):
    """utilities.py:169-186: grow tau by 1.5x from 10 until the variable-averaged
    windowed autocorrelation first drops to <= 0.001; returns that lag.  Keeps
    the reference's early exit value len(x) (the number of variables)
    when the series is too short to decorrelate."""
    x = np.asarray(x, dtype=np.float64)
    tau = 10
    while True:
        if 2 > int(len(x[0, :]) / tau):
            return len(x)
        tau = int(tau * 1.5)
        ac = autocorrelation(x, tau, device)
        avg_ac = np.mean(ac, axis=0)
        idx = np.argwhere(avg_ac <= 0.001)
        if len(idx) > 0:
            return idx[0][0]


def clean_samples(x, device=None):
    """utilities.py:189-195: drop the burn-in, then keep every spacing-th sample."""
    x_ = np.copy(np.asarray(x, dtype=np.float64))
    x_ = x_[:, len_burn_in(x_, device):]
    return x_[:, :: uncorrelated_sample_spacing(x_, device)]
