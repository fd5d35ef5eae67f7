"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end of oracle/_build/liboracle.so, the plain-C CPU restatement of
the reference's pCN hot path (see ipmc_oracle.c).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
as the checker / the timed CPU baseline — never as a product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from ip_mcmc_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        h = C.CDLL(LIB_PATH)
        P = C.c_void_p
        h.orc_forward.argtypes = [C.POINTER(_abi.IpmcModel), C.c_int32, C.c_int64, P, P]
        h.orc_potential.argtypes = [C.POINTER(_abi.IpmcModel), C.c_int32, C.c_int64, P, P, P, P]
        h.orc_pcn_sweep.argtypes = [C.POINTER(_abi.IpmcModel), C.POINTER(_abi.IpmcSweep), C.c_int32]
        h.orc_normal_batch.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, C.c_int32, P]
        h.orc_normal_batch.restype = None
        h.orc_uniform_batch.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, P]
        h.orc_uniform_batch.restype = None
        h.orc_log_batch.argtypes = [C.c_int64, P, P]
        h.orc_log_batch.restype = None
        h.orc_sincos_batch.argtypes = [C.c_int64, P, P, P]
        h.orc_sincos_batch.restype = None
        h.orc_philox4x32_10.argtypes = [P, P, P]
        h.orc_philox4x32_10.restype = None
        h.orc_l96_rhs_f64.argtypes = [C.c_int32, C.c_int32, P, P, P]
        h.orc_l96_rhs_f64.restype = None
        h.orc_l96ts_rhs_f64.argtypes = [C.c_int32, C.c_int32, C.c_int32, P, P, P]
        h.orc_l96ts_rhs_f64.restype = None
        h.orc_rusanov_flux_f64.argtypes = [C.c_int32, C.c_double, C.c_double]
        h.orc_rusanov_flux_f64.restype = C.c_double
        h.orc_rusanov_rate_f64.argtypes = [C.c_int32, C.c_int32, P, C.c_double, P]
        h.orc_rusanov_rate_f64.restype = None
        _lib = h
    return _lib


def _np_dtype(dtype):
    return np.float32 if dtype in (np.float32, "float32", "f32", _abi.F32) else np.float64


def _abi_dtype(npd):
    return _abi.F32 if npd == np.float32 else _abi.F64


def _p(a):
    return None if a is None else a.ctypes.data


def model_struct(op, dtype):
    """IpmcModel on host arrays from a device ObservationOperator's parameters."""
    npd = _np_dtype(dtype)
    fields, reals, ints = op._spec()
    m = _abi.IpmcModel()
    m.kind = op.kind
    m.arith = _abi.ARITH_FMA if op.arith == "fma" else _abi.ARITH_REFERENCE
    m.k, m.q = op.k, op.q
    for name, val in fields.items():
        setattr(m, name, val)
    keep = []
    for name, arr in reals.items():
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float64).astype(npd))
        keep.append(a)
        setattr(m, name, a.ctypes.data)
    for name, arr in ints.items():
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.int32))
        keep.append(a)
        setattr(m, name, a.ctypes.data)
    return m, keep


def forward(op, u, dtype=np.float64):
    npd = _np_dtype(dtype)
    m, keep = model_struct(op, npd)
    u = np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(-1, op.k).astype(npd))
    g = np.empty((u.shape[0], op.q), dtype=npd)
    rc = lib().orc_forward(C.byref(m), _abi_dtype(npd), u.shape[0], _p(u), _p(g))
    assert rc == 0, rc
    return g


def potential(op, u, y, ginv, dtype=np.float64):
    npd = _np_dtype(dtype)
    m, keep = model_struct(op, npd)
    u = np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(-1, op.k).astype(npd))
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).astype(npd))
    gi = np.ascontiguousarray(np.asarray(ginv, dtype=np.float64).astype(npd))
    phi = np.empty((u.shape[0],), dtype=npd)
    rc = lib().orc_potential(C.byref(m), _abi_dtype(npd), u.shape[0], _p(u), _p(y), _p(gi), _p(phi))
    assert rc == 0, rc
    return phi


def pcn_sweep(
    op,
    U,
    phi,
    y,
    ginv,
    prior_sqrt,
    beta,
    seed,
    step0,
    n_steps,
    accepts=None,
    calls=None,
    chain_offset=0,
    box=(None, None, None),
    beta_schedule=None,
    sums=None,
    n_threads=1,
    proposal="pcn",
    reg_scale=None,
    prior_chol=None,
    samples=None,
    sample_every=0,
):
    """In-place sweep on numpy arrays U [C, k] and phi [C] (dtype from U).
    proposal 'pcn': v = sqrt(1-beta^2) u + beta w; 'rw': v = u + beta w.
    reg_scale: StandardRWAccepter regularizer scale (phi then holds I).
    prior_chol: [k, k] lower Cholesky factor of a non-diagonal prior (w = L·ξ)."""
    npd = U.dtype.type
    assert U.flags.c_contiguous and phi.dtype == U.dtype
    m, keep = model_struct(op, npd)
    cv = lambda a: None if a is None else np.ascontiguousarray(np.asarray(a, dtype=np.float64).astype(npd))
    y, gi, sq = cv(y), cv(ginv), cv(prior_sqrt)
    lo, hi, off = (cv(b) for b in box)
    rs = cv(reg_scale)
    ch = cv(prior_chol)
    sched = None if beta_schedule is None else np.ascontiguousarray(beta_schedule, dtype=np.float64)
    keep += [y, gi, sq, lo, hi, off, sched, rs, ch]
    s = _abi.IpmcSweep()
    s.dtype = _abi_dtype(npd)
    s.n_chains = U.shape[0]
    s.chain_offset = chain_offset
    s.u = _p(U)
    s.phi = _p(phi)
    s.accepts = _p(accepts)
    s.calls = _p(calls)
    s.y, s.gamma_inv, s.prior_sqrt = _p(y), _p(gi), _p(sq)
    s.box_lo, s.box_hi, s.box_off = _p(lo), _p(hi), _p(off)
    s.beta = float(beta)
    s.contraction = float(np.sqrt(1 - beta**2)) if proposal == "pcn" else 1.0
    s.beta_schedule = _p(sched)
    s.proposal = _abi.PROPOSAL_RW if proposal == "rw" else _abi.PROPOSAL_PCN
    s.reg_scale = _p(rs)
    s.prior_chol = _p(ch)
    s.seed = seed
    s.step0 = step0
    s.n_steps = n_steps
    if sums is not None:
        s.sum_u, s.sum_u2 = _p(sums[0]), _p(sums[1])
    if samples is not None:  # [C, n_samples, k]: in-launch samples every sample_every steps (0: the final state)
        assert samples.flags.c_contiguous and samples.dtype == U.dtype and samples.shape[0] == U.shape[0]
        s.sample_out = _p(samples)
        s.sample_stride = samples.shape[1] * samples.shape[2]
        s.sample_every = sample_every
        s.sample_step_stride = samples.shape[2]
    rc = lib().orc_pcn_sweep(C.byref(m), C.byref(s), n_threads)
    assert rc == 0, rc


def init_phi(op, U, y, ginv, reg_scale=None):
    """phi[c] = Φ(U_c) (+ ½Σ(reg_scale_i U_ci)²), the sweep's accept potential."""
    npd = U.dtype.type
    m, keep = model_struct(op, npd)
    cv = lambda a: None if a is None else np.ascontiguousarray(np.asarray(a, dtype=np.float64).astype(npd))
    y, gi, rs = cv(y), cv(ginv), cv(reg_scale)
    phi = np.empty(U.shape[0], dtype=npd)
    s = _abi.IpmcSweep()
    s.dtype = _abi_dtype(npd)
    s.n_chains = U.shape[0]
    s.u, s.phi, s.y, s.gamma_inv, s.reg_scale = _p(U), _p(phi), _p(y), _p(gi), _p(rs)
    lib().orc_init_phi.argtypes = [C.POINTER(_abi.IpmcModel), C.POINTER(_abi.IpmcSweep)]
    rc = lib().orc_init_phi(C.byref(m), C.byref(s))
    assert rc == 0, rc
    return phi


def normals(seed, chain_offset, n, step, k):
    out = np.empty((n, k), dtype=np.float64)
    lib().orc_normal_batch(seed, chain_offset, n, step, k, _p(out))
    return out


def uniforms(seed, chain_offset, n, step):
    out = np.empty((n,), dtype=np.float64)
    lib().orc_uniform_batch(seed, chain_offset, n, step, _p(out))
    return out


def det_log(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    lib().orc_log_batch(x.size, _p(x), _p(out))
    return out


def sincos_2pi(t):
    t = np.ascontiguousarray(t, dtype=np.float64)
    s, c = np.empty_like(t), np.empty_like(t)
    lib().orc_sincos_batch(t.size, _p(t), _p(s), _p(c))
    return s, c


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.empty(4, dtype=np.uint32)
    lib().orc_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def l96_rhs(x, F, arith="reference"):
    x = np.ascontiguousarray(x, dtype=np.float64)
    F = np.ascontiguousarray(np.broadcast_to(np.asarray(F, dtype=np.float64), x.shape))
    out = np.empty_like(x)
    lib().orc_l96_rhs_f64(_abi.ARITH_FMA if arith == "fma" else _abi.ARITH_REFERENCE, x.size, _p(x), _p(F), _p(out))
    return out


def l96ts_rhs(x, K, J, p, arith="reference"):
    """Two-scale Lorenz-96 RHS, p = (F, h, c, b)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    assert x.size == K * (1 + J) and p.size == 4
    out = np.empty_like(x)
    lib().orc_l96ts_rhs_f64(_abi.ARITH_FMA if arith == "fma" else _abi.ARITH_REFERENCE, K, J, _p(x), _p(p), _p(out))
    return out


def rusanov_flux(a, b, arith="reference"):
    return lib().orc_rusanov_flux_f64(_abi.ARITH_FMA if arith == "fma" else _abi.ARITH_REFERENCE, a, b)


def rusanov_rate(w, dx, arith="reference"):
    """dudt for interior cells 1..N of w (N+2 values incl. ghosts)."""
    w = np.ascontiguousarray(w, dtype=np.float64)
    r = np.zeros_like(w)
    lib().orc_rusanov_rate_f64(_abi.ARITH_FMA if arith == "fma" else _abi.ARITH_REFERENCE, w.size - 2, _p(w), dx, _p(r))
    return r


def autocorr_ref(x):
    """MCMCSampler.autocorr (sampler.py:43-54) restated: x_ = x - mean(x),
    np.correlate(x_, x_, 'full')[-len(x):] / r[0], all ones for r[0] == 0."""
    x = np.asarray(x, dtype=np.float64)
    x_ = x - np.mean(x)
    r = np.correlate(x_, x_, mode="full")[-len(x):]
    if r[0] == 0:
        return np.ones_like(r)
    return r / r[0]


def burn_in(x, window=50, threshold=0.03):
    """len_burn_in for chains x of shape (C, n_vars, len) or (n_vars, len) (f64)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    single = x.ndim == 2
    if single:
        x = x[None]
    out = np.empty(x.shape[0], dtype=np.int64)
    h = lib()
    h.orc_burn_in.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int64, C.c_int32, C.c_double, C.c_void_p]
    rc = h.orc_burn_in(_p(x), x.shape[0], x.shape[1], x.shape[2], window, threshold, _p(out))
    assert rc == 0, "series shorter than the window"
    return int(out[0]) if single else out
