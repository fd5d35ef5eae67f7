"""The C-ABI's argument checks (include/ipmc.h), exercised on the CPU.

Every call here fails validation (or is a no-op) before anything reaches the
device, so no GPU is needed: the library returns the documented status code
and ipmc_last_error() says why.  The pointers are dummies that are never
dereferenced.  This is the boundary's equivalent of the reference's
`assert 0 <= beta <= 1` (proposer.py:75) and ValueError paths.
"""
import ctypes as C

import pytest

from ip_mcmc_amd import _abi, _lib

DUMMY = 0x10000  # a non-NULL "device pointer"; never dereferenced by these calls


@pytest.fixture(scope="module")
def h():
    return _lib.lib()


def _model(kind=_abi.MODEL_LORENZ96, k=40, q=40, dim=40, n_steps=10):
    m = _abi.IpmcModel()
    m.kind, m.arith, m.k, m.q, m.dim, m.n_steps, m.dt = kind, _abi.ARITH_FMA, k, q, dim, n_steps, 0.01
    m.x0 = m.theta0 = m.A = DUMMY
    return m


def _sweep(n=8, k=40):
    s = _abi.IpmcSweep()
    s.dtype, s.n_chains, s.n_steps = _abi.F64, n, 1
    s.u = s.phi = s.y = s.gamma_inv = s.prior_sqrt = DUMMY
    s.beta, s.contraction = 0.5, 0.75 ** 0.5
    return s


def _status(h, rc, code, text):
    assert rc == code, (rc, h.ipmc_last_error())
    assert text in h.ipmc_last_error().decode()


def test_model_checks(h):
    sweep = C.byref(_sweep())
    _status(h, h.ipmc_pcn_sweep(None, sweep, None), _abi.ERR_INVALID, "model is NULL")
    m = _model(k=0)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "k and q must be positive")
    m = _model()
    m.theta0 = None
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "theta0 is NULL")
    m = _model()
    m.arith = 9
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "bad arith")
    m = _model(kind=_abi.MODEL_LORENZ63, k=4, q=6)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "Lorenz-63")
    m = _model(q=39)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "Lorenz-96")
    m = _model(kind=_abi.MODEL_BURGERS, k=3, q=5, dim=256)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "Burgers")
    m = _model(kind=_abi.MODEL_LORENZ96_2S, k=3, q=29, dim=6)
    m.fast_per_slow = 4
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_INVALID, "q == 5K")
    m = _model(kind=_abi.MODEL_LORENZ96_2S, k=3, q=5 * 65, dim=65)
    m.fast_per_slow = 4
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_UNSUPPORTED, "K <= 64")
    m = _model(kind=42)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_UNSUPPORTED, "unknown model kind")
    m = _model(kind=_abi.MODEL_LINEAR, k=65, q=1)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), sweep, None), _abi.ERR_UNSUPPORTED, "k > 64")


def test_sweep_checks(h):
    m = C.byref(_model())
    _status(h, h.ipmc_pcn_sweep(m, None, None), _abi.ERR_INVALID, "sweep is NULL")
    s = _sweep()
    s.dtype = 5
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "dtype")
    s = _sweep()
    s.proposal = 7
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "proposal")
    for beta in (1.5, -0.1, float("nan")):
        s = _sweep()
        s.beta = beta
        _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "beta has to be in [0,1]")
    s = _sweep()
    s.beta, s.proposal = 1.5, _abi.PROPOSAL_RW  # RW step sizes are not bounded by 1
    s.u = None
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "is NULL")
    s = _sweep(n=-1)
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "negative count")
    s = _sweep()
    s.sample_out, s.sample_stride = DUMMY, 39
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sample_stride < k")
    s = _sweep()
    s.sum_u2 = DUMMY
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sum_u2 needs sum_u")
    # no chains or no steps: a no-op (nothing is launched)
    assert h.ipmc_pcn_sweep(m, C.byref(_sweep(n=0)), None) == _abi.OK
    s = _sweep()
    s.n_steps = 0
    assert h.ipmc_pcn_sweep(m, C.byref(s), None) == _abi.OK


def test_layout_checks(h):
    m = _model(dim=41, k=41, q=41)
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(_sweep(k=41)), None), _abi.ERR_UNSUPPORTED,
            "no kernel compiled for dim=41")
    m = _model()
    s = _sweep()
    s.lanes_per_chain = 16  # d=40 has no 16-lane instantiation
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(s), None), _abi.ERR_UNSUPPORTED, "lanes_per_chain=16")
    m = _model(kind=_abi.MODEL_LORENZ63, k=3, q=6, dim=3)
    s = _sweep(k=3)
    s.spec_width = 3
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(s), None), _abi.ERR_UNSUPPORTED, "power of two")
    s = _sweep(k=3)
    s.chains_per_lane = 2
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(s), None), _abi.ERR_UNSUPPORTED, "one chain per lane")
    s = _sweep(k=3)
    s.lanes_per_chain = 4
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(s), None), _abi.ERR_UNSUPPORTED, "one chain per lane")
    m = _model()
    s = _sweep()
    s.lanes_per_chain, s.spec_width = 8, 16  # 128 lanes per chain > one wavefront
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(s), None), _abi.ERR_UNSUPPORTED, "<= 64")
    s = _sweep()
    s.chains_per_lane, s.spec_width, s.dtype = 2, 4, _abi.F32
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(s), None), _abi.ERR_UNSUPPORTED, "one chain per lane group")
    m = _model(kind=_abi.MODEL_BURGERS, k=3, q=5, dim=258)
    m.n_windows, m.win_lo, m.win_hi = 5, DUMMY, DUMMY
    _status(h, h.ipmc_pcn_sweep(C.byref(m), C.byref(_sweep(k=3)), None), _abi.ERR_UNSUPPORTED, "multiple of 4")


def test_eval_and_rng_checks(h):
    m = C.byref(_model())
    _status(h, h.ipmc_forward(m, 7, 4, DUMMY, DUMMY, None), _abi.ERR_INVALID, "dtype")
    _status(h, h.ipmc_forward(m, _abi.F64, -1, DUMMY, DUMMY, None), _abi.ERR_INVALID, "n must be >= 0")
    _status(h, h.ipmc_forward(m, _abi.F64, 4, None, DUMMY, None), _abi.ERR_INVALID, "u / out is NULL")
    _status(h, h.ipmc_potential(m, _abi.F64, 4, DUMMY, None, DUMMY, DUMMY, None), _abi.ERR_INVALID,
            "y / gamma_inv is NULL")
    assert h.ipmc_forward(m, _abi.F64, 0, None, None, None) == _abi.OK
    _status(h, h.ipmc_normal(1, 0, -1, 0, 4, _abi.F64, DUMMY, None), _abi.ERR_INVALID, "negative count")
    _status(h, h.ipmc_normal(1, 0, 4, 0, 4, 9, DUMMY, None), _abi.ERR_INVALID, "bad dtype")
    _status(h, h.ipmc_uniform(1, 0, 4, 0, None, None), _abi.ERR_INVALID, "out is NULL")
    assert h.ipmc_uniform(1, 0, 0, 0, None, None) == _abi.OK


def test_diagnostics_checks(h):
    _status(h, h.ipmc_autocorr(DUMMY, _abi.F64, 1, 10, 10, 1, 11, DUMMY, None), _abi.ERR_INVALID,
            "exceeds the series length")
    _status(h, h.ipmc_autocorr(DUMMY, _abi.F64, 1, 9000, 9000, 1, 9001, DUMMY, None), _abi.ERR_INVALID,
            "exceeds the series length")  # the long-series path checks the same way
    _status(h, h.ipmc_autocorr(DUMMY, _abi.F64, -1, 10, 10, 1, 5, DUMMY, None), _abi.ERR_INVALID, "negative")
    assert h.ipmc_autocorr(None, _abi.F64, 0, 10, 10, 1, 5, None, None) == _abi.OK
    _status(h, h.ipmc_burn_in(DUMMY, _abi.F64, 2, 3, 49, 147, 49, 1, 50, 0.03, DUMMY, DUMMY, None),
            _abi.ERR_INVALID, "shorter than the window")
    _status(h, h.ipmc_burn_in(DUMMY, 5, 2, 3, 60, 180, 60, 1, 50, 0.03, DUMMY, DUMMY, None), _abi.ERR_INVALID,
            "bad dtype")
    _status(h, h.ipmc_burn_in(DUMMY, _abi.F64, 2, 3, 60, 180, 60, 1, 50, 0.03, None, DUMMY, None),
            _abi.ERR_INVALID, "NULL")
    assert h.ipmc_burn_in(None, _abi.F64, 0, 3, 60, 180, 60, 1, 50, 0.03, None, None, None) == _abi.OK


def test_auto_layout(h):
    """The layout the sweep picks by itself: fp64 d=40 -> 2 lanes per
    chain; fp32 -> two chains per lane group as f32x2, 2 lanes; d=256 -> 16 lanes."""
    m = _model()
    assert h.ipmc_auto_layout(C.byref(m), _abi.F64, 65536) == 102
    assert h.ipmc_auto_layout(C.byref(m), _abi.F32, 65536) == 202
    assert h.ipmc_auto_lanes(C.byref(m), _abi.F64, 65536) == 2
    m = _model(dim=256, k=256, q=256)
    assert h.ipmc_auto_layout(C.byref(m), _abi.F64, 131072) == 116
    assert h.ipmc_auto_layout(None, _abi.F64, 1) == 0


# (dim, dtype, chains) -> cpl * 100 + lpc: the measured-fastest layout, or one
# within 4 % of it, of profiles/r1/lanes_layout_rule.txt (d=40 at 32 768 and
# 65 536 chains: profiles/r2/lanes_inplace.txt, lanes_scan_d40_r2k.txt, after
# the in-place RK4 stages; fp32 at 16 384 chains on 8 interleaved lanes x 2
# chains: profiles/r3/layouts_l8il.jsonl)
LAYOUT_TABLE = [
    (8, "f64", 16384, 104), (8, "f64", 65536, 101), (8, "f32", 16384, 104), (8, "f32", 65536, 202),
    (16, "f64", 16384, 104), (16, "f64", 65536, 101), (16, "f32", 16384, 208), (16, "f32", 65536, 202),
    (40, "f64", 8192, 108), (40, "f64", 16384, 104), (40, "f64", 32768, 102), (40, "f64", 65536, 102),
    (40, "f32", 8192, 108), (40, "f32", 16384, 208), (40, "f32", 32768, 204), (40, "f32", 65536, 202),
    (80, "f64", 16384, 104), (80, "f64", 65536, 104), (80, "f32", 16384, 208), (80, "f32", 65536, 204),
    # below one wave per SIMD (speculative sweeps): DPP halos (profiles/r1/l96_small_layouts.jsonl)
    (40, "f64", 1, 104), (40, "f64", 64, 104), (40, "f64", 1024, 104), (40, "f32", 1, 104), (40, "f32", 1024, 104),
]


@pytest.mark.parametrize("dim,dt,chains,want", LAYOUT_TABLE)
def test_auto_layout_follows_the_layout_scans(h, dim, dt, chains, want):
    m = _model(dim=dim, k=dim, q=dim)
    assert h.ipmc_auto_layout(C.byref(m), _abi.F64 if dt == "f64" else _abi.F32, chains) == want


def test_python_layer_raises_with_the_library_message():
    from ip_mcmc_amd._lib import IpmcError, call

    with pytest.raises(IpmcError, match="beta has to be in"):
        s = _sweep()
        s.beta = 2.0
        call("ipmc_pcn_sweep", C.byref(_model()), C.byref(s), None)


def test_chain_id_and_step_ranges(h):
    """Global chain ids live in one 32-bit Philox counter word and pCN steps
    below 2^63 (the host-draw range starts there): anything outside would alias
    other chains' draws, so the ABI rejects it before launching."""
    m = C.byref(_model())
    s = _sweep()
    s.chain_offset = (1 << 32) - 4  # 8 chains -> ids up to 2^32 + 3
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "<= 2^32")
    s = _sweep()
    s.step0 = (1 << 63) - 1
    s.n_steps = 2
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "below 2^63")
    _status(h, h.ipmc_normal(1, (1 << 32) - 1, 2, 0, 4, _abi.F64, DUMMY, None), _abi.ERR_INVALID, "<= 2^32")
    _status(h, h.ipmc_uniform(1, 1 << 32, 1, 0, DUMMY, None), _abi.ERR_INVALID, "<= 2^32")
    _status(h, h.ipmc_uniform(1, -1, 1, 0, DUMMY, None), _abi.ERR_INVALID, "negative")
    # the last valid id is fine for validation (n = 0 -> no launch)
    assert h.ipmc_uniform(1, 1 << 32, 0, 0, DUMMY, None) == _abi.OK


def _plan(h, model, sweep):
    p = _abi.IpmcPlan()
    rc = h.ipmc_plan_sweep(C.byref(model), C.byref(sweep), C.byref(p))
    assert rc == _abi.OK, h.ipmc_last_error()
    return p.lanes_per_chain, p.chains_per_lane, p.spec_width


def test_plan_sweep_reports_what_the_sweep_runs(h):
    """ipmc_plan_sweep comes from the same code path as ipmc_pcn_sweep's kernel
    choice, including the speculation of multi-step launches (which may run on
    another layout than ipmc_auto_layout's one-step pick)."""
    m = _model(dim=40, k=40, q=40)
    s = _sweep(n=65536)
    assert _plan(h, m, s) == (2, 1, 1)  # headline: 2 lanes per chain, sequential
    s.dtype = _abi.F32
    assert _plan(h, m, s) == (2, 2, 1)  # packed fp32 pairs
    s = _sweep(n=8192)
    assert h.ipmc_auto_layout(C.byref(m), _abi.F64, 8192) == 108  # 8 interleaved lanes fill the GPU
    assert _plan(h, m, s) == (8, 1, 1)
    s.n_steps = 16
    assert _plan(h, m, s) == (8, 1, 1)  # short launches: sequential
    s.n_steps = 512
    assert _plan(h, m, s) == (4, 1, 2)  # long launches speculate on DPP quads, 2 slots (one wave per SIMD)
    s.dtype = _abi.F32
    assert _plan(h, m, s) == (4, 1, 2)  # fp32 the same
    s.n_steps = 16
    assert _plan(h, m, s) == (8, 1, 1)
    s.dtype = _abi.F64
    s3 = _sweep(n=32768)
    s3.n_steps = 2
    assert _plan(h, m, s3) == (2, 1, 1)  # 32 768 chains fill the GPU sequentially
    s3 = _sweep(n=16384)
    s3.n_steps = 8
    assert _plan(h, m, s3) == (4, 1, 1)  # so do 16 384 on 4 lanes: no speculation
    s3 = _sweep(n=2048)
    s3.n_steps = 16
    assert _plan(h, m, s3) == (4, 1, 8)  # slots up to one wave per SIMD
    s = _sweep(n=1)
    s.n_steps = 16
    assert _plan(h, m, s) == (4, 1, 64)  # one chain: its slots span a whole block
    s.spec_width = 1
    assert _plan(h, m, s) == (4, 1, 1)
    s.spec_width = 3
    rc = h.ipmc_plan_sweep(C.byref(m), C.byref(s), C.byref(_abi.IpmcPlan()))
    _status(h, rc, _abi.ERR_UNSUPPORTED, "power of two")
    # small models: one lane per slot
    ml = _model(kind=_abi.MODEL_LORENZ63, k=3, q=6, dim=3)
    s = _sweep(n=4096)
    s.n_steps = 128
    assert _plan(h, ml, s) == (1, 1, 16)  # cfg 2: width 16 (profiles/r1/spec_cfg2.txt)
    # two-scale: K lanes per chain (K=36: 2 slow variables per lane)
    mt = _model(kind=_abi.MODEL_LORENZ96_2S, k=3, q=30, dim=6)
    mt.fast_per_slow = 4
    s = _sweep(n=65536)
    assert _plan(h, mt, s) == (2, 1, 1)  # K=6 J<=4: 3 slow variables per lane, pairs of lanes (DPP halos)
    s2 = _sweep(n=1024)
    s2.n_steps = 16
    assert _plan(h, mt, s2) == (6, 1, 10)  # a small ensemble speculates on 6 lanes per chain (latency)
    mt.fast_per_slow = 8
    assert _plan(h, mt, s) == (6, 1, 1)
    mt = _model(kind=_abi.MODEL_LORENZ96_2S, k=3, q=180, dim=36)
    mt.fast_per_slow = 10
    assert _plan(h, mt, s)[0] == 18
    # Burgers N=256: 32 lanes of 8 cells
    mb = _model(kind=_abi.MODEL_BURGERS, k=3, q=5, dim=256)
    mb.n_windows = 5
    mb.win_lo = mb.win_hi = DUMMY
    s = _sweep(n=2048)
    assert _plan(h, mb, s) == (32, 1, 1)
    s = _sweep(n=1)
    s.n_steps = 8
    assert _plan(h, mb, s) == (32, 1, 8)
    rc = h.ipmc_plan_sweep(None, C.byref(s), C.byref(_abi.IpmcPlan()))
    _status(h, rc, _abi.ERR_INVALID, "model is NULL")


def test_unsupported_layout_sets_the_error_message(h):
    """A forced layout with no compiled kernel reports why (not a stale message)."""
    m = C.byref(_model(dim=40, k=40, q=40))
    s = _sweep()
    s.beta = 2.0
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "beta")  # leave a message behind
    s = _sweep()
    s.lanes_per_chain = 3
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_UNSUPPORTED, "lanes_per_chain=3")


def test_pcn_run_validation(h):
    """ipmc_pcn_run checks its block arithmetic before launching anything, and
    every block goes through ipmc_pcn_sweep's own checks."""
    m = C.byref(_model())
    _status(h, h.ipmc_pcn_run(m, None, 1, 1, 40, None), _abi.ERR_INVALID, "sweep is NULL")
    _status(h, h.ipmc_pcn_run(m, C.byref(_sweep()), -1, 1, 40, None), _abi.ERR_INVALID, "negative count")
    _status(h, h.ipmc_pcn_run(m, C.byref(_sweep()), 1, -1, 40, None), _abi.ERR_INVALID, "negative count")
    _status(h, h.ipmc_pcn_run(m, C.byref(_sweep()), 1, 1 << 31, 40, None), _abi.ERR_INVALID, "< 2^31")
    s = _sweep()
    s.step0 = (1 << 62)
    _status(h, h.ipmc_pcn_run(m, C.byref(s), 1 << 43, 1 << 20, 40, None), _abi.ERR_INVALID, "below 2^63")
    s = _sweep()
    s.sample_out, s.sample_stride = DUMMY, 40
    _status(h, h.ipmc_pcn_run(m, C.byref(s), 2, 3, -1, None), _abi.ERR_INVALID, "sample_block_stride")
    s = _sweep()
    s.beta = 2.0  # the per-block checks of ipmc_pcn_sweep
    _status(h, h.ipmc_pcn_run(m, C.byref(s), 2, 3, 40, None), _abi.ERR_INVALID, "beta has to be in")
    assert h.ipmc_pcn_run(m, C.byref(_sweep()), 0, 5, 40, None) == _abi.OK  # no block: nothing to do


def test_sample_every_validation(h):
    """ipmc_sweep.sample_every (ABI 9): in-launch recording needs a sample
    buffer whose rows and sample slots hold k values."""
    m = C.byref(_model())
    s = _sweep()
    s.sample_every = -1
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sample_every must be in")
    s.sample_every = 1 << 31
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sample_every must be in")
    s.sample_every = 2
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sample_every needs sample_out")
    s.sample_out, s.sample_stride, s.sample_step_stride = DUMMY, 400, 39
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sample_step_stride >= k")
    s.sample_step_stride, s.sample_stride = 40, 39
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "sample_stride >= k")
    s.sample_stride, s.n_steps = 400, 0
    assert h.ipmc_pcn_sweep(m, C.byref(s), None) == _abi.OK  # no step, no in-launch sample: nothing to copy


def test_sample_every_rejects_overlapping_layouts(h):
    """With n_s = n_steps / sample_every samples per chain, a chain's samples
    may not run into the next chain's rows ([chain, sample, k] needs
    sample_stride >= (n_s-1)*sample_step_stride + k, [sample, chain, k] needs
    sample_step_stride >= (n_chains-1)*sample_stride + k)."""
    m = C.byref(_model())
    s = _sweep(n=8)
    s.n_steps, s.sample_every, s.sample_out = 10, 2, DUMMY
    s.sample_stride, s.sample_step_stride = 40, 40  # the sample_every = 0 convention: overlaps
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "samples overlap")
    s.sample_stride, s.sample_step_stride = 199, 40  # one element short of [chain, 5 samples, 40]
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "samples overlap")
    s.sample_stride, s.sample_step_stride = 40, 319  # one element short of [5 samples, 8 chains, 40]
    _status(h, h.ipmc_pcn_sweep(m, C.byref(s), None), _abi.ERR_INVALID, "samples overlap")


def test_pcn_draws_and_copy_validation(h):
    """ipmc_pcn_draws / ipmc_copy_rows_d2h (ABI 10) argument checks (no GPU call)."""
    _status(h, h.ipmc_pcn_draws(1, 0, 4, 0, 3, 0, _abi.F64, DUMMY, None, DUMMY, None, None), _abi.ERR_INVALID,
            "k must be positive")
    _status(h, h.ipmc_pcn_draws(1, 0, 4, 0, 3, 2, 7, DUMMY, None, DUMMY, None, None), _abi.ERR_INVALID, "bad dtype")
    _status(h, h.ipmc_pcn_draws(1, (1 << 32) - 2, 4, 0, 3, 2, _abi.F64, DUMMY, None, DUMMY, None, None),
            _abi.ERR_INVALID, "2^32")
    _status(h, h.ipmc_pcn_draws(1, 0, 4, (1 << 63) - 2, 3, 2, _abi.F64, DUMMY, None, DUMMY, None, None),
            _abi.ERR_INVALID, "below 2^63")
    _status(h, h.ipmc_pcn_draws(1, 0, 4, 0, 3, 2, _abi.F64, DUMMY, None, None, None, None), _abi.ERR_INVALID,
            "w is NULL")
    _status(h, h.ipmc_pcn_draws(1, 0, 4, 0, 3, 2, _abi.F64, None, None, DUMMY, None, None), _abi.ERR_INVALID,
            "both NULL")
    assert h.ipmc_pcn_draws(1, 0, 4, 0, 0, 2, _abi.F64, DUMMY, None, DUMMY, None, None) == _abi.OK  # nothing to draw
    _status(h, h.ipmc_copy_rows_d2h(DUMMY, 8, DUMMY, 16, 16, 4, None), _abi.ERR_INVALID, "pitch < width")
    _status(h, h.ipmc_copy_rows_d2h(None, 16, DUMMY, 16, 16, 4, None), _abi.ERR_INVALID, "NULL")
    _status(h, h.ipmc_copy_rows_d2h(DUMMY, 16, DUMMY, 16, -1, 4, None), _abi.ERR_INVALID, "negative")
    assert h.ipmc_copy_rows_d2h(DUMMY, 16, DUMMY, 16, 16, 0, None) == _abi.OK
