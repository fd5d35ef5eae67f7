"""ipmc_pcn_run (MCMCSampler.run's sampling loop in one C call) gives the bits
of the per-sample launches it replaces: samples, moments, accept counts and
the chain state, for constant and scheduled step sizes and small (speculative)
and large ensembles."""
import contextlib
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return torch.device("cuda", 0)


def _sampler(op, y, gamma, var_step, chains_seed=5, **skw):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             MCMCSampler, PhiloxRNG, VarSteppCNProposer, pCNAccepter)

    prior = GaussianDistribution(np.zeros(op.k), np.eye(op.k))
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(op.q), gamma**2 * np.eye(op.q)))
    prop = VarSteppCNProposer(lambda i: 0.1 + 0.4 / (1 + i), prior) if var_step else ConstSteppCNProposer(0.3, prior)
    acc = CountedAccepter(pCNAccepter(pot))
    return MCMCSampler(prop, acc, PhiloxRNG(chains_seed), **skw), acc


def _run(op, y, gamma, var_step, u0, keep, verbose, skw, **kw):
    s, acc = _sampler(op, y, gamma, var_step, **skw)
    s.verbose = verbose  # verbose keeps the per-sample launch loop (it prints every sample)
    with contextlib.redirect_stdout(io.StringIO()):
        out = s.run(u0, keep=keep, **kw)
    return out, np.asarray(acc.accepts), s.state.u


def _case(case, rng):
    """(operator, data, noise std, chains, sampler options) of one kernel family."""
    from ip_mcmc_amd import (BurgersOperator, LinearOperator, Lorenz63Operator, Lorenz96Operator,
                             TwoScaleLorenz96Operator)

    if case.startswith("linear"):
        op = LinearOperator(rng.normal(size=(3, 4)))
        return op, rng.normal(size=3), 0.5, (1 if case == "linear1" else 4096), {}
    if case in ("l63", "l63_f32"):
        op = Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=40)
        # fp32: two speculative slots per lane (v_pk_* pairs)
        return op, op(np.zeros(3)) + 0.2 * rng.normal(size=6), 0.5, 64, ({"dtype": np.float32} if case == "l63_f32" else {})
    if case == "burgers":
        op = BurgersOperator(N=32, dt_mode="cfl", T=0.3)
        return op, op(np.zeros(3)) + 0.05 * rng.normal(size=5), 0.1, 16, {}
    if case in ("l63_hi", "linear_hi"):  # broad posteriors: the speculative sweeps run the accept path
        op = (Lorenz63Operator(x0=(1.0, 2.0, 20.0), dt=0.01, n_steps=40) if case == "l63_hi"
              else LinearOperator(rng.normal(size=(3, 4))))
        return op, op(np.zeros(op.k)) + 0.2 * rng.normal(size=op.q), 50.0, 64, {}
    if case == "burgers_hi":  # broad posterior: the Burgers sweep speculates along the accept path
        op = BurgersOperator(N=32, dt_mode="cfl", T=0.3)
        return op, op(np.zeros(3)) + 0.05 * rng.normal(size=5), 5.0, 16, {}
    if case == "l96_hi":
        op = Lorenz96Operator(8, 8.0, dt=0.01, n_steps=50)
        return op, op(np.zeros(8)) + 0.1 * rng.normal(size=8), 10.0, 300, {}
    if case in ("ts", "ts_hi"):
        op = TwoScaleLorenz96Operator(4, 2, dt=0.005, n_steps=40)
        return op, op(np.zeros(3)) + 0.1 * rng.normal(size=op.q), (0.5 if case == "ts" else 50.0), 40, {}
    if case in ("ts6", "ts6_hi"):  # K=6 J=4: three slow variables per lane, pairs of lanes
        op = TwoScaleLorenz96Operator(6, 4, dt=0.005, n_steps=30)
        return op, op(np.zeros(3)) + 0.1 * rng.normal(size=op.q), (0.5 if case == "ts6" else 50.0), 40, {}
    op = Lorenz96Operator(8, 8.0, dt=0.01, n_steps=50)
    y = op(np.zeros(8)) + 0.1 * rng.normal(size=8)
    skw = {}
    if case in ("l96_seq", "l96_f32"):
        skw["spec_width"] = 1  # the sequential kernels (packed pairs in f32)
    if case == "l96_f32":
        skw["dtype"] = np.float32
    return op, y, 0.2, 300, skw


@pytest.mark.parametrize("case", ["linear1", "linear4096", "l96", "l96_var", "l96_seq", "l96_f32", "l63", "l63_f32",
                                  "burgers", "ts", "l63_hi", "linear_hi", "ts_hi", "ts6", "ts6_hi", "l96_hi",
                                  "burgers_hi"])
@pytest.mark.parametrize("keep", ["samples", "moments"])
def test_pcn_run_equals_per_sample_launches(dev, case, keep):
    """In-launch samples (ipmc_sweep.sample_every, several samples per launch
    through ipmc_pcn_run) equal one launch per sample, for every kernel
    family: sequential, speculative, packed fp32."""
    rng = np.random.default_rng(2)
    op, y, gamma, n, skw = _case(case, rng)
    u0 = 0.1 * rng.normal(size=(n, op.k))
    kw = dict(n_samples=37, burn_in=25, sample_interval=6)
    a = _run(op, y, gamma, case.endswith("var"), u0, keep, False, skw, **kw)
    b = _run(op, y, gamma, case.endswith("var"), u0, keep, True, skw, **kw)
    if keep == "samples":
        assert a[0].shape == (n, 37, op.k) and np.array_equal(a[0], b[0])
    else:
        assert np.array_equal(a[0]["sum_u"], b[0]["sum_u"]) and np.array_equal(a[0]["sum_u2"], b[0]["sum_u2"])
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[1].sum() > 0


def test_interval_one_runs_across_sample_boundaries(dev):
    """sample_interval=1 (the reference studies' recording): one chain still
    runs multi-step launches (speculation across samples) with the same bits."""
    rng = np.random.default_rng(6)
    op, y, gamma, _, _ = _case("l96", rng)
    u0 = 0.1 * rng.normal(size=op.k)
    a = _run(op, y, gamma, False, u0, "samples", False, {}, n_samples=300, burn_in=0, sample_interval=1)
    b = _run(op, y, gamma, False, u0, "samples", True, {}, n_samples=300, burn_in=0, sample_interval=1)
    assert a[0].shape == (300, 8) and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_pcn_run_streams_to_a_file(dev, tmp_path):
    """run(sample_file=...) through ipmc_pcn_run, flushing every 5 samples,
    equals the in-memory run."""
    from ip_mcmc_amd import LinearOperator

    rng = np.random.default_rng(3)
    op = LinearOperator(rng.normal(size=(2, 4)))
    y = rng.normal(size=2)
    u0 = 0.1 * rng.normal(size=(64, 4))
    s1, _ = _sampler(op, y, 0.5, False)
    mem = s1.run(u0, n_samples=23, burn_in=10, sample_interval=3)
    s2, _ = _sampler(op, y, 0.5, False)
    f = s2.run(u0, n_samples=23, burn_in=10, sample_interval=3, sample_file=str(tmp_path / "s.npy"), flush_every=5)
    assert np.array_equal(np.asarray(f), mem)


@pytest.mark.parametrize("case", ["l96", "l96_seq", "l96_f32", "linear1", "burgers"])
def test_overlapped_sample_copy(dev, case, monkeypatch):
    """Large in-memory sample arrays go to the host in blocks of samples on a
    copy stream while the later blocks sweep (rectangular D2H copies into the
    page-locked result; f32 converted on the device first).  Forced on at a
    small size here: the result equals the per-sample launch loop's, for an
    uneven split (37 samples in 8 blocks) and a single chain."""
    from ip_mcmc_amd import sampler as S

    rng = np.random.default_rng(11)
    op, y, gamma, n, skw = _case(case, rng)
    u0 = 0.1 * rng.normal(size=(n, op.k)) if n > 1 else 0.1 * rng.normal(size=op.k)
    kw = dict(n_samples=37, burn_in=7, sample_interval=4)
    b = _run(op, y, gamma, False, u0, "samples", True, skw, **kw)
    monkeypatch.setattr(S, "OVERLAP_COPY_MIN_BYTES", 0)
    a = _run(op, y, gamma, False, u0, "samples", False, skw, **kw)
    assert a[0].dtype == np.float64 and a[0].shape == b[0].shape
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


@pytest.mark.parametrize("case", ["l96", "l63_hi", "linear1", "burgers", "ts6_hi"])
def test_launch_length_does_not_change_the_chains(dev, case, monkeypatch):
    """The sampler splits burn-in and sample intervals into launches of at most
    sampler.STEPS_PER_LAUNCH steps (16 384 by default, so most runs are one
    launch per block): with the cap forced to 7 -- burn-in, intervals and the
    in-launch sample blocks all split, speculative rounds cut at every launch
    boundary -- samples, accept counts and the final state are the same bits."""
    from ip_mcmc_amd import sampler as S

    rng = np.random.default_rng(12)
    op, y, gamma, n, skw = _case(case, rng)
    n = min(n, 64)
    u0 = 0.1 * rng.normal(size=(n, op.k)) if n > 1 else 0.1 * rng.normal(size=op.k)
    kw = dict(n_samples=9, burn_in=50, sample_interval=20)
    a = _run(op, y, gamma, False, u0, "samples", False, skw, **kw)
    monkeypatch.setattr(S, "STEPS_PER_LAUNCH", 7)
    b = _run(op, y, gamma, False, u0, "samples", False, skw, **kw)
    assert a[0].shape == b[0].shape
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert np.asarray(a[1]).sum() > 0
