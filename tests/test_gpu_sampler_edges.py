"""MCMCSampler.run edge cases on the device: no samples, a zero sample
interval, one chain vs a stack of one, f32 output dtype, and the schedule's
step count (sampler.py:18-26) against the accept/call counters."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _sampler(dtype=np.float64, seed=3):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             LinearOperator, MCMCSampler, pCNAccepter)

    g = np.array([3.0, 1.0, 4.0, 1.0])
    pot = EvolutionPotential(LinearOperator(g), np.array([30.0]), GaussianDistribution(0, 0.25))
    acc = CountedAccepter(pCNAccepter(pot))
    return MCMCSampler(ConstSteppCNProposer(0.5, GaussianDistribution(np.zeros(4), np.eye(4))), acc, seed,
                       dtype=dtype), acc


def test_no_samples_and_zero_interval():
    s, acc = _sampler()
    out = s.run(np.zeros((5, 4)), n_samples=0, burn_in=10, sample_interval=3)
    assert out.shape == (5, 0, 4) and out.dtype == np.float64
    assert np.all(np.asarray(acc.calls) == 7)  # max(0, 10 - 3) + 0
    s, acc = _sampler()
    out = s.run(np.zeros((5, 4)), n_samples=4, burn_in=6, sample_interval=0)
    assert out.shape == (5, 4, 4)
    assert np.all(np.asarray(acc.calls) == 6)  # the burn-in only; every sample is the same state
    assert np.array_equal(out[:, 0], out[:, 3])


def test_single_chain_equals_stack_of_one():
    s1, a1 = _sampler()
    one = s1.run(np.zeros(4), n_samples=6, burn_in=20, sample_interval=5)
    s2, a2 = _sampler()
    stack = s2.run(np.zeros((1, 4)), n_samples=6, burn_in=20, sample_interval=5)
    assert one.shape == (6, 4) and stack.shape == (1, 6, 4)
    assert np.array_equal(one, stack[0])
    assert a1.accepts == int(np.asarray(a2.accepts)[0]) and a1.calls == 15 + 30


def test_f32_samples_come_back_as_float64():
    s, _ = _sampler(np.float32)
    out = s.run(np.zeros((3, 4)), n_samples=5, burn_in=4, sample_interval=2)
    assert out.dtype == np.float64 and out.shape == (3, 5, 4)
    assert np.array_equal(out, out.astype(np.float32).astype(np.float64))  # f32 values, widened


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("flush", [1, 3, 10, 25])
def test_streaming_to_npy_equals_in_memory(tmp_path, dtype, flush):
    """run(sample_file=...) through the double-buffered writer (one buffer when
    every sample fits, a partial last block otherwise) = the in-memory samples,
    for one chain ((n, k) file, the reference's layout) and for a stack."""
    for u0 in (np.zeros(4), np.zeros((7, 4))):
        s1, _ = _sampler(dtype)
        mem = s1.run(u0, n_samples=10, burn_in=4, sample_interval=2)
        s2, _ = _sampler(dtype)
        path = str(tmp_path / f"s_{flush}_{np.dtype(dtype).name}_{u0.ndim}.npy")
        f = s2.run(u0, n_samples=10, burn_in=4, sample_interval=2, sample_file=path, flush_every=flush)
        assert f.shape == mem.shape and f.dtype == np.float64
        assert np.array_equal(np.asarray(f), mem)
        assert np.array_equal(np.load(path), mem)
