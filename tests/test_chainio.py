"""On-disk chains (.npy, load_or_compute) and exact checkpoint / resume."""
import os

import numpy as np
import pytest


def test_load_or_compute_contract(tmp_path):
    from ip_mcmc_amd.chainio import load_or_compute

    calls = []

    def f(n):
        calls.append(n)
        return np.arange(n, dtype=np.float64)

    p = str(tmp_path / "chain")
    a = load_or_compute(p, f, (5,))
    b = load_or_compute(p, f, (5,))
    assert calls == [5] and np.array_equal(a, b) and os.path.exists(p + ".npy")


def test_npy_sink_is_numpy_loadable(tmp_path):
    from ip_mcmc_amd.chainio import NpySampleSink

    s = NpySampleSink(str(tmp_path / "s.npy"), (3, 7, 2))
    full = np.random.default_rng(0).normal(size=(3, 7, 2))
    s.write(0, full[:, :4])
    s.write(4, full[:, 4:])
    got = s.close()
    assert np.array_equal(np.load(str(tmp_path / "s.npy")), full) and np.array_equal(got, full)
    one = NpySampleSink(str(tmp_path / "one.npy"), (5, 2))
    one.write(0, full[0, :3])
    one.write(3, full[0, 3:5])
    assert np.array_equal(one.close(), full[0, :5])


def test_state_roundtrip(tmp_path):
    from ip_mcmc_amd.chainio import ChainState, load_state, save_state

    st = ChainState(np.ones((4, 3)), np.arange(4.0), np.arange(4), None, 2**63 + 11, 12345, 77, "float32")
    p = save_state(str(tmp_path / "st"), st)
    r = load_state(p)
    assert r.seed == st.seed and r.step == 12345 and r.proposer_i == 77 and r.dtype == "float32"
    assert np.array_equal(r.u, st.u) and np.array_equal(r.phi, st.phi) and r.calls is None


@pytest.mark.gpu
def test_resume_is_exact_and_streaming_matches(tmp_path):
    """run(n1) -> checkpoint -> save/load -> run(n2) equals one run of n1+n2 samples,
    bit for bit; sample_file streaming equals the in-memory samples."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             Lorenz96Operator, MCMCSampler, PhiloxRNG, VarSteppCNProposer, pCNAccepter)
    from ip_mcmc_amd.chainio import load_state, save_state

    op = Lorenz96Operator(8, 8.0, dt=0.01, n_steps=50)
    y = op(np.zeros(8)) + 0.05
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(8), 0.01 * np.eye(8)))
    prior = GaussianDistribution(np.zeros(8), np.eye(8))
    for make in (lambda: ConstSteppCNProposer(0.3, prior), lambda: VarSteppCNProposer(lambda i: 0.1 + 0.2 / i, prior)):
        u0 = np.zeros((33, 8))
        s_full = MCMCSampler(make(), CountedAccepter(pCNAccepter(pot)), PhiloxRNG(5))
        full = s_full.run(u0, n_samples=12, burn_in=30, sample_interval=5)
        s1 = MCMCSampler(make(), CountedAccepter(pCNAccepter(pot)), PhiloxRNG(5))
        a = s1.run(u0, n_samples=7, burn_in=30, sample_interval=5)
        p = save_state(str(tmp_path / "ck"), s1.checkpoint())
        s2 = MCMCSampler(make(), CountedAccepter(pCNAccepter(pot)), PhiloxRNG(999))
        b = s2.run(load_state(p), n_samples=5, burn_in=0, sample_interval=5, sample_file=str(tmp_path / "b.npy"),
                   flush_every=2)
        assert np.array_equal(np.concatenate([a, np.asarray(b)], axis=1), full)
        assert np.array_equal(s2.checkpoint().u, s_full.checkpoint().u)
        assert np.array_equal(s2.checkpoint().accepts, s_full.checkpoint().accepts)
