"""fp32 vs fp64: the stated floating-point tolerance.

Per chain the two precisions part ways under the chaotic forward map, so the
bar is statistical: with the same Philox draws and u_0 in both precisions, the
posterior mean of every parameter component agrees within 3 Monte-Carlo
standard errors,
    z_i = |m32_i - m64_i| / sqrt(se32_i^2 + se64_i^2) < 3   for every i,
se = between-chain standard deviation of the per-chain time averages / sqrt(C).
(tools/precision_sweep.py is the full-size version; profiles/r1/precision_sweep.jsonl.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

Z_TOL = 3.0


def _means(d, n_rk, beta, dtype, chains, n_samples):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             Lorenz96Operator, MCMCSampler, pCNAccepter)

    G = Lorenz96Operator(d, 8.0, dt=0.005, n_steps=n_rk)
    k = np.arange(d)
    y = G(0.5 * np.sin(2 * np.pi * k / d)) + 0.1 * np.random.default_rng(3).normal(size=d)
    acc = CountedAccepter(pCNAccepter(EvolutionPotential(G, y, GaussianDistribution(np.zeros(d), 0.01 * np.eye(d)))))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(d), np.eye(d))), acc, 11, dtype=dtype)
    u0 = 0.05 * np.random.default_rng(5).normal(size=(chains, d))
    mom = s.run(u0, n_samples=n_samples, burn_in=20, sample_interval=1, keep="moments")
    return mom["sum_u"] / mom["n"], np.asarray(acc.accepts)


@pytest.mark.parametrize("d,n_rk,beta", [(40, 2000, 0.2), (256, 1000, 0.02)])
def test_fp32_posterior_means_within_3_mcse_of_fp64(d, n_rk, beta):
    import torch

    assert torch.cuda.is_available()
    chains, n_samples = 4096, 100
    m64, a64 = _means(d, n_rk, beta, np.float64, chains, n_samples)
    m32, a32 = _means(d, n_rk, beta, np.float32, chains, n_samples)
    se64 = m64.std(axis=0, ddof=1) / np.sqrt(chains)
    se32 = m32.std(axis=0, ddof=1) / np.sqrt(chains)
    z = np.abs(m32.mean(axis=0) - m64.mean(axis=0)) / np.sqrt(se64**2 + se32**2)
    assert np.all(np.isfinite(z))
    assert z.max() < Z_TOL, (z.max(), np.argmax(z))
    # the accept totals agree within 3 binomial standard errors as well
    steps = chains * (n_samples + 19)
    p = a64.sum() / steps
    assert abs(int(a32.sum()) - int(a64.sum())) < 3 * np.sqrt(2 * steps * p * (1 - p)) + 1
