"""fp32 vs fp64: the stated floating-point tolerance.

Per chain the two precisions part ways under the chaotic forward map, so the
bar is statistical.  The two precisions run from independent u_0 draws (of
one distribution) with independent Philox seeds, so their posterior-mean
estimates are independent and the test can fail (with a shared u_0 the
short runs' time averages stay correlated through it and the z's shrink):
for every parameter component i
    z_i = |m32_i - m64_i| / sqrt(se32_i^2 + se64_i^2),
se = between-chain standard deviation of the per-chain time averages / sqrt(C),
max_i z_i < Z_MAX(d) (family-wise false alarm ~0.2 %: 4.0 for d = 40, 4.5 for
d = 256) and mean_i z_i^2 < 1 + 3 sqrt(2/d) (a chi-square bound on all
components at once); the accept totals agree within 4 between-chain standard
errors.  A third run repeats fp32 with the fp64 run's seed and reports the
fraction of chains with identical accept counts (paired: same u_0 and draws,
so only the arithmetic differs).  (tools/precision_sweep.py is the full-size version;
profiles/r1/precision_sweep.jsonl.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

Z_MAX = {40: 4.0, 256: 4.5}


def _means(d, n_rk, beta, dtype, chains, n_samples, seed, u0_seed):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             Lorenz96Operator, MCMCSampler, pCNAccepter)

    G = Lorenz96Operator(d, 8.0, dt=0.005, n_steps=n_rk)
    k = np.arange(d)
    y = G(0.5 * np.sin(2 * np.pi * k / d)) + 0.1 * np.random.default_rng(3).normal(size=d)
    acc = CountedAccepter(pCNAccepter(EvolutionPotential(G, y, GaussianDistribution(np.zeros(d), 0.01 * np.eye(d)))))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(d), np.eye(d))), acc, seed, dtype=dtype)
    u0 = 0.05 * np.random.default_rng(u0_seed).normal(size=(chains, d))
    mom = s.run(u0, n_samples=n_samples, burn_in=20, sample_interval=1, keep="moments")
    return mom["sum_u"] / mom["n"], np.asarray(acc.accepts, dtype=np.float64)


@pytest.mark.parametrize("d,n_rk,beta", [(40, 2000, 0.2), (256, 1000, 0.02)])
def test_fp32_posterior_means_within_mcse_of_fp64(d, n_rk, beta):
    import torch

    assert torch.cuda.is_available()
    chains, n_samples = 4096, 100
    m64, a64 = _means(d, n_rk, beta, np.float64, chains, n_samples, 11, 5)
    m32, a32 = _means(d, n_rk, beta, np.float32, chains, n_samples, 12, 6)  # independent u_0 and draws
    se64 = m64.std(axis=0, ddof=1) / np.sqrt(chains)
    se32 = m32.std(axis=0, ddof=1) / np.sqrt(chains)
    z = np.abs(m32.mean(axis=0) - m64.mean(axis=0)) / np.sqrt(se64**2 + se32**2)
    assert np.all(np.isfinite(z))
    print(f"d={d}: max z {z.max():.2f}, mean z^2 {np.mean(z**2):.2f}")
    assert z.max() < Z_MAX[d], (z.max(), np.argmax(z))
    assert np.mean(z**2) < 1 + 3 * np.sqrt(2 / d), np.mean(z**2)
    za = abs(a32.sum() - a64.sum()) / np.sqrt(chains * (a32.var(ddof=1) + a64.var(ddof=1)))
    assert za < 4.0, za
    # paired: the fp64 run's draws in fp32
    _, a32p = _means(d, n_rk, beta, np.float32, chains, n_samples, 11, 5)
    print(f"d={d}: paired fp32/fp64 chains with identical accept counts {np.mean(a32p == a64):.3f}")
    assert a32p.sum() > 0
