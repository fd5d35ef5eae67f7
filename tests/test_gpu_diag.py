"""Device chain diagnostics (ipmc_autocorr) vs the reference's MCMCSampler.autocorr."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_autocorr_matches_reference_fixture(golden):
    from ip_mcmc_amd.diagnostics import autocorr

    got = autocorr(golden["ac_x"])
    np.testing.assert_allclose(got, golden["ac_ref"], rtol=1e-10, atol=1e-12)
    assert np.all(got[5] == 1.0)  # constant series: the reference returns ones


def test_autocorr_lags_and_dtypes():
    from ip_mcmc_amd import MCMCSampler
    from ip_mcmc_amd.diagnostics import autocorr

    x = np.random.default_rng(1).normal(size=(3, 7, 500)).cumsum(axis=-1)
    got = autocorr(x, max_lag=50)
    ref = np.stack([MCMCSampler.autocorr(s)[:50] for s in x.reshape(-1, 500)]).reshape(3, 7, 50)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
    got32 = autocorr(torch.as_tensor(x, dtype=torch.float32).cuda(), max_lag=50).cpu().numpy()
    np.testing.assert_allclose(got32, ref, rtol=0, atol=2e-5)


def test_autocorrelation_windows_and_chain_layout():
    """helpers.autocorrelation (helpers.py:41-54) restated with the reference's
    per-window MCMCSampler.autocorr, and the (C, n, k) chain layout."""
    from ip_mcmc_amd import MCMCSampler
    from ip_mcmc_amd.diagnostics import autocorrelation, chain_autocorr

    s = np.random.default_rng(2).normal(size=(3, 1000)).cumsum(axis=1)
    tau = 100
    ref = np.zeros((3, tau))
    for i in range(1000 // tau):
        for var in range(3):
            ref[var] += MCMCSampler.autocorr(s[var, i * tau:(i + 1) * tau])
    ref /= 1000 // tau
    np.testing.assert_allclose(autocorrelation(s, tau), ref, rtol=1e-10, atol=1e-12)
    samples = np.random.default_rng(3).normal(size=(4, 64, 5))
    got = chain_autocorr(samples, 10)
    assert got.shape == (4, 5, 10)
    np.testing.assert_allclose(got[2, 3], MCMCSampler.autocorr(samples[2, :, 3])[:10], rtol=1e-10, atol=1e-12)
