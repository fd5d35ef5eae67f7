"""Device chain diagnostics (ipmc_autocorr, ipmc_burn_in) vs the reference's outputs and the oracle."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_autocorr_matches_reference_fixture(golden):
    from ip_mcmc_amd.diagnostics import autocorr

    got = autocorr(golden["ac_x"])
    np.testing.assert_allclose(got, golden["ac_ref"], rtol=1e-10, atol=1e-12)
    assert np.all(got[5] == 1.0)  # constant series: the reference returns ones


def test_sampler_autocorr_is_the_device_kernel(golden):
    """MCMCSampler.autocorr (sampler.py:43-54) runs ipmc_autocorr and reproduces the reference's outputs."""
    from ip_mcmc_amd import MCMCSampler

    for x, ref in zip(golden["ac_x"], golden["ac_ref"]):
        np.testing.assert_allclose(MCMCSampler.autocorr(x), ref, rtol=1e-10, atol=1e-12)


def test_autocorr_lags_and_dtypes(orc):
    from ip_mcmc_amd.diagnostics import autocorr

    x = np.random.default_rng(1).normal(size=(3, 7, 500)).cumsum(axis=-1)
    got = autocorr(x, max_lag=50)
    ref = np.stack([orc.autocorr_ref(s)[:50] for s in x.reshape(-1, 500)]).reshape(3, 7, 50)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
    got32 = autocorr(torch.as_tensor(x, dtype=torch.float32).cuda(), max_lag=50).cpu().numpy()
    np.testing.assert_allclose(got32, ref, rtol=0, atol=2e-5)


def test_autocorr_of_series_longer_than_lds(orc):
    """Series over 8 192 samples (MCMCSampler.autocorr on a whole long chain,
    sampler.py:43-54 accepts any length) go through the LDS-tiled kernel:
    all lags of a 12 000-sample chain, partial lags of a batch, a constant
    series (ones), f32 input, and a strided (C, n, k) chain layout."""
    from ip_mcmc_amd import MCMCSampler
    from ip_mcmc_amd.diagnostics import autocorr, chain_autocorr

    rng = np.random.default_rng(11)
    x = rng.normal(size=12000).cumsum()
    np.testing.assert_allclose(MCMCSampler.autocorr(x), orc.autocorr_ref(x), rtol=1e-10, atol=1e-12)
    b = rng.normal(size=(3, 9001)).cumsum(axis=-1)
    b[1] = 2.5
    got = autocorr(b, max_lag=700)
    assert got.shape == (3, 700) and np.all(got[1] == 1.0)
    for i in (0, 2):
        np.testing.assert_allclose(got[i], orc.autocorr_ref(b[i])[:700], rtol=1e-10, atol=1e-12)
    got32 = autocorr(torch.as_tensor(b, dtype=torch.float32).cuda(), max_lag=300).cpu().numpy()
    np.testing.assert_allclose(got32[0], orc.autocorr_ref(b[0].astype(np.float32))[:300], rtol=0, atol=2e-5)
    samples = rng.normal(size=(2, 10000, 3)).cumsum(axis=1)
    got = chain_autocorr(samples, 257)
    np.testing.assert_allclose(got[1, 2], orc.autocorr_ref(samples[1, :, 2])[:257], rtol=1e-10, atol=1e-12)


def test_autocorrelation_windows_and_chain_layout(orc):
    """helpers.autocorrelation (helpers.py:41-54) restated with the reference's
    per-window MCMCSampler.autocorr (the oracle's restatement), and the (C, n, k) chain layout."""
    from ip_mcmc_amd.diagnostics import autocorrelation, chain_autocorr

    s = np.random.default_rng(2).normal(size=(3, 1000)).cumsum(axis=1)
    tau = 100
    ref = np.zeros((3, tau))
    for i in range(1000 // tau):
        for var in range(3):
            ref[var] += orc.autocorr_ref(s[var, i * tau:(i + 1) * tau])
    ref /= 1000 // tau
    np.testing.assert_allclose(autocorrelation(s, tau), ref, rtol=1e-10, atol=1e-12)
    samples = np.random.default_rng(3).normal(size=(4, 64, 5))
    got = chain_autocorr(samples, 10)
    assert got.shape == (4, 5, 10)
    np.testing.assert_allclose(got[2, 3], orc.autocorr_ref(samples[2, :, 3])[:10], rtol=1e-10, atol=1e-12)


# ------------------------------------------------------ burn-in (§8(f) #2)
def test_burn_in_matches_reference_fixture(golden, orc):
    """ipmc_burn_in vs the reference's len_burn_in (utilities.py:134-167): identical indices."""
    from ip_mcmc_amd.diagnostics import burn_in_lengths, len_burn_in

    for i in range(int(golden["bi_count"])):
        assert len_burn_in(golden[f"bi_x_{i}"]) == int(golden[f"bi_out_{i}"]), i
    B = golden["bi_batch_x"]
    assert np.array_equal(burn_in_lengths(B), golden["bi_batch_out"])
    # run()'s (C, n_samples, k) layout
    assert np.array_equal(burn_in_lengths(np.ascontiguousarray(B.transpose(0, 2, 1)), layout="time_vars"),
                          golden["bi_batch_out"])
    # fp32 input: the oracle on the same fp32-rounded values
    B32 = torch.as_tensor(B, dtype=torch.float32).cuda()
    want = orc.burn_in(B32.double().cpu().numpy())
    assert np.array_equal(burn_in_lengths(B32).cpu().numpy(), want)


def test_burn_in_large_batch_vs_oracle(orc):
    """65 536-chain-scale batch semantics on 2 048 chains x 4 vars x 3 000 samples."""
    from ip_mcmc_amd.diagnostics import burn_in_lengths

    rng = np.random.default_rng(5)
    C, k, n = 2048, 4, 3000
    t = np.arange(n)
    drift = rng.uniform(1, 10, size=(C, k, 1)) * np.exp(-t / rng.uniform(30, 600, size=(C, 1, 1)))
    x = 0.3 + drift + 0.05 * rng.normal(size=(C, k, n)).cumsum(axis=-1) / np.sqrt(t + 1)
    got = burn_in_lengths(x)
    assert np.array_equal(got, orc.burn_in(x))
    assert len(set(got.tolist())) > 20


def test_spacing_and_clean_samples_match_reference_fixture(golden):
    from ip_mcmc_amd.diagnostics import clean_samples, uncorrelated_sample_spacing

    for j in range(3):
        x = golden[f"us_x_{j}"]
        assert uncorrelated_sample_spacing(x) == int(golden[f"us_out_{j}"])
        assert np.array_equal(clean_samples(x), golden[f"cs_out_{j}"])


def test_burn_in_rejects_short_series():
    from ip_mcmc_amd.diagnostics import burn_in_lengths

    with pytest.raises(ValueError):
        burn_in_lengths(np.zeros((2, 3, 49)))
