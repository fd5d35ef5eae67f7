"""The statistics behind the stated fp tolerances (tools/posterior_agreement.py)
on synthetic chains whose answer is known, on the CPU: independent stationary
AR(1) ensembles of one distribution give calibrated z / T² and R̂ ≈ 1; a
shifted mean is caught by z and T²; over-dispersed starts that have not
relaxed are caught by R̂ and the half-vs-half z; correlated components do not
break the whitened T²/d (they do widen mean z²'s spread)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import posterior_agreement as PA  # noqa: E402


def _ar1(rng, C, n, d, rho, sd=1.0, start_sd=None, mean=0.0, mix=None):
    """(C, n, d) block-mean-like AR(1) traces around `mean`, stationary unless
    start_sd differs from sd; `mix` (d, d) correlates the components."""
    x = np.empty((C, n, d))
    e = rng.normal(size=(C, n, d))
    if mix is not None:
        e = e @ mix.T
    x[:, 0] = (start_sd if start_sd is not None else sd) * e[:, 0]
    for t in range(1, n):
        x[:, t] = rho * x[:, t - 1] + np.sqrt(1 - rho**2) * sd * e[:, t]
    return x + mean


def test_independent_stationary_ensembles_are_calibrated():
    rng = np.random.default_rng(1)
    zs, t2s = [], []
    for _ in range(6):
        a = PA.summarize(_ar1(rng, 2048, 40, 40, 0.6), 10)
        b = PA.summarize(_ar1(rng, 2048, 40, 40, 0.6), 10)
        c = PA.compare(a, b)
        zs.append(c["max_z"])
        t2s.append(c["t2_over_d"])
        assert a["half_z_max"] < 4.0 and a["half_var_z_max"] < 4.0
    assert max(zs) < 4.0
    band = 3.5 * np.sqrt(2 / 40)
    assert all(abs(t - 1) < band for t in t2s) and abs(np.mean(t2s) - 1) < 0.25


def test_a_shifted_posterior_mean_is_caught():
    rng = np.random.default_rng(2)
    a = PA.summarize(_ar1(rng, 2048, 40, 40, 0.6), 10)
    shift = np.zeros(40)
    shift[7] = 0.05  # ~6 standard errors of one component
    b = PA.summarize(_ar1(rng, 2048, 40, 40, 0.6, mean=shift), 10)
    c = PA.compare(a, b)
    assert c["max_z"] > 4.0


def test_unrelaxed_overdispersed_starts_fail_stationarity():
    """Chains still relaxing from over-dispersed starts: the spread shrinks
    between the halves (caught); a stationary ensemble of the same slow
    chains passes although its R̂ is far above 1."""
    rng = np.random.default_rng(3)
    a = PA.summarize(_ar1(rng, 2048, 40, 40, 0.9, sd=0.3, start_sd=3.0), 10)
    assert a["half_var_z_max"] > 4.0
    b = PA.summarize(_ar1(rng, 2048, 40, 40, 0.9, sd=0.3), 10)
    assert b["half_var_z_max"] < 4.0 and b["half_z_max"] < 4.0 and b["rhat_max"] > 1.2


def test_correlated_components_keep_the_whitened_statistic():
    rng = np.random.default_rng(4)
    d = 40
    mix = np.eye(d) + 0.9 * np.ones((d, d)) / np.sqrt(d)  # one strong common mode
    t2 = []
    for _ in range(6):
        a = PA.summarize(_ar1(rng, 2048, 30, d, 0.5, mix=mix), 6)
        b = PA.summarize(_ar1(rng, 2048, 30, d, 0.5, mix=mix), 6)
        t2.append(PA.compare(a, b)["t2_over_d"])
    assert all(abs(t - 1) < 3.5 * np.sqrt(2 / d) for t in t2)
