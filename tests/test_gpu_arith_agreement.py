"""The benched arithmetic against the reference's, on a stationary posterior at
the headline shape.

bench.py times the FMA forward map; the chains pinned bit for bit to the
reference fixtures run REFERENCE arith (no FMA, lorenz.py:77-81's order).
tools/posterior_agreement.py (`arith`) runs both on the forcing-field
posterior at the headline shape (Lorenz-96 d=40, 2 000 RK4 steps, f64) with
the reference's own noise recipe (lorenz_mcmc.py:100-112: γ = r·sd(X_k)) at
r = 2, where the chaotic time average's misfit noise is below one unit
(sqrt(d)·σ_ε/γ ≈ 0.5; at the reference's r = 0.5 it is ~2 and the chains
stick: R̂ 2.1 after 2 400 steps, profiles/r4/posterior_explore_r05.jsonl), from
independent prior draws u_0 with independent Philox seeds, long enough to
reach stationarity; it discards the burn-in diagnostics.burn_in_lengths finds
and estimates Monte-Carlo standard errors by batch means.  The stated
tolerance:

* the ensemble is stationary after the burn-in: the chains' first-half and
  second-half means agree in mean and in spread (|z| < Z_MAX for every
  component; exact for independent chains whatever their autocorrelation --
  split-R̂, which also asks every chain to have explored the posterior, is
  reported);
* the posterior means of the two arithmetics agree: max_i |z_i| < Z_MAX
  (family-wise false alarm ~0.25 % over 40 components) and both mean z² and
  the whitened T²/d lie in 1 ± 3.5·sqrt(2/d) (two-sided: a statistic far below
  1 means the standard errors are mis-calibrated);
* paired (same u_0 and draws): at least PAIRED_MIN of the chains make the same
  accept decisions over the whole run.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

D = 40
PAIRED_MIN = 0.99
Z_MAX = 4.0
BAND = 3.5 * np.sqrt(2 / D)
# (chains, blocks, steps per block, beta, noise level r): 4 800 pCN steps per chain
RUN = (8192, 96, 50, 0.3, 2.0)


def test_fma_and_reference_posteriors_agree_at_the_headline_shape():
    import torch

    import posterior_agreement as PA

    assert torch.cuda.is_available()
    chains, n_seg, seg_len, beta, noise_r = RUN
    r = PA.measure("arith", chains, n_seg, seg_len, beta, noise_r)
    print(r)
    PA.record(r, "posterior_agreement.jsonl")
    assert r["d"] == D and r["rk4_steps"] == 2000 and r["chains"] == chains
    assert "burn_in_capped_from" not in r, r  # the burn-in ends inside the run
    for arm in ("fma_float64", "reference_float64"):
        a = r[arm]
        assert 0.02 < a["accept_rate"] < 0.98, a
        assert a["half_z_max"] < Z_MAX and a["half_var_z_max"] < Z_MAX, a
    assert r["max_z"] < Z_MAX, r
    assert abs(r["mean_z2"] - 1) < BAND, r
    assert abs(r["t2_over_d"] - 1) < BAND, r
    assert r["paired_identical_accept_counts"] >= PAIRED_MIN, r


# the reference's own noise level r = 0.5 (lorenz_mcmc.py:92): the chains stick
# for thousands of steps (R-hat 2.1 after 2 400), so 50 000 pCN steps per chain
# (R-hat 1.05; profiles/r5/posterior_r05_long.jsonl), unpaired
RUN_R05 = (8192, 40, 1250, 0.2, 0.5)


def test_fma_and_reference_posteriors_agree_at_the_references_noise_level():
    import torch

    import posterior_agreement as PA

    assert torch.cuda.is_available()
    chains, n_seg, seg_len, beta, noise_r = RUN_R05
    r = PA.measure("arith", chains, n_seg, seg_len, beta, noise_r, paired=False)
    print(r)
    assert r["d"] == D and r["noise_r"] == 0.5 and r["pcn_steps"] == 50000
    assert "burn_in_capped_from" not in r, r
    for arm in ("fma_float64", "reference_float64"):
        a = r[arm]
        assert 0.02 < a["accept_rate"] < 0.98, a
        assert a["half_z_max"] < Z_MAX and a["half_var_z_max"] < Z_MAX, a
        assert a["rhat_max"] < 1.2, a
    assert r["max_z"] < Z_MAX, r
    assert abs(r["mean_z2"] - 1) < BAND, r
    assert abs(r["t2_over_d"] - 1) < BAND, r


def test_fp32_and_fp64_posteriors_agree_at_the_references_noise_level():
    """The precision twin of the test above: fp32 against fp64
    (both FMA arith) at the headline shape and the reference's own r = 0.5
    (lorenz_mcmc.py:92,111-112), 50 000 pCN steps per chain from independent
    u_0 and seeds, the same stationarity and agreement bounds.  Config 5's
    shape at r = 0.5 (10 min of GPU) stays a recorded tool run:
    profiles/r5/posterior_prec_r05_long.jsonl."""
    import torch

    import posterior_agreement as PA

    assert torch.cuda.is_available()
    chains, n_seg, seg_len, beta, noise_r = RUN_R05
    r = PA.measure("prec40", chains, n_seg, seg_len, beta, noise_r, paired=False)
    print(r)
    PA.record(r, "posterior_agreement.jsonl")
    assert r["d"] == D and r["noise_r"] == 0.5 and r["pcn_steps"] == 50000 and r["rk4_steps"] == 2000
    assert "burn_in_capped_from" not in r, r
    for arm in ("fma_float64", "fma_float32"):
        a = r[arm]
        assert 0.02 < a["accept_rate"] < 0.98, a
        assert a["half_z_max"] < Z_MAX and a["half_var_z_max"] < Z_MAX, a
        assert a["rhat_max"] < 1.2, a
    assert r["max_z"] < Z_MAX, r
    assert abs(r["mean_z2"] - 1) < BAND, r
    assert abs(r["t2_over_d"] - 1) < BAND, r
