"""fp32 vs fp64 on a stationary posterior at config 5's shape: the stated
floating-point tolerance.

Per chain the two precisions part ways under the chaotic forward map, so the
bar is statistical.  tools/posterior_agreement.py (`prec`) runs fp64 and fp32
on the forcing-field posterior at d=256 with config 5's 10 000 RK4 steps per
forward map (the reference's noise recipe, lorenz_mcmc.py:100-112, γ = r·sd(X_k)
at r = 2: misfit noise below one unit; at r = 0.5, R̂ 2.7 after 1 200 steps),
from independent prior draws u_0 with independent Philox seeds, discards the
burn-in diagnostics.burn_in_lengths finds and estimates Monte-Carlo standard
errors by batch means.  The stated tolerance:

* stationarity of the ensemble: first vs second half of the post-burn-in run,
  |z| < Z_MAX for the mean and for the spread (split-R̂ reported);
* the posterior means agree: max_i |z_i| < Z_MAX (family-wise false alarm
  ~0.3 % over 256 components) and mean z² and the whitened T²/d within
  1 ± 3.5·sqrt(2/256) = 1 ± 0.31, two-sided (round 3's independent-seed test
  gave mean z² = 0.38 on short transient runs: that run would now fail);
* paired fp32 (the fp64 run's u_0 and draws) is reported: the fraction of
  chains whose accept counts stay identical.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

D = 256
Z_MAX = 4.5
BAND = 3.5 * np.sqrt(2 / D)
# (chains, blocks, steps per block, beta, noise level r): 2 400 pCN steps per chain
RUN = (8192, 48, 50, 0.3, 2.0)


def test_fp32_and_fp64_posteriors_agree_at_config5_shape():
    import torch

    import posterior_agreement as PA

    assert torch.cuda.is_available()
    chains, n_seg, seg_len, beta, noise_r = RUN
    r = PA.measure("prec", chains, n_seg, seg_len, beta, noise_r)
    print(r)
    PA.record(r, "posterior_agreement.jsonl")
    assert r["d"] == D and r["rk4_steps"] == 10000 and r["chains"] == chains
    assert "burn_in_capped_from" not in r, r
    for arm in ("fma_float64", "fma_float32"):
        a = r[arm]
        assert 0.02 < a["accept_rate"] < 0.98, a
        assert a["half_z_max"] < Z_MAX and a["half_var_z_max"] < Z_MAX, a
    assert r["max_z"] < Z_MAX, r
    assert abs(r["mean_z2"] - 1) < BAND, r
    assert abs(r["t2_over_d"] - 1) < BAND, r
    assert 0 <= r["paired_identical_accept_counts"] <= 1
