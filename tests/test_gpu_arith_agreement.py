"""The benched arithmetic against the reference's at the headline shape.

bench.py times the FMA forward map; the chains pinned bit for bit to the
reference fixtures run REFERENCE arith (no FMA, lorenz.py:77-81's order).  At
65 536 chains x d=40 x 2 000 RK4 steps in f64 (tools/arith_agreement.py,
profiles/r3/arith_agreement.jsonl) this states how far apart they are:

* paired (same u_0, same Philox draws): at least PAIRED_MIN of the chains make
  identical accept decisions over the whole run (identical accept counts);
* independent seeds: the posterior-mean estimates of every one of the 40
  components agree within Z_MAX Monte-Carlo standard errors (family-wise
  false-alarm probability ~0.25 % at Z_MAX = 4 over 40 components), and the
  mean z² is below 1 + 3·sqrt(2/40) (a chi-square bound on all 40 at once).
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

PAIRED_MIN = 0.99
Z_MAX = 4.0
MEAN_Z2_MAX = 1 + 3 * np.sqrt(2 / 40)


@pytest.mark.parametrize("beta,start", [(0.2, "zero"), (0.02, "posterior")])
def test_fma_and_reference_arith_agree_at_the_headline_shape(beta, start):
    import torch

    import arith_agreement as A

    assert torch.cuda.is_available()
    r = A.measure(beta, 40, chains=65536, start=start)
    print(r)
    assert r["chains"] == 65536
    assert r["paired_identical_accept_counts"] >= PAIRED_MIN, r
    assert r["indep_max_z"] < Z_MAX, r
    assert r["indep_mean_z2"] < MEAN_Z2_MAX, r
    assert r["accept_rate_fma"] > 0 and r["accept_rate_ref"] > 0
