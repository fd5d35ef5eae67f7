"""Debug: which speculative ts / Burgers sweep sums differ from the oracle.

  [IPMC_LIB_PATH=variant] python tools/probes/spec_tree_debug.py [case-prefix ...]
  (round 5 ran `bur128` against variant builds whose walk read the proposals by
  __shfl -- from every lane of the chain: correct, profiles/r5/walk_shfl_all_lanes.txt;
  under the first lane's branch, the source lanes inactive: wrong sums,
  profiles/r5/walk_shfl_first_lane.txt)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_parity as T  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from ip_mcmc_amd import BurgersOperator, TwoScaleLorenz96Operator  # noqa: E402

dev = torch.device("cuda", 0)
dtype = torch.float64
rng = np.random.default_rng(31)
cases = []
for K, J, arith in ((6, 4, "fma"), (3, 1, "reference"), (11, 2, "fma")):
    op = TwoScaleLorenz96Operator(K=K, J=J, x0=rng.normal(size=K * (1 + J)), dt=0.004, n_steps=25, arith=arith)
    cases.append((f"ts{K}", op, (1, 0, 2, 64 // K)))
for N, arith in ((128, "reference"), (256, "fma")):
    op = BurgersOperator(N=N, dt_mode="cfl", T=0.2, arith=arith)
    cases.append((f"bur{N}", op, (1, 0, 2, 4, 16) if N == 128 else (1, 0, 2, 8)))
only = sys.argv[1:]
for name, op, widths in cases:
    if only and not any(name.startswith(o) for o in only):
        continue
    for scale in (0.2, 3.0):
        U0, phi0, y, ginv, sq = T._problem(op, 19, dtype, orc, seed=3)
        ginv = ginv * scale
        phi0 = orc.potential(op, U0, y, ginv, T._np(dtype)).astype(np.float64)
        for n in (1, 2, 3, 5, 17):
            o = T._sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 8, 2**32 - 3, n, dtype, want_sums=True)
            for w in widths:
                d = T._sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 8, 2**32 - 3, n, dtype, dev, spec=w,
                                    want_sums=True)
                same = all(np.array_equal(d[k], o[k]) for k in ("u", "phi", "acc", "calls"))
                bad = np.where(~np.all(d["sum_u"] == o["sum_u"], axis=1))[0]
                if not same or len(bad):
                    print(name, scale, "n", n, "w", w, "state_same", same, "bad chains", bad.tolist(),
                          "acc", o["acc"][bad].tolist(), flush=True)
                    for c in bad[:2]:
                        print("   dev", d["sum_u"][c], "orc", o["sum_u"][c], "u0", U0[c], "u", o["u"][c], flush=True)
print("done")
