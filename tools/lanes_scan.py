"""Time the Lorenz-96 sweep for every layout (lanes per chain x chains per lane).

  python tools/lanes_scan.py [chains] [d] [rk_steps]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench as B  # noqa: E402
from ip_mcmc_amd import Lorenz96Operator  # noqa: E402
from ip_mcmc_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
chains = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
d = int(sys.argv[2]) if len(sys.argv) > 2 else 40
n = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
op = Lorenz96Operator(d, 8.0, dt=0.005, n_steps=n)
y = op(np.zeros(d)) + 0.1 * np.random.default_rng(3).normal(size=d)
flop = 30 * d * n
for dt, cpls in ((torch.float32, (1, 2)), (torch.float64, (1,))):
    for cpl in cpls:
        for lanes in (1, 2, 4, 8, 16):
            try:
                w = B.Workload(op, y, chains, 0, dt, dev, lanes, d=d)
                w.s.chains_per_lane = cpl
                el, k = B.timed(w, 3, 1, 1)
            except Exception as e:  # no instantiation for this layout
                print(f"{str(dt):14s} cpl={cpl} lanes={lanes:2d}  n/a ({str(e)[:60]})", flush=True)
                continue
            tf = chains * flop / (k * 1e-3) / 1e12
            print(f"{str(dt):14s} cpl={cpl} lanes={lanes:2d}  {k:9.3f} ms/sweep  {chains / (k * 1e-3):12.0f} "
                  f"pCN steps/s  {tf:6.1f} TFLOP/s", flush=True)
    m, _ = op.model(dt, dev)
    auto = lib().ipmc_auto_layout(C.byref(m), 0 if dt == torch.float32 else 1, chains)
    print(f"{str(dt):14s} auto layout: chains_per_lane={auto // 100} lanes={auto % 100}", flush=True)
