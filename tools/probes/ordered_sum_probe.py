"""The posterior mean's chain-ordered column sum: device (ipmc_ordered_sum) vs
the host library (ipmc_host_ordered_sum) on the headline's per-chain sums
(65 536 x 40), a rank's share of them at 8 GPUs (8 192 x 40) and config 5's
(2^17 x 256 per GPU of 8); same bits asserted.

  python tools/probes/ordered_sum_probe.py  -> one JSON line per shape
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ip_mcmc_amd import _hostlib  # noqa: E402
from ip_mcmc_amd import device as D  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    for n, k in ((65536, 40), (8192, 40), (131072, 256)):
        a = rng.normal(size=(n, k))
        rows = torch.as_tensor(a, device=dev)
        acc = torch.zeros(k, dtype=torch.float64, device=dev)
        D.ordered_sum(rows, acc)  # warm
        torch.cuda.synchronize()
        reps = 20
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(reps):
            acc.zero_()
            D.ordered_sum(rows, acc)
        ev1.record()
        torch.cuda.synchronize()
        dev_ms = ev0.elapsed_time(ev1) / reps
        want = np.zeros(k)
        t0 = time.perf_counter()
        for _ in range(reps):
            want[:] = 0
            _hostlib.ordered_sum(a, want)
        host_ms = (time.perf_counter() - t0) / reps * 1e3
        assert np.array_equal(acc.cpu().numpy(), want)
        print(json.dumps({"rows": n, "k": k, "device_ms": dev_ms, "host_ms": host_ms, "bit_equal": True}), flush=True)


if __name__ == "__main__":
    main()
