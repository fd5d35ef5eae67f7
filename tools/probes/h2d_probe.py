"""H2D of the headline u_0 (65 536 x 40 f64) through device.to_device:
pageable vs page-locked staging, repeated (the staging block is recycled)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ip_mcmc_amd import device as dev  # noqa: E402


def main():
    d = torch.device("cuda", 0)
    x = np.zeros((65536, 40))
    torch.zeros(1, device=d)
    for label, thr in (("pinned", 1 << 22), ("pageable", 1 << 62)):
        dev.PINNED_H2D_MIN_BYTES = thr
        for i in range(4):
            torch.cuda.synchronize(d)
            t = time.perf_counter()
            y = dev.to_device(x, torch.float64, d)
            t1 = time.perf_counter()
            torch.cuda.synchronize(d)
            t2 = time.perf_counter()
            print(f"{label} {i}: host {1e3 * (t1 - t):.2f} ms, to completion {1e3 * (t2 - t):.2f} ms", flush=True)
            del y


if __name__ == "__main__":
    main()
