"""Kernel-leg time of the headline sweep in FMA and REFERENCE arith (bench.py's
Workload: device-resident state, one pCN step per launch, HIP events), for the
libipmc.so that IPMC_LIB_PATH selects (occupancy / code-shape A/Bs).

  IPMC_LIB_PATH=... python tools/probes/arith_kernel_probe.py [tag] [steps] [dtype] [workload]
  -> one JSON line per arithmetic
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "default"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dt = torch.float64 if (len(sys.argv) <= 3 or sys.argv[3] == "f64") else torch.float32
    key = sys.argv[4] if len(sys.argv) > 4 else "cfg3"
    dev = torch.device("cuda", 0)
    prob = bench.make_problem(key)
    for arith, p in (("fma", prob), ("reference", prob.reference_arith())):
        w = bench.Workload(p, prob.chains, 0, dt, dev)
        el, kms = bench.timed(w, steps, 10, 1, settle_s=0.3)
        print(json.dumps({"tag": tag, "lib": os.environ.get("IPMC_LIB_PATH", "product"), "workload": key,
                          "arith": arith, "dtype": str(dt).split(".")[-1], "chains": prob.chains, "steps": steps,
                          "kernel_ms": kms, "pcn_steps_per_s": prob.chains * steps / el,
                          "tflops": prob.chains * prob.flop / (kms * 1e-3) / 1e12, "lanes": w.lanes}), flush=True)
        del w
        torch.cuda.synchronize(dev)


if __name__ == "__main__":
    main()
