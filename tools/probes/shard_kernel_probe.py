"""Kernel-leg time of the metric's 8-GPU share on one GPU: 8 192 chains of the
headline problem (global chain ids from 7 x 8 192, rank 7 of 8), one launch of
K pCN steps (the driver's K = 20), HIP events on the launch stream, for the
libipmc.so that IPMC_LIB_PATH selects (layout / schedule A/Bs of
l96_sweep_kernel<double, 40, 8, true>).

  IPMC_LIB_PATH=... python tools/probes/shard_kernel_probe.py [tag] [steps] [chains] [repeats] [sums]
  -> one JSON line per repeat
`sums`: the launches also accumulate the per-chain sums of u and u^2
(ipmc_sweep.sum_u / sum_u2), as MCMCSampler.run(keep="moments") does.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "default"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    chains = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    sums = len(sys.argv) > 5 and sys.argv[5] == "sums"
    dev = torch.device("cuda", 0)
    prob = bench.make_problem("cfg3")
    w = bench.Workload(prob, chains, 7 * chains, torch.float64, dev, per_launch=steps)
    if sums:
        su = torch.zeros((chains, prob.k), dtype=torch.float64, device=dev)
        su2 = torch.zeros_like(su)
        w.s.sum_u, w.s.sum_u2 = su.data_ptr(), su2.data_ptr()
    for r in range(reps):
        el, kms = bench.timed(w, steps, steps, 1, settle_s=0.3 if r == 0 else 0.1)
        print(json.dumps({"tag": tag, "lib": os.environ.get("IPMC_LIB_PATH", "product"), "chains": chains,
                          "chain_offset": 7 * chains, "steps_per_launch": steps, "sums": sums, "rep": r, "kernel_ms": kms,
                          "ms_per_pcn_step": kms / steps, "kernel_pcn_steps_per_s": chains * steps / (kms * 1e-3),
                          "tflops": chains * steps * prob.flop / (kms * 1e-3) / 1e12, "lanes": w.lanes,
                          "spec_width": w.spec_width}), flush=True)


if __name__ == "__main__":
    main()
