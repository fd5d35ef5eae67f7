"""Where the wall time of bench.py's end-to-end leg goes outside the GPU work,
for the metric's 8-GPU share on one GPU (8 192 chains, K = 20 by default):
bench.timed_run's warm-up, then `reps` timed run_sharded calls, each with the
sampler's own split (set-up, Φ(u_0) and sweep GPU time, tail) and the gather;
the last one under cProfile (top functions by own time to stderr).

  python tools/probes/shard_e2e_profile.py [chains] [steps] [reps] [tag]
  -> one JSON line per timed run
"""
import cProfile
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from ip_mcmc_amd.shard import run_sharded  # noqa: E402


def main():
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    tag = sys.argv[4] if len(sys.argv) > 4 else "default"
    dev = torch.device("cuda", 0)
    prob = bench.make_problem("cfg3")
    make = bench.sampler_factory(prob, np.float64, dev)
    u0 = torch.zeros((chains, prob.k), dtype=torch.float64, device=dev)
    kw = dict(n_samples=1, burn_in=0, sample_interval=steps, keep="moments", gather="mean", results="device")
    run_sharded(make, u0, **dict(kw, sample_interval=5))
    w = bench.Workload(prob, chains, 0, torch.float64, dev)
    for r in range(reps):
        w.settle_clocks(0.3)
        torch.cuda.synchronize(dev)
        pr = cProfile.Profile() if r == reps - 1 else None
        t0 = time.perf_counter()
        if pr:
            pr.enable()
        res = run_sharded(make, u0, **kw)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if pr:
            pr.disable()
        tm = res["sampler"].last_run_timing
        print(json.dumps({"tag": tag, "chains": chains, "steps": steps, "rep": r, "profiled": pr is not None,
                          "wall_ms": el * 1e3, "pcn_steps_per_s": chains * steps / el,
                          "run_ms": res["run_seconds"] * 1e3, "gather_ms": res["gather_seconds"] * 1e3,
                          "setup_ms": tm["setup_s"] * 1e3, "phi0_gpu_ms": tm["phi0_gpu_ms"],
                          "sweeps_gpu_ms": tm["sweeps_gpu_ms"], "tail_ms": tm["tail_ms"],
                          "outside_run_ms": (el - res["run_seconds"]) * 1e3 - res["gather_seconds"] * 1e3}),
              flush=True)
        if pr:  # own time per function in microseconds (pstats prints milliseconds at best)
            st = pstats.Stats(pr)
            rows = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:40]
            for (fn, line, name), (cc, nc, tt, ct, _) in rows:
                print(f"{tt * 1e6:9.1f} us own {ct * 1e6:9.1f} us cum {nc:5d} calls  {os.path.basename(fn)}:{line}({name})",
                      file=sys.stderr)


if __name__ == "__main__":
    main()
