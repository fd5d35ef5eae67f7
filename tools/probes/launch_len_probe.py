"""Per-step time of the headline sweep in launches of 1, 20 and 152 pCN steps
(bench.py's Workload: device-resident state, HIP events around the whole
sequence of launches), interleaved -- does a long launch cost more per step
than one-step launches?

  python tools/probes/launch_len_probe.py [reps]   -> one JSON line per (rep, launch length)
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    prob = bench.make_problem("cfg3")
    steps = 60
    ws = {n: bench.Workload(prob, prob.chains, 0, torch.float64, dev, per_launch=n) for n in (1, 20, 60)}
    ws[1].settle_clocks(0.5)
    for rep in range(reps):
        for n, w in ws.items():
            w.settle_clocks(0.2)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record()
            for m in w.launches(steps):
                w.step(m)
            b.record()
            torch.cuda.synchronize(dev)
            wall = time.perf_counter() - t0
            print(json.dumps({"rep": rep, "steps_per_launch": n, "steps": steps, "gpu_ms_per_step": a.elapsed_time(b) / steps,
                              "wall_ms_per_step": wall * 1e3 / steps}), flush=True)


if __name__ == "__main__":
    main()
