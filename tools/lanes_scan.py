"""Time the L96 sweep kernel for every lanes-per-chain layout (tools only)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench as B

dev = torch.device("cuda", 0)
op, y = B.problem()
chains = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
for dt in (torch.float32, torch.float64):
    for lanes in (1, 2, 4, 8):
        try:
            w = B.Workload(op, y, chains, 0, dt, dev, lanes)
            el, k = B.timed(w, 5, 2, 1)
        except Exception as e:  # no instantiation
            print(dt, lanes, "n/a", e, flush=True)
            continue
        tf = chains * B.FLOP_PER_STEP / (k * 1e-3) / 1e12
        print(f"{str(dt):14s} lanes={lanes}  {k:8.3f} ms/sweep  {chains / (k * 1e-3):12.0f} pCN steps/s  {tf:6.1f} TFLOP/s", flush=True)
