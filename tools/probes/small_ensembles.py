"""The headline problem (bench.py's config 3: d=40, 2 000 RK4 steps, its
posterior and acceptance) with small ensembles: sequential sweeps vs
speculation inside one wave vs speculation over a whole block (auto).

  python tools/probes/small_ensembles.py [chains ...]

One JSON line per (chains, dtype, mode): pCN steps/s, accept rate, steps per
launch 256, 2 warm-up launches then 4 timed (HIP events).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench as B  # noqa: E402

PER_LAUNCH = 256


def run(op, y, n, dtype, spec, dev):
    w = B.Workload(op, y, n, 0, dtype, dev)
    if spec < 0:  # the widest speculation inside one wave for the auto layout
        spec = max(1, 64 // w.lanes)
    w.s.n_steps, w.s.spec_width = PER_LAUNCH, spec
    for _ in range(2):
        B.call("ipmc_pcn_sweep", B.C.byref(w.model), B.C.byref(w.s), w.stream)
        w.s.step0 += PER_LAUNCH
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(4):
        B.call("ipmc_pcn_sweep", B.C.byref(w.model), B.C.byref(w.s), w.stream)
        w.s.step0 += PER_LAUNCH
    b.record()
    torch.cuda.synchronize(dev)
    sec = a.elapsed_time(b) / 1e3
    return n * 4 * PER_LAUNCH / sec, float(w.acc.sum().item()) / (n * 6 * PER_LAUNCH), w.lanes


def main():
    dev = torch.device("cuda", 0)
    op, y = B.problem()
    for n in [int(a) for a in sys.argv[1:]] or (1, 64, 256, 1024, 4096, 8192):
        for dtype in (torch.float64, torch.float32):
            for mode, spec in (("sequential", 1), ("wave", -1), ("auto", 0)):
                rate, acc, lanes = run(op, y, n, dtype, spec, dev)
                print(json.dumps({"chains": n, "dtype": str(dtype).split(".")[-1], "mode": mode, "spec_width": spec,
                                  "lanes_per_chain": lanes, "pcn_steps_per_s": rate, "accept_rate": acc}),
                      flush=True)


if __name__ == "__main__":
    main()
