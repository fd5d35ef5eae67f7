"""Sample streaming to .npy (run(sample_file=...)) vs in-memory samples at the
headline shape (Lorenz-96 d=40, 2 000 RK4 steps, 65 536 chains, every 10th step
recorded).  Also times the previous synchronous writer (D2H + file write with
the GPU idle at every flush) for comparison.

  python tools/probes/stream_probe.py [n_samples] [dir]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import ip_mcmc_amd.sampler as S  # noqa: E402
from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution,  # noqa: E402
                         Lorenz96Operator, MCMCSampler, pCNAccepter)


class SyncWriter:
    """The writer before double buffering: synchronous .double().cpu() per flush."""

    def __init__(self, sink, shape, dtype, device, n_buf, single):
        self.sink, self.single = sink, single
        self.buffer = torch.empty(shape, dtype=dtype, device=device)

    def flush(self, i0, nb):
        blk = self.buffer[:, :nb, :].double().cpu().numpy()
        self.sink.write(i0, blk[0] if self.single else blk)
        return self.buffer

    def finish(self):
        pass


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 36
    d = sys.argv[2] if len(sys.argv) > 2 else tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    G = Lorenz96Operator(40, 8.0, dt=0.005, n_steps=2000)
    y = G(np.zeros(40)) + 0.1 * np.random.default_rng(3).normal(size=40)
    pot = EvolutionPotential(G, y, GaussianDistribution(np.zeros(40), 0.01 * np.eye(40)))
    u0 = np.zeros((65536, 40))
    good = S._StreamingWriter
    res = {}
    for name in ("memory", "stream_double_buffered", "stream_sync", "memory"):
        S._StreamingWriter = SyncWriter if name == "stream_sync" else good
        s = MCMCSampler(ConstSteppCNProposer(0.2, GaussianDistribution(np.zeros(40), np.eye(40))), pCNAccepter(pot), 7)
        path = os.path.join(d, f"{name}.npy") if name.startswith("stream") else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = s.run(u0, n_samples=n, burn_in=1, sample_interval=10, sample_file=path)
        wall = time.perf_counter() - t0
        res[name] = (wall, out)
        print(json.dumps({"mode": name, "n_samples": n, "chains": 65536, "wall_s": wall,
                          "pcn_steps_per_s": 65536 * 10 * n / wall, "bytes": int(np.asarray(out).nbytes)}), flush=True)
        if path:
            assert np.array_equal(np.asarray(out), res["memory"][1])
            del out
            os.remove(path)
    S._StreamingWriter = good


if __name__ == "__main__":
    main()
