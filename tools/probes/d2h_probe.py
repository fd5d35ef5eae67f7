"""D2H cost of a (65536, 20, 40) f64 sample array (the sampler_e2e output):
pageable .cpu() vs a pinned host buffer, and chunked async copies on a side stream."""
import time

import torch

dev = torch.device("cuda", 0)
x = torch.randn((65536, 20, 40), dtype=torch.float64, device=dev)
torch.cuda.synchronize()
for _ in range(2):
    t = time.perf_counter(); y = x.cpu(); dt = time.perf_counter() - t
print(f"pageable .cpu(): {dt*1e3:.1f} ms ({x.numel()*8/dt/1e9:.1f} GB/s)")
t = time.perf_counter(); h = torch.empty(x.shape, dtype=x.dtype, pin_memory=True); ta = time.perf_counter() - t
for _ in range(2):
    t = time.perf_counter(); h.copy_(x); torch.cuda.synchronize(); dt = time.perf_counter() - t
print(f"pinned alloc {ta*1e3:.1f} ms; pinned copy: {dt*1e3:.1f} ms ({x.numel()*8/dt/1e9:.1f} GB/s)")
t = time.perf_counter(); n = h.numpy().copy(); dt = time.perf_counter() - t
print(f"host copy out of the pinned buffer: {dt*1e3:.1f} ms")
s = torch.cuda.Stream()
blk = torch.empty((65536, 40), dtype=torch.float64, pin_memory=True)
t = time.perf_counter()
for i in range(20):
    with torch.cuda.stream(s):
        blk.copy_(x[:, i, :], non_blocking=True)
    s.synchronize()
dt = time.perf_counter() - t
print(f"20 strided per-sample blocks into one pinned block: {dt*1e3:.1f} ms")
