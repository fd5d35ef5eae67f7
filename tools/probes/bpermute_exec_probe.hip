// What a cross-lane read (__shfl = ds_bpermute_b32) returns when its source
// lane is inactive (EXEC off) on gfx950: the root-cause probe for the wrong
// recorded sums of round 4's speculative walk (tools/probes/walk_shfl_probe.py,
// DESIGN.md §5).  One wave; lane i holds 100 + i.
//   A: all lanes active, lane i reads lane i ^ 1            -> 100 + (i ^ 1)
//   B: only even lanes active, lane i reads lane i + 1 (odd, inactive)
//   C: only even lanes active, lane i reads lane i (itself, active)
//   D: lanes < 32 active, lane i reads lane i + 32 (inactive)
//   E: a loop whose trip count is (lane / 16) + 1: in iteration t only the
//      lanes with lane / 16 >= t remain; each reads lane (lane + 16) % 64
//  hipcc --offload-arch=gfx950 -O2 tools/probes/bpermute_exec_probe.hip -o /tmp/bp && /tmp/bp
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(int* out) {
  const int i = threadIdx.x;
  const int val = 100 + i;
  int a = __shfl(val, i ^ 1, 64);
  int b = -1, c = -1, d = -1;
  if ((i & 1) == 0) {
    b = __shfl(val, i + 1, 64);
    c = __shfl(val, i, 64);
  }
  if (i < 32) d = __shfl(val, i + 32, 64);
  int e = 0;
  const int trips = i / 16 + 1;
  for (int t = 0; t < trips; ++t) e = e * 1000 + __shfl(val, (i + 16) % 64, 64);
  out[0 * 64 + i] = a;
  out[1 * 64 + i] = b;
  out[2 * 64 + i] = c;
  out[3 * 64 + i] = d;
  out[4 * 64 + i] = e;
}

int main() {
  int* d = nullptr;
  int h[5 * 64];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  hipFree(d);
  const char* name[5] = {"A all active, read i^1", "B even active, read odd i+1", "C even active, read self",
                         "D i<32 active, read i+32", "E divergent loop, read (i+16)%64"};
  for (int k = 0; k < 5; ++k) {
    std::printf("%s:", name[k]);
    for (int i = 0; i < 64; i += (k == 4 ? 1 : 8)) std::printf(" %d", h[k * 64 + i]);
    std::printf("\n");
  }
  return 0;
}
