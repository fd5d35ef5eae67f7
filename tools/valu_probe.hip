// VALU throughput probe for MI355X: v_fma_f32, v_pk_fma_f32, v_fma_f64 at
// 1/2/4/8 waves per SIMD (256-thread blocks, 256*W blocks).  Prints TFLOP/s.
// Used to pin the roofline peak of the VALU-bound pCN sweep.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o build/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
  const float t = threadIdx.x * 1e-7f;
  if constexpr (MODE == 0) {
    float a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
    float b = 0.999f, c = 1e-3f;
    for (int i = 0; i < iters; ++i) {
#define F(a) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
      F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
#undef F
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  } else if constexpr (MODE == 1) {
    f2 a0 = {t, t}, a1 = {t + 1, t}, a2 = {t + 2, t}, a3 = {t + 3, t}, a4 = {t + 4, t}, a5 = {t + 5, t},
       a6 = {t + 6, t}, a7 = {t + 7, t};
    f2 b = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
    for (int i = 0; i < iters; ++i) {
#define F(a) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
      F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
#undef F
    }
    f2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
  } else {
    double a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
    double b = 0.999, c = 1e-3;
    for (int i = 0; i < iters; ++i) {
#define F(a) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
      F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
#undef F
    }
    out[blockIdx.x * 256 + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
  }
}

template <int MODE>
static double run(int waves, float* buf, int iters) {
  const int blocks = 256 * waves;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, buf, iters);  // warm
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, buf, iters);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double flop = (double)blocks * 256 * iters * 8 * 2 * (MODE == 1 ? 2 : 1);
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  float* buf;
  hipMalloc(&buf, 256 * 256 * 16 * sizeof(float));
  const int iters = 1 << 16;
  const char* names[3] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_f64"};
  for (int w : {1, 2, 4, 8}) {
    printf("waves/SIMD=%d  %s %.1f TF  %s %.1f TF  %s %.1f TF\n", w, names[0], run<0>(w, buf, iters), names[1],
           run<1>(w, buf, iters), names[2], run<2>(w, buf, iters));
  }
  hipFree(buf);
  return 0;
}
