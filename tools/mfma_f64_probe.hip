// f64 MFMA probe for MI355X (gfx950): can the matrix pipe take work off the
// FP64 VALU in the Lorenz-96 sweep?  Prints
//  1. the lane maps of v_mfma_f64_4x4x4_4b_f64 and v_mfma_f64_16x16x4_f64:
//     for a one-hot A (lane p = 1, every other lane 0) and B[lane] = lane,
//     which D lanes/registers receive which B lane;
//  2. the issue rate of each (cycles per MFMA per SIMD, 1/2/4 waves per SIMD);
//  3. overlap: a loop of independent v_fma_f64 alone, MFMA alone, and both
//     interleaved in the same wave (time of the mix vs the sum and the max).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_probe.hip -o build/mfma_f64_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void map_4x4(int p, double* out) {
  const int l = threadIdx.x;
  const double a = (l == p) ? 1.0 : 0.0;
  const double b = 1000.0 + l;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

__global__ void map_16x16(int p, double* out) {
  const int l = threadIdx.x;
  const double a = (l == p) ? 1.0 : 0.0;
  const double b = 1000.0 + l;
  d4 c = {0, 0, 0, 0};
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[4 * l + r] = d[r];
}

// MODE 0: 8 independent v_fma_f64 chains; 1: 4x4x4 MFMA (8 independent
// accumulators); 2: 16x16x4 MFMA (4 independent accumulators); 3: MODE 0 +
// MODE 1 interleaved (one MFMA per VFMA_PER_MFMA FMAs); 4: MODE 0 + MODE 2.
template <int MODE, int VFMA_PER_MFMA>
__global__ __launch_bounds__(256) void rate(double* out, int iters) {
  const double t = threadIdx.x * 1e-7;
  double a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
  double m0 = t, m1 = t, m2 = t, m3 = t, m4 = t, m5 = t, m6 = t, m7 = t;
  d4 q0 = {t, t, t, t}, q1 = q0, q2 = q0, q3 = q0;
  const double b = 0.999, c = 1e-3;
  const double av = (threadIdx.x & 3) == 0 ? 1.0 : 0.0;
  for (int i = 0; i < iters; ++i) {
#define F(a) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
#define M(m) m = __builtin_amdgcn_mfma_f64_4x4x4f64(av, c, m, 0, 0, 0)
#define Q(q) q = __builtin_amdgcn_mfma_f64_16x16x4f64(av, c, q, 0, 0, 0)
    if constexpr (MODE == 0) {
      F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
    } else if constexpr (MODE == 1) {
      M(m0); M(m1); M(m2); M(m3); M(m4); M(m5); M(m6); M(m7);
    } else if constexpr (MODE == 2) {
      Q(q0); Q(q1); Q(q2); Q(q3);
    } else if constexpr (MODE == 3) {
      // 8 MFMAs and 8 * VFMA_PER_MFMA FMAs per iteration
#pragma unroll
      for (int r = 0; r < VFMA_PER_MFMA; ++r) {
        F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
        if (r == 0) { M(m0); M(m1); M(m2); M(m3); }
        if (r == VFMA_PER_MFMA / 2) { M(m4); M(m5); M(m6); M(m7); }
      }
    } else {
#pragma unroll
      for (int r = 0; r < VFMA_PER_MFMA; ++r) {
        F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
        if (r == 0) { Q(q0); Q(q1); }
        if (r == VFMA_PER_MFMA / 2) { Q(q2); Q(q3); }
      }
    }
#undef F
#undef M
#undef Q
  }
  d4 qs = q0 + q1 + q2 + q3;
  out[blockIdx.x * 256 + threadIdx.x] =
      a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + m0 + m1 + m2 + m3 + m4 + m5 + m6 + m7 + qs[0] + qs[1] + qs[2] + qs[3];
}

template <int MODE, int V>
static float time_ms(int waves, double* buf, int iters) {
  const int blocks = 256 * waves;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((rate<MODE, V>), dim3(blocks), dim3(256), 0, 0, buf, iters);  // warm
  hipEventRecord(a, 0);
  hipLaunchKernelGGL((rate<MODE, V>), dim3(blocks), dim3(256), 0, 0, buf, iters);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  double* d;
  double h[256];
  hipMalloc(&d, 256 * 4 * 256 * 8 * sizeof(double));
  printf("# v_mfma_f64_4x4x4_4b_f64: one-hot A at lane p, B[lane] = 1000 + lane -> D lanes that got B\n");
  for (int p = 0; p < 64; ++p) {
    hipLaunchKernelGGL(map_4x4, dim3(1), dim3(64), 0, 0, p, d);
    hipMemcpy(h, d, 64 * sizeof(double), hipMemcpyDeviceToHost);
    printf("A lane %2d:", p);
    for (int l = 0; l < 64; ++l)
      if (h[l] != 0.0) printf(" D[%d]=B[%d]", l, (int)(h[l] - 1000.0 + 0.5));
    printf("\n");
  }
  printf("# v_mfma_f64_16x16x4_f64: D lane.reg that got B\n");
  for (int p = 0; p < 64; ++p) {
    hipLaunchKernelGGL(map_16x16, dim3(1), dim3(64), 0, 0, p, d);
    hipMemcpy(h, d, 256 * sizeof(double), hipMemcpyDeviceToHost);
    printf("A lane %2d:", p);
    int shown = 0;
    for (int i = 0; i < 256; ++i)
      if (h[i] != 0.0 && shown < 6) {
        printf(" D[%d.%d]=B[%d]", i / 4, i % 4, (int)(h[i] - 1000.0 + 0.5));
        ++shown;
      }
    printf("\n");
  }
  const int iters = 4096;
  const double clk = 2.1e9;  // nominal, only for a rough cycles figure
  for (int w = 1; w <= 4; w *= 2) {
    const float f = time_ms<0, 1>(w, d, iters);
    const float m4 = time_ms<1, 1>(w, d, iters);
    const float m16 = time_ms<2, 1>(w, d, iters);
    // per SIMD: w waves each issue iters*8 FMAs / iters*8 4x4 MFMAs / iters*4 16x16 MFMAs
    printf("waves/SIMD %d: vfma64 %.3f ms (%.2f cyc/instr/SIMD @2.1GHz)  mfma4x4 %.3f ms (%.2f)  mfma16x16 %.3f ms "
           "(%.2f)\n",
           w, f, f * 1e-3 * clk / (iters * 8.0 * w), m4, m4 * 1e-3 * clk / (iters * 8.0 * w), m16,
           m16 * 1e-3 * clk / (iters * 4.0 * w));
    const float x2 = time_ms<3, 2>(w, d, iters), x4 = time_ms<3, 4>(w, d, iters), x8 = time_ms<3, 8>(w, d, iters);
    const float f2 = time_ms<0, 1>(w, d, 2 * iters), f4 = time_ms<0, 1>(w, d, 4 * iters),
                f8 = time_ms<0, 1>(w, d, 8 * iters);
    printf("  mix 4x4: 1 MFMA per 2/4/8 FMAs: %.3f / %.3f / %.3f ms; FMAs alone %.3f / %.3f / %.3f ms; MFMAs alone "
           "%.3f\n",
           x2, x4, x8, f2, f4, f8, m4);
    const float y2 = time_ms<4, 2>(w, d, iters), y4 = time_ms<4, 4>(w, d, iters), y8 = time_ms<4, 8>(w, d, iters);
    printf("  mix 16x16: 1 MFMA per 4/8/16 FMAs: %.3f / %.3f / %.3f ms; MFMAs alone %.3f\n", y2, y4, y8, m16);
  }
  hipFree(d);
  return 0;
}
