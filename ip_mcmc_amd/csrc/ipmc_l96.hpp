// Lorenz-96 forward map + pCN sweep kernels.
//
// G(u): forcing field F = theta0 + u (one forcing per slow variable of the
// single-scale Lorenz-96 of lorenz.py:73-88, J = 0), x(0) = x0, classical RK4
// with fixed dt for n_steps steps, G_k = time average of X_k over the n
// post-step states.  The state of one chain lives in VGPRs of a group of LPC
// lanes (M = D/LPC components per lane); the cyclic neighbours X_{k-2},
// X_{k-1}, X_{k+1} that cross a lane boundary come from the neighbour lanes by
// DPP (LPC 2/4) or ds_bpermute (LPC 8/16).  Nothing touches HBM inside the RK
// loop: the kernel is VALU-bound.
#pragma once

#include "ipmc_sweep_common.hpp"

namespace ipmc {

// dX/dt for the lane's M components.
//   FM:  out_k = fma(X_{k+1} - X_{k-2}, X_{k-1}, F_k - X_k)          3 VALU ops
//   REF: out_k = ((-X_k) - (X_{k-1} X_{k-2} - X_{k-1} X_{k+1})) + F_k  lorenz.py:77-81
template <typename T, int M, int LPC, bool FM>
__device__ __forceinline__ void l96_rhs(const T (&s)[M], const T (&F)[M], T (&o)[M], int lane) {
  static_assert(M >= 2, "Lorenz-96 needs at least 2 components per lane");
  const T sl1 = group_prev<LPC>(s[M - 1], lane);
  const T sl2 = group_prev<LPC>(s[M - 2], lane);
  const T sr1 = group_next<LPC>(s[0], lane);
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const T xm1 = (j >= 1) ? s[j - 1] : sl1;
    const T xm2 = (j >= 2) ? s[j - 2] : ((j == 1) ? sl1 : sl2);
    const T xp1 = (j < M - 1) ? s[j + 1] : sr1;
    if constexpr (FM) {
      o[j] = madd<true>(xp1 - xm2, xm1, F[j] - s[j]);
    } else {
      T t = -s[j];
      t = t - (xm1 * xm2 - xm1 * xp1);
      o[j] = t + F[j];
    }
  }
}

// Time-averaged RK4 trajectory: g[j] = (Σ_{n=1..N} x_n[j]) / N.
template <typename T, int M, int LPC, bool FM>
__device__ __forceinline__ void l96_forward(const T (&F)[M], const T* __restrict__ x0, T h, int nsteps, int lane,
                                            T (&g)[M]) {
  const T h2 = h * (T)0.5;
  const T h6 = h / (T)6;
  T x[M], ob[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    x[j] = x0[j];
    ob[j] = (T)0;
  }
  for (int n = 0; n < nsteps; ++n) {
    T k[M], acc[M], xs[M];
    l96_rhs<T, M, LPC, FM>(x, F, k, lane);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      acc[j] = k[j];
      xs[j] = madd<FM>(h2, k[j], x[j]);
    }
    l96_rhs<T, M, LPC, FM>(xs, F, k, lane);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      acc[j] = madd<FM>((T)2, k[j], acc[j]);
      xs[j] = madd<FM>(h2, k[j], x[j]);
    }
    l96_rhs<T, M, LPC, FM>(xs, F, k, lane);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      acc[j] = madd<FM>((T)2, k[j], acc[j]);
      xs[j] = madd<FM>(h, k[j], x[j]);
    }
    l96_rhs<T, M, LPC, FM>(xs, F, k, lane);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      acc[j] = acc[j] + k[j];
      x[j] = madd<FM>(h6, acc[j], x[j]);
      ob[j] = ob[j] + x[j];
    }
  }
  const T nn = (T)nsteps;
#pragma unroll
  for (int j = 0; j < M; ++j) g[j] = ob[j] / nn;
}

template <typename T, int M, int LPC, bool FM>
__device__ __forceinline__ T l96_potential(const T (&v)[M], const T* __restrict__ th0, const T* __restrict__ x0,
                                           const T* __restrict__ y, const T* __restrict__ ginv, T h, int nsteps,
                                           int lane) {
  T F[M], g[M];
#pragma unroll
  for (int j = 0; j < M; ++j) F[j] = th0[j] + v[j];
  l96_forward<T, M, LPC, FM>(F, x0, h, nsteps, lane, g);
  T r[M];
#pragma unroll
  for (int j = 0; j < M; ++j) r[j] = (y[j] - g[j]) * ginv[j];
  return (T)0.5 * ordered_sumsq<T, M, LPC, FM>(r, lane, (T)0);
}

constexpr int kL96Block = 256;

// Occupancy target (waves per SIMD) the register allocator is held to: the
// state needs ~6 arrays of M values live in the RK loop (x, F, time-average,
// k-sum, stage, rhs), plus ~40 registers of addressing / RNG / loop state.
template <typename T, int M>
constexpr int l96_waves_per_simd() {
  constexpr int regs = 6 * M * (int)(sizeof(T) / 4) + 40;
  constexpr int w = 512 / regs;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// n_steps pCN steps per launch; u / Φ(u) / accept counts updated in place.
template <typename T, int D, int LPC, bool FM>
__global__ __launch_bounds__(kL96Block, (l96_waves_per_simd<T, D / LPC>())) void l96_sweep_kernel(const ipmc_model m, const ipmc_sweep s) {
  constexpr int M = D / LPC;
  __shared__ T vpark[M][kL96Block];  // proposal parked in LDS while G runs
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * kL96Block + threadIdx.x;
  const int64_t chain = tid / LPC;
  const int sub = (int)(tid % LPC);
  if (chain >= s.n_chains) return;  // whole lane groups leave together
  const uint64_t gid = (uint64_t)(s.chain_offset + chain);
  const int c0 = sub * M;
  T* __restrict__ u = (T*)s.u + chain * D + c0;
  const T beta = (T)s.beta, contr = (T)s.contraction, h = (T)m.dt;
  T* phi = (T*)s.phi;
  T phu = phi[chain];
  int64_t nacc = 0, ncalls = 0;
  for (int64_t st = 0; st < s.n_steps; ++st) {
    const uint64_t step = s.step0 + (uint64_t)st;
    // Opaque per-step offset: keeps the loop-invariant per-component constants
    // (theta0, x0, y, 1/gamma, sqrt C) from being hoisted into 5*M VGPRs for
    // the whole launch; they are re-read from L1/L2 once per pCN step instead.
    int cl = c0;
    asm volatile("" : "+v"(cl));
    const T bs = s.beta_schedule ? (T)s.beta_schedule[2 * st] : beta;
    const T cs = s.beta_schedule ? (T)s.beta_schedule[2 * st + 1] : contr;
    T v[M];
    pcn_propose<T, M>(u, (const T*)s.prior_sqrt + cl, cs, bs, s.seed, gid, step, c0, v);
    if (box_valid<T, M, LPC>(s, c0, v, lane)) {
      ++ncalls;
#pragma unroll
      for (int j = 0; j < M; ++j) vpark[j][threadIdx.x] = v[j];
      const T phv = l96_potential<T, M, LPC, FM>(v, (const T*)m.theta0 + cl, (const T*)m.x0 + cl,
                                                 (const T*)s.y + cl, (const T*)s.gamma_inv + cl, h, m.n_steps, lane);
      // memory clobber: re-read v from LDS instead of keeping it live in VGPRs across G
      asm volatile("" ::: "memory");
      if (pcn_accept<T>(phu, phv, s.seed, gid, step)) {
#pragma unroll
        for (int j = 0; j < M; ++j) u[j] = vpark[j][threadIdx.x];
        phu = phv;
        ++nacc;
      }
    }
    if (s.sum_u) {
      double* su = s.sum_u + chain * D + c0;
      double* su2 = s.sum_u2 ? s.sum_u2 + chain * D + c0 : nullptr;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const double ud = (double)u[j];
        su[j] += ud;
        if (su2) su2[j] += ud * ud;
      }
    }
  }
  if (sub == 0) {
    phi[chain] = phu;
    if (s.accepts) s.accepts[chain] += nacc;
    if (s.calls) s.calls[chain] += ncalls;
  }
  if (s.sample_out) {
    T* so = (T*)s.sample_out + chain * s.sample_stride + c0;
#pragma unroll
    for (int j = 0; j < M; ++j) so[j] = u[j];
  }
}

// G(u) or Φ(u) for n parameter vectors (no proposal): out = g [n, D] or phi [n].
template <typename T, int D, int LPC, bool FM, bool PHI>
__global__ __launch_bounds__(kL96Block, (l96_waves_per_simd<T, D / LPC>())) void l96_eval_kernel(const ipmc_model m, int64_t n, const T* __restrict__ uin,
                                                              const T* __restrict__ yin,
                                                              const T* __restrict__ ginvin, T* __restrict__ out) {
  constexpr int M = D / LPC;
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * kL96Block + threadIdx.x;
  const int64_t chain = tid / LPC;
  const int sub = (int)(tid % LPC);
  if (chain >= n) return;
  const int c0 = sub * M;
  const T* u = uin + chain * D + c0;
  const T* th0 = (const T*)m.theta0 + c0;
  const T* x0 = (const T*)m.x0 + c0;
  const T h = (T)m.dt;
  T v[M];
#pragma unroll
  for (int j = 0; j < M; ++j) v[j] = u[j];
  if constexpr (PHI) {
    const T ph = l96_potential<T, M, LPC, FM>(v, th0, x0, yin + c0, ginvin + c0, h, m.n_steps, lane);
    if (sub == 0) out[chain] = ph;
  } else {
    T F[M], g[M];
#pragma unroll
    for (int j = 0; j < M; ++j) F[j] = th0[j] + v[j];
    l96_forward<T, M, LPC, FM>(F, x0, h, m.n_steps, lane, g);
#pragma unroll
    for (int j = 0; j < M; ++j) out[chain * D + c0 + j] = g[j];
  }
}

}  // namespace ipmc
