// Small-state forward maps, one chain per lane (LPC = 1):
//   LINEAR    G(u) = A (theta0 + u)                    stuart_examples.py:69-70
//   LORENZ63  RK4 Lorenz-63, theta = (sigma, rho, b) = theta0 + u, observations the
//             time averages of (x, y, z, x^2, y^2, z^2) (lorenz_mcmc.py:17-40 pattern)
#pragma once

#include "ipmc_sweep_common.hpp"

namespace ipmc {

constexpr int kSmallBlock = 64;
constexpr int kSmallKMax = 64;  // linear: k <= 64 (proposal parked in LDS)

template <typename T, bool FM>
__device__ __forceinline__ void l63_rhs(T sg, T rh, T bb, const T (&s)[3], T (&o)[3]) {
  if constexpr (FM) {
    o[0] = sg * (s[1] - s[0]);
    o[1] = madd<true>(s[0], rh - s[2], -s[1]);
    o[2] = madd<true>(s[0], s[1], -(bb * s[2]));
  } else {
    o[0] = sg * (s[1] - s[0]);
    o[1] = s[0] * (rh - s[2]) - s[1];
    o[2] = s[0] * s[1] - bb * s[2];
  }
}

// RK4 steps per loop iteration (default 8).  Config 2 runs one wave per SIMD,
// where a round is one forward map at a single wave's issue rate: unrolled
// steps let the scheduler overlap one step's moment updates and k-sum with the
// next step's right-hand side (same operations, same bits): config 2 453 ->
// 498 M steps/s in f64, 549 -> 615 M in fp32 by 8 against the compiler's own
// choice (by 4: 497 / 604 M; profiles/r4/l63_unroll_ab2.jsonl,
// l63_unroll_ab3.jsonl).  0: the compiler's choice.
#ifndef IPMC_L63_UNROLL
#define IPMC_L63_UNROLL 8
#endif
#if IPMC_L63_UNROLL > 0
#define IPMC_STR_(x) #x
#define IPMC_L63_UNROLL_PRAGMA(n) _Pragma(IPMC_STR_(unroll n))
#define IPMC_L63_RK_UNROLL IPMC_L63_UNROLL_PRAGMA(IPMC_L63_UNROLL)
#else
#define IPMC_L63_RK_UNROLL
#endif

template <typename T, bool FM>
__device__ __forceinline__ void l63_forward(T sg, T rh, T bb, const T* __restrict__ x0, T h, int nsteps, T (&g)[6]) {
  const T h2 = h * (T)0.5, h6 = h / (T)6;
  T x[3] = {x0[0], x0[1], x0[2]};
  T ob[6] = {0, 0, 0, 0, 0, 0};
  IPMC_L63_RK_UNROLL
  for (int n = 0; n < nsteps; ++n) {
    T k1[3], k2[3], k3[3], k4[3], xs[3];
    l63_rhs<T, FM>(sg, rh, bb, x, k1);
#pragma unroll
    for (int i = 0; i < 3; ++i) xs[i] = madd<FM>(h2, k1[i], x[i]);
    l63_rhs<T, FM>(sg, rh, bb, xs, k2);
#pragma unroll
    for (int i = 0; i < 3; ++i) xs[i] = madd<FM>(h2, k2[i], x[i]);
    l63_rhs<T, FM>(sg, rh, bb, xs, k3);
#pragma unroll
    for (int i = 0; i < 3; ++i) xs[i] = madd<FM>(h, k3[i], x[i]);
    l63_rhs<T, FM>(sg, rh, bb, xs, k4);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      // ((k1 + 2 k2) + 2 k3) + k4: 2k is exact, so FMA arith fuses the
      // doublings (3 VALU ops instead of 5, the same bits as the oracle's form)
      const T a = FM ? madd<true>((T)2, k3[i], madd<true>((T)2, k2[i], k1[i])) + k4[i]
                     : ((k1[i] + (T)2 * k2[i]) + (T)2 * k3[i]) + k4[i];
      x[i] = madd<FM>(h6, a, x[i]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ob[i] = ob[i] + x[i];
      ob[3 + i] = madd<FM>(x[i], x[i], ob[3 + i]);
    }
  }
  const T nn = (T)nsteps;
#pragma unroll
  for (int i = 0; i < 6; ++i) g[i] = ob[i] / nn;
}

#ifndef IPMC_L63_PK  // experiments (tools/build_variant.sh): 0 = the scalar fp32 loop
#define IPMC_L63_PK 1
#endif

// fp32: the same RK4 with components (x, y) held as one f32x2 pair P and z
// scalar.  Everything elementwise over the components -- the stage inputs,
// the k-sum, the update and the moments -- is one v_pk_*_f32 for x and y
// (per-element IEEE operations, so the bits of l63_forward<float>); only the
// right-hand side, whose three rates have different formulas, stays scalar.
// 51 -> 42 VALU ops per RK4 step: config 2 runs one wave per SIMD (4 096
// chains x 16 speculative slots), where a single wave's issue rate, not its
// dependent chain, bounds a round, so fewer instructions are
// a shorter round.
template <bool FM>
__device__ __forceinline__ void l63_rhs_pk(float sg, float rh, float bb, f32x2 p, float z, f32x2& kp, float& kz) {
  const float s[3] = {p.x, p.y, z};
  float o[3];
  l63_rhs<float, FM>(sg, rh, bb, s, o);
  kp = f32x2{o[0], o[1]};
  kz = o[2];
}

template <bool FM>
__device__ __forceinline__ void l63_forward_pk(float sg, float rh, float bb, const float* __restrict__ x0, float h,
                                               int nsteps, float (&g)[6]) {
  const float h2 = h * 0.5f, h6 = h / 6.0f;
  const f32x2 H2 = {h2, h2}, H = {h, h}, H6 = {h6, h6}, TWO = {2.0f, 2.0f};
  f32x2 P = {x0[0], x0[1]};
  float z = x0[2];
  f32x2 obP = {0.0f, 0.0f}, ob2P = {0.0f, 0.0f};
  float obz = 0.0f, ob2z = 0.0f;
  IPMC_L63_RK_UNROLL
  for (int n = 0; n < nsteps; ++n) {
    f32x2 k1, k2, k3, k4, xs;
    float k1z, k2z, k3z, k4z, xsz;
    l63_rhs_pk<FM>(sg, rh, bb, P, z, k1, k1z);
    xs = madd<FM>(H2, k1, P);
    xsz = madd<FM>(h2, k1z, z);
    l63_rhs_pk<FM>(sg, rh, bb, xs, xsz, k2, k2z);
    xs = madd<FM>(H2, k2, P);
    xsz = madd<FM>(h2, k2z, z);
    l63_rhs_pk<FM>(sg, rh, bb, xs, xsz, k3, k3z);
    xs = madd<FM>(H, k3, P);
    xsz = madd<FM>(h, k3z, z);
    l63_rhs_pk<FM>(sg, rh, bb, xs, xsz, k4, k4z);
    // l63_forward's ((k1 + 2 k2) + 2 k3) + k4 in the same per-element operations
    const f32x2 a = FM ? madd<true>(TWO, k3, madd<true>(TWO, k2, k1)) + k4 : ((k1 + TWO * k2) + TWO * k3) + k4;
    const float az = FM ? madd<true>(2.0f, k3z, madd<true>(2.0f, k2z, k1z)) + k4z
                        : ((k1z + 2.0f * k2z) + 2.0f * k3z) + k4z;
    P = madd<FM>(H6, a, P);
    z = madd<FM>(h6, az, z);
    obP = obP + P;
    obz = obz + z;
    ob2P = madd<FM>(P, P, ob2P);
    ob2z = madd<FM>(z, z, ob2z);
  }
  const float nn = (float)nsteps;
  g[0] = obP.x / nn;
  g[1] = obP.y / nn;
  g[2] = obz / nn;
  g[3] = ob2P.x / nn;
  g[4] = ob2P.y / nn;
  g[5] = ob2z / nn;
}

// The forward map of small_potential / small_eval_kernel: packed components for fp32.
template <typename T, bool FM>
__device__ __forceinline__ void l63_G(T sg, T rh, T bb, const T* __restrict__ x0, T h, int nsteps, T (&g)[6]) {
  if constexpr (sizeof(T) == 4 && IPMC_L63_PK) l63_forward_pk<FM>(sg, rh, bb, x0, h, nsteps, g);
  else l63_forward<T, FM>(sg, rh, bb, x0, h, nsteps, g);
}

// Φ for the lane's chain; v is read from the LDS park (column `col`).
template <typename T, int MODEL, bool FM>
__device__ __forceinline__ T small_potential(const ipmc_model& m, const T* __restrict__ v, int vstride,
                                             const T* __restrict__ y, const T* __restrict__ ginv) {
  const T* th0 = (const T*)m.theta0;
  T s = (T)0;
  if constexpr (MODEL == IPMC_MODEL_LORENZ63) {
    T g[6];
    l63_G<T, FM>(th0[0] + v[0], th0[1] + v[vstride], th0[2] + v[2 * vstride], (const T*)m.x0, (T)m.dt, m.n_steps,
                 g);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const T r = (y[i] - g[i]) * ginv[i];
      s = madd<FM>(r, r, s);
    }
  } else {
    const T* A = (const T*)m.A;
    const int k = m.k;
    for (int i = 0; i < m.q; ++i) {
      T acc = (T)0;
      for (int j = 0; j < k; ++j) acc = madd<FM>(A[(int64_t)i * k + j], th0[j] + v[j * vstride], acc);
      const T r = (y[i] - acc) * ginv[i];
      s = madd<FM>(r, r, s);
    }
  }
  return (T)0.5 * s;
}

// ½ Σ_j (c_j v_j)², v strided (StandardRWAccepter regularizer, accepter.py:104-106)
template <typename T, bool FM>
__device__ __forceinline__ T small_regularizer(int k, const T* __restrict__ c, const T* __restrict__ v, int vstride) {
  T s = (T)0;
  for (int j = 0; j < k; ++j) {
    const T t = c[j] * v[j * vstride];
    s = madd<FM>(t, t, s);
  }
  return (T)0.5 * s;
}

template <typename T, int MODEL, bool FM>
__global__ __launch_bounds__(kSmallBlock) void small_sweep_kernel(const ipmc_model m, const ipmc_sweep s) {
  __shared__ T vpark[kSmallKMax * kSmallBlock];
  const int64_t chain = (int64_t)blockIdx.x * kSmallBlock + threadIdx.x;
  if (chain >= s.n_chains) return;
  const int k = m.k;
  const uint64_t gid = (uint64_t)(s.chain_offset + chain);
  T* __restrict__ u = (T*)s.u + chain * k;
  const T* sq = (const T*)s.prior_sqrt;
  const T* chol = (const T*)s.prior_chol;
  const T* lo = (const T*)s.box_lo;
  const T* hi = (const T*)s.box_hi;
  const T* off = (const T*)s.box_off;
  const T beta = (T)s.beta, contr = (T)s.contraction;
  T* phi = (T*)s.phi;
  T* v = vpark + threadIdx.x;  // v[j * kSmallBlock]
  T phu = phi[chain];
  const bool rw = (s.proposal == IPMC_PROPOSAL_RW);
  int64_t nacc = 0, ncalls = 0;
  for (int64_t st = 0; st < s.n_steps; ++st) {
    const uint64_t step = s.step0 + (uint64_t)st;
    const T bs = s.beta_schedule ? (T)s.beta_schedule[2 * st] : beta;
    const T cs = s.beta_schedule ? (T)s.beta_schedule[2 * st + 1] : contr;
    double z0 = 0.0, z1 = 0.0;
    bool ok = true;
    if (chol) {
      // non-diagonal prior (chol_noise's order): ξ parked first, then
      // w_j = Σ_{i<=j} L[j][i] ξ_i for descending j, each v_j replacing ξ_j
      for (int j = 0; j < k; j += 2) {
        normal_pair(s.seed, gid, step, (uint32_t)(j >> 1), z0, z1);
        v[j * kSmallBlock] = (T)z0;
        if (j + 1 < k) v[(j + 1) * kSmallBlock] = (T)z1;
      }
      for (int j = k - 1; j >= 0; --j) {
        T w = (T)0;
        for (int i = 0; i <= j; ++i) w = w + v[i * kSmallBlock] * chol[(int64_t)j * k + i];
        const T vj = propose_one<T>(rw, u[j], w, cs, bs);
        v[j * kSmallBlock] = vj;
        const T t = vj + (off ? off[j] : (T)0);
        if (lo && !(lo[j] < t)) ok = false;
        if (hi && !(t < hi[j])) ok = false;
      }
    } else {
      for (int j = 0; j < k; ++j) {
        if ((j & 1) == 0) normal_pair(s.seed, gid, step, (uint32_t)(j >> 1), z0, z1);
        const T w = sq[j] * (T)((j & 1) ? z1 : z0);
        const T vj = propose_one<T>(rw, u[j], w, cs, bs);
        v[j * kSmallBlock] = vj;
        const T t = vj + (off ? off[j] : (T)0);
        if (lo && !(lo[j] < t)) ok = false;
        if (hi && !(t < hi[j])) ok = false;
      }
    }
    if (ok) {
      ++ncalls;
      T phv = small_potential<T, MODEL, FM>(m, v, kSmallBlock, (const T*)s.y, (const T*)s.gamma_inv);
      if (s.reg_scale) phv = phv + small_regularizer<T, FM>(k, (const T*)s.reg_scale, v, kSmallBlock);
      if (pcn_accept<T>(phu, phv, s.seed, gid, step)) {
        for (int j = 0; j < k; ++j) u[j] = v[j * kSmallBlock];
        phu = phv;
        ++nacc;
      }
    }
    if (s.sum_u) {
      for (int j = 0; j < k; ++j) {
        const double ud = (double)u[j];
        s.sum_u[chain * k + j] += ud;
        if (s.sum_u2) s.sum_u2[chain * k + j] += ud * ud;
      }
    }
    const int64_t sl = sample_slot(s, st);
    if (sl >= 0) {
      T* so = (T*)s.sample_out + chain * s.sample_stride + sl * s.sample_step_stride;
      for (int j = 0; j < k; ++j) so[j] = u[j];
    }
  }
  phi[chain] = phu;
  if (s.accepts) s.accepts[chain] += nacc;
  if (s.calls) s.calls[chain] += ncalls;
  if (s.sample_out && s.sample_every == 0) {
    T* so = (T*)s.sample_out + chain * s.sample_stride;
    for (int j = 0; j < k; ++j) so[j] = u[j];
  }
}

// ------------------------------------------------------------ speculation
// Small ensembles leave most of the GPU idle and a chain's steps are a
// latency-bound sequence.  With S lanes per chain, lane s is node s of a
// speculation tree (ipmc_spec_tree.hpp): it evaluates step st + depth(s) from
// the proposal of its origin node (or the current state) with the
// counter-based draws of that step, so it is exactly the proposal the
// sequential chain makes if the decisions before it go the node's way.  The
// chain walks the tree along the real decisions (the nodes off its path are
// discarded and redone), so u, Φ, the counters, the sums and the samples are
// bit-identical to the one-lane kernel; a round advances the chain by up to S
// steps in about one forward-map latency.
// gfx950 only: the f64 linear kernel's LDS (small_spec_lds_bytes) is 96 KiB at
// the default 256 threads, static_assert'ed against kLdsBytesPerCU.
#ifndef IPMC_SPEC_BLOCK  // block-size experiments (tools/build_variant.sh)
#define IPMC_SPEC_BLOCK 256
#endif
constexpr int kSpecBlock = IPMC_SPEC_BLOCK;
#ifndef IPMC_SPEC_K3  // 0: Lorenz-63 with the generic k <= 8 registers (A/B)
#define IPMC_SPEC_K3 1
#endif
constexpr int kSpecKMax = 8;
// linear G: A [q, k], y [q] and 1/γ [q] staged in LDS when q (k + 2) fits
constexpr int kSpecLinLds = 1024;

// Linear Φ with A, y, 1/γ from LDS and θ0 from registers: the operations and
// order of small_potential<LINEAR> (same bits), without a global-memory round
// trip per element in every speculative round.
template <typename T, bool FM>
__device__ __forceinline__ T lin_potential_staged(const T* As, const T* ys, const T* gs, const T (&th0)[kSpecKMax],
                                                  int q, int k, const T* v, int vstride) {
  T s = (T)0;
  for (int i = 0; i < q; ++i) {
    T acc = (T)0;
#pragma unroll
    for (int j = 0; j < kSpecKMax; ++j)
      if (j < k) acc = madd<FM>(As[i * k + j], th0[j] + v[j * vstride], acc);
    const T r = (ys[i] - acc) * gs[i];
    s = madd<FM>(r, r, s);
  }
  return (T)0.5 * s;
}

// Linear G: a round is a few FMAs of Φ, so its latency is the Philox /
// Box–Muller draws of the slots' steps.  The draws do not depend on the chain
// state, so the linear sweep computes them ahead, kPreFactor*S steps at a time
// spread over the group's lanes (w = sqrt(C)·ξ or L·ξ, and log r, in the
// sequential kernel's operations), into LDS; a round then reads them and only
// forms v, Φ(v) and the comparison -- the same bits, a much shorter round.
constexpr int kPreFactor = 4;
constexpr int kPreLds = kPreFactor * kSpecBlock;  // steps per block (all groups)

// LDS of one small_spec_kernel block: the proposal park, the linear model's
// constants and (linear) the pre-drawn w / log r.  f64 at kSpecBlock = 256 is
// 96 KiB -- it fits gfx950's 160 KiB per CU only (64 KiB on gfx942): a larger
// IPMC_SPEC_BLOCK or kPreFactor has to stay under the limit.
template <typename T, int MODEL>
constexpr size_t small_spec_lds_bytes() {
  return sizeof(T) * (size_t)kSpecKMax * kSpecBlock + sizeof(T) * (MODEL == IPMC_MODEL_LINEAR ? kSpecLinLds : 1) +
         (MODEL == IPMC_MODEL_LINEAR ? (sizeof(T) * (size_t)kPreLds * kSpecKMax + sizeof(double) * kPreLds)
                                     : sizeof(T) + sizeof(double));
}

template <typename T, int MODEL, bool FM, int S>
__global__ __launch_bounds__(kSpecBlock) void small_spec_kernel(const ipmc_model m, const ipmc_sweep s) {
  static_assert(small_spec_lds_bytes<T, MODEL>() <= kLdsBytesPerCU,
                "small_spec_kernel: LDS per block exceeds the CU's LDS (gfx950: 160 KiB)");
  constexpr bool PRE = (MODEL == IPMC_MODEL_LINEAR);
  constexpr int C = kPreFactor * S;  // steps of draws a group holds
  __shared__ T vpark[kSpecKMax * kSpecBlock];
  __shared__ T lin_c[MODEL == IPMC_MODEL_LINEAR ? kSpecLinLds : 1];
  __shared__ T pre_w[PRE ? kPreLds * kSpecKMax : 1];    // [group][step in chunk][j]
  __shared__ double pre_lr[PRE ? kPreLds : 1];           // [group][step in chunk]: log r
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int sub = t & (S - 1);
  const int gbase = lane & ~(S - 1);
  const unsigned long long gmask = (S == 64) ? ~0ull : ((1ull << S) - 1);
  const int64_t chain = ((int64_t)blockIdx.x * kSpecBlock + t) / S;
  // Lorenz-63 has k = 3 (ipmc_validate_model): the per-chain registers and
  // the per-round loops are sized to it at compile time
  constexpr bool K3 = IPMC_SPEC_K3 && MODEL == IPMC_MODEL_LORENZ63;
  constexpr int KM = K3 ? 3 : kSpecKMax;
  const int k = K3 ? 3 : m.k;
  // per-problem constants, read once per launch instead of once per round
  bool staged = false;
  if constexpr (MODEL == IPMC_MODEL_LINEAR) {
    const int q = m.q, nA = m.q * k;
    staged = q * (k + 2) <= kSpecLinLds;
    if (staged) {
      for (int i = t; i < nA; i += kSpecBlock) lin_c[i] = ((const T*)m.A)[i];
      for (int i = t; i < q; i += kSpecBlock) {
        lin_c[nA + i] = ((const T*)s.y)[i];
        lin_c[nA + q + i] = ((const T*)s.gamma_inv)[i];
      }
    }
    __syncthreads();  // every thread of the block, before any leaves
  }
  if (chain >= s.n_chains) return;  // whole groups leave together
  const uint64_t gid = (uint64_t)(s.chain_offset + chain);
  T* __restrict__ u = (T*)s.u + chain * k;
  const T* sq = (const T*)s.prior_sqrt;
  const T* chol = (const T*)s.prior_chol;
  const T* lo = (const T*)s.box_lo;
  const T* hi = (const T*)s.box_hi;
  const T* off = (const T*)s.box_off;
  const T beta = (T)s.beta, contr = (T)s.contraction;
  const bool rw = (s.proposal == IPMC_PROPOSAL_RW);
  T* phi = (T*)s.phi;
  T* v = vpark + t;                       // this lane's proposal, v[j * kSpecBlock]
  const T* vgroup = vpark + (t - sub);    // lane 0 of the group
  const T* rs = (const T*)s.reg_scale;
  T ur[KM], sqr[KM], lor[KM], hir[KM], offr[KM], rsr[KM], th0r[KM];
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    const bool in = j < k;
    ur[j] = in ? u[j] : (T)0;
    sqr[j] = (in && sq) ? sq[j] : (T)0;
    lor[j] = (in && lo) ? lo[j] : (T)0;
    hir[j] = (in && hi) ? hi[j] : (T)0;
    offr[j] = (in && off) ? off[j] : (T)0;
    rsr[j] = (in && rs) ? rs[j] : (T)0;
    th0r[j] = (in && MODEL == IPMC_MODEL_LINEAR) ? ((const T*)m.theta0)[j] : (T)0;
  }
  T phu = phi[chain];
  int64_t nacc = 0, ncalls = 0;
  SampleClock clk(s);
  int64_t st = 0;
  // PRE: draws of steps [pbase, pbase + C) of this group, in pre_w / pre_lr
  const int grp = (t - sub) / S;  // this group's index in the block
  T* gw = pre_w + (PRE ? grp * C * KM : 0);
  double* glr = pre_lr + (PRE ? grp * C : 0);
  int64_t pbase = 0, pend = 0;
  // w_j of step tt (sqrt(C_jj)·ξ_j or Σ_{i<=j} L_ji ξ_i), in the sequential kernel's order
  auto draw_w = [&](uint64_t step, T (&w)[KM]) {
    double z0 = 0.0, z1 = 0.0;
    T xi[(KM + 1) & ~1];
    if (chol) {
#pragma unroll
      for (int j = 0; j < KM; j += 2) {
        if (j < k) normal_pair(s.seed, gid, step, (uint32_t)(j >> 1), z0, z1);
        xi[j] = (T)z0;
        xi[j + 1] = (T)z1;
      }
    }
#pragma unroll
    for (int j = 0; j < KM; ++j) {
      w[j] = (T)0;
      if (j < k) {
        if (chol) {
#pragma unroll
          for (int i = 0; i <= j; ++i) w[j] = w[j] + xi[i] * chol[j * k + i];
        } else {
          if ((j & 1) == 0) normal_pair(s.seed, gid, step, (uint32_t)(j >> 1), z0, z1);
          w[j] = sqr[j] * (T)((j & 1) ? z1 : z0);
        }
      }
    }
  };
  // The speculation tree (ipmc_sweep_common.hpp, ipmc_spec_tree.hpp): lane
  // `sub` of the group is node `sub` of the tree for the chain's recent
  // acceptance rate; its proposal starts from its origin node's, formed one
  // level earlier.  Config 2 accepts 88 %: the tree there is the accept chain
  // (~7 steps per round at S = 16); a chain accepting nothing gets the reject
  // chain (S steps per round).
  SpecGuess guess(spec_accept_prior(s, chain));
  // this lane's node of the current tree, reloaded only when the tree changes
  // (a table load per round is most of a linear round's latency)
  int ctb = -1, maxlvl = 0;
  SpecNode nd{};
  unsigned long long nanc = 0, nedge = 0;
  while (st < s.n_steps) {
    const int64_t left = s.n_steps - st;
    const int tb = guess.bucket();
    if (tb != ctb) {  // uniform per group
      nd = kSpecTrees.nd[tb][sub];
      maxlvl = kSpecTrees.maxlvl[tb][S];
      nanc = kSpecTrees.anc[tb][sub];
      nedge = kSpecTrees.edge[tb][sub];
      ctb = tb;
    }
    const bool act = nd.depth < left;  // this node's step is in the launch
    const int64_t tt = st + nd.depth;
    if constexpr (PRE) {
      // refill when this round's slots reach past the held draws (uniform per group)
      if (st + S > pend && pend < s.n_steps) {
        pbase = st;
        pend = st + C;
        wave_sync_lds();  // the previous chunk's reads are done
#pragma unroll
        for (int r = 0; r < kPreFactor; ++r) {  // independent draws: the compiler interleaves them
          const int i = sub + r * S;
          const int64_t ti = pbase + i;
          if (ti < s.n_steps) {
            const uint64_t step = s.step0 + (uint64_t)ti;
            T w[KM];
            draw_w(step, w);
#pragma unroll
            for (int j = 0; j < KM; ++j) gw[i * KM + j] = w[j];
            glr[i] = det_log(accept_uniform(s.seed, gid, step));
          }
        }
        wave_sync_lds();
      }
    }
    // this node's proposal noise w (step tt)
    T w[KM];
    if (act) {
      if constexpr (PRE) {
        const int pi = (int)(tt - pbase);
#pragma unroll
        for (int j = 0; j < KM; ++j) w[j] = gw[pi * KM + j];
      } else {
        draw_w(s.step0 + (uint64_t)tt, w);
      }
    }
    const T bs = (act && s.beta_schedule) ? (T)s.beta_schedule[2 * tt] : beta;
    const T cs = (act && s.beta_schedule) ? (T)s.beta_schedule[2 * tt + 1] : contr;
    // the proposals level by level: a node's origin was formed one level before
    T vr[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) vr[j] = (T)0;
    for (int lv = 0; lv <= maxlvl; ++lv) {
      if (act && nd.lvl == lv) {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
          if (j < k) {
            const T o = nd.orig < 0 ? ur[j] : vgroup[j * kSpecBlock + nd.orig];
            vr[j] = propose_one<T>(rw, o, w[j], cs, bs);
            v[j * kSpecBlock] = vr[j];
          }
        }
      }
      wave_sync_lds();
    }
    bool ok = false, acc = false;
    T phv = (T)0;
    double lr = 0.0;
    if (act) {
      ok = true;
#pragma unroll
      for (int j = 0; j < KM; ++j) {
        if (j < k) {
          const T tb = vr[j] + offr[j];  // + 0 when there is no offset: the same bits as v_j
          if (lo && !(lor[j] < tb)) ok = false;
          if (hi && !(tb < hir[j])) ok = false;
        }
      }
      if (ok) {
        if constexpr (MODEL == IPMC_MODEL_LINEAR) {
          const int nA = m.q * k;
          phv = staged ? lin_potential_staged<T, FM>(lin_c, lin_c + nA, lin_c + nA + m.q, th0r, m.q, k, v, kSpecBlock)
                       : small_potential<T, MODEL, FM>(m, v, kSpecBlock, (const T*)s.y, (const T*)s.gamma_inv);
        } else {
          phv = small_potential<T, MODEL, FM>(m, v, kSpecBlock, (const T*)s.y, (const T*)s.gamma_inv);
        }
        if (rs) {
          T r2 = (T)0;  // small_regularizer's order
#pragma unroll
          for (int j = 0; j < KM; ++j) {
            if (j < k) {
              const T tj = rsr[j] * v[j * kSpecBlock];
              r2 = madd<FM>(tj, tj, r2);
            }
          }
          phv = phv + (T)0.5 * r2;
        }
        lr = PRE ? glr[tt - pbase] : det_log(accept_uniform(s.seed, gid, s.step0 + (uint64_t)tt));
      }
    }
    // pcn_accept against the state this node proposed from: the chain's, or its origin node's proposal
    const T pho = __shfl(phv, gbase + (nd.orig < 0 ? 0 : nd.orig), 64);
    if (ok) acc = (double)((nd.orig < 0 ? phu : pho) - phv) > lr;
    const unsigned long long accm = (__ballot(acc) >> gbase) & gmask;
    const unsigned long long okm = (__ballot(ok) >> gbase) & gmask;
    // the walk resolved in parallel: each lane tests whether its node is on the path
    const unsigned long long path = (__ballot(act && ((accm ^ nedge) & nanc) == 0) >> gbase) & gmask;
    const SpecRound rd = spec_path_round(path, accm, okm);
    const T phf = __shfl(phv, gbase + (rd.win >= 0 ? rd.win : 0), 64);
    if (sub == 0 && (s.sum_u || (s.sample_every > 0 && clk.next < st + rd.used))) {
      // the states after each settled step, in step order: the same walk again
      const bool sums = s.sum_u != nullptr;
      RoundSums<KM> rsum(sums ? s.sum_u + chain * k : nullptr, (sums && s.sum_u2) ? s.sum_u2 + chain * k : nullptr,
                         sums ? k : 0);
      spec_path_replay(path, accm, [&](int q, int la) {
                  if (sums) {
#pragma unroll
                    for (int j = 0; j < KM; ++j)
                      if (j < k) rsum.add(j, la >= 0 ? (double)vgroup[j * kSpecBlock + la] : (double)ur[j]);
                  }
                  if (s.sample_every > 0 && clk.next == st + q) {
                    const int64_t sl = clk.take(clk.next);
                    T* so = (T*)s.sample_out + chain * s.sample_stride + sl * s.sample_step_stride;
#pragma unroll
                    for (int j = 0; j < KM; ++j)
                      if (j < k) so[j] = la >= 0 ? vgroup[j * kSpecBlock + la] : ur[j];
                  }
                });
      if (sums) rsum.store();
    }
    if (rd.win >= 0) {
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (j < k) ur[j] = vgroup[j * kSpecBlock + rd.win];
      phu = phf;
    }
    nacc += rd.nar;
    ncalls += rd.calls;
    guess.settle(rd.nar, rd.used);
    wave_sync_lds();  // the parks are rewritten next round
    st += rd.used;
  }
  if (sub == 0) {
    phi[chain] = phu;
    if (s.accepts) s.accepts[chain] += nacc;
    if (s.calls) s.calls[chain] += ncalls;
#pragma unroll
    for (int j = 0; j < KM; ++j)
      if (j < k) u[j] = ur[j];
    if (s.sample_out && s.sample_every == 0) {
      T* so = (T*)s.sample_out + chain * s.sample_stride;
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (j < k) so[j] = ur[j];
    }
  }
}

template <typename T, int MODEL, bool FM, bool PHI>
__global__ __launch_bounds__(kSmallBlock) void small_eval_kernel(const ipmc_model m, int64_t n,
                                                                 const T* __restrict__ uin,
                                                                 const T* __restrict__ y,
                                                                 const T* __restrict__ ginv, T* __restrict__ out) {
  const int64_t chain = (int64_t)blockIdx.x * kSmallBlock + threadIdx.x;
  if (chain >= n) return;
  const T* v = uin + chain * m.k;
  if constexpr (PHI) {
    out[chain] = small_potential<T, MODEL, FM>(m, v, 1, y, ginv);
  } else {
    const T* th0 = (const T*)m.theta0;
    if constexpr (MODEL == IPMC_MODEL_LORENZ63) {
      T g[6];
      l63_G<T, FM>(th0[0] + v[0], th0[1] + v[1], th0[2] + v[2], (const T*)m.x0, (T)m.dt, m.n_steps, g);
#pragma unroll
      for (int i = 0; i < 6; ++i) out[chain * 6 + i] = g[i];
    } else {
      const T* A = (const T*)m.A;
      for (int i = 0; i < m.q; ++i) {
        T acc = (T)0;
        for (int j = 0; j < m.k; ++j) acc = madd<FM>(A[(int64_t)i * m.k + j], th0[j] + v[j], acc);
        out[chain * m.q + i] = acc;
      }
    }
  }
}

}  // namespace ipmc
