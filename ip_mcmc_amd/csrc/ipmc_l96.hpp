// Lorenz-96 forward map + pCN sweep kernels.
//
// G(u): forcing field F = theta0 + u (one forcing per slow variable of the
// single-scale Lorenz-96 of lorenz.py:73-88, J = 0), x(0) = x0, classical RK4
// with fixed dt for n_steps steps, G_k = time average of X_k over the n
// post-step states.  The state of one chain lives in VGPRs of a group of LPC
// lanes (M = D/LPC components per lane); the cyclic neighbours X_{k-2},
// X_{k-1}, X_{k+1} that cross a lane boundary come from the neighbour lanes by
// DPP: quad permutations (LPC 2/4), row rotations (LPC 16; LPC 8 with two
// chains interleaved per row in the sequential kernels, shifts and a select in
// the speculative one).  Nothing touches HBM inside the RK
// loop: the kernel is VALU-bound.
#pragma once

#include "ipmc_sweep_common.hpp"

namespace ipmc {

// One classical RK4 stage with every rate consumed as soon as it is computed
// (no array of rates; cf. ts_stage in ipmc_l96ts.hip):
//   STAGE 1:   k = f(x);  acc = k;          xs = x + c k
//   STAGE 2/3: k = f(xs); acc = 2k + acc;   xs = x + c k   (in place)
//   STAGE 4:   k = f(xs); acc = acc + k;    x = x + c acc;  ob = ob + x
// The same operations as the textbook form (l96_rhs, then the updates), so the
// bits do not change.  The stage input's halos are fetched before anything is
// written, and the old X_{j-1}, X_{j-2} ride along in p1, p2, so `in` may alias
// `xs`: one array of M values fewer live in the RK loop.
template <typename V, int M, int LPC, bool FM, int STAGE, bool IL>
__device__ __forceinline__ void l96_stage(V (&in)[M], V (&xs)[M], V (&x)[M], V (&acc)[M], V (&ob)[M],
                                          const V (&F)[M], V c, V two, int lane) {
  static_assert(M >= 2, "Lorenz-96 needs at least 2 components per lane");
  const V sr1 = group_next<LPC, IL>(in[0], lane);
  V p2 = group_prev<LPC, IL>(in[M - 2], lane);
  V p1 = group_prev<LPC, IL>(in[M - 1], lane);
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const V cur = in[j];
    const V xp1 = (j < M - 1) ? in[j + 1] : sr1;
    V k;
    if constexpr (FM) {
      k = madd<true>(xp1 - p2, p1, F[j] - cur);
    } else {
      V t = -cur;
      t = t - (p1 * p2 - p1 * xp1);
      k = t + F[j];
    }
    p2 = p1;
    p1 = cur;
    if constexpr (STAGE == 1) {
      acc[j] = k;
      xs[j] = madd<FM>(c, k, x[j]);
    } else if constexpr (STAGE == 4) {
      acc[j] = acc[j] + k;
      x[j] = madd<FM>(c, acc[j], x[j]);
      ob[j] = ob[j] + x[j];
    } else {
      // 2k is exact, so fma(2, k, acc) rounds once exactly as the reference
      // order's acc + 2k does: fused in both arithmetic modes (one op, not two)
      acc[j] = madd<true>(two, k, acc[j]);
      xs[j] = madd<FM>(c, k, x[j]);
    }
  }
}

// IPMC_L96_RK_PER_ITER RK4 steps per loop iteration up to IPMC_L96_PAIR_MAX_M
// components per lane (l96_forward; profiles/r6/shard_kernel_ab10.jsonl)
#ifndef IPMC_L96_PAIR_MAX_M
#define IPMC_L96_PAIR_MAX_M 10
#endif
#ifndef IPMC_L96_RK_PER_ITER
#define IPMC_L96_RK_PER_ITER 4
#endif

// Time-averaged RK4 trajectory: g[j] = (Σ_{n=1..N} x_n[j]) / N.
// V is the per-lane storage type (float, double, or f32x2 = two fp32 chains),
// S the scalar type of the problem constants, IL: interleaved groups of 8
// (group_vlane, ipmc_device.hpp).
template <typename V, int M, int LPC, bool FM, bool IL = false, typename S>
__device__ __forceinline__ void l96_forward(const V (&F)[M], const S* __restrict__ x0, V h, int nsteps, int lane,
                                            V (&g)[M]) {
  using P = Splat<V>;
  const V h2 = h * P::of((S)0.5);
  const V h6 = h / P::of((S)6);
  const V two = P::of((S)2);
  V x[M], ob[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    x[j] = P::of(x0[j]);
    ob[j] = P::of((S)0);
  }
  // R RK4 steps per loop iteration where a lane's step is short (M <= 10):
  // the loop's scalar counter / compare / branch then issue once per R steps.
  // A wave alone on its SIMD (8 192 chains of d=40 on 8 lanes: M = 5, 127
  // instructions per step) issues every instruction in its own 4-cycle slot,
  // scalar ones included: R = 2 / 4 run the 8 192-chain sweep 1.5-2.2 / 2.4-
  // 3.5 % faster, 16 384 chains (M = 10) ~1 %; at M = 20 R = 2 gains ~1 % at
  // one wave per SIMD but not at the headline's two, so M = 20 keeps R = 1
  // (profiles/r6/shard_kernel_ab9.jsonl, shard_kernel_ab10.jsonl).  The
  // loads' s_waitcnt at the loop top, satisfied after the first step, cost
  // nothing (the `pw` A/B, same files).  The R = 1 loop is written
  // out as before: the packed fp32 headline kernel's VGPR numbering -- worth
  // 10 % of its time at one wave per SIMD -- follows the source's shape.
  constexpr int R = (M <= IPMC_L96_PAIR_MAX_M) ? IPMC_L96_RK_PER_ITER : 1;
  if constexpr (R > 1) {
    auto rk4 = [&]() {
      V acc[M], xs[M];
      l96_stage<V, M, LPC, FM, 1, IL>(x, xs, x, acc, ob, F, h2, two, lane);
      l96_stage<V, M, LPC, FM, 2, IL>(xs, xs, x, acc, ob, F, h2, two, lane);
      l96_stage<V, M, LPC, FM, 3, IL>(xs, xs, x, acc, ob, F, h, two, lane);
      l96_stage<V, M, LPC, FM, 4, IL>(xs, xs, x, acc, ob, F, h6, two, lane);
    };
    int n = 0;
    for (; n + R <= nsteps; n += R) {
#pragma unroll
      for (int r = 0; r < R; ++r) rk4();
    }
    for (; n < nsteps; ++n) rk4();
  } else {
    for (int n = 0; n < nsteps; ++n) {
      V acc[M], xs[M];
      l96_stage<V, M, LPC, FM, 1, IL>(x, xs, x, acc, ob, F, h2, two, lane);
      l96_stage<V, M, LPC, FM, 2, IL>(xs, xs, x, acc, ob, F, h2, two, lane);
      l96_stage<V, M, LPC, FM, 3, IL>(xs, xs, x, acc, ob, F, h, two, lane);
      l96_stage<V, M, LPC, FM, 4, IL>(xs, xs, x, acc, ob, F, h6, two, lane);
    }
  }
  const V nn = P::of((S)nsteps);
#pragma unroll
  for (int j = 0; j < M; ++j) g[j] = ob[j] / nn;
}

constexpr int kL96Block = 256;
static_assert(kL96Block == kL96SpecBlockLanes, "block-wide speculation spans one block");
// block-wide rounds index kSpecTrees.nd[tb][slot] with slot < kL96Block / LPC
static_assert(kL96Block <= kSpecNodes, "block-wide speculation slots index the spec-tree tables");

// LDS staging for the in-order misfit / regularizer sums of wide groups
// (LPC >= 8, group_sumsq); one element otherwise.
template <int M, int LPC>
constexpr int l96_stage_len() {
  return LPC >= 8 ? M * kL96Block : 1;
}

template <typename V, int M, int LPC, bool FM, bool IL = false, typename S>
__device__ __forceinline__ V l96_potential(const V (&v)[M], const S* __restrict__ th0, const S* __restrict__ x0,
                                           const S* __restrict__ y, const S* __restrict__ ginv, V h, int nsteps,
                                           int lane, V* stage) {
  using P = Splat<V>;
  V F[M], g[M];
#pragma unroll
  for (int j = 0; j < M; ++j) F[j] = P::of(th0[j]) + v[j];
  l96_forward<V, M, LPC, FM, IL>(F, x0, h, nsteps, lane, g);
  V r[M];
#pragma unroll
  for (int j = 0; j < M; ++j) r[j] = (P::of(y[j]) - g[j]) * P::of(ginv[j]);
  return P::of((S)0.5) * group_sumsq<V, M, LPC, FM, kL96Block, IL>(r, lane, stage, P::of((S)0));
}

// Occupancy target (waves per SIMD) the register allocator is held to: the
// RK loop keeps 5 arrays of M values live (x, F, time-average, k-sum, stage;
// l96_stage consumes each rate as it is computed), the proposal / accept stage
// ~40 registers of addressing / RNG / loop state around it.  The target is
// sized for 6 arrays (fp64 M = 17-20: see below).
// (fp32 one chain per lane group: the compiler's SLP packing needs ~96; every
// variant gets at least 104 registers, i.e. at most 4 waves, since the
// proposal / accept stage spills below that: 20-56 B per lane at 5 waves for
// M <= 5, e.g. d=40 at 8 lanes per chain.)
// fp64 at 17-20 components per lane (the headline's d=40 on 2 lanes): held to
// two waves.  Left free, the compiler took 258 (REFERENCE) / 271 (FMA)
// registers, one wave per SIMD.  At two waves it spilled what lives across G
// (the lane's chain index and addresses, Φ(u): 12 / 80 B per lane); with
// IPMC_L96_PARK the sequential sweep recomputes the lane state from the
// thread index after G and parks Φ(u) in LDS, so nothing spills: the headline
// kernel 3.20 -> 3.13 ms (FMA; profiles/r5/park_ab.jsonl), REFERENCE arith
// 5.24 -> 4.89 ms (profiles/r5/arith_waves_ab.jsonl).
#ifndef IPMC_L96_PARK  // 0: the lane state kept in registers across G (A/B)
#define IPMC_L96_PARK 1
#endif
// (LPC >= 8 stages the misfit through another M x 256 LDS array: two blocks of
// it do not fit the CU's 160 KiB, so those layouts stay at one wave.)
template <typename T, int M, bool FM = true, int LPC = 1>
constexpr int l96_waves_per_simd() {
#ifdef IPMC_L96_WAVES  // occupancy experiments (tools/)
  return IPMC_L96_WAVES;
#endif
  if constexpr ((!FM || IPMC_L96_PARK) && sizeof(T) == 8 && M >= 17 && M <= 20 && LPC < 8) return 2;
  constexpr int want = 6 * M * (int)(sizeof(T) / 4) + (sizeof(T) == 8 ? 40 : 96);
  constexpr int regs = want < 104 ? 104 : want;
  constexpr int w = 512 / regs;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// The packed fp32 kernel: 5 arrays of M f32x2 in the RK loop plus two chains'
// proposal / accept state (~76 registers); at least 196 registers (<40,4>
// spills in the proposal stage below that).  Two waves up to M = 17: a 257th
// register (the dense-prior proposal path pushed <256,16> to 256 VGPRs + 9
// AGPRs) halves the occupancy of every ensemble larger than one wave per SIMD,
// e.g. config 5's d=256 (121 -> 110 ms per f32 sweep; profiles/r2).
template <int M>
constexpr int l96_pk_waves_per_simd() {
#ifdef IPMC_PK_WAVES  // occupancy experiments (tools/)
  return IPMC_PK_WAVES;
#endif
  constexpr int want = 10 * M + 80;
  constexpr int w = 512 / (want < 196 ? 196 : want);
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// n_steps pCN steps per launch; u / Φ(u) / accept counts updated in place.
template <typename T, int D, int LPC, bool FM>
__global__ __launch_bounds__(kL96Block, (l96_waves_per_simd<T, D / LPC, FM, LPC>())) void l96_sweep_kernel(const ipmc_model m, const ipmc_sweep s) {
  constexpr int M = D / LPC;
  constexpr bool IL = (LPC == 8);  // interleaved groups of 8 (group_vlane)
  __shared__ T vpark[M][kL96Block];  // proposal parked in LDS while G runs
  __shared__ T stage[l96_stage_len<M, LPC>()];
#if IPMC_L96_PARK
  __shared__ T phpark[kL96Block];  // Φ(u) parked in LDS while G runs
#endif
  const int lane = threadIdx.x & 63;
  // the lane's chain, component block and addresses, from the thread index;
  // with IPMC_L96_PARK recomputed every pCN step behind an opaque copy of the
  // index, so none of it stays live across G
  struct Lane {
    int64_t chain;
    int sub, c0;
    uint64_t gid;
    T* u;
  };
  auto lane_state = [&](int tx) {
    Lane l;
    const int64_t tid = (int64_t)blockIdx.x * kL96Block + group_vlane<LPC, IL>(tx);
    l.chain = tid / LPC;
    l.sub = (int)(tid % LPC);
    l.c0 = l.sub * M;
    l.gid = (uint64_t)(s.chain_offset + l.chain);
    l.u = (T*)s.u + l.chain * D + l.c0;
    return l;
  };
  Lane L0 = lane_state(threadIdx.x);
  if (L0.chain >= s.n_chains) return;  // whole lane groups leave together
  const T beta = (T)s.beta, contr = (T)s.contraction, h = (T)m.dt;
  T* phi = (T*)s.phi;
  T phu = phi[L0.chain];
  const bool rw = (s.proposal == IPMC_PROPOSAL_RW);
  int nacc = 0, ncalls = 0;  // per launch (n_steps <= INT32_MAX, checked by the API)
  for (int64_t st = 0; st < s.n_steps; ++st) {
    const uint64_t step = s.step0 + (uint64_t)st;
#if IPMC_L96_PARK
    int tx = threadIdx.x;
    asm volatile("" : "+v"(tx));
    const Lane L = lane_state(tx);
#else
    const Lane& L = L0;
#endif
    const int64_t chain = L.chain;
    const int c0 = L.c0;
    const uint64_t gid = L.gid;
    T* __restrict__ u = L.u;
    // Opaque per-step offset: keeps the loop-invariant per-component constants
    // (theta0, x0, y, 1/gamma, sqrt C) from being hoisted into 5*M VGPRs for
    // the whole launch; they are re-read from L1/L2 once per pCN step instead.
    // The proposal takes it as its first component too, so the Philox rounds on
    // the (constant) normal slots are recomputed each step rather than hoisted
    // and spilled to scratch around G (36 B per lane: 1.6x the compulsory HBM
    // bytes of the headline sweep, profiles/r2/pmc_l96_f64_hoisted.json).
    int cl = c0;
    asm volatile("" : "+v"(cl));
    const T bs = s.beta_schedule ? (T)s.beta_schedule[2 * st] : beta;
    const T cs = s.beta_schedule ? (T)s.beta_schedule[2 * st + 1] : contr;
    T v[M];
    pcn_propose<T, M>(u, (const T*)s.prior_sqrt + cl, cs, bs, s.seed, gid, step, cl, v, rw,
                      (const T*)s.prior_chol, D);
    if (box_valid<T, M, LPC, IL>(s, c0, v, lane)) {
      ++ncalls;
      const T reg = s.reg_scale
                        ? regularizer<T, M, LPC, FM, T, kL96Block, IL>((const T*)s.reg_scale + cl, v, lane, stage)
                        : (T)0;
#pragma unroll
      for (int j = 0; j < M; ++j) vpark[j][threadIdx.x] = v[j];
#if IPMC_L96_PARK
      phpark[threadIdx.x] = phu;
#endif
      T phv = l96_potential<T, M, LPC, FM, IL>(v, (const T*)m.theta0 + cl, (const T*)m.x0 + cl, (const T*)s.y + cl,
                                           (const T*)s.gamma_inv + cl, h, m.n_steps, lane, stage);
      if (s.reg_scale) phv = phv + reg;  // I(v) = Φ(v) + regularizer (accepter.py:106)
      // memory clobber: re-read v from LDS instead of keeping it live in VGPRs across G
      asm volatile("" ::: "memory");
#if IPMC_L96_PARK
      phu = phpark[threadIdx.x];
      int ty = threadIdx.x;
      asm volatile("" : "+v"(ty));
      const Lane La = lane_state(ty);
      const uint64_t gida = La.gid;
      T* __restrict__ ua = La.u;
#else
      const uint64_t gida = gid;
      T* __restrict__ ua = u;
#endif
      if (pcn_accept<T>(phu, phv, s.seed, gida, step)) {
#pragma unroll
        for (int j = 0; j < M; ++j) ua[j] = vpark[j][threadIdx.x];
        phu = phv;
        ++nacc;
      }
    }
    if (s.sum_u) {
      RoundSums<M> rsum(s.sum_u + chain * D + c0, s.sum_u2 ? s.sum_u2 + chain * D + c0 : nullptr, M);
#pragma unroll
      for (int j = 0; j < M; ++j) rsum.add(j, (double)u[j]);
      rsum.store();
    }
    const int64_t sl = sample_slot(s, st);
    if (sl >= 0) {
      T* so = (T*)s.sample_out + chain * s.sample_stride + sl * s.sample_step_stride + c0;
#pragma unroll
      for (int j = 0; j < M; ++j) so[j] = u[j];
    }
  }
#if IPMC_L96_PARK
  int te = threadIdx.x;
  asm volatile("" : "+v"(te));
  const Lane Le = lane_state(te);
#else
  const Lane& Le = L0;
#endif
  if (Le.sub == 0) {
    phi[Le.chain] = phu;
    if (s.accepts) s.accepts[Le.chain] += nacc;
    if (s.calls) s.calls[Le.chain] += ncalls;
  }
  if (s.sample_out && s.sample_every == 0) {
    T* so = (T*)s.sample_out + Le.chain * s.sample_stride + Le.c0;
#pragma unroll
    for (int j = 0; j < M; ++j) so[j] = Le.u[j];
  }
}

// Speculative sweep for ensembles too small to fill the GPU (as
// small_spec_kernel, ipmc_small.hpp): S slots of LPC lanes per chain
// (S*LPC <= 64, one wavefront, or one chain per block); slot s is node s of
// the speculation tree for the chain's recent acceptance rate
// (ipmc_spec_tree.hpp): it proposes step st + depth(s) from its origin node's
// proposal (or the current state), and the chain walks the tree along the real
// decisions (spec_walk, ipmc_sweep_common.hpp).  The state lives in registers
// of every slot (ur) and the proposals in the LDS park.  Bit-identical to
// l96_sweep_kernel.
template <typename T, int D, int LPC, bool FM>
__global__ __launch_bounds__(kL96Block) void l96_spec_kernel(const ipmc_model m, const ipmc_sweep s, int S) {
  constexpr int M = D / LPC;
  __shared__ T vpark[M][kL96Block];
  __shared__ T stage[l96_stage_len<M, LPC>()];
  // G == kL96Block: one chain per block, its slots spread over the block's
  // waves (one per SIMD of the CU, so a round takes the same time), combined
  // through LDS instead of a wave ballot
  __shared__ unsigned long long wmask[2][kL96Block / 64];
  __shared__ T phpark[kL96Block];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int G = S * LPC;  // lanes per chain: a power of two <= 64, or kL96Block
  const int64_t tid = (int64_t)blockIdx.x * kL96Block + t;
  const int64_t chain = tid / G;
  const int r = (int)(tid % G);
  const int slot = r / LPC, sub = r % LPC;
  const int gbase = lane - r;  // the chain's first lane in the wavefront
  if (chain >= s.n_chains) return;
  const uint64_t gid = (uint64_t)(s.chain_offset + chain);
  const int c0 = sub * M;
  T* __restrict__ u = (T*)s.u + chain * D + c0;
  const T beta = (T)s.beta, contr = (T)s.contraction, h = (T)m.dt;
  T* phi = (T*)s.phi;
  T ur[M];
#pragma unroll
  for (int j = 0; j < M; ++j) ur[j] = u[j];
  T phu = phi[chain];
  const bool rw = (s.proposal == IPMC_PROPOSAL_RW);
  const unsigned long long gmask = (G >= 64) ? ~0ull : ((1ull << G) - 1);
  int nacc = 0, ncalls = 0;
  SampleClock clk(s);
  int64_t st = 0;
  SpecGuess guess(spec_accept_prior(s, chain));  // the speculation tree (ipmc_sweep_common.hpp)
  const int lane0 = t - r + sub;  // slot 0's lane for my components
  while (st < s.n_steps) {
    const int64_t left = s.n_steps - st;
    const int tb = guess.bucket();
    const SpecNode nd = kSpecTrees.nd[tb][slot];
    const int maxlvl = kSpecTrees.maxlvl[tb][S];
    const bool act = nd.depth < left;  // uniform per slot: this node's step is in the launch
    const int64_t tt = st + nd.depth;
    const int og = nd.orig < 0 ? 0 : nd.orig;
    bool ok = false;
    T phv = (T)0;
    double lr = 0.0;
    int cl = c0;
    asm volatile("" : "+v"(cl));
    const uint64_t step = s.step0 + (uint64_t)tt;
    T w[M];
    if (act) pcn_noise<T, M>((const T*)s.prior_sqrt + cl, s.seed, gid, step, c0, w, (const T*)s.prior_chol, D);
    const T bs = (act && s.beta_schedule) ? (T)s.beta_schedule[2 * tt] : beta;
    const T cs = (act && s.beta_schedule) ? (T)s.beta_schedule[2 * tt + 1] : contr;
    // the proposals level by level: a node's origin was formed one level before
    T v[M];
#pragma unroll
    for (int j = 0; j < M; ++j) v[j] = (T)0;
    for (int lv = 0; lv <= maxlvl; ++lv) {
      if (act && nd.lvl == lv) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
          v[j] = propose_one<T>(rw, nd.orig < 0 ? ur[j] : vpark[j][lane0 + og * LPC], w[j], cs, bs);
          vpark[j][t] = v[j];
        }
      }
      if (G <= 64) wave_sync_lds();
      else __syncthreads();
    }
    if (act) {  // uniform per slot
      ok = box_valid<T, M, LPC>(s, c0, v, lane);
      if (ok) {
        const T reg = s.reg_scale
                          ? regularizer<T, M, LPC, FM, T, kL96Block>((const T*)s.reg_scale + cl, v, lane, stage)
                          : (T)0;
        phv = l96_potential<T, M, LPC, FM>(v, (const T*)m.theta0 + cl, (const T*)m.x0 + cl, (const T*)s.y + cl,
                                           (const T*)s.gamma_inv + cl, h, m.n_steps, lane, stage);
        if (s.reg_scale) phv = phv + reg;
        lr = det_log(accept_uniform(s.seed, gid, step));
      }
    }
    // pcn_accept against the state this node proposed from: the chain's, or
    // its origin node's proposal (whose Φ that slot's lanes hold)
    T pho;
    if (G <= 64) {
      pho = __shfl(phv, gbase + og * LPC, 64);
    } else {
      phpark[t] = phv;
      __syncthreads();
      pho = phpark[og * LPC];
    }
    const bool acc = ok && (double)((nd.orig < 0 ? phu : pho) - phv) > lr;
    // one bit per slot: the slot's lane sub == 0, at bit slot*LPC
    SpecRound rd;
    T phf;
    unsigned long long accm = 0, path = 0;  // G <= 64: the chain's bits, one per slot
    const SpecNode* tree = kSpecTrees.nd[tb];
    if (G <= 64) {
      // the walk resolved in parallel (spec_on_path): every lane tests its own
      // node against the slots' decisions, a ballot gathers the path -- no
      // cross-lane read inside a data-dependent loop
      accm = spec_slot_bits((__ballot(acc && sub == 0) >> gbase) & gmask, S, LPC);
      const unsigned long long okm = spec_slot_bits((__ballot(ok && sub == 0) >> gbase) & gmask, S, LPC);
      path = spec_slot_bits((__ballot(spec_on_path(tb, slot, accm, act) && sub == 0) >> gbase) & gmask, S, LPC);
      rd = spec_path_round(path, accm, okm);
      phf = __shfl(phv, gbase + (rd.win >= 0 ? rd.win : 0) * LPC, 64);
    } else {
      const unsigned long long ab = __ballot(acc && sub == 0), ob = __ballot(ok && sub == 0);
      if (lane == 0) {
        wmask[0][t >> 6] = ab;
        wmask[1][t >> 6] = ob;
      }
      __syncthreads();
      rd = spec_walk(
          S, left,
          [&](int n) {
            const int bit = n * LPC;
            return spec_step_bits(tree, n, 0, wmask[0][bit >> 6] >> (bit & 63), wmask[1][bit >> 6] >> (bit & 63));
          },
          [](int, int) {});
      phf = phpark[(rd.win >= 0 ? rd.win : 0) * LPC];
    }
    if (slot == 0 && (s.sum_u || (s.sample_every > 0 && clk.next < st + rd.used))) {
      // the states after each settled step, in step order: the same walk again
      const bool sums = s.sum_u != nullptr;
      RoundSums<M> rsum(sums ? s.sum_u + chain * D + c0 : nullptr,
                        (sums && s.sum_u2) ? s.sum_u2 + chain * D + c0 : nullptr, sums ? M : 0);
      auto visit = [&](int q, int la) {
        if (sums) {
#pragma unroll
          for (int j = 0; j < M; ++j) rsum.add(j, la >= 0 ? (double)vpark[j][lane0 + la * LPC] : (double)ur[j]);
        }
        if (s.sample_every > 0 && clk.next == st + q) {
          const int64_t sl = clk.take(clk.next);
          T* so = (T*)s.sample_out + chain * s.sample_stride + sl * s.sample_step_stride + c0;
#pragma unroll
          for (int j = 0; j < M; ++j) so[j] = la >= 0 ? vpark[j][lane0 + la * LPC] : ur[j];
        }
      };
      if (G <= 64) {
        spec_path_replay(path, accm, visit);
      } else {
        spec_replay(
            rd.used,
            [&](int n) {
              const int bit = n * LPC;
              return spec_step_bits(tree, n, 0, wmask[0][bit >> 6] >> (bit & 63), wmask[1][bit >> 6] >> (bit & 63));
            },
            visit);
      }
      if (sums) rsum.store();
    }
    if (rd.win >= 0) {
#pragma unroll
      for (int j = 0; j < M; ++j) ur[j] = vpark[j][lane0 + rd.win * LPC];
      phu = phf;
    }
    nacc += rd.nar;
    ncalls += rd.calls;
    guess.settle(rd.nar, rd.used);
    if (G <= 64) wave_sync_lds();  // the parks are rewritten next round
    else __syncthreads();
    st += rd.used;
  }
  if (slot == 0) {
#pragma unroll
    for (int j = 0; j < M; ++j) u[j] = ur[j];
    if (sub == 0) {
      phi[chain] = phu;
      if (s.accepts) s.accepts[chain] += nacc;
      if (s.calls) s.calls[chain] += ncalls;
    }
    if (s.sample_out && s.sample_every == 0) {
      T* so = (T*)s.sample_out + chain * s.sample_stride + c0;
#pragma unroll
      for (int j = 0; j < M; ++j) so[j] = ur[j];
    }
  }
}

// fp32, two chains per lane group (x = chain 2p, y = chain 2p+1): the RK loop
// runs on f32x2 so every FLOP is a v_pk_*_f32; proposal and accept stay per
// chain (scalar), so the bits equal the one-chain kernel's.
template <int D, int LPC, bool FM>
__global__ __launch_bounds__(kL96Block, (l96_pk_waves_per_simd<D / LPC>())) void l96_sweep_pk_kernel(
    const ipmc_model m, const ipmc_sweep s) {
  constexpr int M = D / LPC;
  using V = f32x2;
  constexpr bool IL = (LPC == 8);  // interleaved groups of 8 (group_vlane)
  __shared__ V vpark[M][kL96Block];
  __shared__ V stage[l96_stage_len<M, LPC>()];
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * kL96Block + group_vlane<LPC, IL>(threadIdx.x);
  const int64_t pair = tid / LPC;
  const int sub = (int)(tid % LPC);
  const int64_t ca = 2 * pair;
  if (ca >= s.n_chains) return;
  const bool has_b = ca + 1 < s.n_chains;
  const int64_t cb = has_b ? ca + 1 : ca;  // a phantom B duplicates A and is never written
  const uint64_t ga = (uint64_t)(s.chain_offset + ca), gb = (uint64_t)(s.chain_offset + cb);
  const int c0 = sub * M;
  float* __restrict__ ua = (float*)s.u + ca * D + c0;
  float* __restrict__ ub = (float*)s.u + cb * D + c0;
  const float beta = (float)s.beta, contr = (float)s.contraction;
  const V h = Splat<V>::of((float)m.dt);
  float* phi = (float*)s.phi;
  float pa = phi[ca], pb = phi[cb];
  int na = 0, nb = 0, ka = 0, kb = 0;  // per launch (n_steps <= INT32_MAX)
  for (int64_t st = 0; st < s.n_steps; ++st) {
    const uint64_t step = s.step0 + (uint64_t)st;
    int cl = c0;
    asm volatile("" : "+v"(cl));
    const float bs = s.beta_schedule ? (float)s.beta_schedule[2 * st] : beta;
    const float cs = s.beta_schedule ? (float)s.beta_schedule[2 * st + 1] : contr;
    const float* sq = (const float*)s.prior_sqrt + cl;
    const bool rw = (s.proposal == IPMC_PROPOSAL_RW);
    // the proposal's component base: opaque per step (no hoisted, spilled
    // Philox rounds, as in l96_sweep_kernel) except at M = 20, whose spill-free
    // register assignment with the hoisted form measured 7 % faster (d=40,
    // 1.77 vs 1.91 ms; the RK loop's instructions are identical, their VGPR
    // numbering is not: profiles/r2/pk_codegen.txt)
    const int pc0 = (M == 20) ? c0 : cl;
    // propose A, park it, then B: one chain's proposal live at a time (the
    // two-chain proposal stage otherwise spills past the occupancy target)
    bool oka, okb;
    {
      float va[M];
      pcn_propose<float, M>(ua, sq, cs, bs, s.seed, ga, step, pc0, va, rw, (const float*)s.prior_chol, D);
      oka = box_valid<float, M, LPC, IL>(s, c0, va, lane);
#pragma unroll
      for (int j = 0; j < M; ++j) vpark[j][threadIdx.x].x = va[j];
    }
    asm volatile("" ::: "memory");
    {
      float vb[M];
      pcn_propose<float, M>(ub, sq, cs, bs, s.seed, gb, step, pc0, vb, rw, (const float*)s.prior_chol, D);
      okb = has_b && box_valid<float, M, LPC, IL>(s, c0, vb, lane);
#pragma unroll
      for (int j = 0; j < M; ++j) vpark[j][threadIdx.x].y = vb[j];
    }
    asm volatile("" ::: "memory");
    if (oka || okb) {
      ka += oka;
      kb += okb;
      V v[M];
#pragma unroll
      for (int j = 0; j < M; ++j) v[j] = vpark[j][threadIdx.x];
      const V reg = s.reg_scale
                        ? regularizer<V, M, LPC, FM, float, kL96Block, IL>((const float*)s.reg_scale + cl, v, lane,
                                                                         stage)
                        : V{0.f, 0.f};
      V ph = l96_potential<V, M, LPC, FM, IL>(v, (const float*)m.theta0 + cl, (const float*)m.x0 + cl,
                                          (const float*)s.y + cl, (const float*)s.gamma_inv + cl, h, m.n_steps,
                                          lane, stage);
      if (s.reg_scale) ph = ph + reg;
      asm volatile("" ::: "memory");
      if (oka && pcn_accept<float>(pa, ph.x, s.seed, ga, step)) {
#pragma unroll
        for (int j = 0; j < M; ++j) ua[j] = vpark[j][threadIdx.x].x;
        pa = ph.x;
        ++na;
      }
      if (okb && pcn_accept<float>(pb, ph.y, s.seed, gb, step)) {
#pragma unroll
        for (int j = 0; j < M; ++j) ub[j] = vpark[j][threadIdx.x].y;
        pb = ph.y;
        ++nb;
      }
    }
    if (s.sum_u) {  // chain a's sums, then chain b's (RoundSums: batched loads and stores)
      {
        RoundSums<M> rsum(s.sum_u + ca * D + c0, s.sum_u2 ? s.sum_u2 + ca * D + c0 : nullptr, M);
#pragma unroll
        for (int j = 0; j < M; ++j) rsum.add(j, (double)ua[j]);
        rsum.store();
      }
      if (has_b) {
        RoundSums<M> rsum(s.sum_u + cb * D + c0, s.sum_u2 ? s.sum_u2 + cb * D + c0 : nullptr, M);
#pragma unroll
        for (int j = 0; j < M; ++j) rsum.add(j, (double)ub[j]);
        rsum.store();
      }
    }
    const int64_t sl = sample_slot(s, st);
    if (sl >= 0) {
      float* so = (float*)s.sample_out + ca * s.sample_stride + sl * s.sample_step_stride + c0;
#pragma unroll
      for (int j = 0; j < M; ++j) so[j] = ua[j];
      if (has_b) {
        float* sb = (float*)s.sample_out + cb * s.sample_stride + sl * s.sample_step_stride + c0;
#pragma unroll
        for (int j = 0; j < M; ++j) sb[j] = ub[j];
      }
    }
  }
  if (sub == 0) {
    phi[ca] = pa;
    if (s.accepts) s.accepts[ca] += na;
    if (s.calls) s.calls[ca] += ka;
    if (has_b) {
      phi[cb] = pb;
      if (s.accepts) s.accepts[cb] += nb;
      if (s.calls) s.calls[cb] += kb;
    }
  }
  if (s.sample_out && s.sample_every == 0) {
    float* so = (float*)s.sample_out + ca * s.sample_stride + c0;
#pragma unroll
    for (int j = 0; j < M; ++j) so[j] = ua[j];
    if (has_b) {
      float* sb = (float*)s.sample_out + cb * s.sample_stride + c0;
#pragma unroll
      for (int j = 0; j < M; ++j) sb[j] = ub[j];
    }
  }
}

// G(u) or Φ(u) for n parameter vectors (no proposal): out = g [n, D] or phi [n].
template <typename T, int D, int LPC, bool FM, bool PHI>
__global__ __launch_bounds__(kL96Block, (l96_waves_per_simd<T, D / LPC, FM, LPC>())) void l96_eval_kernel(const ipmc_model m, int64_t n, const T* __restrict__ uin,
                                                              const T* __restrict__ yin,
                                                              const T* __restrict__ ginvin, T* __restrict__ out) {
  constexpr int M = D / LPC;
  constexpr bool IL = (LPC == 8);  // interleaved groups of 8 (group_vlane)
  __shared__ T stage[PHI ? l96_stage_len<M, LPC>() : 1];
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * kL96Block + group_vlane<LPC, IL>(threadIdx.x);
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
    const T ph = l96_potential<T, M, LPC, FM, IL>(v, th0, x0, yin + c0, ginvin + c0, h, m.n_steps, lane, stage);
    if (sub == 0) out[chain] = ph;
  } else {
    T F[M], g[M];
#pragma unroll
    for (int j = 0; j < M; ++j) F[j] = th0[j] + v[j];
    l96_forward<T, M, LPC, FM, IL>(F, x0, h, m.n_steps, lane, g);
#pragma unroll
    for (int j = 0; j < M; ++j) out[chain * D + c0 + j] = g[j];
  }
}

}  // namespace ipmc
