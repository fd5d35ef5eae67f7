// Shared pieces of every pCN sweep kernel: proposal, ordered misfit, accept.
//
// One chain is owned by a group of LPC consecutive lanes (LPC in {1,2,4,8,16});
// lane `sub` of the group owns parameter components [sub*M, sub*M + M).
// Everything a group computes is a function of (seed, global chain id, global
// step) only, so results are independent of LPC, of the grid and of sharding.
#pragma once

#include "../../include/ipmc.h"
#include "ipmc_device.hpp"

namespace ipmc {

// pCN: v = contraction*u + beta*(sqrt(C_ii) * xi_i)   (proposer.py:81-82)
// RW:  v = u + beta*(sqrt(C_ii) * xi_i)               (proposer.py:29-30, beta = sqrt(2 delta))
// in the reference's expression order: products first, then the sum, no FMA.
template <typename T>
__device__ __forceinline__ T propose_one(bool rw, T u, T w, T contr, T beta) {
  return rw ? u + beta * w : contr * u + beta * w;
}

// Non-diagonal prior (sweep.prior_chol = L, the lower Cholesky factor of C,
// row-major [k, k]): w_j = Σ_{i<=j} L[j][i] ξ_i, summed in ascending i from
// +0 with no FMA (oracle/orc_models.inc: the same order).  The group's lane
// owning components [c0, c0+M) draws ξ_0 .. ξ_{c0+M-1} itself (the proposal is
// a negligible part of a step next to G).
template <typename T, int M>
__device__ __forceinline__ void chol_propose(const T* __restrict__ u, const T* __restrict__ L, int k, T contr,
                                             T beta, uint64_t seed, uint64_t gid, uint64_t step, int c0, T (&v)[M],
                                             bool rw) {
  T w[M];
#pragma unroll
  for (int j = 0; j < M; ++j) w[j] = (T)0;
  const int iend = c0 + M;
  for (int i = 0; i < iend; i += 2) {
    double z0, z1;
    normal_pair(seed, gid, step, (uint32_t)(i >> 1), z0, z1);
    const T x0 = (T)z0, x1 = (T)z1;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int r = c0 + j;
      if (i <= r) w[j] = w[j] + x0 * L[(int64_t)r * k + i];
      if (i + 1 <= r) w[j] = w[j] + x1 * L[(int64_t)r * k + i + 1];
    }
  }
#pragma unroll
  for (int j = 0; j < M; ++j) v[j] = propose_one<T>(rw, u[j], w[j], contr, beta);
}

template <typename T, int M>
__device__ __forceinline__ void pcn_propose(const T* __restrict__ u, const T* __restrict__ sq, T contr, T beta,
                                            uint64_t seed, uint64_t gid, uint64_t step, int c0, T (&v)[M],
                                            bool rw = false, const T* __restrict__ chol = nullptr, int k = 0) {
  if (chol) {
    chol_propose<T, M>(u, chol, k, contr, beta, seed, gid, step, c0, v, rw);
    return;
  }
  if constexpr (M % 2 == 0) {
    // c0 is even whenever M is even: pairs never straddle lanes
#pragma unroll
    for (int j = 0; j < M; j += 2) {
      double z0, z1;
      normal_pair(seed, gid, step, (uint32_t)((c0 + j) >> 1), z0, z1);
      const T w0 = sq[j] * (T)z0;
      const T w1 = sq[j + 1] * (T)z1;
      v[j] = propose_one<T>(rw, u[j], w0, contr, beta);
      v[j + 1] = propose_one<T>(rw, u[j + 1], w1, contr, beta);
    }
  } else {
    double z0 = 0.0, z1 = 0.0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int c = c0 + j;
      if (j == 0 || (c & 1) == 0) normal_pair(seed, gid, step, (uint32_t)(c >> 1), z0, z1);
      const T w = sq[j] * (T)((c & 1) ? z1 : z0);
      v[j] = propose_one<T>(rw, u[j], w, contr, beta);
    }
  }
}

// s = Σ_i r_i^2 over the chain's q = LPC*M residuals in component order
// (lane 0's M values, then lane 1's, ...), identical on every lane of the group.
template <typename T, int M, int LPC, bool FM, int S = 0, bool IL = false>
__device__ __forceinline__ T ordered_sumsq(const T (&r)[M], int lane, T s) {
  if constexpr (S == LPC) {
    return s;
  } else {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const T x = group_bcast<LPC, S, IL>(r[j], lane);
      s = madd<FM>(x, x, s);
    }
    return ordered_sumsq<T, M, LPC, FM, S + 1, IL>(r, lane, s);
  }
}

// The same in-order sum through LDS for wide groups (LPC >= 8): each lane
// parks its M values in `stage` (M rows of BLK, this thread's column) and every
// lane of the group reads the chain's LPC*M values back in order -- broadcast
// LDS reads instead of LPC*M cross-lane moves, which the compiler would issue
// all at once and spill (d = 256: 345 VGPRs of spill without this).
template <typename V, int M, int LPC, bool FM, int BLK, bool IL = false>
__device__ __forceinline__ V ordered_sumsq_lds(const V (&r)[M], V* stage, V s) {
  const int t = group_vlane<LPC, IL>(threadIdx.x);  // the group's lanes are consecutive columns
  const int base = t & ~(LPC - 1);
#pragma unroll
  for (int j = 0; j < M; ++j) stage[j * BLK + t] = r[j];
  wave_sync_lds();
#pragma unroll 1
  for (int sub = 0; sub < LPC; ++sub) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const V x = stage[j * BLK + base + sub];
      s = madd<FM>(x, x, s);
    }
  }
  wave_sync_lds();  // the stage is reused by the next sum
  return s;
}

template <typename V, int M, int LPC, bool FM, int BLK, bool IL = false>
__device__ __forceinline__ V group_sumsq(const V (&r)[M], int lane, V* stage, V s) {
  if constexpr (LPC >= 8 && BLK > 0) return ordered_sumsq_lds<V, M, LPC, FM, BLK, IL>(r, stage, s);
  else return ordered_sumsq<V, M, LPC, FM, 0, IL>(r, lane, s);
}

// StandardRWAccepter regularizer ½ Σ_i (c_i v_i)² over the chain's components
// in component order (accepter.py:104-106 with the reference's sqrt-covariance
// factor); c = reg_scale + this lane's offset.
template <typename V, int M, int LPC, bool FM, typename S, int BLK = 0, bool IL = false>
__device__ __forceinline__ V regularizer(const S* __restrict__ c, const V (&v)[M], int lane, V* stage = nullptr) {
  using P = Splat<V>;
  V t[M];
#pragma unroll
  for (int j = 0; j < M; ++j) t[j] = P::of(c[j]) * v[j];
  return P::of((S)0.5) * group_sumsq<V, M, LPC, FM, BLK, IL>(t, lane, stage, P::of((S)0));
}

// ConstrainAccepter box: lo < v + off < hi for every component of the chain.
template <typename T, int M, int LPC, bool IL = false>
__device__ __forceinline__ bool box_valid(const ipmc_sweep& s, int c0, const T (&v)[M], int lane) {
  if (!s.box_lo && !s.box_hi) return true;
  const T* lo = (const T*)s.box_lo;
  const T* hi = (const T*)s.box_hi;
  const T* off = (const T*)s.box_off;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const T t = v[j] + (off ? off[c0 + j] : (T)0);
    if (lo && !(lo[c0 + j] < t)) ok = false;
    if (hi && !(t < hi[c0 + j])) ok = false;
  }
  return group_all<LPC, IL>(ok, lane);
}

// In-launch recording (ipmc_sweep.sample_every > 0, sampler.py:23-28): u
// after step j (0-based in this launch) is sample (j+1)/every - 1 when
// (j+1) % every == 0.
// Sequential sweeps: from the (wave-uniform) step counter after G -- nothing
// extra is live across G, whose RK loop may hold every register (a clock
// carried across G changed the packed M = 20 kernel's register assignment).
__device__ __forceinline__ int64_t sample_slot(const ipmc_sweep& s, int64_t j) {
  return (s.sample_every > 0 && (j + 1) % s.sample_every == 0) ? (j + 1) / s.sample_every - 1 : -1;
}
// Speculative sweeps (several steps per round): tracked incrementally by the
// recording lane -- `next` is the next such j -- so no step pays a division.
struct SampleClock {
  int64_t next, slot, every;
  __device__ explicit SampleClock(const ipmc_sweep& s)
      : next(s.sample_every > 0 ? s.sample_every - 1 : INT64_MAX), slot(0), every(s.sample_every) {}
  // the state after step j is a sample: its slot (advancing the clock), else -1
  __device__ __forceinline__ int64_t take(int64_t j) {
    if (j != next) return -1;
    next += every;
    return slot++;
  }
};

// ---------------------------------------------------------- speculation
// A speculative round evaluates the next S steps of a chain at once, slot s
// taking step st+s under a guess of the decisions before it: reject mode (the
// steps before it rejected: every slot proposes from the current state, the
// first acceptance ends the round) or accept mode (accepted: slot s proposes
// from slot s-1's proposal, the first rejection ends the round).  The slot
// where the guess first fails still decided correctly (its inputs were
// right), so a round settles `used` steps either way and the results are
// bit-identical to the sequential chain; the guess only changes how many.
// A chain guesses "accept" while it accepted at least half of its recent
// steps: accepted and settled steps summed over its rounds with weight 3/4 per
// round back (~4 rounds).  Rounds 1-3 used the whole launch's ratio, which
// lags behind a posterior whose acceptance changes along the run (burn-in, a
// step-size schedule) once launches are long (sampler.STEPS_PER_LAUNCH).
// Before its first round: `prior`.
struct SpecGuess {
  float a, n;  // recency-weighted accepted / settled steps
  __device__ __forceinline__ explicit SpecGuess(bool prior) : a(prior ? 1.f : 0.f), n(1.f) {}
  __device__ __forceinline__ bool accept_mode() const {
#ifdef IPMC_SPEC_REJECT_ONLY  // experiments (tools/build_variant.sh): the reject path only
    return false;
#endif
    return 2.f * a >= n;
  }
  __device__ __forceinline__ void settle(int nar, int used) {
#ifdef IPMC_SPEC_GUESS_CUMULATIVE  // experiments: rounds 1-3's whole-launch ratio
    if (fresh) a = n = 0.f;
    fresh = false;
    a += (float)nar;
    n += (float)used;
#else
    a = fmaf(0.75f, a, (float)nar);
    n = fmaf(0.75f, n, (float)used);
#endif
  }
#ifdef IPMC_SPEC_GUESS_CUMULATIVE
  bool fresh = true;
#endif
};
// The prior at a launch's first round: the chain's accept counter over the
// steps it has counted before the launch (step0 - accepts_step0: a resumed or
// continued run counts from its own first step, not from global step 0);
// accept mode without any history.
__device__ __forceinline__ bool spec_accept_prior(const ipmc_sweep& s, int64_t chain) {
  if (!s.accepts || s.step0 <= s.accepts_step0) return true;
  return (uint64_t)(2 * s.accepts[chain]) >= s.step0 - s.accepts_step0;
}

struct SpecRound {
  int first;  // the first slot whose guess failed (S: none)
  int used;   // steps settled by the round
  int nar;    // accepted steps among them
  int win;    // the slot whose proposal is the chain's new state (-1: unchanged)
};
// From the slots' decisions: slot s's at bit s*L of acc_bits (L lanes per slot).
__device__ __forceinline__ SpecRound spec_round(bool amode, unsigned long long acc_bits, int S, int L, int64_t left) {
  const int lim = left < S ? (int)left : S;
  SpecRound r;
  if (!amode) {
    r.first = acc_bits ? __builtin_ctzll(acc_bits) / L : S;
    r.used = r.first < S ? r.first + 1 : lim;
    r.nar = r.first < S ? 1 : 0;
    r.win = r.first < S ? r.first : -1;
  } else {
    unsigned long long ev = 0;  // the evaluated slots' bits
    for (int q = 0; q < lim; ++q) ev |= 1ull << (q * L);
    const unsigned long long rej = ev & ~acc_bits;
    r.first = rej ? __builtin_ctzll(rej) / L : S;
    r.used = r.first < S ? r.first + 1 : lim;
    r.nar = r.first < S ? r.first : lim;
    r.win = r.nar - 1;
  }
  return r;
}
// The slot whose proposal is the chain's state after step st+q of the round (-1: the old state).
__device__ __forceinline__ int spec_last_acc(const SpecRound& r, bool amode, int q) {
  return amode ? (q < r.nar ? q : r.nar - 1) : (q == r.first ? r.first : -1);
}

// Running sums Σu, Σu² (ipmc_sweep.sum_u / sum_u2) of a lane's n <= N
// components over the steps a round (or a step) settles, held in registers
// meanwhile: one batched load before and one store after.  A `+=` on global
// memory per step and component compiles to a dependent load / add / store
// chain -- 2n memory round trips per settled step, as long as the forward map
// itself for a short one (Lorenz-63: config 2 through MCMCSampler.run with
// keep="moments").  The additions are the per-step ones in step order: the
// same bits.
template <int N>
struct RoundSums {
  double a[N], b[N];
  double* su;
  double* su2;
  int n;
  __device__ __forceinline__ RoundSums(double* su_, double* su2_, int n_) : su(su_), su2(su2_), n(n_) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      a[j] = j < n ? su[j] : 0.0;
      b[j] = (su2 && j < n) ? su2[j] : 0.0;
    }
  }
  __device__ __forceinline__ void add(int j, double ud) {
    a[j] = a[j] + ud;
    b[j] = b[j] + ud * ud;
  }
  __device__ __forceinline__ void store() {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j < n) {
        su[j] = a[j];
        if (su2) su2[j] = b[j];
      }
    }
  }
};

// accept iff Φ(u) − Φ(v) > log r   ⇔ exp(Φ(u) − Φ(v)) > r   (accepter.py:62, 121-122)
template <typename T>
__device__ __forceinline__ bool pcn_accept(T phu, T phv, uint64_t seed, uint64_t gid, uint64_t step) {
  const double r = accept_uniform(seed, gid, step);
  return (double)(phu - phv) > det_log(r);
}

}  // namespace ipmc
