// Shared pieces of every pCN sweep kernel: proposal, ordered misfit, accept.
//
// One chain is owned by a group of LPC consecutive lanes (LPC in {1,2,4,8,16});
// lane `sub` of the group owns parameter components [sub*M, sub*M + M).
// Everything a group computes is a function of (seed, global chain id, global
// step) only, so results are independent of LPC, of the grid and of sharding.
#pragma once

#include "../../include/ipmc.h"
#include "ipmc_device.hpp"
#include "ipmc_spec_tree.hpp"

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
__device__ __forceinline__ void chol_noise(const T* __restrict__ L, int k, uint64_t seed, uint64_t gid, uint64_t step,
                                           int c0, T (&w)[M]) {
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
}

// A step's proposal noise w for components [c0, c0+M): sqrt(C_jj)·ξ_j, or
// Σ_{i<=j} L_ji ξ_i with a Cholesky factor.
template <typename T, int M>
__device__ __forceinline__ void pcn_noise(const T* __restrict__ sq, uint64_t seed, uint64_t gid, uint64_t step, int c0,
                                          T (&w)[M], const T* __restrict__ chol = nullptr, int k = 0) {
  if (chol) {
    chol_noise<T, M>(chol, k, seed, gid, step, c0, w);
    return;
  }
  if constexpr (M % 2 == 0) {
    // c0 is even whenever M is even: pairs never straddle lanes
#pragma unroll
    for (int j = 0; j < M; j += 2) {
      double z0, z1;
      normal_pair(seed, gid, step, (uint32_t)((c0 + j) >> 1), z0, z1);
      w[j] = sq[j] * (T)z0;
      w[j + 1] = sq[j + 1] * (T)z1;
    }
  } else {
    double z0 = 0.0, z1 = 0.0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int c = c0 + j;
      if (j == 0 || (c & 1) == 0) normal_pair(seed, gid, step, (uint32_t)(c >> 1), z0, z1);
      w[j] = sq[j] * (T)((c & 1) ? z1 : z0);
    }
  }
}

template <typename T, int M>
__device__ __forceinline__ void pcn_propose(const T* __restrict__ u, const T* __restrict__ sq, T contr, T beta,
                                            uint64_t seed, uint64_t gid, uint64_t step, int c0, T (&v)[M],
                                            bool rw = false, const T* __restrict__ chol = nullptr, int k = 0) {
  T w[M];
  pcn_noise<T, M>(sq, seed, gid, step, c0, w, chol, k);
#pragma unroll
  for (int j = 0; j < M; ++j) v[j] = propose_one<T>(rw, u[j], w[j], contr, beta);
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
// A speculative round evaluates several future steps of a chain at once, its
// S slots taking the first S nodes of a speculation tree (ipmc_spec_tree.hpp):
// node n proposes step st + depth(n) from the proposal of its origin node (or
// the chain's state) with that step's draws, so it is exactly the proposal
// the sequential chain makes there if the decisions before it go the way the
// node's path says.  The chain then walks the tree along the real decisions
// (spec_walk): every visited node's decision is the sequential chain's, and
// the round settles the steps up to the first node whose next node is not
// among the slots.  Results are bit-identical to the sequential chain for any
// tree; the tree, picked by the chain's recent acceptance rate, only sets how
// many steps a round settles.
static __constant__ const SpecTrees kSpecTrees = make_spec_trees();

#ifndef IPMC_SPEC_TREE  // 0: rounds 3-4's two paths only, reject or accept chain (A/B)
#define IPMC_SPEC_TREE 1
#endif
#ifndef IPMC_SPEC_MEMORY  // the acceptance estimate's weight per round back (A/B)
#define IPMC_SPEC_MEMORY 0.75f
#endif

// The chain's recent acceptance rate: accepted and settled steps summed over
// its rounds with weight 3/4 per round back (~4 rounds).  A chain's accepts
// come in bursts (a chain leaving a local minimum accepts several steps in a
// row), which a short memory follows; rounds 1-3 used the whole launch's
// ratio, which also lags behind a posterior whose acceptance changes along
// the run (burn-in, a step-size schedule) once launches are long
// (sampler.STEPS_PER_LAUNCH).  Before its first round: `prior`.
struct SpecGuess {
  float a, n;  // recency-weighted accepted / settled steps
  __device__ __forceinline__ explicit SpecGuess(float prior) : a(prior), n(1.f) {}
  // the tree: the grid bucket nearest the estimated acceptance rate
  __device__ __forceinline__ int bucket() const {
#ifdef IPMC_SPEC_REJECT_ONLY  // experiments (tools/build_variant.sh): the reject chain only
    return 0;
#endif
#if IPMC_SPEC_TREE
    const float p = a / n;  // the grid's midpoints in fp32 (any tree is correct; this only picks one)
    int b = 0;
#pragma unroll
    for (int i = 0; i + 1 < kSpecBuckets; ++i) b += p > (float)(0.5 * (kSpecGridP[i] + kSpecGridP[i + 1])) ? 1 : 0;
    return b;
#else
    return 2.f * a >= n ? kSpecBuckets - 1 : 0;
#endif
  }
  __device__ __forceinline__ void settle(int nar, int used) {
#ifdef IPMC_SPEC_GUESS_CUMULATIVE  // experiments: rounds 1-3's whole-launch ratio
    if (fresh) a = n = 0.f;
    fresh = false;
    a += (float)nar;
    n += (float)used;
#else
    a = fmaf(IPMC_SPEC_MEMORY, a, (float)nar);
    n = fmaf(IPMC_SPEC_MEMORY, n, (float)used);
#endif
  }
#ifdef IPMC_SPEC_GUESS_CUMULATIVE
  bool fresh = true;
#endif
};
// The prior at a launch's first round: the chain's acceptance over the steps
// it has counted before the launch (step0 - accepts_step0: a resumed or
// continued run counts from its own first step, not from global step 0); 1
// without any history.
__device__ __forceinline__ float spec_accept_prior(const ipmc_sweep& s, int64_t chain) {
  if (!s.accepts || s.step0 <= s.accepts_step0) return 1.f;
  return (float)s.accepts[chain] / (float)(s.step0 - s.accepts_step0);
}

struct SpecRound {
  int used;   // steps settled by the round
  int nar;    // accepted steps among them
  int win;    // the node whose proposal is the chain's new state (-1: unchanged)
  int calls;  // evaluated (in-box) proposals among them
};
// What the walk needs of node n: its decision, whether its proposal was
// evaluated (ConstrainAccepter) and the next node after a reject / an accept.
struct SpecStep {
  bool acc, ok;
  int next_rej, next_acc;
};
// Walk the round's tree from node 0 along the decisions (node(n) -> SpecStep),
// calling visit(q, la) for every settled step q = 0, 1, ... with la the node
// whose proposal is the state after step st+q (-1: the round's starting
// state).  Stops after `left` steps or at a next node outside the S slots.
template <class Node, class Visit>
__device__ __forceinline__ SpecRound spec_walk(int S, int64_t left, Node&& node, Visit&& visit) {
  SpecRound r{0, 0, -1, 0};
  int n = 0;
  while (true) {
    const SpecStep x = node(n);
    r.calls += x.ok ? 1 : 0;
    if (x.acc) {
      ++r.nar;
      r.win = n;
    }
    visit(r.used, r.win);
    ++r.used;
    const int c = x.acc ? x.next_acc : x.next_rej;
    if (r.used >= left || c < 0 || c >= S) break;
    n = c;
  }
  return r;
}
// The same path again for the recorded states, as a counted loop over the
// `used` steps the walk settled (visit(q, la) as in spec_walk).  Kept apart
// from spec_walk: a cross-lane read of the proposals inside the walk's
// data-dependent loop gave wrong states in the Burgers kernel with two chains
// per wave (tools/probes/spec_tree_debug.py), the counted loop and LDS reads
// do not.
template <class Node, class Visit>
__device__ __forceinline__ void spec_replay(int used, Node&& node, Visit&& visit) {
  int n = 0, la = -1;
  for (int q = 0; q < used; ++q) {
    const SpecStep x = node(n);
    if (x.acc) la = n;
    visit(q, la);
    n = x.acc ? x.next_acc : x.next_rej;
  }
}
// In-wave rounds (S <= 64 slots, one decision bit per slot): the walk
// resolved in parallel.  Every lane computes whether its own node lies on the
// realized path (spec_on_path), a ballot gathers the path, and the path's
// nodes in index order are its steps in order (a child's index exceeds its
// parent's).  `path`, `acc`, `ok` hold one bit per slot (bit n = node n).
__device__ __forceinline__ bool spec_on_path(int tb, int node, unsigned long long acc, bool act) {
  return act && ((acc ^ kSpecTrees.edge[tb][node]) & kSpecTrees.anc[tb][node]) == 0;
}
__device__ __forceinline__ SpecRound spec_path_round(unsigned long long path, unsigned long long acc,
                                                     unsigned long long ok) {
  SpecRound r;
  r.used = __builtin_popcountll(path);
  r.nar = __builtin_popcountll(path & acc);
  r.calls = __builtin_popcountll(path & ok);
  const unsigned long long pa = path & acc;
  r.win = pa ? 63 - __builtin_clzll(pa) : -1;  // the deepest accepted node of the path
  return r;
}
// One bit per slot (bit n = slot n) from a ballot holding slot n's bit at
// n*L (L lanes per slot, S slots, S*L <= 64).
__device__ __forceinline__ unsigned long long spec_slot_bits(unsigned long long m, int S, int L) {
  if (L == 1) return m;
  unsigned long long b = 0;
  for (int n = 0; n < S; ++n) b |= ((m >> (n * L)) & 1ull) << n;
  return b;
}
// visit(q, la) over the path's steps, as spec_walk's
template <class Visit>
__device__ __forceinline__ void spec_path_replay(unsigned long long path, unsigned long long acc, Visit&& visit) {
  int la = -1, q = 0;
  while (path) {
    const int n = __builtin_ctzll(path);
    path &= path - 1;
    if ((acc >> n) & 1ull) la = n;
    visit(q++, la);
  }
}

// Node n's step from the slots' decision bits (bit n*L of acc / ok, L lanes
// per slot) and the tree table.
__device__ __forceinline__ SpecStep spec_step_bits(const SpecNode* tree, int n, int L, unsigned long long acc,
                                                   unsigned long long ok) {
  const SpecNode& x = tree[n];
  return SpecStep{((acc >> (n * L)) & 1ull) != 0, ((ok >> (n * L)) & 1ull) != 0, x.child[0], x.child[1]};
}
__device__ __forceinline__ int spec_pack_children(const SpecNode& x) {
  return (int)(uint16_t)x.child[0] | ((int)x.child[1] << 16);
}
__device__ __forceinline__ SpecStep spec_step_packed(int packed, int n, int L, unsigned long long acc,
                                                     unsigned long long ok) {
  return SpecStep{((acc >> (n * L)) & 1ull) != 0, ((ok >> (n * L)) & 1ull) != 0,
                  (int)(int16_t)(packed & 0xFFFF), packed >> 16};
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
