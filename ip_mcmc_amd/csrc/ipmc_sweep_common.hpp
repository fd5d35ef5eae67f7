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

// v = contraction*u + beta*(sqrt(C_ii) * xi_i)     (proposer.py:81-82; the
// expression order of the reference: two products, then the sum, no FMA)
template <typename T, int M>
__device__ __forceinline__ void pcn_propose(const T* __restrict__ u, const T* __restrict__ sq, T contr, T beta,
                                            uint64_t seed, uint64_t gid, uint64_t step, int c0, T (&v)[M]) {
  if constexpr (M % 2 == 0) {
    // c0 is even whenever M is even: pairs never straddle lanes
#pragma unroll
    for (int j = 0; j < M; j += 2) {
      double z0, z1;
      normal_pair(seed, gid, step, (uint32_t)((c0 + j) >> 1), z0, z1);
      const T w0 = sq[j] * (T)z0;
      const T w1 = sq[j + 1] * (T)z1;
      v[j] = contr * u[j] + beta * w0;
      v[j + 1] = contr * u[j + 1] + beta * w1;
    }
  } else {
    double z0 = 0.0, z1 = 0.0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int c = c0 + j;
      if (j == 0 || (c & 1) == 0) normal_pair(seed, gid, step, (uint32_t)(c >> 1), z0, z1);
      const T w = sq[j] * (T)((c & 1) ? z1 : z0);
      v[j] = contr * u[j] + beta * w;
    }
  }
}

// s = Σ_i r_i^2 over the chain's q = LPC*M residuals in component order
// (lane 0's M values, then lane 1's, ...), identical on every lane of the group.
template <typename T, int M, int LPC, bool FM, int S = 0>
__device__ __forceinline__ T ordered_sumsq(const T (&r)[M], int lane, T s) {
  if constexpr (S == LPC) {
    return s;
  } else {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const T x = group_bcast<LPC, S>(r[j], lane);
      s = madd<FM>(x, x, s);
    }
    return ordered_sumsq<T, M, LPC, FM, S + 1>(r, lane, s);
  }
}

// ConstrainAccepter box: lo < v + off < hi for every component of the chain.
template <typename T, int M, int LPC>
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
  return group_all<LPC>(ok, lane);
}

// accept iff Φ(u) − Φ(v) > log r   ⇔ exp(Φ(u) − Φ(v)) > r   (accepter.py:62, 121-122)
template <typename T>
__device__ __forceinline__ bool pcn_accept(T phu, T phv, uint64_t seed, uint64_t gid, uint64_t step) {
  const double r = accept_uniform(seed, gid, step);
  return (double)(phu - phv) > det_log(r);
}

}  // namespace ipmc
