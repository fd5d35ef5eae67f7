// Device building blocks for the pCN sweep kernels (gfx950 / CDNA4).
//
//  * the counter-based draws (Philox4x32-10, deterministic log / sincos,
//    Box–Muller) come from ipmc_rng.hpp, compiled for host and device.
//  * Cross-lane halo exchange for chains spread over 2/4 lanes (DPP quad_perm,
//    no LDS traffic) or 8/16 lanes (ds_bpermute).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ipmc_rng.hpp"

namespace ipmc {

// LDS per CU on gfx950 (MI355X): the static LDS of any block must fit this.
constexpr size_t kLdsBytesPerCU = 160 * 1024;

// Philox draws, deterministic log / sincos, Box–Muller and the proposal
// noise element: ipmc_rng.hpp (shared with the host library).

// ------------------------------------------------------------- arithmetic
// madd<FMA>(a, b, c) = c + a*b, fused (one rounding) or not (two roundings).
template <bool FM>
__device__ __forceinline__ float madd(float a, float b, float c) {
  if constexpr (FM) return __builtin_fmaf(a, b, c);
  else return c + a * b;
}
template <bool FM>
__device__ __forceinline__ double madd(double a, double b, double c) {
  if constexpr (FM) return __builtin_fma(a, b, c);
  else return c + a * b;
}

// ------------------------------------------------------------- cross-lane
// DPP quad_perm control words (lane i of each quad reads lane sel_i).
constexpr int qperm(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) { return dpp_f32<CTRL>(v); }
template <int CTRL>
__device__ __forceinline__ double dpp(double v) { return dpp_f64<CTRL>(v); }

// Two fp32 chains packed per lane (x = chain 2p, y = chain 2p+1): every
// arithmetic op is a v_pk_*_f32 with per-component IEEE semantics, i.e. the
// same bits as two scalar evaluations.
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <bool FM>
__device__ __forceinline__ f32x2 madd(f32x2 a, f32x2 b, f32x2 c) {
  if constexpr (FM) return __builtin_elementwise_fma(a, b, c);
  else return c + a * b;
}
template <int CTRL>
__device__ __forceinline__ f32x2 dpp(f32x2 v) {
  f32x2 r;
  r.x = dpp_f32<CTRL>(v.x);
  r.y = dpp_f32<CTRL>(v.y);
  return r;
}

__device__ __forceinline__ float shfl(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ double shfl(double v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ f32x2 shfl(f32x2 v, int src) {
  f32x2 r;
  r.x = __shfl(v.x, src, 64);
  r.y = __shfl(v.y, src, 64);
  return r;
}

// scalar -> storage type (splat for packed pairs)
template <typename V>
struct Splat {
  template <typename S>
  __device__ static __forceinline__ V of(S s) { return (V)s; }
};
template <>
struct Splat<f32x2> {
  __device__ static __forceinline__ f32x2 of(float s) { return f32x2{s, s}; }
};

// Value of `v` held by the previous / next lane of this chain's lane group
// (cyclic inside the group of LPC lanes; groups are LPC-aligned).
// DPP row rotations (rows of 16 lanes): row_ror:1 makes lane i read lane
// (i-1) mod 16 of its row, row_ror:15 lane (i+1) mod 16.
constexpr int kRowRor1 = 0x121;
constexpr int kRowRor15 = 0x12F;

// (DPP movs take VALU issue slots -- 24 of the 224 instructions of a d=40
// RK4 step at LPC 4 -- but moving these halos to ds_bpermute measured 10 %
// slower: profiles/r1/halo_dpp_vs_lds.txt.)
// Half rows (LPC 8) have no rotation of their own: lane i reads lane i-1
// (row_shr:1) except at the half's first lane, which reads the half's last
// (row_shl:7), and the select is one v_cndmask per dword -- three VALU ops
// instead of a ds_bpermute round trip, whose latency one wave per SIMD (the
// 8 192-chain ensemble on 8 lanes) cannot hide.
constexpr int kRowShl1 = 0x101;
constexpr int kRowShl7 = 0x107;
constexpr int kRowShr1 = 0x111;
constexpr int kRowShr7 = 0x117;
constexpr int kRowRor2 = 0x122;
constexpr int kRowRor14 = 0x12E;

// Interleaved groups of 8 (IL; the sequential Lorenz-96 kernels): each row of
// 16 lanes holds two chains, one on its even lanes and one on its odd lanes,
// so a DPP row rotation by 2 is a halo move for both -- one VALU op per dword,
// as for LPC 16.  The lane's place in its group follows from the virtual
// thread index group_vlane(t): chain = vt / 8, sub = vt % 8.
template <int LPC, bool IL>
__device__ __forceinline__ int group_vlane(int t) {
  if constexpr (IL && LPC == 8) return (t & ~15) | ((t & 1) << 3) | ((t >> 1) & 7);
  else return t;
}

template <int LPC, bool IL = false, typename T>
__device__ __forceinline__ T group_prev(T v, int lane) {
  if constexpr (LPC == 1) return v;
  else if constexpr (LPC == 2) return dpp<qperm(1, 0, 3, 2)>(v);
  else if constexpr (LPC == 4) return dpp<qperm(3, 0, 1, 2)>(v);
  else if constexpr (LPC == 8 && IL) return dpp<kRowRor2>(v);
  else if constexpr (LPC == 8) {
    const T a = dpp<kRowShr1>(v), b = dpp<kRowShl7>(v);
    return (lane & 7) == 0 ? b : a;
  } else if constexpr (LPC == 16) return dpp<kRowRor1>(v);
  else return shfl(v, (lane & ~(LPC - 1)) | ((lane - 1) & (LPC - 1)));
}
template <int LPC, bool IL = false, typename T>
__device__ __forceinline__ T group_next(T v, int lane) {
  if constexpr (LPC == 1) return v;
  else if constexpr (LPC == 2) return dpp<qperm(1, 0, 3, 2)>(v);
  else if constexpr (LPC == 4) return dpp<qperm(1, 2, 3, 0)>(v);
  else if constexpr (LPC == 8 && IL) return dpp<kRowRor14>(v);
  else if constexpr (LPC == 8) {
    const T a = dpp<kRowShl1>(v), b = dpp<kRowShr7>(v);
    return (lane & 7) == 7 ? b : a;
  } else if constexpr (LPC == 16) return dpp<kRowRor15>(v);
  else return shfl(v, (lane & ~(LPC - 1)) | ((lane + 1) & (LPC - 1)));
}
// Value of `v` held by lane `s` of this chain's group.
template <int LPC, int S, bool IL = false, typename T>
__device__ __forceinline__ T group_bcast(T v, int lane) {
  if constexpr (LPC == 1) return v;
  else if constexpr (LPC <= 4) {
    // within a quad: group base lane b = (i & ~(LPC-1)); source = b + S
    if constexpr (LPC == 2) return dpp<qperm(S, S, 2 + S, 2 + S)>(v);
    else return dpp<qperm(S, S, S, S)>(v);
  } else if constexpr (LPC == 8 && IL) {
    return shfl(v, (lane & ~15) | (S << 1) | (lane & 1));
  } else {
    return shfl(v, (lane & ~(LPC - 1)) | S);
  }
}

// LDS written by lanes of this wavefront is visible to the whole wavefront.
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// All lanes of the group hold `ok`: true iff every lane's ok is true.
template <int LPC, bool IL = false>
__device__ __forceinline__ bool group_all(bool ok, int lane) {
  if constexpr (LPC == 1) return ok;
  const unsigned long long m = __ballot(ok);
  if constexpr (LPC == 8 && IL) {  // this chain's lanes: every other lane of the row
    const unsigned long long g = (m >> (lane & ~15)) & (0x5555ull << (lane & 1));
    return g == (0x5555ull << (lane & 1));
  }
  const unsigned long long g = (m >> (lane & ~(LPC - 1))) & ((1ull << LPC) - 1);
  return g == ((1ull << LPC) - 1);
}

}  // namespace ipmc
