// Device building blocks for the pCN sweep kernels (gfx950 / CDNA4).
//
//  * Philox4x32-10 counter-based RNG: ctr = (slot, chain, step_lo, step_hi),
//    key = (seed_lo, seed_hi). slot j -> normal pair (2j, 2j+1) of the
//    proposal (proposer.py:81-82's w ~ N(0, C)), slot 0xFFFFFFFF -> the accept
//    uniform (accepter.py:62's rng.random()).
//  * Deterministic log / sincos(2*pi*t) built from + - * / in a fixed order,
//    so every draw is bit-identical to the CPU oracle.
//  * Cross-lane halo exchange for chains spread over 2/4 lanes (DPP quad_perm,
//    no LDS traffic) or 8/16 lanes (ds_bpermute).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ipmc {

// LDS per CU on gfx950 (MI355X): the static LDS of any block must fit this.
constexpr size_t kLdsBytesPerCU = 160 * 1024;

// ---------------------------------------------------------------- Philox
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += W0;
      k1 += W1;
    }
    const uint32_t lo0 = M0 * c0, hi0 = __umulhi(M0, c0);
    const uint32_t lo1 = M1 * c2, hi1 = __umulhi(M1, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return {c0, c1, c2, c3};
}

__device__ __forceinline__ u32x4 philox_draw(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot) {
  return philox4x32_10(slot, (uint32_t)chain, (uint32_t)step, (uint32_t)(step >> 32), (uint32_t)seed,
                       (uint32_t)(seed >> 32));
}

// ------------------------------------------------------ deterministic math
// Bit-identical to oracle/orc_rng.c (same constants, same operation order;
// compiled with -ffp-contract=off so no operation is fused).
__device__ __forceinline__ double det_log(double x) {
  if (x == 0.0) return -__builtin_inf();
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  int e = (int)((b >> 52) & 0x7ff) - 1023;
  double m = __longlong_as_double((long long)((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull));
  if (m > 0x1.6a09e667f3bcdp+0) {
    m = m * 0.5;
    e = e + 1;
  }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double p = 0x1.642c8590b2164p-5;
  p = p * z + 0x1.8618618618618p-5;
  p = p * z + 0x1.af286bca1af28p-5;
  p = p * z + 0x1.e1e1e1e1e1e1ep-5;
  p = p * z + 0x1.1111111111111p-4;
  p = p * z + 0x1.3b13b13b13b14p-4;
  p = p * z + 0x1.745d1745d1746p-4;
  p = p * z + 0x1.c71c71c71c71cp-4;
  p = p * z + 0x1.2492492492492p-3;
  p = p * z + 0x1.999999999999ap-3;
  p = p * z + 0x1.5555555555555p-2;
  const double s2 = s + s;
  const double lm = s2 + s2 * (z * p);
  const double de = (double)e;
  return de * 0x1.62e42fee00000p-1 + (de * 0x1.a39ef35793c76p-33 + lm);
}

__device__ __forceinline__ void det_sincos_2pi(double t, double& so, double& co) {
  const double y = t * 4.0;
  int qi = (int)y;
  double r = y - (double)qi;
  if (r > 0.5) {
    r = r - 1.0;
    qi = qi + 1;
  }
  const double phi = r * 0x1.921fb54442d18p+0;
  const double z = phi * phi;
  double ps = 0x1.952c77030ad4ap-49;
  ps = ps * z + -0x1.ae7f3e733b81fp-41;
  ps = ps * z + 0x1.6124613a86d09p-33;
  ps = ps * z + -0x1.ae64567f544e4p-26;
  ps = ps * z + 0x1.71de3a556c734p-19;
  ps = ps * z + -0x1.a01a01a01a01ap-13;
  ps = ps * z + 0x1.1111111111111p-7;
  ps = ps * z + -0x1.5555555555555p-3;
  const double sv = phi + phi * (z * ps);
  double pc = -0x1.6827863b97d97p-53;
  pc = pc * z + 0x1.ae7f3e733b81fp-45;
  pc = pc * z + -0x1.93974a8c07c9dp-37;
  pc = pc * z + 0x1.1eed8eff8d898p-29;
  pc = pc * z + -0x1.27e4fb7789f5cp-22;
  pc = pc * z + 0x1.a01a01a01a01ap-16;
  pc = pc * z + -0x1.6c16c16c16c17p-10;
  pc = pc * z + 0x1.5555555555555p-5;
  pc = pc * z + -0x1.0000000000000p-1;
  const double cv = 1.0 + z * pc;
  switch (qi & 3) {
    case 0: so = sv;  co = cv;  break;
    case 1: so = cv;  co = -sv; break;
    case 2: so = -sv; co = -cv; break;
    default: so = -cv; co = sv; break;
  }
}

// Box–Muller pair for components (2*slot, 2*slot+1).
__device__ __forceinline__ void normal_pair(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot,
                                            double& z0, double& z1) {
  const u32x4 o = philox_draw(seed, chain, step, slot);
  const uint64_t a = ((((uint64_t)o.x << 32) | o.y) >> 11) + 1;
  const uint64_t b = (((uint64_t)o.z << 32) | o.w) >> 11;
  const double u1 = (double)a * 0x1.0p-53;
  const double u2 = (double)b * 0x1.0p-53;
  const double rad = __builtin_sqrt(-2.0 * det_log(u1));
  double sv, cv;
  det_sincos_2pi(u2, sv, cv);
  z0 = rad * cv;
  z1 = rad * sv;
}

__device__ __forceinline__ double accept_uniform(uint64_t seed, uint64_t chain, uint64_t step) {
  const u32x4 o = philox_draw(seed, chain, step, 0xFFFFFFFFu);
  const uint64_t a = (((uint64_t)o.x << 32) | o.y) >> 11;
  return (double)a * 0x1.0p-53;
}

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
