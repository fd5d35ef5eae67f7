// Counter-based draws of the pCN path, compiled for the device (every sweep
// kernel, hipcc) AND for the host (libipmc_host.so, g++): one source, so the
// host library's draws are the kernels' bits by construction.
//
//  * Philox4x32-10 (Random123): ctr = (slot, chain, step_lo, step_hi),
//    key = (seed_lo, seed_hi).  slot j -> normal pair (2j, 2j+1) of the
//    proposal (proposer.py:81-82's w ~ N(0, C)), slot 0xFFFFFFFF -> the accept
//    uniform (accepter.py:62's rng.random()).
//  * Deterministic log / sincos(2*pi*t) built from + - * / in a fixed order
//    (IEEE sqrt and division only), bit-identical to oracle/orc_rng.c
//    (DESIGN.md §4).  Both compilers run with -ffp-contract=off, so nothing is
//    fused.
//  * draw_w: one component of a step's proposal noise, sqrt(C_jj)·ξ_j or
//    Σ_{i<=j} L_ji ξ_i (chol_noise's order) -- ipmc_pcn_draws' element.
#pragma once

#include <stdint.h>

#ifdef __HIP__
#define IPMC_HD __host__ __device__ __forceinline__
#else
#define IPMC_HD inline __attribute__((always_inline))
#endif

namespace ipmc {

struct u32x4 {
  uint32_t x, y, z, w;
};

IPMC_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

IPMC_HD u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += W0;
      k1 += W1;
    }
    const uint32_t lo0 = M0 * c0, hi0 = mulhi32(M0, c0);
    const uint32_t lo1 = M1 * c2, hi1 = mulhi32(M1, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return {c0, c1, c2, c3};
}

IPMC_HD u32x4 philox_draw(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot) {
  return philox4x32_10(slot, (uint32_t)chain, (uint32_t)step, (uint32_t)(step >> 32), (uint32_t)seed,
                       (uint32_t)(seed >> 32));
}

IPMC_HD double det_log(double x) {
  if (x == 0.0) return -__builtin_inf();
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  int e = (int)((b >> 52) & 0x7ff) - 1023;
  double m = __builtin_bit_cast(double, (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
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

IPMC_HD void det_sincos_2pi(double t, double& so, double& co) {
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
IPMC_HD void normal_pair(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot, double& z0, double& z1) {
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

// The standard normal ξ_j of (chain, step) in f64.
IPMC_HD double normal_component(uint64_t seed, uint64_t chain, uint64_t step, int j) {
  double z0, z1;
  normal_pair(seed, chain, step, (uint32_t)(j >> 1), z0, z1);
  return (j & 1) ? z1 : z0;
}

// A 53-bit uniform in [0, 1) from Philox slot `slot`.
IPMC_HD double slot_uniform(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot) {
  const u32x4 o = philox_draw(seed, chain, step, slot);
  const uint64_t a = (((uint64_t)o.x << 32) | o.y) >> 11;
  return (double)a * 0x1.0p-53;
}

// The accept uniform r of (chain, step): slot 0xFFFFFFFF.
IPMC_HD double accept_uniform(uint64_t seed, uint64_t chain, uint64_t step) {
  return slot_uniform(seed, chain, step, 0xFFFFFFFFu);
}

// Component j of the proposal noise w of (chain gid, step): sqrt(C_jj)·ξ_j
// for a diagonal prior (sq), else Σ_{i<=j} L_ji ξ_i summed in ascending i
// from +0 with no FMA (chol_noise / oracle/orc_models.inc: the same order),
// in the chain dtype T.
template <typename T>
IPMC_HD T draw_w(uint64_t seed, uint64_t gid, uint64_t step, int j, int k, const T* sq, const T* chol) {
  double z0, z1;
  if (chol) {
    T wj = (T)0;
    for (int ii = 0; ii <= j; ii += 2) {
      normal_pair(seed, gid, step, (uint32_t)(ii >> 1), z0, z1);
      wj = wj + (T)z0 * chol[(int64_t)j * k + ii];
      if (ii + 1 <= j) wj = wj + (T)z1 * chol[(int64_t)j * k + ii + 1];
    }
    return wj;
  }
  normal_pair(seed, gid, step, (uint32_t)(j >> 1), z0, z1);
  return sq[j] * (T)((j & 1) ? z1 : z0);
}

}  // namespace ipmc
