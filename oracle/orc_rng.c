/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orc_rng.h).
 * Philox4x32-10 and the deterministic log / sincos used by Box–Muller.
 */
#include "orc_rng.h"

#include <math.h>

#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int round = 0; round < 10; ++round) {
    if (round > 0) {
      k0 += PHILOX_W0;
      k1 += PHILOX_W1;
    }
    uint64_t p0 = (uint64_t)PHILOX_M0 * (uint64_t)c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * (uint64_t)c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

static double as_double(uint64_t b) {
  union { uint64_t u; double d; } v;
  v.u = b;
  return v.d;
}
static uint64_t as_bits(double d) {
  union { uint64_t u; double d; } v;
  v.d = d;
  return v.u;
}

/* 2^-53 */
#define TWO_M53 0x1.0p-53

/* log(x) for x in [0, +inf), normal x (and 0 -> -inf). Reduction x = m 2^e,
 * m in (sqrt(1/2), sqrt(2)], s = (m-1)/(m+1), log m = 2 atanh(s) as an odd
 * series in s truncated after s^23 (|s| <= 0.1716, truncation < 1e-18). */
double orc_log(double x) {
  if (x == 0.0) return -INFINITY;
  uint64_t b = as_bits(x);
  int e = (int)((b >> 52) & 0x7ff) - 1023;
  double m = as_double((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
  if (m > 0x1.6a09e667f3bcdp+0) {
    m = m * 0.5;
    e = e + 1;
  }
  double f = m - 1.0;
  double s = f / (2.0 + f);
  double z = s * s;
  double p = 0x1.642c8590b2164p-5; /* 1/23 */
  p = p * z + 0x1.8618618618618p-5; /* 1/21 */
  p = p * z + 0x1.af286bca1af28p-5; /* 1/19 */
  p = p * z + 0x1.e1e1e1e1e1e1ep-5; /* 1/17 */
  p = p * z + 0x1.1111111111111p-4; /* 1/15 */
  p = p * z + 0x1.3b13b13b13b14p-4; /* 1/13 */
  p = p * z + 0x1.745d1745d1746p-4; /* 1/11 */
  p = p * z + 0x1.c71c71c71c71cp-4; /* 1/9 */
  p = p * z + 0x1.2492492492492p-3; /* 1/7 */
  p = p * z + 0x1.999999999999ap-3; /* 1/5 */
  p = p * z + 0x1.5555555555555p-2; /* 1/3 */
  double s2 = s + s;
  double lm = s2 + s2 * (z * p);
  double de = (double)e;
  return de * 0x1.62e42fee00000p-1 + (de * 0x1.a39ef35793c76p-33 + lm);
}

/* sin(2 pi t), cos(2 pi t) for t in [0, 1). Exact quadrant reduction in turns,
 * then Taylor polynomials on |phi| <= pi/4 (truncation < 1e-19). */
void orc_sincos_2pi(double t, double* s_out, double* c_out) {
  double y = t * 4.0;
  int qi = (int)y;
  double r = y - (double)qi;
  if (r > 0.5) {
    r = r - 1.0;
    qi = qi + 1;
  }
  double phi = r * 0x1.921fb54442d18p+0; /* pi/2 */
  double z = phi * phi;
  double ps = 0x1.952c77030ad4ap-49; /* +1/17! */
  ps = ps * z + -0x1.ae7f3e733b81fp-41; /* -1/15! */
  ps = ps * z + 0x1.6124613a86d09p-33;  /* +1/13! */
  ps = ps * z + -0x1.ae64567f544e4p-26; /* -1/11! */
  ps = ps * z + 0x1.71de3a556c734p-19;  /* +1/9! */
  ps = ps * z + -0x1.a01a01a01a01ap-13; /* -1/7! */
  ps = ps * z + 0x1.1111111111111p-7;   /* +1/5! */
  ps = ps * z + -0x1.5555555555555p-3;  /* -1/3! */
  double sv = phi + phi * (z * ps);
  double pc = -0x1.6827863b97d97p-53; /* -1/18! */
  pc = pc * z + 0x1.ae7f3e733b81fp-45;  /* +1/16! */
  pc = pc * z + -0x1.93974a8c07c9dp-37; /* -1/14! */
  pc = pc * z + 0x1.1eed8eff8d898p-29;  /* +1/12! */
  pc = pc * z + -0x1.27e4fb7789f5cp-22; /* -1/10! */
  pc = pc * z + 0x1.a01a01a01a01ap-16;  /* +1/8! */
  pc = pc * z + -0x1.6c16c16c16c17p-10; /* -1/6! */
  pc = pc * z + 0x1.5555555555555p-5;   /* +1/4! */
  pc = pc * z + -0x1.0000000000000p-1;  /* -1/2! */
  double cv = 1.0 + z * pc;
  switch (qi & 3) {
    case 0: *s_out = sv;  *c_out = cv;  break;
    case 1: *s_out = cv;  *c_out = -sv; break;
    case 2: *s_out = -sv; *c_out = -cv; break;
    default: *s_out = -cv; *c_out = sv; break;
  }
}

static void philox_draw(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot, uint32_t o[4]) {
  uint32_t ctr[4] = {slot, (uint32_t)chain, (uint32_t)step, (uint32_t)(step >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  orc_philox4x32_10(ctr, key, o);
}

void orc_normal_pair(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot, double z[2]) {
  uint32_t o[4];
  philox_draw(seed, chain, step, slot, o);
  uint64_t a = ((((uint64_t)o[0] << 32) | o[1]) >> 11) + 1; /* (0, 2^53] */
  uint64_t b = (((uint64_t)o[2] << 32) | o[3]) >> 11;       /* [0, 2^53) */
  double u1 = (double)a * TWO_M53;
  double u2 = (double)b * TWO_M53;
  double rad = sqrt(-2.0 * orc_log(u1));
  double sv, cv;
  orc_sincos_2pi(u2, &sv, &cv);
  z[0] = rad * cv;
  z[1] = rad * sv;
}

double orc_normal(uint64_t seed, uint64_t chain, uint64_t step, uint32_t comp) {
  double z[2];
  orc_normal_pair(seed, chain, step, comp >> 1, z);
  return z[comp & 1];
}

double orc_accept_uniform(uint64_t seed, uint64_t chain, uint64_t step) {
  uint32_t o[4];
  philox_draw(seed, chain, step, 0xFFFFFFFFu, o);
  uint64_t a = (((uint64_t)o[0] << 32) | o[1]) >> 11;
  return (double)a * TWO_M53;
}
