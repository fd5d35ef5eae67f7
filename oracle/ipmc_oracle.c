/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's pCN hot path (ochsnerd/ip_mcmc,
 * sampler.py / proposer.py / accepter.py / potential.py + the forward maps of
 * report/scripts) over many independent chains, on HOST pointers, with the
 * same structs as include/ipmc.h.  It is the parity checker for libipmc.so and
 * the "port" CPU baseline of bench.py; the product path never loads it.
 *
 * Pinned against the reference by tests/test_oracle_golden.py (fixtures made
 * by tests/golden/make_golden.py from the reference itself).
 *
 * Build: oracle/Makefile  ->  oracle/_build/liboracle.so
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/ipmc.h"
#include "orc_rng.h"

#define REAL double
#define SFX(n) n##_f64
#define FMA(a, b, c) fma((a), (b), (c))
#include "orc_models.inc"
#undef REAL
#undef SFX
#undef FMA

#define REAL float
#define SFX(n) n##_f32
#define FMA(a, b, c) fmaf((a), (b), (c))
#include "orc_models.inc"
#undef REAL
#undef SFX
#undef FMA

static int check_model(const ipmc_model* m) {
  if (!m || m->k <= 0 || m->q <= 0) return IPMC_ERR_INVALID;
  switch (m->kind) {
    case IPMC_MODEL_LINEAR: return (m->A && m->theta0) ? IPMC_OK : IPMC_ERR_INVALID;
    case IPMC_MODEL_LORENZ63:
      return (m->k == 3 && m->q == 6 && m->x0 && m->theta0 && m->n_steps > 0) ? IPMC_OK : IPMC_ERR_INVALID;
    case IPMC_MODEL_LORENZ96:
      return (m->dim == m->k && m->q == m->dim && m->x0 && m->theta0 && m->n_steps > 0) ? IPMC_OK
                                                                                       : IPMC_ERR_INVALID;
    case IPMC_MODEL_LORENZ96_2S:
      return (m->k == 3 && m->dim > 0 && m->fast_per_slow > 0 && m->q == 5 * m->dim && m->x0 && m->theta0 &&
              m->n_steps > 0)
                 ? IPMC_OK
                 : IPMC_ERR_INVALID;
    case IPMC_MODEL_BURGERS:
      return (m->k == 3 && m->q == m->n_windows && m->x0 && m->theta0 && m->win_lo && m->win_hi && m->dim > 1)
                 ? IPMC_OK
                 : IPMC_ERR_INVALID;
    default: return IPMC_ERR_UNSUPPORTED;
  }
}

int orc_forward(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, void* g) {
  int st = check_model(m);
  if (st) return st;
  if (dtype == IPMC_F64) return forward_f64(m, n, (const double*)u, (double*)g);
  if (dtype == IPMC_F32) return forward_f32(m, n, (const float*)u, (float*)g);
  return IPMC_ERR_INVALID;
}

int orc_potential(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, const void* y,
                  const void* ginv, void* phi) {
  int st = check_model(m);
  if (st) return st;
  if (dtype == IPMC_F64)
    return potential_f64(m, n, (const double*)u, (const double*)y, (const double*)ginv, (double*)phi);
  if (dtype == IPMC_F32)
    return potential_f32(m, n, (const float*)u, (const float*)y, (const float*)ginv, (float*)phi);
  return IPMC_ERR_INVALID;
}

/* n_threads <= 1: serial.  Chains are split into contiguous blocks. */
int orc_pcn_sweep(const ipmc_model* m, const ipmc_sweep* s, int32_t n_threads) {
  int st = check_model(m);
  if (st) return st;
  if (!s || !s->u || !s->phi || !s->y || !s->gamma_inv || !s->prior_sqrt) return IPMC_ERR_INVALID;
  if (s->proposal == IPMC_PROPOSAL_PCN && !(s->beta >= 0.0 && s->beta <= 1.0)) return IPMC_ERR_INVALID;
  const int64_t C = s->n_chains;
  if (n_threads < 1) n_threads = 1;
#pragma omp parallel for num_threads(n_threads) schedule(static)
  for (int64_t t = 0; t < n_threads; ++t) {
    int64_t b = C * t / n_threads, e = C * (t + 1) / n_threads;
    if (s->dtype == IPMC_F64)
      sweep_range_f64(m, s, b, e);
    else
      sweep_range_f32(m, s, b, e);
  }
  return IPMC_OK;
}

int orc_init_phi(const ipmc_model* m, const ipmc_sweep* s) {
  int st = check_model(m);
  if (st) return st;
  return s->dtype == IPMC_F64 ? init_phi_f64(m, s) : init_phi_f32(m, s);
}

void orc_normal_batch(uint64_t seed, int64_t chain_offset, int64_t n, uint64_t step, int32_t k, double* out) {
  for (int64_t c = 0; c < n; ++c)
    for (int32_t i = 0; i < k; ++i)
      out[c * k + i] = orc_normal(seed, (uint64_t)(chain_offset + c), step, (uint32_t)i);
}

void orc_uniform_batch(uint64_t seed, int64_t chain_offset, int64_t n, uint64_t step, double* out) {
  for (int64_t c = 0; c < n; ++c) out[c] = orc_accept_uniform(seed, (uint64_t)(chain_offset + c), step);
}

void orc_log_batch(int64_t n, const double* x, double* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = orc_log(x[i]);
}

void orc_sincos_batch(int64_t n, const double* t, double* s, double* c) {
  for (int64_t i = 0; i < n; ++i) orc_sincos_2pi(t[i], &s[i], &c[i]);
}

/* Lorenz-96 right-hand side (for the lorenz.py:114-171 known-answer tests and
 * the RHS fixtures), fp64, either arithmetic. */
void orc_l96_rhs_f64(int32_t arith, int32_t d, const double* x, const double* F, double* out) {
  l96_rhs_f64(arith == IPMC_ARITH_FMA, d, x, F, out);
}

/* Two-scale Lorenz-96 right-hand side (lorenz.py:44-101), fp64; p = (F, h, c, b). */
void orc_l96ts_rhs_f64(int32_t arith, int32_t K, int32_t J, const double* x, const double* p, double* out) {
  const double hc = p[1] * p[2], hJ = p[1] / (double)J;
  l96ts_rhs_f64(arith == IPMC_ARITH_FMA, K, J, p[0], hc, hJ, p[3], p[2], x, out);
}

/* Rusanov pieces for the rusanov.py:112-170 known-answer tests. */
double orc_rusanov_flux_f64(int32_t arith, double a, double b) {
  return rus_flux_f64(arith == IPMC_ARITH_FMA, a, b);
}
void orc_rusanov_rate_f64(int32_t arith, int32_t N, const double* w, double dx, double* r) {
  rus_rate_f64(arith == IPMC_ARITH_FMA, N, w, -dx, 0.0, 0, r);
}


int orc_abi_version(void) { return IPMC_ABI_VERSION; }
