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
#define FMAX(a, b) fmax((a), (b))
#define FABS(a) fabs(a)
#include "orc_models.inc"
#undef REAL
#undef SFX
#undef FMA
#undef FMAX
#undef FABS

#define REAL float
#define SFX(n) n##_f32
#define FMA(a, b, c) fmaf((a), (b), (c))
#define FMAX(a, b) fmaxf((a), (b))
#define FABS(a) fabsf(a)
#include "orc_models.inc"
#undef REAL
#undef SFX
#undef FMA
#undef FMAX
#undef FABS

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
  if (!s || !s->u || !s->phi || !s->y || !s->gamma_inv || (!s->prior_sqrt && !s->prior_chol)) return IPMC_ERR_INVALID;
  if (s->proposal == IPMC_PROPOSAL_PCN && !(s->beta >= 0.0 && s->beta <= 1.0)) return IPMC_ERR_INVALID;
  if (s->sample_every < 0 || (s->sample_every > 0 && (!s->sample_out || s->sample_step_stride < m->k)))
    return IPMC_ERR_INVALID;
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

/* numpy pairwise_sum (loops_utils.h.src) for any n, recursive as numpy's. */
static double np_pairwise_any(const double* a, int64_t n) {
  if (n <= 128) return np_pairwise_f64(a, (int)n);
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise_any(a, n2) + np_pairwise_any(a + n2, n - n2);
}

/* len_burn_in (report/scripts/burgers/utilities.py:134-167) for C chains of
 * contiguous (n_vars, len) f64 blocks: moving_avg via np.cumsum
 * (:139-142), means via np.mean (:155), changed flags (:156-159), search
 * from the end (:162-165).  Returns 0, or -1 if len < window. */
int orc_burn_in(const double* x, int64_t n_chains, int32_t n_vars, int64_t len, int32_t w, double thr,
                int64_t* out) {
  if (len < w || w <= 0) return -1;
  const int64_t n_avgs = len - w + 1, L = n_avgs - 1;
  double* cs = (double*)malloc(sizeof(double) * (size_t)len);
  double* avgs = (double*)malloc(sizeof(double) * (size_t)(n_vars * n_avgs));
  double* means = (double*)malloc(sizeof(double) * (size_t)n_vars);
  unsigned char* ch = (unsigned char*)malloc((size_t)(L > 0 ? L : 1));
  for (int64_t c = 0; c < n_chains; ++c) {
    const double* xc = x + c * n_vars * len;
    for (int v = 0; v < n_vars; ++v) {
      const double* y = xc + v * len;
      cs[0] = y[0];
      for (int64_t t = 1; t < len; ++t) cs[t] = cs[t - 1] + y[t];
      double* av = avgs + v * n_avgs;
      av[0] = cs[w - 1] / (double)w;
      for (int64_t j = 1; j < n_avgs; ++j) av[j] = (cs[j + w - 1] - cs[j - 1]) / (double)w;
      means[v] = np_pairwise_any(y, len) / (double)len;
    }
    for (int64_t i = 0; i < L; ++i) {
      int any = 0;
      for (int v = 0; v < n_vars && !any; ++v) {
        const double* av = avgs + v * n_avgs;
        any = fabs((av[i] - av[i + 1]) / means[v]) > thr;
      }
      ch[i] = (unsigned char)any;
    }
    int64_t res = len - 1;
    for (int64_t i = L - w - 2; i > 0; --i) {
      int all = 1;
      for (int64_t j = i; j < i + w + 1 && all; ++j) all = ch[j];
      if (all) {
        res = i;
        break;
      }
    }
    out[c] = res;
  }
  free(cs);
  free(avgs);
  free(means);
  free(ch);
  return 0;
}

/* Two-scale Lorenz-96 right-hand side (lorenz.py:44-101), fp64; p = (F, h, c, b). */
void orc_l96ts_rhs_f64(int32_t arith, int32_t K, int32_t J, const double* x, const double* p, double* out) {
  const double hc = p[1] * p[2], hJ = p[1] / (double)J;
  l96ts_rhs_f64(arith == IPMC_ARITH_FMA, K, J, p[0], hc, hJ, p[3], p[2], x, out);
}

/* Rusanov pieces for the rusanov.py:112-170 known-answer tests. */
/* FMA arith: the kernels' F2 flux and rate, in the reference's units
 * (F = F2/4, dudt = c1 (F2_{i+1/2} - F2_{i-1/2})). */
double orc_rusanov_flux_f64(int32_t arith, double a, double b) {
  if (arith != IPMC_ARITH_FMA) return rus_flux_f64(a, b);
  return 0.25 * fma(fmax(fabs(a + a), fabs(b + b)), a - b, a * a + b * b); /* rus_rate_f2 */
}
void orc_rusanov_rate_f64(int32_t arith, int32_t N, const double* w, double dx, double* r) {
  if (arith != IPMC_ARITH_FMA) {
    rus_rate_f64(N, w, -dx, 0.0, 0, r);
    return;
  }
  const double c1 = 0.25 * (1.0 / -dx);
  rus_rate_f2_f64(N, w, 0, 0.0, r);
  for (int i = 1; i <= N; ++i) r[i] = c1 * r[i];
}


int orc_abi_version(void) { return IPMC_ABI_VERSION; }
