/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Host sanitizer run of the CPU restatement (sanitizers on host
 * code).  Built with -fsanitize=address,undefined by `make -C oracle asan`
 * and run by tests/test_oracle_sanitized.py: every model's forward map and
 * potential in both dtypes and arithmetic modes, pCN and RW sweeps with the
 * box constraint, schedules, sums and regularizer, init_phi and len_burn_in,
 * on small ragged shapes.  Exit status 0 and no sanitizer report is the pass.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ipmc.h"

int orc_forward(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, void* g);
int orc_potential(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, const void* y, const void* ginv,
                  void* phi);
int orc_pcn_sweep(const ipmc_model* m, const ipmc_sweep* s, int32_t n_threads);
int orc_init_phi(const ipmc_model* m, const ipmc_sweep* s);
int orc_burn_in(const double* x, int64_t n_chains, int32_t n_vars, int64_t len, int32_t w, double thr,
                int64_t* out);

static uint64_t rs = 88172645463325252ull;
static double rnd(void) { /* xorshift64, uniform [-1, 1) */
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (double)(rs >> 11) * 0x1.0p-52 - 1.0;
}

/* a real array of n values in the requested dtype (heap, exact size) */
static void* arr(int32_t dtype, int64_t n, double scale, double shift) {
  void* p = malloc((size_t)(n > 0 ? n : 1) * (dtype == IPMC_F64 ? 8 : 4));
  for (int64_t i = 0; i < n; ++i) {
    const double v = shift + scale * rnd();
    if (dtype == IPMC_F64) ((double*)p)[i] = v;
    else ((float*)p)[i] = (float)v;
  }
  return p;
}

static void cfree(const void* p) { free((void*)p); }

static int failures = 0;
#define CHECK(expr)                                                          \
  do {                                                                       \
    int rc_ = (expr);                                                        \
    if (rc_ != IPMC_OK) {                                                    \
      fprintf(stderr, "FAIL %s:%d rc=%d: %s\n", __FILE__, __LINE__, rc_, #expr); \
      ++failures;                                                            \
    }                                                                        \
  } while (0)

static void run_model(ipmc_model* m, int32_t dtype, int64_t C, int proposal, int with_reg) {
  const int k = m->k, q = m->q;
  void* u = arr(dtype, C * k, 0.2, 0.0);
  void* y = arr(dtype, q, 0.5, 1.0);
  void* gi = arr(dtype, q, 0.5, 5.0);
  void* g = arr(dtype, C * q, 0.0, 0.0);
  void* phi = arr(dtype, C, 0.0, 0.0);
  void* sq = arr(dtype, k, 0.3, 1.0);
  void* lo = arr(dtype, k, 0.0, -0.5);
  void* reg = arr(dtype, k, 0.3, 1.0);
  void* samp = arr(dtype, C * (k + 1), 0.0, 0.0);
  double* sched = (double*)malloc(sizeof(double) * 2 * 5);
  for (int i = 0; i < 5; ++i) {
    sched[2 * i] = 0.1 + 0.05 * i;
    sched[2 * i + 1] = proposal == IPMC_PROPOSAL_PCN ? sqrt(1 - sched[2 * i] * sched[2 * i]) : 1.0;
  }
  double* su = (double*)calloc((size_t)(C * k), sizeof(double));
  double* su2 = (double*)calloc((size_t)(C * k), sizeof(double));
  int64_t* acc = (int64_t*)calloc((size_t)C, sizeof(int64_t));
  int64_t* calls = (int64_t*)calloc((size_t)C, sizeof(int64_t));
  CHECK(orc_forward(m, dtype, C, u, g));
  CHECK(orc_potential(m, dtype, C, u, y, gi, phi));
  ipmc_sweep s;
  memset(&s, 0, sizeof(s));
  s.dtype = dtype;
  s.n_chains = C;
  s.chain_offset = 12345;
  s.u = u;
  s.phi = phi;
  s.accepts = acc;
  s.calls = calls;
  s.y = y;
  s.gamma_inv = gi;
  s.prior_sqrt = sq;
  s.beta = 0.3;
  s.contraction = proposal == IPMC_PROPOSAL_PCN ? sqrt(1 - 0.09) : 1.0;
  s.proposal = proposal;
  s.reg_scale = with_reg ? reg : NULL;
  s.seed = 0xABCDEFull;
  s.step0 = (1ull << 32) - 2;
  s.n_steps = 5;
  if (with_reg) CHECK(orc_init_phi(m, &s));
  CHECK(orc_pcn_sweep(m, &s, 1));
  s.box_lo = lo;
  s.beta_schedule = sched;
  s.sum_u = su;
  s.sum_u2 = su2;
  s.sample_out = samp;
  s.sample_stride = k + 1;
  s.step0 += 5;
  CHECK(orc_pcn_sweep(m, &s, 3));
  free(u), free(y), free(gi), free(g), free(phi), free(sq), free(lo), free(reg), free(samp), free(sched);
  free(su), free(su2), free(acc), free(calls);
}

int main(void) {
  for (int dt = 0; dt < 2; ++dt) {
    const int32_t dtype = dt ? IPMC_F64 : IPMC_F32;
    for (int arith = 0; arith < 2; ++arith) {
      for (int prop = 0; prop < 2; ++prop) {
        ipmc_model m;
        /* linear */
        memset(&m, 0, sizeof(m));
        m.kind = IPMC_MODEL_LINEAR, m.arith = arith, m.k = 5, m.q = 3;
        m.A = arr(dtype, 15, 1.0, 0.0), m.theta0 = arr(dtype, 5, 1.0, 0.0);
        run_model(&m, dtype, 7, prop, prop);
        cfree(m.A), cfree(m.theta0);
        /* Lorenz-63 */
        memset(&m, 0, sizeof(m));
        m.kind = IPMC_MODEL_LORENZ63, m.arith = arith, m.k = 3, m.q = 6, m.dim = 3, m.n_steps = 20, m.dt = 0.01;
        m.x0 = arr(dtype, 3, 1.0, 5.0), m.theta0 = arr(dtype, 3, 0.0, 10.0);
        run_model(&m, dtype, 5, prop, prop);
        cfree(m.x0), cfree(m.theta0);
        /* Lorenz-96 */
        memset(&m, 0, sizeof(m));
        m.kind = IPMC_MODEL_LORENZ96, m.arith = arith, m.k = m.q = m.dim = 9, m.n_steps = 15, m.dt = 0.005;
        m.x0 = arr(dtype, 9, 1.0, 8.0), m.theta0 = arr(dtype, 9, 0.0, 8.0);
        run_model(&m, dtype, 6, prop, prop);
        cfree(m.x0), cfree(m.theta0);
        /* two-scale Lorenz-96 */
        memset(&m, 0, sizeof(m));
        m.kind = IPMC_MODEL_LORENZ96_2S, m.arith = arith, m.k = 3, m.dim = 5, m.q = 25, m.n_steps = 10;
        m.dt = 0.004, m.fast_per_slow = 3, m.moment_mode = prop, m.coupling_c = 1.0;
        m.x0 = arr(dtype, 5 * 4, 1.0, 0.0), m.theta0 = arr(dtype, 3, 0.0, 9.0);
        run_model(&m, dtype, 4, prop, prop);
        cfree(m.x0), cfree(m.theta0);
        /* Burgers, both time-stepping modes */
        for (int mode = 0; mode < 2; ++mode) {
          memset(&m, 0, sizeof(m));
          const int N = 40;
          m.kind = IPMC_MODEL_BURGERS, m.arith = arith, m.k = 3, m.q = 2, m.n_windows = 2, m.dim = N;
          m.dt_mode = mode, m.dt = 1e-3, m.n_steps = 30, m.t_end = 0.05, m.cfl = 0.5, m.nu = mode ? 0.0 : 1e-3;
          m.dx = 2.0 / N, m.meas_scale = 10.0, m.meas_dx = 2.0 / N, m.max_iter = 100000;
          double* xc = (double*)malloc(sizeof(double) * (N + 2));
          float* xcf = (float*)malloc(sizeof(float) * (N + 2));
          for (int i = 0; i < N + 2; ++i) xc[i] = -1.0 - 1.0 / N + i * 2.0 / N, xcf[i] = (float)xc[i];
          int32_t wl[2] = {5, 20}, wh[2] = {12, 40};
          m.x0 = dtype == IPMC_F64 ? (void*)xc : (void*)xcf;
          m.win_lo = wl, m.win_hi = wh;
          m.theta0 = arr(dtype, 3, 0.0, 0.5);
          run_model(&m, dtype, 3, prop, prop);
          free(xc), free(xcf), cfree(m.theta0);
        }
      }
    }
  }
  /* len_burn_in on ragged lengths incl. len == window */
  for (int64_t len = 50; len <= 400; len += 117) {
    double* x = (double*)malloc(sizeof(double) * 3 * 2 * (size_t)len);
    for (int64_t i = 0; i < 3 * 2 * len; ++i) x[i] = 1.0 + rnd();
    int64_t out[3];
    CHECK(orc_burn_in(x, 3, 2, len, 50, 0.03, out));
    free(x);
  }
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("oracle selftest ok\n");
  return 0;
}
