// libipmc.so — C-ABI entry points (include/ipmc.h): argument checks, kernel
// choice and launch.  Small-state models (linear, Lorenz-63) and the RNG
// probes live here; Lorenz-96 and Burgers in their own translation units.
#include <stdarg.h>
#include <algorithm>
#include <stdio.h>

#include "ipmc_internal.hpp"
#include "ipmc_small.hpp"

namespace ipmc {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return IPMC_ERR_DEVICE;
  }
  return IPMC_OK;
}

static int fail(int code, const char* msg) {
  set_error("%s", msg);
  return code;
}

// The Philox counter holds the global chain id in one 32-bit word and the pCN
// step in two (ipmc_device.hpp); host-side draws (rng.py) use steps from
// kHostStepBase on.  Ids or steps outside these ranges would alias other
// chains' draws, so they are rejected.
constexpr int64_t kChainIdLimit = int64_t(1) << 32;
constexpr uint64_t kHostStepBase = uint64_t(1) << 63;

static int check_chain_range(int64_t chain_offset, int64_t n_chains) {
  if (n_chains < 0 || chain_offset < 0) return fail(IPMC_ERR_INVALID, "negative count");
  if (chain_offset > kChainIdLimit - n_chains)
    return fail(IPMC_ERR_INVALID, "global chain ids (chain_offset + n_chains) must be <= 2^32");
  return IPMC_OK;
}

static int check_model(const ipmc_model* m) {
  if (!m) return fail(IPMC_ERR_INVALID, "model is NULL");
  if (m->k <= 0 || m->q <= 0) return fail(IPMC_ERR_INVALID, "model k and q must be positive");
  if (!m->theta0) return fail(IPMC_ERR_INVALID, "model theta0 is NULL");
  if (m->arith != IPMC_ARITH_FMA && m->arith != IPMC_ARITH_REFERENCE) return fail(IPMC_ERR_INVALID, "bad arith");
  switch (m->kind) {
    case IPMC_MODEL_LINEAR:
      if (!m->A) return fail(IPMC_ERR_INVALID, "linear model: A is NULL");
      if (m->k > kSmallKMax) return fail(IPMC_ERR_UNSUPPORTED, "linear model: k > 64");
      return IPMC_OK;
    case IPMC_MODEL_LORENZ63:
      if (m->k != 3 || m->q != 6) return fail(IPMC_ERR_INVALID, "Lorenz-63: k must be 3 and q 6");
      if (!m->x0 || m->n_steps <= 0) return fail(IPMC_ERR_INVALID, "Lorenz-63: x0 / n_steps");
      return IPMC_OK;
    case IPMC_MODEL_LORENZ96:
      if (m->dim != m->k || m->q != m->dim) return fail(IPMC_ERR_INVALID, "Lorenz-96: k and q must equal dim");
      if (!m->x0 || m->n_steps <= 0) return fail(IPMC_ERR_INVALID, "Lorenz-96: x0 / n_steps");
      return IPMC_OK;
    case IPMC_MODEL_LORENZ96_2S:
      if (m->k != 3 || m->dim <= 0 || m->fast_per_slow <= 0 || m->q != 5 * m->dim)
        return fail(IPMC_ERR_INVALID, "two-scale Lorenz-96: k must be 3, K, J > 0 and q == 5K");
      if (!m->x0 || m->n_steps <= 0) return fail(IPMC_ERR_INVALID, "two-scale Lorenz-96: x0 / n_steps");
      if (m->dim > 64) return fail(IPMC_ERR_UNSUPPORTED, "two-scale Lorenz-96: K <= 64");
      return IPMC_OK;
    case IPMC_MODEL_BURGERS:
      if (m->k != 3 || m->q != m->n_windows || !m->win_lo || !m->win_hi || !m->x0 || m->dim < 2)
        return fail(IPMC_ERR_INVALID, "Burgers: k must be 3, q == n_windows, windows/centres set");
      return IPMC_OK;
  }
  return fail(IPMC_ERR_UNSUPPORTED, "unknown model kind");
}

static bool l96_has(int D, int dtype, int lpc, int cpl) {
  if (dtype == IPMC_F64) return cpl == 1 && l96_has_f64(D, lpc);
  return l96_has_f32(D, lpc, cpl);
}

// Layout choice for Lorenz-96 (lanes per chain LPC, chains per lane group CPL),
// from the layout scans of profiles/r1/lanes_scan_*.txt and lanes_layout_rule.txt:
//  1. the fewest lanes per chain whose halos go by DPP (LPC 1, 2, 4, 8, 16) that
//     still gives every SIMD one wave (kWaveLanes lanes), packed fp32 (CPL 2)
//     first; more lanes only add halo work, fewer leave SIMDs idle.  With more
//     than 20 components per lane (the in-place RK4 state, l96_stage, no
//     longer fits 256 VGPRs) the next layout (LPC 2 -> 4, <= 4 waves).
//     d=40, 65 536 chains, LPC 2 vs 4 on the same box: packed fp32 1.75 vs
//     1.85 ms, fp64 3.32 vs 3.37 ms (profiles/r2/lanes_scan_d40_r2k.txt);
//     (LPC 8 since round 3: two chains interleaved per row of 16 lanes, one
//     DPP row rotation per halo dword, group_vlane in ipmc_device.hpp; d=40,
//     8 192 chains: 14.7 / 17.1 M steps/s at 20 / 200 steps per launch, 10.4 /
//     10.8 M with ds_bpermute halos, profiles/r3/bench_8192_l8dpp.jsonl);
//  2. else any compiled layout reaching one wave;
//  3. else (an ensemble below one wave per SIMD, where the speculative sweep
//     fills lanes with slots) the most DPP lanes per chain that keep >= 4
//     components per lane: a chain's RK4 step is then a latency chain, and
//     LPC 8 (round 1, halos through LDS) was 1.6x slower (d=40 at 1 / 64 /
//     1 024 chains: LPC 4 0.050 / 0.050 / 0.054 ms per step vs LPC 8 0.080 /
//     0.084 / 0.087).
// The most lanes per chain whose halos go by DPP (LPC 1, 2, 4, 16) with >= 4
// components per lane, 0 if none is compiled: the layout of latency-bound
// chains (small ensembles, speculative slots).
static int l96_dpp_lpc(int D, int dtype, int cpl) {
  static const int dpp[4] = {1, 2, 4, 16};
  int lpc = 0;
  for (int i = 0; i < 4; ++i)
    if (D % dpp[i] == 0 && D / dpp[i] >= 4 && l96_has(D, dtype, dpp[i], cpl)) lpc = dpp[i];
  return lpc;
}

static void l96_layout(int D, int dtype, int64_t n_chains, int& lpc, int& cpl) {
  constexpr int64_t kWaveLanes = 65536;  // 256 CUs x 4 SIMDs x 64 lanes
  static const int dpp[5] = {1, 2, 4, 8, 16};
  static const int all[5] = {1, 2, 4, 8, 16};
  const int ncpl = dtype == IPMC_F32 ? 2 : 1;
  const int cpls[2] = {ncpl, 1};
  auto ok = [&](int l, int c) { return D % l == 0 && D / l >= 2 && l96_has(D, dtype, l, c); };
  for (int ci = 0; ci < ncpl; ++ci) {
    const int c = cpls[ci];
    const int64_t groups = (n_chains + c - 1) / c;
    for (int i = 0; i < 5; ++i) {
      int l = dpp[i];
      if (!ok(l, c) || groups * l < kWaveLanes) continue;
      // beyond 20 components per lane the in-place RK4 state (5 arrays) no
      // longer fits 256 VGPRs: split the chain over twice the lanes
      if (D / l > 20 && l <= 2 && ok(2 * l, c) && groups * 2 * l <= 4 * kWaveLanes) l *= 2;
      lpc = l;
      cpl = c;
      return;
    }
  }
  for (int ci = 0; ci < ncpl; ++ci) {
    const int c = cpls[ci];
    const int64_t groups = (n_chains + c - 1) / c;
    for (int i = 0; i < 5; ++i) {
      if (ok(all[i], c) && groups * all[i] >= kWaveLanes) {
        lpc = all[i];
        cpl = c;
        return;
      }
    }
  }
  lpc = 0;
  for (int ci = ncpl - 1; ci >= 0 && !lpc; --ci) {  // one chain per lane group first
    cpl = cpls[ci];
    lpc = l96_dpp_lpc(D, dtype, cpl);
    for (int i = 0; i < 5 && !lpc; ++i)
      if (ok(all[i], cpl)) lpc = all[i];
  }
}

// The whole Lorenz-96 sweep plan (layout and speculation width) for a launch:
// the one place ipmc_pcn_sweep and ipmc_plan_sweep take it from.
static int l96_plan(const ipmc_model& m, const ipmc_sweep& s, int& lpc, int& cpl, int& spec) {
  l96_layout(m.dim, s.dtype, s.n_chains, lpc, cpl);
  if (s.chains_per_lane) cpl = s.chains_per_lane;
  if (s.lanes_per_chain) lpc = s.lanes_per_chain;
  if (!lpc || !l96_has(m.dim, s.dtype, lpc, cpl)) {
    set_error("Lorenz-96: no kernel compiled for dim=%d lanes_per_chain=%d chains_per_lane=%d", m.dim, lpc, cpl);
    return IPMC_ERR_UNSUPPORTED;
  }
  // speculation (l96_spec_kernel): spec_width slots of lpc lanes per chain,
  // auto = the widest keeping the ensemble within one wave per SIMD
  spec = s.spec_width;
  if (spec < 0 || spec > kL96SpecBlockLanes || (spec & (spec - 1)))
    return fail(IPMC_ERR_UNSUPPORTED, "spec_width must be a power of two <= 256");
  if (spec == 0) {
    spec = 1;
    // an auto layout that already fills a wave per SIMD (since LPC 8 halos go
    // by DPP: 8 192 chains of d=40 on 8 lanes) runs sequentially unless the
    // launch is long: a launch lasts as long as its slowest chain, which costs
    // speculation most on short launches (bench problem, 8 192 chains, 20 /
    // 200 / 512 steps per launch: 8 lanes sequential 14.7 / 17.1 / -- M
    // steps/s, 4 lanes x 2 slots 10.7 / 17.7 / 18.8 M)
    const int64_t groups = (s.n_chains + cpl - 1) / cpl;
    const bool fills = !s.lanes_per_chain && groups * lpc >= 65536;
    if (s.n_steps > 1 && s.chains_per_lane != 2 && (!fills || s.n_steps >= 256)) {
      // speculative slots run on the quad / row DPP layout (l96_dpp_lpc: the
      // speculative kernel's LPC 8 halos take two DPP moves and a select)
      int l = lpc;
      if (!s.lanes_per_chain) {
        const int d = l96_dpp_lpc(m.dim, s.dtype, 1);
        if (d) l = d;
      }
      // slots fill at most one wave per SIMD.  A launch lasts as long as its
      // slowest chain, and on the bench problem (chains burning in from u = 0)
      // wider speculation loses most where launches are short: 8 192 chains,
      // 20 / 200 / 512 steps per launch, 4 lanes x 2 slots (this rule) 11.4 /
      // 18.0 / 18.8 M steps/s, 2 lanes x 8 slots (two waves per SIMD, round 3's
      // earlier rule) 5.9 / 15.6 / 18.9 M, sequential on 8 lanes 10.4 / 10.8 M
      // (profiles/r3/bench_8192_short.jsonl, bench_shards_l4.jsonl); on
      // config_bench's problem, which accepts almost nothing, 19.6 vs 20.2 M.
      const int64_t cap = 65536;
      int w = 1;
      while (w * 2 * l <= 64 && s.n_chains * (int64_t)l * w * 2 <= cap) w *= 2;
      // a whole block of slots per chain (4 waves on the CU's 4 SIMDs) while
      // the ensemble stays within one wave per SIMD
      if (w * l == 64 && s.n_chains * (int64_t)kL96SpecBlockLanes <= 65536) w = kL96SpecBlockLanes / l;
      if (w > 1) {
        spec = w;
        lpc = l;
      }
    }
  }
  if (spec > 1) {
    if (spec * lpc > 64 && spec * lpc != kL96SpecBlockLanes)
      return fail(IPMC_ERR_UNSUPPORTED, "Lorenz-96: spec_width * lanes_per_chain must be <= 64 or 256");
    if (cpl == 2) {
      if (s.chains_per_lane == 2)
        return fail(IPMC_ERR_UNSUPPORTED, "Lorenz-96: speculation runs one chain per lane group");
      cpl = 1;  // the packed fp32 layout is for full ensembles; fp32 one-chain kernels speculate
    }
  }
  return IPMC_OK;
}

template <typename T, int MODEL, bool FM>
static int small_sweep_launch(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  const int64_t blocks = (s.n_chains + kSmallBlock - 1) / kSmallBlock;
  hipLaunchKernelGGL((small_sweep_kernel<T, MODEL, FM>), dim3((unsigned)blocks), dim3(kSmallBlock), 0, st, m, s);
  return check_launch("small_sweep_kernel");
}

template <typename T>
static int small_sweep(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  const bool fm = m.arith == IPMC_ARITH_FMA;
  if (m.kind == IPMC_MODEL_LORENZ63)
    return fm ? small_sweep_launch<T, IPMC_MODEL_LORENZ63, true>(m, s, st)
              : small_sweep_launch<T, IPMC_MODEL_LORENZ63, false>(m, s, st);
  return fm ? small_sweep_launch<T, IPMC_MODEL_LINEAR, true>(m, s, st)
            : small_sweep_launch<T, IPMC_MODEL_LINEAR, false>(m, s, st);
}

// Speculation width for the small models (lanes per chain, small_spec_kernel):
// spec_width if given (a power of two <= 64), else the widest that keeps
// the ensemble within one wave per SIMD (1024 SIMDs x 64 lanes), when a launch
// has more than one step to speculate over: wider groups waste more work after
// the first acceptance and the machine turns throughput-bound (cfg 2, 4 096
// chains, accept 5 %: width 16 = 299 M steps/s, 64 = 153 M, 1 = 67 M;
// profiles/r1/spec_cfg2.txt).  -1: invalid request.
static int small_spec_width(const ipmc_model& m, const ipmc_sweep& s) {
  const int req = s.spec_width;
  if (req > 0) {
    if (req > 64 || (req & (req - 1))) return -1;
    if (req > 1 && m.k > kSpecKMax) return -1;
    return req;
  }
  int w = 1;
  if (m.k <= kSpecKMax && s.n_steps > 1)
    while (w < 64 && s.n_chains * (int64_t)w * 2 <= 65536) w *= 2;
  return w;
}

template <typename T, int MODEL, bool FM>
static int small_spec_launch(const ipmc_model& m, const ipmc_sweep& s, int w, hipStream_t st) {
  const int64_t blocks = (s.n_chains * w + kSpecBlock - 1) / kSpecBlock;
  switch (w) {
#define IPMC_SPEC(W)                                                                                           \
  case W:                                                                                                      \
    hipLaunchKernelGGL((small_spec_kernel<T, MODEL, FM, W>), dim3((unsigned)blocks), dim3(kSpecBlock), 0, st, m, \
                       s);                                                                                     \
    return check_launch("small_spec_kernel");
    IPMC_SPEC(2) IPMC_SPEC(4) IPMC_SPEC(8) IPMC_SPEC(16) IPMC_SPEC(32) IPMC_SPEC(64)
#undef IPMC_SPEC
  }
  return fail(IPMC_ERR_UNSUPPORTED, "speculation width must be a power of two <= 64");
}

template <typename T>
static int small_spec(const ipmc_model& m, const ipmc_sweep& s, int w, hipStream_t st) {
  const bool fm = m.arith == IPMC_ARITH_FMA;
  if (m.kind == IPMC_MODEL_LORENZ63)
    return fm ? small_spec_launch<T, IPMC_MODEL_LORENZ63, true>(m, s, w, st)
              : small_spec_launch<T, IPMC_MODEL_LORENZ63, false>(m, s, w, st);
  return fm ? small_spec_launch<T, IPMC_MODEL_LINEAR, true>(m, s, w, st)
            : small_spec_launch<T, IPMC_MODEL_LINEAR, false>(m, s, w, st);
}

template <typename T, int MODEL, bool FM>
static int small_eval_launch(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv,
                             void* out, bool phi, hipStream_t st) {
  const int64_t blocks = (n + kSmallBlock - 1) / kSmallBlock;
  if (phi)
    hipLaunchKernelGGL((small_eval_kernel<T, MODEL, FM, true>), dim3((unsigned)blocks), dim3(kSmallBlock), 0, st, m,
                       n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);
  else
    hipLaunchKernelGGL((small_eval_kernel<T, MODEL, FM, false>), dim3((unsigned)blocks), dim3(kSmallBlock), 0, st, m,
                       n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);
  return check_launch("small_eval_kernel");
}

template <typename T>
static int small_eval(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                      bool phi, hipStream_t st) {
  const bool fm = m.arith == IPMC_ARITH_FMA;
  if (m.kind == IPMC_MODEL_LORENZ63)
    return fm ? small_eval_launch<T, IPMC_MODEL_LORENZ63, true>(m, n, u, y, ginv, out, phi, st)
              : small_eval_launch<T, IPMC_MODEL_LORENZ63, false>(m, n, u, y, ginv, out, phi, st);
  return fm ? small_eval_launch<T, IPMC_MODEL_LINEAR, true>(m, n, u, y, ginv, out, phi, st)
            : small_eval_launch<T, IPMC_MODEL_LINEAR, false>(m, n, u, y, ginv, out, phi, st);
}

template <typename T>
__global__ void normal_kernel(uint64_t seed, int64_t c_off, int64_t n, uint64_t step, int k, T* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * k) return;
  const int64_t c = i / k;
  const int j = (int)(i % k);
  double z0, z1;
  normal_pair(seed, (uint64_t)(c_off + c), step, (uint32_t)(j >> 1), z0, z1);
  out[i] = (T)((j & 1) ? z1 : z0);
}

// phi[c] = phi[c] + ½ Σ_j (c_j u_cj)²  (the sweep's I = Φ + regularizer, in its order)
template <typename T, bool FM>
__global__ void reg_add_kernel(int64_t n, int k, const T* __restrict__ u, const T* __restrict__ c, T* phi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  phi[i] = phi[i] + small_regularizer<T, FM>(k, c, u + i * k, 1);
}

// ipmc_pcn_draws: one thread per (step, chain, component), grid-stride.  w is
// formed with pcn_propose's / chol_noise's operations (draw_w, ipmc_rng.hpp:
// the same bits as the sweep kernels' proposal noise and as the host
// library's ipmc_host_pcn_draws); the j = 0 thread also writes log r.
template <typename T>
__global__ void draws_kernel(uint64_t seed, int64_t c_off, int64_t n, uint64_t step0, int64_t total, int k,
                             const T* __restrict__ sq, const T* __restrict__ chol, T* __restrict__ w,
                             double* __restrict__ log_r) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sc = i / k;
    const int j = (int)(i - sc * k);
    const int64_t s = sc / n;
    const uint64_t gid = (uint64_t)(c_off + (sc - s * n));
    const uint64_t step = step0 + (uint64_t)s;
    w[i] = draw_w<T>(seed, gid, step, j, k, sq, chol);
    if (j == 0 && log_r) log_r[sc] = det_log(accept_uniform(seed, gid, step));
  }
}

__global__ void uniform_kernel(uint64_t seed, int64_t c_off, int64_t n, uint64_t step, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = accept_uniform(seed, (uint64_t)(c_off + i), step);
}

static int dispatch_eval(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, const void* y,
                         const void* ginv, void* out, bool phi, void* stream) {
  int rc = check_model(m);
  if (rc) return rc;
  if (dtype != IPMC_F32 && dtype != IPMC_F64) return fail(IPMC_ERR_INVALID, "dtype must be IPMC_F32 or IPMC_F64");
  if (n < 0) return fail(IPMC_ERR_INVALID, "n must be >= 0");
  if (n == 0) return IPMC_OK;
  if (!u || !out) return fail(IPMC_ERR_INVALID, "u / out is NULL");
  if (phi && (!y || !ginv)) return fail(IPMC_ERR_INVALID, "y / gamma_inv is NULL");
  hipStream_t st = (hipStream_t)stream;
  switch (m->kind) {
    case IPMC_MODEL_LINEAR:
    case IPMC_MODEL_LORENZ63:
      return dtype == IPMC_F64 ? small_eval<double>(*m, n, u, y, ginv, out, phi, st)
                               : small_eval<float>(*m, n, u, y, ginv, out, phi, st);
    case IPMC_MODEL_LORENZ96: {
      int lpc, cpl;
      l96_layout(m->dim, IPMC_F64, n, lpc, cpl);  // eval kernels run one chain per lane group
      if (!lpc || !l96_has(m->dim, dtype, lpc, 1)) return fail(IPMC_ERR_UNSUPPORTED, "Lorenz-96: no kernel compiled for this dim");
      return dtype == IPMC_F64 ? l96_eval_f64(*m, n, u, y, ginv, out, phi, lpc, st)
                               : l96_eval_f32(*m, n, u, y, ginv, out, phi, lpc, st);
    }
    case IPMC_MODEL_BURGERS:
      return burgers_eval(*m, dtype, n, u, y, ginv, out, phi, st);
    case IPMC_MODEL_LORENZ96_2S:
      return l96ts_eval(*m, dtype, n, u, y, ginv, out, phi, st);
  }
  return fail(IPMC_ERR_UNSUPPORTED, "unknown model kind");
}

}  // namespace ipmc

using namespace ipmc;

extern "C" {

int ipmc_abi_version(void) { return IPMC_ABI_VERSION; }

const char* ipmc_last_error(void) { return g_err; }

int ipmc_auto_lanes(const ipmc_model* m, int32_t dtype, int64_t n_chains) {
  return ipmc_auto_layout(m, dtype, n_chains) % 100;
}

int ipmc_auto_layout(const ipmc_model* m, int32_t dtype, int64_t n_chains) {
  if (!m) return 0;
  if (m->kind == IPMC_MODEL_LORENZ96) {
    int lpc, cpl;
    l96_layout(m->dim, dtype, n_chains, lpc, cpl);
    return cpl * 100 + lpc;
  }
  return 101;
}

int ipmc_plan_sweep(const ipmc_model* m, const ipmc_sweep* s, ipmc_plan* out) {
  int rc = check_model(m);
  if (rc) return rc;
  if (!s || !out) return fail(IPMC_ERR_INVALID, "sweep / out is NULL");
  if (s->dtype != IPMC_F32 && s->dtype != IPMC_F64) return fail(IPMC_ERR_INVALID, "dtype must be IPMC_F32/F64");
  int lanes = 1, cpl = 1, spec = 1;
  switch (m->kind) {
    case IPMC_MODEL_LINEAR:
    case IPMC_MODEL_LORENZ63:
      spec = small_spec_width(*m, *s);
      if (spec < 0)
        return fail(IPMC_ERR_UNSUPPORTED, "small models: spec_width must be a power of two <= 64, and 1 for k > 8");
      break;
    case IPMC_MODEL_LORENZ96:
      rc = l96_plan(*m, *s, lanes, cpl, spec);
      break;
    case IPMC_MODEL_BURGERS:
      rc = burgers_plan(*m, *s, lanes, spec);
      break;
    case IPMC_MODEL_LORENZ96_2S:
      rc = l96ts_plan(*m, *s, lanes, spec);
      break;
    default:
      return fail(IPMC_ERR_UNSUPPORTED, "unknown model kind");
  }
  if (rc) return rc;
  out->lanes_per_chain = lanes;
  out->chains_per_lane = cpl;
  out->spec_width = spec;
  out->reserved = 0;
  return IPMC_OK;
}

int ipmc_pcn_sweep(const ipmc_model* m, const ipmc_sweep* s, void* stream) {
  int rc = check_model(m);
  if (rc) return rc;
  if (!s) return fail(IPMC_ERR_INVALID, "sweep is NULL");
  if (s->dtype != IPMC_F32 && s->dtype != IPMC_F64) return fail(IPMC_ERR_INVALID, "dtype must be IPMC_F32/F64");
  if (s->proposal != IPMC_PROPOSAL_PCN && s->proposal != IPMC_PROPOSAL_RW)
    return fail(IPMC_ERR_INVALID, "proposal must be IPMC_PROPOSAL_PCN or IPMC_PROPOSAL_RW");
  if (s->proposal == IPMC_PROPOSAL_PCN && !(s->beta >= 0.0 && s->beta <= 1.0))
    return fail(IPMC_ERR_INVALID, "beta has to be in [0,1]");
  if (s->n_steps < 0) return fail(IPMC_ERR_INVALID, "negative count");
  rc = check_chain_range(s->chain_offset, s->n_chains);
  if (rc) return rc;
  if (s->n_steps > 0x7fffffff) return fail(IPMC_ERR_INVALID, "n_steps per launch must be < 2^31");
  if (s->step0 > kHostStepBase - (uint64_t)s->n_steps)
    return fail(IPMC_ERR_INVALID, "pCN steps must stay below 2^63 (the host-draw range)");
  if (s->sample_every < 0 || s->sample_every > 0x7fffffff)
    return fail(IPMC_ERR_INVALID, "sample_every must be in [0, 2^31)");
  if (s->sample_every > 0 && (!s->sample_out || s->sample_step_stride < m->k || s->sample_stride < m->k))
    return fail(IPMC_ERR_INVALID, "sample_every needs sample_out, sample_stride >= k and sample_step_stride >= k");
  if (s->sample_every > 0 && s->n_chains > 1) {
    // the n_s samples of a chain must not reach into another chain's rows
    const int64_t ns = s->n_steps / s->sample_every;
    if (ns > 0) {
      const bool chain_major = (s->sample_stride - m->k) / s->sample_step_stride >= ns - 1;
      const bool sample_major = (s->sample_step_stride - m->k) / s->sample_stride >= s->n_chains - 1;
      if (!chain_major && !sample_major)
        return fail(IPMC_ERR_INVALID,
                    "sample_every: the samples overlap; need sample_stride >= (n_s-1)*sample_step_stride + k or "
                    "sample_step_stride >= (n_chains-1)*sample_stride + k, n_s = n_steps / sample_every");
    }
  }
  if (s->n_chains == 0 || s->n_steps == 0) {
    if (s->n_chains > 0 && s->sample_out && s->sample_every == 0) {
      // no step: the sample is the current state
      const size_t es = s->dtype == IPMC_F64 ? 8 : 4;
      hipStream_t st = (hipStream_t)stream;
      if (hipMemcpy2DAsync(s->sample_out, (size_t)s->sample_stride * es, s->u, (size_t)m->k * es,
                           (size_t)m->k * es, (size_t)s->n_chains, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail(IPMC_ERR_DEVICE, "sample copy failed");
    }
    return IPMC_OK;
  }
  if (!s->u || !s->phi || !s->y || !s->gamma_inv || (!s->prior_sqrt && !s->prior_chol))
    return fail(IPMC_ERR_INVALID, "u / phi / y / gamma_inv / prior_sqrt (or prior_chol) is NULL");
  if (s->sample_out && s->sample_stride < m->k) return fail(IPMC_ERR_INVALID, "sample_stride < k");
  if (s->sum_u2 && !s->sum_u) return fail(IPMC_ERR_INVALID, "sum_u2 needs sum_u");
  hipStream_t st = (hipStream_t)stream;
  switch (m->kind) {
    case IPMC_MODEL_LINEAR:
    case IPMC_MODEL_LORENZ63: {
      if (s->chains_per_lane > 1 || s->lanes_per_chain > 1)
        return fail(IPMC_ERR_UNSUPPORTED, "small models run one chain per lane (spec_width adds speculative lanes)");
      const int w = small_spec_width(*m, *s);
      if (w < 0)
        return fail(IPMC_ERR_UNSUPPORTED, "small models: spec_width must be a power of two <= 64, and 1 for k > 8");
      if (w > 1) return s->dtype == IPMC_F64 ? small_spec<double>(*m, *s, w, st) : small_spec<float>(*m, *s, w, st);
      return s->dtype == IPMC_F64 ? small_sweep<double>(*m, *s, st) : small_sweep<float>(*m, *s, st);
    }
    case IPMC_MODEL_LORENZ96: {
      int lpc, cpl, spec;
      rc = l96_plan(*m, *s, lpc, cpl, spec);
      if (rc) return rc;
      return s->dtype == IPMC_F64 ? l96_sweep_f64(*m, *s, lpc, spec, st)
                                  : l96_sweep_f32(*m, *s, lpc, cpl, spec, st);
    }
    case IPMC_MODEL_BURGERS:
      return burgers_sweep(*m, *s, st);
    case IPMC_MODEL_LORENZ96_2S:
      return l96ts_sweep(*m, *s, st);
  }
  return fail(IPMC_ERR_UNSUPPORTED, "unknown model kind");
}

int ipmc_pcn_run(const ipmc_model* m, const ipmc_sweep* s, int64_t n_blocks, int64_t block_steps,
                 int64_t sample_block_stride, void* stream) {
  if (!s) return fail(IPMC_ERR_INVALID, "sweep is NULL");
  if (n_blocks < 0 || block_steps < 0) return fail(IPMC_ERR_INVALID, "negative count");
  if (block_steps > 0x7fffffff) return fail(IPMC_ERR_INVALID, "block_steps must be < 2^31");
  if (n_blocks > 0 && (uint64_t)block_steps > 0 &&
      (uint64_t)n_blocks > (kHostStepBase - s->step0) / (uint64_t)block_steps)
    return fail(IPMC_ERR_INVALID, "pCN steps must stay below 2^63 (the host-draw range)");
  if (s->sample_out && sample_block_stride < 0) return fail(IPMC_ERR_INVALID, "negative sample_block_stride");
  const size_t es = s->dtype == IPMC_F64 ? 8 : 4;
  ipmc_sweep b = *s;
  b.n_steps = block_steps;
  for (int64_t i = 0; i < n_blocks; ++i) {  // sampler.py:23-28, one launch per block
    b.step0 = s->step0 + (uint64_t)(i * block_steps);
    if (s->sample_out) b.sample_out = (char*)s->sample_out + (size_t)(i * sample_block_stride) * es;
    if (s->beta_schedule) b.beta_schedule = s->beta_schedule + 2 * i * block_steps;
    const int rc = ipmc_pcn_sweep(m, &b, stream);
    if (rc) return rc;
  }
  return IPMC_OK;
}

int ipmc_init_phi(const ipmc_model* m, const ipmc_sweep* s, void* stream) {
  if (!s) return fail(IPMC_ERR_INVALID, "sweep is NULL");
  int rc = dispatch_eval(m, s->dtype, s->n_chains, s->u, s->y, s->gamma_inv, s->phi, true, stream);
  if (rc || !s->reg_scale || s->n_chains == 0) return rc;
  const int64_t blocks = (s->n_chains + 255) / 256;
  const bool fm = m->arith == IPMC_ARITH_FMA;
  hipStream_t st = (hipStream_t)stream;
  if (s->dtype == IPMC_F64) {
    if (fm)
      hipLaunchKernelGGL((reg_add_kernel<double, true>), dim3((unsigned)blocks), dim3(256), 0, st, s->n_chains, m->k,
                         (const double*)s->u, (const double*)s->reg_scale, (double*)s->phi);
    else
      hipLaunchKernelGGL((reg_add_kernel<double, false>), dim3((unsigned)blocks), dim3(256), 0, st, s->n_chains,
                         m->k, (const double*)s->u, (const double*)s->reg_scale, (double*)s->phi);
  } else {
    if (fm)
      hipLaunchKernelGGL((reg_add_kernel<float, true>), dim3((unsigned)blocks), dim3(256), 0, st, s->n_chains, m->k,
                         (const float*)s->u, (const float*)s->reg_scale, (float*)s->phi);
    else
      hipLaunchKernelGGL((reg_add_kernel<float, false>), dim3((unsigned)blocks), dim3(256), 0, st, s->n_chains,
                         m->k, (const float*)s->u, (const float*)s->reg_scale, (float*)s->phi);
  }
  return check_launch("reg_add_kernel");
}

int ipmc_potential(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, const void* y,
                   const void* gamma_inv, void* phi, void* stream) {
  return dispatch_eval(m, dtype, n, u, y, gamma_inv, phi, true, stream);
}

int ipmc_forward(const ipmc_model* m, int32_t dtype, int64_t n, const void* u, void* g, void* stream) {
  return dispatch_eval(m, dtype, n, u, nullptr, nullptr, g, false, stream);
}

int ipmc_normal(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step, int32_t k, int32_t dtype,
                void* out, void* stream) {
  if (k < 0) return fail(IPMC_ERR_INVALID, "negative count");
  const int rc = check_chain_range(chain_offset, n_chains);
  if (rc) return rc;
  if (dtype != IPMC_F32 && dtype != IPMC_F64) return fail(IPMC_ERR_INVALID, "bad dtype");
  const int64_t total = n_chains * k;
  if (total == 0) return IPMC_OK;
  if (!out) return fail(IPMC_ERR_INVALID, "out is NULL");
  const int64_t blocks = (total + 255) / 256;
  if (dtype == IPMC_F64)
    hipLaunchKernelGGL(normal_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, seed,
                       chain_offset, n_chains, step, k, (double*)out);
  else
    hipLaunchKernelGGL(normal_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, seed,
                       chain_offset, n_chains, step, k, (float*)out);
  return check_launch("normal_kernel");
}

int ipmc_uniform(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step, double* out, void* stream) {
  const int rc = check_chain_range(chain_offset, n_chains);
  if (rc) return rc;
  if (n_chains == 0) return IPMC_OK;
  if (!out) return fail(IPMC_ERR_INVALID, "out is NULL");
  const int64_t blocks = (n_chains + 255) / 256;
  hipLaunchKernelGGL(uniform_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, seed, chain_offset,
                     n_chains, step, out);
  return check_launch("uniform_kernel");
}

int ipmc_pcn_draws(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step0, int64_t n_steps,
                   int32_t k, int32_t dtype, const void* prior_sqrt, const void* prior_chol, void* w,
                   double* log_r, void* stream) {
  if (k <= 0 || n_steps < 0) return fail(IPMC_ERR_INVALID, "k must be positive and n_steps >= 0");
  int rc = check_chain_range(chain_offset, n_chains);
  if (rc) return rc;
  if (dtype != IPMC_F32 && dtype != IPMC_F64) return fail(IPMC_ERR_INVALID, "bad dtype");
  if (step0 > kHostStepBase || (uint64_t)n_steps > kHostStepBase - step0)
    return fail(IPMC_ERR_INVALID, "pCN steps must stay below 2^63 (the host-draw range)");
  if (n_chains == 0 || n_steps == 0) return IPMC_OK;
  if (!w) return fail(IPMC_ERR_INVALID, "w is NULL");
  if (!prior_sqrt && !prior_chol) return fail(IPMC_ERR_INVALID, "prior_sqrt and prior_chol are both NULL");
  if (n_chains > INT64_MAX / k / n_steps) return fail(IPMC_ERR_INVALID, "n_steps * n_chains * k overflows");
  const int64_t total = n_steps * n_chains * k;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 65536);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IPMC_F64)
    hipLaunchKernelGGL(draws_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, st, seed, chain_offset, n_chains,
                       step0, total, k, (const double*)prior_sqrt, (const double*)prior_chol, (double*)w, log_r);
  else
    hipLaunchKernelGGL(draws_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, st, seed, chain_offset, n_chains,
                       step0, total, k, (const float*)prior_sqrt, (const float*)prior_chol, (float*)w, log_r);
  return check_launch("draws_kernel");
}

int ipmc_copy_rows_d2h(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t width,
                       int64_t rows, void* stream) {
  if (rows < 0 || width < 0) return fail(IPMC_ERR_INVALID, "negative count");
  if (rows == 0 || width == 0) return IPMC_OK;
  if (!dst || !src) return fail(IPMC_ERR_INVALID, "dst / src is NULL");
  if (dst_pitch < width || src_pitch < width) return fail(IPMC_ERR_INVALID, "pitch < width");
  const hipError_t e = hipMemcpy2DAsync(dst, (size_t)dst_pitch, src, (size_t)src_pitch, (size_t)width,
                                        (size_t)rows, hipMemcpyDeviceToHost, (hipStream_t)stream);
  if (e != hipSuccess) {
    set_error("hipMemcpy2DAsync: %s", hipGetErrorString(e));
    return IPMC_ERR_DEVICE;
  }
  return IPMC_OK;
}

}  // extern "C"
