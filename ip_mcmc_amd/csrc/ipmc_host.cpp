// libipmc_host.so: the pCN path's counter-based draws on the host CPU
// (include/ipmc_host.h).  Same source as the device draws (ipmc_rng.hpp), built
// by g++ with -ffp-contract=off, so every value equals libipmc.so's.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../include/ipmc.h"
#include "../../include/ipmc_host.h"
#include "ipmc_rng.hpp"

using namespace ipmc;

namespace {

thread_local char g_err[256] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

// the device library's ranges (ipmc_api.hip): 32-bit global chain ids, pCN
// steps below 2^63 (host-side GaussianDistribution draws live above)
constexpr int64_t kChainIdLimit = int64_t(1) << 32;
constexpr uint64_t kHostStepBase = uint64_t(1) << 63;
// below this many elements one thread does the block (config 1's one chain)
constexpr int64_t kParallelMin = int64_t(1) << 16;

int check_chain_range(int64_t chain_offset, int64_t n_chains) {
  if (n_chains < 0 || chain_offset < 0) return fail(IPMC_ERR_INVALID, "negative count");
  if (chain_offset > kChainIdLimit - n_chains)
    return fail(IPMC_ERR_INVALID, "global chain ids (chain_offset + n_chains) must be <= 2^32");
  return IPMC_OK;
}

// fn(i0, i1) over [0, total) in contiguous slices, one per thread
template <typename F>
void parallel_for(int64_t total, int n_threads, F fn) {
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  if (total < kParallelMin) nt = 1;
  nt = (int)std::min<int64_t>(nt, std::max<int64_t>(1, total / 4096));
  if (nt <= 1) {
    fn((int64_t)0, total);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int t = 0; t < nt; ++t) {
    const int64_t i0 = total * t / nt, i1 = total * (t + 1) / nt;
    th.emplace_back([=] { fn(i0, i1); });
  }
  for (auto& x : th) x.join();
}

// draws_kernel's element loop (ipmc_api.hip), element i = (s, c, j) row-major
template <typename T>
void draws(uint64_t seed, int64_t c_off, int64_t n, uint64_t step0, int64_t total, int k, const T* sq,
           const T* chol, T* w, double* log_r, int n_threads) {
  parallel_for(total, n_threads, [=](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t sc = i / k;
      const int j = (int)(i - sc * k);
      const int64_t s = sc / n;
      const uint64_t gid = (uint64_t)(c_off + (sc - s * n));
      const uint64_t step = step0 + (uint64_t)s;
      w[i] = draw_w<T>(seed, gid, step, j, k, sq, chol);
      if (j == 0 && log_r) log_r[sc] = det_log(accept_uniform(seed, gid, step));
    }
  });
}

}  // namespace

extern "C" {

int ipmc_host_abi_version(void) { return IPMC_HOST_ABI_VERSION; }

const char* ipmc_host_last_error(void) { return g_err; }

int ipmc_host_pcn_draws(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step0, int64_t n_steps,
                        int32_t k, int32_t dtype, const void* prior_sqrt, const void* prior_chol, void* w,
                        double* log_r, int32_t n_threads) {
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
  if (dtype == IPMC_F64)
    draws<double>(seed, chain_offset, n_chains, step0, total, k, (const double*)prior_sqrt,
                  (const double*)prior_chol, (double*)w, log_r, n_threads);
  else
    draws<float>(seed, chain_offset, n_chains, step0, total, k, (const float*)prior_sqrt, (const float*)prior_chol,
                 (float*)w, log_r, n_threads);
  return IPMC_OK;
}

int ipmc_host_normal(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step, int32_t k,
                     int32_t dtype, void* out) {
  if (k < 0) return fail(IPMC_ERR_INVALID, "negative count");
  const int rc = check_chain_range(chain_offset, n_chains);
  if (rc) return rc;
  if (dtype != IPMC_F32 && dtype != IPMC_F64) return fail(IPMC_ERR_INVALID, "bad dtype");
  const int64_t total = n_chains * k;
  if (total == 0) return IPMC_OK;
  if (!out) return fail(IPMC_ERR_INVALID, "out is NULL");
  for (int64_t i = 0; i < total; ++i) {  // normal_kernel's element
    const double z = normal_component(seed, (uint64_t)(chain_offset + i / k), step, (int)(i % k));
    if (dtype == IPMC_F64)
      ((double*)out)[i] = z;
    else
      ((float*)out)[i] = (float)z;
  }
  return IPMC_OK;
}

int ipmc_host_uniform(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step, double* out) {
  const int rc = check_chain_range(chain_offset, n_chains);
  if (rc) return rc;
  if (n_chains == 0) return IPMC_OK;
  if (!out) return fail(IPMC_ERR_INVALID, "out is NULL");
  for (int64_t c = 0; c < n_chains; ++c) out[c] = accept_uniform(seed, (uint64_t)(chain_offset + c), step);
  return IPMC_OK;
}

int ipmc_host_step_uniforms(uint64_t seed, int64_t chain, uint64_t step, int32_t n, double* out) {
  if (n < 0 || chain < 0 || chain >= kChainIdLimit) return fail(IPMC_ERR_INVALID, "bad chain id or count");
  if (n > 0x10000) return fail(IPMC_ERR_INVALID, "at most 65536 uniforms per step");
  if (n == 0) return IPMC_OK;
  if (!out) return fail(IPMC_ERR_INVALID, "out is NULL");
  for (int32_t i = 0; i < n; ++i) out[i] = slot_uniform(seed, (uint64_t)chain, step, 0xFFFFFFFFu - (uint32_t)i);
  return IPMC_OK;
}

int ipmc_host_ordered_sum(const double* rows, int64_t n_rows, int64_t k, int64_t row_stride, double div,
                          double* acc) {
  if (n_rows < 0 || k < 0 || row_stride < k) return fail(IPMC_ERR_INVALID, "bad shape");
  if (n_rows == 0 || k == 0) return IPMC_OK;
  if (!rows || !acc) return fail(IPMC_ERR_INVALID, "NULL pointer");
  // one pass over the rows, every column in its own sequential chain (the
  // columns vectorise: each one's additions keep their order), the running
  // sums in a local buffer; div == 1 adds the rows as they are.  Memory-bound:
  // one streaming pass beats round 4's column tiles (a pass over the rows per
  // tile) 2.4x -- 2^18 x 256 values in 0.095 vs 0.228 s on the 8-core build
  // container -- and threads over columns were slower still (each re-reads
  // every row's cache lines).
  std::vector<double> a(acc, acc + k);
  double* __restrict__ ap = a.data();
  const double* __restrict__ x = rows;
  if (div == 1.0) {
    for (int64_t r = 0; r < n_rows; ++r, x += row_stride)
      for (int64_t j = 0; j < k; ++j) ap[j] = ap[j] + x[j];
  } else {
    for (int64_t r = 0; r < n_rows; ++r, x += row_stride)
      for (int64_t j = 0; j < k; ++j) ap[j] = ap[j] + x[j] / div;
  }
  for (int64_t j = 0; j < k; ++j) acc[j] = ap[j];
  return IPMC_OK;
}

}  // extern "C"
