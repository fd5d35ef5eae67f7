// Chain diagnostics on the device: batched normalised autocorrelation.
//
// For every series x (one chain's samples of one component, or one window of
// it) this computes what MCMCSampler.autocorr does for one series
// (sampler.py:43-54): x_ = x - mean(x), r[tau] = sum_t x_[t] x_[t+tau]
// (np.correlate(x_, x_, 'full')[-n:]), out = r / r[0], or all ones when
// r[0] == 0 (a constant series).  helpers.autocorrelation (helpers.py:41-54)
// is this over windows of tau_max samples, averaged on the host.
//
// One workgroup per series: the series is staged once in LDS (coalesced
// strided load), the mean is a block reduction, and each thread owns lags
// tau = tid, tid + 256, ... with the inner sum over t read from LDS.
#include "ipmc_internal.hpp"

namespace ipmc {

constexpr int kAcBlock = 256;
constexpr int kAcMaxLen = 8192;  // doubles staged per series (64 KiB LDS)

template <typename T>
__global__ __launch_bounds__(kAcBlock) void autocorr_kernel(const T* __restrict__ x, int64_t n_series, int64_t len,
                                                             int64_t stride_series, int64_t stride_t, int max_lag,
                                                             double* __restrict__ out) {
  __shared__ double xs[kAcMaxLen];
  __shared__ double red[kAcBlock];
  const int64_t s = blockIdx.x;
  if (s >= n_series) return;
  const T* src = x + s * stride_series;
  double part = 0.0;
  for (int64_t t = threadIdx.x; t < len; t += kAcBlock) {
    const double v = (double)src[t * stride_t];
    xs[t] = v;
    part += v;
  }
  red[threadIdx.x] = part;
  __syncthreads();
  for (int off = kAcBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  const double mean = red[0] / (double)len;
  __syncthreads();
  for (int64_t t = threadIdx.x; t < len; t += kAcBlock) xs[t] = xs[t] - mean;
  __syncthreads();
  // r[0] first (every thread needs it for the normalisation)
  double r0p = 0.0;
  for (int64_t t = threadIdx.x; t < len; t += kAcBlock) r0p += xs[t] * xs[t];
  red[threadIdx.x] = r0p;
  __syncthreads();
  for (int off = kAcBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  const double r0 = red[0];
  double* o = out + s * max_lag;
  for (int tau = threadIdx.x; tau < max_lag; tau += kAcBlock) {
    if (r0 == 0.0) {
      o[tau] = 1.0;
      continue;
    }
    double r = 0.0;
    for (int64_t t = 0; t + tau < len; ++t) r += xs[t] * xs[t + tau];
    o[tau] = r / r0;
  }
}

}  // namespace ipmc

using namespace ipmc;

extern "C" int ipmc_autocorr(const void* x, int32_t dtype, int64_t n_series, int64_t len, int64_t stride_series,
                             int64_t stride_t, int32_t max_lag, double* out, void* stream) {
  if (n_series < 0 || len < 0 || max_lag < 0) {
    set_error("ipmc_autocorr: negative size");
    return IPMC_ERR_INVALID;
  }
  if (n_series == 0 || max_lag == 0) return IPMC_OK;
  if (len == 0 || !x || !out) {
    set_error("ipmc_autocorr: empty series or NULL pointer");
    return IPMC_ERR_INVALID;
  }
  if (len > kAcMaxLen) {
    set_error("ipmc_autocorr: series longer than %d samples (split into windows)", kAcMaxLen);
    return IPMC_ERR_UNSUPPORTED;
  }
  if (max_lag > len) {
    set_error("ipmc_autocorr: max_lag %d exceeds the series length %lld", max_lag, (long long)len);
    return IPMC_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IPMC_F64)
    hipLaunchKernelGGL(autocorr_kernel<double>, dim3((unsigned)n_series), dim3(kAcBlock), 0, st, (const double*)x,
                       n_series, len, stride_series, stride_t, max_lag, out);
  else if (dtype == IPMC_F32)
    hipLaunchKernelGGL(autocorr_kernel<float>, dim3((unsigned)n_series), dim3(kAcBlock), 0, st, (const float*)x,
                       n_series, len, stride_series, stride_t, max_lag, out);
  else {
    set_error("ipmc_autocorr: bad dtype");
    return IPMC_ERR_INVALID;
  }
  return check_launch("autocorr_kernel");
}
