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
// tau = tid, tid + 256, ... with the inner sum over t read from LDS.  Longer
// series (> kAcMaxLen samples) stream through LDS tiles instead
// (autocorr_long_kernel), with the same summation order.
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

// Series longer than kAcMaxLen: the same sums from global memory.  A block
// owns kAcBlock consecutive lags of one series (grid: series x lag tiles),
// recomputes the mean and r[0] with the short kernel's strided-partials + tree
// order, and streams the series through LDS in tiles of kAcTile samples:
// a = x_[t0 .. t0+kAcTile), b = x_[t0+tau0 .. t0+tau0+kAcTile+kAcBlock).
// Each thread's r[tau] is still the ascending sum over t, so the results equal
// the short kernel's bit for bit.
constexpr int kAcTile = 2048;

template <typename T>
__device__ double ac_block_sum(const T* src, int64_t len, int64_t stride_t, double sub, bool square, double* red) {
  double part = 0.0;
  for (int64_t t = threadIdx.x; t < len; t += kAcBlock) {
    const double v = (double)src[t * stride_t];
    if (square) {
      const double c = v - sub;
      part += c * c;
    } else {
      part += v;
    }
  }
  red[threadIdx.x] = part;
  __syncthreads();
  for (int off = kAcBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(kAcBlock) void autocorr_long_kernel(const T* __restrict__ x, int64_t n_series,
                                                                  int64_t len, int64_t stride_series,
                                                                  int64_t stride_t, int max_lag,
                                                                  double* __restrict__ out) {
  __shared__ double a[kAcTile];
  __shared__ double b[kAcTile + kAcBlock];
  __shared__ double red[kAcBlock];
  const int64_t s = blockIdx.x;
  const int tau0 = blockIdx.y * kAcBlock;
  if (s >= n_series || tau0 >= max_lag) return;
  const T* src = x + s * stride_series;
  const double mean = ac_block_sum(src, len, stride_t, 0.0, false, red) / (double)len;
  const double r0 = ac_block_sum(src, len, stride_t, mean, true, red);
  const int tau = tau0 + (int)threadIdx.x;
  double* o = out + s * max_lag;
  if (r0 == 0.0) {
    if (tau < max_lag) o[tau] = 1.0;
    return;
  }
  double r = 0.0;
  for (int64_t t0 = 0; t0 + tau0 < len; t0 += kAcTile) {
    for (int i = threadIdx.x; i < kAcTile; i += kAcBlock) {
      const int64_t t = t0 + i;
      a[i] = t < len ? (double)src[t * stride_t] - mean : 0.0;
    }
    for (int i = threadIdx.x; i < kAcTile + kAcBlock; i += kAcBlock) {
      const int64_t t = t0 + tau0 + i;
      b[i] = t < len ? (double)src[t * stride_t] - mean : 0.0;
    }
    __syncthreads();
    if (tau < max_lag) {
      const int64_t rem = len - tau - t0;  // terms t0 + i with t0 + i + tau < len
      const int n = rem < kAcTile ? (int)(rem > 0 ? rem : 0) : kAcTile;
      const int sh = (int)threadIdx.x;
      for (int i = 0; i < n; ++i) r += a[i] * b[i + sh];
    }
    __syncthreads();
  }
  if (tau < max_lag) o[tau] = r / r0;
}

// ---------------------------------------------------------------- burn-in
// len_burn_in (burgers/utilities.py:134-167) for a batch of chains.  Per
// chain c with n_vars series of len samples and window w:
//   avg_v[j] = (cs[j+w-1] - cs[j-1]) / w   (cs = np.cumsum, cs[-1] := 0 term absent)
//   changed[i] = any_v |(avg_v[i] - avg_v[i+1]) / mean_v| > thr,  i < L = len - w
//   burn_in = largest i in [1, L-w-2] with changed[i..i+w] all set, else len-1.
// Kernel 1: one thread per series (c, v) streams the series twice (the
// leading and trailing cumulative sums are both sequential sums in np.cumsum's
// order, so their difference is bit-identical to res[l:] - res[:-l]) and ORs
// its flags into a per-chain bitmask.  Kernel 2: one thread per chain scans
// the bitmask from the end.  All arithmetic is fp64.

// numpy pairwise_sum (loops_utils.h.src) of a strided series, iteratively.
template <typename T>
__device__ double np_pairwise_strided(const T* a, int64_t n, int64_t s) {
  int64_t off[48], len[48];
  double left[48];
  int stage[48];
  int sp = 0;
  off[0] = 0;
  len[0] = n;
  stage[0] = 0;
  double ret = 0.0;
  while (sp >= 0) {
    const int64_t o = off[sp], m = len[sp];
    if (m <= 128) {
      const T* b = a + o * s;
      if (m < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < m; ++i) r = r + (double)b[i * s];
        ret = r;
      } else {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = (double)b[j * s];
        int64_t i;
        for (i = 8; i < m - (m % 8); i += 8)
          for (int j = 0; j < 8; ++j) r[j] = r[j] + (double)b[(i + j) * s];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < m; ++i) res = res + (double)b[i * s];
        ret = res;
      }
      --sp;
      continue;
    }
    int64_t n2 = m / 2;
    n2 -= n2 % 8;
    if (stage[sp] == 0) {
      stage[sp] = 1;
      ++sp;
      off[sp] = o;
      len[sp] = n2;
      stage[sp] = 0;
    } else if (stage[sp] == 1) {
      left[sp] = ret;
      stage[sp] = 2;
      ++sp;
      off[sp] = o + n2;
      len[sp] = m - n2;
      stage[sp] = 0;
    } else {
      ret = left[sp] + ret;
      --sp;
    }
  }
  return ret;
}

template <typename T>
__global__ __launch_bounds__(256) void burn_in_flags_kernel(const T* __restrict__ x, int64_t n_chains, int n_vars,
                                                             int64_t len, int64_t s_chain, int64_t s_var,
                                                             int64_t s_t, int w, double thr,
                                                             unsigned* __restrict__ flags, int64_t words) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_chains * n_vars) return;
  const int64_t c = g / n_vars;
  const int v = (int)(g % n_vars);
  const T* a = x + c * s_chain + v * s_var;
  const double mean = np_pairwise_strided<T>(a, len, s_t) / (double)len;
  const double dw = (double)w;
  double lead = (double)a[0];
  for (int64_t t = 1; t < w; ++t) lead = lead + (double)a[t * s_t];
  double trail = 0.0;
  double prev = lead / dw;
  unsigned* fl = flags + c * words;
  unsigned word = 0;
  const int64_t L = len - w;
  for (int64_t j = 1; j <= L; ++j) {
    lead = lead + (double)a[(j + w - 1) * s_t];
    trail = (j == 1) ? (double)a[0] : trail + (double)a[(j - 1) * s_t];
    const double cur = (lead - trail) / dw;
    const double ch = fabs((prev - cur) / mean);
    const int64_t i = j - 1;
    if (ch > thr) word |= 1u << (i & 31);
    if ((i & 31) == 31 || j == L) {
      if (word) atomicOr(fl + (i >> 5), word);
      word = 0;
    }
    prev = cur;
  }
}

__global__ void burn_in_search_kernel(int64_t n_chains, int64_t len, int w, const unsigned* __restrict__ flags,
                                      int64_t words, int64_t* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_chains) return;
  const unsigned* fl = flags + c * words;
  const int64_t L = len - w;
  const int64_t top = L - w - 2;
  int64_t run = 0, res = len - 1;
  for (int64_t j = L - 1; j >= 1; --j) {
    run = ((fl[j >> 5] >> (j & 31)) & 1u) ? run + 1 : 0;
    if (j <= top && run >= w + 1) {
      res = j;
      break;
    }
  }
  out[c] = res;
}

// The chain-ordered column sums behind the many-chain posterior mean
// (shard.ordered_sum_sharded): acc[j] = (((acc[j] + x_0j/div) + x_1j/div) + ...)
// strictly in row order, the additions of ipmc_host_ordered_sum (same IEEE
// operations, -ffp-contract=off: the same bits).  The sum of a column is one
// dependent chain of adds, so the kernel keeps that chain fed: a block owns 64
// columns; wave 0 holds one column per lane and adds chunk c (<= 8 192 values)
// from LDS while waves 1-15 stream chunk c + 1 from global memory into the other
// LDS buffer (coalesced, many loads in flight) -- one barrier per chunk.  A
// lane walking the rows straight from global memory waits out a load latency
// per row or per unrolled group (2.5 ms for 65 536 x 40 values on the MI355X,
// more than the host library's one pass).
constexpr int kOsCols = 64;     // columns per block (wave 0: one per lane)
constexpr int kOsBuf = 8192;    // doubles per LDS buffer: 8192 / kc rows per chunk
constexpr int kOsBlock = 1024;  // wave 0 adds, waves 1-15 load
constexpr int kOsLoaders = kOsBlock / 64 - 1;
constexpr int kOsPerLane = 16;  // rows per loader lane and chunk (>= ceil(8192 / kOsLoaders / 1))

__global__ __launch_bounds__(kOsBlock) void ordered_sum_kernel(const double* __restrict__ x, int64_t n_rows, int64_t k,
                                                              int64_t stride, double div, double* __restrict__ acc) {
  __shared__ double buf[2][kOsBuf];
  const int t = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * kOsCols;
  const int kc = (int)((k - c0) < kOsCols ? (k - c0) : kOsCols);
  // rows per chunk: the buffer's rows, and at most what the loaders cover in one pass
  const int R = (kOsBuf / kc) < kOsLoaders * kOsPerLane ? (kOsBuf / kc) : kOsLoaders * kOsPerLane;
  const int64_t n_chunks = (n_rows + R - 1) / R;
  auto rows_of = [&](int64_t chunk) {
    const int64_t left = n_rows - chunk * R;
    return (int)(left < R ? left : R);
  };
  // loader lane l of waves 1-15: column l % 64, rows l / 64, + 15, + 30, ...
  // of the chunk -- all of its loads issued before any LDS write, so each lane
  // has up to kOsPerLane in flight and the block ~15 x 64 x 16 (no division
  // per element)
  const int lj = (t - 64) & 63, lr = (t - 64) >> 6;
  auto load = [&](int64_t chunk, int b) {  // chunk -> buf[b], row-major [rows][kc]
    if (lj >= kc) return;
    const int rows = rows_of(chunk);
    const double* src = x + chunk * R * stride + c0 + lj;
    double* dst = buf[b] + lj;
    double v[kOsPerLane];
#pragma unroll
    for (int u = 0; u < kOsPerLane; ++u) {
      const int r = lr + kOsLoaders * u;
      v[u] = r < rows ? src[r * stride] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kOsPerLane; ++u) {
      const int r = lr + kOsLoaders * u;
      if (r < rows) dst[r * kc] = v[u];
    }
  };
  double a = 0.0;
  if (t < kc) a = acc[c0 + t];
  if (t >= 64) load(0, 0);
  __syncthreads();
  for (int64_t c = 0; c < n_chunks; ++c) {
    if (t < 64) {
      if (t < kc) {
        const int rows = rows_of(c);
        const double* bb = buf[c & 1] + t;
        if (div == 1.0) {
#pragma unroll 8
          for (int r = 0; r < rows; ++r) a = a + bb[r * kc];
        } else {
#pragma unroll 8
          for (int r = 0; r < rows; ++r) a = a + bb[r * kc] / div;
        }
      }
    } else if (c + 1 < n_chunks) {
      load(c + 1, (int)((c + 1) & 1));
    }
    __syncthreads();  // chunk c consumed and chunk c + 1 in place
  }
  if (t < kc) acc[c0 + t] = a;
}

// The posterior mean's first stage (shard.block_sum): out[b][j] = (((0 +
// x_{bB,j}/div) + x_{bB+1,j}/div) + ...) over the rows of block b (B
// consecutive rows, the last block possibly shorter), strictly in row order --
// the additions of ipmc_host_ordered_sum from zero on each block, so the same
// bits.  Blocks are independent: one lane per (block, column), its loads issued
// kBsUnroll rows ahead of its adds; a block's B dependent adds are the critical
// path (B = 1 024: tens of microseconds for any number of blocks that fits the
// chip), where a whole-column chain over 65 536 rows takes ~0.7 ms.
constexpr int kBsThreads = 256;
constexpr int kBsUnroll = 16;

__global__ __launch_bounds__(kBsThreads) void block_sums_kernel(const double* __restrict__ x, int64_t n_rows, int64_t k,
                                                               int64_t stride, int64_t B, double div,
                                                               double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * kBsThreads + threadIdx.x;
  const int64_t nb = (n_rows + B - 1) / B;
  if (t >= nb * k) return;
  const int64_t b = t / k, j = t - b * k;
  const int64_t r0 = b * B;
  const int64_t rows = (n_rows - r0) < B ? (n_rows - r0) : B;
  const double* p = x + r0 * stride + j;
  double s = 0.0;
  int64_t r = 0;
  for (; r + kBsUnroll <= rows; r += kBsUnroll) {
    double v[kBsUnroll];
#pragma unroll
    for (int u = 0; u < kBsUnroll; ++u) v[u] = p[(r + u) * stride];
    if (div == 1.0) {
#pragma unroll
      for (int u = 0; u < kBsUnroll; ++u) s = s + v[u];
    } else {
#pragma unroll
      for (int u = 0; u < kBsUnroll; ++u) s = s + v[u] / div;
    }
  }
  for (; r < rows; ++r) s = div == 1.0 ? s + p[r * stride] : s + p[r * stride] / div;
  out[b * k + j] = s;
}

}  // namespace ipmc

using namespace ipmc;

extern "C" int ipmc_ordered_sum(const double* rows, int64_t n_rows, int64_t k, int64_t row_stride, double div,
                                double* acc, void* stream) {
  if (n_rows < 0 || k < 0 || row_stride < k) {
    set_error("ipmc_ordered_sum: bad shape (n_rows, k >= 0, row_stride >= k)");
    return IPMC_ERR_INVALID;
  }
  if (n_rows == 0 || k == 0) return IPMC_OK;
  if (!rows || !acc) {
    set_error("ipmc_ordered_sum: NULL pointer");
    return IPMC_ERR_INVALID;
  }
  hipLaunchKernelGGL(ordered_sum_kernel, dim3((unsigned)((k + kOsCols - 1) / kOsCols)), dim3(kOsBlock), 0,
                     (hipStream_t)stream, rows, n_rows, k, row_stride, div, acc);
  return check_launch("ordered_sum_kernel");
}

extern "C" int ipmc_block_sums(const double* rows, int64_t n_rows, int64_t k, int64_t row_stride, int64_t block_rows,
                               double div, double* out, void* stream) {
  if (n_rows < 0 || k < 0 || row_stride < k || block_rows <= 0) {
    set_error("ipmc_block_sums: bad shape (n_rows, k >= 0, row_stride >= k, block_rows > 0)");
    return IPMC_ERR_INVALID;
  }
  if (n_rows == 0 || k == 0) return IPMC_OK;
  if (!rows || !out) {
    set_error("ipmc_block_sums: NULL pointer");
    return IPMC_ERR_INVALID;
  }
  const int64_t lanes = (n_rows + block_rows - 1) / block_rows * k;
  hipLaunchKernelGGL(block_sums_kernel, dim3((unsigned)((lanes + kBsThreads - 1) / kBsThreads)), dim3(kBsThreads), 0,
                     (hipStream_t)stream, rows, n_rows, k, row_stride, block_rows, div, out);
  return check_launch("block_sums_kernel");
}

extern "C" int ipmc_burn_in(const void* x, int32_t dtype, int64_t n_chains, int32_t n_vars, int64_t len,
                            int64_t stride_chain, int64_t stride_var, int64_t stride_t, int32_t window,
                            double threshold, uint32_t* flags_scratch, int64_t* out, void* stream) {
  if (n_chains < 0 || n_vars <= 0 || len < 0 || window <= 0) {
    set_error("ipmc_burn_in: bad sizes (n_vars and window must be positive)");
    return IPMC_ERR_INVALID;
  }
  if (n_chains == 0) return IPMC_OK;
  if (len < window) {
    set_error("ipmc_burn_in: series of %lld samples shorter than the window %d", (long long)len, window);
    return IPMC_ERR_INVALID;
  }
  if (!x || !out || !flags_scratch) {
    set_error("ipmc_burn_in: NULL pointer");
    return IPMC_ERR_INVALID;
  }
  if (dtype != IPMC_F64 && dtype != IPMC_F32) {
    set_error("ipmc_burn_in: bad dtype");
    return IPMC_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t words = (len + 31) / 32;
  if (hipMemsetAsync(flags_scratch, 0, (size_t)(n_chains * words) * sizeof(uint32_t), st) != hipSuccess) {
    set_error("ipmc_burn_in: memset failed");
    return IPMC_ERR_DEVICE;
  }
  const int64_t ns = n_chains * n_vars;
  const unsigned nb = (unsigned)((ns + 255) / 256);
  if (dtype == IPMC_F64)
    hipLaunchKernelGGL(burn_in_flags_kernel<double>, dim3(nb), dim3(256), 0, st, (const double*)x, n_chains, n_vars,
                       len, stride_chain, stride_var, stride_t, window, threshold, (unsigned*)flags_scratch, words);
  else
    hipLaunchKernelGGL(burn_in_flags_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)x, n_chains, n_vars,
                       len, stride_chain, stride_var, stride_t, window, threshold, (unsigned*)flags_scratch, words);
  int rc = check_launch("burn_in_flags_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(burn_in_search_kernel, dim3((unsigned)((n_chains + 255) / 256)), dim3(256), 0, st, n_chains, len,
                     window, (const unsigned*)flags_scratch, words, out);
  return check_launch("burn_in_search_kernel");
}

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
  if (max_lag > len) {
    set_error("ipmc_autocorr: max_lag %d exceeds the series length %lld", max_lag, (long long)len);
    return IPMC_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  if (len > kAcMaxLen) {
    if (n_series > 0x7fffffff) {
      set_error("ipmc_autocorr: at most 2^31 - 1 long series per call");
      return IPMC_ERR_INVALID;
    }
    const dim3 grid((unsigned)n_series, (unsigned)((max_lag + kAcBlock - 1) / kAcBlock));
    if (dtype == IPMC_F64)
      hipLaunchKernelGGL(autocorr_long_kernel<double>, grid, dim3(kAcBlock), 0, st, (const double*)x, n_series, len,
                         stride_series, stride_t, max_lag, out);
    else if (dtype == IPMC_F32)
      hipLaunchKernelGGL(autocorr_long_kernel<float>, grid, dim3(kAcBlock), 0, st, (const float*)x, n_series, len,
                         stride_series, stride_t, max_lag, out);
    else {
      set_error("ipmc_autocorr: bad dtype");
      return IPMC_ERR_INVALID;
    }
    return check_launch("autocorr_long_kernel");
  }
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
