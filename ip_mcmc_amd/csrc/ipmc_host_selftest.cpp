// Sanitizer driver for libipmc_host.so's source (ipmc_host.cpp), host code only:
//   make -C ip_mcmc_amd/csrc host-asan   (-fsanitize=address,undefined)
//   make -C ip_mcmc_amd/csrc host-tsan   (-fsanitize=thread: parallel_for's slices)
// run by tests/test_host_sanitized.py.  Drives every entry point of
// include/ipmc_host.h on ragged shapes -- thread counts that do not divide the
// element count, the Cholesky-prior path, f32 and f64, row_stride > k,
// div != 1, empty inputs -- and every error return.  Each result is also
// checked: the threaded draws equal the one-thread draws and ipmc_rng.hpp's
// element functions, the ordered sum equals a plain loop in row order.
// Prints "host selftest ok" and exits 0, or names the first failed check.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ipmc.h"
#include "../../include/ipmc_host.h"
#include "ipmc_rng.hpp"

namespace {

int g_checks = 0;

void check(bool ok, const char* what) {
  ++g_checks;
  if (!ok) {
    std::fprintf(stderr, "FAILED: %s (%s)\n", what, ipmc_host_last_error());
    std::exit(1);
  }
}

void expect_error(int rc, const char* what) {
  check(rc == IPMC_ERR_INVALID, what);
  check(std::strlen(ipmc_host_last_error()) > 0, "an error leaves a message");
}

template <typename T>
bool same_bits(const std::vector<T>& a, const std::vector<T>& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0;
}

template <typename T>
void draws_case(int64_t n_chains, int64_t n_steps, int k, bool chol, uint64_t seed, int64_t c_off, uint64_t step0) {
  const int dt = sizeof(T) == 8 ? IPMC_F64 : IPMC_F32;
  std::vector<T> sq(k), L(chol ? (size_t)k * k : 0);
  for (int j = 0; j < k; ++j) sq[j] = (T)(0.5 + 0.1 * j);
  for (int j = 0; j < k && chol; ++j)
    for (int i = 0; i <= j; ++i) L[(size_t)j * k + i] = (T)(i == j ? 1.0 + 0.01 * j : 0.3 / (1 + j - i));
  const size_t total = (size_t)(n_steps * n_chains * k);
  std::vector<T> w1(total), wt(total);
  std::vector<double> lr1((size_t)(n_steps * n_chains)), lrt(lr1.size());
  const void* psq = chol ? nullptr : sq.data();
  const void* pch = chol ? L.data() : nullptr;
  check(ipmc_host_pcn_draws(seed, c_off, n_chains, step0, n_steps, k, dt, psq, pch, w1.data(), lr1.data(), 1) == 0,
        "pcn_draws, one thread");
  for (int nt : {0, 3, 7, 64}) {
    std::fill(wt.begin(), wt.end(), (T)0);
    check(ipmc_host_pcn_draws(seed, c_off, n_chains, step0, n_steps, k, dt, psq, pch, wt.data(), lrt.data(), nt) ==
              0,
          "pcn_draws, threads");
    check(same_bits(w1, wt) && same_bits(lr1, lrt), "threaded draws equal the one-thread draws");
  }
  // log_r may be NULL
  check(ipmc_host_pcn_draws(seed, c_off, n_chains, step0, n_steps, k, dt, psq, pch, wt.data(), nullptr, 5) == 0,
        "pcn_draws without log_r");
  check(same_bits(w1, wt), "draws without log_r");
  // spot checks against the element functions
  for (int64_t s = 0; s < n_steps; s += std::max<int64_t>(1, n_steps / 3))
    for (int64_t c = 0; c < n_chains; c += std::max<int64_t>(1, n_chains / 5)) {
      const uint64_t gid = (uint64_t)(c_off + c), st = step0 + (uint64_t)s;
      for (int j = 0; j < k; ++j) {
        const T e = ipmc::draw_w<T>(seed, gid, st, j, k, chol ? nullptr : sq.data(), chol ? L.data() : nullptr);
        check(std::memcmp(&e, &w1[(size_t)((s * n_chains + c) * k + j)], sizeof(T)) == 0, "w element");
      }
      const double l = ipmc::det_log(ipmc::accept_uniform(seed, gid, st));
      check(std::memcmp(&l, &lr1[(size_t)(s * n_chains + c)], 8) == 0, "log r element");
    }
}

void ordered_sum_case(int64_t n_rows, int64_t k, int64_t stride, double div) {
  std::vector<double> rows((size_t)std::max<int64_t>(1, n_rows * stride));
  for (size_t i = 0; i < rows.size(); ++i) rows[i] = std::sin(0.37 * (double)i) * (1.0 + (double)(i % 11));
  std::vector<double> acc(k), ref(k);
  for (int64_t j = 0; j < k; ++j) acc[j] = ref[j] = 0.25 * (double)j;
  check(ipmc_host_ordered_sum(rows.data(), n_rows, k, stride, div, acc.data()) == 0, "ordered_sum");
  for (int64_t r = 0; r < n_rows; ++r)
    for (int64_t j = 0; j < k; ++j) {
      const double x = rows[(size_t)(r * stride + j)];
      ref[j] = ref[j] + (div == 1.0 ? x : x / div);
    }
  check(same_bits(acc, ref), "ordered_sum equals the row-order loop");
}

}  // namespace

int main() {
  check(ipmc_host_abi_version() == IPMC_HOST_ABI_VERSION, "abi version");

  // draws: single-thread sizes, and blocks above the parallel threshold whose
  // element count no thread count divides
  draws_case<double>(1, 5, 4, false, 7, 0, 0);
  draws_case<float>(3, 2, 5, true, 7, 11, 100);
  draws_case<double>(4097, 7, 3, false, 0xFFFFFFFFFFFFFFFFull, 0, 0);
  draws_case<double>(1031, 13, 7, true, 42, (int64_t(1) << 32) - 1031, (uint64_t(1) << 63) - 13);
  draws_case<float>(2053, 9, 5, false, 3, 5, 17);
  draws_case<float>(997, 11, 9, true, 3, 5, 17);
  {
    std::vector<double> w(8);
    check(ipmc_host_pcn_draws(1, 0, 0, 0, 5, 4, IPMC_F64, nullptr, nullptr, nullptr, nullptr, 1) == 0,
          "zero chains is a no-op");
    check(ipmc_host_pcn_draws(1, 0, 3, 0, 0, 4, IPMC_F64, nullptr, nullptr, nullptr, nullptr, 1) == 0,
          "zero steps is a no-op");
    const double sq[4] = {1, 1, 1, 1};
    expect_error(ipmc_host_pcn_draws(1, 0, 1, 0, 1, 0, IPMC_F64, sq, nullptr, w.data(), nullptr, 1), "k = 0");
    expect_error(ipmc_host_pcn_draws(1, 0, 1, 0, -1, 4, IPMC_F64, sq, nullptr, w.data(), nullptr, 1), "n_steps < 0");
    expect_error(ipmc_host_pcn_draws(1, -1, 1, 0, 1, 4, IPMC_F64, sq, nullptr, w.data(), nullptr, 1),
                 "negative chain offset");
    expect_error(ipmc_host_pcn_draws(1, 0, -1, 0, 1, 4, IPMC_F64, sq, nullptr, w.data(), nullptr, 1),
                 "negative chain count");
    expect_error(ipmc_host_pcn_draws(1, int64_t(1) << 32, 1, 0, 1, 4, IPMC_F64, sq, nullptr, w.data(), nullptr, 1),
                 "chain ids beyond 2^32");
    expect_error(ipmc_host_pcn_draws(1, 0, 1, 0, 1, 4, 99, sq, nullptr, w.data(), nullptr, 1), "bad dtype");
    expect_error(ipmc_host_pcn_draws(1, 0, 1, uint64_t(1) << 63, 1, 4, IPMC_F64, sq, nullptr, w.data(), nullptr, 1),
                 "steps at 2^63");
    expect_error(ipmc_host_pcn_draws(1, 0, 1, (uint64_t(1) << 63) - 1, 2, 4, IPMC_F64, sq, nullptr, w.data(), nullptr,
                                     1),
                 "steps crossing 2^63");
    expect_error(ipmc_host_pcn_draws(1, 0, 1, 0, 1, 4, IPMC_F64, sq, nullptr, nullptr, nullptr, 1), "w NULL");
    expect_error(ipmc_host_pcn_draws(1, 0, 1, 0, 1, 4, IPMC_F64, nullptr, nullptr, w.data(), nullptr, 1),
                 "no prior");
    expect_error(ipmc_host_pcn_draws(1, 0, int64_t(1) << 31, 0, int64_t(1) << 40, 64, IPMC_F64, sq, nullptr, w.data(),
                                     nullptr, 1),
                 "element count overflow");
  }

  // normals and uniforms: the element functions, ragged k, both dtypes
  for (int k : {0, 1, 5, 40}) {
    const int64_t n = 37, off = 1000;
    std::vector<double> z64((size_t)(n * k) + 1);
    std::vector<float> z32((size_t)(n * k) + 1);
    check(ipmc_host_normal(9, off, n, 123, k, IPMC_F64, z64.data()) == 0, "normal f64");
    check(ipmc_host_normal(9, off, n, 123, k, IPMC_F32, z32.data()) == 0, "normal f32");
    for (int64_t i = 0; i < n * k; ++i) {
      const double e = ipmc::normal_component(9, (uint64_t)(off + i / k), 123, (int)(i % k));
      check(std::memcmp(&e, &z64[(size_t)i], 8) == 0 && z32[(size_t)i] == (float)e, "normal element");
    }
  }
  expect_error(ipmc_host_normal(9, 0, 1, 0, -1, IPMC_F64, nullptr), "normal k < 0");
  expect_error(ipmc_host_normal(9, 0, 1, 0, 3, 7, nullptr), "normal bad dtype");
  expect_error(ipmc_host_normal(9, 0, 1, 0, 3, IPMC_F64, nullptr), "normal out NULL");
  expect_error(ipmc_host_normal(9, (int64_t(1) << 32) - 1, 2, 0, 3, IPMC_F64, nullptr), "normal chain range");
  check(ipmc_host_normal(9, 0, 0, 0, 3, IPMC_F64, nullptr) == 0, "normal empty");
  {
    std::vector<double> r(33);
    check(ipmc_host_uniform(5, 7, 33, 9, r.data()) == 0, "uniform");
    for (int c = 0; c < 33; ++c) {
      const double e = ipmc::accept_uniform(5, (uint64_t)(7 + c), 9);
      check(r[(size_t)c] == e && e >= 0.0 && e < 1.0, "uniform element");
    }
    expect_error(ipmc_host_uniform(5, 0, 1, 9, nullptr), "uniform out NULL");
    expect_error(ipmc_host_uniform(5, -3, 1, 9, r.data()), "uniform chain range");
    check(ipmc_host_uniform(5, 0, 0, 9, nullptr) == 0, "uniform empty");
    std::vector<double> u(70000);
    check(ipmc_host_step_uniforms(5, 7, 9, 65536, u.data()) == 0, "step uniforms");
    check(u[0] == r[0], "step uniform 0 is the accept uniform");
    check(u[65535] == ipmc::slot_uniform(5, 7, 9, 0xFFFFFFFFu - 65535u), "last step uniform");
    expect_error(ipmc_host_step_uniforms(5, 7, 9, 65537, u.data()), "too many step uniforms");
    expect_error(ipmc_host_step_uniforms(5, -1, 9, 1, u.data()), "step uniforms chain < 0");
    expect_error(ipmc_host_step_uniforms(5, int64_t(1) << 32, 9, 1, u.data()), "step uniforms chain >= 2^32");
    expect_error(ipmc_host_step_uniforms(5, 7, 9, -1, u.data()), "step uniforms n < 0");
    expect_error(ipmc_host_step_uniforms(5, 7, 9, 1, nullptr), "step uniforms out NULL");
    check(ipmc_host_step_uniforms(5, 7, 9, 0, nullptr) == 0, "step uniforms empty");
  }

  // ordered sum: ragged strides, div != 1, empty
  ordered_sum_case(1, 1, 1, 1.0);
  ordered_sum_case(1000, 40, 40, 1.0);
  ordered_sum_case(1000, 40, 123, 1.0);
  ordered_sum_case(333, 257, 300, 7.0);
  ordered_sum_case(5, 3, 3, 0.5);
  ordered_sum_case(0, 4, 4, 2.0);
  {
    double acc[2] = {1, 2};
    check(ipmc_host_ordered_sum(nullptr, 0, 2, 2, 1.0, acc) == 0 && acc[0] == 1 && acc[1] == 2, "no rows");
    check(ipmc_host_ordered_sum(nullptr, 3, 0, 0, 1.0, nullptr) == 0, "no columns");
    expect_error(ipmc_host_ordered_sum(acc, 1, 2, 1, 1.0, acc), "row_stride < k");
    expect_error(ipmc_host_ordered_sum(acc, -1, 2, 2, 1.0, acc), "n_rows < 0");
    expect_error(ipmc_host_ordered_sum(nullptr, 1, 2, 2, 1.0, acc), "rows NULL");
    expect_error(ipmc_host_ordered_sum(acc, 1, 2, 2, 1.0, nullptr), "acc NULL");
  }
  std::printf("host selftest ok: %d checks\n", g_checks);
  return 0;
}
