// A non-Python caller of the C-ABI (include/ipmc.h): the headline problem's
// pCN sweep from plain host C++ -- hipMalloc'ed buffers, ipmc_model /
// ipmc_sweep filled by hand, ipmc_init_phi + ipmc_pcn_sweep on a stream.
// This is what a C, C++, Go (cgo) or Rust (FFI) binding of the reference's hot
// path does.
//
//   l96_pcn [n_chains] [n_steps] [--dump file]
//
// Problem: single-scale Lorenz-96 d=40, forcing F = 8 + u, x0 = 8 + 0.01 e_0,
// RK4 dt = 0.005 for 200 steps, y_k = 8 + (k mod 5)/8, 1/γ = 10, prior N(0, I),
// pCN β = 0.2, seed 7, u_0[c][k] = ((7c + 13k) mod 17 − 8)/64 (every input is
// exactly representable, so tests/test_gpu_c_api.py rebuilds it in numpy and
// checks the result against the CPU oracle bit for bit).  Prints one JSON line;
// --dump writes u [n, 40] f64, Φ [n] f64 and accepts [n] int64.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ipmc.h"

#define HIP_OK(x)                                                             \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(2);                                                           \
    }                                                                         \
  } while (0)
#define IPMC_OK_(x)                                                           \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_ != IPMC_OK) {                                                     \
      std::fprintf(stderr, "%s -> %d: %s\n", #x, rc_, ipmc_last_error());     \
      std::exit(3);                                                           \
    }                                                                         \
  } while (0)

template <typename T>
static T* to_device(const std::vector<T>& h) {
  T* d = nullptr;
  HIP_OK(hipMalloc(&d, h.size() * sizeof(T)));
  HIP_OK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  int64_t n = 4096, steps = 10;
  const char* dump = nullptr;
  int pos = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--dump") && i + 1 < argc) dump = argv[++i];
    else if (pos == 0) n = std::atoll(argv[i]), ++pos;
    else steps = std::atoll(argv[i]);
  }
  if (ipmc_abi_version() != IPMC_ABI_VERSION) {
    std::fprintf(stderr, "libipmc ABI %d, header %d\n", ipmc_abi_version(), IPMC_ABI_VERSION);
    return 4;
  }
  const int D = 40;
  std::vector<double> x0(D, 8.0), th0(D, 8.0), y(D), ginv(D, 10.0), sq(D, 1.0), u(n * D), phi(n);
  std::vector<int64_t> acc(n, 0);
  x0[0] += 0.01;
  for (int k = 0; k < D; ++k) y[k] = 8.0 + (k % 5) / 8.0;
  for (int64_t c = 0; c < n; ++c)
    for (int k = 0; k < D; ++k) u[c * D + k] = (double)((7 * c + 13 * k) % 17 - 8) / 64.0;

  double *dx0 = to_device(x0), *dth0 = to_device(th0), *dy = to_device(y), *dg = to_device(ginv),
         *dsq = to_device(sq), *du = to_device(u), *dphi = to_device(phi);
  int64_t* dacc = to_device(acc);
  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));

  ipmc_model m;
  std::memset(&m, 0, sizeof m);
  m.kind = IPMC_MODEL_LORENZ96;
  m.arith = IPMC_ARITH_FMA;
  m.k = m.q = m.dim = D;
  m.n_steps = 200;
  m.dt = 0.005;
  m.x0 = dx0;
  m.theta0 = dth0;

  ipmc_sweep s;
  std::memset(&s, 0, sizeof s);
  s.dtype = IPMC_F64;
  s.n_chains = n;
  s.u = du;
  s.phi = dphi;
  s.accepts = dacc;
  s.y = dy;
  s.gamma_inv = dg;
  s.prior_sqrt = dsq;
  s.beta = 0.2;
  s.contraction = std::sqrt(1.0 - s.beta * s.beta);
  s.proposal = IPMC_PROPOSAL_PCN;
  s.seed = 7;
  s.step0 = 0;
  s.n_steps = steps;

  ipmc_plan plan;
  IPMC_OK_(ipmc_plan_sweep(&m, &s, &plan));
  IPMC_OK_(ipmc_init_phi(&m, &s, st));
  hipEvent_t a, b;
  HIP_OK(hipEventCreate(&a));
  HIP_OK(hipEventCreate(&b));
  HIP_OK(hipEventRecord(a, st));
  IPMC_OK_(ipmc_pcn_sweep(&m, &s, st));
  HIP_OK(hipEventRecord(b, st));
  HIP_OK(hipStreamSynchronize(st));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, a, b));

  HIP_OK(hipMemcpy(u.data(), du, u.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(phi.data(), dphi, phi.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(acc.data(), dacc, acc.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
  int64_t total = 0;
  double usum = 0.0;
  for (int64_t c = 0; c < n; ++c) total += acc[c];
  for (double v : u) usum += v;
  std::printf("{\"chains\": %lld, \"pcn_steps\": %lld, \"accepts\": %lld, \"sum_u\": %.17g, \"sweep_ms\": %.4f, "
              "\"pcn_steps_per_s\": %.6g, \"lanes_per_chain\": %d, \"spec_width\": %d}\n",
              (long long)n, (long long)steps, (long long)total, usum, ms, n * steps / (ms * 1e-3),
              plan.lanes_per_chain, plan.spec_width);
  if (dump) {
    FILE* f = std::fopen(dump, "wb");
    if (!f) return 5;
    std::fwrite(u.data(), sizeof(double), u.size(), f);
    std::fwrite(phi.data(), sizeof(double), phi.size(), f);
    std::fwrite(acc.data(), sizeof(int64_t), acc.size(), f);
    std::fclose(f);
  }
  for (void* p : {(void*)dx0, (void*)dth0, (void*)dy, (void*)dg, (void*)dsq, (void*)du, (void*)dphi, (void*)dacc})
    HIP_OK(hipFree(p));
  HIP_OK(hipStreamDestroy(st));
  return 0;
}
