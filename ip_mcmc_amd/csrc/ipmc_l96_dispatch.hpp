// Lorenz-96 instantiation table and launchers (included by ipmc_l96_f32.hip
// and ipmc_l96_f64.hip, one dtype per translation unit so they build in parallel).
#pragma once

#include "ipmc_internal.hpp"
#include "ipmc_l96.hpp"

namespace ipmc {

// State dims with a compiled kernel. Each (D, LPC) needs M = D/LPC >= 2
// components per lane and at most 160 B of state per lane-array (6 arrays of
// M live in VGPRs).
#define IPMC_L96_DIMS(X) \
  X(4) X(6) X(8) X(10) X(12) X(16) X(20) X(24) X(32) X(36) X(40) X(48) X(60) X(64) X(80) X(128) X(160) X(256)

template <typename T, int D, int LPC>
constexpr bool l96_ok() {
  return LPC <= 16 && D % LPC == 0 && D / LPC >= 2 && (D / LPC) * (int)sizeof(T) <= 160;
}

// An (D, LPC) pair with no instantiation: report it through ipmc_last_error.
inline int l96_unsupported(const ipmc_model& m, int lpc, const char* what) {
  set_error("Lorenz-96: no %s kernel compiled for dim=%d lanes_per_chain=%d", what, m.dim, lpc);
  return IPMC_ERR_UNSUPPORTED;
}

// spec > 1: the speculative kernel with spec slots of LPC lanes per chain.
template <typename T, int D, int LPC, bool FM>
int l96_launch_sweep(const ipmc_model& m, const ipmc_sweep& s, int spec, hipStream_t st) {
  if (spec > 1) {
    const int64_t blocks = (s.n_chains * LPC * spec + kL96Block - 1) / kL96Block;
    hipLaunchKernelGGL((l96_spec_kernel<T, D, LPC, FM>), dim3((unsigned)blocks), dim3(kL96Block), 0, st, m, s,
                       spec);
    return check_launch("l96_spec_kernel");
  }
  const int64_t threads = s.n_chains * LPC;
  const int64_t blocks = (threads + kL96Block - 1) / kL96Block;
  hipLaunchKernelGGL((l96_sweep_kernel<T, D, LPC, FM>), dim3((unsigned)blocks), dim3(kL96Block), 0, st, m, s);
  return check_launch("l96_sweep_kernel");
}

template <typename T, int D, int LPC, bool FM>
int l96_launch_eval(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                    bool phi, hipStream_t st) {
  const int64_t threads = n * LPC;
  const int64_t blocks = (threads + kL96Block - 1) / kL96Block;
  if (phi)
    hipLaunchKernelGGL((l96_eval_kernel<T, D, LPC, FM, true>), dim3((unsigned)blocks), dim3(kL96Block), 0, st, m, n,
                       (const T*)u, (const T*)y, (const T*)ginv, (T*)out);
  else
    hipLaunchKernelGGL((l96_eval_kernel<T, D, LPC, FM, false>), dim3((unsigned)blocks), dim3(kL96Block), 0, st, m,
                       n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);
  return check_launch("l96_eval_kernel");
}

template <typename T, int D, bool FM>
int l96_sweep_d(const ipmc_model& m, const ipmc_sweep& s, int lpc, int spec, hipStream_t st) {
  switch (lpc) {
#define IPMC_CASE(L)                                                                         \
  case L:                                                                                    \
    if constexpr (l96_ok<T, D, L>()) return l96_launch_sweep<T, D, L, FM>(m, s, spec, st); \
    break;
    IPMC_CASE(1) IPMC_CASE(2) IPMC_CASE(4) IPMC_CASE(8) IPMC_CASE(16)
#undef IPMC_CASE
  }
  return l96_unsupported(m, lpc, "sweep");
}

template <int D, int LPC, bool FM>
int l96_launch_sweep_pk(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  const int64_t pairs = (s.n_chains + 1) / 2;
  const int64_t blocks = (pairs * LPC + kL96Block - 1) / kL96Block;
  hipLaunchKernelGGL((l96_sweep_pk_kernel<D, LPC, FM>), dim3((unsigned)blocks), dim3(kL96Block), 0, st, m, s);
  return check_launch("l96_sweep_pk_kernel");
}

// packed fp32 pairs: 8 bytes of storage per component, like fp64
template <int D, bool FM>
int l96_sweep_pk_d(const ipmc_model& m, const ipmc_sweep& s, int lpc, hipStream_t st) {
  switch (lpc) {
#define IPMC_CASE(L)                                                                     \
  case L:                                                                                \
    if constexpr (l96_ok<double, D, L>()) return l96_launch_sweep_pk<D, L, FM>(m, s, st); \
    break;
    IPMC_CASE(1) IPMC_CASE(2) IPMC_CASE(4) IPMC_CASE(8) IPMC_CASE(16)
#undef IPMC_CASE
  }
  return l96_unsupported(m, lpc, "packed fp32 sweep");
}

// The dispatchers below take the arithmetic mode as a template argument: each
// (dtype, mode) pair is its own translation unit (ipmc_l96_f{32,64}{,_ref}.hip),
// so the four build in parallel.
template <bool FM>
int l96_sweep_pk_f(const ipmc_model& m, const ipmc_sweep& s, int lpc, hipStream_t st) {
  switch (m.dim) {
#define IPMC_DIM(D) \
  case D: return l96_sweep_pk_d<D, FM>(m, s, lpc, st);
    IPMC_L96_DIMS(IPMC_DIM)
#undef IPMC_DIM
  }
  return l96_unsupported(m, lpc, "dimension's");
}

template <typename T, int D, bool FM>
int l96_eval_d(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
               int lpc, hipStream_t st) {
  switch (lpc) {
#define IPMC_CASE(L)                                                                                  \
  case L:                                                                                             \
    if constexpr (l96_ok<T, D, L>()) return l96_launch_eval<T, D, L, FM>(m, n, u, y, ginv, out, phi, st); \
    break;
    IPMC_CASE(1) IPMC_CASE(2) IPMC_CASE(4) IPMC_CASE(8) IPMC_CASE(16)
#undef IPMC_CASE
  }
  return l96_unsupported(m, lpc, "evaluation");
}

template <typename T, bool FM>
int l96_sweep_tf(const ipmc_model& m, const ipmc_sweep& s, int lpc, int spec, hipStream_t st) {
  switch (m.dim) {
#define IPMC_DIM(D) \
  case D: return l96_sweep_d<T, D, FM>(m, s, lpc, spec, st);
    IPMC_L96_DIMS(IPMC_DIM)
#undef IPMC_DIM
  }
  return l96_unsupported(m, lpc, "dimension's");
}

template <typename T, bool FM>
int l96_eval_tf(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
                int lpc, hipStream_t st) {
  switch (m.dim) {
#define IPMC_DIM(D) \
  case D: return l96_eval_d<T, D, FM>(m, n, u, y, ginv, out, phi, lpc, st);
    IPMC_L96_DIMS(IPMC_DIM)
#undef IPMC_DIM
  }
  return l96_unsupported(m, lpc, "dimension's");
}

template <typename T, int D>
bool l96_has_d(int lpc) {
  switch (lpc) {
    case 1: return l96_ok<T, D, 1>();
    case 2: return l96_ok<T, D, 2>();
    case 4: return l96_ok<T, D, 4>();
    case 8: return l96_ok<T, D, 8>();
    case 16: return l96_ok<T, D, 16>();
  }
  return false;
}

template <typename T>
bool l96_has_t(int D, int lpc) {
  switch (D) {
#define IPMC_DIM(DD) \
  case DD: return l96_has_d<T, DD>(lpc);
    IPMC_L96_DIMS(IPMC_DIM)
#undef IPMC_DIM
  }
  return false;
}

}  // namespace ipmc
