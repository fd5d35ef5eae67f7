// Lorenz-96 kernels, fp32 instantiations, REFERENCE arithmetic (no FMA; lorenz.py:77-81).
#include "ipmc_l96_dispatch.hpp"

namespace ipmc {

int l96_sweep_f32_ref(const ipmc_model& m, const ipmc_sweep& s, int lpc, int cpl, int spec, hipStream_t st) {
  return cpl == 2 ? l96_sweep_pk_f<false>(m, s, lpc, st) : l96_sweep_tf<float, false>(m, s, lpc, spec, st);
}
int l96_eval_f32_ref(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                     bool phi, int lpc, hipStream_t st) {
  return l96_eval_tf<float, false>(m, n, u, y, ginv, out, phi, lpc, st);
}

}  // namespace ipmc
