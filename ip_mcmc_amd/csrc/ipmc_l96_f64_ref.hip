// Lorenz-96 kernels, fp64 instantiations, REFERENCE arithmetic (no FMA; lorenz.py:77-81).
#include "ipmc_l96_dispatch.hpp"

namespace ipmc {

int l96_sweep_f64_ref(const ipmc_model& m, const ipmc_sweep& s, int lpc, int spec, hipStream_t st) {
  return l96_sweep_tf<double, false>(m, s, lpc, spec, st);
}
int l96_eval_f64_ref(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                     bool phi, int lpc, hipStream_t st) {
  return l96_eval_tf<double, false>(m, n, u, y, ginv, out, phi, lpc, st);
}

}  // namespace ipmc
