// Lorenz-96 kernels, fp64 instantiations, FMA arithmetic (REFERENCE:
// ipmc_l96_f64_ref.hip; one mode per translation unit so they build in parallel).
#include "ipmc_l96_dispatch.hpp"

namespace ipmc {

int l96_sweep_f64_ref(const ipmc_model& m, const ipmc_sweep& s, int lpc, int spec, hipStream_t st);
int l96_eval_f64_ref(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                     bool phi, int lpc, hipStream_t st);

int l96_sweep_f64(const ipmc_model& m, const ipmc_sweep& s, int lpc, int spec, hipStream_t st) {
  return m.arith == IPMC_ARITH_FMA ? l96_sweep_tf<double, true>(m, s, lpc, spec, st)
                                   : l96_sweep_f64_ref(m, s, lpc, spec, st);
}
int l96_eval_f64(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
                 int lpc, hipStream_t st) {
  return m.arith == IPMC_ARITH_FMA ? l96_eval_tf<double, true>(m, n, u, y, ginv, out, phi, lpc, st)
                                   : l96_eval_f64_ref(m, n, u, y, ginv, out, phi, lpc, st);
}
bool l96_has_f64(int D, int lpc) { return l96_has_t<double>(D, lpc); }

}  // namespace ipmc
