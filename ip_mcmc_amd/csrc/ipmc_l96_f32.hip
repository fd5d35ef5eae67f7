// Lorenz-96 kernels, fp32 instantiations.
#include "ipmc_l96_dispatch.hpp"

namespace ipmc {

int l96_sweep_f32(const ipmc_model& m, const ipmc_sweep& s, int lpc, int cpl, int spec, hipStream_t st) {
  return cpl == 2 ? l96_sweep_pk(m, s, lpc, st) : l96_sweep_t<float>(m, s, lpc, spec, st);
}
int l96_eval_f32(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
                 int lpc, hipStream_t st) {
  return l96_eval_t<float>(m, n, u, y, ginv, out, phi, lpc, st);
}
bool l96_has_f32(int D, int lpc, int cpl) {
  return cpl == 2 ? l96_has_t<double>(D, lpc) : l96_has_t<float>(D, lpc);
}

}  // namespace ipmc
