// Lorenz-96 kernels, fp32 instantiations (one chain per lane group, and two
// packed as f32x2), FMA arithmetic (REFERENCE: ipmc_l96_f32_ref.hip; one mode
// per translation unit so they build in parallel).
// The lane-state park (IPMC_L96_PARK, ipmc_l96.hpp) is an fp64 occupancy device
// (two waves at 17-20 components per lane).  In this unit it changes no
// kernel's occupancy, yet with it the compiler schedules the packed sweep's RK
// loop differently (the same 427 instructions, reordered): 1.85 instead of
// 1.67 ms per headline f32 sweep, three interleaved A/Bs
// (profiles/r5/f32_ab.jsonl).  Off here: the round-4 code and schedule.
#define IPMC_L96_PARK 0
#include "ipmc_l96_dispatch.hpp"

namespace ipmc {

int l96_sweep_f32_ref(const ipmc_model& m, const ipmc_sweep& s, int lpc, int cpl, int spec, hipStream_t st);
int l96_eval_f32_ref(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                     bool phi, int lpc, hipStream_t st);

int l96_sweep_f32(const ipmc_model& m, const ipmc_sweep& s, int lpc, int cpl, int spec, hipStream_t st) {
  if (m.arith != IPMC_ARITH_FMA) return l96_sweep_f32_ref(m, s, lpc, cpl, spec, st);
  return cpl == 2 ? l96_sweep_pk_f<true>(m, s, lpc, st) : l96_sweep_tf<float, true>(m, s, lpc, spec, st);
}
int l96_eval_f32(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
                 int lpc, hipStream_t st) {
  return m.arith == IPMC_ARITH_FMA ? l96_eval_tf<float, true>(m, n, u, y, ginv, out, phi, lpc, st)
                                   : l96_eval_f32_ref(m, n, u, y, ginv, out, phi, lpc, st);
}
bool l96_has_f32(int D, int lpc, int cpl) {
  return cpl == 2 ? l96_has_t<double>(D, lpc) : l96_has_t<float>(D, lpc);
}

}  // namespace ipmc
