// Burgers (Rusanov FV + SSPRK2) kernels — placeholder until the wave-cooperative kernel lands.
#include "ipmc_internal.hpp"

namespace ipmc {

int burgers_sweep(const ipmc_model&, const ipmc_sweep&, hipStream_t) {
  set_error("Burgers sweep: not built yet");
  return IPMC_ERR_UNSUPPORTED;
}
int burgers_eval(const ipmc_model&, int32_t, int64_t, const void*, const void*, const void*, void*, bool,
                 hipStream_t) {
  set_error("Burgers eval: not built yet");
  return IPMC_ERR_UNSUPPORTED;
}

}  // namespace ipmc
