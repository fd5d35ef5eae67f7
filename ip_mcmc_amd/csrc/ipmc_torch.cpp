// torch.ops.ipmc.* — the TORCH_LIBRARY front end of libipmc (SURVEY §8(b):
// "a torch op via TORCH_LIBRARY ... a C-ABI twin for non-torch callers").
//
// Each op checks its tensors (device, dtype, contiguity, shape) and calls the
// C-ABI entry point of include/ipmc.h on the given HIP stream; there is no
// compute here and no CPU kernel: the ops are registered for the CUDA (= HIP
// on ROCm) dispatch key only, so a CPU tensor raises instead of falling back.
//
// `model` is the address of an ipmc_model (host struct whose arrays are device
// pointers) built by ObservationOperator.model() and kept alive by the caller;
// `stream` is a hipStream_t as an integer (torch.cuda.current_stream().cuda_stream).
#include <torch/library.h>

#include <optional>

#include "../../include/ipmc.h"

namespace {

void check_rc(int rc, const char* fn) { TORCH_CHECK(rc == IPMC_OK, fn, " failed (", rc, "): ", ipmc_last_error()); }

int32_t real_dtype(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kDouble || t.scalar_type() == at::kFloat, name, " must be float32 or float64");
  return t.scalar_type() == at::kDouble ? IPMC_F64 : IPMC_F32;
}

void dense(const at::Tensor& t, const char* name, const at::Tensor& like) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.device() == like.device(), name, " must be on ", like.device());
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void same_real(const at::Tensor& t, const char* name, const at::Tensor& u, int64_t numel) {
  dense(t, name, u);
  TORCH_CHECK(t.scalar_type() == u.scalar_type(), name, " must have u's dtype");
  TORCH_CHECK(t.numel() == numel, name, " must have ", numel, " elements, not ", t.numel());
}

const ipmc_model* as_model(int64_t model) {
  TORCH_CHECK(model != 0, "model must be the address of an ipmc_model (ObservationOperator.model())");
  return reinterpret_cast<const ipmc_model*>(static_cast<intptr_t>(model));
}

// n_steps pCN steps of every chain, u / phi / accepts updated in place
// (ipmc_pcn_sweep; MCMCSampler.run's fast path, sampler.py:12-41).
void pcn_sweep(at::Tensor u, at::Tensor phi, at::Tensor accepts, const at::Tensor& y, const at::Tensor& gamma_inv,
               const at::Tensor& prior_sqrt, int64_t model, double beta, double contraction, int64_t seed,
               int64_t chain_offset, int64_t step0, int64_t n_steps, int64_t stream, int64_t proposal,
               std::optional<at::Tensor> sum_u, std::optional<at::Tensor> sum_u2) {
  const ipmc_model* m = as_model(model);
  TORCH_CHECK(u.dim() == 2 && u.size(1) == m->k, "u must be [n_chains, ", m->k, "]");
  dense(u, "u", u);
  const int32_t dt = real_dtype(u, "u");
  const int64_t C = u.size(0);
  same_real(phi, "phi", u, C);
  dense(accepts, "accepts", u);
  TORCH_CHECK(accepts.scalar_type() == at::kLong && accepts.numel() == C, "accepts must be int64 [n_chains]");
  same_real(y, "y", u, m->q);
  same_real(gamma_inv, "gamma_inv", u, m->q);
  same_real(prior_sqrt, "prior_sqrt", u, m->k);
  ipmc_sweep s{};
  s.dtype = dt;
  s.n_chains = C;
  s.chain_offset = chain_offset;
  s.u = u.data_ptr();
  s.phi = phi.data_ptr();
  s.accepts = accepts.data_ptr<int64_t>();
  s.y = y.data_ptr();
  s.gamma_inv = gamma_inv.data_ptr();
  s.prior_sqrt = prior_sqrt.data_ptr();
  s.beta = beta;
  s.contraction = contraction;
  s.proposal = static_cast<int32_t>(proposal);
  s.seed = static_cast<uint64_t>(seed);
  s.step0 = static_cast<uint64_t>(step0);
  s.n_steps = n_steps;
  for (auto* acc : {&sum_u, &sum_u2}) {
    if (!acc->has_value()) continue;
    const at::Tensor& t = acc->value();
    dense(t, "sum_u/sum_u2", u);
    TORCH_CHECK(t.scalar_type() == at::kDouble && t.numel() == C * m->k, "sum_u/sum_u2 must be float64 [n_chains, k]");
  }
  if (sum_u.has_value()) s.sum_u = sum_u->data_ptr<double>();
  if (sum_u2.has_value()) {
    TORCH_CHECK(sum_u.has_value(), "sum_u2 needs sum_u");
    s.sum_u2 = sum_u2->data_ptr<double>();
  }
  check_rc(ipmc_pcn_sweep(m, &s, reinterpret_cast<void*>(static_cast<intptr_t>(stream))), "ipmc_pcn_sweep");
}

// phi[c] = Φ(u_c) (ipmc_potential; EvolutionPotential.__call__ minus the constant, potential.py:53-54).
void potential(const at::Tensor& u, const at::Tensor& y, const at::Tensor& gamma_inv, at::Tensor phi, int64_t model,
               int64_t stream) {
  const ipmc_model* m = as_model(model);
  TORCH_CHECK(u.dim() == 2 && u.size(1) == m->k, "u must be [n, ", m->k, "]");
  dense(u, "u", u);
  const int32_t dt = real_dtype(u, "u");
  same_real(y, "y", u, m->q);
  same_real(gamma_inv, "gamma_inv", u, m->q);
  same_real(phi, "phi", u, u.size(0));
  check_rc(ipmc_potential(m, dt, u.size(0), u.data_ptr(), y.data_ptr(), gamma_inv.data_ptr(), phi.data_ptr(),
                          reinterpret_cast<void*>(static_cast<intptr_t>(stream))),
           "ipmc_potential");
}

// g[c] = G(u_c) (ipmc_forward; the observation operators of lorenz_mcmc.py, stuart_examples.py, utilities.py).
void forward(const at::Tensor& u, at::Tensor g, int64_t model, int64_t stream) {
  const ipmc_model* m = as_model(model);
  TORCH_CHECK(u.dim() == 2 && u.size(1) == m->k, "u must be [n, ", m->k, "]");
  dense(u, "u", u);
  const int32_t dt = real_dtype(u, "u");
  same_real(g, "g", u, u.size(0) * m->q);
  check_rc(ipmc_forward(m, dt, u.size(0), u.data_ptr(), g.data_ptr(),
                        reinterpret_cast<void*>(static_cast<intptr_t>(stream))),
           "ipmc_forward");
}

// the header this front end was compiled against (torch_ops.load() compares it
// with the ctypes mirror, so a stale build that would pass stale structs raises)
int64_t abi_version() { return IPMC_ABI_VERSION; }

}  // namespace

TORCH_LIBRARY(ipmc, m) {
  m.def(
      "pcn_sweep(Tensor(a!) u, Tensor(b!) phi, Tensor(c!) accepts, Tensor y, Tensor gamma_inv, Tensor prior_sqrt, "
      "int model, float beta, float contraction, int seed, int chain_offset, int step0, int n_steps, int stream=0, "
      "int proposal=0, Tensor(d!)? sum_u=None, Tensor(e!)? sum_u2=None) -> ()");
  m.def("potential(Tensor u, Tensor y, Tensor gamma_inv, Tensor(a!) phi, int model, int stream=0) -> ()");
  m.def("forward(Tensor u, Tensor(a!) g, int model, int stream=0) -> ()");
  m.def("abi_version() -> int", &abi_version);
}

TORCH_LIBRARY_IMPL(ipmc, CUDA, m) {
  m.impl("pcn_sweep", &pcn_sweep);
  m.impl("potential", &potential);
  m.impl("forward", &forward);
}
