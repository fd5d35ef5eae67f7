// Host-side internals shared by the libipmc translation units.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/ipmc.h"

namespace ipmc {

// lanes of one Lorenz-96 speculative chain when its slots span a whole block
constexpr int kL96SpecBlockLanes = 256;


void set_error(const char* fmt, ...);
int check_launch(const char* what);

// Lorenz-96 dispatch (ipmc_l96_f{32,64}.hip; REFERENCE arith in ipmc_l96_f{32,64}_ref.hip).
// Returns IPMC_ERR_UNSUPPORTED when (D, lpc) has no instantiation.
// spec > 1: speculative sweep with `spec` slots per chain (one chain per lane group only).
int l96_sweep_f32(const ipmc_model& m, const ipmc_sweep& s, int lpc, int cpl, int spec, hipStream_t st);
int l96_sweep_f64(const ipmc_model& m, const ipmc_sweep& s, int lpc, int spec, hipStream_t st);
int l96_eval_f32(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
                 int lpc, hipStream_t st);
int l96_eval_f64(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out, bool phi,
                 int lpc, hipStream_t st);
bool l96_has_f32(int D, int lpc, int cpl);  // cpl: chains per lane group (1, or 2 packed)
bool l96_has_f64(int D, int lpc);

// Burgers (ipmc_burgers.hip)
int burgers_sweep(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st);
// lanes per chain and speculation width burgers_sweep would use
int burgers_plan(const ipmc_model& m, const ipmc_sweep& s, int& lanes, int& spec);
int burgers_eval(const ipmc_model& m, int32_t dtype, int64_t n, const void* u, const void* y, const void* ginv,
                 void* out, bool phi, hipStream_t st);

// Two-scale Lorenz-96 with the moment observation (ipmc_l96ts.hip)
int l96ts_sweep(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st);
int l96ts_plan(const ipmc_model& m, const ipmc_sweep& s, int& lanes, int& spec);
int l96ts_eval(const ipmc_model& m, int32_t dtype, int64_t n, const void* u, const void* y, const void* ginv,
               void* out, bool phi, hipStream_t st);

}  // namespace ipmc
