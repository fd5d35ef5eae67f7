/*
 * ipmc.h — C-ABI of the MI355X many-chain pCN sampler (libipmc.so).
 *
 * This is the drop-in boundary for the reference's hot path, the pCN
 * Metropolis–Hastings step with an evolution-equation misfit potential:
 *
 *   reference (ochsnerd/ip_mcmc, pure Python, one chain)      this ABI (many chains, device)
 *   ------------------------------------------------------    -----------------------------------
 *   MCMCSampler.run / _step           sampler.py:12-41        ipmc_pcn_sweep   (n_steps steps/launch)
 *   MCMCSampler.run sampling loop     sampler.py:23-28        ipmc_pcn_run     (one launch per sample, in C)
 *   ConstSteppCNProposer.__call__     proposer.py:81-82       ipmc_pcn_sweep   (proposal stage)
 *   VarSteppCNProposer.__call__       proposer.py:110-115     ipmc_pcn_sweep   (host passes beta per launch)
 *   ProbabilisticAccepter.__call__    accepter.py:59-62       ipmc_pcn_sweep   (accept stage)
 *   pCNAccepter.accept_probability    accepter.py:121-122     ipmc_pcn_sweep   (exp(Φu−Φv) > r)
 *   CountedAccepter.__call__          accepter.py:20-27       ipmc_sweep.accepts (per-chain counter)
 *   ConstrainAccepter.__call__        accepter.py:52-55       ipmc_sweep.box_lo/box_hi/box_off
 *   EvolutionPotential.__call__       potential.py:53-54      ipmc_potential
 *   G(u) observation operators        lorenz_mcmc.py:55-68,   ipmc_forward
 *                                     stuart_examples.py:69-70,
 *                                     burgers/utilities.py:40-41
 *   GaussianDistribution.sample       distribution.py:114-118 ipmc_normal (counter-based N(0,I))
 *   MCMCSampler._step with a Python G / constraint / noise model
 *                                     sampler.py:35-41,       ipmc_pcn_draws (a block of steps' w and log r
 *                                     potential.py:48-54,     for the host-side step; G runs in the caller)
 *                                     accepter.py:39-62
 *   ConstStep/VarStepStandardRWProposer proposer.py:14-56     ipmc_sweep.proposal = IPMC_PROPOSAL_RW
 *   StandardRWAccepter._I             accepter.py:104-106     ipmc_sweep.reg_scale, ipmc_init_phi
 *   Lorenz96.__call__ (J > 0) + moment_function
 *                                     lorenz.py:44-101,       IPMC_MODEL_LORENZ96_2S
 *                                     lorenz_mcmc.py:17-40
 *   MCMCSampler.autocorr              sampler.py:43-54        ipmc_autocorr
 *   len_burn_in                       burgers/utilities.py:134-167  ipmc_burn_in
 *   np.mean over the samples          sampler.py:20-28 callers ipmc_block_sums (the many-chain posterior
 *                                     (e.g. stuart_examples.py)  mean's fixed-order block sums, on the device)
 *
 * The reference has no FFI of its own (it is duck-typed Python); these entry
 * points are what a ctypes binding of its plugin API binds.
 *
 * Conventions
 *  - Every pointer inside the structs and every data pointer argument is a
 *    DEVICE pointer (hipMalloc / torch CUDA tensor) for libipmc.so; the CPU
 *    oracle (oracle/liboracle.so) implements the same structs on HOST pointers.
 *  - Arrays are dense row-major; per-chain arrays are [n_chains, k] with k
 *    contiguous. Real arrays have the dtype given by `dtype` (float or double).
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *    Calls are asynchronous on that stream and never synchronise the host.
 *  - Return value: IPMC_OK or an ipmc_status error; ipmc_last_error() gives
 *    a message (thread-local).
 *  - Randomness is counter-based (Philox4x32-10). The draw for (chain, step,
 *    component) is a pure function of (seed, global chain id, global pCN step,
 *    component), so results do not depend on sharding or launch splitting.
 *    Global chain ids are 32-bit (chain_offset + n_chains <= 2^32, else IPMC_ERR_INVALID).
 */
#ifndef IPMC_H
#define IPMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPMC_ABI_VERSION 13

/* entry points kept for older callers but no longer on the product path */
#if defined(__GNUC__) || defined(__clang__)
#define IPMC_DEPRECATED(msg) __attribute__((deprecated(msg)))
#else
#define IPMC_DEPRECATED(msg)
#endif

typedef enum {
  IPMC_OK = 0,
  IPMC_ERR_INVALID = 1,     /* bad argument (shape, null pointer, range) */
  IPMC_ERR_UNSUPPORTED = 2, /* valid request the library does not implement */
  IPMC_ERR_DEVICE = 3       /* HIP runtime error (launch / memory) */
} ipmc_status;

typedef enum { IPMC_F32 = 0, IPMC_F64 = 1 } ipmc_dtype;

typedef enum {
  IPMC_MODEL_LINEAR = 0,    /* G(u) = A (theta0 + u)                  stuart_examples.py:69-70 */
  IPMC_MODEL_LORENZ63 = 1,  /* RK4 Lorenz-63, moments time-averaged   (no reference; lorenz_mcmc.py:17-40 pattern) */
  IPMC_MODEL_LORENZ96 = 2,  /* RK4 single-scale Lorenz-96, forcing field theta0+u, time-averaged X   lorenz.py:73-88 */
  IPMC_MODEL_BURGERS = 3,   /* Rusanov FV + SSPRK2 Burgers, windowed trapz observations   burgers/rusanov.py, utilities.py */
  IPMC_MODEL_LORENZ96_2S = 4 /* RK4 two-scale Lorenz-96 (lorenz.py:44-101), theta = (F, h, b), time-averaged
                                5K moments (lorenz_mcmc.py:17-40, 55-68) */
} ipmc_model_kind;

typedef enum {
  IPMC_ARITH_FMA = 0,       /* fused multiply-add form (fast path, bit-exact vs oracle in the same mode) */
  IPMC_ARITH_REFERENCE = 1  /* no FMA anywhere; reference expression order (lorenz.py:77-81) */
} ipmc_arith;

typedef enum { IPMC_DT_FIXED = 0, IPMC_DT_CFL = 1 } ipmc_dt_mode;

typedef enum { IPMC_PROPOSAL_PCN = 0, IPMC_PROPOSAL_RW = 1 } ipmc_proposal;

/* Forward-map description. Fields not used by a model are ignored. */
typedef struct ipmc_model {
  int32_t kind;       /* ipmc_model_kind */
  int32_t arith;      /* ipmc_arith */
  int32_t k;          /* parameter dimension (length of u) */
  int32_t q;          /* observation dimension (length of G(u)) */
  int32_t dim;        /* state dimension: L96 d; Burgers N interior cells; L63 3 */
  int32_t n_steps;    /* time steps of the integrator (fixed-dt models) */
  double dt;          /* time step */
  const void* x0;     /* [dim] initial state (L63/L96); Burgers: [dim+2] cell centres incl. ghosts */
  const void* theta0; /* [k] prior-mean offset: the model evaluates at theta = theta0 + u */
  const void* A;      /* LINEAR: [q, k] matrix */
  /* Burgers (IPMC_MODEL_BURGERS) */
  int32_t dt_mode;    /* ipmc_dt_mode */
  int32_t n_windows;  /* == q */
  const int32_t* win_lo; /* [q] first cell (interior index) of each trapz window  utilities.py:93-98 */
  const int32_t* win_hi; /* [q] one-past-last cell */
  double dx;          /* cell width (reference: linspace retstep) */
  double t_end;       /* CFL mode: integrate while t < t_end (rusanov.py:40-45) */
  double cfl;         /* CFL mode: dt = cfl*dx/max|u| (reference 0.5, rusanov.py:102-109) */
  double nu;          /* viscosity of the optional central-difference term (0 = reference scheme) */
  double meas_scale;  /* observation scale (reference 10, utilities.py:107) */
  double meas_dx;     /* trapz spacing x[2]-x[1] of the interior centres (utilities.py:91) */
  int32_t max_iter;   /* CFL mode: step cap; a chain that hits it is invalid (Φ = +inf) */
  int32_t reserved;
  /* Two-scale Lorenz-96 (IPMC_MODEL_LORENZ96_2S): dim = K slow variables, state K(1+J) */
  int32_t fast_per_slow; /* J (lorenz.py:21-22) */
  int32_t moment_mode;   /* 0: the reference moment_function (Ybar_k = Y_{k,0}, lorenz_mcmc.py:32, Q8); 1: block mean */
  double coupling_c;     /* c, time-scale ratio (lorenz.py:27-28), fixed; theta = (F, h, b) = theta0 + u */
} ipmc_model;

/* One launch of n_steps pCN steps for n_chains chains. */
typedef struct ipmc_sweep {
  int32_t dtype;            /* ipmc_dtype of u/phi/y/gamma_inv/prior_sqrt/box_* */
  int32_t lanes_per_chain;  /* 0 = auto; otherwise a divisor of the state dim (kernel layout only: results are identical) */
  int32_t chains_per_lane;  /* 0 = auto; 2 = two fp32 chains packed per lane group (v_pk_*_f32), 1 = one (layout only) */
  int32_t spec_width;       /* speculative steps per round (0 = auto, 1 = off; a power of two): spec_width lane
                               groups per chain each evaluate one of the next steps from the current state, the
                               first acceptance ends the round -- results identical, small ensembles run faster.
                               Lorenz-63 / linear (k <= 8), Lorenz-96 (spec_width * lanes_per_chain <= 64, or = 256:
                               the slots of one chain over the 4 waves of a block),
                               Burgers (spec_width * lanes of a chain <= 64, or = 256), two-scale Lorenz-96 (any width
                               with spec_width * K <= 64). */
  int64_t n_chains;
  int64_t chain_offset;     /* global id of chain 0 of this shard (RNG counter); chain_offset + n_chains <= 2^32 */
  void* u;                  /* [n_chains, k] in/out current state */
  void* phi;                /* [n_chains] in/out cached Φ(u) */
  int64_t* accepts;         /* [n_chains] in/out accept counters (may be NULL) */
  int64_t* calls;           /* [n_chains] in/out count of proposals that passed the box (may be NULL);
                               = the inner CountedAccepter's calls under ConstrainAccepter(CountedAccepter(..)) */
  const void* y;            /* [q] data */
  const void* gamma_inv;    /* [q] 1/γ_i, diagonal noise covariance Γ = diag(γ²) */
  const void* prior_sqrt;   /* [k] sqrt of the diagonal prior covariance (NULL if prior_chol is set) */
  const void* box_lo;       /* [k] or NULL: ConstrainAccepter box, valid iff lo < v+off < hi for all i */
  const void* box_hi;       /* [k] or NULL */
  const void* box_off;      /* [k] or NULL (treated as 0) */
  double beta;              /* pCN step size, 0 <= beta <= 1 */
  double contraction;       /* sqrt(1 - beta^2), computed by the host (proposer.py:77) */
  const double* beta_schedule; /* optional [n_steps][2] (beta, contraction) of each step of this launch,
                                  overriding beta/contraction (VarSteppCNProposer, proposer.py:110-115;
                                  VarStepStandardRWProposer, proposer.py:53-56, with beta = sqrt(2)*sqrt(delta(i))) */
  int32_t proposal;         /* ipmc_proposal: PCN v = contraction*u + beta*w (proposer.py:82),
                               RW v = u + beta*w (proposer.py:30, beta = sqrt(2 delta)) */
  int32_t reserved1;
  const void* reg_scale;    /* optional [k]: accept on I = Φ + ½Σ(reg_scale_i v_i)² instead of Φ
                               (StandardRWAccepter, accepter.py:98-106); `phi` then caches I(u) */
  uint64_t seed;            /* Philox key */
  uint64_t step0;           /* global pCN step index of the first step of this launch; step0 + n_steps <= 2^63
                               (steps from 2^63 on are the host-draw range, rng.py) */
  int64_t n_steps;          /* pCN steps in this launch */
  void* sample_out;         /* optional [n_chains, *] : u after the last step, row stride sample_stride elements */
  int64_t sample_stride;
  double* sum_u;            /* optional [n_chains, k] running sum of u after every step (f64) */
  double* sum_u2;           /* optional [n_chains, k] running sum of u^2 */
  const void* prior_chol;   /* optional [k, k] row-major lower Cholesky factor L of a NON-diagonal prior covariance
                               (GaussianDistribution.L): w_j = sum_{i<=j} L[j][i] xi_i in ascending i, overriding
                               prior_sqrt (which may then be NULL); proposer.py:81-82's w ~ N(0, C) */
  int64_t sample_every;     /* 0: sample_out receives u after the last step of the launch (above).  > 0: samples
                               inside the launch, MCMCSampler.run's recording (sampler.py:23-28): u after every
                               step j (0-based in this launch) with (j+1) % sample_every == 0 goes to
                               sample_out + ((j+1)/sample_every - 1)*sample_step_stride (+ chain*sample_stride);
                               nothing else is written.  One launch then covers many samples and the speculative
                               sweeps run across sample boundaries. */
  int64_t sample_step_stride; /* elements between consecutive samples of one chain (>= k when sample_every > 0);
                                 with n_s = n_steps / sample_every samples per chain the rows may not overlap:
                                 sample_stride >= (n_s-1)*sample_step_stride + k ([chain, sample, k]) or
                                 sample_step_stride >= (n_chains-1)*sample_stride + k ([sample, chain, k]) */
  uint64_t accepts_step0;   /* (ABI 11) global pCN step at which the `accepts` counters started counting
                               (MCMCSampler.run zeroes them at its first step; 0 = from step 0).  A speculative
                               sweep's first round picks its speculation tree by the chain's acceptance over the
                               steps since then (step0 - accepts_step0); results never depend on it. */
} ipmc_sweep;

/* pCN sweep: n_steps x (propose v, Φ(v) = ½‖(y−G(v))/γ‖², accept iff Φ(u)−Φ(v) > log r). */
int ipmc_pcn_sweep(const ipmc_model* model, const ipmc_sweep* sweep, void* stream);

/* MCMCSampler.run's sampling loop (sampler.py:23-28) in one call: n_blocks
   consecutive ipmc_pcn_sweep launches of block_steps steps each, block b
   starting at global step sweep->step0 + b*block_steps (sweep->n_steps is
   ignored) and, if sweep->sample_out is set, writing u after its last step to
   sample_out + b*sample_block_stride elements (rows still sweep->sample_stride
   apart: samples [n_chains, n_samples, k] take sample_block_stride = k);
   beta_schedule, if set, holds all n_blocks*block_steps steps; sum_u / sum_u2
   accumulate over every step.  The same results as the n_blocks calls, without
   a host round trip per sample.  With sweep->sample_every > 0 each block
   records its in-launch samples from sample_out + b*sample_block_stride. */
int ipmc_pcn_run(const ipmc_model* model, const ipmc_sweep* sweep, int64_t n_blocks, int64_t block_steps,
                 int64_t sample_block_stride, void* stream);
/* sweep->phi[c] = the accept potential of sweep->u[c] for every chain: Φ(u), or
   I(u) = Φ(u) + ½Σ(reg_scale_i u_i)² when sweep->reg_scale is set (call before the first sweep). */
int ipmc_init_phi(const ipmc_model* model, const ipmc_sweep* sweep, void* stream);

/* Φ(u) for n parameter vectors u [n, k] -> phi [n]  (EvolutionPotential.__call__ minus the constant). */
int ipmc_potential(const ipmc_model* model, int32_t dtype, int64_t n, const void* u,
                   const void* y, const void* gamma_inv, void* phi, void* stream);

/* G(u) for n parameter vectors u [n, k] -> g [n, q]. */
int ipmc_forward(const ipmc_model* model, int32_t dtype, int64_t n, const void* u, void* g,
                 void* stream);

/* The proposal's standard normals: out[c, i] = ξ(seed, chain_offset + c, step, i), [n_chains, k]. */
int ipmc_normal(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step, int32_t k,
                int32_t dtype, void* out, void* stream);

/* The accept uniforms: out[c] = r(seed, chain_offset + c, step) in [0,1), always double. */
int ipmc_uniform(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step, double* out,
                 void* stream);

/* The random inputs of n_steps pCN steps for a HOST-side step (MCMCSampler.run with a Python forward map,
   constraint predicate or noise model, sampler.py:35-41): for step s in [0, n_steps) (global pCN step
   step0 + s) and chain c, w[(s*n_chains + c)*k + j] = the proposal noise exactly as the sweep kernels form
   it -- prior_sqrt[j] * xi_j, or sum_{i<=j} prior_chol[j][i] * xi_i in ascending i from +0 (no FMA) --
   in dtype, and, if log_r is not NULL, log_r[s*n_chains + c] = log r with the kernels' deterministic log
   (accept iff (double)(phi_u - phi_v) > log_r, accepter.py:62).  step0 + n_steps <= 2^63. */
int ipmc_pcn_draws(uint64_t seed, int64_t chain_offset, int64_t n_chains, uint64_t step0, int64_t n_steps,
                   int32_t k, int32_t dtype, const void* prior_sqrt, const void* prior_chol, void* w,
                   double* log_r, void* stream);

/* Asynchronous rectangular copy device -> host (page-locked for overlap) on `stream`: `rows` rows of
   `width` bytes, row r from src + r*src_pitch to dst + r*dst_pitch (the sampler's block-wise sample
   copy; inside libipmc so that it runs on the HIP runtime the caller's stream belongs to). */
int ipmc_copy_rows_d2h(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t width,
                       int64_t rows, void* stream);

/* Batched normalised autocorrelation (MCMCSampler.autocorr, sampler.py:43-54):
   series s is x[s*stride_series + t*stride_t], t < len (any len; series over 8192 samples stream through LDS tiles);
   out[s, tau] = r[tau]/r[0], r[tau] = Σ_t x_[t] x_[t+tau], x_ = x - mean(x), tau < max_lag <= len;
   all ones for a constant series.  out is double [n_series, max_lag]. */
int ipmc_autocorr(const void* x, int32_t dtype, int64_t n_series, int64_t len, int64_t stride_series,
                  int64_t stride_t, int32_t max_lag, double* out, void* stream);

/* Batched burn-in detection (len_burn_in, report/scripts/burgers/utilities.py:134-167):
   chain c, variable v, sample t is x[c*stride_chain + v*stride_var + t*stride_t], t < len;
   out[c] = the reference's burn-in index for that chain (window = avg_window = 50 and
   threshold = accepted_change = 0.03 in the reference).  flags_scratch: uint32
   [n_chains * ceil(len/32)] device scratch (overwritten).  Requires len >= window. */
int ipmc_burn_in(const void* x, int32_t dtype, int64_t n_chains, int32_t n_vars, int64_t len, int64_t stride_chain,
                 int64_t stride_var, int64_t stride_t, int32_t window, double threshold, uint32_t* flags_scratch,
                 int64_t* out, void* stream);

/* DEPRECATED since ABI 13 -- not on the product path: the posterior mean is ipmc_block_sums (below) + the
   block sums in block order, which no rank has to wait for.  Kept (exported, tested) for callers of ABI 12.
   (ABI 12) acc[j] = (((acc[j] + rows[0][j]/div) + rows[1][j]/div) + ...) for j < k over the n_rows rows
   (row r at rows + r*row_stride doubles), strictly in row order -- one dependent chain of adds per column,
   equal bit for bit to ipmc_host_ordered_sum (ipmc_host.h); div == 1 adds the rows as they are.
   Device pointers; acc [k] in/out. */
IPMC_DEPRECATED("ipmc_block_sums (ABI 13) forms the posterior mean")
int ipmc_ordered_sum(const double* rows, int64_t n_rows, int64_t k, int64_t row_stride, double div, double* acc,
                     void* stream);

/* (ABI 13) out[b][j] = (((0 + rows[bB][j]/div) + rows[bB+1][j]/div) + ...) for j < k over the rows of block b
   (B = block_rows consecutive rows; the last block holds the n_rows % B left over), each block from zero
   strictly in row order -- the first stage of the many-chain posterior mean (shard.block_sum: block sums,
   then the block sums in block order), equal bit for bit to ipmc_host_ordered_sum on each block from zero.
   Blocks run in parallel.  Device pointers; out [ceil(n_rows / B), k]. */
int ipmc_block_sums(const double* rows, int64_t n_rows, int64_t k, int64_t row_stride, int64_t block_rows,
                    double div, double* out, void* stream);

/* Lorenz-96 layout of a ONE-step launch (no speculation) when lanes_per_chain = chains_per_lane = 0:
   returns lanes_per_chain, and chains_per_lane * 100 + lanes_per_chain from ipmc_auto_layout.
   Multi-step launches may speculate on another layout: ipmc_plan_sweep reports that. */
int ipmc_auto_lanes(const ipmc_model* model, int32_t dtype, int64_t n_chains);
int ipmc_auto_layout(const ipmc_model* model, int32_t dtype, int64_t n_chains);

/* The kernel plan ipmc_pcn_sweep(model, sweep) would run, from the same code path: lanes per chain
   (per speculative slot), chains per lane group (2 = packed fp32 pairs) and speculation width
   (1 = sequential).  Reads only the sweep's dtype, n_chains, n_steps, lanes_per_chain,
   chains_per_lane and spec_width; returns the error ipmc_pcn_sweep would for an unsupported layout. */
typedef struct ipmc_plan {
  int32_t lanes_per_chain;
  int32_t chains_per_lane;
  int32_t spec_width;
  int32_t reserved;
} ipmc_plan;
int ipmc_plan_sweep(const ipmc_model* model, const ipmc_sweep* sweep, ipmc_plan* out);

const char* ipmc_last_error(void);
int ipmc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* IPMC_H */
