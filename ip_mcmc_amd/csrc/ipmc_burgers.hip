// Burgers forward map (Rusanov FV + SSPRK2, burgers/rusanov.py:6-109) and its
// pCN sweep.
//
// Layout: one chain per group of GS lanes (GS in {16, 32, 64}, groups aligned
// inside a wavefront); lane `sub` owns CPL consecutive interior cells
// [sub*CPL + 1, sub*CPL + CPL] in VGPRs (N = nlive*CPL, nlive <= GS; lanes past
// nlive hold no cells).  The ghost cells are explicit values on the first and
// last live lane (the IC sets them, rusanov.py:32, and the first step reads
// them before any boundary condition is applied).  Interface fluxes between
// lanes use the neighbour lane's edge cell (DPP wave_shr:1 / wave_shl:1,
// below); each lane computes
// CPL+1 fluxes, the shared edge flux bit-identically on both sides.  CFL mode
// reduces max|w| over the group every step (exact, order-free); fixed-dt mode
// keeps a per-lane guard and reduces once.  The final interior state is staged
// in LDS and lane 0 of the group evaluates the Measurer windows in numpy's
// pairwise summation order (so REFERENCE arith equals np.trapz bit for bit).
#include "ipmc_internal.hpp"
#include "ipmc_sweep_common.hpp"

namespace ipmc {

constexpr int kBurBlock = 256;
// block-wide rounds index kSpecTrees.nd[tb][slot] with slot < kBurBlock / GS
static_assert(kBurBlock <= kSpecNodes, "block-wide speculation slots index the spec-tree tables");

// Rusanov flux F = ½(f(a)+f(b)) − ½·max(|a|,|b|)·(b−a), f(w) = w²/2
// (rusanov.py:92-96), REFERENCE arith: the reference's operation order.
template <typename T>
__device__ __forceinline__ T rus_flux_ref(T a, T b) {
  const T half = (T)0.5;
  const T aa = a < (T)0 ? -a : a, ab = b < (T)0 ? -b : b;
  const T sp = ab > aa ? ab : aa;
  const T fa = (half * a) * a, fb = (half * b) * b;
  const T favg = half * (fa + fb);
  return favg - (half * sp) * (b - a);
}

// max(|a|, |b|) as ONE v_max with abs source modifiers.  fmax(fabs, fabs) in
// C++ compiles to a canonicalising v_max per operand plus the max (the compiler
// cannot prove the DPP-moved and loop-carried values canonical), i.e. 3 VALU
// ops.  The hardware max is IEEE maxNum, the same value as C fmax for every
// input these kernels produce (no signalling NaNs); the oracle uses fmax.
__device__ __forceinline__ double max_abs(double a, double b) {
  double r;
  asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float max_abs(float a, float b) {
  float r;
  asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ double abs_of(double a) { return __builtin_fabs(a); }
__device__ __forceinline__ float abs_of(float a) { return __builtin_fabsf(a); }
__device__ __forceinline__ double max_of(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ float max_of(float a, float b) { return __builtin_fmaxf(a, b); }

// ds_swizzle in bit mode (and 0x1F, xor 0x10): lane i reads lane i ^ 16 of
// its 32-lane half; no address operand, no LDS storage.
__device__ __forceinline__ float swz_xor16(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
}
__device__ __forceinline__ double swz_xor16(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffff), 0x401F);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x401F);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// max over the GS-lane group (GS-aligned in the wave), every lane gets it:
// DPP xor 1 / xor 2 (quad_perm), row_half_mirror (8), row_mirror (16) inside a
// row, ds_swizzle xor 16 across the two rows of a 32-lane half, and for
// GS = 64 the two halves' values by readlane.  maxNum is exact and order-free,
// so any tree gives the same value.  (Five __shfl_xor levels -- a
// ds_bpermute round trip each, in the CFL loop's critical path every step --
// took cfg 4 CFL 0.466 ms.)
constexpr int kDppRowMirror = 0x140;
constexpr int kDppRowHalfMirror = 0x141;

template <int GS, typename T>
__device__ __forceinline__ T group_max_abs(T m) {
  static_assert(GS == 16 || GS == 32 || GS == 64, "Burgers groups are 16, 32 or 64 lanes");
  m = max_of(m, dpp<qperm(1, 0, 3, 2)>(m));
  m = max_of(m, dpp<qperm(2, 3, 0, 1)>(m));
  m = max_of(m, dpp<kDppRowHalfMirror>(m));
  m = max_of(m, dpp<kDppRowMirror>(m));
  if constexpr (GS >= 32) m = max_of(m, swz_xor16(m));
  if constexpr (GS == 64) m = max_of(__shfl(m, 0, 64), __shfl(m, 32, 64));
  return m;
}

// max |w| over the lane's cells (NaN ignored, as the reference's np.max of a
// finite state never sees one before the CFL guard trips)
template <int CPL, typename T>
__device__ __forceinline__ T lane_max_abs(const T (&w)[CPL], bool live) {
  T m = (T)0;
  if (live) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) m = max_abs(m, w[j]);  // m >= 0
  }
  return m;
}

// REFERENCE arith: dudt = (F_{i+½} − F_{i−½})/(−dx) for the lane's cells from
// state s (+ halos hl / hr); VISC adds ν(u_{i+1} − 2u_i + u_{i−1})/dx².
template <typename T>
struct RusConst {
  T mdx, c1, nudx2;  // −dx, the F2 scale ¼/(−dx), ν/dx²
};

template <typename T, int CPL, bool VISC>
__device__ __forceinline__ void rus_rate(const T (&s)[CPL], T hl, T hr, const RusConst<T>& k, T (&r)[CPL]) {
  T fl = rus_flux_ref<T>(hl, s[0]);
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const T right = (j + 1 < CPL) ? s[j + 1] : hr;
    const T left = (j > 0) ? s[j - 1] : hl;
    const T fr = rus_flux_ref<T>(s[j], right);
    T v = (fr - fl) / k.mdx;
    if (VISC) {  // the central-difference form
      const T lap = (right - (s[j] + s[j])) + left;
      v = v + k.nudx2 * lap;
    }
    r[j] = v;
    fl = fr;
  }
}

// FMA arith: the flux in the scale F2 = 4F,
//   F2(a, b) = fma(max(d_a, d_b), a − b, e_a + e_b),  e = w·w,  d = 2|w| [+ 4ν/dx],
// with e and d formed once per cell (d as one fma with an abs source modifier,
// so the viscous flux costs nothing), i.e. max, sub, add, fma per interface,
// and dudt = c1·(F2_{i+½} − F2_{i−½}), c1 = ¼/(−dx), folded into the update's
// dt.  In fp64 an SSPRK2 step takes 173 VALU instructions per lane of 8 cells
// (187 with the earlier pre-scaled flux fma(c2·s, b−a, c1·(a²+b²)), 7 ops per
// interface; profiles/r2/burgers_f2_ab.jsonl).  fp32 runs the same arithmetic
// on cell pairs (rus_rate_pk).  The flux differences of the viscous term are
// the central-difference Laplacian; REFERENCE arith keeps that form.
template <typename T, int CPL, bool VISC>
__device__ __forceinline__ void rus_rate_f2(const T (&s)[CPL], T hl, T hr, T cv2, T (&r)[CPL]) {
  T x[CPL + 2], e[CPL + 2], d[CPL + 2];
  x[0] = hl;
  x[CPL + 1] = hr;
#pragma unroll
  for (int j = 0; j < CPL; ++j) x[j + 1] = s[j];
#pragma unroll
  for (int i = 0; i < CPL + 2; ++i) {
    e[i] = x[i] * x[i];
    d[i] = VISC ? madd<true>(abs_of(x[i]), (T)2, cv2) : x[i] + x[i];
  }
  auto flux = [&](int i) {
    const T sp = VISC ? max_of(d[i], d[i + 1]) : max_abs(d[i], d[i + 1]);
    return madd<true>(sp, x[i] - x[i + 1], e[i] + e[i + 1]);
  };
  T fl = flux(0);
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const T fr = flux(j + 1);
    r[j] = fr - fl;
    fl = fr;
  }
}

struct BurCtx {
  int sub, lane, nlive;
};

// Halo exchange inside the group: value of the previous lane's last cell and
// the next lane's first cell (or the ghosts at the ends).
// DPP wave_shr:1 / wave_shl:1 (GFX9 whole-wave shifts; no LDS round trip):
// the lanes they leave without a source are group ends, which take ghosts.
constexpr int kDppWaveShl1 = 0x130;
constexpr int kDppWaveShr1 = 0x138;

template <typename T, int CPL>
__device__ __forceinline__ void halos(const T (&s)[CPL], T gl, T gr, const BurCtx& c, T& hl, T& hr) {
  hl = dpp<kDppWaveShr1>(s[CPL - 1]);
  hr = dpp<kDppWaveShl1>(s[0]);
  if (c.sub == 0) hl = gl;
  if (c.sub == c.nlive - 1) hr = gr;
}

// fp32 FMA arith: rus_rate_f2 on cell pairs P[p] = (w[p], w[p+H]), H = CPL/2,
// so every flux, rate and update is a v_pk_*_f32 on two cells (the max is two
// v_max_f32 with abs modifiers: there is no packed max).  Pair p's neighbours
// are pairs p-1 and p+1 except at the ends: Q = [(hl, w[H-1]), P[0..H-1],
// (w[H], hr)], so the interface w[H-1]|w[H] is evaluated twice, bit-identically.
// The viscous wave speed max(2|a|, 2|b|) + 4ν/dx equals rus_rate_f2's
// max(fma(|a|, 2, 4ν/dx), fma(|b|, 2, 4ν/dx)) exactly (2|w| is exact and
// rounding is monotone).
template <int H, bool VISC>
__device__ __forceinline__ void rus_rate_pk(const f32x2 (&X)[H], float hl, float hr, f32x2 cv2, f32x2 (&r)[H]) {
  f32x2 q[H + 2], e[H + 2], d[H + 2];
  q[0] = f32x2{hl, X[H - 1].x};
#pragma unroll
  for (int p = 0; p < H; ++p) q[p + 1] = X[p];
  q[H + 1] = f32x2{X[0].y, hr};
#pragma unroll
  for (int i = 0; i < H + 2; ++i) {
    e[i] = q[i] * q[i];
    d[i] = q[i] + q[i];
  }
  auto flux = [&](int i) {
    f32x2 sp = f32x2{max_abs(d[i].x, d[i + 1].x), max_abs(d[i].y, d[i + 1].y)};
    if (VISC) sp = sp + cv2;
    return madd<true>(sp, q[i] - q[i + 1], e[i] + e[i + 1]);
  };
  f32x2 fl = flux(0);
#pragma unroll
  for (int p = 0; p < H; ++p) {
    const f32x2 fr = flux(p + 1);
    r[p] = fr - fl;
    fl = fr;
  }
}

// Integrate the Riemann IC (left, right, jump) to the end; returns validity.
// w holds the final interior cells of this lane.  VISC is a compile-time
// switch: a runtime flag made the compiler evaluate the diffusion term for
// every cell and select it away (6 extra VALU ops per cell and stage).
template <typename T, int CPL, int GS, bool FM, bool VISC>
__device__ bool burgers_integrate(const ipmc_model& m, T left, T right, T jump, const BurCtx& c, T (&w)[CPL]) {
  const bool live = c.sub < c.nlive;
  const T* xc = (const T*)m.x0;
  const int c0 = c.sub * CPL + 1;  // first owned cell (ghost-inclusive index)
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int idx = live ? c0 + j : 1;
    w[j] = (xc[idx] < jump) ? left : right;
  }
  const int N = m.dim;
  T gl = (xc[0] < jump) ? left : right;
  T gr = (xc[N + 1] < jump) ? left : right;
  const T dx = (T)m.dx, mdx = -dx;
  const T cfl_dx = (T)m.cfl * dx;
  const T rdx = (T)1 / mdx;
  const RusConst<T> kc{mdx, (T)0.25 * rdx, (T)m.nu / (dx * dx)};
  const T cv2 = ((T)4 * (T)m.nu) / dx;  // the viscous term in the F2 scale
  const T tend = (T)m.t_end;
  const T dtf = (T)m.dt;
  const bool cflmode = (m.dt_mode == IPMC_DT_CFL);
  bool valid = true;
  bool lane_ok = true;
  // One SSPRK2 step of size dt, rusanov.py:62-74.  REFERENCE: u* = u + dt L(u);
  // u* += dt L(u*); u = (u + u*)/2.  FMA arith folds the average into the
  // stages: u_half = fma(dt/2, L(u), u) next to u*, then
  // u = fma(dt/2, L(u*), u_half) (one VALU op per cell fewer; dt/2 is exact),
  // with dt scaled by c1 for the F2 flux (dudt = c1 ΔF2).
  constexpr bool PK = FM && sizeof(T) == 4;
  constexpr int H = CPL / 2;
  f32x2 P[H];  // PK: the state as cell pairs (w[p], w[p+H])
  if constexpr (PK) {
#pragma unroll
    for (int p = 0; p < H; ++p) P[p] = f32x2{(float)w[p], (float)w[p + H]};
  }
  auto step = [&](T dt0) {
    const T dt = FM ? dt0 * kc.c1 : dt0;
    const T hdt = dt * (T)0.5;
    if constexpr (PK) {
      const f32x2 dtv{(float)dt, (float)dt}, hdtv{(float)hdt, (float)hdt}, cvv{(float)cv2, (float)cv2};
      f32x2 r[H], S[H];
      float hl = dpp<kDppWaveShr1>(P[H - 1].y), hr = dpp<kDppWaveShl1>(P[0].x);
      if (c.sub == 0) hl = (float)gl;
      if (c.sub == c.nlive - 1) hr = (float)gr;
      rus_rate_pk<H, VISC>(P, hl, hr, cvv, r);
#pragma unroll
      for (int p = 0; p < H; ++p) {
        S[p] = madd<true>(dtv, r[p], P[p]);
        P[p] = madd<true>(hdtv, r[p], P[p]);
      }
      hl = dpp<kDppWaveShr1>(S[H - 1].y);
      hr = dpp<kDppWaveShl1>(S[0].x);
      if (c.sub == 0) hl = S[0].x;  // BC on u*
      if (c.sub == c.nlive - 1) hr = S[H - 1].y;
      rus_rate_pk<H, VISC>(S, hl, hr, cvv, r);
#pragma unroll
      for (int p = 0; p < H; ++p) P[p] = madd<true>(hdtv, r[p], P[p]);
      gl = P[0].x;
      gr = P[H - 1].y;
    } else {
      T hl, hr, r[CPL], ws[CPL];
      halos<T, CPL>(w, gl, gr, c, hl, hr);
      if constexpr (FM)
        rus_rate_f2<T, CPL, VISC>(w, hl, hr, cv2, r);
      else
        rus_rate<T, CPL, VISC>(w, hl, hr, kc, r);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        ws[j] = madd<FM>(dt, r[j], w[j]);
        if constexpr (FM) w[j] = madd<true>(hdt, r[j], w[j]);
      }
      const T gls = ws[0], grs = ws[CPL - 1];  // BC on u*, used by the first / last live lane only
      halos<T, CPL>(ws, gls, grs, c, hl, hr);
      if constexpr (FM)
        rus_rate_f2<T, CPL, VISC>(ws, hl, hr, cv2, r);
      else
        rus_rate<T, CPL, VISC>(ws, hl, hr, kc, r);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        if constexpr (FM) {
          w[j] = madd<true>(hdt, r[j], w[j]);
        } else {
          ws[j] = ws[j] + dt * r[j];
          w[j] = (w[j] + ws[j]) / (T)2;
        }
      }
      gl = w[0];
      gr = w[CPL - 1];
    }
  };
  // max|w| over the lane's cells (order-free: maxNum of absolute values)
  auto lane_max = [&]() -> T {
    if constexpr (PK) {
      float mx = 0.0f;
      if (live) {
#pragma unroll
        for (int p = 0; p < H; ++p) mx = max_abs(max_abs(mx, P[p].x), P[p].y);
      }
      return (T)mx;
    } else {
      return lane_max_abs<CPL>(w, live);
    }
  };
  if (cflmode) {
    // dt = cfl dx / max|w| over the group each step, while t < t_end (the
    // reference's overshooting loop, rusanov.py:40-45, 102-109)
    T t = (T)0;
    int iters = 0;
    for (;;) {
      const T mx = group_max_abs<GS>(lane_max());
      if (!(t < tend)) break;
      if (iters >= m.max_iter) {
        valid = false;
        break;
      }
      const T dt = cfl_dx / mx;
      t = t + dt;
      ++iters;
      step(dt);
    }
  } else {
    // fixed dt: a uniform trip count, and a per-lane CFL guard reduced once
    const int n = m.n_steps;
    for (int it = 0; it < n; ++it) {
      const T mx = lane_max();
      if (!(mx * dtf <= cfl_dx)) lane_ok = false;
      step(dtf);
    }
  }
  if constexpr (PK) {
#pragma unroll
    for (int p = 0; p < H; ++p) {
      w[p] = P[p].x;
      w[p + H] = P[p].y;
    }
  }
  if (!cflmode) {
    // the group is valid iff every live lane kept max|w| dt <= cfl dx
    const unsigned long long bad = __ballot(!lane_ok);
    const unsigned long long gmask = (GS == 64 ? ~0ull : ((1ull << GS) - 1)) << (c.lane & ~(GS - 1));
    valid = (bad & gmask) == 0;
  }
  return valid;
}

// numpy pairwise sum (loops_utils.h.src, n <= 128) of the trapz terms
// (mdx * (v[i+1] + v[i])) / 2, i = 0..n-1, with v in LDS.
template <typename T>
__device__ T trapz_pairwise(const T* v, int n, T mdx) {
  auto term = [&](int i) { return (mdx * (v[i + 1] + v[i])) / (T)2.0; };
  if (n < 8) {
    T res = (T)0;
    for (int i = 0; i < n; ++i) res = res + term(i);
    return res;
  }
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = term(j);
  int i;
  for (i = 8; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + term(i + j);
  }
  T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + term(i);
  return res;
}


// G(theta) for the chain, state staged through `row` (this chain's N
// interior cells in LDS).  Lane 0 of the group evaluates the windows and,
// for PHI, the misfit; g_out (if set) receives G.  Returns Φ (+inf if the
// integration was invalid) on lane 0 of the group.
template <typename T, int CPL, int GS, bool FM>
__device__ T burgers_phi(const ipmc_model& m, const T (&v)[3], const BurCtx& c, T* row, const T* y, const T* ginv,
                         T* g_out) {
  const T* th0 = (const T*)m.theta0;
  const T left = (T)1 + (th0[0] + v[0]);
  const T right = th0[1] + v[1];
  const T jump = th0[2] + v[2];
  T w[CPL];
  const bool valid = (m.nu != 0.0) ? burgers_integrate<T, CPL, GS, FM, true>(m, left, right, jump, c, w)
                                   : burgers_integrate<T, CPL, GS, FM, false>(m, left, right, jump, c, w);
  if (c.sub < c.nlive) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) row[c.sub * CPL + j] = w[j];
  }
  wave_sync_lds();
  T phi = (T)0;
  if (c.sub == 0) {
    const T mdxm = (T)m.meas_dx;
    T acc = (T)0;
    for (int j = 0; j < m.q; ++j) {
      T gj = (T)__builtin_nan("");
      const int lo = m.win_lo[j], hi = m.win_hi[j];
      int nt = hi - lo - 1;
      if (nt < 0) nt = 0;
      // a window outside [0, N) or wider than 129 cells is not measurable: G = NaN
      if (valid && (nt == 0 || (lo >= 0 && lo + nt + 1 <= m.dim && nt <= 128)))
        gj = (T)m.meas_scale * trapz_pairwise<T>(row + lo, nt, mdxm);
      if (g_out) g_out[j] = gj;
      if (y) {
        const T r = (y[j] - gj) * ginv[j];
        acc = madd<FM>(r, r, acc);
      }
    }
    phi = valid ? (T)0.5 * acc : (T)__builtin_inf();
  }
  wave_sync_lds();  // row is reused by the next evaluation
  return phi;
}

constexpr int kBurQMax = 64;

// S speculative slots of GS lanes per chain (S = 1: the sequential chain; S·GS
// <= 64, or = kBurBlock: one chain per block, its slots on the block's waves,
// combined through LDS): slot s is node s of the speculation tree for the
// chain's recent acceptance rate (ipmc_spec_tree.hpp), and the chain walks the
// tree along the real decisions (spec_walk, ipmc_sweep_common.hpp) --
// bit-identical to S = 1.
template <typename T, int CPL, int GS, bool FM>
__global__ __launch_bounds__(kBurBlock) void burgers_sweep_kernel(const ipmc_model m, const ipmc_sweep s, int S) {
  __shared__ T lds[kBurBlock * CPL];
  __shared__ unsigned long long bmask[2][kBurBlock / 64];  // block-wide rounds: the waves' ballots
  __shared__ T vpk[4][kBurBlock];                          // and every slot's v and Φ(v)
  const int lane = threadIdx.x & 63;
  const int G = S * GS;
  const int64_t tid = (int64_t)blockIdx.x * kBurBlock + threadIdx.x;
  const int64_t chain = tid / G;
  const int r = (int)(tid % G);
  const int slot = r / GS;
  const int cbase = lane - r;
  const BurCtx c{r - slot * GS, lane, m.dim / CPL};
  if (chain >= s.n_chains) return;
  T* row = lds + (threadIdx.x & ~(GS - 1)) * CPL;
  const uint64_t gid = (uint64_t)(s.chain_offset + chain);
  T* u = (T*)s.u + chain * 3;
  T ur[3] = {u[0], u[1], u[2]};  // every lane of the chain keeps the chain state
  const T* sq = (const T*)s.prior_sqrt;
  const T beta = (T)s.beta, contr = (T)s.contraction;
  T* phi = (T*)s.phi;
  T phu = phi[chain];
  const unsigned long long gmask = (G >= 64) ? ~0ull : ((1ull << G) - 1);
  int nacc = 0, ncalls = 0;
  SampleClock clk(s);
  int64_t st = 0;
  SpecGuess guess(spec_accept_prior(s, chain));  // the speculation tree (ipmc_sweep_common.hpp)
  const bool rw = s.proposal == IPMC_PROPOSAL_RW;
  const T* chol = (const T*)s.prior_chol;
  while (st < s.n_steps) {
    const int64_t left = s.n_steps - st;
    const int tb = S > 1 ? guess.bucket() : 0;
    const SpecNode nd = kSpecTrees.nd[tb][slot];
    const int maxlvl = kSpecTrees.maxlvl[tb][S];
    const bool act = nd.depth < left;  // uniform per slot
    const int64_t tt = st + nd.depth;
    const int og = nd.orig < 0 ? 0 : nd.orig;
    bool ok = false;
    T phv = (T)0;
    double lr = 0.0;
    const uint64_t step = s.step0 + (uint64_t)tt;
    T w[3];
    if (act) pcn_noise<T, 3>(sq, s.seed, gid, step, 0, w, chol, 3);
    const T bs = (act && s.beta_schedule) ? (T)s.beta_schedule[2 * tt] : beta;
    const T cs = (act && s.beta_schedule) ? (T)s.beta_schedule[2 * tt + 1] : contr;
    // the proposals level by level (every lane of a slot holds its proposal):
    // a node's origin was formed one level before
    T v[3] = {(T)0, (T)0, (T)0};
    for (int lv = 0; lv <= maxlvl; ++lv) {
      T o[3];
      if (G <= 64) {
#pragma unroll
        for (int j = 0; j < 3; ++j) o[j] = __shfl(v[j], cbase + og * GS, 64);
      } else {
        const int t = threadIdx.x;
#pragma unroll
        for (int j = 0; j < 3; ++j) vpk[j][t] = v[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 3; ++j) o[j] = vpk[j][og * GS];
        __syncthreads();
      }
      if (act && nd.lvl == lv) {
#pragma unroll
        for (int j = 0; j < 3; ++j) v[j] = propose_one<T>(rw, nd.orig < 0 ? ur[j] : o[j], w[j], cs, bs);
      }
    }
    if (act) {  // uniform per slot
      ok = true;
      if (s.box_lo || s.box_hi) {
        const T* lo = (const T*)s.box_lo;
        const T* hi = (const T*)s.box_hi;
        const T* off = (const T*)s.box_off;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const T t = v[j] + (off ? off[j] : (T)0);
          if (lo && !(lo[j] < t)) ok = false;
          if (hi && !(t < hi[j])) ok = false;
        }
      }
      if (ok) {
        phv = burgers_phi<T, CPL, GS, FM>(m, v, c, row, (const T*)s.y, (const T*)s.gamma_inv, nullptr);
        phv = __shfl(phv, lane & ~(GS - 1), 64);
        if (s.reg_scale) phv = phv + regularizer<T, 3, 1, FM>((const T*)s.reg_scale, v, lane);
        lr = det_log(accept_uniform(s.seed, gid, step));
      }
    }
    // pcn_accept against the state this node proposed from: the chain's, or
    // its origin node's proposal (whose Φ that slot's lanes hold)
    T pho;
    if (G <= 64) {
      pho = __shfl(phv, cbase + og * GS, 64);
    } else {
      const int t = threadIdx.x;
#pragma unroll
      for (int j = 0; j < 3; ++j) vpk[j][t] = v[j];
      vpk[3][t] = phv;
      __syncthreads();
      pho = vpk[3][og * GS];
    }
    const bool acc = ok && (double)((nd.orig < 0 ? phu : pho) - phv) > lr;
    // one bit per slot (its first lane, bit slot*GS of the chain's lanes)
    const SpecNode* tree = kSpecTrees.nd[tb];
    unsigned long long accm = 0, path = 0;  // G <= 64: the chain's bits, one per slot
    // a block-wide chain's node n from the table and the waves' ballots in LDS
    auto node = [&](int n) {
      const int bit = n * GS;
      return spec_step_bits(tree, n, 0, bmask[0][bit >> 6] >> (bit & 63), bmask[1][bit >> 6] >> (bit & 63));
    };
    SpecRound rd;
    T phf;
    if (G <= 64) {
      // the walk resolved in parallel (spec_on_path, as ipmc_l96.hpp): no
      // cross-lane read inside a data-dependent loop
      accm = spec_slot_bits((__ballot(acc && c.sub == 0) >> cbase) & gmask, S, GS);
      const unsigned long long okm = spec_slot_bits((__ballot(ok && c.sub == 0) >> cbase) & gmask, S, GS);
      path = spec_slot_bits((__ballot(spec_on_path(tb, slot, accm, act) && c.sub == 0) >> cbase) & gmask, S, GS);
      rd = spec_path_round(path, accm, okm);
      phf = __shfl(phv, cbase + (rd.win >= 0 ? rd.win : 0) * GS, 64);
    } else {
      const int t = threadIdx.x;
      const unsigned long long ab = __ballot(acc && c.sub == 0), ob = __ballot(ok && c.sub == 0);
      if (lane == 0) {
        bmask[0][t >> 6] = ab;
        bmask[1][t >> 6] = ob;
      }
      __syncthreads();
      rd = spec_walk(S, left, node, [](int, int) {});
      phf = vpk[3][(rd.win >= 0 ? rd.win : 0) * GS];
    }
    if (G <= 64 && (s.sum_u || s.sample_every > 0)) {  // the recorded states read the parked proposals
      const int t = threadIdx.x;
#pragma unroll
      for (int j = 0; j < 3; ++j) vpk[j][t] = v[j];
      wave_sync_lds();
    }
    const int t0 = threadIdx.x - r;  // the chain's first thread in the block
    // the proposal of slot q from the LDS park (every lane of the chain runs this, uniform per chain)
    auto slot_v = [&](int q, T (&out)[3]) {
#pragma unroll
      for (int j = 0; j < 3; ++j) out[j] = vpk[j][t0 + q * GS];
    };
    T vf[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) vf[j] = __shfl(v[j], cbase + (rd.win >= 0 ? rd.win : 0) * GS, 64);
    if (G > 64) slot_v(rd.win >= 0 ? rd.win : 0, vf);
    if (s.sum_u || s.sample_every > 0) {  // uniform per chain (only lane r == 0 keeps the clock)
      // the states after each settled step, in step order: the same walk again
      const bool sums = s.sum_u && r == 0;
      RoundSums<3> rsum(sums ? s.sum_u + chain * 3 : nullptr, (sums && s.sum_u2) ? s.sum_u2 + chain * 3 : nullptr,
                        sums ? 3 : 0);
      auto visit = [&](int q, int la) {
        T vq[3];
        slot_v(la >= 0 ? la : 0, vq);
        if (r == 0) {
          if (sums) {
#pragma unroll
            for (int j = 0; j < 3; ++j) rsum.add(j, la >= 0 ? (double)vq[j] : (double)ur[j]);
          }
          if (s.sample_every > 0 && clk.next == st + q) {
            // the state after step st+q is a sample
            const int64_t sl = clk.take(clk.next);
            T* so = (T*)s.sample_out + chain * s.sample_stride + sl * s.sample_step_stride;
#pragma unroll
            for (int j = 0; j < 3; ++j) so[j] = la >= 0 ? vq[j] : ur[j];
          }
        }
      };
      if (G <= 64) spec_path_replay(path, accm, visit);
      else spec_replay(rd.used, node, visit);
      if (sums) rsum.store();
    }
    if (G > 64) __syncthreads();  // bmask / vpk are rewritten next round
    else wave_sync_lds();
    if (rd.win >= 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) ur[j] = vf[j];
      phu = phf;
    }
    nacc += rd.nar;
    ncalls += rd.calls;
    guess.settle(rd.nar, rd.used);
    st += rd.used;
  }
  if (r == 0) {
    phi[chain] = phu;
    if (s.accepts) s.accepts[chain] += nacc;
    if (s.calls) s.calls[chain] += ncalls;
#pragma unroll
    for (int j = 0; j < 3; ++j) u[j] = ur[j];
    if (s.sample_out && s.sample_every == 0) {
      T* so = (T*)s.sample_out + chain * s.sample_stride;
#pragma unroll
      for (int j = 0; j < 3; ++j) so[j] = ur[j];
    }
  }
}

template <typename T, int CPL, int GS, bool FM, bool PHI>
__global__ __launch_bounds__(kBurBlock) void burgers_eval_kernel(const ipmc_model m, int64_t n,
                                                                 const T* __restrict__ uin, const T* __restrict__ y,
                                                                 const T* __restrict__ ginv, T* __restrict__ out) {
  __shared__ T lds[kBurBlock * CPL];
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * kBurBlock + threadIdx.x;
  const int64_t chain = tid / GS;
  const BurCtx c{(int)(tid % GS), lane, m.dim / CPL};
  if (chain >= n) return;
  T* row = lds + (threadIdx.x & ~(GS - 1)) * CPL;
  const T v[3] = {uin[chain * 3], uin[chain * 3 + 1], uin[chain * 3 + 2]};
  const T ph = burgers_phi<T, CPL, GS, FM>(m, v, c, row, PHI ? y : nullptr, ginv, PHI ? nullptr : out + chain * m.q);
  if (PHI && c.sub == 0) out[chain] = ph;
}

// ------------------------------------------------------------------ host
// Supported layouts: CPL cells per lane, GS lanes per chain.
static bool fit(int N, int c, int& cpl, int& gs) {
  if (N % c) return false;
  const int need = N / c;
  const int groups[3] = {16, 32, 64};
  for (int g : groups) {
    if (need <= g) {
      cpl = c;
      gs = g;
      return true;
    }
  }
  return false;
}

// Prefer 8 cells per lane (more independent work per lane between halo
// exchanges); 4 when a chain does not fit 8-cell lanes.  Measured on cfg 4
// (N=256): 8 cells beat 4 even for 2 048 chains, where 4 would double the
// waves per SIMD (profiles/r1/configs.jsonl).  lanes_per_chain > 0
// (ipmc_sweep) forces CPL = N / lanes_per_chain.
static bool pick(int N, int64_t n_chains, int lanes, int& cpl, int& gs) {
  (void)n_chains;
  if (lanes > 0) return (N % lanes == 0) && fit(N, N / lanes, cpl, gs);
  return fit(N, 8, cpl, gs) || fit(N, 4, cpl, gs);
}

// Speculation width: spec_width if given (a power of two, S·GS <= 64), else for
// multi-step launches the widest keeping the ensemble within one wave per SIMD.
template <int GS>
static int burgers_spec(const ipmc_sweep& s) {
  if (s.spec_width > 0) {
    const int w = s.spec_width;
    return ((w & (w - 1)) == 0 && (w * GS <= 64 || w * GS == kBurBlock)) ? w : -1;
  }
  int w = 1;
  if (s.n_steps > 1) {
    while (w * 2 * GS <= 64 && s.n_chains * (int64_t)GS * w * 2 <= 65536) w *= 2;
    // a whole block of slots per chain while the ensemble stays within one wave per SIMD
    if (w * GS == 64 && s.n_chains * (int64_t)kBurBlock <= 65536) w = kBurBlock / GS;
  }
  return w;
}

template <typename T, int CPL, int GS, bool FM>
static int launch_sweep(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  const int S = burgers_spec<GS>(s);
  if (S < 1) {
    set_error("Burgers: spec_width must be a power of two with spec_width * %d lanes <= 64 or = 256", GS);
    return IPMC_ERR_UNSUPPORTED;
  }
  const int64_t blocks = (s.n_chains * GS * S + kBurBlock - 1) / kBurBlock;
  hipLaunchKernelGGL((burgers_sweep_kernel<T, CPL, GS, FM>), dim3((unsigned)blocks), dim3(kBurBlock), 0, st, m, s,
                     S);
  return check_launch("burgers_sweep_kernel");
}

template <typename T, int CPL, int GS, bool FM>
static int launch_eval(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                       bool phi, hipStream_t st) {
  const int64_t blocks = (n * GS + kBurBlock - 1) / kBurBlock;
  if (phi)
    hipLaunchKernelGGL((burgers_eval_kernel<T, CPL, GS, FM, true>), dim3((unsigned)blocks), dim3(kBurBlock), 0, st,
                       m, n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);
  else
    hipLaunchKernelGGL((burgers_eval_kernel<T, CPL, GS, FM, false>), dim3((unsigned)blocks), dim3(kBurBlock), 0, st,
                       m, n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);
  return check_launch("burgers_eval_kernel");
}

template <typename T, bool FM, typename F>
static int dispatch(int cpl, int gs, F&& f) {
#define IPMC_BUR(C, G) \
  if (cpl == C && gs == G) return f.template operator()<T, C, G, FM>();
  IPMC_BUR(8, 16) IPMC_BUR(8, 32) IPMC_BUR(8, 64) IPMC_BUR(4, 16) IPMC_BUR(4, 32) IPMC_BUR(4, 64)
#undef IPMC_BUR
  return IPMC_ERR_UNSUPPORTED;
}

static int validate(const ipmc_model& m, int64_t n_chains, int lanes, int& cpl, int& gs) {
  if (m.q > kBurQMax) {
    set_error("Burgers: at most %d observation windows", kBurQMax);
    return IPMC_ERR_UNSUPPORTED;
  }
  if (!pick(m.dim, n_chains, lanes, cpl, gs) || (cpl != 4 && cpl != 8)) {
    set_error("Burgers: N=%d must be a multiple of 4 and at most 512 (lanes_per_chain=%d: N/lanes must be 4 or 8)",
              m.dim, lanes);
    return IPMC_ERR_UNSUPPORTED;
  }
  return IPMC_OK;
}

struct SweepLauncher {
  const ipmc_model& m;
  const ipmc_sweep& s;
  hipStream_t st;
  template <typename T, int C, int G, bool FM>
  int operator()() {
    return launch_sweep<T, C, G, FM>(m, s, st);
  }
};

struct EvalLauncher {
  const ipmc_model& m;
  int64_t n;
  const void *u, *y, *ginv;
  void* out;
  bool phi;
  hipStream_t st;
  template <typename T, int C, int G, bool FM>
  int operator()() {
    return launch_eval<T, C, G, FM>(m, n, u, y, ginv, out, phi, st);
  }
};

int burgers_sweep(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  int cpl, gs;
  int rc = validate(m, s.n_chains, s.lanes_per_chain, cpl, gs);
  if (rc) return rc;
  SweepLauncher l{m, s, st};
  const bool fm = m.arith == IPMC_ARITH_FMA;
  if (s.dtype == IPMC_F64) return fm ? dispatch<double, true>(cpl, gs, l) : dispatch<double, false>(cpl, gs, l);
  return fm ? dispatch<float, true>(cpl, gs, l) : dispatch<float, false>(cpl, gs, l);
}

int burgers_plan(const ipmc_model& m, const ipmc_sweep& s, int& lanes, int& spec) {
  int cpl, gs;
  const int rc = validate(m, s.n_chains, s.lanes_per_chain, cpl, gs);
  if (rc) return rc;
  lanes = gs;
  spec = gs == 16 ? burgers_spec<16>(s) : gs == 32 ? burgers_spec<32>(s) : burgers_spec<64>(s);
  if (spec < 1) {
    set_error("Burgers: spec_width must be a power of two with spec_width * %d lanes <= 64 or = 256", gs);
    return IPMC_ERR_UNSUPPORTED;
  }
  return IPMC_OK;
}

int burgers_eval(const ipmc_model& m, int32_t dtype, int64_t n, const void* u, const void* y, const void* ginv,
                 void* out, bool phi, hipStream_t st) {
  int cpl, gs;
  int rc = validate(m, n, 0, cpl, gs);
  if (rc) return rc;
  EvalLauncher l{m, n, u, y, ginv, out, phi, st};
  const bool fm = m.arith == IPMC_ARITH_FMA;
  if (dtype == IPMC_F64) return fm ? dispatch<double, true>(cpl, gs, l) : dispatch<double, false>(cpl, gs, l);
  return fm ? dispatch<float, true>(cpl, gs, l) : dispatch<float, false>(cpl, gs, l);
}

}  // namespace ipmc
