// Two-scale Lorenz-96 (lorenz.py:44-101 with J > 0) forward map, observed by
// the time-averaged moment function of lorenz_mcmc.py:17-40, and its pCN sweep.
//
// Layout: one chain per group of L = K/SPL consecutive lanes, floor(64/L)
// chains per wave (groups need not be power-of-two aligned: K=6 at SPL 1 packs
// 10 chains = 60 live lanes per wave); lane i owns the SPL slow variables
// X_{i*SPL..i*SPL+SPL-1} and their fast blocks Y_{k,0..J-1} in VGPRs (1+J
// values per slow variable and RK4 array).  The fast blocks are cyclic inside
// the block (np.roll of Y_in[k, :]) so they never leave the lane; the slow
// neighbours X_{k-2}, X_{k-1}, X_{k+1} (cyclic mod K) of the lane's first and
// last slow variables come from the neighbouring lanes: by ds_bpermute in
// general, by one DPP quad_perm swap when L = 2 (SPL 3 for K = 6), and not at
// all when L = 1 (SPL 6 for K = 6: the whole chain in one lane).
// theta = (F, h, b) = theta0 + u is the same on every lane of the group.
// Lane k accumulates the five moments of slot k; Φ sums the 5K residuals in
// observation order (every lane gathers them, so all lanes hold Φ).
#include "ipmc_internal.hpp"
#include "ipmc_sweep_common.hpp"

namespace ipmc {

constexpr int kTsBlock = 256;

#ifndef IPMC_TS_PK
#define IPMC_TS_PK 1
#endif

// SPL 3 and 6 are compiled for K = 6 (the reference's K=6 J=4 study,
// lorenz_mcmc.py:87-88): lanes per chain fixed at 2 (DPP halos) and 1 (none).
// (A ring of K/3 lanes for K = 36, 5 chains = 60 live lanes per wave instead of
// 54, measured slower: f64 needs one wave and AGPR spills at 3 x 11 values per
// RK array, 0.94 vs 1.11 M pCN steps/s; fp32 1.53 vs 1.69 M;
// profiles/r5/ts36_layouts.jsonl.)
template <int SPL>
constexpr int ts_fixed_lanes() {
  return SPL == 3 ? 2 : (SPL == 6 ? 1 : 0);
}
// the (SPL, J) pairs a kernel is compiled for
template <int SPL, int J>
constexpr bool ts_compiled() {
  return SPL == 1 || (SPL == 2 && J <= 10) || (SPL > 2 && J <= 4);
}

// The slow ring's halos (K > 32, two slow variables per lane) through LDS --
// one row per lane written once per stage, three neighbour reads -- instead of
// three ds_bpermute: 1-1.6 % faster on K=36 J=10 in f64 and fp32, four
// interleaved A/Bs (profiles/r5/ts36_layouts.jsonl); 0 for the permute form.
#ifndef IPMC_TS_LDS_HALO
#define IPMC_TS_LDS_HALO 1
#endif

// Occupancy target (waves per SIMD) for the sweep kernel: 4 RK4 arrays of
// 1 + J values per lane plus the chain state.
template <typename T, int J, int SPL>
constexpr int ts_waves() {
#ifdef IPMC_TS_WAVES  // layout experiments (tools/)
  return IPMC_TS_WAVES;
#endif
  if constexpr (SPL == 6) return sizeof(T) == 8 ? 1 : 2;
  if constexpr (SPL == 3) return sizeof(T) == 8 ? 2 : 3;
  if constexpr (SPL == 2) return sizeof(T) == 8 ? (J <= 4 ? 3 : 2) : (J <= 2 ? 4 : (J <= 8 ? 3 : 2));
  return sizeof(T) == 8 ? (J <= 4 ? 4 : (J <= 10 ? 3 : 2)) : (J <= 2 ? 5 : (J <= 8 ? 4 : (J <= 10 ? 3 : 2)));
}

struct TsCtx {
  int K, sub, base;  // base = first lane of the group, sub = k
};

// lane -> (chain, k) for the packed layout; chain < 0 for the idle tail lanes.
__device__ __forceinline__ int64_t ts_chain(int K, TsCtx& c) {
  const int lane = threadIdx.x & 63;
  const int cpw = 64 / K;
  const int slot = lane / K;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  c.K = K;
  c.sub = lane - slot * K;
  c.base = slot * K;
  return slot < cpw ? wave * cpw + slot : -1;
}

// numpy pairwise_sum order (n <= 128) of a compile-time-sized array.
template <typename T, int J>
__device__ __forceinline__ T np_pairwise(const T (&a)[J], int off) {
  if constexpr (J < 8) {
    T res = (T)0;
#pragma unroll
    for (int i = 0; i < J; ++i) res = res + a[off + i];
    return res;
  } else {
    T r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[off + j];
    constexpr int full = J - (J % 8);
#pragma unroll
    for (int i = 8; i < full; i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + a[off + i + j];
    }
    T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int i = full; i < J; ++i) res = res + a[off + i];
    return res;
  }
}

// state s[0] = X_k, s[1 + j] = Y_{k,j}
template <typename T, int J>
__device__ __forceinline__ T block_mean(const T (&s)[1 + J]) {
  T y[J];
#pragma unroll
  for (int j = 0; j < J; ++j) y[j] = s[1 + j];
  return np_pairwise<T, J>(y, 0) / (T)J;
}

// Per-evaluation coefficients: theta = (F, h, b), hc = h c (fast_slow_fact,
// lorenz.py:42), hJ = h / J (lorenz.py:98); FMA arith also folds the block
// mean's 1/J into hc (hcJ = hc / J) and c into the fast rate (chJ = c hJ,
// cb = c b), so no stage needs a division or the final scaling by c.
template <typename T>
struct TsCoef {
  T F, hc, hJ, bb, cc, hcJ, chJ, cb;
};

template <typename T>
__device__ __forceinline__ TsCoef<T> ts_coef(T F, T h, T bb, T cc, int J) {
  TsCoef<T> k;
  k.F = F;
  k.bb = bb;
  k.cc = cc;
  k.hc = h * cc;
  k.hJ = h / (T)J;
  k.hcJ = k.hc / (T)J;
  k.chJ = cc * k.hJ;
  k.cb = cc * bb;
  return k;
}

// dX_k/dt (lorenz.py:77-86) and dY_{k,j}/dt (lorenz.py:94-99).
// REFERENCE: yb = block mean, the reference's operation order.
// FMA: ys = block SUM, t = fma(x_{k+1} - x_{k-2}, x_{k-1}, F - X); fma(-hc/J, ys, t).
template <typename T, bool FM>
__device__ __forceinline__ T ts_slow(T X, T xm1, T xm2, T xp1, const TsCoef<T>& k, T ys) {
  const T F = k.F, hc = k.hc, yb = ys;
  if constexpr (FM) {
    const T t = madd<true>(xp1 - xm2, xm1, F - X);
    return madd<true>(-k.hcJ, ys, t);
  } else {
    T t = -X;
    t = t - (xm1 * xm2 - xm1 * xp1);
    t = t + F;
    return t - hc * yb;
  }
}

// REFERENCE: c (((-y) - b (y_{j+1} y_{j+2} - y_{j-1} y_{j+1})) + hJ X).
// FMA: fma(-c b, y_{j+1} (y_{j+2} - y_{j-1}), fma(-c, y, qX)) with qX = c hJ X
// computed once per slow variable and stage.
template <typename T, bool FM>
__device__ __forceinline__ T ts_fast(T y, T yp1, T yp2, T ym1, T X, T qX, const TsCoef<T>& k) {
  if constexpr (FM) {
    const T nl = yp1 * (yp2 - ym1);
    return madd<true>(-k.cb, nl, madd<true>(-k.cc, y, qX));
  } else {
    T t = -y;
    t = t - k.bb * (yp1 * yp2 - ym1 * yp1);
    t = t + k.hJ * X;
    return t * k.cc;
  }
}

// FMA arith's block sum (REFERENCE: block_mean).
template <typename T, int J>
__device__ __forceinline__ T block_sum(const T (&s)[1 + J]) {
  T y[J];
#pragma unroll
  for (int j = 0; j < J; ++j) y[j] = s[1 + j];
  return np_pairwise<T, J>(y, 0);
}

// Slow neighbours of a lane holding SPL >= 2 slow variables Xo: p1 = X_{k0-1},
// p2 = X_{k0-2} (the previous lane's last two) and n0 = X_{k0+SPL} (the next
// lane's first), cyclic over the group's L = K/SPL lanes.
template <int SPL, typename T>
__device__ __forceinline__ void ts_halo(const T (&Xo)[SPL], const TsCtx& c, T& p1, T& p2, T& n0) {
  constexpr int LF = ts_fixed_lanes<SPL>();
  if constexpr (LF == 1) {  // the whole ring in this lane
    p1 = Xo[SPL - 1];
    p2 = Xo[SPL - 2];
    n0 = Xo[0];
  } else if constexpr (LF == 2) {  // previous = next = the other lane of the (pair-aligned) group
    p1 = dpp<qperm(1, 0, 3, 2)>(Xo[SPL - 1]);
    p2 = dpp<qperm(1, 0, 3, 2)>(Xo[SPL - 2]);
    n0 = dpp<qperm(1, 0, 3, 2)>(Xo[0]);
  } else {
    const int L = c.K / SPL;
    const int prev = c.base + (c.sub + L - 1) % L, next = c.base + (c.sub + 1) % L;
#if IPMC_TS_LDS_HALO
    __shared__ T ring[kTsBlock][SPL];  // the wave's slow variables, one row per lane
    const int w0 = threadIdx.x & ~63;
#pragma unroll
    for (int a = 0; a < SPL; ++a) ring[threadIdx.x][a] = Xo[a];
    wave_sync_lds();
    p1 = ring[w0 + prev][SPL - 1];
    p2 = ring[w0 + prev][SPL - 2];
    n0 = ring[w0 + next][0];
    wave_sync_lds();  // read before the next stage rewrites the ring
#else
    p1 = shfl(Xo[SPL - 1], prev);
    p2 = shfl(Xo[SPL - 2], prev);
    n0 = shfl(Xo[0], next);
#endif
  }
}

// One classical RK4 stage over the lane's SPL slow variables k = sub*SPL + a
// and their fast blocks, with each rate k consumed as soon as it is computed:
//   STAGE 1: acc = k;           out = base + c*k     (in = x, out = xs)
//   STAGE 2/3: acc = 2k + acc;  out = base + c*k     (in = out = xs)
//   STAGE 4: acc = acc + k;     out = base + c*acc   (in = xs, out = x)
// -- the same operations as the textbook form, so the bits do not change, but
// no separate array of rates: `in` may alias `out` because every value an
// element still needs is read before it is overwritten (the old X and block
// mean, the old Y_{k,0}, Y_{k,1} for the cyclic wrap and the previous old Y).
// Slow neighbours across lanes come by ds_bpermute, cyclic over the group's
// L = K/SPL lanes, before anything is written.
template <typename T, int J, bool FM, int SPL, int STAGE>
__device__ __forceinline__ void ts_stage(T (&in)[SPL][1 + J], T (&out)[SPL][1 + J], T (&base)[SPL][1 + J],
                                         T (&acc)[SPL][1 + J], T cst, const TsCoef<T>& kc, const TsCtx& c) {
  auto upd = [&](int a, int i, T k) {
    if constexpr (STAGE == 1) acc[a][i] = k;
    else if constexpr (STAGE == 4) acc[a][i] = acc[a][i] + k;
    else acc[a][i] = madd<FM>((T)2, k, acc[a][i]);
    if constexpr (STAGE == 4) out[a][i] = madd<FM>(cst, acc[a][i], base[a][i]);
    else out[a][i] = madd<FM>(cst, k, base[a][i]);
  };
  const int L = c.K / SPL;
  T Xo[SPL], yb[SPL], kX[SPL];
#pragma unroll
  for (int a = 0; a < SPL; ++a) {
    Xo[a] = in[a][0];
    yb[a] = FM ? block_sum<T, J>(in[a]) : block_mean<T, J>(in[a]);
  }
  if constexpr (SPL == 1) {
    const T xm1 = __shfl(Xo[0], c.base + (c.sub + L - 1) % L, 64);
    const T xm2 = __shfl(Xo[0], c.base + (c.sub + L - 2) % L, 64);
    const T xp1 = __shfl(Xo[0], c.base + (c.sub + 1) % L, 64);
    kX[0] = ts_slow<T, FM>(Xo[0], xm1, xm2, xp1, kc, yb[0]);
  } else {
    T p1, p2, n0;  // X_{k0-1}, X_{k0-2}, X_{k0+SPL}
    ts_halo<SPL, T>(Xo, c, p1, p2, n0);
#pragma unroll
    for (int a = 0; a < SPL; ++a) {
      const T xm1 = a >= 1 ? Xo[a - 1] : p1;
      const T xm2 = a >= 2 ? Xo[a - 2] : (a == 1 ? p1 : p2);
      const T xp1 = a + 1 < SPL ? Xo[a + 1] : n0;
      kX[a] = ts_slow<T, FM>(Xo[a], xm1, xm2, xp1, kc, yb[a]);
    }
  }
#pragma unroll
  for (int a = 0; a < SPL; ++a) {
    upd(a, 0, kX[a]);
    const T qX = FM ? kc.chJ * Xo[a] : (T)0;
    const T y0 = in[a][1], y1 = in[a][1 + (1 % J)];
    T prev = in[a][J];  // old Y_{k,J-1}: the j = 0 element's left neighbour
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const T y = in[a][1 + j];  // elements >= j are not yet overwritten
      const T yp1 = (j + 1 < J) ? in[a][2 + j] : y0;
      const T yp2 = (j + 2 < J) ? in[a][3 + j] : ((j + 2 - J) == 0 ? y0 : y1);
      const T k = ts_fast<T, FM>(y, yp1, yp2, prev, Xo[a], qX, kc);
      prev = y;
      upd(a, 1 + j, k);
    }
  }
}

// fp32 with J even: each fast block held as H = J/2 pairs of f32x2,
// Y[p] = (Y_{k,p}, Y_{k,p+H}), so the fast rates and RK4 updates are
// v_pk_*_f32 on two fast variables.  The block's cyclic neighbours of pair p
// are pairs p±1, p+2 with the halves swapped each time the index wraps past H
// (ts_pair); every per-element operation is the scalar kernel's, so the bits
// are the same (the block sum / mean still adds the scalars in numpy's order).
template <int H>
__device__ __forceinline__ f32x2 ts_pair(const f32x2 (&y)[H], const f32x2& old0, const f32x2& old1, int i) {
  // pair i of the cyclic sequence, i in [-1, H + 1]; indices >= H read the
  // saved old pairs 0 / 1 (the in-place stage has overwritten them)
  const int w = i < 0 ? -1 : i / H;
  const int j = i - w * H;
  const f32x2 v = (w >= 1) ? (j == 0 ? old0 : old1) : y[j];
  return (w & 1) ? __builtin_shufflevector(v, v, 1, 0) : v;
}

template <int J>
__device__ __forceinline__ float ts_pk_sum(const f32x2 (&y)[J / 2], bool mean) {
  constexpr int H = J / 2;
  float a[J];
#pragma unroll
  for (int p = 0; p < H; ++p) {
    a[p] = y[p].x;
    a[p + H] = y[p].y;
  }
  const float sm = np_pairwise<float, J>(a, 0);
  return mean ? sm / (float)J : sm;
}

template <int J, bool FM, int SPL, int STAGE>
__device__ __forceinline__ void ts_stage_pk(float (&xin)[SPL], f32x2 (&yin)[SPL][J / 2], float (&xout)[SPL],
                                            f32x2 (&yout)[SPL][J / 2], float (&xb)[SPL], f32x2 (&yb)[SPL][J / 2],
                                            float (&xa)[SPL], f32x2 (&ya)[SPL][J / 2], float cst,
                                            const TsCoef<float>& kc, const TsCoef<f32x2>& kv, const TsCtx& c) {
  constexpr int H = J / 2;
  auto upd = [&](auto& acc, auto& out, const auto& base, auto k, auto cs) {
    using V = decltype(k);
    if constexpr (STAGE == 1) acc = k;
    else if constexpr (STAGE == 4) acc = acc + k;
    else acc = madd<FM>(Splat<V>::of(2.0f), k, acc);
    if constexpr (STAGE == 4) out = madd<FM>(cs, acc, base);
    else out = madd<FM>(cs, k, base);
  };
  const f32x2 csv{cst, cst};
  const int L = c.K / SPL;
  float Xo[SPL], ybk[SPL], kX[SPL];
#pragma unroll
  for (int a = 0; a < SPL; ++a) {
    Xo[a] = xin[a];
    ybk[a] = ts_pk_sum<J>(yin[a], !FM);
  }
  if constexpr (SPL == 1) {
    const float xm1 = __shfl(Xo[0], c.base + (c.sub + L - 1) % L, 64);
    const float xm2 = __shfl(Xo[0], c.base + (c.sub + L - 2) % L, 64);
    const float xp1 = __shfl(Xo[0], c.base + (c.sub + 1) % L, 64);
    kX[0] = ts_slow<float, FM>(Xo[0], xm1, xm2, xp1, kc, ybk[0]);
  } else {
    float p1, p2, n0;
    ts_halo<SPL, float>(Xo, c, p1, p2, n0);
#pragma unroll
    for (int a = 0; a < SPL; ++a) {
      const float xm1 = a >= 1 ? Xo[a - 1] : p1;
      const float xm2 = a >= 2 ? Xo[a - 2] : (a == 1 ? p1 : p2);
      const float xp1 = a + 1 < SPL ? Xo[a + 1] : n0;
      kX[a] = ts_slow<float, FM>(Xo[a], xm1, xm2, xp1, kc, ybk[a]);
    }
  }
#pragma unroll
  for (int a = 0; a < SPL; ++a) {
    upd(xa[a], xout[a], xb[a], kX[a], cst);
    const f32x2 Xv{Xo[a], Xo[a]};
    const float q = FM ? kc.chJ * Xo[a] : 0.0f;
    const f32x2 qX{q, q};
    const f32x2 old0 = yin[a][0], old1 = yin[a][1 % H];
    f32x2 prevp = ts_pair<H>(yin[a], old0, old1, -1);  // old pair -1 (= pair H-1, swapped)
#pragma unroll
    for (int p = 0; p < H; ++p) {
      const f32x2 y = yin[a][p];  // pairs >= p are not yet overwritten
      const f32x2 yp1 = ts_pair<H>(yin[a], old0, old1, p + 1);
      const f32x2 yp2 = ts_pair<H>(yin[a], old0, old1, p + 2);
      const f32x2 k = ts_fast<f32x2, FM>(y, yp1, yp2, prevp, Xv, qX, kv);
      prevp = y;
      upd(ya[a][p], yout[a][p], yb[a][p], k, csv);
    }
  }
}

// ts_phi for fp32 with J even: the fast blocks as pairs (ts_stage_pk).
template <int J, bool FM, int SPL>
__device__ float ts_phi_pk(const ipmc_model& m, const float (&v)[3], const TsCtx& c, int kq, const float* __restrict__ y,
                           const float* __restrict__ ginv, float* g_out) {
  constexpr int H = J / 2;
  const int K = c.K;
  const int k0 = kq * SPL;
  const float* th0 = (const float*)m.theta0;
  const float F = th0[0] + v[0], h = th0[1] + v[1], bb = th0[2] + v[2];
  const TsCoef<float> kc = ts_coef<float>(F, h, bb, (float)m.coupling_c, J);
  TsCoef<f32x2> kv;
  kv.F = f32x2{kc.F, kc.F};
  kv.hc = f32x2{kc.hc, kc.hc};
  kv.hJ = f32x2{kc.hJ, kc.hJ};
  kv.bb = f32x2{kc.bb, kc.bb};
  kv.cc = f32x2{kc.cc, kc.cc};
  kv.hcJ = f32x2{kc.hcJ, kc.hcJ};
  kv.chJ = f32x2{kc.chJ, kc.chJ};
  kv.cb = f32x2{kc.cb, kc.cb};
  const float rJ = 1.0f / (float)J;
  const float hh = (float)m.dt, h2 = hh * 0.5f, h6 = hh / 6.0f;
  const float* x0 = (const float*)m.x0;
  float X[SPL], ob[SPL][5];
  f32x2 Y[SPL][H];
#pragma unroll
  for (int i = 0; i < SPL; ++i) {
    X[i] = x0[k0 + i];
    const float* yb0 = x0 + K + (k0 + i) * J;
#pragma unroll
    for (int p = 0; p < H; ++p) Y[i][p] = f32x2{yb0[p], yb0[p + H]};
#pragma unroll
    for (int b = 0; b < 5; ++b) ob[i][b] = 0.0f;
  }
  const bool refmom = (m.moment_mode == 0);
  for (int n = 0; n < m.n_steps; ++n) {
    float xa[SPL], xs[SPL];
    f32x2 ya[SPL][H], ys[SPL][H];
    ts_stage_pk<J, FM, SPL, 1>(X, Y, xs, ys, X, Y, xa, ya, h2, kc, kv, c);
    ts_stage_pk<J, FM, SPL, 2>(xs, ys, xs, ys, X, Y, xa, ya, h2, kc, kv, c);
    ts_stage_pk<J, FM, SPL, 3>(xs, ys, xs, ys, X, Y, xa, ya, hh, kc, kv, c);
    ts_stage_pk<J, FM, SPL, 4>(xs, ys, X, Y, X, Y, xa, ya, h6, kc, kv, c);
#pragma unroll
    for (int a = 0; a < SPL; ++a) {
      const float Xa = X[a];
      const float yb = refmom ? Y[a][0].x : (FM ? ts_pk_sum<J>(Y[a], false) * rJ : ts_pk_sum<J>(Y[a], true));
      ob[a][0] = ob[a][0] + Xa;
      ob[a][1] = ob[a][1] + yb;
      ob[a][2] = madd<FM>(Xa, Xa, ob[a][2]);
      ob[a][3] = madd<FM>(Xa, yb, ob[a][3]);
      ob[a][4] = madd<FM>(yb, yb, ob[a][4]);
    }
  }
  const float nn = (float)m.n_steps;
  float r[SPL][5];
#pragma unroll
  for (int a = 0; a < SPL; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const int k = k0 + a;
      const float g = ob[a][b] / nn;
      if (g_out) g_out[b * K + k] = g;
      r[a][b] = y ? (y[b * K + k] - g) * ginv[b * K + k] : 0.0f;
    }
  float s = 0.0f;
  if (y) {
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      for (int l = 0; l < K / SPL; ++l) {  // observation order: slow variable l*SPL + a of moment b
#pragma unroll
        for (int a = 0; a < SPL; ++a) {
          const float val = __shfl(r[a][b], c.base + l, 64);
          s = madd<FM>(val, val, s);
        }
      }
    }
  }
  return 0.5f * s;
}

// Φ(theta0 + v) for the group; g_out (per chain, [5K]) receives G if set.
// kq: k behind an opaque register copy made once per pCN step, so the
// per-lane constants (x0 block, y, 1/gamma) are re-read each step instead of
// being hoisted into VGPRs for the whole sweep.
template <typename T, int J, bool FM, int SPL>
__device__ T ts_phi(const ipmc_model& m, const T (&v)[3], const TsCtx& c, int kq, const T* __restrict__ y,
                    const T* __restrict__ ginv, T* g_out) {
  if constexpr (sizeof(T) == 4 && J % 2 == 0 && IPMC_TS_PK)
    return ts_phi_pk<J, FM, SPL>(m, v, c, kq, y, ginv, g_out);
  const int K = c.K;
  const int k0 = kq * SPL;  // this lane's first slow variable
  const T* th0 = (const T*)m.theta0;
  const T F = th0[0] + v[0], h = th0[1] + v[1], bb = th0[2] + v[2];
  const TsCoef<T> kc = ts_coef<T>(F, h, bb, (T)m.coupling_c, J);
  const T rJ = (T)1 / (T)J;
  const T hh = (T)m.dt, h2 = hh * (T)0.5, h6 = hh / (T)6;
  const T* x0 = (const T*)m.x0;
  T x[SPL][1 + J];
  T ob[SPL][5];
#pragma unroll
  for (int i = 0; i < SPL; ++i) {
    x[i][0] = x0[k0 + i];
#pragma unroll
    for (int j = 0; j < J; ++j) x[i][1 + j] = x0[K + (k0 + i) * J + j];
#pragma unroll
    for (int b = 0; b < 5; ++b) ob[i][b] = (T)0;
  }
  const bool refmom = (m.moment_mode == 0);
  for (int n = 0; n < m.n_steps; ++n) {
    T acc[SPL][1 + J], xs[SPL][1 + J];
    ts_stage<T, J, FM, SPL, 1>(x, xs, x, acc, h2, kc, c);
    ts_stage<T, J, FM, SPL, 2>(xs, xs, x, acc, h2, kc, c);
    ts_stage<T, J, FM, SPL, 3>(xs, xs, x, acc, hh, kc, c);
    ts_stage<T, J, FM, SPL, 4>(xs, x, x, acc, h6, kc, c);
#pragma unroll
    for (int a = 0; a < SPL; ++a) {
      const T X = x[a][0];
      // FMA arith: the block mean as sum * (1/J) (REFERENCE: np.mean's division)
      const T yb = refmom ? x[a][1] : (FM ? block_sum<T, J>(x[a]) * rJ : block_mean<T, J>(x[a]));
      ob[a][0] = ob[a][0] + X;
      ob[a][1] = ob[a][1] + yb;
      ob[a][2] = madd<FM>(X, X, ob[a][2]);
      ob[a][3] = madd<FM>(X, yb, ob[a][3]);
      ob[a][4] = madd<FM>(yb, yb, ob[a][4]);
    }
  }
  const T nn = (T)m.n_steps;
  T r[SPL][5];
#pragma unroll
  for (int a = 0; a < SPL; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const int k = k0 + a;
      const T g = ob[a][b] / nn;
      if (g_out) g_out[b * K + k] = g;
      r[a][b] = y ? (y[b * K + k] - g) * ginv[b * K + k] : (T)0;
    }
  T s = (T)0;
  if (y) {
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      for (int l = 0; l < K / SPL; ++l) {  // observation order: slow variable l*SPL + a of moment b
#pragma unroll
        for (int a = 0; a < SPL; ++a) {
          const T val = __shfl(r[a][b], c.base + l, 64);
          s = madd<FM>(val, val, s);
        }
      }
    }
  }
  return (T)0.5 * s;
}

// Sweep with S speculative slots per chain (S = 1: the plain sequential chain).
// A chain owns S consecutive groups of L = K/SPL lanes; slot s is node s of
// the speculation tree for the chain's recent acceptance rate (see
// small_spec_kernel, ipmc_spec_tree.hpp) -- bit-identical to S = 1.
// ⌊64 / (S·L)⌋ chains per wave.
template <typename T, int J, bool FM, int SPL>
__global__ __launch_bounds__(kTsBlock, (ts_waves<T, J, SPL>())) void l96ts_sweep_kernel(const ipmc_model m,
                                                                                      const ipmc_sweep s, int S) {
  __shared__ T vpk[3][kTsBlock];  // the proposals, for the recorded states of a round
  const int lane = threadIdx.x & 63;
  const int K = m.dim, L = K / SPL, G = S * L;
  const int cpw = 64 / G;
  const int q = lane / G, r = lane - q * G;
  const int slot = r / L;
  const int cbase = q * G;  // the chain's first lane in the wave
  TsCtx c{K, r - slot * L, cbase + slot * L};
  const int64_t chain = q < cpw ? (((int64_t)blockIdx.x * kTsBlock + threadIdx.x) >> 6) * cpw + q : -1;
  if (chain < 0 || chain >= s.n_chains) return;
  const uint64_t gid = (uint64_t)(s.chain_offset + chain);
  T* u = (T*)s.u + chain * 3;
  T ur[3] = {u[0], u[1], u[2]};
  const T* sq = (const T*)s.prior_sqrt;
  const T beta = (T)s.beta, contr = (T)s.contraction;
  const bool rw = (s.proposal == IPMC_PROPOSAL_RW);
  T* phi = (T*)s.phi;
  T phu = phi[chain];
  int nacc = 0, ncalls = 0;
  SampleClock clk(s);
  int64_t st = 0;
  SpecGuess guess(spec_accept_prior(s, chain));  // the speculation tree (ipmc_sweep_common.hpp)
  const T* chol = (const T*)s.prior_chol;
  const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1);
  while (st < s.n_steps) {
    const int64_t left = s.n_steps - st;
    const int tb = S > 1 ? guess.bucket() : 0;
    const SpecNode nd = kSpecTrees.nd[tb][slot];
    const int maxlvl = kSpecTrees.maxlvl[tb][S];
    const bool act = nd.depth < left;  // uniform per slot
    const int64_t tt = st + nd.depth;
    const int ol = cbase + (nd.orig < 0 ? 0 : nd.orig) * L;  // the origin slot's first lane
    int kq = c.sub;
    asm volatile("" : "+v"(kq));
    bool ok = false, acc = false;
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
#pragma unroll
      for (int j = 0; j < 3; ++j) o[j] = __shfl(v[j], ol, 64);
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
        phv = ts_phi<T, J, FM, SPL>(m, v, c, kq, (const T*)s.y, (const T*)s.gamma_inv, nullptr);
        if (s.reg_scale) phv = phv + regularizer<T, 3, 1, FM>((const T*)s.reg_scale, v, lane);
        lr = det_log(accept_uniform(s.seed, gid, step));
      }
    }
    // pcn_accept against the state this node proposed from: the chain's, or
    // its origin node's proposal (whose Φ that slot's lanes hold)
    const T pho = __shfl(phv, ol, 64);
    if (ok) acc = (double)((nd.orig < 0 ? phu : pho) - phv) > lr;
    // one bit per slot (its first lane, at bit slot*L of the chain's lanes); the
    // walk resolved in parallel (spec_on_path, as ipmc_l96.hpp): no cross-lane
    // read inside a data-dependent loop
    const unsigned long long accm = spec_slot_bits((__ballot(acc && c.sub == 0) >> cbase) & gmask, S, L);
    const unsigned long long okm = spec_slot_bits((__ballot(ok && c.sub == 0) >> cbase) & gmask, S, L);
    const unsigned long long path =
        spec_slot_bits((__ballot(spec_on_path(tb, slot, accm, act) && c.sub == 0) >> cbase) & gmask, S, L);
    const SpecRound rd = spec_path_round(path, accm, okm);
    const int wl = cbase + (rd.win >= 0 ? rd.win : 0) * L;  // the new state's slot, first lane
    T vf[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) vf[j] = __shfl(v[j], wl, 64);
    const T phf = __shfl(phv, wl, 64);
    if (s.sum_u || s.sample_every > 0) {  // uniform per chain (only lane r == 0 keeps the clock)
      // the states after each settled step, in step order: the path again, the
      // proposals read from the LDS park, written by lane r == 0
      const bool sums = s.sum_u && r == 0;
      RoundSums<3> rsum(sums ? s.sum_u + chain * 3 : nullptr, (sums && s.sum_u2) ? s.sum_u2 + chain * 3 : nullptr,
                        sums ? 3 : 0);
#pragma unroll
      for (int j = 0; j < 3; ++j) vpk[j][threadIdx.x] = v[j];
      wave_sync_lds();
      const int t0 = (threadIdx.x & ~63) + cbase;  // the chain's first thread in the block
      spec_path_replay(
          path, accm,
          [&](int q, int la) {
            T vq[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) vq[j] = vpk[j][t0 + (la >= 0 ? la : 0) * L];
            if (r == 0) {
              if (sums) {
#pragma unroll
                for (int j = 0; j < 3; ++j) rsum.add(j, la >= 0 ? (double)vq[j] : (double)ur[j]);
              }
              if (s.sample_every > 0 && clk.next == st + q) {
                const int64_t sl = clk.take(clk.next);
                T* so = (T*)s.sample_out + chain * s.sample_stride + sl * s.sample_step_stride;
#pragma unroll
                for (int j = 0; j < 3; ++j) so[j] = la >= 0 ? vq[j] : ur[j];
              }
            }
          });
      if (sums) rsum.store();
      wave_sync_lds();  // the park is rewritten next round
    }
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

template <typename T, int J, bool FM, int SPL, bool PHI>
__global__ __launch_bounds__(kTsBlock) void l96ts_eval_kernel(const ipmc_model m, int64_t n, const T* __restrict__ uin,
                                                              const T* __restrict__ y, const T* __restrict__ ginv,
                                                              T* __restrict__ out) {
  TsCtx c;
  int64_t chain = ts_chain(m.dim / SPL, c);
  c.K = m.dim;
  if (chain < 0 || chain >= n) return;
  const T v[3] = {uin[chain * 3], uin[chain * 3 + 1], uin[chain * 3 + 2]};
  const T ph = ts_phi<T, J, FM, SPL>(m, v, c, c.sub, PHI ? y : nullptr, ginv, PHI ? nullptr : out + chain * m.q);
  if (PHI && c.sub == 0) out[chain] = ph;
}

// blocks for n chains of G lanes each, ⌊64/G⌋ chains per wave
static int64_t ts_blocks(int G, int64_t n) {
  const int64_t cpw = 64 / G;
  const int64_t waves = (n + cpw - 1) / cpw;
  return (waves * 64 + kTsBlock - 1) / kTsBlock;
}

#define IPMC_TS_J(X) X(1) X(2) X(4) X(8) X(10) X(16)

// Slow variables per lane: 2 when K is even, a chain would otherwise fill a
// wave alone (K > 32: K=36 packs 3 chains = 54 lanes instead of 1 = 36) and the
// doubled state still fits (J <= 10); for K = 6 with J <= 4 (the thesis
// problem) kTs6Spl: 3 = pairs of lanes, all 64 lanes live, halos by one DPP
// swap (6 lanes per chain leave 4 idle lanes per wave and ds_bpermute halos);
// 1 otherwise.  lanes_per_chain = K, K/2 (K even, J <= 10) or, for K = 6 and
// J <= 4, 2 or 1 selects it explicitly.  -1: unsupported request.
#ifndef IPMC_TS6_SPL  // layout experiments (tools/)
#define IPMC_TS6_SPL 3
#endif
static int ts_spl(const ipmc_model& m, const ipmc_sweep* s) {
  const int K = m.dim, J = m.fast_per_slow;
  const bool two_ok = (K % 2 == 0) && J <= 10;
  const bool six_ok = (K == 6) && J <= 4;
  if (s && s->lanes_per_chain > 0) {
    if (s->lanes_per_chain == K) return 1;
    if (two_ok && s->lanes_per_chain == K / 2) return 2;
    if (six_ok && s->lanes_per_chain == 2) return 3;
    if (six_ok && s->lanes_per_chain == 1) return 6;
    return -1;
  }
  // K = 6 pairs of lanes for ensembles that fill the GPU by themselves (>= 32 768
  // chains = one wave per SIMD of pairs) or one-step launches; a smaller
  // ensemble's multi-step launch speculates, and its rounds are latency chains:
  // 6 lanes per chain (5 values per lane instead of 15) and up to 10 slots --
  // the reference's K=6 J=4 study with 1 024 chains ran 1.46x slower on pairs
  // (profiles/r3/example_lorenz_thesis.json vs profiles/r2).
  if (six_ok && (!s || s->n_steps <= 1 || s->n_chains >= 32768)) return IPMC_TS6_SPL;
  return (two_ok && K > 32) ? 2 : 1;
}

// Speculation width: spec_width if given (S·L <= 64), else, for multi-step
// launches, the widest that keeps the ensemble within one wave per SIMD.
static int ts_spec(const ipmc_sweep& s, int L) {
  const int smax = 64 / L;
  if (s.spec_width > 0) return s.spec_width <= smax ? s.spec_width : -1;
  if (s.n_steps <= 1) return 1;
  const int64_t fit = 65536 / (s.n_chains * (int64_t)L);
  return (int)(fit < 1 ? 1 : (fit > smax ? smax : fit));
}

template <typename T, bool FM, int SPL>
static int ts_sweep_t(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  const int L = m.dim / SPL;
  const int S = ts_spec(s, L);
  if (S < 1) {
    set_error("two-scale Lorenz-96: spec_width * lanes per chain (%d) must be <= 64", L);
    return IPMC_ERR_UNSUPPORTED;
  }
  const int64_t blocks = ts_blocks(L * S, s.n_chains);
  switch (m.fast_per_slow) {
#define IPMC_J(J)                                                                                                  \
  case J:                                                                                                          \
    if constexpr (ts_compiled<SPL, J>()) {                                     \
      hipLaunchKernelGGL((l96ts_sweep_kernel<T, J, FM, SPL>), dim3((unsigned)blocks), dim3(kTsBlock), 0, st, m, s, \
                         S);                                                                                       \
      return check_launch("l96ts_sweep_kernel");                                                                   \
    }                                                                                                              \
    break;
    IPMC_TS_J(IPMC_J)
#undef IPMC_J
  }
  set_error("two-scale Lorenz-96: no kernel compiled for J=%d (1, 2, 4, 8, 10, 16)", m.fast_per_slow);
  return IPMC_ERR_UNSUPPORTED;
}

template <typename T, bool FM, int SPL>
static int ts_eval_t(const ipmc_model& m, int64_t n, const void* u, const void* y, const void* ginv, void* out,
                     bool phi, hipStream_t st) {
  const int64_t blocks = ts_blocks(m.dim / SPL, n);
  switch (m.fast_per_slow) {
#define IPMC_J(J)                                                                                                 \
  case J:                                                                                                         \
    if constexpr (ts_compiled<SPL, J>()) {                                    \
      if (phi)                                                                                                    \
        hipLaunchKernelGGL((l96ts_eval_kernel<T, J, FM, SPL, true>), dim3((unsigned)blocks), dim3(kTsBlock), 0,   \
                           st, m, n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);                          \
      else                                                                                                        \
        hipLaunchKernelGGL((l96ts_eval_kernel<T, J, FM, SPL, false>), dim3((unsigned)blocks), dim3(kTsBlock), 0,  \
                           st, m, n, (const T*)u, (const T*)y, (const T*)ginv, (T*)out);                          \
      return check_launch("l96ts_eval_kernel");                                                                   \
    }                                                                                                             \
    break;
    IPMC_TS_J(IPMC_J)
#undef IPMC_J
  }
  set_error("two-scale Lorenz-96: no kernel compiled for J=%d (1, 2, 4, 8, 10, 16)", m.fast_per_slow);
  return IPMC_ERR_UNSUPPORTED;
}

int l96ts_sweep(const ipmc_model& m, const ipmc_sweep& s, hipStream_t st) {
  if (m.dim > 64) {
    set_error("two-scale Lorenz-96: K <= 64");
    return IPMC_ERR_UNSUPPORTED;
  }
  const int spl = ts_spl(m, &s);
  if (spl < 0) {
    set_error("two-scale Lorenz-96: lanes_per_chain must be K, (K even, J <= 10) K/2 or (K = 6, J <= 4) 2 or 1");
    return IPMC_ERR_UNSUPPORTED;
  }
  const bool fm = m.arith == IPMC_ARITH_FMA;
#define IPMC_TS_SPL_SWEEP(P)                                                                                       \
  if (spl == P) {                                                                                                  \
    if (s.dtype == IPMC_F64) return fm ? ts_sweep_t<double, true, P>(m, s, st) : ts_sweep_t<double, false, P>(m, s, st); \
    return fm ? ts_sweep_t<float, true, P>(m, s, st) : ts_sweep_t<float, false, P>(m, s, st);                       \
  }
  IPMC_TS_SPL_SWEEP(2)
  IPMC_TS_SPL_SWEEP(3)
  IPMC_TS_SPL_SWEEP(6)
#undef IPMC_TS_SPL_SWEEP
  if (s.dtype == IPMC_F64) return fm ? ts_sweep_t<double, true, 1>(m, s, st) : ts_sweep_t<double, false, 1>(m, s, st);
  return fm ? ts_sweep_t<float, true, 1>(m, s, st) : ts_sweep_t<float, false, 1>(m, s, st);
}

int l96ts_plan(const ipmc_model& m, const ipmc_sweep& s, int& lanes, int& spec) {
  if (m.dim > 64) {
    set_error("two-scale Lorenz-96: K <= 64");
    return IPMC_ERR_UNSUPPORTED;
  }
  const int spl = ts_spl(m, &s);
  if (spl < 0) {
    set_error("two-scale Lorenz-96: lanes_per_chain must be K, (K even, J <= 10) K/2 or (K = 6, J <= 4) 2 or 1");
    return IPMC_ERR_UNSUPPORTED;
  }
  lanes = m.dim / spl;
  spec = ts_spec(s, lanes);
  if (spec < 1) {
    set_error("two-scale Lorenz-96: spec_width * lanes per chain (%d) must be <= 64", lanes);
    return IPMC_ERR_UNSUPPORTED;
  }
  return IPMC_OK;
}

int l96ts_eval(const ipmc_model& m, int32_t dtype, int64_t n, const void* u, const void* y, const void* ginv,
               void* out, bool phi, hipStream_t st) {
  if (m.dim > 64) {
    set_error("two-scale Lorenz-96: K <= 64");
    return IPMC_ERR_UNSUPPORTED;
  }
  const bool fm = m.arith == IPMC_ARITH_FMA;
  const int spl = ts_spl(m, nullptr);
#define IPMC_TS_SPL_EVAL(P)                                                                                        \
  if (spl == P) {                                                                                                  \
    if (dtype == IPMC_F64)                                                                                         \
      return fm ? ts_eval_t<double, true, P>(m, n, u, y, ginv, out, phi, st)                                       \
                : ts_eval_t<double, false, P>(m, n, u, y, ginv, out, phi, st);                                     \
    return fm ? ts_eval_t<float, true, P>(m, n, u, y, ginv, out, phi, st)                                          \
              : ts_eval_t<float, false, P>(m, n, u, y, ginv, out, phi, st);                                        \
  }
  IPMC_TS_SPL_EVAL(2)
  IPMC_TS_SPL_EVAL(3)
  IPMC_TS_SPL_EVAL(6)
#undef IPMC_TS_SPL_EVAL
  if (dtype == IPMC_F64)
    return fm ? ts_eval_t<double, true, 1>(m, n, u, y, ginv, out, phi, st)
              : ts_eval_t<double, false, 1>(m, n, u, y, ginv, out, phi, st);
  return fm ? ts_eval_t<float, true, 1>(m, n, u, y, ginv, out, phi, st)
            : ts_eval_t<float, false, 1>(m, n, u, y, ginv, out, phi, st);
}

}  // namespace ipmc
