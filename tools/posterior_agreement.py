"""Stationary posterior comparisons behind the stated floating-point tolerances.

  python tools/posterior_agreement.py arith  [chains] [segments] [seg_len] [beta] [r] [nopair]
  python tools/posterior_agreement.py prec   [chains] [segments] [seg_len] [beta] [r] [nopair]
  -> one JSON line per comparison

Two pairs of samplers are compared on the same posterior:
  * ``arith``: the benched FMA forward map against REFERENCE arith (no FMA,
    lorenz.py:77-81's operation order, the mode pinned bit for bit to the
    reference fixtures) at the headline shape: Lorenz-96 d=40, 2 000 RK4 steps,
    f64 (BASELINE config 3);
  * ``prec``: fp32 against fp64 at config 5's shape: d=256, 10 000 RK4 steps.

The posterior.  The forcing-field problem of bench.py (F = 8 + u, u_true =
0.5 sin(2πk/d), prior N(0, I), y = G(u_true) + η) with the reference's own
noise recipe (lorenz_mcmc.py:100-112: Γ = r²·diag(var of the observed
quantity along the truth's trajectory)): γ = r·sd(X_k).  The time-averaged
observation of a chaotic run moves by σ_ε ≈ 0.5 (d=40, T=10) / 0.3 (d=256,
T=50) under any perturbation a pCN step makes (`chaos`), so each proposal's
misfit carries a noise of sd ≈ sqrt(d)·σ_ε/γ: with bench.py's γ = 0.1 that is
~50 units (the chains freeze where they land: 0.2 % accepted, falling), at the
reference's r = 0.5 (γ ≈ 1.8) ~2 (8-9 % accepted, the chains stick: split-R̂
2.1 after 2 400 steps at d=40, profiles/r4/posterior_explore_r05.jsonl), at
r = 2 (γ ≈ 7.3) ~0.5: a noisy-likelihood chain that mixes.

The run.  Independent u_0 for each sampler, drawn from the prior (over-
dispersed against the posterior) with independent seeds, and independent
Philox seeds: nothing is shared, so the comparison can fail.  Each sampler
runs ``segments`` blocks of ``seg_len`` pCN steps through MCMCSampler.run
(keep="moments", resumed from its own checkpoint between blocks): the
per-chain block means B[c, j, i] are the batch means.

The statistics (all per parameter component i):
  * burn-in: diagnostics.burn_in_lengths (the reference's len_burn_in,
    burgers/utilities.py:134-167, on the device) over the ensemble's
    block-mean trace of the forcing F = 8 + u (its relative-change test needs
    a mean away from 0 and, flagging a change in ANY of the d variables, a
    trace with the noise averaged down); that many blocks, and at least the
    first quarter of the run, are discarded from every chain (a trace without
    a sustained change returns len - 1 in the reference's heuristic,
    utilities.py:160-165: nothing to discard);
  * MCSE by batch means over the post-burn-in blocks, batches merged until
    their lag-1 autocorrelation is below 0.1; the across-chain standard error
    (sd over chains of the per-chain means / sqrt(C)) is reported beside it
    and the larger of the two is used;
  * stationarity of the ensemble over the post-burn-in run: the chains'
    first-half and second-half means have the same mean (per-chain difference
    z) and the same spread (paired z of the squared deviations) -- exact for
    independent chains whatever their autocorrelation; split-R̂ over the batch
    means is reported beside them (it also asks each chain to have explored
    the posterior: a stationary chain a few autocorrelation times long reads
    R̂² ≈ 1 + (τ − 1)/h);
  * agreement: z_i = (m_A,i − m_B,i) / sqrt(se_A,i² + se_B,i²); max |z_i|,
    mean z_i², and the whitened statistic T²/d = Δᵀ(S_A/C + S_B/C)⁻¹Δ / d
    with S the between-chain covariance of the per-chain means (a chi-square
    with d degrees of freedom over d for independent estimates, whatever the
    correlation between components);
  * paired (same u_0, same draws, only the arithmetic differs): the fraction
    of chains with identical accept counts.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DT = 0.005
R_NOISE = 2.0  # the noise level r of lorenz_mcmc.py:111-112 (the reference used 0.5 for its 5K moments)


def truth_sd(d, F, n_spin=2000, n_traj=20000, dt=DT):
    """Pooled sd of the instantaneous X_k along the truth's trajectory (host RK4)."""
    from ip_mcmc_amd import Lorenz96Operator as L

    x = L.spinup(d, F, dt=dt, n_steps=n_spin)
    xs = np.empty((n_traj // 10, d))
    for t in range(n_traj):
        k1 = L.rhs(x, F)
        k2 = L.rhs(x + 0.5 * dt * k1, F)
        k3 = L.rhs(x + 0.5 * dt * k2, F)
        k4 = L.rhs(x + dt * k3, F)
        x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        if t % 10 == 9:
            xs[t // 10] = x
    return float(xs.std())


def problem(d, n_rk, r=R_NOISE):
    """(y, gamma, u_true, x0) of the forcing-field posterior at (d, n_rk)."""
    from ip_mcmc_amd import Lorenz96Operator

    k = np.arange(d)
    u_true = 0.5 * np.sin(2 * np.pi * k / d)
    op = Lorenz96Operator(d, 8.0, dt=DT, n_steps=n_rk)
    gamma = r * truth_sd(d, 8.0 + u_true)
    y = op(u_true) + gamma * np.random.default_rng(3).normal(size=d)
    return y, gamma, u_true, op.x0


def blocks(d, n_rk, y, gamma, x0, arith, dtype, seed, u0, n_seg, seg_len):
    """Per-chain block means (C, n_seg, d) f64, accept counts (C,) and the
    sampler's wall seconds."""
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             Lorenz96Operator, MCMCSampler, PhiloxRNG, pCNAccepter)

    op = Lorenz96Operator(d, 8.0, x0=x0, dt=DT, n_steps=n_rk, arith=arith)
    acc = CountedAccepter(pCNAccepter(EvolutionPotential(op, y, GaussianDistribution(np.zeros(d),
                                                                                      gamma**2 * np.eye(d)))))
    s = MCMCSampler(ConstSteppCNProposer(BETA[0], GaussianDistribution(np.zeros(d), np.eye(d))), acc,
                    PhiloxRNG(seed), dtype=dtype)
    C = u0.shape[0]
    B = np.empty((C, n_seg, d))
    state = u0
    wall = 0.0
    for j in range(n_seg):
        t0 = time.perf_counter()
        mom = s.run(state, n_samples=1, burn_in=0, sample_interval=seg_len, keep="moments")
        wall += time.perf_counter() - t0
        B[:, j] = mom["sum_u"] / mom["n"]
        state = s.checkpoint()
        print(f"[posterior_agreement] {arith} {np.dtype(dtype).name} block {j + 1}/{n_seg} "
              f"({wall:.1f} s)", file=sys.stderr, flush=True)  # progress: long runs stay visibly alive
    return B, np.asarray(state.accepts, dtype=np.int64), wall


BETA = [0.2]


def burn_in_blocks(B, window, theta0=8.0):
    """diagnostics.burn_in_lengths on the ensemble's block-mean trace of the
    forcing theta = theta0 + u (lorenz_mcmc.py:64's theta = prior_mean + u):
    the average over the chains of each block mean, one series of d
    variables.  The reference heuristic (utilities.py:134-167) flags a
    moving-average change |d avg / mean| > 3 % of the variable's own mean in
    ANY variable and ends the burn-in at the last run of avg_window + 1 such
    changes: on one chain's trace of 40 (or 256) noisy components some
    component changes by 3 % almost every block, and on the perturbation u
    (mean ~0) every one does -- the ensemble mean (noise / sqrt(C)) of theta is
    the trace it can read."""
    from ip_mcmc_amd.diagnostics import burn_in_lengths

    trace = np.ascontiguousarray((B + theta0).mean(axis=0)[None])  # (1, n, d)
    return burn_in_lengths(trace, avg_window=window, layout="time_vars")


def _batches(P):
    """Batch means of P (C, n, d): consecutive blocks merged until the batch
    means' lag-1 autocorrelation is below 0.1 (or 8 batches are left).
    Returns (Q (C, nb, d), batch size in blocks, that lag-1 autocorrelation)."""
    C, n, d = P.shape
    bs = 1
    while True:
        nb = n // bs
        Q = P[:, :nb * bs].reshape(C, nb, bs, d).mean(axis=2)
        if nb < 4:
            return Q, bs, None
        c = Q - Q.mean(axis=1, keepdims=True)
        r1 = np.sum(c[:, 1:] * c[:, :-1], axis=(0, 1)) / np.maximum(np.sum(c * c, axis=(0, 1)), 1e-300)
        if np.max(r1) < 0.1 or nb < 16:
            return Q, bs, float(np.max(r1))
        bs *= 2


def _split_rhat(Q):
    """Split-R̂ per component over the batch means Q (C, nb, d): each chain's
    batches cut in two halves; on (nearly) uncorrelated batches, so the
    within-chain autocorrelation does not inflate it (on raw autocorrelated
    blocks a stationary chain reads R̂² ≈ 1 + (τ − 1)/h)."""
    h = Q.shape[1] // 2
    S = np.concatenate([Q[:, :h], Q[:, h:2 * h]], axis=0)  # (2C, h, d)
    W = S.var(axis=1, ddof=1).mean(axis=0)
    Bv = h * S.mean(axis=1).var(axis=0, ddof=1)
    return np.sqrt(((h - 1) / h * W + Bv / h) / W)


def summarize(B, burn):
    """Estimator, MCSE and stationarity statistics of one sampler's blocks."""
    C, n, d = B.shape
    P = B[:, burn:]
    m_chain = P.mean(axis=1)  # (C, d)
    m = m_chain.mean(axis=0)
    se_chain = m_chain.std(axis=0, ddof=1) / np.sqrt(C)
    Q, bs, r1 = _batches(P)
    se_bm = Q.reshape(-1, d).std(axis=0, ddof=1) / np.sqrt(Q.shape[0] * Q.shape[1])
    se = np.maximum(se_chain, se_bm)
    rhat = _split_rhat(Q)
    # the ensemble is stationary over the post-burn-in run: the chains' first-
    # half and second-half means have the same mean (per-chain difference z)
    # and the same spread (paired z of the squared deviations) -- both exact
    # for independent chains whatever their autocorrelation, unlike R̂, which
    # also asks every chain to have explored the posterior (split-R̂ is
    # reported; a stationary chain as short as a few autocorrelation times
    # reads above 1)
    h = P.shape[1] // 2
    m1, m2 = P[:, :h].mean(axis=1), P[:, h:2 * h].mean(axis=1)
    dif = m1 - m2
    zh = np.abs(dif.mean(axis=0)) / (dif.std(axis=0, ddof=1) / np.sqrt(C))
    mu = 0.5 * (m1.mean(axis=0) + m2.mean(axis=0))
    dv = (m1 - mu) ** 2 - (m2 - mu) ** 2
    zv = np.abs(dv.mean(axis=0)) / (dv.std(axis=0, ddof=1) / np.sqrt(C))
    return {"m": m, "se": se, "se_chain": se_chain, "se_bm": se_bm, "batch_blocks": bs, "batch_r1": r1,
            "rhat_max": float(rhat.max()), "half_z_max": float(zh.max()), "half_var_z_max": float(zv.max()),
            "m_chain": m_chain}


def compare(sa, sb):
    d = sa["m"].shape[0]
    delta = sa["m"] - sb["m"]
    z = np.abs(delta) / np.sqrt(sa["se"]**2 + sb["se"]**2)
    C = sa["m_chain"].shape[0]
    S = np.cov(sa["m_chain"], rowvar=False) / C + np.cov(sb["m_chain"], rowvar=False) / sb["m_chain"].shape[0]
    S = np.atleast_2d(S)
    t2 = float(delta @ np.linalg.solve(S, delta))
    return {"max_z": float(z.max()), "mean_z2": float(np.mean(z**2)), "t2_over_d": t2 / d,
            "se_ratio_bm_over_chain": float(np.median(sa["se_bm"] / sa["se_chain"]))}


def record(rec, name):
    """Append `rec` to $IPMC_RECORD_DIR/name when the variable is set (GPU
    sessions keep the tests' measurements beside their log)."""
    d = os.environ.get("IPMC_RECORD_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name), "a") as f:
            f.write(json.dumps(rec) + "\n")


def measure(kind, chains, n_seg, seg_len, beta=0.2, r=R_NOISE, window=None, paired=True):
    """One comparison; returns the JSON record."""
    BETA[0] = beta
    if kind == "arith":
        d, n_rk = 40, 2000
        runs = (("fma", np.float64, 11, 5), ("reference", np.float64, 12, 6))
    elif kind == "prec":
        d, n_rk = 256, 10000
        runs = (("fma", np.float64, 11, 5), ("fma", np.float32, 12, 6))
    elif kind == "prec40":  # fp32 vs fp64 at the headline shape (the reference's noise level: tests/)
        d, n_rk = 40, 2000
        runs = (("fma", np.float64, 11, 5), ("fma", np.float32, 12, 6))
    else:
        raise ValueError(kind)
    t0 = time.perf_counter()
    y, gamma, u_true, x0 = problem(d, n_rk, r)
    window = window or max(5, n_seg // 10)
    out = {"kind": kind, "d": d, "rk4_steps": n_rk, "chains": chains, "segments": n_seg, "seg_len": seg_len,
           "pcn_steps": n_seg * seg_len, "beta": beta, "noise_r": r, "gamma": gamma, "burn_in_window": window}
    res = []
    for arith, dt, seed, u0_seed in runs:
        u0 = np.random.default_rng(u0_seed).normal(size=(chains, d))  # prior draws
        B, acc, wall = blocks(d, n_rk, y, gamma, x0, arith, dt, seed, u0, n_seg, seg_len)
        res.append((B, acc, wall, u0))
    # the reference heuristic returns len - 1 when a trace never shows
    # avg_window + 1 consecutive significant changes (utilities.py:160-165):
    # nothing to discard.  At least the first quarter is discarded anyway.
    bi = [np.where(b >= n_seg - 1, 0, b) for b in (burn_in_blocks(B, window) for B, *_ in res)]
    out["burn_in_heuristic_blocks"] = [int(b.max()) for b in bi]
    burn = max(int(max(b.max() for b in bi)), n_seg // 4)
    if burn > n_seg // 2:
        out["burn_in_capped_from"] = burn
        burn = n_seg // 2
    out["burn_in_blocks"] = burn
    out["burn_in_steps"] = burn * seg_len
    sums = [summarize(B, burn) for B, *_ in res]
    names = [f"{a}_{np.dtype(t).name}" for a, t, *_ in runs]
    for nm, sm, (B, acc, wall, _) in zip(names, sums, res):
        out[nm] = {"accept_rate": float(acc.sum()) / (chains * n_seg * seg_len), "rhat_max": sm["rhat_max"],
                   "half_z_max": sm["half_z_max"], "half_var_z_max": sm["half_var_z_max"],
                   "batch_blocks": sm["batch_blocks"], "batch_r1": sm["batch_r1"],
                   "mcse_median": float(np.median(sm["se"])), "post_mean_range": [float(sm["m"].min()),
                                                                                  float(sm["m"].max())],
                   "wall_s": wall}
    out.update(compare(*sums))
    out["u_true_rms_dev"] = float(np.sqrt(np.mean((sums[0]["m"] - u_true)**2)))
    if paired:
        arith, dt, seed, u0_seed = runs[1]
        Bp, accp, _ = blocks(d, n_rk, y, gamma, x0, arith, dt, runs[0][2], res[0][3], n_seg, seg_len)
        out["paired_identical_accept_counts"] = float(np.mean(accp == res[0][1]))
        out["paired_identical_block_means"] = float(np.mean(np.all(Bp == res[0][0], axis=(1, 2))))
    out["wall_s"] = time.perf_counter() - t0
    return out


def chaos(d, n_rk, n=32, hs=(1e-7, 1e-5, 1e-3, 1e-1)):
    """sd over n nearby u of the time-averaged observation (the misfit noise a
    pCN proposal of size h meets), on the device."""
    import torch

    from ip_mcmc_amd import Lorenz96Operator

    op = Lorenz96Operator(d, 8.0, dt=DT, n_steps=n_rk)
    rng = np.random.default_rng(0)
    u = rng.normal(size=(1, d))
    rec = {"d": d, "rk4_steps": n_rk}
    for h in hs:
        U = np.repeat(u, n, axis=0) + h * rng.normal(size=(n, d))
        g = op.forward_device(torch.as_tensor(U, device="cuda"), torch.float64).cpu().numpy()
        rec[f"sigma_eps_h{h:g}"] = float(g.std(axis=0, ddof=1).mean())
    return rec


if __name__ == "__main__":
    kind = sys.argv[1] if len(sys.argv) > 1 else "arith"
    if kind == "chaos":
        for d, n in ((40, 2000), (256, 10000)):
            print(json.dumps(chaos(d, n)), flush=True)
        sys.exit(0)
    a = sys.argv[2:]
    chains = int(a[0]) if len(a) > 0 else (8192 if kind == "arith" else 16384)
    n_seg = int(a[1]) if len(a) > 1 else 60
    seg_len = int(a[2]) if len(a) > 2 else 50
    beta = float(a[3]) if len(a) > 3 else 0.2
    r = float(a[4]) if len(a) > 4 else R_NOISE
    paired = not (len(a) > 5 and a[5] == "nopair")
    print(json.dumps(measure(kind, chains, n_seg, seg_len, beta, r, paired=paired)), flush=True)
