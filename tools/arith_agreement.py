"""FMA vs REFERENCE arithmetic at the headline shape (65 536 chains, Lorenz-96
d=40, 2 000 RK4 steps, f64): how far the benched FMA forward map moves the
chains from the reference's operation order (lorenz.py:77-81, unfused).

  python tools/arith_agreement.py [n_steps] [beta ...]  -> JSON lines

Per beta, three runs of MCMCSampler on the bench problem (y = G(u_true) +
N(0, 0.1²), u_true = 0.5 sin(2πk/40)):
  FMA seed A, REFERENCE seed A (paired: same u_0, same draws) and REFERENCE
  seed B (independent draws).
Paired: the fraction of chains whose accept counts are identical and whose
final states are bit-identical.  Independent: the posterior-mean estimate
(mean over chains of each chain's time average) of FMA-A against REF-B per
component, z_i = |m_F - m_R| / sqrt(se_F² + se_R²), se = between-chain sd / sqrt(C)
-- a test that can fail, as the two runs share no draws.
tests/test_gpu_arith_agreement.py asserts the stated tolerances on the same
quantities; profiles/r3/arith_agreement.jsonl records a full run.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

D, N_RK, DT, GAMMA = 40, 2000, 0.005, 0.1


def problem(arith):
    from ip_mcmc_amd import Lorenz96Operator

    op = Lorenz96Operator(D, 8.0, dt=DT, n_steps=N_RK, arith=arith)
    k = np.arange(D)
    u_true = 0.5 * np.sin(2 * np.pi * k / D)
    return op, u_true


def run(arith, seed, beta, u0, n_steps, y, x0):
    from ip_mcmc_amd import (ConstSteppCNProposer, CountedAccepter, EvolutionPotential, GaussianDistribution,
                             Lorenz96Operator, MCMCSampler, PhiloxRNG, pCNAccepter)

    op = Lorenz96Operator(D, 8.0, x0=x0, dt=DT, n_steps=N_RK, arith=arith)
    acc = CountedAccepter(pCNAccepter(EvolutionPotential(op, y, GaussianDistribution(np.zeros(D),
                                                                                      GAMMA**2 * np.eye(D)))))
    s = MCMCSampler(ConstSteppCNProposer(beta, GaussianDistribution(np.zeros(D), np.eye(D))), acc, PhiloxRNG(seed))
    mom = s.run(u0, n_samples=n_steps, burn_in=1, sample_interval=1, keep="moments")
    return {"mean": mom["sum_u"] / mom["n"], "accepts": np.asarray(acc.accepts).copy(), "u": s.state.u.copy()}


def compare(fa, ra, rb, n_steps):
    C = fa["mean"].shape[0]
    same_acc = float(np.mean(fa["accepts"] == ra["accepts"]))
    same_u = float(np.mean(np.all(fa["u"] == ra["u"], axis=1)))
    mF, mR = fa["mean"].mean(axis=0), rb["mean"].mean(axis=0)
    seF = fa["mean"].std(axis=0, ddof=1) / np.sqrt(C)
    seR = rb["mean"].std(axis=0, ddof=1) / np.sqrt(C)
    z = np.abs(mF - mR) / np.sqrt(seF**2 + seR**2)
    zp = np.abs(mF - ra["mean"].mean(axis=0)) / np.sqrt(seF**2 + seR**2)
    return {"chains": C, "pcn_steps": n_steps,
            "accept_rate_fma": float(fa["accepts"].sum()) / (C * n_steps),
            "accept_rate_ref": float(ra["accepts"].sum()) / (C * n_steps),
            "paired_identical_accept_counts": same_acc, "paired_identical_final_state": same_u,
            "paired_max_accept_count_diff": int(np.max(np.abs(fa["accepts"] - ra["accepts"]))),
            "indep_max_z": float(z.max()), "indep_mean_z2": float(np.mean(z**2)),
            "paired_max_z": float(zp.max())}


def measure(beta, n_steps, chains=65536, start="posterior"):
    op, u_true = problem("fma")
    y = op(u_true) + GAMMA * np.random.default_rng(3).normal(size=D)
    if start == "posterior":  # near the truth: the chains accept at a rate that exercises the decisions
        u0 = u_true[None, :] + 0.01 * np.random.default_rng(5).normal(size=(chains, D))
    else:  # the bench's start (u = 0)
        u0 = np.zeros((chains, D))
    t0 = time.perf_counter()
    fa = run("fma", 11, beta, u0, n_steps, y, op.x0)
    ra = run("reference", 11, beta, u0, n_steps, y, op.x0)
    rb = run("reference", 12, beta, u0, n_steps, y, op.x0)
    res = compare(fa, ra, rb, n_steps)
    res.update({"beta": beta, "start": start, "wall_s": time.perf_counter() - t0})
    return res


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    betas = [float(b) for b in sys.argv[2:]] or [0.2, 0.05, 0.02]
    print(json.dumps(measure(0.2, n, start="zero")), flush=True)
    for b in betas:
        print(json.dumps(measure(b, n)), flush=True)
