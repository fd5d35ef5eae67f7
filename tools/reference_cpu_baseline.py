"""Time the REFERENCE as-is on the headline workload (SURVEY §8(d) CPU baseline (i)).

Runs only in the build container (needs /root/reference): the reference's
MCMCSampler + ConstSteppCNProposer + pCNAccepter + EvolutionPotential +
GaussianDistribution, with G = classical RK4 (dt 0.005, 2000 steps, time
average) over the reference's own Lorenz96 RHS object (lorenz.py:13-111, J=0,
d=40) -- the reference has no RK4 driver, so this is the smallest wrapper that
makes its code run config 3.  One chain per process, P processes; stdout of
the sampler suppressed; --steps 60 keeps every process busy for > 30 s (1.7
pCN steps/s per core).  Writes profiles/r4/reference_cpu_cfg3.json, which
bench.py reports next to its own cpu_baseline (clearly labelled: measured
here, not on the GPU box).

  python tools/reference_cpu_baseline.py [--procs P] [--steps S]
  python tools/reference_cpu_baseline.py --config 1 [--samples N]

--config 1 times the reference's own config-1 script composition instead
(stuart_examples.py:58-109, example 2.1: the closure G, pCNProposer(0.25),
CountedAccepter(pCNAccepter), scalar noise, default burn-in 1 000 and interval
200, one chain) -> profiles/r3/reference_cpu_cfg1.json, beside
examples/stuart_reference.py's run of the same composition through
ip_mcmc_amd's host step.
"""
import argparse
import contextlib
import io
import json
import multiprocessing as mp
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _setup():
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "ip_mcmc"))
    sys.path.insert(0, os.path.join(REF, "report", "scripts"))
    import matplotlib

    matplotlib.use("Agg")
    import ip_mcmc

    ip_mcmc.pCNProposer = ip_mcmc.ConstSteppCNProposer  # stale name in lorenz.py:8
    import lorenz

    return ip_mcmc, lorenz


def worker(args):
    seed, steps = args
    import numpy as np

    ip_mcmc, lorenz = _setup()
    D, N, DT, BETA, GAMMA = 40, 2000, 0.005, 0.2, 0.1

    def G_of(F):
        f = lorenz.Lorenz96(D, 0, F, 0.0, 0.0, 0.0)
        return lambda x: f(0.0, x)

    def rk4_avg(F, x0):
        f = G_of(F)
        x = np.array(x0)
        ob = np.zeros(D)
        h2, h6 = DT * 0.5, DT / 6.0
        for _ in range(N):
            k1 = f(x)
            k2 = f(x + h2 * k1)
            k3 = f(x + h2 * k2)
            k4 = f(x + DT * k3)
            x = x + h6 * (((k1 + 2.0 * k2) + 2.0 * k3) + k4)
            ob = ob + x
        return ob / N

    x0 = np.full(D, 8.0)
    x0[0] += 0.01
    k = np.arange(D)
    y = rk4_avg(8.0 + 0.5 * np.sin(2 * np.pi * k / D), x0) + GAMMA * np.random.default_rng(3).normal(size=D)
    noise = ip_mcmc.GaussianDistribution(np.zeros(D), GAMMA**2 * np.eye(D))
    prior = ip_mcmc.GaussianDistribution(np.zeros(D), np.eye(D))
    pot = ip_mcmc.EvolutionPotential(lambda u: rk4_avg(8.0 + u, x0), y, noise)
    sampler = ip_mcmc.MCMCSampler(ip_mcmc.ConstSteppCNProposer(BETA, prior), ip_mcmc.pCNAccepter(pot),
                                  np.random.default_rng(seed))
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        sampler.run(np.zeros(D), n_samples=steps, burn_in=0, sample_interval=1)
    return time.perf_counter() - t0


def config1(n_samples):
    import numpy as np

    ip_mcmc, _ = _setup()
    g = np.array([int(x) for x in str(np.pi) if x != "."])[:1]
    u = np.array([int(x) for x in str(np.e) if x != "."])[:1]

    def G(u):
        return np.dot(g, u)

    prior = ip_mcmc.GaussianDistribution(mean=np.zeros_like(u), covariance=np.identity(1))
    noise = ip_mcmc.GaussianDistribution(mean=0, covariance=0.5**2)
    rng = np.random.default_rng(1)
    data = G(u) + noise.sample(rng)
    acc = ip_mcmc.CountedAccepter(ip_mcmc.pCNAccepter(potential=ip_mcmc.EvolutionPotential(G, data, noise)))
    sampler = ip_mcmc.MCMCSampler(ip_mcmc.pCNProposer(beta=0.25, prior=prior), acc, rng)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        samples = sampler.run(u_0=np.zeros_like(u), n_samples=n_samples)
    el = time.perf_counter() - t0
    steps = 800 + n_samples * 200
    rec = {"value": steps / el, "unit": "pCN steps/s", "cores": 1, "kind": "reference",
           "sample": f"stuart_examples.py example 2.1 as composed there, one chain, n_samples={n_samples} "
                     f"({steps} pCN steps), reference MCMCSampler on numpy/scipy",
           "accept_ratio": float(acc.ratio()), "sample_mean": float(samples.mean()), "wall_s": el,
           "host": platform.processor() or platform.machine(),
           "measured_on": "build container (the reference does not exist on the GPU box)"}
    out = os.path.join(REPO, "profiles", "r3", "reference_cpu_cfg1.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--samples", type=int, default=500)
    args = ap.parse_args()
    if args.config == 1:
        config1(args.samples)
        return
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(args.procs) as pool:
        times = pool.map(worker, [(i, args.steps) for i in range(args.procs)])
    wall = time.perf_counter() - t0
    per_proc = [args.steps / t for t in times]
    rec = {
        "value": float(sum(per_proc)),
        "unit": "pCN steps/s",
        "cores": args.procs,
        "kind": "reference",
        "per_core": float(sum(per_proc) / args.procs),
        "sample": f"{args.procs} processes x 1 chain x {args.steps} pCN steps of config 3 (d=40, 2000 RK4 "
                  f"steps, f64) through the reference MCMCSampler/pCNAccepter/EvolutionPotential with the "
                  f"reference Lorenz96 RHS; 2 G evaluations per step (Φ(u) recomputed, accepter.py:122); "
                  f"{min(times):.1f}-{max(times):.1f} s of sampling per process",
        "seconds_per_process": [float(t) for t in times],
        "host": platform.processor() or platform.machine(),
        "measured_on": "build container (the reference does not exist on the GPU box)",
        "wall_s": wall,
    }
    out = os.path.join(REPO, "profiles", "r4", "reference_cpu_cfg3.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
