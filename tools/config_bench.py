"""Throughput of the BASELINE configs other than the headline (one GPU).

  python tools/config_bench.py [cfg2 cfg4 cfg4full cfg5 ...]

cfg2     Lorenz-63, 500 RK4 steps, 4 096 chains; SURVEY §8(d): prior N(0, diag(1, 1, 0.1)),
         y = the long-run moment means of the truth, Γ = r²·diag(var of the instantaneous moments),
         r = 0.5 (lorenz_mcmc.py:106-112's construction)
cfg4     Burgers N=256, fixed dt 1e-3 x 1000, 2 048 chains (= 16 384 / 8 GPUs)
cfg4full Burgers as cfg4 with all 16 384 chains on one GPU
cfg4cfl  Burgers N=256, reference CFL time stepping, 2 048 chains
cfg4visc Burgers N=256 with viscosity nu = 1e-3 (central differences), fixed dt 1e-3 x 1000, 2 048 chains
cfg5     Lorenz-96 d=256, 10 000 RK4 steps, 131 072 chains (= 2^20 / 8 GPUs)
l96xN    the headline problem with N chains (N = 1, 64, 1024: speculative sweeps; 8192..65536: the
         per-GPU share of a strong-scaled 65 536-chain run)
ts6      two-scale Lorenz-96 K=6 J=4 (the thesis problem, lorenz_mcmc.py:87-88), T=20 (4 000 RK4 steps), 65 536 chains
ts36     two-scale Lorenz-96 K=36 J=10, 2 000 RK4 steps of 0.002, 16 384 chains
"""
import ctypes as C
import json
import re
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ip_mcmc_amd import (BurgersOperator, Lorenz63Operator, Lorenz96Operator, TwoScaleLorenz96Operator,  # noqa: E402
                         _abi)
from ip_mcmc_amd._lib import call, lib  # noqa: E402


def l63_truth_moments(theta=(10.0, 28.0, 8.0 / 3.0), dt=0.01, spinup=1000, n=50000):
    """Mean and variance over a long truth trajectory (T = n·dt after the
    spin-up) of the instantaneous moments (x, y, z, x², y², z²): the data and
    the noise scale of config 2, built as lorenz_mcmc.py:100-112 builds its own
    (moment_function over a long simulation, np.mean / np.var along time)."""
    s, r, b = theta
    x = Lorenz63Operator.spinup(theta, dt=dt, n_steps=spinup)
    f = lambda x: np.array([s * (x[1] - x[0]), x[0] * (r - x[2]) - x[1], x[0] * x[1] - b * x[2]])
    traj = np.empty((n, 3))
    for t in range(n):
        k1 = f(x)
        k2 = f(x + 0.5 * dt * k1)
        k3 = f(x + 0.5 * dt * k2)
        k4 = f(x + dt * k3)
        x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        traj[t] = x
    mom = np.concatenate([traj, traj**2], axis=1)
    return mom.mean(axis=0), mom.var(axis=0)


CFG2_R = 0.5  # noise level r (lorenz_mcmc.py:92)


def cfg2_problem():
    """(operator, y, 1/γ, prior sqrt-diagonal, beta) of config 2."""
    x0 = Lorenz63Operator.spinup(n_steps=1000)
    op = Lorenz63Operator(x0=x0, dt=0.01, n_steps=500)
    mean, var = l63_truth_moments()
    return op, mean, 1.0 / (CFG2_R * np.sqrt(var)), np.array([1.0, 1.0, np.sqrt(0.1)]), 0.2


def make(cfg):
    if cfg == "cfg2":
        op, y, ginv, sq, beta = cfg2_problem()
        return op, 4096, beta, sq, 80 * 500, (y, ginv)
    if cfg == "cfg2g1":  # round 1-2's config 2 (gamma = 1 for every moment, y = G(0) + N(0, 1))
        x0 = Lorenz63Operator.spinup(n_steps=1000)
        op = Lorenz63Operator(x0=x0, dt=0.01, n_steps=500)
        return op, 4096, 0.2, np.array([1.0, 1.0, np.sqrt(0.1)]), 80 * 500, 1.0
    if cfg in ("cfg4", "cfg4full", "cfg4cfl", "cfg4visc"):
        if cfg == "cfg4cfl":
            op = BurgersOperator(N=256, dt_mode="cfl")
        elif cfg == "cfg4visc":  # BASELINE's "viscous Burgers": central-difference diffusion, nu = 1e-3
            op = BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=1000, nu=1e-3)
        else:
            op = BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=1000)
        n = 16384 if cfg == "cfg4full" else 2048
        return op, n, 0.15, np.full(3, 0.25), 30 * 256 * 1000, 0.05
    mt = re.fullmatch(r"cfg4n(\d+)", cfg)
    if mt:  # config 4's share with another number of fixed time steps (per-pCN-step overhead fits)
        nst = int(mt.group(1))
        op = BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=nst)
        return op, 2048, 0.15, np.full(3, 0.25), 30 * 256 * nst, 0.05
    if cfg == "cfg5":
        op = Lorenz96Operator(256, 8.0, dt=0.005, n_steps=10000)
        return op, 131072, 0.2, np.ones(256), 30 * 256 * 10000, 0.1
    if cfg == "ts6":
        op = TwoScaleLorenz96Operator(K=6, J=4, dt=0.005, n_steps=4000)
        return op, 65536, 0.5, np.sqrt([10.0, 1.0, 10.0]), 45 * 30 * 4000, 0.5
    if cfg == "ts36":
        op = TwoScaleLorenz96Operator(K=36, J=10, dt=0.002, n_steps=2000, moments="mean")
        return op, 16384, 0.5, np.sqrt([10.0, 1.0, 10.0]), 45 * 396 * 2000, 0.5
    if cfg.startswith("l96"):
        # the headline problem with few chains (the reference runs one): speculation
        # territory; "l96d80x16384": another dimension; "l96mx64": the mixing
        # posterior of tools/posterior_agreement.py (gamma = 0.5 sd(X) = 1.8,
        # the reference's noise recipe) instead of gamma = 0.1, whose chains
        # accept almost nothing -- the best case for a speculative sweep
        mt = re.fullmatch(r"l96(m?)(?:d(\d+))?x(\d+)", cfg)
        d = int(mt.group(2) or 40)
        op = Lorenz96Operator(d, 8.0, dt=0.005, n_steps=2000)
        return op, int(mt.group(3)), 0.2, np.ones(d), 30 * d * 2000, (1.8 if mt.group(1) else 0.1)
    raise SystemExit(f"unknown config {cfg}")


def run(cfg, dtype, steps=10, lanes=0, per_launch=1, spec=None, warmup=3, cpl=0):
    dev = torch.device("cuda", 0)
    op, n, beta, sq, flop, gamma = make(cfg)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64)).to(dtype).to(dev).contiguous()
    m, _ = op.model(dtype, dev)
    u = torch.zeros((n, op.k), dtype=dtype, device=dev)
    if isinstance(gamma, tuple):  # (y, 1/γ) given by the config
        y, gi = t(gamma[0]), t(gamma[1])
    else:
        g0 = op.forward_device(u[:1].clone())[0].double().cpu().numpy()
        y = t(np.nan_to_num(g0) + gamma * np.random.default_rng(1).normal(size=op.q))
        gi = t(np.full(op.q, 1 / gamma))
    sqt = t(sq)
    phi = torch.empty(n, dtype=dtype, device=dev)
    adt = _abi.F64 if dtype == torch.float64 else _abi.F32
    st = torch.cuda.current_stream(dev).cuda_stream
    call("ipmc_potential", C.byref(m), adt, n, u.data_ptr(), y.data_ptr(), gi.data_ptr(), phi.data_ptr(), st)
    acc = torch.zeros(n, dtype=torch.int64, device=dev)
    s = _abi.IpmcSweep()
    s.dtype, s.n_chains = adt, n
    if isinstance(op, (Lorenz63Operator,)):
        s.spec_width = lanes  # small models: the ":" option is the speculation width
    else:
        s.lanes_per_chain = lanes
    if spec is not None:
        s.spec_width = spec
    s.chains_per_lane = cpl
    s.u, s.phi, s.accepts = u.data_ptr(), phi.data_ptr(), acc.data_ptr()
    s.y, s.gamma_inv, s.prior_sqrt = y.data_ptr(), gi.data_ptr(), sqt.data_ptr()
    s.beta, s.contraction = beta, float(np.sqrt(1 - beta**2))
    s.seed, s.n_steps = 5, per_launch
    # warm-up: the clocks ramp over the first ~0.1 s of load, so a fixed
    # number of short launches left the first config of a run ~7 % slow
    t_w = time.perf_counter()
    nw = 0
    while nw < warmup or time.perf_counter() - t_w < 0.25:
        call("ipmc_pcn_sweep", C.byref(m), C.byref(s), st)
        s.step0 += per_launch
        nw += 1
        if nw % 8 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record()
        call("ipmc_pcn_sweep", C.byref(m), C.byref(s), st)
        b.record()
        s.step0 += per_launch
    torch.cuda.synchronize(dev)
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) / per_launch
    res = {
        "config": cfg,
        "dtype": str(dtype).split(".")[-1],
        "chains": n,
        "ms_per_sweep": ms,
        "pcn_steps_per_s": n / (ms * 1e-3),
        "tflops_algorithmic": n * flop / (ms * 1e-3) / 1e12,
        "accept_rate": float(acc.sum().item()) / (n * (steps + nw) * per_launch),
    }
    if per_launch > 1:
        res["steps_per_launch"] = per_launch
    if lanes:
        res["lanes_forced"] = lanes
    if spec is not None:
        res["spec_width"] = spec
    # the kernel plan this sweep ran (ipmc_plan_sweep: the launch's own code path)
    p = _abi.IpmcPlan()
    call("ipmc_plan_sweep", C.byref(m), C.byref(s), C.byref(p))
    res["plan"] = {"lanes_per_chain": p.lanes_per_chain, "chains_per_lane": p.chains_per_lane,
                   "spec_width": p.spec_width}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    cfgs = sys.argv[1:] or ["cfg2", "cfg4", "cfg4full", "cfg4cfl", "cfg5"]
    # "cfg4:64" forces 64 lanes per chain (small models: speculation width), "cfg2@128" runs
    # 128 pCN steps per launch, "l96x1~1" sets spec_width 1 (no speculation), "^2" two
    # fp32 chains per lane group, "!f32" one dtype only
    for c in cfgs:
        name = re.match(r"[a-z0-9]+", c).group(0)
        opt = {k: int(v) for k, v in re.findall(r"([:@~^])(\d+)", c)}
        dts = [torch.float64, torch.float32]
        if "!f32" in c:
            dts = [torch.float32]
        elif "!f64" in c:
            dts = [torch.float64]
        for dt in dts:
            if opt.get("^") and dt != torch.float32:
                continue
            run(name, dt, lanes=opt.get(":", 0), per_launch=opt.get("@", 1), spec=opt.get("~"), cpl=opt.get("^", 0))
