"""Headline benchmark: pCN steps/s on Lorenz-96 d=40, 2000 RK4 steps, 65 536 chains.

  python bench.py [--gpus N --steps K --warmup W] [--workload cfg3|cfg4|cfg5]
  (N > 1: started once, it launches torch.distributed.run with N ranks itself;
   under an external torch.distributed.run WORLD_SIZE must equal N)

A "step" is one pCN step of every chain of the ensemble: propose, run the
forward map (cfg3: 2000 RK4 steps of Lorenz-96, d=40), evaluate Φ, accept or
reject.  value is SURVEY §8(d)'s timed region with the data in HBM: the
drop-in ``MCMCSampler.run`` end to end, through the sharded entry point
``shard.run_sharded`` -- u_0 already on the device, Φ(u_0), exactly K pCN
steps of every chain in the fused libipmc kernels, the per-chain sums and
states left in HBM (results='device'; Φ and the accept counts come back),
the block-sum posterior mean and the final gather over the ranks (RCCL at
N > 1) -- bracketed by barrier + synchronize, max over ranks.  The same run
handing over host buffers (H2D of u_0, D2H of states and sums) is
extra.run_e2e_pcie, the PCIe-inclusive rate.
value = all chains of all ranks x K / that time.  The chains are independent
units, sharded over the ranks with no collective on the data path (global
chain ids, so every chain is the one-GPU run's bit for bit).  BASELINE's
metric is 65 536 chains over the whole node, so cfg3 splits them over the N
GPUs (strong scaling, the default: 8 192 chains per GPU at N = 8), and at
N > 1 "extra.weak_scaling" carries 65 536 chains on every GPU under its own
metric string.  Configs 4 and 5 state their ensembles per node too, so
--workload cfg4 / cfg5 split them the same way.  Every rank holds only its
own block of u_0 (run_sharded(n_total=...)).

extra.kernel_*: the same sweep kernel on device-resident state (raw
ipmc_pcn_sweep launches, one pCN step per launch for a full GPU, HIP events
on the launch stream) -- the number the roofline is computed on.

roofline: VALU-bound (no MFMA, no HBM traffic inside the RK loop). achieved =
algorithmic FLOP per launch / average kernel time of the kernel leg's timed
launches; algorithmic FLOP per pCN step per chain = 30·d·n (SURVEY §8(d)
counting rule).
cpu_baseline: the C oracle (same arithmetic, bit-exact), a bounded sample of
the same workload on this host's cores, rank 0 at N=1 only; the reference
itself, timed in the build container by tools/reference_cpu_baseline.py, is
attached as cpu_baseline.reference_recorded.

--workload cfg4 / cfg5 times BASELINE's configs 4 (viscous Burgers N=256,
1 000 FD steps, 16 384 chains over the node) and 5 (Lorenz-96 d=256, 10 000
RK4 steps, 2^20 chains over the node, fp32 beside fp64) the same way; the
default cfg3 line carries short end-to-end runs of both in extra.configs.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from ip_mcmc_amd import BurgersOperator, Lorenz96Operator, _abi  # noqa: E402
from ip_mcmc_amd._lib import call  # noqa: E402

ITEM = {"f64": 8, "f32": 4}
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}  # MI355X vector (spec), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
METRIC_CHAINS = 65536  # cfg3's metric ensemble: 65 536 chains over the node (BASELINE.json "metric")
METRIC = "pCN steps/sec (whole node), Lorenz-96 d=40 T=2000, 65 536 chains"
WORKLOAD_CHAINS = {"cfg3": METRIC_CHAINS, "cfg4": 16384, "cfg5": 1 << 20}  # per node, as BASELINE states them


def ensemble(workload, world, chains=None, scaling=None):
    """(scaling, total chains over the node) of a bench run.  Every BASELINE
    workload states its ensemble per node (cfg3's metric: 65 536 chains over
    the whole node), so the default is strong scaling: the node's ensemble
    split over the N GPUs (8 192 chains per GPU at N = 8).  --scaling weak
    runs --chains (default: the workload's ensemble) on EVERY GPU; cfg3's line
    carries that figure beside value (extra.weak_scaling)."""
    scaling = scaling or "strong"
    per = int(chains or WORKLOAD_CHAINS[workload])
    return scaling, per * (world if scaling == "weak" else 1)


def metric_name(workload, prob_name, total_chains):
    """The line's metric: BASELINE's own string exactly when the run is its
    configuration (cfg3 with 65 536 chains over the node), else the same form
    naming the chains actually run, so a line never quotes one ensemble's
    name for another's throughput."""
    grouped = f"{total_chains:,}".replace(",", " ")
    if workload == "cfg3":
        return METRIC if total_chains == METRIC_CHAINS else \
            f"pCN steps/sec (whole node), Lorenz-96 d=40 T=2000, {grouped} chains"
    return f"pCN steps/sec (whole node), {prob_name}, {total_chains} chains"


class Problem:
    """One BASELINE workload: forward map, data, noise, prior and pCN step."""

    def __init__(self, key, name, op, y, gamma, prior_sqrt, beta, chains, flop, mix_ceiling, steps, warmup, data):
        self.key, self.name, self.op, self.y = key, name, op, np.asarray(y, dtype=np.float64)
        self.gamma = np.broadcast_to(np.asarray(gamma, dtype=np.float64), self.y.shape).copy()
        self.sq = np.asarray(prior_sqrt, dtype=np.float64)
        self.beta, self.chains, self.flop = beta, chains, flop
        self.mix_ceiling, self.steps, self.warmup, self.data = mix_ceiling, steps, warmup, data
        self.k = op.k

    def reference_arith(self):
        """The same problem with the forward map in REFERENCE arith (no FMA, the
        reference's operation order: lorenz.py:77-81, rusanov.py:62-96)."""
        import copy

        p = copy.copy(self)
        p.op = copy.copy(self.op)
        p.op.arith, p.op._cache = "reference", {}
        return p


def make_problem(key):
    """cfg3 (the headline), cfg4, cfg5 of BASELINE.json / SURVEY §8(d)."""
    if key == "cfg3":
        d, n = 40, 2000
        op = Lorenz96Operator(d, forcing_mean=8.0, dt=0.005, n_steps=n)  # x0: 1000-step spin-up from 8 + 0.01 e0
        k = np.arange(d)
        y = op(0.5 * np.sin(2 * np.pi * k / d)) + 0.1 * np.random.default_rng(3).normal(size=d)
        # 30 algorithmic FLOP per component and RK4 step in 20 VALU ops (10 of
        # them FMA): at most 30 / (2 x 20) of the all-FMA peak
        return Problem(key, "lorenz96_d40_rk4_2000_pcn", op, y, 0.1, np.ones(d), 0.2, 65536, 30 * d * n, 30 / 40,
                       200, 10, "synthetic (forcing-field inverse problem, F = 8 + u, y = G(0.5 sin(2 pi k/40)) + "
                       "N(0, 0.1^2), seed 3; prior N(0, I); u_0 = 0)")
    if key == "cfg4":
        # burgers_beta.py:25-87 at N=256 (SURVEY §8(d) cfg 4), viscous (nu = 1e-3), fixed dt 1e-3 x 1 000
        op = BurgersOperator(N=256, dt_mode="fixed", dt=1e-3, n_steps=1000, nu=1e-3)
        y = op(np.array([0.025, -0.025, -0.02])) + 0.05 * np.random.default_rng(3).normal(size=5)
        return Problem(key, "burgers_n256_fd1000_viscous_pcn", op, y, 0.05, np.full(3, 0.25), 0.15, 16384,
                       30 * 256 * 1000, None, 100, 5, "synthetic (Riemann-IC inverse problem, theta = [1.5, 0.25, "
                       "-0.5] + u, y = G([0.025, -0.025, -0.02]) + N(0, 0.05^2), seed 3; prior N(0, 0.25^2 I))")
    if key == "cfg5":
        d, n = 256, 10000
        op = Lorenz96Operator(d, forcing_mean=8.0, dt=0.005, n_steps=n)
        k = np.arange(d)
        y = op(0.5 * np.sin(2 * np.pi * k / d)) + 0.1 * np.random.default_rng(3).normal(size=d)
        return Problem(key, "lorenz96_d256_rk4_10000_pcn", op, y, 0.1, np.ones(d), 0.2, 1 << 20, 30 * d * n, 30 / 40,
                       4, 1, "synthetic (forcing-field inverse problem, d=256, y = G(0.5 sin(2 pi k/256)) + "
                       "N(0, 0.1^2), seed 3; prior N(0, I); u_0 = 0)")
    if key == "cfg3_mixing":
        # the headline's shape and kernel on a posterior the chains sample: the
        # reference's noise recipe (lorenz_mcmc.py:100-112, gamma = r sd(X_k))
        # at r = 2, tools/posterior_agreement.py:91-100
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import posterior_agreement as PA

        d, n = 40, 2000
        y, gamma, _, x0 = PA.problem(d, n, 2.0)
        op = Lorenz96Operator(d, forcing_mean=8.0, x0=x0, dt=0.005, n_steps=n)
        return Problem(key, "lorenz96_d40_rk4_2000_pcn_mixing", op, y, gamma, np.ones(d), 0.2, 65536, 30 * d * n,
                       30 / 40, 200, 10, f"synthetic (forcing-field problem, gamma = 2 sd(X_k) = {gamma:.3f}; "
                                         "prior N(0, I); u_0 = 0)")
    raise SystemExit(f"unknown workload {key}")


CFG5_PARITY_NOTE = ("no floor: 10 000 RK4 steps = 50 time units run far past Lorenz-96's predictability horizon "
                    "(rounding differences grow ~e^(1.7 t)), so G in any two arithmetics are unrelated and paired "
                    "streams part at the first steps; bit-exact streams at config 5 are REFERENCE arith's (GPU == "
                    "oracle, tests/test_gpu_paired_streams.py; its rate: extra.configs.cfg5.reference_f64), the "
                    "precision claim the stationary fp32/fp64 tolerance (tests/test_gpu_tolerance.py)")


def _hist(x, edges):
    c, _ = np.histogram(x, bins=edges)
    return {"edges": [int(e) for e in edges], "counts": [int(v) for v in c]}


def paired_streams(prob, chains, steps, dtype, dev):
    """The accept/reject index streams of the benched FMA forward map against
    REFERENCE arith (the reference's operation order, pinned bit for bit to the
    reference fixtures: lorenz.py:77-81, rusanov.py:62-96), on `prob` itself:
    the same seed, u_0 = 0 and global chain ids, so both arms draw the same
    proposals and uniforms (accepter.py:59-62,121-122's rule on the same
    numbers); only G's rounding differs.  One pCN step per launch; after each
    the accept counters give every chain's decision.  A chain whose decisions
    agree at every step has the same states bit for bit in both arms (the
    proposal never reads G), which is checked.  Returns the record."""
    arms = [Workload(p, chains, 0, dtype, dev) for p in (prob, prob.reference_arith())]
    dec = []
    for w in arms:
        D = torch.empty((steps, chains), dtype=torch.int8, device=dev)
        prev = w.acc.clone()
        for t in range(steps):
            w.step(1)
            D[t] = (w.acc - prev).to(torch.int8)
            prev.copy_(w.acc)
        dec.append(D)
    torch.cuda.synchronize(dev)
    diff = dec[0] != dec[1]
    div = diff.any(dim=0)
    first = torch.argmax(diff.to(torch.int8), dim=0)[div].cpu().numpy()
    same = ~div
    ident = float(same.float().mean().item())
    state_eq = bool(torch.equal(arms[0].u[same], arms[1].u[same]))
    phf, phr = arms[0].phi[same].double(), arms[1].phi[same].double()
    rel = float(((phf - phr).abs() / phr.abs().clamp_min(1e-300)).max().item()) if phf.numel() else None
    edges = [e for e in sorted({0, 1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, steps}) if e <= steps]
    return {"workload": prob.name, "chains": chains, "steps": steps, "dtype": "f64" if dtype == torch.float64 else
            "f32", "identical_accept_stream_frac": ident, "diverged_chains": int(div.sum().item()),
            "first_divergence_step_hist": _hist(first, edges),
            "accept_rate_fma": float(dec[0].float().mean().item()),
            "accept_rate_reference": float(dec[1].float().mean().item()),
            "identical_chains_states_bit_equal": state_eq, "identical_chains_phi_max_rel_diff": rel,
            "how": "same seed, u_0 = 0 and chain ids in both arms; one pCN step per launch; decisions from the accept "
                   "counters; FMA arith (benched) vs REFERENCE arith (the reference's operation order)"}


# ------------------------------------------------------------ kernel leg
class Workload:
    """Device-resident chains swept by raw ipmc_pcn_sweep launches (the kernel leg)."""

    def __init__(self, prob, n_chains, chain_offset, dtype, dev, lanes=0, chains_per_lane=0, per_launch=1,
                 spec_width=0):
        self.dev, self.dtype = dev, dtype
        self.n_chains, self.per_launch = n_chains, per_launch
        self.model, self._keep = prob.op.model(dtype, dev)
        t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64)).to(dtype).to(dev).contiguous()
        self.y, self.ginv, self.sq = t(prob.y), t(1.0 / prob.gamma), t(prob.sq)
        self.u = torch.zeros((n_chains, prob.k), dtype=dtype, device=dev)
        self.phi = torch.empty(n_chains, dtype=dtype, device=dev)
        self.acc = torch.zeros(n_chains, dtype=torch.int64, device=dev)
        self.stream = torch.cuda.current_stream(dev).cuda_stream
        adt = _abi.F64 if dtype == torch.float64 else _abi.F32
        call("ipmc_potential", C.byref(self.model), adt, n_chains, self.u.data_ptr(), self.y.data_ptr(),
             self.ginv.data_ptr(), self.phi.data_ptr(), self.stream)
        s = _abi.IpmcSweep()
        s.dtype, s.lanes_per_chain, s.chains_per_lane, s.spec_width = adt, lanes, chains_per_lane, spec_width
        s.n_chains, s.chain_offset = n_chains, chain_offset
        s.u, s.phi, s.accepts = self.u.data_ptr(), self.phi.data_ptr(), self.acc.data_ptr()
        s.y, s.gamma_inv, s.prior_sqrt = self.y.data_ptr(), self.ginv.data_ptr(), self.sq.data_ptr()
        s.beta, s.contraction = prob.beta, float(np.sqrt(1 - prob.beta**2))
        s.seed, s.step0, s.n_steps = 2, 0, per_launch
        self.s = s
        # the plan the sweep runs (ipmc_plan_sweep: same code path as the launch)
        self.lanes, self.chains_per_lane, self.spec_width = sweep_plan(self.model, s)

    def settle_clocks(self, seconds):
        """Untimed G evaluations of the chains' current u (ipmc_potential into a
        scratch Φ: the chain state is untouched) for `seconds` of wall time, so
        that a short timed region does not start on idle clocks (they ramp over
        ~0.1-0.3 s of load: 65 536 chains ran 18.9 M steps/s at K = 20 after 5
        warm-up steps, 20.4 M at K = 200; profiles/r3/bench_65536_k20.jsonl)."""
        if seconds <= 0:
            return
        scratch = torch.empty_like(self.phi)
        t0 = time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < seconds:
            call("ipmc_potential", C.byref(self.model), self.s.dtype, self.n_chains, self.u.data_ptr(),
                 self.y.data_ptr(), self.ginv.data_ptr(), scratch.data_ptr(), self.stream)
            i += 1
            if i % 4 == 0:
                torch.cuda.synchronize(self.dev)
        torch.cuda.synchronize(self.dev)

    def launches(self, n_steps):
        """Launch sizes covering exactly n_steps pCN steps."""
        full, rem = divmod(n_steps, self.per_launch)
        return [self.per_launch] * full + ([rem] if rem else [])

    def step(self, n=1):
        """One launch of n pCN steps for every chain."""
        self.s.n_steps = n
        call("ipmc_pcn_sweep", C.byref(self.model), C.byref(self.s), self.stream)
        self.s.step0 += n


def sweep_plan(model, sweep):
    """(lanes per chain, chains per lane group, speculation width) of the kernel
    ipmc_pcn_sweep runs for this model and sweep."""
    p = _abi.IpmcPlan()
    call("ipmc_plan_sweep", C.byref(model), C.byref(sweep), C.byref(p))
    return p.lanes_per_chain, p.chains_per_lane, p.spec_width


def pmc_record(dtype, chains, lanes, d=40, n_rk=2000):
    """The committed rocprofv3 PMC passes of this sweep kernel (same dtype,
    chains, shape and lanes-per-chain layout): profiles/r*/pmc_l96_<dtype>.json,
    newest round first -- HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE,
    corrected as MI355X_MICROARCH.md's HBM section prescribes), clock and VALU
    issue rate -- with its path, or (None, None)."""
    import glob

    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"pmc_l96_{dtype}.json")), reverse=True):
        rec = json.load(open(path))
        names = " ".join(rec.get("kernel", []))
        if (rec.get("chains") == chains and rec.get("d") == d and rec.get("rk4_steps") == n_rk
                and f"{d}, {lanes}, true" in names):
            return rec, os.path.relpath(path, REPO)
    return None, None


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def barrier(world):
    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(x, world, dev):
    """The max of x over the ranks of the process group (RCCL on the device
    with backend "nccl"); x itself without one."""
    if dist.is_initialized():
        t = torch.tensor([x], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        x = float(t.item())
    return x


def timed(w, steps, warmup, world, settle_s=0.0):
    """Exactly `steps` pCN steps of every chain (after `warmup` untimed ones,
    and settle_s seconds of untimed G evaluations that leave the chains as
    they are), bracketed by barrier + synchronize; (max-rank wall seconds, mean
    kernel ms per full launch of w.per_launch steps, from HIP events on the
    launch stream)."""
    w.settle_clocks(settle_s)
    for n in w.launches(warmup):
        w.step(n)
    torch.cuda.synchronize(w.dev)
    barrier(world)
    torch.cuda.synchronize(w.dev)
    sizes = w.launches(steps)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in sizes]
    t0 = time.perf_counter()
    for (a, b), n in zip(ev, sizes):
        a.record()
        w.step(n)
        b.record()
    torch.cuda.synchronize(w.dev)
    barrier(world)
    torch.cuda.synchronize(w.dev)
    el = time.perf_counter() - t0
    full = [a.elapsed_time(b) for (a, b), n in zip(ev, sizes) if n == w.per_launch] or \
           [a.elapsed_time(b) * w.per_launch / n for (a, b), n in zip(ev, sizes)]
    kern_ms = float(np.mean(full))
    return max_over_ranks(el, world, w.dev), kern_ms


# --------------------------------------------------------- end-to-end leg
def sampler_factory(prob, dtype_np, dev, seed=2):
    """make(chain_offset) -> the drop-in sampler of `prob` (the reference's
    composition: ConstSteppCNProposer + pCNAccepter(EvolutionPotential))."""
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, MCMCSampler, PhiloxRNG,
                             pCNAccepter)

    prior = GaussianDistribution(np.zeros(prob.k), np.diag(prob.sq**2))
    noise = GaussianDistribution(np.zeros(prob.y.shape[0]), np.diag(prob.gamma**2))

    def make(chain_offset=0):
        pot = EvolutionPotential(prob.op, prob.y, noise)
        return MCMCSampler(ConstSteppCNProposer(prob.beta, prior), pCNAccepter(pot), PhiloxRNG(seed),
                           dtype=dtype_np, device=dev, chain_offset=chain_offset)

    return make


def timed_run(prob, dtype_np, dev, total_chains, steps, warmup, world, gather="all", seed=2, settle=None,
              resident=True):
    """SURVEY §8(d)'s timed region: shard.run_sharded(u_0, exactly `steps`
    pCN steps, keep='moments') bracketed by barrier + synchronize,
    after an untimed run of `warmup` steps of the same shape and `settle()`
    (the kernel leg's untimed G evaluations: the clocks drop within the ~10 ms
    the host takes between legs and ramp back over ~0.1-0.3 s, so the timed
    run of a K=20 line otherwise starts on them: 3.35 instead of 3.2 ms per
    step, profiles/r5/e2e_trace_summary.json).  resident (gather='mean'): u_0
    is a device tensor written before the timed region and the per-chain
    results stay in HBM (results='device'), so no PCIe transfer is timed -- the
    task's `value`; resident=False hands over host buffers both ways (the
    PCIe-inclusive rate, extra.run_e2e_pcie).  Returns the record and the
    gathered result."""
    from ip_mcmc_amd.shard import run_sharded

    from ip_mcmc_amd.shard import chain_range, world_info

    make = sampler_factory(prob, dtype_np, dev, seed)
    resident = resident and gather == "mean"
    kw = {"results": "device"} if resident else {}
    # only this rank's block of u_0 (run_sharded(n_total=...)): no rank holds the node's ensemble
    lo, hi = chain_range(total_chains, world_info()[0], world)
    if resident:  # in HBM before the timed region starts
        u0 = torch.zeros((hi - lo, prob.k), dtype=torch.float64, device=dev)
    else:
        u0 = np.full((hi - lo, prob.k), 0.0)  # written, i.e. resident (np.zeros maps its pages on first touch)
    kw["n_total"] = total_chains
    if warmup > 0:
        run_sharded(make, u0, n_samples=1, burn_in=0, sample_interval=warmup, keep="moments", gather=gather, **kw)
    if settle is not None:
        settle()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    res = run_sharded(make, u0, n_samples=1, burn_in=0, sample_interval=steps, keep="moments", gather=gather, **kw)
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    smp = res["sampler"]
    assert smp.last_path == "device" and smp.state.steps_this_run == steps
    tm = smp.last_run_timing
    rec = {"pcn_steps_per_s": total_chains * steps / el, "wall_s": el, "ms_per_step": el / steps * 1e3,
           "steps": steps, "total_chains": total_chains, "chains_per_gpu": hi - lo, "u0_rows_per_rank": hi - lo,
           "accept_rate": float(res["accepts"].sum()) / (total_chains * steps),
           "run_seconds_rank0": res["run_seconds"], "gather_ms": res["gather_seconds"] * 1e3,
           "setup_ms": tm["setup_s"] * 1e3, "phi0_gpu_ms": tm["phi0_gpu_ms"], "sweeps_gpu_ms": tm["sweeps_gpu_ms"],
           "tail_ms": tm["tail_ms"], "data_in_hbm": bool(resident)}
    return rec, res


def e2e_samples(prob, n_chains, chain_offset, dtype_np, dev, world, n_samples=20):
    """MCMCSampler.run with samples: host u_0 (n_chains x k) in, n_samples
    samples 1 step apart back on the host (page-locked, copied in blocks while
    later blocks sweep)."""
    make = sampler_factory(prob, dtype_np, dev)
    s = make(chain_offset)
    u0 = np.full((n_chains, prob.k), 0.0)
    # warm run of the same size: device allocations, and the page-locked result
    # block that torch's host allocator recycles once the caller drops it
    s.run(u0, n_samples=n_samples, burn_in=1, sample_interval=1)
    torch.cuda.synchronize(dev)
    barrier(world)
    t0 = time.perf_counter()
    out = s.run(u0, n_samples=n_samples, burn_in=1, sample_interval=1)
    el = time.perf_counter() - t0
    assert out.shape == (n_chains, n_samples, prob.k)
    barrier(world)
    el_max = max_over_ranks(el, world, dev)
    tm = s.last_run_timing
    return {"pcn_steps_per_s": world * n_chains * n_samples / el_max, "wall_s": el_max, "samples": n_samples,
            "sample_bytes_per_rank": int(out.nbytes), "setup_ms": tm["setup_s"] * 1e3,
            "sweeps_gpu_ms": tm["sweeps_gpu_ms"], "tail_ms_after_sweeps": tm["tail_ms"],
            "copy_overlapped": tm["copy_overlapped"],
            "note": "MCMCSampler.run(u0 host (chains x k), n_samples, burn_in=1, sample_interval=1): H2D of u0, "
                    "Phi(u0), the sweeps, D2H of the (chains, n_samples, k) f64 samples; tail = wall after set-up "
                    "not covered by the GPU sweeps (launch gaps + the last copy block + epilogue)"}


def config_line(key, dev, world, steps=None, warmup=None, chains=None):
    """A short end-to-end run of config 4 or 5 as BASELINE states it (the
    ensemble over the node): f64, and for config 5 f32 beside it with the
    posterior-mean difference of the two short runs in between-chain standard
    errors (a smoke of the fp32-vs-fp64 comparison; the stated tolerance is
    the stationary test, tests/test_gpu_tolerance.py)."""
    prob = make_problem(key)
    total = chains or prob.chains
    st, wu = steps or prob.steps, prob.warmup if warmup is None else warmup
    gather = "mean"
    rec64, r64 = timed_run(prob, np.float64, dev, total, st, wu, world, gather=gather)
    out = {"workload": prob.name, "f64": rec64, "flop_per_chain_step": prob.flop,
           "tflops_f64": total * prob.flop * st / rec64["wall_s"] / 1e12}
    if key == "cfg5":
        # REFERENCE arith: the arithmetic whose accept streams are the reference's at this length
        recr = timed_run(prob.reference_arith(), np.float64, dev, total, st, wu, world, gather=gather)[0]
        out["reference_f64"] = recr
        out["tflops_reference_f64"] = total * prob.flop * st / recr["wall_s"] / 1e12
        rec32, r32 = timed_run(prob, np.float32, dev, total, st, wu, world, gather=gather, seed=3)
        out["f32"] = rec32
        out["tflops_f32"] = total * prob.flop * st / rec32["wall_s"] / 1e12
        out["f32_over_f64"] = rec32["pcn_steps_per_s"] / rec64["pcn_steps_per_s"]
        out["posterior_mean_max_abs_diff_f32_f64"] = float(np.max(np.abs(r32["mean"] - r64["mean"])))
        tf_ref = out["tflops_reference_f64"]
        out["arith_parity"] = {
            "bit_exact_arith": "reference",
            "bit_exact_pcn_steps_per_s": recr["pcn_steps_per_s"],
            "fma_pcn_steps_per_s": rec64["pcn_steps_per_s"],
            "fma_paired_identical_accept_frac": None,  # filled from parity.cfg5 when the paired run is in the line
            "tflops_reference_f64": tf_ref,
            "reference_frac_of_peak": tf_ref / PEAK_TFLOPS["f64"],
            "reference_op_ceiling_frac": CFG5_REFERENCE_CEILING,
            "note": "at config 5 the bit-exact accept streams (GPU == oracle == the reference's operation order, "
                    "lorenz.py:77-81) are REFERENCE arith's: its rate is bit_exact_pcn_steps_per_s.  The FMA chains "
                    "(fma_pcn_steps_per_s, the faster rate) are not the reference's chains: 50 time units of chaos "
                    "part the paired streams at the first steps (fma_paired_identical_accept_frac); their claim is "
                    "the stated stationary tolerance.  REFERENCE arith issues 32 FP64 ops (no FMA) per component "
                    "and RK4 step plus 24 DPP moves per 16 components (the d=256 kernel's loop, hipcc -S): "
                    "30 FLOP / (2 x 33.5 slots) = 0.448 of the FP64 peak is its op-mix ceiling (at the ~2.15 GHz "
                    "the chip holds under this load, ~0.40).  reference_frac_of_peak is end to end over the "
                    "run's steps + Phi(u_0), which counts no FLOP of Phi(u_0): with 4 steps the kernel's own "
                    "fraction is 5/4 of it"}
    return out


# REFERENCE arith's op-mix ceiling at d=256 on 16 lanes: 30 FLOP per component
# and RK4 step in 32 unfused FP64 ops + 24 DPP moves / 16 components
CFG5_REFERENCE_CEILING = 30 / (2 * (32 + 24 / 16))


def cpu_baseline(prob, dtype_np, budget_s=15.0):
    """The C oracle on this host's cores: a bounded sample of the same
    workload (chains x 1 pCN step), scaled to pCN steps/s."""
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    ginv = 1.0 / prob.gamma
    phi0 = O.potential(prob.op, np.zeros((1, prob.k), dtype=dtype_np), prob.y, ginv, dtype_np)[0]

    def run(nc):
        U = np.zeros((nc, prob.k), dtype=dtype_np)  # every chain starts at u = 0, as on the GPU
        phi = np.full(nc, phi0, dtype=dtype_np)
        acc = np.zeros(nc, dtype=np.int64)
        t0 = time.perf_counter()
        O.pcn_sweep(prob.op, U, phi, prob.y, ginv, prob.sq, prob.beta, 2, 0, 1, accepts=acc, n_threads=threads)
        return time.perf_counter() - t0

    t1 = run(threads)  # one chain-step per thread, calibration
    per = t1 / threads  # wall seconds per chain-step with all threads busy
    n = int(max(threads, min(1_000_000, budget_s / max(per, 1e-9))))
    n = (n // threads) * threads
    el = run(n)
    return {"value": n / el, "unit": "pCN steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} chains x 1 pCN step of the {prob.name} workload "
                      f"({'f64' if dtype_np == np.float64 else 'f32'}), C oracle, {threads} threads, {el:.1f} s"}


def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: run N ranks under
    torch.distributed.run as a child process (nothing here has touched the GPU)
    and relay its exit code; its rank 0 prints the line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {n} ranks: {' '.join(cmd)}")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def auto_per_launch(chains_per_rank):
    """pCN steps per launch of the kernel leg: 1 when the rank's chains fill a
    wave per SIMD on their own (>= 16 384 chains, one launch per step), else
    512, so that the sweep speculates over the steps of a launch
    (ipmc_plan_sweep).  A launch lasts as long as its slowest chain, so short
    speculative launches lose to the chains that accept early: 8 192 chains
    run sequentially on 8 interleaved lanes below 256 steps per launch and
    speculate on 4 lanes x 2 slots from there (ipmc_plan_sweep): 14.4 / 16.6 /
    17.8 M steps/s on this problem at 20 / 200 / 1 024 timed steps, where round
    3's first rule (2 lanes x 8 slots) ran 5.9 / 15.6 / 18.9 M
    (profiles/r3/bench_8192_*.jsonl)."""
    return 1 if chains_per_rank >= 16384 else 512


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed pCN steps (default: the workload's, cfg3 200)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed pCN steps first (default: cfg3 10)")
    ap.add_argument("--workload", default="cfg3", choices=["cfg3", "cfg4", "cfg5"],
                    help="cfg3: the headline (Lorenz-96 d=40, 65 536 chains); cfg4: viscous Burgers N=256, 16 384 "
                         "chains; cfg5: Lorenz-96 d=256, 10 000 RK4 steps, 2^20 chains (f32 beside f64)")
    ap.add_argument("--chains", type=int, default=None,
                    help="total chains (strong, the default) or chains per GPU (weak); default: the workload's")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (the default for every workload: BASELINE states the ensembles per node, cfg3's "
                         "metric 65 536 chains over the whole node): --chains split over the GPUs; weak: --chains on "
                         "every GPU")
    ap.add_argument("--steps-per-launch", type=int, default=0,
                    help="pCN steps per kernel launch of the kernel leg (0 = auto)")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--spec-width", type=int, default=0, help="speculative slots per chain (0 = auto, 1 = off)")
    ap.add_argument("--settle", type=float, default=0.3,
                    help="seconds of untimed G evaluations before the warm-up steps (clock ramp; 0 = off)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the short cfg4 / cfg5 runs in extra.configs")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the paired FMA / REFERENCE accept-stream runs (parity.*; N = 1 only)")
    ap.add_argument("--pmc-file", default=None,
                    help="a tools/pmc_summarize.py record of this box's PMC passes for roofline.traffic (default: the "
                         "newest committed profiles/r*/pmc_l96_<dtype>.json of the same kernel and layout)")
    ap.add_argument("--kernel-only", action="store_true",
                    help="profiling runs: the kernel leg only (no end-to-end leg, extras or CPU baseline), so a "
                         "rocprofv3 trace or PMC pass holds the timed sweep launches and nothing else; the line's "
                         "value is then the kernel leg's rate (marked kernel_only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the product path) or gloo (rehearsal of the N-rank logic)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 (rehearsing N ranks on a one-GPU box; needs --dist-backend gloo)")
    args = ap.parse_args()

    if args.share_device and args.dist_backend != "gloo":
        raise SystemExit("--share-device needs --dist-backend gloo (RCCL wants one GPU per rank)")
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", 0 if args.share_device else local)
    torch.cuda.set_device(dev)
    # a process group for N > 1, and for one rank under a launcher
    # (torch.distributed.run sets MASTER_ADDR): then every collective of the
    # line -- barriers, the gathers, the max over ranks -- runs over RCCL even
    # on a one-GPU box (tests/test_gpu_bench_dist.py)
    grouped = world > 1 or (env_world is not None and "MASTER_ADDR" in os.environ)
    if grouped:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    log(f"rank {rank}/{world} on {dev}: building the {args.workload} problem")
    prob = make_problem(args.workload)
    steps = args.steps if args.steps is not None else prob.steps
    warmup = args.warmup if args.warmup is not None else prob.warmup
    args.scaling, total_chains = ensemble(args.workload, world, args.chains, args.scaling)
    from ip_mcmc_amd.shard import chain_range

    lo_rank, hi_rank = chain_range(total_chains, rank, world)  # this rank's global chain ids
    per_rank = hi_rank - lo_rank
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    ndt = np.float64 if args.dtype == "f64" else np.float32

    # 1. kernel leg: device-resident sweeps, HIP events (the roofline's kernel time)
    # (a launch never exceeds the timed steps: the plan reported is the one timed)
    per_launch = min(args.steps_per_launch or auto_per_launch(per_rank), max(1, steps))
    w = Workload(prob, per_rank, lo_rank, tdt, dev, args.lanes, per_launch=per_launch,
                 spec_width=args.spec_width)
    log(f"kernel leg: {steps} pCN steps ({args.dtype}, {per_rank} chains/GPU, {per_launch} steps/launch, "
        f"lanes={w.lanes}, spec_width={w.spec_width})")
    el_k, kern_ms = timed(w, steps, warmup, world, args.settle)
    kernel_rate = total_chains * steps / el_k
    log(f"kernel leg: {el_k:.3f} s, kernel {kern_ms:.3f} ms/launch, {kernel_rate / 1e6:.2f} M steps/s")
    lanes_k, cpl_k, spec_k = w.lanes, w.chains_per_lane, w.spec_width
    # the end-to-end legs settle the clocks on the kernel leg's chains (their
    # swept state, untouched: ipmc_potential into a scratch Φ)
    settle = lambda: w.settle_clocks(args.settle)  # noqa: E731
    if args.kernel_only:
        args.no_extra = args.no_configs = args.no_cpu = True

    # 2. value: MCMCSampler.run end to end through shard.run_sharded
    # the job's result on every rank: the posterior mean (fixed-order block
    # sums, bit-identical for any N) and every chain's Φ and accept
    # count; the per-chain states and sums stay on their rank
    gather_mode = "mean"
    if args.kernel_only:
        e2e = {"pcn_steps_per_s": kernel_rate, "wall_s": el_k, "ms_per_step": el_k / steps * 1e3,
               "accept_rate": None, "gather_ms": 0.0, "kernel_only": True}
        res = {"phi": np.zeros(0), "mean": np.zeros(0), "accepts": np.zeros(0)}
    else:
        log(f"end-to-end leg: run_sharded({total_chains} chains, {steps} steps, keep='moments', gather={gather_mode})")
        e2e, res = timed_run(prob, ndt, dev, total_chains, steps, warmup, world, gather=gather_mode, settle=settle)
    value = e2e["pcn_steps_per_s"]
    log(f"end-to-end: {e2e['wall_s']:.3f} s, {value / 1e6:.2f} M steps/s")
    e2e_pcie = None
    if not args.kernel_only:
        # the same run handing over host buffers (u_0 in, states and sums out):
        # the PCIe-inclusive rate, never value
        e2e_pcie = timed_run(prob, ndt, dev, total_chains, steps, warmup, world, gather=gather_mode, settle=settle,
                             resident=False)[0]
        log(f"end-to-end with host buffers: {e2e_pcie['pcn_steps_per_s'] / 1e6:.2f} M steps/s")
    gather = {"ms": e2e["gather_ms"], "mode": gather_mode,
              "bytes_per_rank": int(per_rank * (3 * prob.k + 2) * 8 if gather_mode == "all" else per_rank * 16),
              "what": "every chain's Phi and accept count (all_gather_into_tensor) and the posterior mean "
                      "(block sums of 1 024 chains on each rank's GPU, shared blocks and block sums in one all_gather)",
              "collective": (f"all_gather_into_tensor ({'RCCL' if args.dist_backend == 'nccl' else 'gloo'})"
                             + (" + block-sum all_gather" if gather_mode == "mean" else "")
                             if grouped else "none (one rank)"),
              "rows": int(res["phi"].shape[0]), "inside_timed_region": not args.kernel_only}
    assert np.isfinite(res["phi"]).all() and np.isfinite(res["mean"]).all()
    accept_rate = e2e["accept_rate"]
    del res

    extra = {"kernel_pcn_steps_per_s": kernel_rate, "kernel_ms": kern_ms,
             "kernel_note": "device-resident state, raw ipmc_pcn_sweep launches of steps_per_launch steps, HIP "
                            "events on the launch stream (the roofline's kernel time); no H2D / D2H / gather",
             "run_e2e_moments": e2e, "run_e2e_pcie": e2e_pcie}
    parity = {}
    if not args.no_parity and world == 1 and not args.kernel_only:
        # north_star's bit-exact accept streams, for the arithmetic value is
        # timed in: paired FMA / REFERENCE runs of the benched problems
        # (DESIGN.md §6 states and tests/test_gpu_paired_streams.py asserts the floors)
        pp = paired_streams(prob, per_rank, max(steps, 200), tdt, dev)
        log(f"paired FMA/REFERENCE accept streams ({args.workload}): {pp['identical_accept_stream_frac']:.5f} "
            f"identical over {pp['steps']} steps")
        parity["paired_identical_accept_frac"] = pp["identical_accept_stream_frac"]
        parity[args.workload] = pp
        if args.workload == "cfg3" and not args.no_configs:
            for key, ch, st in (("cfg4", 16384, 200), ("cfg5", 16384, 100)):
                pp = paired_streams(make_problem(key), ch, st, tdt, dev)
                log(f"paired FMA/REFERENCE accept streams ({key}): {pp['identical_accept_stream_frac']:.5f}")
                parity[key] = pp
        if "cfg5" in parity:
            parity["cfg5"]["note"] = CFG5_PARITY_NOTE
    if not args.no_extra and args.workload == "cfg3":
        # one-step launches: 40 steps are plenty; speculative launches (small
        # shards) are timed over the headline's steps, as short ones are slow
        xs = min(steps, 40) if per_launch == 1 else steps
        other = torch.float32 if tdt == torch.float64 else torch.float64
        key = "f32" if other == torch.float32 else "f64"
        w2 = Workload(prob, per_rank, lo_rank, other, dev, args.lanes, per_launch=per_launch)
        el2, k2 = timed(w2, xs, 2, world)
        log(f"{key}: kernel {k2:.3f} ms/launch")
        extra[f"{key}_kernel_pcn_steps_per_s"] = total_chains * xs / el2
        extra[f"{key}_kernel_ms"] = k2
        extra[f"{key}_kernel_tflops"] = per_rank * per_launch * prob.flop / (k2 * 1e-3) / 1e12
        del w2
        e2 = timed_run(prob, np.float32 if key == "f32" else np.float64, dev, total_chains, min(steps, 100), 2,
                       world, gather=gather_mode, settle=settle)[0]
        extra[f"{key}_run_pcn_steps_per_s"] = e2["pcn_steps_per_s"]
        # the reference's operation order (no FMA in the forward map): the
        # arithmetic whose accept streams are pinned to the reference fixtures
        pref = prob.reference_arith()
        w3 = Workload(pref, per_rank, lo_rank, tdt, dev, args.lanes, per_launch=per_launch)
        xr = min(xs, 20) if per_launch == 1 else xs
        el3, k3 = timed(w3, xr, 2, world)
        log(f"reference arith ({args.dtype}): kernel {k3:.3f} ms/launch")
        extra["reference_arith_kernel_pcn_steps_per_s"] = total_chains * xr / el3
        extra["reference_arith_kernel_ms"] = k3
        extra["reference_arith_kernel_tflops"] = per_rank * per_launch * prob.flop / (k3 * 1e-3) / 1e12
        del w3
        # REFERENCE arith end to end: the same timed region as value
        er = timed_run(pref, ndt, dev, total_chains, steps, 2, world, gather=gather_mode, settle=settle)[0]
        log(f"reference arith end to end: {er['pcn_steps_per_s'] / 1e6:.2f} M steps/s")
        parity["reference_arith_value"] = er["pcn_steps_per_s"]
        parity["reference_arith_run_e2e_moments"] = er
        # the headline's shape and kernel on a posterior the chains sample
        # (the rate should not depend on acceptance)
        pmix = make_problem("cfg3_mixing")
        em = timed_run(pmix, ndt, dev, total_chains, steps, 2, world, gather=gather_mode, settle=settle)[0]
        log(f"mixing posterior end to end: {em['pcn_steps_per_s'] / 1e6:.2f} M steps/s, "
            f"{em['accept_rate']:.3f} accepted")
        extra["mixing_posterior"] = dict(em, workload=pmix.name, data=pmix.data, over_value=em["pcn_steps_per_s"] / value,
                                         accept_rate_value=accept_rate)
        if world > 1:  # the other scaling beside the line: 65 536 chains per GPU / over the node
            other_s = "strong" if args.scaling == "weak" else "weak"
            n_other = ensemble(args.workload, world, None, other_s)[1]
            wk, _ = timed_run(prob, ndt, dev, n_other, steps, 2, world, gather=gather_mode, settle=settle)
            extra[f"{other_s}_scaling"] = {"pcn_steps_per_s": wk["pcn_steps_per_s"], "total_chains": n_other,
                                           "chains_per_gpu": wk["chains_per_gpu"], "ms_per_step": wk["ms_per_step"],
                                           "steps": wk["steps"], "timed": "run_sharded end to end, keep='moments'",
                                           "metric": metric_name(args.workload, prob.name, n_other)}
        extra["run_e2e_samples"] = e2e_samples(prob, per_rank, lo_rank, ndt, dev, world)
    if not args.no_configs and args.workload == "cfg3":
        cfgs = {}
        for key in ("cfg4", "cfg5"):
            log(f"extra.configs: {key} end to end")
            cfgs[key] = config_line(key, dev, world)
        if "cfg5" in parity and "arith_parity" in cfgs["cfg5"]:
            cfgs["cfg5"]["arith_parity"]["fma_paired_identical_accept_frac"] = \
                parity["cfg5"]["identical_accept_stream_frac"]
            cfgs["cfg5"]["arith_parity"]["fma_paired"] = {k: parity["cfg5"][k] for k in ("chains", "steps")}
        extra["configs"] = cfgs
    del settle, w

    flop = per_rank * per_launch * prob.flop
    achieved = flop / (kern_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    is_l96_40 = args.workload == "cfg3"
    pmc, pmc_src = pmc_record(args.dtype, per_rank, lanes_k) if (per_launch == 1 and is_l96_40) else (None, None)
    if args.pmc_file:
        pmc, pmc_src = json.load(open(args.pmc_file)), os.path.relpath(os.path.abspath(args.pmc_file), REPO)
    traffic = None if pmc is None else pmc["hbm_bytes_per_launch"]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log("CPU baseline (C oracle)")
        cpu = cpu_baseline(prob, ndt)
        import glob

        recs = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "reference_cpu_cfg3.json")), reverse=True)
        if is_l96_40 and recs:  # the reference itself, timed in the build container (tools/), newest round
            cpu["reference_recorded"] = json.load(open(recs[0]))
            cpu["reference_recorded"]["source"] = os.path.relpath(recs[0], REPO)

    if rank == 0:
        item = ITEM[args.dtype]
        line = {
            "metric": metric_name(args.workload, prob.name, total_chains),
            "value": value,
            "unit": "pCN steps/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": e2e["ms_per_step"],
            "higher_is_better": True,
            "kernel_only": bool(args.kernel_only),
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": prob.data,
            "config": {
                "workload": prob.name,
                "timed": "shard.run_sharded -> MCMCSampler.run(u_0 (chains x k) f64 in HBM, n_samples=1, burn_in=0, "
                         "sample_interval=steps, keep='moments', results='device') end to end: Phi(u_0), the fused "
                         "sweeps, the per-chain sums and states left in HBM, Phi and the accept counts to the host, "
                         "the block-sum posterior mean and the gather over ranks; max over ranks (the same run with "
                         "host buffers both ways, PCIe included: extra.run_e2e_pcie)",
                "chains_per_gpu": per_rank,
                "total_chains": total_chains,
                "k": prob.k,
                "beta": prob.beta,
                "arith": "fma",
                "kernel_leg_steps_per_launch": per_launch,
                "lanes_per_chain": lanes_k,
                "chains_per_lane": cpl_k,
                "spec_width": spec_k,
                # the benched arithmetic against the reference's operation order (parity.*)
                "arith_parity": None if not parity else {
                    "paired_identical_accept_stream_frac": parity.get("paired_identical_accept_frac"),
                    "paired_chains": parity.get(args.workload, {}).get("chains"),
                    "paired_steps": parity.get(args.workload, {}).get("steps"),
                    "reference_arith_value": parity.get("reference_arith_value")},
                "parallelism": f"{total_chains} chains sharded over {world} GPU(s) ({args.scaling} scaling)",
                "clock_settle_s": args.settle,
                "clock_settle": "untimed G evaluations of the kernel leg's chains before the kernel leg's and before "
                                "each end-to-end leg's timed region (after its warm-up run)",
            },
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": achieved / peak,
                "traffic": traffic,
                "traffic_unit": "bytes/launch (HBM, rocprofv3 PMC)",
                "traffic_source": pmc_src,
                "algorithmic_bytes": per_rank * per_launch * (prob.k * item + 2 * (item + 8)),
                "hbm_GBps": None if traffic is None else traffic / (kern_ms * 1e-3) / 1e9,
                "hbm_frac": None if traffic is None else traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "kernel_ms": kern_ms,
                "kernel_time_source": "HIP events around the kernel leg's timed launches (extra.kernel_*); "
                                      "tools/trace_summary.py restricts a rocprofv3 kernel trace to the same launches",
                "flop_per_launch": flop,
                "clock_GHz_pmc": None if pmc is None else pmc.get("effective_clock_GHz"),
                "valu_issue_per_simd_cycle_pmc": None if pmc is None else pmc.get("valu_issue_per_simd_cycle"),
                "mix_ceiling_frac": prob.mix_ceiling,
                "note": "vector-ALU bound (FP64 pipe; packed FP32 for f32), no MFMA and no HBM traffic in the "
                        "forward map's time loop: algorithmic FLOP = 30*d*n per chain-step (cfg3/cfg5; Burgers "
                        "30*N*n), on the kernel leg's launch time",
            },
            "cpu_baseline": cpu,
            "accept_rate": accept_rate,
            "parity": parity or None,
            "final_gather": gather,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
