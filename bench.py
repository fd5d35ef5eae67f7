"""Headline benchmark: pCN steps/s on Lorenz-96 d=40, 2000 RK4 steps, 65 536 chains.

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: started once, it launches torch.distributed.run with N ranks itself;
   under an external torch.distributed.run WORLD_SIZE must equal N)

A "step" is one pCN step of every chain of the batch: propose, run the forward
map (2000 RK4 steps of Lorenz-96, d=40), evaluate Φ, accept or reject -- the
fused libipmc kernel.  The metric's 65 536 chains are split over the N GPUs
(strong scaling, the default; global chain ids rank*65536/N + i); the weak
number (65 536 chains per GPU) is carried in "extra" for N > 1.  When a GPU
holds fewer chains than fill it, one launch runs several pCN steps
(--steps-per-launch, auto), so the speculative sweep can fill the lanes;
results are bit-identical to one step per launch.  Inputs are resident in HBM
before the timed region.  value = all chains of all ranks x K / max-rank wall
time.  Arithmetic: float64 with the FMA forward map (the reference computes in
float64); "extra" carries float32, the REFERENCE-arith (no FMA, the
reference's operation order) throughput, and MCMCSampler.run end to end
(host u_0 in, samples back on the host).

roofline: VALU-bound (no MFMA, no HBM traffic inside the RK loop). achieved =
algorithmic FLOP per launch / average kernel time from HIP events on the
launch stream; algorithmic FLOP per pCN step per chain = 30·d·n = 2.4 MFLOP
(SURVEY §8(d) counting rule).
cpu_baseline: the C oracle (same arithmetic, bit-exact), a bounded sample of
the same workload on this host's cores, rank 0 at N=1 only; the reference
itself, timed in the build container by tools/reference_cpu_baseline.py, is
attached as cpu_baseline.reference_recorded.
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

from ip_mcmc_amd import Lorenz96Operator, _abi  # noqa: E402
from ip_mcmc_amd._lib import call  # noqa: E402

D, N_RK, DT, BETA, GAMMA = 40, 2000, 0.005, 0.2, 0.1
ITEM = {"f64": 8, "f32": 4}
# 30 algorithmic FLOP per component and RK4 step in 20 VALU ops (10 of them
# FMA): at most 30 / (2 x 20) of the all-FMA peak
MIX_CEILING = 30 / 40
CHAINS_PER_GPU = 65536
FLOP_PER_STEP = 30 * D * N_RK  # 2.4e6
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}  # MI355X vector (spec), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0


def problem():
    """Config 3: forcing-field inverse problem."""
    op = Lorenz96Operator(D, forcing_mean=8.0, dt=DT, n_steps=N_RK)  # x0: 1000-step spin-up from 8 + 0.01 e0
    k = np.arange(D)
    u_true = 0.5 * np.sin(2 * np.pi * k / D)  # F_true = 8 + 0.5 sin(2πk/40)
    g_true = op(u_true)
    y = g_true + GAMMA * np.random.default_rng(3).normal(size=D)
    return op, y


class Workload:
    def __init__(self, op, y, n_chains, chain_offset, dtype, dev, lanes=0, d=D, chains_per_lane=0, per_launch=1,
                 spec_width=0):
        self.dev, self.dtype = dev, dtype
        self.n_chains, self.per_launch = n_chains, per_launch
        self.model, self._keep = op.model(dtype, dev)
        t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64)).to(dtype).to(dev).contiguous()
        self.y, self.ginv, self.sq = t(y), t(np.full(d, 1 / GAMMA)), t(np.ones(d))
        self.u = torch.zeros((n_chains, d), dtype=dtype, device=dev)
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
        s.beta, s.contraction = BETA, float(np.sqrt(1 - BETA**2))
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


def pmc_record(dtype, chains, lanes):
    """The committed rocprofv3 PMC passes of this sweep kernel (same dtype,
    chains, shape and lanes-per-chain layout): profiles/r*/pmc_l96_<dtype>.json,
    newest round first -- HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE,
    corrected as MI355X_MICROARCH.md's HBM section prescribes), clock and VALU
    issue rate -- with its path, or (None, None)."""
    import glob

    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"pmc_l96_{dtype}.json")), reverse=True):
        rec = json.load(open(path))
        names = " ".join(rec.get("kernel", []))
        if (rec.get("chains") == chains and rec.get("d") == D and rec.get("rk4_steps") == N_RK
                and f"{D}, {lanes}, true" in names):
            return rec, os.path.relpath(path, REPO)
    return None, None


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world, dev):
    if world > 1:
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


def cpu_baseline(op, y, dtype_np, budget_s=15.0):
    """The C oracle on this host's cores: a bounded sample of the same
    workload (chains x 1 pCN step), scaled to pCN steps/s."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))

    ginv = np.full(D, 1 / GAMMA)
    phi0 = O.potential(op, np.zeros((1, D), dtype=dtype_np), y, ginv, dtype_np)[0]

    def run(nc):
        U = np.zeros((nc, D), dtype=dtype_np)  # every chain starts at u = 0, as on the GPU
        phi = np.full(nc, phi0, dtype=dtype_np)
        acc = np.zeros(nc, dtype=np.int64)
        t0 = time.perf_counter()
        O.pcn_sweep(op, U, phi, y, ginv, np.ones(D), BETA, 2, 0, 1, accepts=acc, n_threads=threads)
        return time.perf_counter() - t0

    t1 = run(threads)  # one chain-step per thread, calibration
    per = t1 / threads  # wall seconds per chain-step with all threads busy
    n = int(max(threads, min(1_000_000, budget_s / max(per, 1e-9))))
    n = (n // threads) * threads
    el = run(n)
    return {"value": n / el, "unit": "pCN steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} chains x 1 pCN step of the headline workload (d=40, 2000 RK4 steps, "
                      f"{'f64' if dtype_np == np.float64 else 'f32'}), C oracle, {threads} threads, {el:.1f} s"}


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
    """pCN steps per launch: 1 when the rank's chains fill a wave per SIMD on
    their own (>= 16 384 chains, one launch per step), else 512, so that the
    sweep speculates over the steps of a launch (ipmc_plan_sweep).  A launch
    lasts as long as its slowest chain, so short speculative launches lose to
    the chains that accept early: 8 192 chains run sequentially on 8
    interleaved lanes below 256 steps per launch and speculate on 4 lanes x 2
    slots from there (ipmc_plan_sweep): 14.4 / 16.6 / 17.8 M steps/s on this
    problem at 20 / 200 / 1 024 timed steps, where round 3's first rule (2
    lanes x 8 slots) ran 5.9 / 15.6 / 18.9 M (profiles/r3/bench_8192_*.jsonl)."""
    return 1 if chains_per_rank >= 16384 else 512


def e2e_run(op, y, n_chains, chain_offset, dtype_np, dev, world, n_samples=20):
    """MCMCSampler.run end to end (SURVEY §8(d)'s timed region): host u_0
    (n_chains x 40) in, n_samples samples 1 step apart back on the host
    (page-locked, copied in blocks while later blocks sweep)."""
    from ip_mcmc_amd import (ConstSteppCNProposer, EvolutionPotential, GaussianDistribution, MCMCSampler,
                             PhiloxRNG, pCNAccepter)

    prior = GaussianDistribution(np.zeros(D), np.eye(D))
    pot = EvolutionPotential(op, y, GaussianDistribution(np.zeros(D), GAMMA**2 * np.eye(D)))
    u0 = np.full((n_chains, D), 0.0)  # written, i.e. resident (np.zeros maps its pages on first touch, inside run())
    s = MCMCSampler(ConstSteppCNProposer(BETA, prior), pCNAccepter(pot), PhiloxRNG(2), dtype=dtype_np, device=dev,
                    chain_offset=chain_offset)
    # warm run of the same size: device allocations, and the page-locked result
    # block that torch's host allocator recycles once the caller drops it
    s.run(u0, n_samples=n_samples, burn_in=1, sample_interval=1)
    torch.cuda.synchronize(dev)
    barrier(world)
    t0 = time.perf_counter()
    out = s.run(u0, n_samples=n_samples, burn_in=1, sample_interval=1)
    el = time.perf_counter() - t0
    assert out.shape == (n_chains, n_samples, D)
    barrier(world)
    el_max = max_over_ranks(el, world, dev)
    tm = s.last_run_timing
    return {"pcn_steps_per_s": world * n_chains * n_samples / el_max, "wall_s": el_max, "samples": n_samples,
            "sample_bytes_per_rank": int(out.nbytes), "setup_ms": tm["setup_s"] * 1e3,
            "sweeps_gpu_ms": tm["sweeps_gpu_ms"], "tail_ms_after_sweeps": tm["tail_ms"],
            "copy_overlapped": tm["copy_overlapped"],
            "note": "MCMCSampler.run(u0 host (chains x 40), n_samples, burn_in=1, sample_interval=1): H2D of u0, "
                    "Phi(u0), the sweeps, D2H of the (chains, n_samples, 40) f64 samples; tail = wall after set-up "
                    "not covered by the GPU sweeps (launch gaps + the last copy block + epilogue)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--chains", type=int, default=CHAINS_PER_GPU,
                    help="total chains (strong, the default) or chains per GPU (weak)")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong: --chains split over the GPUs (the metric's 65 536; default); "
                         "weak: --chains per GPU")
    ap.add_argument("--steps-per-launch", type=int, default=0, help="pCN steps per kernel launch (0 = auto)")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--spec-width", type=int, default=0, help="speculative slots per chain (0 = auto, 1 = off)")
    ap.add_argument("--settle", type=float, default=0.3,
                    help="seconds of untimed G evaluations before the warm-up steps (clock ramp; 0 = off)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
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
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    log(f"rank {rank}/{world} on {dev}: building the problem")
    op, y = problem()
    total_chains = args.chains * (world if args.scaling == "weak" else 1)
    if total_chains % world:
        raise SystemExit("--scaling strong needs --chains divisible by the number of GPUs")
    per_rank = total_chains // world
    # (a launch never exceeds the timed steps: the plan reported is the one timed)
    per_launch = min(args.steps_per_launch or auto_per_launch(per_rank), max(1, args.steps))
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    w = Workload(op, y, per_rank, rank * per_rank, tdt, dev, args.lanes, per_launch=per_launch,
                 spec_width=args.spec_width)
    log(f"timing {args.steps} pCN steps ({args.dtype}, {per_rank} chains/GPU, {per_launch} steps/launch, "
        f"lanes={w.lanes}, spec_width={w.spec_width})")
    el, kern_ms = timed(w, args.steps, args.warmup, world, args.settle)
    log(f"{args.dtype}: {el:.3f} s, kernel {kern_ms:.3f} ms/launch")
    value = total_chains * args.steps / el

    # final gather of the per-chain results (the path's one exchange): accept
    # rate and posterior-mean state over all chains of all ranks
    from ip_mcmc_amd.shard import gather_chains

    # (after the timed region: per-chain state u, Φ and accept counts of every
    # rank to every rank; all_gather_into_tensor = RCCL over xGMI at N > 1)
    torch.cuda.synchronize(w.dev)
    barrier(world)
    tg = time.perf_counter()
    host = (lambda t: t.cpu()) if args.dist_backend == "gloo" else (lambda t: t)
    u_all = gather_chains(host(w.u), total_chains)
    phi_all = gather_chains(host(w.phi.view(-1, 1)), total_chains)
    acc_all = gather_chains(host(w.acc.view(-1, 1)), total_chains)
    torch.cuda.synchronize(w.dev)
    gather_ms = (time.perf_counter() - tg) * 1e3
    gather = {"ms": gather_ms, "bytes_per_rank": int(w.u.numel() * w.u.element_size() + w.phi.numel() *
                                                     w.phi.element_size() + w.acc.numel() * 8),
              "collective": (f"all_gather_into_tensor ({'RCCL' if args.dist_backend == 'nccl' else 'gloo'})"
                             if world > 1 else "none (one rank)"),
              "rows": int(u_all.shape[0])}
    assert bool(torch.isfinite(phi_all).all())
    del u_all, phi_all
    accept_rate = float(acc_all.double().sum().item()) / (total_chains * (args.steps + args.warmup))

    extra = {}
    if not args.no_extra:
        # one-step launches: 40 steps are plenty; speculative launches (small
        # shards) are timed over the headline's steps, as short ones are slow
        xs = min(args.steps, 40) if per_launch == 1 else args.steps
        other = torch.float32 if tdt == torch.float64 else torch.float64
        key = "f32" if other == torch.float32 else "f64"
        w2 = Workload(op, y, per_rank, rank * per_rank, other, dev, args.lanes, per_launch=per_launch)
        el2, k2 = timed(w2, xs, 2, world)
        log(f"{key}: kernel {k2:.3f} ms/launch")
        extra[f"{key}_pcn_steps_per_s"] = total_chains * xs / el2
        extra[f"{key}_kernel_ms"] = k2
        extra[f"{key}_tflops"] = per_rank * per_launch * FLOP_PER_STEP / (k2 * 1e-3) / 1e12
        del w2
        # the reference's operation order (no FMA in the forward map): the
        # arithmetic whose accept streams are pinned to the reference fixtures
        op_ref = Lorenz96Operator(D, forcing_mean=8.0, x0=op.x0, dt=DT, n_steps=N_RK, arith="reference")
        w3 = Workload(op_ref, y, per_rank, rank * per_rank, tdt, dev, args.lanes, per_launch=per_launch)
        xr = min(xs, 20) if per_launch == 1 else xs
        el3, k3 = timed(w3, xr, 2, world)
        log(f"reference arith ({args.dtype}): kernel {k3:.3f} ms/launch")
        extra["reference_arith_pcn_steps_per_s"] = total_chains * xr / el3
        extra["reference_arith_kernel_ms"] = k3
        extra["reference_arith_tflops"] = per_rank * per_launch * FLOP_PER_STEP / (k3 * 1e-3) / 1e12
        del w3
        if world > 1:  # weak scaling beside the strong line: 65 536 chains per GPU
            w4 = Workload(op, y, CHAINS_PER_GPU, rank * CHAINS_PER_GPU, tdt, dev, args.lanes, per_launch=1)
            el4, k4 = timed(w4, xs, 2, world)
            extra["weak_scaling"] = {"pcn_steps_per_s": world * CHAINS_PER_GPU * xs / el4,
                                     "total_chains": world * CHAINS_PER_GPU, "ms_per_step": el4 / xs * 1e3,
                                     "kernel_ms": k4, "steps": xs}
            del w4
        extra["run_e2e"] = e2e_run(op, y, per_rank, rank * per_rank, np.float64 if tdt == torch.float64
                                   else np.float32, dev, world)
        extra["run_e2e_pcn_steps_per_s"] = extra["run_e2e"]["pcn_steps_per_s"]

    flop = per_rank * per_launch * FLOP_PER_STEP
    achieved = flop / (kern_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    pmc, pmc_src = pmc_record(args.dtype, per_rank, w.lanes) if per_launch == 1 else (None, None)
    traffic = None if pmc is None else pmc["hbm_bytes_per_launch"]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log("CPU baseline (C oracle)")
        cpu = cpu_baseline(op, y, np.float64 if tdt == torch.float64 else np.float32)
        ref_rec = os.path.join(REPO, "profiles", "r1", "reference_cpu_cfg3.json")
        if os.path.exists(ref_rec):  # the reference itself, timed in the build container (tools/)
            cpu["reference_recorded"] = json.load(open(ref_rec))

    if rank == 0:
        line = {
            "metric": "pCN steps/sec (whole node), Lorenz-96 d=40 T=2000, 65 536 chains",
            "value": value,
            "unit": "pCN steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (forcing-field inverse problem, y = G(u_true) + N(0, 0.1^2), seed 3)",
            "config": {
                "workload": "lorenz96_d40_rk4_2000_pcn",
                "chains_per_gpu": per_rank,
                "total_chains": total_chains,
                "d": D,
                "rk4_steps": N_RK,
                "dt": DT,
                "beta": BETA,
                "arith": "fma",
                "steps_per_launch": per_launch,
                "lanes_per_chain": w.lanes,
                "chains_per_lane": w.chains_per_lane,
                "spec_width": w.spec_width,
                "parallelism": f"{total_chains} chains sharded over {world} GPU(s) ({args.scaling} scaling)",
                "clock_settle_s": args.settle,
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
                "algorithmic_bytes": per_rank * per_launch * (D * ITEM[args.dtype] + 2 * (ITEM[args.dtype] + 8)),
                "hbm_GBps": None if traffic is None else traffic / (kern_ms * 1e-3) / 1e9,
                "hbm_frac": None if traffic is None else traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "kernel_ms": kern_ms,
                "flop_per_launch": flop,
                "clock_GHz_pmc": None if pmc is None else pmc.get("effective_clock_GHz"),
                "valu_issue_per_simd_cycle_pmc": None if pmc is None else pmc.get("valu_issue_per_simd_cycle"),
                "mix_ceiling_frac": MIX_CEILING,
                "note": "vector-ALU bound (FP64 pipe; packed FP32 for f32), no MFMA and no HBM traffic in the "
                        "RK loop: algorithmic FLOP = 30*d*n per chain-step, issued as 20 VALU ops of which 10 "
                        "FMA, so the op mix caps achieved/peak at mix_ceiling_frac (x clock/2.4 GHz); "
                        "valu_issue_per_simd_cycle 0.25 = a wave64 op every 4 cycles = the pipe issuing every "
                        "slot (traffic_source holds the PMC passes)",
            },
            "cpu_baseline": cpu,
            "accept_rate": accept_rate,
            "final_gather": gather,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
