"""Headline benchmark: pCN steps/s on Lorenz-96 d=40, 2000 RK4 steps, 65 536 chains.

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: launched by torch.distributed.run, one process per GPU)

A "step" is one pCN sweep: every chain of the batch proposes, runs its
forward map (2000 RK4 steps of Lorenz-96, d=40), evaluates Φ and accepts or
rejects -- one launch of the fused libipmc kernel.  Each GPU owns 65 536
chains (weak scaling; global chain ids rank*65536 + i), inputs resident in
HBM before the timed region.  value = all chains of all ranks x K / max-rank
wall time.  Arithmetic: float64 (the reference computes in float64); the
float32 throughput of the same workload is reported in "extra".

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
    def __init__(self, op, y, n_chains, chain_offset, dtype, dev, lanes=0, d=D, chains_per_lane=0):
        self.dev, self.dtype = dev, dtype
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
        s.dtype, s.lanes_per_chain, s.chains_per_lane = adt, lanes, chains_per_lane
        s.n_chains, s.chain_offset = n_chains, chain_offset
        s.u, s.phi, s.accepts = self.u.data_ptr(), self.phi.data_ptr(), self.acc.data_ptr()
        s.y, s.gamma_inv, s.prior_sqrt = self.y.data_ptr(), self.ginv.data_ptr(), self.sq.data_ptr()
        s.beta, s.contraction = BETA, float(np.sqrt(1 - BETA**2))
        s.seed, s.step0, s.n_steps = 2, 0, 1
        self.s = s
        # the plan the sweep runs (ipmc_plan_sweep: same code path as the launch)
        self.lanes, self.chains_per_lane, self.spec_width = sweep_plan(self.model, s)

    def step(self):
        call("ipmc_pcn_sweep", C.byref(self.model), C.byref(self.s), self.stream)
        self.s.step0 += 1


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


def timed(w, steps, warmup, world):
    for _ in range(warmup):
        w.step()
    torch.cuda.synchronize(w.dev)
    barrier(world)
    torch.cuda.synchronize(w.dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record()
        w.step()
        b.record()
    torch.cuda.synchronize(w.dev)
    barrier(world)
    torch.cuda.synchronize(w.dev)
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=w.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, kern_ms


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chains", type=int, default=CHAINS_PER_GPU, help="chains per GPU (weak) or in total (strong)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --chains per GPU (default); strong: --chains split over the GPUs")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the product path) or gloo (rehearsal of the N-rank logic)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 (rehearsing N ranks on a one-GPU box; needs --dist-backend gloo)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_device and args.dist_backend != "gloo":
        raise SystemExit("--share-device needs --dist-backend gloo (RCCL wants one GPU per rank)")
    dev = torch.device("cuda", 0 if args.share_device else local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    log(f"rank {rank}/{world} on {dev}: building the problem")
    op, y = problem()
    if args.scaling == "strong":
        if args.chains % world:
            raise SystemExit("--scaling strong needs --chains divisible by the number of GPUs")
        args.chains //= world  # chains per rank from here on
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    w = Workload(op, y, args.chains, rank * args.chains, tdt, dev, args.lanes)
    log(f"timing {args.steps} sweeps ({args.dtype}, {args.chains} chains/GPU, lanes={w.lanes})")
    el, kern_ms = timed(w, args.steps, args.warmup, world)
    log(f"{args.dtype}: {el:.3f} s, kernel {kern_ms:.3f} ms/launch")
    total_steps = world * args.chains * args.steps
    value = total_steps / el

    # final gather of the per-chain results (the path's one exchange): accept
    # rate and posterior-mean state over all chains of all ranks
    from ip_mcmc_amd.shard import gather_chains

    # (after the timed region: per-chain state u, Φ and accept counts of every
    # rank to every rank; all_gather_into_tensor = RCCL over xGMI at N > 1)
    torch.cuda.synchronize(w.dev)
    barrier(world)
    tg = time.perf_counter()
    host = (lambda t: t.cpu()) if args.dist_backend == "gloo" else (lambda t: t)
    u_all = gather_chains(host(w.u), world * args.chains)
    phi_all = gather_chains(host(w.phi.view(-1, 1)), world * args.chains)
    acc_all = gather_chains(host(w.acc.view(-1, 1)), world * args.chains)
    torch.cuda.synchronize(w.dev)
    gather_ms = (time.perf_counter() - tg) * 1e3
    gather = {"ms": gather_ms, "bytes_per_rank": int(w.u.numel() * w.u.element_size() + w.phi.numel() *
                                                     w.phi.element_size() + w.acc.numel() * 8),
              "collective": (f"all_gather_into_tensor ({'RCCL' if args.dist_backend == 'nccl' else 'gloo'})"
                             if world > 1 else "none (one rank)"),
              "rows": int(u_all.shape[0])}
    assert bool(torch.isfinite(phi_all).all())
    del u_all, phi_all
    accept_rate = float(acc_all.double().sum().item()) / (world * args.chains * (args.steps + args.warmup))

    extra = {}
    if not args.no_extra:
        other = torch.float32 if tdt == torch.float64 else torch.float64
        w2 = Workload(op, y, args.chains, rank * args.chains, other, dev, args.lanes)
        el2, k2 = timed(w2, args.steps, args.warmup, world)
        log(f"{other}: kernel {k2:.3f} ms/launch")
        key = "f32" if other == torch.float32 else "f64"
        extra[f"{key}_pcn_steps_per_s"] = world * args.chains * args.steps / el2
        extra[f"{key}_kernel_ms"] = k2
        extra[f"{key}_tflops"] = args.chains * FLOP_PER_STEP / (k2 * 1e-3) / 1e12
        del w2

    flop = args.chains * FLOP_PER_STEP
    achieved = flop / (kern_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    pmc, pmc_src = pmc_record(args.dtype, args.chains, w.lanes)
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
                "chains_per_gpu": args.chains,
                "total_chains": world * args.chains,
                "d": D,
                "rk4_steps": N_RK,
                "dt": DT,
                "beta": BETA,
                "arith": "fma",
                "lanes_per_chain": w.lanes,
                "chains_per_lane": w.chains_per_lane,
                "spec_width": w.spec_width,
                "parallelism": f"chains sharded over {world} GPU(s)",
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
                "algorithmic_bytes": args.chains * (D * ITEM[args.dtype] + 2 * (ITEM[args.dtype] + 8)),
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
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
