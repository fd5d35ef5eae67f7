"""MCMCSampler — drop-in for ``ip_mcmc/sampler.py`` on many chains at once.

Reference (sampler.py:6-54): ``MCMCSampler(proposal, acceptance, rng)``;
``run(u_0, n_samples, burn_in=1000, sample_interval=200)`` advances ONE chain
``max(0, burn_in − sample_interval) + n_samples·sample_interval`` steps
(:18-26), records the state after every block of ``sample_interval`` steps
(:28) and returns a float64 array (n_samples, k).

Here ``u_0`` may be one state (k,) — same return shape as the reference — or
a stack (C, k) of C independent chains, returning (C, n_samples, k).  The
step (ConstSteppCNProposer / VarSteppCNProposer / ConstStepStandardRWProposer /
VarStepStandardRWProposer + pCNAccepter or StandardRWAccepter on an
EvolutionPotential with a device forward map, optionally wrapped in
CountedAccepter / ConstrainAccepter(BoxConstraint)) runs as one fused HIP
kernel per block of steps (libipmc ``ipmc_pcn_sweep``).  A composition with
caller Python code in it -- a Python forward map, a constraint predicate, a
non-diagonal noise covariance, a user proposer or accepter -- runs the
host-side step of hostloop.py instead, with the same GPU-drawn Philox stream
(no composition the kernels can run ever takes that path).

Differences from the reference, all deliberate:
  * randomness is the counter-based Philox stream of rng.py, not PCG64;
  * Φ(u) is cached between steps instead of recomputed (accepter.py:122);
  * the per-sample ``print`` (sampler.py:24) happens only with verbose=True.
"""
import ctypes as C
import math
import time

import numpy as np
import torch

from . import _abi
from . import device as dev
from ._lib import UnsupportedOnDevice, call
from .accepter import BoxConstraint, ConstrainAccepter, CountedAccepter, StandardRWAccepter, pCNAccepter
from .distribution import GaussianDistribution
from .potential import EvolutionPotential
from .chainio import ChainState, NpySampleSink
from .rng import PhiloxRNG, resolve_rng

# pCN steps per chain in one kernel launch (launches are split at sample
# boundaries; this bounds a single launch's run time for large ensembles).
# A speculative launch lasts as long as its slowest chain takes to settle the
# launch's steps, and that excess over the mean shrinks with the launch
# length: config 2 (4 096 chains, 88 % accepted) runs 323 / 403 / 447 M steps/s
# at 1 024 / 4 096 / 16 384 steps per launch (profiles/r3/launch_len.jsonl).
STEPS_PER_LAUNCH = 16384
# ... and fewer for heavy ensembles: about LAUNCH_WORK state-component updates
# per launch (~0.5 s on one MI355X; the headline sweep is 5.2e9 per step).
LAUNCH_WORK = 8e11


def _steps_per_launch(model, n_chains):
    """pCN steps per launch so that one launch stays around half a second."""
    rk = model.n_steps if model.n_steps > 0 else 1000
    state = max(1, model.dim) * (1 + max(0, model.fast_per_slow))
    per_step = float(n_chains) * rk * state
    return int(max(1, min(STEPS_PER_LAUNCH, LAUNCH_WORK // max(per_step, 1.0))))


class _Plan:
    """The device form of a proposer/accepter composition."""

    def __init__(self, proposer, accepter):
        if getattr(proposer, "kind", None) not in ("pcn", "rw"):
            raise UnsupportedOnDevice(
                "device sampler needs a ConstSteppCNProposer, VarSteppCNProposer, ConstStepStandardRWProposer or "
                f"VarStepStandardRWProposer, not {type(proposer).__name__}"
            )
        self.proposer = proposer
        self.proposal = _abi.PROPOSAL_RW if proposer.kind == "rw" else _abi.PROPOSAL_PCN
        # w ~ N(0, C): sqrt(C_ii)·ξ_i for a diagonal C, else L·ξ with L the lower
        # Cholesky factor (ipmc_sweep.prior_chol)
        if proposer.w.is_diagonal:
            self.prior_sqrt, self.prior_chol = proposer.w.sqrt_diagonal, None
        else:
            self.prior_sqrt, self.prior_chol = None, proposer.w.L
        self.counted_outer = []  # CountedAccepters that see every step
        self.counted_inner = []  # CountedAccepters inside a ConstrainAccepter
        self.box = None
        self.reg_scale = None
        acc, inside = accepter, False
        while True:
            if isinstance(acc, CountedAccepter):
                (self.counted_inner if inside else self.counted_outer).append(acc)
                acc = acc.accepter
            elif isinstance(acc, ConstrainAccepter):
                if self.box is not None:
                    raise UnsupportedOnDevice("only one ConstrainAccepter is supported on the device")
                if not isinstance(acc.is_valid, BoxConstraint):
                    raise UnsupportedOnDevice(
                        "ConstrainAccepter on the device needs a BoxConstraint (a Python callable cannot run in the kernel)"
                    )
                self.box = acc.is_valid
                inside = True
                acc = acc.accepter
            elif isinstance(acc, pCNAccepter):
                break
            elif isinstance(acc, StandardRWAccepter):
                prior = acc.prior
                if not isinstance(prior, GaussianDistribution) or not prior.is_diagonal:
                    raise UnsupportedOnDevice("StandardRWAccepter on the device needs a diagonal GaussianDistribution prior")
                self.reg_scale = prior.sqrt_diagonal  # apply_sqrt_covariance's diagonal (Q6)
                break
            else:
                raise UnsupportedOnDevice(
                    f"device sampler needs a pCNAccepter or StandardRWAccepter, not {type(acc).__name__}"
                )
        pot = acc.theta
        if not isinstance(pot, EvolutionPotential):
            raise UnsupportedOnDevice(f"the accepter's potential must be an EvolutionPotential, not {type(pot).__name__}")
        self.potential = pot
        self.G = pot.G
        self.y_eff, self.gamma_inv = pot.device_terms()
        if proposer.w.k != self.G.k:
            raise ValueError(f"prior dimension {proposer.w.k} != forward map k = {self.G.k}")
        if self.reg_scale is not None and self.reg_scale.shape[0] != self.G.k:
            raise ValueError("StandardRWAccepter prior dimension != forward map k")


class MCMCSampler:
    def __init__(
        self,
        proposal,
        acceptance,
        rng,
        dtype=np.float64,
        device=None,
        lanes_per_chain=0,
        chain_offset=0,
        verbose=False,
        spec_width=0,
    ):
        """Reference signature (sampler.py:7-10) plus device options:
        dtype (np.float64 or np.float32), device, lanes_per_chain (kernel
        layout, 0 = auto), chain_offset (global id of chain 0, for sharding),
        spec_width (speculative steps per round for small ensembles: 0 = auto,
        1 = off; results are identical either way)."""
        self.proposer = proposal
        self.accepter = acceptance
        self.rng = rng
        self.dtype = dtype
        self.device = device
        self.lanes_per_chain = int(lanes_per_chain)
        self.chain_offset = int(chain_offset)
        self.verbose = verbose
        self.spec_width = int(spec_width)
        # state of the last run (device tensors), for inspection / continuation
        self.state = None
        self.last_run_seconds = None
        # keep_device_sums: a keep="moments" device run leaves its (sum_u,
        # sum_u2) device tensors in last_device_sums (shard.run_sharded sums
        # them on the device for the posterior mean); off by default
        self.keep_device_sums = False
        self.last_device_sums = None
        # pre_sync: a callable f(sums) that a keep="moments" device run calls
        # with its (sum_u, sum_u2) device tensors after the sweeps are queued
        # and before its one synchronisation, so that device work on the sums
        # and its page-locked copies ride the same wait (shard.run_sharded's
        # block sums); its return value is left in pre_sync_result
        self.pre_sync = None
        self.pre_sync_result = None
        # "device" (fused kernels), "host" / "host-generic" (hostloop.py) for the last run
        self.last_path = None
        self.last_run_timing = None

    # ------------------------------------------------------------------ run
    def run(self, u_0, n_samples, burn_in=1000, sample_interval=200, keep="samples", sample_file=None,
            flush_every=None, results="host"):
        """Run the chain(s).  keep='samples' returns the samples like the
        reference; keep='moments' returns a dict of per-chain sums of u and u²
        over every post-burn-in step (no sample array); keep='last' returns
        the final states (C, k).

        results='device' (keep='moments' or 'last', device path) leaves the
        per-chain results in HBM: the sums / last states come back as device
        tensors and the checkpoint's states stay on the device (ChainState.u is
        copied to the host on first access); only Φ and the counters are
        copied.  u_0 may then be a device tensor too, so a run starts and ends
        in HBM.  The host tier always returns host arrays.

        u_0 may be a ChainState (``checkpoint()`` / ``chainio.load_state``):
        the run then continues those chains exactly (same Φ cache, Philox
        position and proposer counter).  sample_file='x.npy' streams the
        samples into a np.load-compatible file block by block (every
        ``flush_every`` samples) and returns it memory-mapped."""
        if keep not in ("samples", "moments", "last"):
            raise ValueError("keep must be 'samples', 'moments' or 'last'")
        if results not in ("host", "device"):
            raise ValueError("results must be 'host' or 'device'")
        if results == "device" and keep == "samples":
            raise ValueError("results='device' keeps keep='moments' or 'last' in HBM")
        on_dev = results == "device"
        t_entry = time.perf_counter()
        self.last_device_sums = self.pre_sync_result = None
        try:
            plan = _Plan(self.proposer, self.accepter)
        except UnsupportedOnDevice as e:
            # a Python forward map / constraint / noise model or a caller's own
            # proposer or accepter: the host-side step (hostloop.py), with the
            # same counter-based draws from the GPU
            from . import hostloop

            return hostloop.run(self, u_0, n_samples, burn_in, sample_interval, keep, sample_file, str(e))
        self.last_path = "device"
        device = dev.resolve_device(self.device)
        td = dev.torch_dtype(self.dtype)
        k = plan.G.k
        resume = isinstance(u_0, ChainState)
        if resume:
            u_src = u_0.u_device if u_0.u_device is not None else u_0.u
            if u_src.shape[1] != k:
                raise ValueError(f"ChainState has k={u_src.shape[1]}, forward map k={k}")
            single = False
            U = dev.to_device(u_src, td, device).clone()
        elif isinstance(u_0, torch.Tensor):
            single = u_0.dim() <= 1
            U = u_0.reshape(-1, k).to(device=device, dtype=td).clone().contiguous()
        else:
            arr = np.asarray(u_0, dtype=np.float64)
            single = arr.ndim <= 1
            U = dev.to_device(arr.reshape(-1, k), td, device).clone()
        n_chains = U.shape[0]
        n_samples = int(n_samples)
        sample_interval = int(sample_interval)
        if n_samples < 0 or sample_interval < 0:
            raise ValueError("n_samples and sample_interval must be >= 0")

        # the seed is resolved once and kept, so the Philox position carries
        # over between runs like the reference's one Generator (code.org:12-13)
        if not isinstance(self.rng, PhiloxRNG):
            self.rng = resolve_rng(self.rng)
        rng = self.rng
        accept_kind = "rw_reg" if plan.reg_scale is not None else "pcn"
        if resume:
            _check_resume(u_0, self.chain_offset, accept_kind)
            rng.seed, rng.step = u_0.seed, u_0.step
            if hasattr(plan.proposer, "i"):
                plan.proposer.i = u_0.proposer_i
        if isinstance(self.accepter, CountedAccepter):
            self.accepter.reset()  # sampler.py:15-16

        cur_stream = torch.cuda.current_stream(device)  # looked up once (~13 us a call)
        stream = cur_stream.cuda_stream
        phi = torch.empty((n_chains,), dtype=td, device=device)
        accepts = torch.zeros((n_chains,), dtype=torch.int64, device=device)
        calls = torch.zeros((n_chains,), dtype=torch.int64, device=device) if plan.counted_inner else None
        y_t = dev.const_to_device(plan.y_eff, td, device)
        gi_t = dev.const_to_device(plan.gamma_inv, td, device)
        sq_t = None if plan.prior_sqrt is None else dev.const_to_device(plan.prior_sqrt, td, device)
        chol_t = None if plan.prior_chol is None else dev.const_to_device(plan.prior_chol, td, device)
        keep_alive = [y_t, gi_t, sq_t, chol_t]
        box_ptrs = (None, None, None)
        if plan.box is not None:
            arrs = plan.box.arrays(k)
            ts = [None if a is None else dev.const_to_device(a, td, device) for a in arrs]
            keep_alive += [t for t in ts if t is not None]
            box_ptrs = tuple(dev.ptr(t) for t in ts)
        reg_t = None if plan.reg_scale is None else dev.const_to_device(plan.reg_scale, td, device)
        keep_alive.append(reg_t)
        model, _ = plan.G.model(td, device)

        sw = _abi.IpmcSweep()
        sw.dtype = dev.abi_dtype(td)
        sw.lanes_per_chain = self.lanes_per_chain
        sw.spec_width = self.spec_width
        sw.n_chains = n_chains
        sw.chain_offset = self.chain_offset
        sw.u = U.data_ptr()
        sw.phi = phi.data_ptr()
        sw.accepts = accepts.data_ptr()
        sw.calls = dev.ptr(calls)
        sw.y = y_t.data_ptr()
        sw.gamma_inv = gi_t.data_ptr()
        sw.prior_sqrt = dev.ptr(sq_t)
        sw.prior_chol = dev.ptr(chol_t)
        sw.box_lo, sw.box_hi, sw.box_off = box_ptrs
        sw.proposal = plan.proposal
        sw.reg_scale = dev.ptr(reg_t)
        const_beta = hasattr(plan.proposer, "device_step")
        if const_beta:
            sw.beta, sw.contraction = plan.proposer.device_step()
        sw.seed = rng.seed
        sw.accepts_step0 = rng.step  # the accept counters start at this run's first step
        # the accept potential of the starting states: Φ(u), or I(u) for StandardRWAccepter
        state_dtype = "float64" if td == torch.float64 else "float32"
        if resume and u_0.phi.shape[0] != n_chains:
            raise ValueError("ChainState phi does not match its u")
        ev_setup = torch.cuda.Event(enable_timing=True)  # the GPU work of the set-up: Φ(u0)
        ev_setup.record(cur_stream)
        if resume and u_0.dtype == state_dtype and u_0.accept_kind != "generic":
            phi.copy_(dev.to_device(u_0.phi, td, device))
        else:
            # a fresh run, a state saved in the other precision (its Φ cache is
            # not this dtype's Φ(u)) or by the generic host tier (no Φ cache):
            # recompute it
            call("ipmc_init_phi", C.byref(model), C.byref(sw), stream)

        step = rng.step
        prop_i = getattr(plan.proposer, "i", 0)

        def launch(n, sample_view=None, sums=None):
            nonlocal step, prop_i
            if n <= 0 and sample_view is None:
                return
            sched = None
            if not const_beta and n > 0:
                sched = torch.as_tensor(plan.proposer.beta_schedule(prop_i, n)).to(device)
                keep_alive.append(sched)
            sw.beta_schedule = dev.ptr(sched)
            if not const_beta:
                sw.beta, sw.contraction = 0.0, 1.0
            sw.step0 = step
            sw.n_steps = n
            sw.sample_every = 0
            if sample_view is not None:
                sw.sample_out = sample_view.data_ptr()
                sw.sample_stride = sample_view.stride(0)
            else:
                sw.sample_out = None
                sw.sample_stride = 0
            sw.sum_u, sw.sum_u2 = (None, None) if sums is None else (sums[0].data_ptr(), sums[1].data_ptr())
            call("ipmc_pcn_sweep", C.byref(model), C.byref(sw), stream)
            step += n
            prop_i += n

        def launch_blocks(nb, interval, first_view, sums):
            """nb samples `interval` steps apart, sample i into first_view's slot
            + i: launches of up to `spl` steps that record their samples inside
            the kernel (ipmc_sweep.sample_every), issued by ipmc_pcn_run -- no
            host round trip per sample, and the speculative sweeps of small
            ensembles run across sample boundaries."""
            nonlocal step, prop_i
            per = max(1, spl // interval)  # samples per launch
            sched = None
            if not const_beta:
                sched = torch.as_tensor(plan.proposer.beta_schedule(prop_i, nb * interval)).to(device)
                keep_alive.append(sched)
                sw.beta, sw.contraction = 0.0, 1.0
            sw.sum_u, sw.sum_u2 = (None, None) if sums is None else (sums[0].data_ptr(), sums[1].data_ptr())
            sw.sample_every = interval if first_view is not None else 0
            sw.sample_step_stride = k
            done = 0
            for n_launch, n_per in ((nb // per, per), (1 if nb % per else 0, nb % per)):
                if n_launch == 0:
                    continue
                sw.step0 = step
                sw.beta_schedule = 0 if sched is None else sched.data_ptr() + 16 * done * interval
                if first_view is not None:
                    sw.sample_out = first_view.data_ptr() + first_view.element_size() * done * k
                    sw.sample_stride = first_view.stride(0)
                else:
                    sw.sample_out = None
                    sw.sample_stride = 0
                call("ipmc_pcn_run", C.byref(model), C.byref(sw), n_launch, n_per * interval, n_per * k, stream)
                done += n_launch * n_per
                step += n_launch * n_per * interval
            prop_i += nb * interval
            sw.sample_every = 0

        t0 = time.perf_counter()
        ev_first = torch.cuda.Event(enable_timing=True)
        ev_first.record(cur_stream)
        spl = _steps_per_launch(model, n_chains)
        n_burn = max(0, burn_in - sample_interval)  # sampler.py:18
        for c0 in range(0, n_burn, spl):
            launch(min(spl, n_burn - c0))

        samples = None
        sums = None
        sink = None
        buf_len = n_samples
        if keep == "samples":
            if sample_file is not None:
                sink = NpySampleSink(sample_file, (n_samples, k) if single else (n_chains, n_samples, k))
                # device staging buffers of <= ~256 MiB between flushes
                auto = max(1, (1 << 28) // max(1, n_chains * k * 8))
                buf_len = max(1, min(n_samples, int(flush_every) if flush_every else auto))
                writer = _StreamingWriter(sink, (n_chains, buf_len, k), td, device, 2 if n_samples > buf_len else 1,
                                          single)
                samples = writer.buffer
            else:
                samples = torch.empty((n_chains, buf_len, k), dtype=td, device=device)
        elif keep == "moments":
            sums = (
                torch.zeros((n_chains, k), dtype=torch.float64, device=device),
                torch.zeros((n_chains, k), dtype=torch.float64, device=device),
            )
        # one launch per sample: the whole loop (up to the next streaming flush)
        # in one ipmc_pcn_run call; consecutive sample slots are k elements apart
        blockwise = (not self.verbose) and 0 < sample_interval <= spl
        # Large in-memory sample arrays go to the host in blocks of samples while
        # the later blocks are still sweeping (copy stream, rectangular D2H
        # copies into the page-locked result): only the last block's copy is
        # left after the sweeps.
        out_bytes = n_chains * n_samples * k * 8
        overlap = (blockwise and keep == "samples" and sink is None and n_samples >= 2
                   and OVERLAP_COPY_MIN_BYTES <= out_bytes <= PINNED_MAX_BYTES and dev.rect_copy_available())
        bounds = [n_samples]
        copies = []  # (first sample, end sample, event after its sweeps)
        src64 = None
        if overlap:
            # the last block is one sample: its copy is all that is left after
            # the sweeps (blocks of ~n/8 samples before it)
            n_blk = min(n_samples - 1, OVERLAP_COPY_BLOCKS - 1)
            bounds = [(j + 1) * (n_samples - 1) // n_blk for j in range(n_blk)] + [n_samples]
            if td != torch.float64:
                # f64 staging for the converted blocks, allocated before any sweep
                # is queued so that no block still in use is handed back to us
                src64 = torch.empty((n_chains, n_samples, k), dtype=torch.float64, device=device)
        i = 0
        while blockwise and i < n_samples:  # sampler.py:23-28
            slot = i % buf_len  # 0: segments end where the staging buffer is full
            nb = min(n_samples - i, buf_len - slot, next(b for b in bounds if b > i) - i)
            launch_blocks(nb, sample_interval, None if samples is None else samples[:, slot, :], sums)
            if sink is not None:
                samples = writer.flush(i - slot, slot + nb)
            if overlap:
                ev = torch.cuda.Event()
                ev.record(cur_stream)
                copies.append((i, i + nb, ev))
            i += nb
        for i in range(0 if not blockwise else n_samples, n_samples):  # sampler.py:23-28
            if self.verbose:
                print(f"Sampling {i + 1}/{n_samples}")
            slot = i % buf_len
            done = 0
            while done < sample_interval:
                n = min(spl, sample_interval - done)
                last = done + n == sample_interval
                view = samples[:, slot, :] if (samples is not None and last) else None
                launch(n, view, sums)
                done += n
            if sample_interval == 0 and samples is not None:
                launch(0, samples[:, slot, :])
            if sink is not None and (slot == buf_len - 1 or i == n_samples - 1):
                samples = writer.flush(i - slot, slot + 1)
        if sink is not None:
            writer.finish()
        ev_swept = torch.cuda.Event(enable_timing=True)
        ev_swept.record(cur_stream)
        # the host copy of the samples goes to page-locked memory (~57 GB/s
        # instead of ~5 GB/s pageable on the MI355X box, profiles/r1/d2h_probe.txt);
        # allocating it here overlaps the allocation with the queued sweeps
        host_out = None
        if keep == "samples" and sink is None:
            host_out = _host_buffer(tuple(samples.shape))
        if overlap:
            copy_stream = torch.cuda.Stream(device=device)
            src = samples if src64 is None else src64
            pitch = n_samples * k * 8
            with torch.cuda.stream(copy_stream):
                for i0, i1, ev in copies:
                    copy_stream.wait_event(ev)
                    if src64 is not None:
                        src64[:, i0:i1].copy_(samples[:, i0:i1])
                    dev.copy_rows_d2h(host_out.data_ptr() + i0 * k * 8, pitch, src.data_ptr() + i0 * k * 8, pitch,
                                      (i1 - i0) * k * 8, n_chains, copy_stream.cuda_stream)
        # the chain state (u, Φ, counters) to page-locked host memory on the
        # sweep stream, queued before the wait: a pageable copy of u alone was
        # ~2-4 ms after the sweeps at the headline size (21 MB)
        # (results='device': the states and sums stay in HBM; Φ and the counters,
        # 16 B per chain, still come back for the checkpoint and the counters)
        state_host = [None if on_dev else _pinned_copy(U)] + [_pinned_copy(t) for t in (phi, accepts, calls)
                                                              if t is not None]
        sums_host = None if (sums is None or on_dev) else [_pinned_copy(t) for t in sums]
        pre = self.pre_sync(sums) if (self.pre_sync is not None and sums is not None) else None
        torch.cuda.synchronize(device)
        self.pre_sync_result = pre
        self.last_run_seconds = time.perf_counter() - t0

        total = step - rng.step
        rng.step = step
        if hasattr(plan.proposer, "i"):
            plan.proposer.i = prop_i

        u_np = U if on_dev else state_host[0].numpy()
        phi_np, acc_np = (t.numpy() for t in state_host[1:3])
        calls_np = state_host[3].numpy() if calls is not None else None
        for ca in plan.counted_outer:
            _bump(ca, np.full(n_chains, total, dtype=np.int64), acc_np, single)
        for ca in plan.counted_inner:
            _bump(ca, calls_np, acc_np, single)
        if self.verbose and isinstance(self.accepter, CountedAccepter):
            print(f"Acceptance ratio: {self.accepter.ratio()}")  # sampler.py:30-31

        prev_acc = u_0.accepts if resume else 0
        prev_calls = u_0.calls if (resume and u_0.calls is not None) else 0
        self.state = ChainState(
            u_np, phi_np, prev_acc + acc_np,
            None if calls_np is None else prev_calls + calls_np, rng.seed, rng.step, prop_i, state_dtype,
            chain_offset=self.chain_offset, accept_kind=accept_kind,
        )
        self.state.steps_this_run = total
        if keep == "samples" and sink is None and not overlap:
            host_out.copy_(samples if samples.dtype == torch.float64 else samples.double())
        # where the wall time went: host set-up (H2D, plan; Φ(u0) is queued) before
        # the first launch, the GPU time of Φ(u0) and of all sweeps, and the rest
        # after set-up that the sweeps do not cover (Φ(u0) still running when the
        # host finished its set-up, launch gaps, the copy tail, host epilogue)
        t_end = time.perf_counter()
        sweeps_ms = ev_first.elapsed_time(ev_swept)
        phi0_ms = ev_setup.elapsed_time(ev_first)
        self.last_run_timing = {"total_s": t_end - t_entry, "setup_s": t0 - t_entry, "phi0_gpu_ms": phi0_ms,
                                "sweeps_gpu_ms": sweeps_ms,
                                "tail_ms": (t_end - t0) * 1e3 - sweeps_ms, "copy_overlapped": bool(overlap)}
        if keep == "samples":
            if sink is not None:
                return sink.close()
            out = host_out.numpy()  # shares the page-locked buffer (kept alive by the array)
            return out[0] if single else out
        self.last_device_sums = sums if (keep == "moments" and self.keep_device_sums) else None
        if keep == "moments":
            n_post = n_samples * sample_interval
            su, su2 = (sums[0], sums[1]) if on_dev else (sums_host[0].numpy(), sums_host[1].numpy())
            res = {"sum_u": su, "sum_u2": su2, "n": n_post}
            if single:
                res = {"sum_u": res["sum_u"][0], "sum_u2": res["sum_u2"][0], "n": n_post}
            return res
        last = U.to(torch.float64, copy=True) if on_dev else np.array(u_np, dtype=np.float64)
        return last[0] if single else last

    def checkpoint(self):
        """ChainState of the last run (save with chainio.save_state; pass it as
        run()'s u_0 to continue the chains exactly)."""
        if self.state is None:
            raise ValueError("No run yet!")
        return self.state

    def _step(self, u, rng):
        """sampler.py:35-41, one host step (API compatibility; not the hot path)."""
        v = self.proposer(u, rng)
        if self.accepter(u, v, rng):
            return v
        return u

    @classmethod
    def autocorr(cls, x):
        """Normalised autocorrelation of a 1-D chain (sampler.py:43-54), all
        len(x) lags, by the ipmc_autocorr kernel (diagnostics.autocorr; ones
        for a constant chain, as the reference)."""
        from .diagnostics import autocorr

        return autocorr(np.asarray(x, dtype=np.float64).reshape(-1))


def _check_resume(state, chain_offset, accept_kind):
    """A ChainState continues exactly only on the same Philox streams (global
    chain ids) and the same accept potential (Φ for pCNAccepter, I = Φ + the
    regularizer for StandardRWAccepter); anything else is an error.  States
    saved before these fields existed carry None and are not checked; states
    of the generic host tier ("generic") cache no potential, and the resuming
    run recomputes it."""
    if state.chain_offset is not None and state.chain_offset != chain_offset:
        raise ValueError(
            f"ChainState was saved with chain_offset={state.chain_offset}, the sampler has {chain_offset}: "
            "the chains would continue on other Philox streams"
        )
    if state.accept_kind not in (None, "generic") and accept_kind != "generic" and state.accept_kind != accept_kind:
        raise ValueError(
            f"ChainState caches the {state.accept_kind!r} accept potential, this sampler accepts on "
            f"{accept_kind!r} (pcn = pCNAccepter's Φ, rw_reg = StandardRWAccepter's Φ + regularizer)"
        )


# page-locked host buffers up to this size; larger sample arrays use pageable
# memory (or stream to disk with run(sample_file=...))
PINNED_MAX_BYTES = 8 << 30
# in-memory sample arrays of at least this many bytes are copied to the host in
# OVERLAP_COPY_BLOCKS blocks of samples while the sweeps run (MCMCSampler.run)
OVERLAP_COPY_MIN_BYTES = 64 << 20
OVERLAP_COPY_BLOCKS = 8


class _StreamingWriter:
    """Double-buffered sample streaming for run(sample_file=...): while the
    sweeps fill one device staging buffer, the previous one goes to page-locked
    host memory on a copy stream and from there to the .npy file, so the GPU
    does not wait for PCIe or the disk (one buffer when everything fits in it)."""

    def __init__(self, sink, shape, dtype, device, n_buf, single):
        self.sink, self.single, self.device = sink, single, device
        self.dev = [torch.empty(shape, dtype=dtype, device=device) for _ in range(n_buf)]
        nbytes = torch.empty((), dtype=dtype).element_size()
        for d in shape:
            nbytes *= int(d)
        pin = nbytes <= PINNED_MAX_BYTES
        self.host = [torch.empty(shape, dtype=dtype, pin_memory=pin) for _ in range(n_buf)]
        self.done = [None] * n_buf  # D2H of buffer b finished
        self.pending = []  # (b, first sample index, samples) copied or in flight, not yet written
        self.copy_stream = torch.cuda.Stream(device=device)
        self.cur = 0

    @property
    def buffer(self):
        return self.dev[self.cur]

    def flush(self, i0, nb):
        """The current buffer holds samples i0 .. i0+nb-1: start its copy to the
        host, write the block before it to the file, and return the buffer the
        next sweeps write into."""
        b = self.cur
        filled = torch.cuda.Event()
        filled.record(torch.cuda.current_stream(self.device))
        self.copy_stream.wait_event(filled)
        with torch.cuda.stream(self.copy_stream):
            self.host[b][:, :nb].copy_(self.dev[b][:, :nb], non_blocking=True)
            self.done[b] = torch.cuda.Event()
            self.done[b].record(self.copy_stream)
        self.pending.append((b, i0, nb))
        if len(self.pending) == len(self.dev):
            self._write_oldest()
        self.cur = (b + 1) % len(self.dev)
        if self.done[self.cur] is not None:
            # the sweeps must not overwrite a buffer its D2H is still reading
            torch.cuda.current_stream(self.device).wait_event(self.done[self.cur])
        return self.dev[self.cur]

    def _write_oldest(self):
        b, i0, nb = self.pending.pop(0)
        self.done[b].synchronize()
        blk = self.host[b][:, :nb].numpy()
        self.sink.write(i0, blk[0] if self.single else blk)

    def finish(self):
        while self.pending:
            self._write_oldest()


def _pinned_copy(t):
    """An asynchronous copy of device tensor t into page-locked host memory
    (torch's caching host allocator recycles the block); read it after the
    stream is synchronised."""
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.numel() * t.element_size() <= PINNED_MAX_BYTES)
    h.copy_(t, non_blocking=True)
    return h


def _host_buffer(shape):
    n = 8
    for d in shape:
        n *= int(d)
    return torch.empty(shape, dtype=torch.float64, pin_memory=n <= PINNED_MAX_BYTES)


def _bump(counted, calls, accepts, single):
    if single:
        counted.calls = int(np.asarray(counted.calls).sum()) + int(calls[0])
        counted.accepts = int(np.asarray(counted.accepts).sum()) + int(accepts[0])
        return
    c0 = np.asarray(counted.calls)
    a0 = np.asarray(counted.accepts)
    counted.calls = (c0 if c0.shape == calls.shape else 0) + calls
    counted.accepts = (a0 if a0.shape == accepts.shape else 0) + accepts
