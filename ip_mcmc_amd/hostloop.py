"""Host-side pCN loop for compositions the fused kernels cannot run.

The reference's plugin API takes any Python callable as the forward map
(``EvolutionPotential(G, data, noise)``, potential.py:48-54; config 1's caller
passes the closure ``G(u) = np.dot(g, u)``, stuart_examples.py:69-70), any
predicate as a constraint (``ConstrainAccepter``, accepter.py:39-55), any
Gaussian noise model and any proposer/accepter implementing its ABCs.  The
fused sweep kernels run a fixed set of device forward maps; for everything else
``MCMCSampler.run`` comes here.  This is not a CPU fallback for device
compositions (those always take the kernels): it is the one place a caller's
Python code has to run, and the GPU still supplies the randomness.

Two tiers:

* **Structured** (vectorised over the chains): a pCN / RW proposer with any
  prior covariance, ``CountedAccepter`` / ``ConstrainAccepter`` layers in any
  order, ``pCNAccepter`` or ``StandardRWAccepter`` (any prior), over an
  ``EvolutionPotential`` with any G and any ``GaussianDistribution`` noise, or
  over any other potential object.  Per block of steps one
  ``ipmc_pcn_draws`` launch produces the proposal noise ``w`` (the sweep
  kernels' own operations: ``sqrt(C_ii)·ξ_i`` or ``Σ_{i<=j} L_ji ξ_i``) and
  ``log r`` (the kernels' deterministic log); the host forms
  ``v = contraction·u + β·w`` (``u + β·w`` for RW) in the chain dtype,
  evaluates the constraints and G, and accepts iff ``(double)(Φu − Φv) > log r``
  -- the kernels' sequence of operations.  For a diagonal noise Φ is
  ``½ Σ_i ((y_i − m_i − g_i)·γ_i⁻¹)²`` summed in component order without FMA,
  so a device-expressible G run through this loop gives the fused kernel's
  bits in REFERENCE arith.  A device ``ObservationOperator`` is evaluated in
  one ``ipmc_forward`` launch per step for all chains; a Python G is called
  once per chain and step, as the reference calls it.
* **Generic** (any other proposer or accepter, e.g. a user subclass of
  ``ProposerBase`` / ``AccepterBase``): the reference's own ``_step``
  (sampler.py:35-41) per chain, with an rng whose ``multivariate_normal`` and
  ``random`` return the same counter-based draws (the reference's MockRNG seam,
  test_utilities.py:11-26).
"""
import numpy as np
import torch

from . import device as dev
from ._lib import call
from .accepter import ConstrainAccepter, CountedAccepter, StandardRWAccepter, pCNAccepter
from .chainio import ChainState, NpySampleSink
from .distribution import GaussianDistribution
from .forward import ObservationOperator
from .potential import EvolutionPotential

# bytes of draws (w) fetched from the device per block of steps
DRAW_BLOCK_BYTES = 64 << 20


# ------------------------------------------------------------------ draws
def device_draws(seed, chain_offset, n_chains, step0, n_steps, k, np_dtype, prior_sqrt, prior_chol, device=None):
    """(w [n_steps, C, k] in np_dtype, log r [n_steps, C] float64) from
    ipmc_pcn_draws on `device`."""
    device = dev.resolve_device(device)
    td = dev.torch_dtype(np_dtype)
    sq = None if prior_sqrt is None else dev.to_device(prior_sqrt, td, device)
    ch = None if prior_chol is None else dev.to_device(prior_chol, td, device)
    w = torch.empty((n_steps, n_chains, k), dtype=td, device=device)
    lr = torch.empty((n_steps, n_chains), dtype=torch.float64, device=device)
    call("ipmc_pcn_draws", seed, chain_offset, n_chains, step0, n_steps, k, dev.abi_dtype(td), dev.ptr(sq),
         dev.ptr(ch), w.data_ptr(), lr.data_ptr(), dev.stream_handle(device))
    return w.cpu().numpy(), lr.cpu().numpy()


def device_raw_draws(seed, chain_offset, n_chains, step0, n_steps, k, device=None):
    """(ξ [n_steps, C, k], r [n_steps, C]) float64: ipmc_normal / ipmc_uniform on `device`."""
    device = dev.resolve_device(device)
    xi = torch.empty((n_steps, n_chains, k), dtype=torch.float64, device=device)
    r = torch.empty((n_steps, n_chains), dtype=torch.float64, device=device)
    st = dev.stream_handle(device)
    for s in range(n_steps):
        call("ipmc_normal", seed, chain_offset, n_chains, step0 + s, k, dev.abi_dtype(torch.float64),
             xi[s].data_ptr(), st)
        call("ipmc_uniform", seed, chain_offset, n_chains, step0 + s, r[s].data_ptr(), st)
    return xi.cpu().numpy(), r.cpu().numpy()


def host_draws(seed, chain_offset, n_chains, step0, n_steps, k, np_dtype, prior_sqrt, prior_chol, device=None):
    """The same (w, log r) from libipmc_host.so (ipmc_host_pcn_draws): the
    kernels' draw arithmetic compiled for the host CPU (csrc/ipmc_rng.hpp)."""
    from . import _hostlib

    return _hostlib.pcn_draws(seed, chain_offset, n_chains, step0, n_steps, k, np_dtype, prior_sqrt, prior_chol)


def host_raw_draws(seed, chain_offset, n_chains, step0, n_steps, k, device=None):
    """The same (ξ, r) from libipmc_host.so (ipmc_host_normal / ipmc_host_uniform)."""
    from . import _hostlib

    xi = np.empty((n_steps, n_chains, k), dtype=np.float64)
    r = np.empty((n_steps, n_chains), dtype=np.float64)
    for s in range(n_steps):
        xi[s] = _hostlib.normals(seed, chain_offset, n_chains, step0 + s, k)
        r[s] = _hostlib.uniforms(seed, chain_offset, n_chains, step0 + s)
    return xi, r


# Where the host step's draws come from: "device" (ipmc_pcn_draws on the GPU),
# "host" (libipmc_host.so, the same bits on the CPU) or "auto" (the GPU when
# torch sees one, else the host library -- BASELINE config 1 on a machine
# without a GPU).
DRAW_SOURCE = "auto"


def draw_source():
    if DRAW_SOURCE != "auto":
        return DRAW_SOURCE
    return "device" if torch.cuda.is_available() else "host"


def _auto_w(*a, **kw):
    return (device_draws if draw_source() == "device" else host_draws)(*a, **kw)


def _auto_raw(*a, **kw):
    return (device_raw_draws if draw_source() == "device" else host_raw_draws)(*a, **kw)


# the providers the loop uses (tests may substitute others)
DRAWS = {"w": _auto_w, "raw": _auto_raw}
# run_structured's one-chain f64 loop on Python floats (tests switch it off to
# compare it with the array loop)
SINGLE_CHAIN_FLOATS = True


class GenericComposition(Exception):
    """The composition is not in the structured tier's vocabulary."""


# ------------------------------------------------------------- structured
class HostPlan:
    """The structured tier's reading of a proposer/accepter composition."""

    def __init__(self, proposer, accepter, k):
        kind = getattr(proposer, "kind", None)
        prior = getattr(proposer, "w", None)
        if kind not in ("pcn", "rw") or not isinstance(prior, GaussianDistribution):
            raise GenericComposition(type(proposer).__name__)
        if prior.k != k:
            raise ValueError(f"prior dimension {prior.k} != state dimension {k}")
        self.proposer = proposer
        self.rw = kind == "rw"
        if prior.is_diagonal:
            self.prior_sqrt, self.prior_chol = prior.sqrt_diagonal, None
        else:
            self.prior_sqrt, self.prior_chol = None, prior.L
        self.layers = []  # ("count", CountedAccepter) | ("constrain", predicate), outermost first
        acc = accepter
        while True:
            if isinstance(acc, CountedAccepter):
                self.layers.append(("count", acc))
                acc = acc.accepter
            elif isinstance(acc, ConstrainAccepter):
                self.layers.append(("constrain", acc.is_valid))
                acc = acc.accepter
            elif isinstance(acc, pCNAccepter):
                self.reg_prior = None
                break
            elif isinstance(acc, StandardRWAccepter):
                self.reg_prior = acc.prior
                break
            else:
                raise GenericComposition(type(acc).__name__)
        self.potential = acc.theta
        self.accept_kind = "pcn" if self.reg_prior is None else "rw_reg"


class _Misfit:
    """Φ for a stack of proposals, in the chain dtype T."""

    def __init__(self, potential, T, device):
        self.T, self.device = T, device
        self.pot = potential
        self.G = None
        if isinstance(potential, EvolutionPotential) and isinstance(potential.rho, GaussianDistribution):
            rho = potential.rho
            self.G = potential.G
            y_eff = np.atleast_1d(np.asarray(potential.y, dtype=np.float64)) - rho.mean
            if rho.k != y_eff.shape[0]:
                raise ValueError(f"data dimension {y_eff.shape[0]} != noise dimension {rho.k}")
            self.diag = rho.is_diagonal
            if self.diag:
                # the kernels' misfit terms: y - m and 1/γ rounded to T
                self.y_eff = y_eff.astype(T)
                self.ginv = (1.0 / np.sqrt(rho.covariance_diagonal)).astype(T)
            else:
                self.y_eff64 = y_eff
                self.Lg = rho.L

    def forward(self, V):
        """G for the rows of V (n, k) -> (n, q)."""
        G = self.G
        if isinstance(G, ObservationOperator):
            td = dev.torch_dtype(self.T)
            g = G.forward_device(dev.to_device(V, td, dev.resolve_device(self.device)), td)
            return g.cpu().numpy()
        rows = [np.atleast_1d(np.asarray(G(v), dtype=np.float64)).reshape(-1) for v in V.astype(np.float64)]
        return np.stack(rows) if rows else np.zeros((0, 0))

    def __call__(self, V):
        T = self.T
        n = V.shape[0]
        if n == 0:
            return np.zeros(0, dtype=T)
        if self.G is None:  # any potential object: its own value (constant included)
            return np.array([float(self.pot(v)) for v in V.astype(np.float64)], dtype=np.float64).astype(T)
        g = self.forward(V)
        q = self.y_eff.shape[0] if self.diag else self.y_eff64.shape[0]
        if g.ndim != 2 or g.shape[1] != q:
            raise ValueError(f"the forward map returned {g.shape[1:] if g.ndim == 2 else g.shape} values per "
                             f"parameter vector, the data have {q}")
        if self.diag:
            r = (self.y_eff[None, :] - g.astype(T)) * self.ginv[None, :]
            s = np.zeros(n, dtype=T)
            for i in range(r.shape[1]):  # component order, no FMA (REFERENCE arith's sum)
                s = s + r[:, i] * r[:, i]
            return T(0.5) * s
        # dense noise Γ = L Lᵀ: ½‖L⁻¹(y − m − G)‖² (−logpdf without its constant)
        from scipy.linalg import solve_triangular

        z = solve_triangular(self.Lg, (self.y_eff64[None, :] - g.astype(np.float64)).T, lower=True)
        return (0.5 * np.sum(z * z, axis=0)).astype(T)


def _regularizer(prior, V, T):
    """StandardRWAccepter's ½‖prior.apply_sqrt_covariance(v)‖² (accepter.py:104-106,
    Q6): diagonal prior in the kernels' order, else through the Cholesky factor."""
    if prior.is_diagonal:
        c = prior.sqrt_diagonal.astype(T)
        s = np.zeros(V.shape[0], dtype=T)
        for j in range(V.shape[1]):
            t = c[j] * V[:, j]
            s = s + t * t
        return T(0.5) * s
    t = V.astype(np.float64) @ prior.L.T
    return (0.5 * np.sum(t * t, axis=1)).astype(T)


class _Recorder:
    """Samples / moments / last state of a host run, like the device path's outputs."""

    def __init__(self, keep, n_chains, n_samples, k, single, sample_file):
        self.keep, self.single = keep, single
        self.sink = None
        self.samples = None
        if keep == "samples":
            if sample_file is not None:
                self.sink = NpySampleSink(sample_file, (n_samples, k) if single else (n_chains, n_samples, k))
            else:
                self.samples = np.empty((n_chains, n_samples, k), dtype=np.float64)
        self.sum_u = self.sum_u2 = None
        if keep == "moments":
            self.sum_u = np.zeros((n_chains, k), dtype=np.float64)
            self.sum_u2 = np.zeros((n_chains, k), dtype=np.float64)

    def record(self, i, u):
        ud = u.astype(np.float64)
        if self.sink is not None:
            self.sink.write(i, ud[0][None, :] if self.single else ud[:, None, :])
        elif self.samples is not None:
            self.samples[:, i, :] = ud

    def accumulate(self, u):
        if self.sum_u is not None:
            ud = u.astype(np.float64)
            self.sum_u += ud
            self.sum_u2 += ud * ud


def _schedule(plan, i0, n, T):
    """(beta, contraction) of proposals i0+1 .. i0+n as T, per step."""
    p = plan.proposer
    if hasattr(p, "device_step"):
        b, c = p.device_step()
        return np.full(n, b, dtype=np.float64).astype(T), np.full(n, c, dtype=np.float64).astype(T)
    sched = p.beta_schedule(i0, n)
    return sched[:, 0].astype(T), sched[:, 1].astype(T)


def _announce(verbose, done_steps, n_burn, interval, n_samples):
    """sampler.py:24's per-sample print, before the block of sample i."""
    if verbose and done_steps >= n_burn and (done_steps - n_burn) % interval == 0:
        i = (done_steps - n_burn) // interval
        if i < n_samples:
            print(f"Sampling {i + 1}/{n_samples}")


def run_structured(plan, U, phi, seed, chain_offset, step, prop_i, n_burn, n_samples, interval, rec, device,
                   verbose=False):
    """Advance the chains (U [C, k] and Φ(U) [C], both dtype T, updated in
    place) by n_burn steps, then n_samples blocks of `interval` steps recording
    the state after each block (sampler.py:18-28).  Returns (accepts, calls per
    count layer, steps run)."""
    T = U.dtype.type
    C_, k = U.shape
    misfit = _Misfit(plan.potential, T, device)
    counts = [np.zeros(C_, dtype=np.int64) for lay in plan.layers if lay[0] == "count"]
    acc_total = np.zeros(C_, dtype=np.int64)
    total = n_burn + n_samples * interval
    block = max(1, min(total, DRAW_BLOCK_BYTES // max(1, C_ * k * U.itemsize)))
    done = 0
    post = 0  # post-burn-in steps done
    # one f64 chain, a Python G and a diagonal noise (the reference's own use,
    # e.g. config 1's script): the same operations on Python floats (IEEE
    # doubles, as numpy's), without numpy's per-call overhead on 1-element arrays
    single = (SINGLE_CHAIN_FLOATS and C_ == 1 and T is np.float64 and misfit.G is not None and misfit.diag
              and not isinstance(misfit.G, ObservationOperator)
              and (plan.reg_prior is None or plan.reg_prior.is_diagonal))
    if single:
        ul, ph = U[0].tolist(), float(phi[0])
        yl, gil = misfit.y_eff.tolist(), misfit.ginv.tolist()
        rsl = None if plan.reg_prior is None else plan.reg_prior.sqrt_diagonal.tolist()
    while done < total:
        nb = min(block, total - done)
        w, log_r = DRAWS["w"](seed, chain_offset, C_, step + done, nb, k, T, plan.prior_sqrt, plan.prior_chol,
                              device)
        betas, contrs = _schedule(plan, prop_i + done, nb, T)
        if single:
            wl, lrl, bl, cl = w[:, 0, :].tolist(), log_r[:, 0].tolist(), betas.tolist(), contrs.tolist()
            for s in range(nb):
                _announce(verbose, done + s, n_burn, interval, n_samples)
                b, ws = bl[s], wl[s]
                if plan.rw:
                    v = [ui + b * wi for ui, wi in zip(ul, ws)]
                else:
                    c = cl[s]
                    v = [c * ui + b * wi for ui, wi in zip(ul, ws)]
                reach, ci = True, 0
                for kind, obj in plan.layers:
                    if kind == "count":
                        counts[ci][0] += reach
                        ci += 1
                    elif reach:
                        reach = bool(obj(np.array(v)))
                if reach:
                    gv = misfit.G(np.array(v))
                    if isinstance(gv, (float, np.floating)):  # a scalar observation (config 1's np.dot)
                        g = [float(gv)]
                    else:
                        g = np.atleast_1d(np.asarray(gv, dtype=np.float64)).reshape(-1).tolist()
                    if len(g) != len(yl):
                        raise ValueError(f"the forward map returned {len(g)} values per parameter vector, the data "
                                         f"have {len(yl)}")
                    sm = 0.0
                    for yi, gv, gi in zip(yl, g, gil):  # component order, no FMA
                        r = (yi - gv) * gi
                        sm = sm + r * r
                    phv = 0.5 * sm
                    if rsl is not None:
                        s2 = 0.0
                        for cj, vj in zip(rsl, v):
                            t = cj * vj
                            s2 = s2 + t * t
                        phv = phv + 0.5 * s2
                    if (ph - phv) > lrl[s]:
                        ul, ph = v, phv
                        acc_total[0] += 1
                if done + s >= n_burn:
                    if rec.sum_u is not None:
                        rec.accumulate(np.array([ul]))
                    post += 1
                    if post % interval == 0:
                        rec.record(post // interval - 1, np.array([ul]))
            done += nb
            continue
        for s in range(nb):
            _announce(verbose, done + s, n_burn, interval, n_samples)
            V = U + betas[s] * w[s] if plan.rw else contrs[s] * U + betas[s] * w[s]
            reach = np.ones(C_, dtype=bool)
            reached = []
            for kind, obj in plan.layers:
                if kind == "count":
                    reached.append(reach.copy())
                else:
                    idx = np.flatnonzero(reach)
                    if idx.size:
                        ok = np.array([bool(obj(V[c])) for c in idx], dtype=bool)
                        reach[idx[~ok]] = False
            idx = np.flatnonzero(reach)
            accepted = np.zeros(C_, dtype=bool)
            if idx.size:
                Vi = V[idx]
                phv = misfit(Vi)
                if plan.reg_prior is not None:
                    phv = phv + _regularizer(plan.reg_prior, Vi, T)
                a = (phi[idx] - phv).astype(np.float64) > log_r[s, idx]
                sel = idx[a]
                U[sel] = Vi[a]
                phi[sel] = phv[a]
                accepted[sel] = True
            acc_total += accepted
            for ci, r in enumerate(reached):
                counts[ci] += r
            if done + s >= n_burn:
                rec.accumulate(U)
                post += 1
                if post % interval == 0:
                    rec.record(post // interval - 1, U)
        done += nb
    if single:
        U[0] = ul
        phi[0] = ph
    return acc_total, counts, total


def initial_phi(plan, U, device):
    T = U.dtype.type
    phi = _Misfit(plan.potential, T, device)(U)
    if plan.reg_prior is not None:
        phi = phi + _regularizer(plan.reg_prior, U, T)
    return phi


# ----------------------------------------------------------------- generic
class StepRNG:
    """The rng handed to a caller's proposer/accepter in the generic tier: the
    draws of one (chain, step), like the reference's MockRNG seam
    (test_utilities.py:11-26).

    Normals come from the step's Philox stream in component order through a
    cursor: the first ``multivariate_normal(mean, cov)`` of a step returns
    mean + sqrt(C)·ξ[0:k] (diagonal C) or mean + L·ξ[0:k] in the kernels'
    order -- the structured tier's and the kernels' proposal -- and a second
    draw in the same step continues with ξ[k:2k] (e.g. a product prior that
    samples its components one by one, distribution.py:57-59).  Uniforms
    likewise: the first ``random()`` is the accept uniform r (Philox slot
    0xFFFFFFFF), further ones come from slots 0xFFFFFFFE, 0xFFFFFFFD, ...  Draws
    beyond the pre-drawn block come from libipmc_host.so (the same bits).
    ``standard_normal``, ``normal``, ``uniform`` and ``lognormal`` use the same
    cursors; any other Generator method raises AttributeError."""

    SUPPORTED = ("multivariate_normal", "random", "standard_normal", "normal", "uniform", "lognormal")

    def __init__(self, seed=0):
        self.seed = int(seed)
        self.gid = self.step = 0
        self.xi = np.zeros(0)
        self.r = 0.0
        self._n = self._u = 0

    def set(self, xi, r, gid=0, step=0):
        self.xi, self.r = np.asarray(xi, dtype=np.float64), float(r)
        self.gid, self.step = int(gid), int(step)
        self._n = self._u = 0

    def __getattr__(self, name):
        raise AttributeError(f"the generic tier's rng supports {', '.join(self.SUPPORTED)}; "
                             f"numpy Generator.{name} has no counter-based twin here")

    # ------------------------------------------------------------ cursors
    def _normals(self, m):
        j0, j1 = self._n, self._n + m
        self._n = j1
        if j1 <= self.xi.shape[0]:
            return self.xi[j0:j1].copy()
        from . import _hostlib

        return _hostlib.normals(self.seed, self.gid, 1, self.step, j1)[0, j0:j1]

    def _uniforms(self, m):
        i0, i1 = self._u, self._u + m
        self._u = i1
        out = np.empty(m)
        extra = None
        for i in range(i0, i1):
            if i == 0:
                out[i - i0] = self.r
            else:
                if extra is None:
                    from . import _hostlib

                    extra = _hostlib.extra_uniforms(self.seed, self.gid, self.step, i1)
                out[i - i0] = extra[i]
        return out

    @staticmethod
    def _count(size):
        if size is None:
            return 1
        return int(np.prod(np.atleast_1d(size)))

    @staticmethod
    def _shape(v, size):
        return float(v[0]) if size is None else v.reshape(size)

    # --------------------------------------------------- Generator methods
    def multivariate_normal(self, mean=None, cov=None, size=None):
        mean = np.atleast_1d(np.asarray(mean, dtype=np.float64))
        k = mean.shape[0]
        cov = np.asarray(cov, dtype=np.float64).reshape(k, k)
        diag = bool(np.all(cov == np.diag(np.diag(cov))))
        L = None if diag else np.linalg.cholesky(cov)
        rows = []
        for _ in range(self._count(size)):
            xi = self._normals(k)
            if diag:
                rows.append(np.sqrt(np.diag(cov)) * xi + mean)
                continue
            w = np.zeros(k)
            for j in range(k):
                a = 0.0
                for i in range(j + 1):
                    a = a + float(xi[i]) * float(L[j, i])
                w[j] = a
            rows.append(w + mean)
        if size is None:
            return rows[0]
        return np.stack(rows).reshape(tuple(np.atleast_1d(size)) + (k,))

    def random(self, size=None):
        return self._shape(self._uniforms(self._count(size)), size)

    def standard_normal(self, size=None):
        return self._shape(self._normals(self._count(size)), size)

    def normal(self, loc=0.0, scale=1.0, size=None):
        return self._shape(loc + scale * self._normals(self._count(size)), size)

    def uniform(self, low=0.0, high=1.0, size=None):
        return self._shape(low + (high - low) * self._uniforms(self._count(size)), size)

    def lognormal(self, mean=0.0, sigma=1.0, size=None):
        return self._shape(np.exp(mean + sigma * self._normals(self._count(size))), size)


def _counted(acc):
    """Every CountedAccepter reachable through .accepter attributes."""
    out = []
    seen = set()
    while acc is not None and id(acc) not in seen:
        seen.add(id(acc))
        if isinstance(acc, CountedAccepter):
            out.append(acc)
        acc = getattr(acc, "accepter", None)
    return out


def run_generic(proposer, accepter, U, seed, chain_offset, step, n_burn, n_samples, interval, rec, device,
                verbose=False):
    """The reference's _step (sampler.py:35-41) per chain with StepRNG draws.
    Returns (CountedAccepters found, their per-chain (calls, accepts), steps
    run, per-chain accept decisions).

    A stateful proposer (a step counter ``i``, like VarStep*, proposer.py:105)
    sees every chain's call of one step with the counter the step starts with,
    and advances once per step, as one chain of the reference would."""
    C_, k = U.shape
    total = n_burn + n_samples * interval
    counted = _counted(accepter)
    per = {id(ca): (np.zeros(C_, dtype=np.int64), np.zeros(C_, dtype=np.int64)) for ca in counted}
    decided = np.zeros(C_, dtype=np.int64)
    rng = StepRNG(seed)
    stateful = hasattr(proposer, "i")
    block = max(1, min(total, DRAW_BLOCK_BYTES // max(1, C_ * k * 8)))
    u_rows = [np.asarray(U[c], dtype=np.float64).copy() for c in range(C_)]
    done = 0
    post = 0
    while done < total:
        nb = min(block, total - done)
        xi, r = DRAWS["raw"](seed, chain_offset, C_, step + done, nb, k, device)
        for s in range(nb):
            _announce(verbose, done + s, n_burn, interval, n_samples)
            i_step = proposer.i if stateful else None
            i_next = i_step
            for c in range(C_):
                before = [(ca.calls, ca.accepts) for ca in counted]
                rng.set(xi[s, c], r[s, c], chain_offset + c, step + done + s)
                if stateful:
                    proposer.i = i_step
                v = proposer(u_rows[c], rng)
                if stateful:
                    i_next = proposer.i
                if accepter(u_rows[c], v, rng):
                    u_rows[c] = np.asarray(v, dtype=np.float64)
                    decided[c] += 1
                for ca, (c0, a0) in zip(counted, before):
                    per[id(ca)][0][c] += int(np.sum(ca.calls)) - int(np.sum(c0))
                    per[id(ca)][1][c] += int(np.sum(ca.accepts)) - int(np.sum(a0))
            if stateful:
                proposer.i = i_next
            if done + s >= n_burn:
                Ucur = np.stack(u_rows)
                rec.accumulate(Ucur)
                post += 1
                if post % interval == 0:
                    rec.record(post // interval - 1, Ucur)
        done += nb
    U[:] = np.stack(u_rows).astype(U.dtype) if C_ else U
    return counted, per, total, decided


# --------------------------------------------------------------------- run
def run(sampler, u_0, n_samples, burn_in, sample_interval, keep, sample_file, reason):
    """MCMCSampler.run for a composition outside the fused kernels' set."""
    from .rng import PhiloxRNG, resolve_rng
    from .sampler import _bump, _check_resume

    if keep not in ("samples", "moments", "last"):
        raise ValueError("keep must be 'samples', 'moments' or 'last'")
    T = np.float64 if dev.torch_dtype(sampler.dtype) == dev.F64 else np.float32
    device = sampler.device  # resolved where a device call needs it (draws, a device G)
    resume = isinstance(u_0, ChainState)
    if resume:
        single = False
        U = np.array(u_0.u, dtype=T)
    else:
        if isinstance(u_0, torch.Tensor):
            u_0 = u_0.detach().cpu().numpy()
        arr = np.asarray(u_0, dtype=np.float64)
        single = arr.ndim <= 1
        U = np.atleast_2d(arr).astype(T).copy()
        if arr.ndim == 0:
            U = U.reshape(1, 1)
    n_chains, k = U.shape
    n_samples, sample_interval = int(n_samples), int(sample_interval)
    if n_samples < 0 or sample_interval < 0:
        raise ValueError("n_samples and sample_interval must be >= 0")
    if not isinstance(sampler.rng, PhiloxRNG):
        sampler.rng = resolve_rng(sampler.rng)
    rng = sampler.rng
    try:
        plan = HostPlan(sampler.proposer, sampler.accepter, k)
    except GenericComposition:
        plan = None
    # a generic run caches no accept potential (its Φ is NaN): "generic" tells a
    # later structured or device run to recompute Φ(u) instead of reusing it
    accept_kind = "generic" if plan is None else plan.accept_kind
    if resume:
        _check_resume(u_0, sampler.chain_offset, accept_kind)
        rng.seed, rng.step = u_0.seed, u_0.step
        if hasattr(sampler.proposer, "i"):
            sampler.proposer.i = u_0.proposer_i
    if isinstance(sampler.accepter, CountedAccepter):
        sampler.accepter.reset()  # sampler.py:15-16
    n_burn = max(0, burn_in - sample_interval)  # sampler.py:18
    # interval 0 records the same state n_samples times (the reference's loop does)
    eff_interval = sample_interval if sample_interval > 0 else 1
    rec = _Recorder(keep, n_chains, n_samples, k, single, sample_file)
    state_dtype = "float64" if T == np.float64 else "float32"
    prop_i = getattr(sampler.proposer, "i", 0)
    import time

    t0 = time.perf_counter()
    calls_np = None
    # sample_interval 0: burn in, then every sample is the same state (the
    # reference's loop runs no step between its records, sampler.py:23-28)
    n_rec = n_samples if sample_interval > 0 else 0
    if plan is not None:
        if (resume and u_0.dtype == state_dtype and u_0.phi.shape[0] == n_chains
                and u_0.accept_kind != "generic"):
            phi = np.array(u_0.phi, dtype=T)
        else:
            phi = initial_phi(plan, U, device)
        acc_np, counts, total = run_structured(plan, U, phi, rng.seed, sampler.chain_offset, rng.step, prop_i,
                                               n_burn, n_rec, eff_interval, rec, device, sampler.verbose)
        ci = 0
        inner = False
        for kind, obj in plan.layers:
            if kind == "count":
                c = counts[ci]
                ci += 1
                _bump(obj, c, acc_np, single)
                if inner and calls_np is None:
                    calls_np = c
            else:
                inner = True
    else:
        phi = np.full(n_chains, np.nan, dtype=T)
        counted = _counted(sampler.accepter)
        prev = [(ca.calls, ca.accepts) for ca in counted]
        counted, per, total, acc_np = run_generic(sampler.proposer, sampler.accepter, U, rng.seed,
                                                  sampler.chain_offset, rng.step, n_burn, n_rec, eff_interval, rec,
                                                  device, sampler.verbose)
        for ca, (c0, a0) in zip(counted, prev):
            # per-chain arrays for many chains, ints for one (the device path's convention)
            c, a = per[id(ca)]
            ca.calls, ca.accepts = c0, a0
            _bump(ca, c, a, single)
    if sample_interval == 0:
        for i in range(n_samples):
            rec.record(i, U)
    sampler.last_run_seconds = time.perf_counter() - t0
    sampler.last_path = "host" if plan is not None else "host-generic"
    sampler.last_host_reason = reason
    rng.step += total
    prop_i += total
    if hasattr(sampler.proposer, "i"):
        sampler.proposer.i = prop_i
    if sampler.verbose and isinstance(sampler.accepter, CountedAccepter):
        print(f"Acceptance ratio: {sampler.accepter.ratio()}")  # sampler.py:30-31
    prev_acc = u_0.accepts if resume else 0
    prev_calls = u_0.calls if (resume and u_0.calls is not None) else 0
    sampler.state = ChainState(U.copy(), np.asarray(phi).copy(), prev_acc + acc_np,
                               None if calls_np is None else prev_calls + calls_np, rng.seed, rng.step, prop_i,
                               state_dtype, chain_offset=sampler.chain_offset, accept_kind=accept_kind)
    sampler.state.steps_this_run = total
    if keep == "samples":
        if rec.sink is not None:
            return rec.sink.close()
        return rec.samples[0] if single else rec.samples
    if keep == "moments":
        n_post = n_samples * sample_interval
        if single:
            return {"sum_u": rec.sum_u[0], "sum_u2": rec.sum_u2[0], "n": n_post}
        return {"sum_u": rec.sum_u, "sum_u2": rec.sum_u2, "n": n_post}
    last = U.astype(np.float64)
    return last[0] if single else last
