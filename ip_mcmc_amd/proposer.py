"""pCN proposers — mirror of ``ip_mcmc/proposer.py`` (the pCN part).

v = sqrt(1 − β²)·u + β·w,  w ~ N(0, C)   (Cotter et al. 2013 eq. 4.8)

The device path draws w = sqrt(C_ii)·ξ_i from the counter-based stream
(rng.py) inside the sweep kernel; ``__call__`` keeps the reference's
single-step host signature for API compatibility.
"""
from abc import ABC, abstractmethod

import numpy as np

from .distribution import GaussianDistribution



def _centred(prior):
    """N(0, C) of the prior N(m, C), as proposer.py builds its noise
    distribution: the prior's Cholesky factor is reused (a new factorization
    per sampler was ~0.2 ms of every run_sharded call before any GPU work)."""
    if isinstance(prior, GaussianDistribution):
        return prior.centred()
    return GaussianDistribution(mean=np.zeros_like(prior.mean), covariance=prior.covariance)

class ProposerBase(ABC):
    """proposer.py:8-11."""

    @abstractmethod
    def __call__(self, u, rng):
        ...


class ConstStepStandardRWProposer(ProposerBase):
    """proposer.py:14-30: v = u + sqrt(2 delta) w, w ~ N(0, C) (Cotter et al. eq. 4.3)."""

    kind = "rw"

    def __init__(self, delta, prior):
        self.prefactor = np.sqrt(2 * delta)
        self.w = _centred(prior)

    def device_step(self):
        return float(self.prefactor), 1.0

    def beta_schedule(self, i0, n):
        return None

    def __call__(self, u, rng):
        return u + self.prefactor * self.w.sample(rng)


class VarStepStandardRWProposer(ProposerBase):
    """proposer.py:33-56: v = u + sqrt(2) sqrt(delta(i)) w with i counted from 1
    (incremented before use); the sampler passes each launch's step sizes to
    the kernel (ipmc_sweep.beta_schedule)."""

    kind = "rw"

    def __init__(self, delta, prior):
        self.prefactor = np.sqrt(2)
        self.delta = delta
        self.i = 0
        self.w = _centred(prior)

    def beta_schedule(self, i0, n):
        sched = np.empty((n, 2), dtype=np.float64)
        sched[:, 0] = [self.prefactor * np.sqrt(self.delta(i0 + j + 1)) for j in range(n)]
        sched[:, 1] = 1.0
        return sched

    def __call__(self, u, rng):
        self.i += 1
        stepsize = self.prefactor * np.sqrt(self.delta(self.i))
        return u + stepsize * self.w.sample(rng)


class PWLinear:
    """Piecewise-linear step schedule (report/scripts/burgers/burgers_beta.py:131-147):
    delta decreases linearly from start_delta until len_burn_in, then stays end_delta."""

    def __init__(self, start_delta, end_delta, len_burn_in):
        self.d_s = start_delta
        self.d_e = end_delta
        self.l = len_burn_in
        self.slope = (start_delta - end_delta) / len_burn_in

    def __call__(self, i):
        if i > self.l:
            return self.d_e
        return self.d_s - self.slope * i

    def __repr__(self):
        return f"pwl_{self.d_s}_{self.d_e}_{self.l}"


class ConstSteppCNProposer(ProposerBase):
    """proposer.py:59-82.  Only the prior covariance is used; a non-zero prior
    mean is ignored (callers sample perturbations around it, Q1)."""

    kind = "pcn"

    def __init__(self, beta, prior):
        assert 0 <= beta <= 1, "beta has to be in [0,1]"
        self.beta = beta
        self.contraction = np.sqrt(1 - beta**2)  # proposer.py:77
        self.w = _centred(prior)

    def device_step(self):
        return float(self.beta), float(self.contraction)

    def beta_schedule(self, i0, n):
        """(beta, contraction) for proposals i0+1 .. i0+n (constant here)."""
        return None

    def __call__(self, u, rng):
        return self.contraction * u + self.beta * self.w.sample(rng)


class VarSteppCNProposer(ProposerBase):
    """proposer.py:85-115: beta(i) for the i-th proposal, i counted from 1
    (incremented before use, :111-112).  The sampler passes the schedule of
    each launch to the kernel (ipmc_sweep.beta_schedule)."""

    kind = "pcn"

    def __init__(self, beta, prior):
        self.beta = beta
        self.i = 0
        self.w = _centred(prior)

    def beta_schedule(self, i0, n):
        b = np.array([float(self.beta(i0 + j + 1)) for j in range(n)], dtype=np.float64)
        if np.any((b < 0) | (b > 1)):
            raise ValueError("beta(i) has to be in [0,1]")
        sched = np.empty((n, 2), dtype=np.float64)
        sched[:, 0] = b
        sched[:, 1] = np.sqrt(1 - b**2)
        return sched

    def __call__(self, u, rng):
        self.i += 1
        b = self.beta(self.i)
        return np.sqrt(1 - b**2) * u + b * self.w.sample(rng)
