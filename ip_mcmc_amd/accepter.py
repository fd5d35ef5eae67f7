"""Accepters — mirror of ``ip_mcmc/accepter.py`` (the pCN part).

The sampler's device path fuses ``pCNAccepter`` (exp(Φ(u) − Φ(v)) > r,
accepter.py:62,121-122), ``CountedAccepter`` (per-chain counters,
accepter.py:13-36) and ``ConstrainAccepter`` with a ``BoxConstraint``
(accepter.py:39-55) into the sweep kernel.  The ``__call__`` methods keep the
reference's one-step host signature for API compatibility.
"""
from abc import ABC, abstractmethod

import numpy as np


class AccepterBase(ABC):
    """accepter.py:6-10."""

    @abstractmethod
    def __call__(self, u, v, rng):
        """Return True if v is accepted"""


class CountedAccepter(AccepterBase):
    """accepter.py:13-36.  With many chains ``accepts`` (and ``calls`` under a
    ConstrainAccepter) are per-chain integer arrays and ``ratio()`` returns the
    per-chain ratios; for one chain they are ints and a float, as in the
    reference."""

    def __init__(self, accepter):
        self.accepter = accepter
        self.calls = 0
        self.accepts = 0

    def __call__(self, u, v, rng):
        accepted = self.accepter(u, v, rng)
        self.calls += 1
        if accepted:
            self.accepts += 1
        return accepted

    def reset(self):
        self.calls = 0
        self.accepts = 0

    def ratio(self):
        if np.all(np.asarray(self.calls) == 0):
            raise ValueError("No samples yet!")
        return np.asarray(self.accepts) / np.asarray(self.calls) if np.ndim(self.accepts) else self.accepts / self.calls


class BoxConstraint:
    """A device-expressible constraint: valid iff lower < v + offset < upper
    componentwise (strict, like is_valid_IC, burgers_wasserstein_chain.py:47-55).
    None bounds are ±inf."""

    def __init__(self, lower=None, upper=None, offset=None):
        self.lower = None if lower is None else np.asarray(lower, dtype=np.float64)
        self.upper = None if upper is None else np.asarray(upper, dtype=np.float64)
        self.offset = None if offset is None else np.asarray(offset, dtype=np.float64)

    def arrays(self, k):
        lo = None if self.lower is None else np.broadcast_to(self.lower, (k,)).copy()
        hi = None if self.upper is None else np.broadcast_to(self.upper, (k,)).copy()
        off = None if self.offset is None else np.broadcast_to(self.offset, (k,)).copy()
        return lo, hi, off

    def __call__(self, v):
        v = np.asarray(v, dtype=np.float64)
        t = v + (0.0 if self.offset is None else self.offset)
        ok = np.ones(t.shape[:-1] if t.ndim > 1 else (), dtype=bool)
        if self.lower is not None:
            ok = ok & np.all(self.lower < t, axis=-1)
        if self.upper is not None:
            ok = ok & np.all(t < self.upper, axis=-1)
        return bool(ok) if np.ndim(ok) == 0 else ok


class ConstrainAccepter(AccepterBase):
    """accepter.py:39-55: reject v without consulting the inner accepter (and
    without drawing its uniform) when ``constraint(v)`` is False.  The device
    path needs a BoxConstraint."""

    def __init__(self, accepter, constraint):
        self.accepter = accepter
        self.is_valid = constraint

    def __call__(self, u, v, rng):
        if self.is_valid(v):
            return self.accepter(u, v, rng)
        return False


class ProbabilisticAccepter(AccepterBase):
    """accepter.py:58-66: accept iff a(u, v) > rng.random() (strict)."""

    def __call__(self, u, v, rng):
        a = self.accept_probability(u, v)
        return a > rng.random()

    @abstractmethod
    def accept_probability(self, u, v):
        ...


class StandardRWAccepter(ProbabilisticAccepter):
    """accepter.py:86-106: a(u, v) = exp(I(u) − I(v)),
    I(w) = Φ(w) + ½‖prior.apply_sqrt_covariance(w)‖².

    The reference applies the sqrt COVARIANCE where its docstring says
    C^{-1/2} (accepter_test.py:29-30 pins that value);
    this keeps the reference's behaviour.  On the device the regularizer is
    ½ Σ_i (sqrt(C_ii) w_i)² (diagonal prior)."""

    def __init__(self, potential, prior):
        self.theta = potential
        self.prior = prior

    def accept_probability(self, u, v):
        Iu = self._I(u)
        Iv = self._I(v)
        return np.exp(Iu - Iv)

    def _I(self, w):
        regularizer = 0.5 * np.linalg.norm(self.prior.apply_sqrt_covariance(w)) ** 2
        return self.theta(w) + regularizer


class pCNAccepter(ProbabilisticAccepter):
    """accepter.py:109-122: a(u, v) = exp(Φ(u) − Φ(v)) (Cotter et al. eq. 4.11)."""

    def __init__(self, potential):
        self.theta = potential

    def accept_probability(self, u, v):
        return np.exp(self.theta(u) - self.theta(v))
