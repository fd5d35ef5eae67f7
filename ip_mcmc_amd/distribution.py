"""Probability distributions — mirror of ``ip_mcmc/distribution.py``.

``GaussianDistribution`` keeps the reference's constructor and methods
(distribution.py:90-146): ``sample``, ``__call__``, ``logpdf``,
``apply_covariance``, ``apply_sqrt_covariance``, ``apply_precision``,
``apply_sqrt_precision`` and the attribute ``k``.  Those are host-side helpers
(problem setup and tests); the sampler's hot path reads only
``covariance_diagonal`` / ``sqrt_diagonal`` and evaluates everything on the GPU.

Deliberate difference: the reference's
``apply_sqrt_covariance`` multiplies by the raw ``scipy.linalg.cho_factor``
output, whose unused upper triangle still holds the input matrix, so it is
wrong for non-diagonal covariances; here it multiplies by the true lower
Cholesky factor.  Both agree for diagonal covariances (every script's case).
"""
from abc import ABC, abstractmethod

import numpy as np

from .rng import PhiloxRNG


def _as_array(x, ndim=1):
    """distribution.py:136-146: scalars become 1-element arrays of ``ndim`` dims."""
    if np.isscalar(x):
        return np.array([x], ndmin=ndim, dtype=float)
    if isinstance(x, list):
        x = np.array(x, dtype=float)
    x = np.asarray(x)
    assert len(x.shape) == ndim, f"Dimension error: {len(x.shape)} instead of {ndim}."
    return x


class DistributionBase(ABC):
    """distribution.py:8-26.  Subclasses define ``k``, the dimension."""

    @abstractmethod
    def sample(self, rng):
        """Return a point sampled from this distribution"""

    @abstractmethod
    def __call__(self, x):
        """Return the value of the distribution at x"""

    @abstractmethod
    def logpdf(self, x):
        """Return the log of value of the distribution at x"""


class GaussianDistribution(DistributionBase):
    """N(mean, covariance) — distribution.py:90-146."""

    def __init__(self, mean=0, covariance=1):
        mean = _as_array(mean, ndim=1).astype(float)
        covariance = _as_array(covariance, ndim=2).astype(float)
        self.k = mean.shape[0]
        assert covariance.shape == (self.k, self.k), "dimension error"
        self.mean = mean
        self.covariance = covariance
        # distribution.py:104 factors C once (scipy cho_factor); a non-SPD
        # covariance fails here as it does there.
        self.L = np.linalg.cholesky(covariance)
        self._logdet = 2.0 * float(np.sum(np.log(np.diag(self.L))))

    def centred(self):
        """N(0, C) sharing this distribution's covariance and its factor L (no
        second factorization, and its diagonal test decided once for both)."""
        self.is_diagonal  # noqa: B018 -- cached on self, so the copy carries it
        w = object.__new__(type(self))
        w.__dict__.update(self.__dict__)
        w.mean = np.zeros_like(self.mean)
        return w

    # ---------------------------------------------------------------- shape
    @property
    def is_diagonal(self):
        # decided once, like the factor L above (every run() asks, three times)
        if getattr(self, "_diag_of", None) is not self.covariance:
            c = self.covariance
            self._is_diag, self._diag_of = bool(np.all(c == np.diag(np.diag(c)))), c
        return self._is_diag

    @property
    def covariance_diagonal(self):
        return np.diag(self.covariance).copy()

    @property
    def sqrt_diagonal(self):
        """sqrt(C_ii) — the proposal scale of the device path (diagonal C only)."""
        if not self.is_diagonal:
            raise ValueError("sqrt_diagonal needs a diagonal covariance")
        return np.sqrt(np.diag(self.covariance))

    def log_normaliser(self):
        """½ (k log 2π + log det C): the constant in −logpdf that Φ drops."""
        return 0.5 * (self.k * np.log(2.0 * np.pi) + self._logdet)

    # ---------------------------------------------------------- densities
    def logpdf(self, x):
        """log N(x; mean, C) with scipy's shape rules: a point of shape (k,)
        (a scalar when k = 1) gives a float, a stack (n, k) gives (n,)."""
        x = np.asarray(x, dtype=float)
        if self.k == 1:
            pts = x.reshape(-1, 1)
            single = x.size == 1 and x.ndim <= 1
        else:
            pts = x.reshape(-1, self.k)
            single = x.ndim == 1
        z = np.linalg.solve(self.L, (pts - self.mean).T)  # L^{-1}(x - m)
        out = -0.5 * np.sum(z * z, axis=0) - self.log_normaliser()
        return float(out[0]) if single else out

    def __call__(self, x):
        return np.exp(self.logpdf(x))

    # ------------------------------------------------------------- sampling
    def sample(self, rng):
        """One draw. ``rng`` is a numpy Generator (the reference's call,
        ``rng.multivariate_normal``, distribution.py:117) or a PhiloxRNG, whose
        draw is mean + L·ξ with ξ the device's counter-based normals."""
        if isinstance(rng, PhiloxRNG):
            xi = rng.host_normals(self.k)
            out = self.mean + self.L @ xi
        else:
            out = rng.multivariate_normal(mean=self.mean, cov=self.covariance)
        return out

    # ------------------------------------------------------------ operators
    def apply_covariance(self, x):
        return self.covariance @ _as_array(x)

    def apply_sqrt_covariance(self, x):
        return self.L @ _as_array(x)

    def apply_precision(self, x):
        x = _as_array(x)
        return np.linalg.solve(self.L.T, np.linalg.solve(self.L, x))

    def apply_sqrt_precision(self, x):
        return np.linalg.solve(self.L.T, _as_array(x))
