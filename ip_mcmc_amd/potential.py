"""Potentials — mirror of ``ip_mcmc/potential.py``.

``EvolutionPotential(G, data, noise)`` (potential.py:42-57) is the hot-path
potential: Φ(u) = −log ρ(y − G(u)) for Gaussian noise ρ = N(m, Γ).  The device
evaluates Φ_dev(u) = ½‖(y − m − G(u))/γ‖² (diagonal Γ = diag(γ²)); the
Gaussian normalising constant ½(q log 2π + log det Γ) cancels in every
Φ(u) − Φ(v) and is added back only where a caller asks for the reference's
absolute value (``__call__``).
"""
from abc import ABC, abstractmethod

import ctypes as C

import numpy as np
import torch

from . import device as dev
from ._lib import UnsupportedOnDevice, call
from .distribution import GaussianDistribution
from .forward import ObservationOperator


class PotentialBase(ABC):
    """potential.py:6-22: L(u; y) = exp(−Φ(u; y))."""

    @abstractmethod
    def __call__(self, u):
        ...

    @abstractmethod
    def exp_minus_potential(self, u):
        """Return exp(-potential(u))"""


class EvolutionPotential(PotentialBase):
    """Potential of the model data = G(u) + η, η ~ noise (potential.py:42-57)."""

    def __init__(self, observation_operator, data, noise_distribution):
        self.G = observation_operator
        self.y = np.atleast_1d(np.asarray(data, dtype=np.float64))
        self.rho = noise_distribution

    # ------------------------------------------------------------ device form
    def device_terms(self):
        """(y − m, 1/γ) of the diagonal-Gaussian misfit, or raise UnsupportedOnDevice."""
        if not isinstance(self.G, ObservationOperator):
            raise UnsupportedOnDevice(
                "EvolutionPotential: the forward map must be a device ObservationOperator "
                "(LinearOperator, Lorenz63Operator, Lorenz96Operator, BurgersOperator); "
                f"got {type(self.G).__name__}"
            )
        if not isinstance(self.rho, GaussianDistribution):
            raise UnsupportedOnDevice("EvolutionPotential: noise must be a GaussianDistribution on the device")
        if not self.rho.is_diagonal:
            raise UnsupportedOnDevice("EvolutionPotential: noise covariance must be diagonal on the device")
        if self.rho.k != self.G.q or self.y.shape[0] != self.G.q:
            raise ValueError(f"data/noise dimension {self.y.shape[0]}/{self.rho.k} != G's q = {self.G.q}")
        y_eff = self.y - self.rho.mean
        ginv = 1.0 / np.sqrt(self.rho.covariance_diagonal)
        return y_eff, ginv

    def phi_device(self, u, dtype=None):
        """Φ_dev for a device tensor u [n, k] -> [n] (no normalising constant)."""
        td = u.dtype if dtype is None else dtype
        u = u.to(td).contiguous()
        y_eff, ginv = self.device_terms()
        m, _ = self.G.model(td, u.device)
        yt = dev.to_device(y_eff, td, u.device)
        gt = dev.to_device(ginv, td, u.device)
        out = torch.empty((u.shape[0],), dtype=td, device=u.device)
        call(
            "ipmc_potential",
            C.byref(m),
            dev.abi_dtype(td),
            u.shape[0],
            u.data_ptr(),
            yt.data_ptr(),
            gt.data_ptr(),
            out.data_ptr(),
            dev.stream_handle(u.device),
        )
        return out

    # ---------------------------------------------------------- reference form
    def __call__(self, u):
        """−noise.logpdf(y − G(u)) (potential.py:53-54); u (k,) -> float, (n, k) -> (n,).
        A device forward map with diagonal Gaussian noise evaluates on the GPU;
        a Python G or another noise model evaluates as the reference does."""
        try:
            self.device_terms()
        except UnsupportedOnDevice:
            single = np.ndim(u) <= 1
            pts = np.atleast_2d(np.asarray(u, dtype=np.float64))
            vals = np.array([-self.rho.logpdf(self.y - np.atleast_1d(np.asarray(self.G(p), dtype=np.float64)))
                             for p in pts], dtype=np.float64).reshape(-1)
            return float(vals[0]) if single else vals
        single = np.ndim(u) <= 1
        arr = np.asarray(u, dtype=np.float64).reshape(-1, self.G.k)
        t = dev.to_device(arr, dev.F64, dev.resolve_device())
        phi = self.phi_device(t).cpu().numpy() + self.rho.log_normaliser()
        return float(phi[0]) if single else phi

    def exp_minus_potential(self, u):
        """noise.pdf(y − G(u)) (potential.py:56-57)."""
        return np.exp(-self(u))
