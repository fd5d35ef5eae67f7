"""Forward maps G(u) ("observation operators") evaluated on the GPU.

In the reference a forward map is any Python callable handed to
``EvolutionPotential(G, data, noise)`` (potential.py:48-51); the scripts build
them from scipy/numpy integrators (lorenz_mcmc.py:43-71,
burgers/utilities.py:17-41, stuart_examples.py:69-70).  Here each forward map
is a device object: calling it on a parameter vector u of shape (k,) or a stack
(C, k) evaluates G on the GPU through ``ipmc_forward``; the sampler hands the
same description to the fused sweep kernel, so G never leaves the device.

  LinearOperator     G(u) = A (theta0 + u)                       stuart_examples.py:69-70
  Lorenz63Operator   RK4 Lorenz-63, moments time-averaged        (no reference; SURVEY §8(d) cfg 2)
  Lorenz96Operator   RK4 single-scale Lorenz-96 forcing field     lorenz.py:73-88, lorenz_mcmc.py:55-68
  TwoScaleLorenz96Operator  RK4 two-scale L96, 5K moments         lorenz.py:44-101, lorenz_mcmc.py:17-71
  BurgersOperator    Rusanov FV + SSPRK2, windowed trapz          burgers/rusanov.py:6-109, utilities.py:17-109

Every operator takes ``arith='fma'`` (default, fused multiply-adds) or
``arith='reference'`` (no FMA; the reference's operation order, e.g.
lorenz.py:77-81); both are bit-exact against the CPU oracle in the same mode.
"""
import ctypes as C

import numpy as np
import torch

from . import _abi
from . import device as dev
from ._lib import call

_ARITH = {"fma": _abi.ARITH_FMA, "reference": _abi.ARITH_REFERENCE}


class ObservationOperator:
    """Base: subclasses set kind/k/q and fill the model struct."""

    kind = None

    def __init__(self, arith="fma"):
        if arith not in _ARITH:
            raise ValueError(f"arith must be 'fma' or 'reference', not {arith!r}")
        self.arith = arith
        self._cache = {}

    # subclasses: return (fields dict, real arrays dict, int arrays dict)
    def _spec(self):
        raise NotImplementedError

    def model(self, dtype, device):
        """(IpmcModel, keep-alive tensors) for `dtype` on `device` (cached)."""
        key = (dtype, str(device))
        hit = self._cache.get(key)
        if hit is not None:
            return hit
        fields, reals, ints = self._spec()
        m = _abi.IpmcModel()
        m.kind = self.kind
        m.arith = _ARITH[self.arith]
        m.k = self.k
        m.q = self.q
        for name, val in fields.items():
            setattr(m, name, val)
        keep = []
        for name, arr in reals.items():
            t = dev.to_device(arr, dtype, device)
            keep.append(t)
            setattr(m, name, t.data_ptr())
        for name, arr in ints.items():
            t = torch.as_tensor(np.asarray(arr, dtype=np.int32)).to(device).contiguous()
            keep.append(t)
            setattr(m, name, t.data_ptr())
        self._cache[key] = (m, keep)
        return m, keep

    def forward_device(self, u, dtype=None):
        """G for a device tensor u [n, k] -> [n, q] (same dtype)."""
        td = u.dtype if dtype is None else dtype
        u = u.to(td).contiguous()
        m, _ = self.model(td, u.device)
        n = u.shape[0]
        out = torch.empty((n, self.q), dtype=td, device=u.device)
        call("ipmc_forward", C.byref(m), dev.abi_dtype(td), n, u.data_ptr(), out.data_ptr(), dev.stream_handle(u.device))
        return out

    def __call__(self, u, dtype=None, device=None):
        """G(u).  numpy in -> numpy float64 out (computed in float64 unless
        dtype says otherwise); a device tensor in -> a device tensor out."""
        if isinstance(u, torch.Tensor) and u.is_cuda:
            uu = u.reshape(-1, self.k)
            g = self.forward_device(uu, dtype)
            return g.reshape(self.q) if u.dim() == 1 else g
        arr = np.asarray(u, dtype=np.float64)
        single = arr.ndim <= 1
        td = dev.torch_dtype(dtype)
        t = dev.to_device(arr.reshape(-1, self.k), td, dev.resolve_device(device))
        g = self.forward_device(t).double().cpu().numpy()
        if single:
            return float(g[0, 0]) if self.q == 1 and arr.ndim == 0 else g[0]
        return g


class LinearOperator(ObservationOperator):
    """G(u) = A (theta0 + u); A of shape (q, k), or a 1-D g for G(u) = <g, u>
    (stuart_examples.py:69-70)."""

    kind = _abi.MODEL_LINEAR

    def __init__(self, A, theta0=None, arith="fma"):
        super().__init__(arith)
        A = np.asarray(A, dtype=np.float64)
        if A.ndim == 1:
            A = A.reshape(1, -1)
        if A.ndim != 2:
            raise ValueError("A must be (q, k) or (k,)")
        self.A = A
        self.q, self.k = A.shape
        if self.k > 64:
            raise ValueError("LinearOperator supports k <= 64 on the device")
        self.theta0 = np.zeros(self.k) if theta0 is None else np.asarray(theta0, dtype=np.float64).reshape(self.k)

    def _spec(self):
        return {}, {"A": self.A, "theta0": self.theta0}, {}


class Lorenz63Operator(ObservationOperator):
    """Lorenz-63 with (sigma, rho, b) = theta0 + u, classical RK4 (dt, n_steps)
    from x0; G = time averages of (x, y, z, x², y², z²) over the n post-step
    states (the moment-function pattern of lorenz_mcmc.py:17-40)."""

    kind = _abi.MODEL_LORENZ63

    def __init__(self, theta0=(10.0, 28.0, 8.0 / 3.0), x0=(1.0, 1.0, 1.0), dt=0.01, n_steps=500, arith="fma"):
        super().__init__(arith)
        self.k, self.q = 3, 6
        self.theta0 = np.asarray(theta0, dtype=np.float64).reshape(3)
        self.x0 = np.asarray(x0, dtype=np.float64).reshape(3)
        self.dt = float(dt)
        self.n_steps = int(n_steps)

    def _spec(self):
        return (
            {"dim": 3, "n_steps": self.n_steps, "dt": self.dt},
            {"theta0": self.theta0, "x0": self.x0},
            {},
        )

    @staticmethod
    def spinup(theta=(10.0, 28.0, 8.0 / 3.0), x0=(1.0, 1.0, 1.0), dt=0.01, n_steps=1000):
        """RK4 spin-up on the host (problem setup only): returns the end state."""
        s, r, b = theta

        def f(x):
            return np.array([s * (x[1] - x[0]), x[0] * (r - x[2]) - x[1], x[0] * x[1] - b * x[2]])

        x = np.asarray(x0, dtype=np.float64).copy()
        for _ in range(n_steps):
            k1 = f(x)
            k2 = f(x + 0.5 * dt * k1)
            k3 = f(x + 0.5 * dt * k2)
            k4 = f(x + dt * k3)
            x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        return x


class Lorenz96Operator(ObservationOperator):
    """Single-scale Lorenz-96 (lorenz.py:73-88, J = 0) with one forcing per slow
    variable: F = forcing_mean + u.  Classical RK4 (dt, n_steps) from the
    shared initial state x0; G_k = time average of X_k over the n post-step
    states (lorenz_mcmc.py:68's time average, uniform steps).

    Unlike LorenzObservationOperator (lorenz_mcmc.py:66), G is stateless: every
    evaluation starts from x0."""

    kind = _abi.MODEL_LORENZ96

    def __init__(self, K=40, forcing_mean=8.0, x0=None, dt=0.005, n_steps=2000, arith="fma"):
        super().__init__(arith)
        self.K = int(K)
        self.k = self.q = self.K
        fm = np.asarray(forcing_mean, dtype=np.float64)
        self.theta0 = np.full(self.K, float(fm)) if fm.ndim == 0 else fm.reshape(self.K)
        if x0 is None:
            x0 = self.spinup(self.K, self.theta0, dt=dt, n_steps=1000)
        self.x0 = np.asarray(x0, dtype=np.float64).reshape(self.K)
        self.dt = float(dt)
        self.n_steps = int(n_steps)

    def _spec(self):
        return (
            {"dim": self.K, "n_steps": self.n_steps, "dt": self.dt},
            {"theta0": self.theta0, "x0": self.x0},
            {},
        )

    @staticmethod
    def rhs(x, F):
        """dX/dt of single-scale Lorenz-96 (host numpy, problem setup)."""
        return (np.roll(x, -1) - np.roll(x, 2)) * np.roll(x, 1) - x + F

    @classmethod
    def spinup(cls, K, F, dt=0.005, n_steps=1000, x_init=None):
        """RK4 spin-up on the host from x = F + 0.01 e_0 (problem setup only)."""
        F = np.broadcast_to(np.asarray(F, dtype=np.float64), (K,))
        x = F.copy() if x_init is None else np.asarray(x_init, dtype=np.float64).copy()
        if x_init is None:
            x[0] += 0.01
        for _ in range(n_steps):
            k1 = cls.rhs(x, F)
            k2 = cls.rhs(x + 0.5 * dt * k1, F)
            k3 = cls.rhs(x + 0.5 * dt * k2, F)
            k4 = cls.rhs(x + dt * k3, F)
            x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        return x


class TwoScaleLorenz96Operator(ObservationOperator):
    """Two-scale Lorenz-96 (lorenz.py:44-101, K slow X_k each coupled to J fast
    Y_{k,j}) observed by the time-averaged moment function of
    lorenz_mcmc.py:17-40: G = time averages over the n post-step RK4 states of
    [X, Ȳ, X², XȲ, Ȳ²] (q = 5K).  theta = (F, h, b) = prior_means + u
    (lorenz_mcmc.py:64), c fixed (lorenz_mcmc.py:121).

    moments='reference' takes Ȳ_k = Y_{k,0} as the reference does
    (lorenz_mcmc.py:32, np.mean of one element); moments='mean'
    takes the block mean over j.  State order as the reference's:
    [X_0..X_{K-1}, Y_{0,0}..Y_{0,J-1}, Y_{1,0}, ...].  Stateless like
    Lorenz96Operator: every evaluation starts from x0.
    Classical RK4 replaces solve_ivp's RK45."""

    kind = _abi.MODEL_LORENZ96_2S
    J_COMPILED = (1, 2, 4, 8, 10, 16)

    def __init__(self, K=6, J=4, prior_means=(12.0, 8.0, 9.0), c=1.0, x0=None, dt=0.005, n_steps=4000,
                 moments="reference", arith="fma"):
        super().__init__(arith)
        self.K, self.J = int(K), int(J)
        if not 1 <= self.K <= 64:
            raise ValueError("TwoScaleLorenz96Operator: 1 <= K <= 64 on the device")
        if self.J not in self.J_COMPILED:
            raise ValueError(f"TwoScaleLorenz96Operator: J must be one of {self.J_COMPILED}")
        if moments not in ("reference", "mean"):
            raise ValueError("moments must be 'reference' or 'mean'")
        self.moments = moments
        self.k, self.q = 3, 5 * self.K
        self.theta0 = np.asarray(prior_means, dtype=np.float64).reshape(3)
        self.c = float(c)
        if x0 is None:
            x0 = self.spinup(self.K, self.J, (10.0, 10.0, self.c, 10.0), dt=dt, n_steps=2000)
        self.x0 = np.asarray(x0, dtype=np.float64).reshape(self.K * (1 + self.J))
        self.dt = float(dt)
        self.n_steps = int(n_steps)

    def _spec(self):
        return (
            {
                "dim": self.K,
                "fast_per_slow": self.J,
                "moment_mode": 0 if self.moments == "reference" else 1,
                "coupling_c": self.c,
                "n_steps": self.n_steps,
                "dt": self.dt,
            },
            {"theta0": self.theta0, "x0": self.x0},
            {},
        )

    @staticmethod
    def rhs(x, K, J, F, h, c, b):
        """d(state)/dt (host numpy, problem setup), lorenz.py:44-101."""
        X, Y = x[:K], x[K:].reshape(K, J)
        dX = -X - (np.roll(X, 1) * np.roll(X, 2) - np.roll(X, 1) * np.roll(X, -1)) + F - h * c * Y.mean(axis=1)
        nl = np.roll(Y, -1, axis=1) * np.roll(Y, -2, axis=1) - np.roll(Y, 1, axis=1) * np.roll(Y, -1, axis=1)
        dY = c * (-Y - b * nl + (h / J) * X[:, None])
        return np.concatenate([dX, dY.reshape(-1)])

    @classmethod
    def spinup(cls, K, J, theta=(10.0, 10.0, 1.0, 10.0), dt=0.005, n_steps=2000, seed=1):
        """RK4 spin-up on the host from default_rng(seed).random, as
        lorenz_mcmc.py:76-79 seeds its truth run (theta = F, h, c, b)."""
        F, h, c, b = theta
        x = np.random.default_rng(seed).random((J + 1) * K)
        for _ in range(n_steps):
            k1 = cls.rhs(x, K, J, F, h, c, b)
            k2 = cls.rhs(x + 0.5 * dt * k1, K, J, F, h, c, b)
            k3 = cls.rhs(x + 0.5 * dt * k2, K, J, F, h, c, b)
            k4 = cls.rhs(x + dt * k3, K, J, F, h, c, b)
            x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        return x


class BurgersOperator(ObservationOperator):
    """Inviscid Burgers by the reference's Rusanov finite-volume scheme
    (burgers/rusanov.py:6-109: SSPRK2, outflow BC, Rusanov flux with
    f(w) = w²/2) from the perturbed Riemann initial condition
    (utilities.py:44-62) with theta = prior_mean + u = (δ1, δ2, σ0):
    w(x, 0) = 1 + δ1 for x < σ0, δ2 otherwise; observed by the reference's
    Measurer (utilities.py:82-109): meas_scale · trapz over windows of width
    `interval` around `points`.

    dt_mode='cfl' reproduces RusanovFVM.integrate (dt = cfl·dx/max|w|, loop
    while t < T, rusanov.py:40-45, 102-109); dt_mode='fixed' takes n_steps
    steps of dt and marks a chain invalid (Φ = +inf) if the CFL bound is ever
    violated.  nu > 0 adds a central-difference viscous term."""

    kind = _abi.MODEL_BURGERS

    def __init__(
        self,
        prior_mean=(1.5, 0.25, -0.5),
        domain=(-1.0, 1.0),
        N=256,
        T=1.0,
        points=(-0.5, -0.25, 0.25, 0.5, 0.75),
        interval=0.1,
        meas_scale=10.0,
        dt_mode="cfl",
        dt=1e-3,
        n_steps=1000,
        cfl=0.5,
        nu=0.0,
        max_iter=1_000_000,
        arith="fma",
    ):
        super().__init__(arith)
        self.k = 3
        self.theta0 = np.asarray(prior_mean, dtype=np.float64).reshape(3)
        self.N = int(N)
        a, b = float(domain[0]), float(domain[1])
        dxc = (b - a) / self.N
        # rusanov.py:18-25: cell centres incl. ghosts, dx = linspace step
        self.x, self.dx = np.linspace(start=a - 0.5 * dxc, stop=b + 0.5 * dxc, num=self.N + 2, retstep=True)
        xv = self.x[1:-1]
        self.meas_dx = xv[1] - xv[0]  # utilities.py:91
        p = np.asarray(points, dtype=np.float64)
        self.win_lo = np.searchsorted(xv, p - interval / 2, side="left")  # utilities.py:93-95
        self.win_hi = np.searchsorted(xv, p + interval / 2, side="left")  # utilities.py:96-98
        self.q = len(p)
        if np.any(self.win_hi - self.win_lo - 1 > 128):
            raise ValueError("BurgersOperator: a measurement window spans more than 129 cells")
        if self.q > 64:
            raise ValueError("BurgersOperator: at most 64 measurement windows")
        self.meas_scale = float(meas_scale)
        if dt_mode not in ("cfl", "fixed"):
            raise ValueError("dt_mode must be 'cfl' or 'fixed'")
        self.dt_mode = dt_mode
        self.dt = float(dt)
        self.n_steps = int(n_steps)
        self.T = float(T)
        self.cfl = float(cfl)
        self.nu = float(nu)
        self.max_iter = int(max_iter)

    def _spec(self):
        return (
            {
                "dim": self.N,
                "n_steps": self.n_steps,
                "dt": self.dt,
                "dt_mode": _abi.DT_CFL if self.dt_mode == "cfl" else _abi.DT_FIXED,
                "n_windows": self.q,
                "dx": float(self.dx),
                "t_end": self.T,
                "cfl": self.cfl,
                "nu": self.nu,
                "meas_scale": self.meas_scale,
                "meas_dx": float(self.meas_dx),
                "max_iter": self.max_iter,
            },
            {"theta0": self.theta0, "x0": self.x},
            {"win_lo": self.win_lo, "win_hi": self.win_hi},
        )
