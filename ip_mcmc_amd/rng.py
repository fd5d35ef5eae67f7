"""Counter-based randomness shared by every chain (Philox4x32-10).

The reference threads ONE ``np.random.Generator`` through every component
(report/code.org:12-13): the proposal draws ``multivariate_normal``
(distribution.py:117) and the accepter draws ``random()`` (accepter.py:62),
in that order, once per step.  A sequential stream cannot be shared by 65 536
concurrent chains, so the device draws are a pure function of
(seed, global chain id, global pCN step, component):

  ctr = (slot, chain, step_lo32, step_hi32), key = (seed_lo32, seed_hi32)
  slot j          -> Box–Muller pair of proposal components (2j, 2j+1)
  slot 0xFFFFFFFF -> the accept uniform r in [0, 1)

``PhiloxRNG`` is the user-facing handle: the sampler reads ``seed`` and
``step`` and advances ``step`` by the pCN steps it ran, so two successive
``run`` calls continue one stream exactly as a Generator would (an int seed or
numpy Generator given to the sampler is resolved into one PhiloxRNG once, on
the first run, and kept).
"""
import numpy as np

_MASK64 = (1 << 64) - 1
# Host-side draws (GaussianDistribution.sample with a PhiloxRNG) use pCN steps
# from this offset on (chain id 0), away from any sampler step: the C-ABI
# rejects sweeps that would reach it, and sampler chain ids may use the whole
# 32-bit counter word (include/ipmc.h).
HOST_STEP_BASE = 1 << 63


class PhiloxRNG:
    def __init__(self, seed=0, step=0):
        self.seed = int(seed) & _MASK64
        self.step = int(step)
        self._host_draws = 0

    def __repr__(self):
        return f"PhiloxRNG(seed={self.seed}, step={self.step})"

    def advance(self, n_steps):
        self.step += int(n_steps)

    # ----------------------------------------------------------- device draws
    def normals(self, n_chains, k, step=None, chain_offset=0, dtype=None, device=None):
        """The proposal's standard normals ξ[c, i] for chains chain_offset + c at `step` (device tensor)."""
        from . import device as dev

        return dev.normals(self.seed, chain_offset, n_chains, self.step if step is None else step, k, dtype, device)

    def uniforms(self, n_chains, step=None, chain_offset=0, device=None):
        """The accept uniforms r[c] in [0, 1) (float64 device tensor)."""
        from . import device as dev

        return dev.uniforms(self.seed, chain_offset, n_chains, self.step if step is None else step, device)

    def host_normals(self, k):
        """k fresh standard normals as a numpy array: ipmc_host_normal of
        libipmc_host.so (the device draws' arithmetic on the CPU; no GPU needed)."""
        from . import _hostlib

        z = _hostlib.normals(self.seed, 0, 1, HOST_STEP_BASE + self._host_draws, k)
        self._host_draws += 1
        return z.reshape(k)


# SURVEY §8(b)'s name for the same handle
PhiloxStream = PhiloxRNG


def resolve_rng(rng):
    """PhiloxRNG | int seed | numpy Generator -> PhiloxRNG.

    A numpy Generator (the reference's RNG) seeds a fresh Philox stream from
    one 63-bit integer drawn from it, so runs stay reproducible from the
    Generator's own seed."""
    if isinstance(rng, PhiloxRNG):
        return rng
    if isinstance(rng, (int, np.integer)):
        return PhiloxRNG(int(rng))
    if isinstance(rng, np.random.Generator):
        return PhiloxRNG(int(rng.integers(0, 2**63 - 1)))
    raise TypeError(f"rng must be a PhiloxRNG, an int seed or a numpy Generator, not {type(rng).__name__}")
