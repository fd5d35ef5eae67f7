"""ip_mcmc_amd — MI355X-native many-chain pCN sampler for Bayesian inverse problems.

Drop-in for the pCN hot path of ochsnerd/ip_mcmc (``ip_mcmc/__init__.py``):
the same class names and signatures, plus a leading chain axis, with the
proposal, the forward map G, the potential and the accept/reject fused into
hand-written HIP kernels for gfx950 (libipmc.so, C-ABI in include/ipmc.h).
"""
from .sampler import MCMCSampler
from .proposer import (
    ConstStepStandardRWProposer,
    ConstSteppCNProposer,
    ProposerBase,
    PWLinear,
    VarStepStandardRWProposer,
    VarSteppCNProposer,
)
from .accepter import (
    AccepterBase,
    BoxConstraint,
    ConstrainAccepter,
    CountedAccepter,
    ProbabilisticAccepter,
    StandardRWAccepter,
    pCNAccepter,
)
from .potential import EvolutionPotential, PotentialBase
from .distribution import DistributionBase, GaussianDistribution
from .forward import (
    BurgersOperator,
    LinearOperator,
    Lorenz63Operator,
    Lorenz96Operator,
    ObservationOperator,
    TwoScaleLorenz96Operator,
)
from .rng import PhiloxRNG, PhiloxStream

# the name report/scripts/stuart_examples.py:6 imports (the package's
# ConstSteppCNProposer under its older name)
pCNProposer = ConstSteppCNProposer
from ._lib import IpmcError, UnsupportedOnDevice

__all__ = [
    "MCMCSampler",
    "ProposerBase",
    "ConstSteppCNProposer",
    "pCNProposer",
    "VarSteppCNProposer",
    "ConstStepStandardRWProposer",
    "VarStepStandardRWProposer",
    "PWLinear",
    "StandardRWAccepter",
    "AccepterBase",
    "BoxConstraint",
    "ConstrainAccepter",
    "CountedAccepter",
    "ProbabilisticAccepter",
    "pCNAccepter",
    "EvolutionPotential",
    "PotentialBase",
    "DistributionBase",
    "GaussianDistribution",
    "BurgersOperator",
    "LinearOperator",
    "Lorenz63Operator",
    "Lorenz96Operator",
    "ObservationOperator",
    "TwoScaleLorenz96Operator",
    "PhiloxRNG",
    "PhiloxStream",
    "IpmcError",
    "UnsupportedOnDevice",
]
