"""Host-side API of ip_mcmc_amd against the reference's own unit tests.

The reference's tests (ip_mcmc/*_test.py) drive the one-step host methods
with its MockRNG; the same assertions hold here (restated, with a local
MockRNG of the same behaviour, test_utilities.py:11-26).  No GPU is used.
"""
import numpy as np
import pytest

from ip_mcmc_amd import (
    BoxConstraint,
    ConstrainAccepter,
    ConstStepStandardRWProposer,
    ConstSteppCNProposer,
    CountedAccepter,
    GaussianDistribution,
    MCMCSampler,
    PWLinear,
    StandardRWAccepter,
    VarStepStandardRWProposer,
    VarSteppCNProposer,
    pCNAccepter,
)


class MockRNG(np.random.Generator):
    def __init__(self, result):
        super().__init__(np.random.PCG64())
        self.result = result

    def normal(self, loc=None, scale=None):
        return self.result

    def multivariate_normal(self, mean=None, cov=None):
        return self.result * np.ones_like(mean)

    def random(self):
        if np.all(0 <= self.result) and np.all(self.result <= 1):
            return self.result
        return 0.5


# distribution_test.py:7-24
def test_gaussian_scalar():
    rng = MockRNG(0)
    g = GaussianDistribution(mean=1, covariance=2)
    assert np.isclose(g.sample(rng), 0)
    assert np.isclose(g.apply_covariance(1), 2)
    assert np.isclose(g.apply_sqrt_covariance(1), np.sqrt(2))
    assert np.isclose(g.apply_precision(1), 0.5)
    assert np.isclose(g.apply_sqrt_precision(1), np.sqrt(0.5))


def test_gaussian_multivariate():
    g = GaussianDistribution(mean=np.array([1, 1, 1]), covariance=np.diagflat([1, 2, 3]))
    assert all(np.isclose([1, 2, 3], g.apply_covariance([1, 1, 1])))
    assert all(np.isclose([1, np.sqrt(2), np.sqrt(3)], g.apply_sqrt_covariance([1, 1, 1])))
    assert all(np.isclose([1, 1 / 2, 1 / 3], g.apply_precision([1, 1, 1])))
    assert all(np.isclose([1, 1 / np.sqrt(2), 1 / np.sqrt(3)], g.apply_sqrt_precision([1, 1, 1])))


def test_gaussian_logpdf_matches_reference(golden):
    g = GaussianDistribution(mean=np.array([1.0, -2.0, 0.5]), covariance=np.diag([0.5, 2.0, 1.5]))
    np.testing.assert_allclose(g.logpdf(golden["gauss_x"]), golden["gauss_logpdf"], rtol=1e-13)
    gf = GaussianDistribution(mean=np.array([0.0, 1.0]), covariance=np.array([[2.0, 0.5], [0.5, 1.0]]))
    np.testing.assert_allclose(gf.logpdf(golden["gaussfull_x"]), golden["gaussfull_logpdf"], rtol=1e-13)
    assert isinstance(g.logpdf(golden["gauss_x"][0]), float)


# proposer_test.py:8-58
def test_rw_proposer_scalar():
    rng = MockRNG(-np.pi)
    delta = np.e
    p = ConstStepStandardRWProposer(delta, GaussianDistribution(100, np.sin(np.e)))
    assert np.isclose(p.prefactor, np.sqrt(2 * delta))
    assert np.isclose(p(-np.e, rng), -np.e - p.prefactor * np.pi)


def test_rw_proposer_multivariate():
    rng = MockRNG(np.array([1, 2]))
    p = ConstStepStandardRWProposer(np.pi, GaussianDistribution(np.array([-1, 2]), np.array([[1, 0], [0, 4]])))
    assert np.isclose(p(np.array([-1, 2]), rng), np.array([-1 + p.prefactor, 2 + 2 * p.prefactor])).all()


def test_pcn_proposer_scalar():
    rng = MockRNG(-np.pi)
    beta = 1 / np.e
    p = ConstSteppCNProposer(beta, GaussianDistribution(mean=0, covariance=2))
    assert np.isclose(p.contraction, np.sqrt(1 - beta**2))
    assert np.isclose(p(-np.pi, rng), np.sqrt(1 - beta**2) * (-np.pi) + beta * -np.pi)


def test_pcn_proposer_multivariate():
    rng = MockRNG(np.array([2, -1]))
    p = ConstSteppCNProposer(0.5, GaussianDistribution(np.array([0, 0]), np.array([[2, 0.5], [0.5, 1]])))
    u = np.array([1, 1])
    assert np.isclose(p(u, rng), np.sqrt(1 - 0.25) * u + 0.5 * np.array([2, -1])).all()


def test_pcn_beta_range_asserted():
    with pytest.raises(AssertionError):
        ConstSteppCNProposer(1.5, GaussianDistribution(0, 1))


def test_var_step_schedules_count_from_one():
    prior = GaussianDistribution(np.zeros(2), np.eye(2))
    p = VarSteppCNProposer(lambda i: 0.1 * i, prior)
    s = p.beta_schedule(0, 3)
    np.testing.assert_allclose(s[:, 0], [0.1, 0.2, 0.3])
    np.testing.assert_allclose(s[:, 1], np.sqrt(1 - s[:, 0] ** 2))
    r = VarStepStandardRWProposer(PWLinear(0.1, 0.001, 10), prior)
    s = r.beta_schedule(9, 3)
    np.testing.assert_allclose(s[:, 0], np.sqrt(2) * np.sqrt([0.1 - 0.0099 * 10, 0.001, 0.001]))


# accepter_test.py:20-42
def test_standard_rw_accepter_regularizer_quirk():
    rng = MockRNG(np.exp(-(np.sqrt(2) + 0.5)) + 0.01)
    a = StandardRWAccepter(lambda u: np.linalg.norm(u), GaussianDistribution(mean=0, covariance=2))
    assert np.isclose(a._I(1), 1 + 1)
    assert np.isclose(a._I(5), 5 + 25)
    assert a(0, 0, rng)
    assert not a(0, np.sqrt(2), rng)


def test_pcn_accepter_probability():
    a = pCNAccepter(lambda x: -np.log(x))  # AnalyticPotential(x*x, x): exp(-Φ) = x
    assert np.isclose(a.accept_probability(1, 1), 1)
    assert np.isclose(a.accept_probability(1, 2), 2)


def test_counted_and_constrain_accepters():
    c = CountedAccepter(pCNAccepter(lambda x: 0.0))
    with pytest.raises(ValueError):
        c.ratio()
    rng = MockRNG(0.5)
    assert c(0, 1, rng)
    assert c.calls == 1 and c.accepts == 1 and c.ratio() == 1.0
    box = BoxConstraint(lower=[-1.0], upper=[1.0], offset=[0.5])
    k = ConstrainAccepter(c, box)
    assert not k(0, np.array([0.6]), rng)  # 1.1 is outside (-1, 1): no inner call
    assert c.calls == 1
    assert k(0, np.array([0.4]), rng) and c.calls == 2
    assert np.array_equal(box(np.array([[0.4], [0.6], [-1.6]])), [True, False, False])


# sampler.py:43-54: the oracle's restatement (the checker of the device kernel
# behind MCMCSampler.autocorr) against the reference's own outputs
def test_autocorr_oracle_matches_reference_fixture(golden, orc):
    got = np.stack([orc.autocorr_ref(x) for x in golden["ac_x"]])
    np.testing.assert_array_equal(got, golden["ac_ref"])
    assert np.all(orc.autocorr_ref(np.ones(7)) == 1)


def test_step_schedule_matches_reference(golden):
    """sampler.py:18-26 step count (fixture from the reference with MockProposer)."""
    for b, n, s, calls in golden["schedule"]:
        assert max(0, b - s) + n * s == calls


def test_steps_per_launch_bounds_launch_work():
    """Heavy ensembles are split into short launches; light ones use the cap."""
    from ip_mcmc_amd import Lorenz96Operator, TwoScaleLorenz96Operator, _abi
    from ip_mcmc_amd.sampler import STEPS_PER_LAUNCH, _steps_per_launch

    def model(op):
        m = _abi.IpmcModel()
        for name, val in op._spec()[0].items():
            setattr(m, name, val)
        return m

    head = Lorenz96Operator(40, 8.0, x0=np.full(40, 8.0), dt=0.005, n_steps=2000)
    cfg5 = Lorenz96Operator(256, 8.0, x0=np.full(256, 8.0), dt=0.005, n_steps=10000)
    assert _steps_per_launch(model(head), 65536) == 152  # 8e11 // 5.24e9
    assert _steps_per_launch(model(cfg5), 131072) == 2
    assert _steps_per_launch(model(head), 4) == STEPS_PER_LAUNCH
    ts = TwoScaleLorenz96Operator(K=36, J=10, x0=np.zeros(396), n_steps=2000)
    assert 1 <= _steps_per_launch(model(ts), 16384) < STEPS_PER_LAUNCH
