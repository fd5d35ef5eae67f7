"""Two-scale Lorenz-96 lane layouts: one or two slow variables per lane
(lanes_per_chain = K or K/2; for K > 32 the ring's halos go through LDS) and,
for K = 6 with J <= 4, three (2 lanes, DPP halos) or all six (1 lane), with
and without speculative slots, equal the oracle bit for bit (G, Φ and
sweeps)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from test_gpu_parity import _assert_same, _np, _problem, _sweep_device, _sweep_oracle  # noqa: E402


@pytest.fixture(scope="module")
def dev_ts():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("K,J", [(2, 4), (6, 4), (4, 10), (36, 10), (40, 2), (64, 1), (8, 8), (48, 8)])
def test_ts_two_slow_per_lane_bit_exact(dev_ts, orc, dtype, K, J):
    from ip_mcmc_amd import TwoScaleLorenz96Operator

    rng = np.random.default_rng(K * 100 + J)
    for arith, mom in (("fma", "mean"), ("reference", "reference")):
        op = TwoScaleLorenz96Operator(K=K, J=J, x0=rng.normal(size=K * (1 + J)), dt=0.004, n_steps=20,
                                      moments=mom, arith=arith)
        U = 0.3 * rng.normal(size=(23, 3))
        # the device forward map with the automatic layout (two per lane for K > 32)
        g = op.forward_device(torch.as_tensor(U, dtype=dtype, device=dev_ts)).cpu().numpy()
        assert np.array_equal(g, orc.forward(op, U, _np(dtype))), (K, J, arith)
        U0, phi0, y, ginv, sq = _problem(op, 29, dtype, orc, seed=K + J)
        ginv = ginv * 0.2
        phi0 = orc.potential(op, U0, y, ginv, _np(dtype)).astype(np.float64)
        o = _sweep_oracle(orc, op, U0, phi0, y, ginv, sq, 0.3, 4, 7, 9, dtype, want_sums=True)
        layouts = [(K, 1), (K // 2, 1), (K // 2, 0), (K, 0)]
        if K == 6 and J <= 4:
            layouts += [(2, 1), (2, 0), (2, 4), (1, 1), (1, 0), (1, 8)]
        for lanes, spec in layouts:
            d = _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 4, 7, 9, dtype, dev_ts, lanes=lanes, spec=spec,
                              want_sums=True)
            _assert_same(d, o, (K, J, arith, lanes, spec))
            assert np.array_equal(d["sum_u"], o["sum_u"]) and np.array_equal(d["samp"], o["u"])


def test_ts_layout_requests_checked(dev_ts, orc):
    from ip_mcmc_amd import TwoScaleLorenz96Operator, UnsupportedOnDevice

    op = TwoScaleLorenz96Operator(K=5, J=4, x0=np.zeros(25), n_steps=5)
    U0, phi0, y, ginv, sq = _problem(op, 4, torch.float64, orc)
    with pytest.raises(UnsupportedOnDevice, match="lanes_per_chain must be K"):
        _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 4, 0, 2, torch.float64, dev_ts, lanes=2)
    op = TwoScaleLorenz96Operator(K=6, J=16, x0=np.zeros(6 * 17), n_steps=5)
    U0, phi0, y, ginv, sq = _problem(op, 4, torch.float64, orc)
    with pytest.raises(UnsupportedOnDevice, match="lanes_per_chain must be K"):
        _sweep_device(op, U0, phi0, y, ginv, sq, 0.3, 4, 0, 2, torch.float64, dev_ts, lanes=3)
