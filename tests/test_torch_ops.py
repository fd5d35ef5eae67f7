"""torch.ops.ipmc (csrc/ipmc_torch.cpp): the TORCH_LIBRARY front end of libipmc.

CPU: the library loads, registers its schemas and has NO CPU kernel (a CPU
tensor raises instead of falling back).  GPU: the ops give exactly the bits of
the C-ABI path and of the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")


def test_torch_ops_registered_without_cpu_kernel():
    from ip_mcmc_amd import Lorenz96Operator, _abi, torch_ops

    ops = torch_ops.load()
    assert ops.abi_version() == _abi.ABI_VERSION == 13
    for name in ("pcn_sweep", "potential", "forward"):
        assert str(getattr(ops, name).default._schema).startswith(f"ipmc::{name}(")
    op = Lorenz96Operator(8, 8.0, dt=0.01, n_steps=5)
    u = torch.zeros((2, 8), dtype=torch.float64)
    with pytest.raises(NotImplementedError):
        ops.forward(u, torch.empty((2, 8), dtype=torch.float64), 1, 0)
    with pytest.raises((NotImplementedError, RuntimeError)):
        torch_ops.potential(op, u, torch.zeros(8, dtype=torch.float64), torch.ones(8, dtype=torch.float64))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_torch_ops_match_c_abi_and_oracle(orc, dtype):
    from ip_mcmc_amd import BurgersOperator, Lorenz96Operator, torch_ops

    dev = torch.device("cuda", 0)
    npd = np.float64 if dtype == torch.float64 else np.float32
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64)).to(dtype).to(dev).contiguous()
    for op, C_, beta, n in ((Lorenz96Operator(40, 8.0, dt=0.005, n_steps=100), 300, 0.2, 6),
                            (BurgersOperator(N=64, dt_mode="fixed", dt=2e-3, n_steps=200), 130, 0.15, 4)):
        rng = np.random.default_rng(4)
        U0 = (0.05 * rng.normal(size=(C_, op.k))).astype(npd).astype(np.float64)
        y = orc.forward(op, 0.02 * rng.normal(size=(1, op.k)))[0] + 0.05 * rng.normal(size=op.q)
        ginv, sq = np.full(op.q, 20.0), np.full(op.k, 0.5)
        # forward / potential vs the oracle
        g = torch_ops.forward(op, t(U0)).cpu().numpy()
        assert np.array_equal(g, orc.forward(op, U0, npd))
        phi = torch_ops.potential(op, t(U0), t(y), t(ginv))
        phio = orc.potential(op, U0, y, ginv, npd)
        assert np.array_equal(phi.cpu().numpy(), phio)
        # sweep with running sums vs the oracle
        U = t(U0)
        acc = torch.zeros(C_, dtype=torch.int64, device=dev)
        su = torch.zeros((C_, op.k), dtype=torch.float64, device=dev)
        su2 = torch.zeros_like(su)
        torch_ops.pcn_sweep(op, U, phi, acc, t(y), t(ginv), t(sq), beta, 17, 3, n, sum_u=su, sum_u2=su2)
        Uo, pho = U0.astype(npd), phio.copy()
        acco = np.zeros(C_, dtype=np.int64)
        so = (np.zeros((C_, op.k)), np.zeros((C_, op.k)))
        orc.pcn_sweep(op, Uo, pho, y, ginv, sq, beta, 17, 3, n, accepts=acco, sums=so, n_threads=8)
        torch.cuda.synchronize(dev)
        assert np.array_equal(U.cpu().numpy(), Uo)
        assert np.array_equal(phi.cpu().numpy(), pho)
        assert np.array_equal(acc.cpu().numpy(), acco)
        assert np.array_equal(su.cpu().numpy(), so[0]) and np.array_equal(su2.cpu().numpy(), so[1])
    # shape errors come back as RuntimeError with the op's message
    with pytest.raises(RuntimeError, match="u must be"):
        torch_ops.forward(op, t(np.zeros((2, op.k + 1))))
