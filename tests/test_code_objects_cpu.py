"""The register budget the headline kernels' occupancy depends on, read from
the built libipmc.so's gfx950 code objects (tools/code_objects.py: the
AMDGPU metadata note of each offload bundle; no GPU needed).

The fp64 headline sweep runs two waves per SIMD only because the lane state is
recomputed after G behind an opaque copy of the thread index and Φ(u) is
parked in LDS (ipmc_l96.hpp, IPMC_L96_PARK): 254 VGPRs, no
scratch.  One register more, or a compiler that hoists the recomputation,
would silently halve the occupancy or add scratch traffic; this test fails
instead.  It also fails on a build with IPMC_L96_PARK=0
(profiles/r6/code_objects_nopark.txt)."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import code_objects as CO  # noqa: E402

LIB = os.environ.get("IPMC_CODEOBJ_LIB", CO.LIB)

# kernel -> waves per SIMD it is built for (l96_waves_per_simd /
# l96_pk_waves_per_simd, ipmc_l96.hpp): a wave target of W leaves 512 / W
# registers (VGPRs + AGPRs) per lane
BUDGET = {
    # the headline (config 3, d=40 on 2 lanes per chain), FMA and REFERENCE arith: two waves
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi2ELb1EEEv10ipmc_model10ipmc_sweep": 2,
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi2ELb0EEEv10ipmc_model10ipmc_sweep": 2,
    # the metric's 8-GPU share (8 192 chains per GPU: d=40 on 8 lanes) and the 16 384-chain layout
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi8ELb1EEEv10ipmc_model10ipmc_sweep": 1,
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi4ELb1EEEv10ipmc_model10ipmc_sweep": 2,
    # config 5 (d=256 on 16 lanes), f64 and packed fp32: two waves
    "_ZN4ipmc16l96_sweep_kernelIdLi256ELi16ELb1EEEv10ipmc_model10ipmc_sweep": 2,
    "_ZN4ipmc19l96_sweep_pk_kernelILi256ELi16ELb1EEEv10ipmc_model10ipmc_sweep": 2,
    # the packed fp32 headline: one wave (348 registers without the park)
    "_ZN4ipmc19l96_sweep_pk_kernelILi40ELi2ELb1EEEv10ipmc_model10ipmc_sweep": 1,
    "_ZN4ipmc19l96_sweep_pk_kernelILi40ELi2ELb0EEEv10ipmc_model10ipmc_sweep": 1,
    # Φ(u_0) of the headline (the eval kernel at the sweep's two-wave target, no park)
    "_ZN4ipmc15l96_eval_kernelIdLi40ELi2ELb1ELb1EEEv10ipmc_modellPKT_S4_S4_PS2_": 2,
    "_ZN4ipmc15l96_eval_kernelIdLi40ELi8ELb1ELb1EEEv10ipmc_modellPKT_S4_S4_PS2_": 1,
}


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} is not built (__graft_entry__.build())")
    return CO.kernels(LIB)


@pytest.mark.parametrize("name", sorted(BUDGET))
def test_headline_kernels_fit_their_occupancy_without_scratch(kernels, name):
    assert name in kernels, f"{name} not in {LIB}"
    regs, scratch, vgpr_spill, _ = CO.budget(kernels[name])
    assert scratch == 0, f"{name}: {scratch} B of scratch per lane"
    assert vgpr_spill == 0, f"{name}: {vgpr_spill} VGPRs spilled"
    waves = BUDGET[name]
    assert regs <= 512 // waves, f"{name}: {regs} VGPRs + AGPRs > {512 // waves} ({waves} waves per SIMD)"


def test_headline_kernel_register_count_is_the_measured_one(kernels):
    """The fp64 headline's 254 registers: a drift of more than a
    few registers means the code shape changed -- re-measure it (the budget
    test above is the hard limit)."""
    regs = CO.budget(kernels["_ZN4ipmc16l96_sweep_kernelIdLi40ELi2ELb1EEEv10ipmc_model10ipmc_sweep"])[0]
    assert 240 <= regs <= 256, regs


# The RK4 loops of the measured kernels, as the library holds them (llvm-objdump
# of the code objects): instruction mix per loop iteration and a fingerprint of
# the instruction text with its register numbering.  The packed fp32 headline
# runs one wave per SIMD, where its VGPR numbering alone moved it 1.68 -> 1.86 ms
# (round 6: the RK4 step written as a lambda, identical instructions); the fp64
# headline's schedule is the one the roofline numbers were measured on.  A
# change here is not an error by itself: re-measure the kernel
# (tools/probes/arith_kernel_probe.py, shard_kernel_probe.py) and record the
# new values with the measurement.
RK_LOOPS = {
    # symbol: (RK4 steps per iteration, DPP moves, instruction mix, fingerprint)
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi2ELb1EEEv10ipmc_model10ipmc_sweep":
        (1, 24, {"v_add_f64": 200, "v_fmac_f64_e32": 140, "v_fma_f64": 60, "v_mov_b32_dpp": 24},
         "4ca7e5e543f92291"),
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi2ELb0EEEv10ipmc_model10ipmc_sweep":
        (1, 24, {"v_add_f64": 360, "v_mul_f64": 240, "v_fmac_f64_e32": 40, "v_mov_b32_dpp": 24},
         "310192a4703db684"),
    "_ZN4ipmc19l96_sweep_pk_kernelILi40ELi2ELb1EEEv10ipmc_model10ipmc_sweep":
        (1, 24, {"v_pk_add_f32": 200, "v_pk_fma_f32": 200, "v_mov_b32_dpp": 24}, "8bf10843bdd030d6"),
    # the metric's 8-GPU share: 4 RK4 steps per iteration (l96_forward, M <= 10)
    "_ZN4ipmc16l96_sweep_kernelIdLi40ELi8ELb1EEEv10ipmc_model10ipmc_sweep":
        (4, 96, {"v_add_f64": 200, "v_fmac_f64_e32": 140, "v_fma_f64": 60, "v_mov_b32_dpp": 96},
         "74f2af144cf85a8d"),
}


@pytest.mark.parametrize("name", sorted(RK_LOOPS))
def test_rk_loops_are_the_measured_ones(name):
    from collections import Counter

    steps, dpp, mix, fp = RK_LOOPS[name]
    body = CO.rk_loop(name, LIB, dpp=dpp)
    got = Counter(x.split()[0] for x in body)
    for op, n in mix.items():
        assert got[op] == n, (name, op, got[op], n)
    # FP64 / packed-FP32 work and DPP moves are the loop: besides them only the
    # loop's counter, compare and branch (5 scalar instructions for the 4-step
    # loop) and the x(0) loads' 2 waits, once per iteration of `steps` RK4 steps
    assert len(body) - sum(mix.values()) <= 7, (name, len(body), dict(got))
    assert CO.fingerprint(body) == fp, (
        f"{name}: the RK4 loop's instructions or register numbering changed (fingerprint "
        f"{CO.fingerprint(body)}); re-measure the kernel and record the new fingerprint with the measurement")
