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
