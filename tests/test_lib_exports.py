"""libipmc.so / liboracle.so load and export what the headers declare (no GPU call)."""
import ctypes
import os
import re

from conftest import REPO


def _declared(header):
    src = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ipmc_\w+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    names = _declared("ipmc.h")
    assert {"ipmc_pcn_sweep", "ipmc_potential", "ipmc_forward", "ipmc_normal", "ipmc_uniform",
            "ipmc_auto_lanes", "ipmc_last_error", "ipmc_abi_version"} <= set(names)


def test_libipmc_exports_every_declared_symbol():
    from ip_mcmc_amd import _abi, _lib

    h = _lib.lib()
    for name in _declared("ipmc.h"):
        assert hasattr(h, name), name
    assert set(_abi.SIGNATURES) == set(_declared("ipmc.h"))
    assert h.ipmc_abi_version() == _abi.ABI_VERSION


def test_struct_layout_matches_header():
    """ctypes mirror sizes equal the C compiler's (checked via the oracle build of the same header)."""
    from ip_mcmc_amd import _abi

    # pointers and doubles are 8-aligned on x86-64 / gfx950 alike
    assert ctypes.sizeof(_abi.IpmcModel) % 8 == 0
    assert ctypes.sizeof(_abi.IpmcSweep) % 8 == 0
    assert _abi.IpmcSweep.calls.offset == _abi.IpmcSweep.accepts.offset + 8
    assert _abi.IpmcModel.max_iter.offset == _abi.IpmcModel.meas_dx.offset + 8


def test_oracle_library_loads(orc):
    from ip_mcmc_amd import _abi

    assert orc.lib().orc_abi_version() == _abi.ABI_VERSION == 13


def test_struct_offsets_match_c_compiler(orc):
    """Every ctypes field offset equals offsetof() in the C compiler's view of include/ipmc.h."""
    import numpy as np
    from ip_mcmc_amd import _abi

    out = np.zeros(128, dtype=np.int64)
    lib = orc.lib()
    lib.orc_layout.argtypes = [ctypes.c_void_p]
    n = lib.orc_layout(out.ctypes.data)
    want = [ctypes.sizeof(_abi.IpmcModel)] + [getattr(_abi.IpmcModel, f).offset for f, _ in _abi.IpmcModel._fields_]
    want += [ctypes.sizeof(_abi.IpmcSweep)] + [getattr(_abi.IpmcSweep, f).offset for f, _ in _abi.IpmcSweep._fields_]
    assert list(out[:n]) == want


def test_libipmc_host_exports_every_declared_symbol():
    """libipmc_host.so (include/ipmc_host.h) loads without a GPU or the HIP
    runtime and exports exactly what its header declares."""
    import subprocess

    from ip_mcmc_amd import _hostlib

    h = _hostlib.lib()
    names = _declared("ipmc_host.h")
    assert set(names) == set(_hostlib.SIGNATURES)
    for name in names:
        assert hasattr(h, name), name
    assert h.ipmc_host_abi_version() == _hostlib.ABI_VERSION
    deps = subprocess.run(["ldd", _hostlib.LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip64" not in deps and "libhsa" not in deps, deps
