"""Loader for the in-tree HIP library ``ip_mcmc_amd/lib/libipmc.so``.

There is no CPU fallback: if the library is missing or a call fails, this
module raises.  Build it with ``python -c "import __graft_entry__ as g; g.build()"``
or ``make -C ip_mcmc_amd/csrc -j8``.
"""
import ctypes as C
import os

from . import _abi

# IPMC_LIB_PATH selects another build of the same library (layout experiments).
LIB_PATH = os.environ.get("IPMC_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                           "libipmc.so")


class IpmcError(RuntimeError):
    """A libipmc call returned an error status."""

    def __init__(self, fn, status, message):
        self.fn = fn
        self.status = status
        super().__init__(f"{fn} failed with {_abi.STATUS_NAMES.get(status, status)}: {message}")


class UnsupportedOnDevice(NotImplementedError):
    """The requested composition has no device implementation."""


_lib = None


def lib():
    """The loaded libipmc (loaded once, signatures bound)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libipmc.so not found at {LIB_PATH}; build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')"
            )
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in _abi.SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        v = h.ipmc_abi_version()
        if v != _abi.ABI_VERSION:
            raise RuntimeError(f"libipmc ABI version {v} != {_abi.ABI_VERSION}")
        _lib = h
    return _lib


def call(name, *args):
    """Call a libipmc entry point; raise IpmcError on a non-zero status."""
    h = lib()
    rc = getattr(h, name)(*args)
    if rc != _abi.OK:
        msg = h.ipmc_last_error().decode(errors="replace")
        if rc == _abi.ERR_UNSUPPORTED:
            raise UnsupportedOnDevice(f"{name}: {msg}")
        raise IpmcError(name, rc, msg)
    return rc
