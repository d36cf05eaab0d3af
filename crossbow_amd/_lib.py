"""ctypes binding of ``libcrossbow_sma.so`` (declared in include/crossbow_sma.h).

The library is the product path: there is no CPU fallback.  Loading fails
loudly when the .so is missing, and every compute entry point fails with
``CBX_ERR_NO_DEVICE`` on a host without an MI355X.

``torch`` is imported before the library is loaded so that, in processes that
also use PyTorch (bench.py, the GPU tests), both share PyTorch's HIP runtime
and RCCL (same SONAMEs) instead of loading a second copy.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401,E402  (see module docstring: one HIP runtime per process)

from ._abi import *  # noqa: F401,F403  (status codes, constants, CbxError)
from ._abi import SIGNATURES, CbxError, bind  # noqa: F401

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libcrossbow_sma.so")

_lib = None


def load(path: str = LIB_PATH):
    """Load the library (building it first if it is absent and hipcc exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        from . import build as _build
        _build.build_lib()
    if not os.path.exists(path):
        raise RuntimeError(f"crossbow_amd native library missing: {path} (run `python -m crossbow_amd.build`)")
    lib = bind(ctypes.CDLL(path))
    _lib = lib
    return lib


def last_error() -> str:
    return load().cbx_last_error().decode(errors="replace")


def check(rc: int) -> int:
    """Raise CbxError on a negative status; return non-negative values."""
    if rc < 0:
        raise CbxError(rc, last_error())
    return rc
