"""crossbow_amd -- MI355X-native synchronous model averaging (SMA) for Crossbow.

The product is ``libcrossbow_sma.so`` (HIP for gfx950, C-ABI in
``include/crossbow_sma.h``).  This package holds its sources (``csrc/``), the
build (``build.py``), and the host-side mirror of Crossbow's interface for the
path: ``TheGPU`` (the JNI natives) and ``ModelManager.trySynchronise``.
"""
from ._lib import (BUF_DATA, BUF_DIFF, BUF_GRADIENT, BUF_LAST, SYNC_ASP, SYNC_BSP, SYNC_SSP,  # noqa: F401
                   UPDATE_DEFAULT, UPDATE_SMA, UPDATE_SYNCHRONOUSEAMSGD, UPDATE_WORKER, CbxError)
from .modelmanager import ModelManager  # noqa: F401
from .thegpu import TheGPU  # noqa: F401
