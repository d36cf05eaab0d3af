"""Python view of the sma.c seam (include/crossbow_sma.h, ``cbx_sma_plan_*``):
the SMA step and the replica optimiser step over device buffers the caller
owns, for a Crossbow build that keeps its own model manager and replaces only
``crossbowSynchronisationSMA`` (clib-multigpu/synch/sma.c:233-248) and
``crossbowKernelOptimiserSMA`` (kernels/optimisers/sma.cu:3-100).

Pointers and streams are plain integers (``tensor.data_ptr()``,
``torch.cuda.Stream().cuda_stream``, or raw ``hipMalloc`` results).  Torch-free:
``lib`` is a bound library (``crossbow_amd._lib.load()`` by default, or a
build bound through ``crossbow_amd._abi.bind``).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple


def _default_lib():
    from . import _lib
    return _lib.load()


def _raise(lib, rc: int, what: str) -> int:
    if rc < 0:
        msg = f"{what}: {lib.cbx_last_error().decode(errors='replace')}"
        try:
            from ._abi import CbxError
        except ImportError:  # loaded as a standalone file (the torch-free test workers)
            raise RuntimeError(f"{rc} {msg}") from None
        raise CbxError(rc, msg)
    return rc


def _ptrs(values: Sequence[Optional[int]]):
    arr = (ctypes.c_void_p * max(1, len(values)))()
    for k, v in enumerate(values):
        arr[k] = v or None
    return arr


def _ints(values: Sequence[int]):
    arr = (ctypes.c_int * max(1, len(values)))()
    for k, v in enumerate(values):
        arr[k] = int(v)
    return arr


class SmaPlan:
    """``cbx_sma_plan_create`` over HIP devices ``devices`` for buffers of
    ``elements`` floats; ``comms`` = the caller's ncclComm_t handles (ints), or
    None to let the plan create them (ncclCommInitAll, more than one device)."""

    def __init__(self, devices: Sequence[int], elements: int, comms: Optional[Sequence[int]] = None, lib=None,
                 buckets: int = 0):
        self.lib = lib if lib is not None else _default_lib()
        self.G = len(devices)
        p = ctypes.c_void_p()
        _raise(self.lib, self.lib.cbx_sma_plan_create(ctypes.byref(p), _ints(devices), self.G, elements,
                                                      _ptrs(comms) if comms is not None else None),
               "cbx_sma_plan_create")
        self._p = p
        if buckets:
            self.set_buckets(buckets)

    def step(self, streams: Sequence[int], z: Sequence[int], last: Optional[Sequence[Optional[int]]],
             replicas: Sequence[Tuple[int, int, int, int, int]], alpha: float, momentum: float,
             first: int = 0) -> int:
        """One SMA step.  ``replicas[id]`` = (device index, w, s, locked, copy).
        Returns 1 when Phase D ran."""
        dev = [r[0] for r in replicas]
        return _raise(self.lib, self.lib.cbx_sma_plan_step(
            self._p, _ptrs(streams), _ptrs(z), _ptrs(last) if last is not None else None, len(replicas),
            _ints(dev), _ptrs([r[1] for r in replicas]), _ptrs([r[2] for r in replicas]),
            _ints([r[3] for r in replicas]), _ints([r[4] for r in replicas]), ctypes.c_float(alpha),
            ctypes.c_float(momentum), first), "cbx_sma_plan_step")

    def ssgd_step(self, streams: Sequence[int], z: Sequence[int], last: Optional[Sequence[Optional[int]]],
                  acc: Sequence[int], replicas: Sequence[Tuple[int, int, int]], momentum: float, wpc: int,
                  first: int = 0) -> None:
        """One synchronous-SGD barrier (update model WORKER).  ``replicas[id]`` =
        (device index, w, locked)."""
        _raise(self.lib, self.lib.cbx_ssgd_plan_step(
            self._p, _ptrs(streams), _ptrs(z), _ptrs(last) if last is not None else None, _ptrs(acc),
            len(replicas), _ints([r[0] for r in replicas]), _ptrs([r[1] for r in replicas]),
            _ints([r[2] for r in replicas]), ctypes.c_float(momentum), wpc, first), "cbx_ssgd_plan_step")

    def average_batchnorm(self, elements: Sequence[int], mean: Sequence[int], variance: Sequence[int],
                          updated: Sequence[int]) -> None:
        """BN running-statistics averaging; ``mean``/``variance``/``updated`` are
        indexed [k * layers + l] (k: position in the plan's devices)."""
        _raise(self.lib, self.lib.cbx_sma_plan_average_batchnorm(
            self._p, len(elements), _ints(elements), _ptrs(mean), _ptrs(variance), _ints(updated)),
            "cbx_sma_plan_average_batchnorm")

    def set_buckets(self, buckets: int) -> None:
        """G > 1: buckets of the all-reduce pipeline (0 = default 8, 1 = in order)."""
        _raise(self.lib, self.lib.cbx_sma_plan_set_buckets(self._p, buckets), "cbx_sma_plan_set_buckets")

    def free(self) -> None:
        if self._p:
            self.lib.cbx_sma_plan_free(self._p)
            self._p = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()


def optimise_buffers(stream: int, w: int, g: int, last: Optional[int], s: int, elements: int,
                     learning_rate: float, momentum: float, weight_decay: float, lib=None) -> None:
    """``cbx_sma_optimise_buffers``: one task's replica optimiser step."""
    lib = lib if lib is not None else _default_lib()
    _raise(lib, lib.cbx_sma_optimise_buffers(stream or None, w, g, last or None, s, elements,
                                             ctypes.c_float(learning_rate), ctypes.c_float(momentum),
                                             ctypes.c_float(weight_decay)), "cbx_sma_optimise_buffers")


def ssgd_accumulate_buffers(stream: int, w: Optional[int], g: int, acc: int, elements: int, learning_rate: float,
                            weight_decay: float, lib=None) -> None:
    """``cbx_ssgd_accumulate_buffers``: one task's synchronous-SGD step."""
    lib = lib if lib is not None else _default_lib()
    _raise(lib, lib.cbx_ssgd_accumulate_buffers(stream or None, w or None, g, acc, elements,
                                                ctypes.c_float(learning_rate), ctypes.c_float(weight_decay)),
           "cbx_ssgd_accumulate_buffers")
