"""ctypes front-end for the CPU SMA oracle (``oracle/sma_oracle.c``).

TEST INFRASTRUCTURE ONLY.  Imported by ``tests/``, by
``__graft_entry__.smoke()`` (as the checker) and by ``bench.py``'s
``cpu_baseline`` leg.  The product package ``crossbow_amd`` never imports it.

Restates ``clib-multigpu/synch/sma.c:13-231`` (phases A-D) and
``clib-multigpu/synch/common.c:3-57`` (the all-reduce); see the C file for the
per-line citations.  Parity unpinned against reference outputs (the reference
holds no fixtures for this path and cannot be built here); cross-checked bit
for bit against an OpenBLAS replay of the reference's saxpy call sequence.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsma_oracle.so")

SEED = 20190701
BUF_Z, BUF_LAST, BUF_S0, BUF_W0 = 0, 1, 16, 17
BASE_MOMENTUM = np.float32(0.9)

_lib = None


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        fpp = ctypes.POINTER(fp)
        ip = ctypes.POINTER(ctypes.c_int)
        L.cbo_splitmix64.restype = ctypes.c_uint64
        L.cbo_splitmix64.argtypes = [ctypes.c_uint64]
        L.cbo_fill_normal.restype = None
        L.cbo_fill_normal.argtypes = [fp, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_float, fp]
        for name in ("cbo_sma_fma", "cbo_sma_blas"):
            f = getattr(L, name)
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_float, ctypes.c_float,
                          fpp, fpp, fpp, fpp, ip, ip, ctypes.c_int, fp]
        L.cbo_sma_accumulate.restype = ctypes.c_int
        L.cbo_sma_accumulate.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_float, fp, fpp, fpp, ip, fp]
        L.cbo_sma_apply.restype = None
        L.cbo_sma_apply.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_float, fp, fp, fp, fpp, ctypes.c_int]
        for name in ("cbo_sma_optimise", "cbo_sma_optimise_blas"):
            f = getattr(L, name)
            f.restype = None if name == "cbo_sma_optimise" else ctypes.c_int
            f.argtypes = [ctypes.c_size_t, ctypes.c_float, ctypes.c_float, ctypes.c_float, fp, fp, fp, fp]
        for name in ("cbo_default_task", "cbo_default_task_blas"):
            f = getattr(L, name)
            f.restype = None if name == "cbo_default_task" else ctypes.c_int
            f.argtypes = [ctypes.c_size_t, ctypes.c_float, ctypes.c_float, ctypes.c_float, fp, fp, fp, fp]
        L.cbo_default_sync.restype = None
        L.cbo_default_sync.argtypes = [ctypes.c_int, ctypes.c_size_t, fp, fpp, ip, ctypes.c_int]
        for name in ("cbo_ssgd_worker", "cbo_ssgd_worker_blas"):
            f = getattr(L, name)
            f.restype = None if name == "cbo_ssgd_worker" else ctypes.c_int
            f.argtypes = [ctypes.c_size_t, ctypes.c_float, ctypes.c_float, fp, fp, fp]
        for name in ("cbo_ssgd_sync", "cbo_ssgd_sync_blas"):
            f = getattr(L, name)
            f.restype = None if name == "cbo_ssgd_sync" else ctypes.c_int
            f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                          fpp, fpp, fpp, fpp, ip, ctypes.c_int, fp]
        L.cbo_bn_average.restype = ctypes.c_int
        L.cbo_bn_average.argtypes = [ctypes.c_int, ctypes.c_int, ip, fpp, fpp, ip]
        L.cbo_blas_open.restype = ctypes.c_int
        L.cbo_blas_open.argtypes = [ctypes.c_char_p]
        L.cbo_blas_name.restype = ctypes.c_char_p
        L.cbo_blas_set_threads.argtypes = [ctypes.c_int]
        L.cbo_bind_core.argtypes = [ctypes.c_int]
        L.cbo_now.restype = ctypes.c_double
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _fpp(arrs):
    fp = ctypes.POINTER(ctypes.c_float)
    if arrs is None:
        return None
    return (fp * len(arrs))(*[(_fp(a) if a is not None else fp()) for a in arrs])


def splitmix64(x: int) -> int:
    return int(lib().cbo_splitmix64(ctypes.c_uint64(x & 0xFFFFFFFFFFFFFFFF)))


def fill_normal(n: int, buffer_id: int, sigma: float, mean: Optional[np.ndarray] = None) -> np.ndarray:
    """``mean + sigma * N(0,1)`` from splitmix64 -> Box-Muller."""
    out = np.empty(n, dtype=np.float32)
    m = _fp(mean) if mean is not None else ctypes.POINTER(ctypes.c_float)()
    lib().cbo_fill_normal(_fp(out), n, (SEED ^ buffer_id) & 0xFFFFFFFFFFFFFFFF, sigma, m)
    return out


@dataclass
class SmaState:
    """All buffers of one SMA step, laid out like the model manager.

    ``z[g]``/``last[g]`` are the base model (and its momentum) on device g;
    ``s[i]``/``w[i]`` are replica i's snapshot and data; replica i lives on
    device ``i % G`` (clib-multigpu/modelmanager.c:51-64).
    """
    G: int
    size: int
    n: int
    alpha: float
    momentum: float
    z: List[np.ndarray]
    last: Optional[List[np.ndarray]]
    s: List[np.ndarray]
    w: List[np.ndarray]
    locked: np.ndarray = field(default=None)
    copy: np.ndarray = field(default=None)
    first: int = 0

    def __post_init__(self):
        if self.locked is None:
            self.locked = np.ones(self.size, dtype=np.int32)
        if self.copy is None:
            self.copy = np.zeros(self.size, dtype=np.int32)
        self.locked = np.ascontiguousarray(self.locked, dtype=np.int32)
        self.copy = np.ascontiguousarray(self.copy, dtype=np.int32)

    def clone(self) -> "SmaState":
        cp = lambda L: None if L is None else [a.copy() for a in L]  # noqa: E731
        return SmaState(self.G, self.size, self.n, self.alpha, self.momentum, cp(self.z), cp(self.last),
                        cp(self.s), cp(self.w), self.locked.copy(), self.copy.copy(), self.first)


def make_state(n: int, G: int, R: int, alpha: float, momentum: float, threads: int = 1) -> SmaState:
    """Synthetic inputs of BASELINE.md 2.3 for ``G`` devices x ``R`` replicas.
    ``threads`` > 1 fills the buffers on that many threads (the C fill
    releases the GIL); the values are the same."""
    size = G * R
    if threads > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            zf = ex.submit(fill_normal, n, BUF_Z, 0.05)
            lf = ex.submit(fill_normal, n, BUF_LAST, 0.001) if momentum > 0 else None
            z = zf.result()
            s = list(ex.map(lambda i: fill_normal(n, BUF_S0 + 2 * i, 0.01, z), range(size)))
            w = list(ex.map(lambda i: fill_normal(n, BUF_W0 + 2 * i, 0.001, s[i]), range(size)))
            last = lf.result() if lf is not None else None
        return SmaState(G, size, n, alpha, momentum, [z.copy() for _ in range(G)],
                        None if last is None else [last.copy() for _ in range(G)], s, w)
    z = fill_normal(n, BUF_Z, 0.05)
    last = fill_normal(n, BUF_LAST, 0.001) if momentum > 0 else None
    s, w = [], []
    for i in range(size):
        si = fill_normal(n, BUF_S0 + 2 * i, 0.01, z)
        s.append(si)
        w.append(fill_normal(n, BUF_W0 + 2 * i, 0.001, si))
    return SmaState(G, size, n, alpha, momentum, [z.copy() for _ in range(G)],
                    None if last is None else [last.copy() for _ in range(G)], s, w)


def _step(fn, st: SmaState, scratch_floats: int) -> int:
    scratch = np.empty(max(1, scratch_floats), dtype=np.float32)
    lp = _fpp(st.last) if st.last is not None else _fpp([None] * st.G)
    return fn(st.G, st.size, st.n, st.alpha, st.momentum, _fpp(st.z), lp, _fpp(st.s), _fpp(st.w),
              st.locked.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
              st.copy.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), st.first, _fp(scratch))


def sma_step(st: SmaState) -> int:
    """One SMA step (fmaf restatement), in place.  Returns Phase-D copy count."""
    if st.momentum > 0 and st.last is None:
        raise ValueError("momentum > 0 requires base-model `last` buffers (model.c:116-120)")
    return _step(lib().cbo_sma_fma, st, (st.G + 1) * st.n)


def sma_accumulate(alpha: float, z: np.ndarray, s: List[np.ndarray], w: List[np.ndarray],
                   copy: Optional[List[int]] = None) -> "tuple[np.ndarray, int]":
    """Phase A of one device over its (locked, id-ordered) replicas; w updated in place."""
    n = z.size
    acc = np.empty(n, dtype=np.float32)
    cp = None
    if copy is not None:
        arr = np.ascontiguousarray(copy, dtype=np.int32)
        cp = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    c = lib().cbo_sma_accumulate(len(s), n, alpha, _fp(z), _fpp(s), _fpp(w), cp, _fp(acc))
    return acc, int(c)


def sma_apply(momentum: float, D: np.ndarray, z: np.ndarray, last: Optional[np.ndarray],
              w: List[np.ndarray], copy: bool) -> None:
    """Phases C and D of one device, in place on z, last and (if copy) w."""
    lp = _fp(last) if last is not None else ctypes.POINTER(ctypes.c_float)()
    lib().cbo_sma_apply(len(w), z.size, momentum, _fp(D), _fp(z), lp, _fpp(w) if w else None, 1 if copy else 0)


def sma_optimise(rate: float, momentum: float, wd: float, w: np.ndarray, g: np.ndarray,
                 last: Optional[np.ndarray], s: np.ndarray, blas: bool = False) -> None:
    """The replica optimiser step of one task (kernels/optimisers/sma.cu:3-100), in place.

    ``rate`` is the negated learning rate (sma.cu:43).  ``blas=True`` replays
    the reference's cuBLAS/memcpy call sequence on OpenBLAS instead.
    """
    if momentum > 0 and last is None:
        raise ValueError("momentum > 0 needs the replica's `last` buffer (model.c:116-120)")
    lp = _fp(last) if last is not None else ctypes.POINTER(ctypes.c_float)()
    if blas:
        if not lib().cbo_blas_is_open():
            blas_open()
        rc = lib().cbo_sma_optimise_blas(w.size, rate, momentum, wd, _fp(w), _fp(g), lp, _fp(s))
        if rc != 0:
            raise RuntimeError("OpenBLAS replay unavailable")
    else:
        lib().cbo_sma_optimise(w.size, rate, momentum, wd, _fp(w), _fp(g), lp, _fp(s))


def default_task(rate: float, momentum: float, wd: float, w: np.ndarray, g: np.ndarray,
                 last: Optional[np.ndarray], z: np.ndarray, blas: bool = False) -> None:
    """DEFAULT task step (kernels/optimisers/default.cu:3-131), in place on w, g,
    last and the device's base model z.  ``rate`` is the negated learning rate."""
    if momentum > 0 and last is None:
        raise ValueError("momentum > 0 needs the replica's `last` buffer (model.c:116-120)")
    lp = _fp(last) if last is not None else ctypes.POINTER(ctypes.c_float)()
    if blas:
        if not lib().cbo_blas_is_open():
            blas_open()
        if lib().cbo_default_task_blas(w.size, rate, momentum, wd, _fp(w), _fp(g), lp, _fp(z)) != 0:
            raise RuntimeError("OpenBLAS replay unavailable")
    else:
        lib().cbo_default_task(w.size, rate, momentum, wd, _fp(w), _fp(g), lp, _fp(z))


def default_sync(st: SmaState) -> None:
    """DEFAULT barrier, single GPU (synch/default.c:5-43): w_i = z for locked i >= first."""
    if st.G != 1:
        raise ValueError("multi-GPU DEFAULT synchronisation is err() in the reference (default.c:46-51)")
    lib().cbo_default_sync(st.size, st.n, _fp(st.z[0]), _fpp(st.w),
                           st.locked.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), st.first)


def ssgd_worker(rate: float, wd: float, w: np.ndarray, g: np.ndarray, acc: np.ndarray, blas: bool = False) -> None:
    """S-SGD task step (kernels/optimisers/synchronoussgd.cu:3-56), in place on g and acc."""
    if blas:
        if not lib().cbo_blas_is_open():
            blas_open()
        if lib().cbo_ssgd_worker_blas(w.size, rate, wd, _fp(w), _fp(g), _fp(acc)) != 0:
            raise RuntimeError("OpenBLAS replay unavailable")
    else:
        lib().cbo_ssgd_worker(w.size, rate, wd, _fp(w), _fp(g), _fp(acc))


def ssgd_sync(st: SmaState, acc: List[np.ndarray], wpc: int, blas: bool = False) -> None:
    """S-SGD barrier (synch/synchronoussgd.c:13-106) on ``st`` (z, last, w) and the
    per-device accumulators ``acc``, in place.  ``st.momentum`` is the base momentum."""
    lp = _fpp(st.last) if st.last is not None else _fpp([None] * st.G)
    args = (st.G, st.size, st.n, int(wpc), st.momentum, _fpp(st.z), lp, _fpp(st.w), _fpp(acc),
            st.locked.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), st.first)
    if blas:
        if not lib().cbo_blas_is_open():
            blas_open()
        if lib().cbo_ssgd_sync_blas(*args, _fp(np.empty(2 * st.n, np.float32))) != 0:
            raise RuntimeError("OpenBLAS replay unavailable")
    else:
        lib().cbo_ssgd_sync(*args, _fp(np.empty(st.n, np.float32)))


def bn_average(mean: List[List[np.ndarray]], var: List[List[np.ndarray]], updated) -> None:
    """BN running-stat averaging (cudnn/cudnnbatchnormparams.c:157-222), in place.

    ``mean[g][l]`` / ``var[g][l]``: layer l's buffers on device g;
    ``updated[g][l]``: that layer had updates on device g since the last call.
    """
    G, L = len(mean), len(mean[0])
    elements = np.array([m.size for m in mean[0]], dtype=np.int32)
    flat_m = [mean[g][l] for g in range(G) for l in range(L)]
    flat_v = [var[g][l] for g in range(G) for l in range(L)]
    upd = np.ascontiguousarray(np.asarray(updated, dtype=np.int32).reshape(G * L))
    lib().cbo_bn_average(G, L, elements.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _fpp(flat_m), _fpp(flat_v),
                         upd.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))


def openblas_path() -> Optional[str]:
    """Locate an OpenBLAS shared object with 32-bit-int cblas (the numpy/scipy wheels')."""
    cands = []
    try:
        import scipy  # noqa: F401
        cands += glob.glob(os.path.join(os.path.dirname(os.path.dirname(scipy.__file__)),
                                        "scipy.libs", "libscipy_openblas-*.so"))
    except Exception:
        pass
    for c in ("libopenblas.so.0", "libopenblas.so"):
        cands.append(c)
    for c in cands:
        h = None
        try:
            h = ctypes.CDLL(c)
        except OSError:
            continue
        if hasattr(h, "cblas_saxpy") or hasattr(h, "scipy_cblas_saxpy"):
            return c
    return None


def blas_open(path: Optional[str] = None) -> str:
    path = path or openblas_path()
    rc = lib().cbo_blas_open(path.encode() if path else None)
    if rc != 0:
        raise RuntimeError(f"OpenBLAS not available (rc={rc}, tried {path})")
    return lib().cbo_blas_name().decode()


def blas_set_threads(k: int) -> None:
    lib().cbo_blas_set_threads(int(k))


def sma_step_blas(st: SmaState) -> int:
    """One SMA step replaying the reference's BLAS call sequence, in place."""
    if not lib().cbo_blas_is_open():
        blas_open()
    return _step(lib().cbo_sma_blas, st, 2 * st.G * st.n + st.n)


def bind_core(core: int) -> int:
    return lib().cbo_bind_core(core)


def unbind() -> int:
    return lib().cbo_unbind()


def now() -> float:
    return lib().cbo_now()


def bytes_per_step(n: int, R: int, momentum: float, G: int = 1) -> int:
    """Algorithmic HBM bytes per step per GPU."""
    m = 1 if momentum > 0 else 0
    if G == 1:
        return (12 * R + 8 + 8 * m) * n
    return (12 * R + 8) * n + (12 + 8 * m) * n
