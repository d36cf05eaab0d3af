"""Shared test helpers: drive the HIP path through the C-ABI and compare with
the CPU oracle on identical inputs (oracle/ is test infrastructure)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


def bits(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def assert_bitexact(got: np.ndarray, want: np.ndarray, what: str = "") -> None:
    g, w = bits(got), bits(want)
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        k = bad[0]
        raise AssertionError(f"{what}: {bad.size} of {g.size} elements differ; first at {k}: "
                             f"got {got[k]!r} want {want[k]!r}")


def make_gpu(n: int, R: int, alpha: float, momentum: float, sync: int = 0, update_type: int = 7,
             devices=(0,)):
    from crossbow_amd import TheGPU
    g = TheGPU()
    g.init(list(devices))
    g.setModel(1, 4 * n)
    g.setModelVariable(0, 1, [n], 4 * n)
    g.setUpdateModelType(update_type)
    g.setEamsgdAlpha(alpha)
    g.setMomentum(momentum, 0)
    g.setModelManager(R, sync)
    return g


def upload(g, st: O.SmaState) -> None:
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_LAST
    for dev in range(st.G):
        g.base_write(dev, BUF_DATA, st.z[dev])
        if st.last is not None:
            g.base_write(dev, BUF_LAST, st.last[dev])
    for i in range(st.size):
        g.replica_write(i, BUF_DIFF, st.s[i])
        g.replica_write(i, BUF_DATA, st.w[i])


def download(g, st: O.SmaState) -> O.SmaState:
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_LAST
    out = st.clone()
    for dev in range(st.G):
        out.z[dev] = g.base_read(dev, BUF_DATA)
        if st.last is not None:
            out.last[dev] = g.base_read(dev, BUF_LAST)
    for i in range(st.size):
        out.s[i] = g.replica_read(i, BUF_DIFF)
        out.w[i] = g.replica_read(i, BUF_DATA)
    return out


def compare_states(got: O.SmaState, want: O.SmaState, exact: bool = True, rtol=1e-5, atol=1e-6) -> None:
    pairs = [("z", got.z, want.z), ("w", got.w, want.w), ("s", got.s, want.s)]
    if want.last is not None:
        pairs.append(("last", got.last, want.last))
    for name, G_, W_ in pairs:
        for k, (a, b) in enumerate(zip(G_, W_)):
            if exact:
                assert_bitexact(a, b, f"{name}[{k}]")
            else:
                np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=f"{name}[{k}]")
