"""The largest model the boundary takes, on the GPU (run with -m gpu).

The natives take the model size as a Java int (TheGPU.setModel(II),
TheGPU.java:268; the reference's `int bytes`, model.h:35), so a model is at
most 2^31 - 1 bytes: n = 536,870,911 floats, whose last byte offsets reach
2^31, where signed 32-bit arithmetic would turn negative.  (The kernels'
own limit is 4 GiB per buffer: unsigned 32-bit byte offsets from a uniform
base, crossbow_amd/csrc/sma_kernels.hip.)  At that size the step is checked
bit for bit against the oracle in every element (through byte offset 2^30
and the ragged tail below 2^31), and by the size-independent conservation
checksum
z' + sum_i w_i' = z + sum_i w_i + 0.9 last, summed on the device in fp64.
Both the fused kernel and the split pipeline (kernel A / one-rank all-reduce /
kernel B over buckets, i.e. per-bucket base offsets) run.  A size that does
not fit a Java int is refused by the wrapper instead of wrapping round.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import assert_bitexact, make_gpu

pytestmark = pytest.mark.gpu

N_MAX = (2**31 - 1) // 4  # 536,870,911 floats = 2,147,483,644 bytes


class _Dev:
    """A zero-copy view of a library device buffer for torch."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False),
                                         "version": 3, "strides": None}


def _view(ptr, n):
    import torch
    return torch.as_tensor(_Dev(ptr, n), device="cuda")


def test_one_past_the_limit_is_refused():
    from crossbow_amd import CbxError, TheGPU
    g = TheGPU()
    g.init([0])
    try:
        with pytest.raises(CbxError, match="Java int"):
            g.setModel(1, 4 * (N_MAX + 1))
        with pytest.raises(CbxError, match="Java int"):
            g.setModelVariable(0, 1, [N_MAX + 1], 4 * (N_MAX + 1))
    finally:
        g.free()


@pytest.mark.timeout(330)
@pytest.mark.parametrize("split", [False, True])
def test_max_size_parity_every_element_and_conservation(split):
    # Every element of z, last and both w against the oracle (no
    # sample): the inputs are cloned on the device before the step, then
    # inputs and outputs come down chunk by chunk (the step is elementwise)
    # and the oracle runs on each chunk.
    import torch
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_LAST
    n, R = N_MAX, 2  # ragged: n % 4 == 3
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        if split:
            g.set_force_split(True)
            g.set_bucket_elements(100_000_000)  # 6 buckets, the last one ragged
        g.fill_synthetic(O.SEED)
        g.wait()
        z, last = _view(g.base_buffer(0, BUF_DATA), n), _view(g.base_buffer(0, BUF_LAST), n)
        s = [_view(g.replica_buffer(i, BUF_DIFF), n) for i in range(R)]
        w = [_view(g.replica_buffer(i, BUF_DATA), n) for i in range(R)]

        def total(ts):
            return sum(float(torch.sum(t, dtype=torch.float64)) for t in ts)

        torch.cuda.synchronize()
        z0, l0, w0 = z.clone(), last.clone(), [t.clone() for t in w]  # s is not written by the step
        before = total([z] + w) + 0.9 * total([last])
        g.lockAny()
        g.synchronise(0, 1, 0, False)
        g.unlockAny()
        g.wait()
        torch.cuda.synchronize()
        after = total([z] + w)
        assert abs(after - before) <= 1e-6 * max(1.0, abs(before)) + 1e-1, (after, before)
        chunk, compared = 1 << 26, 0
        for a in range(0, n, chunk):
            b = min(n, a + chunk)

            def host(t):
                return t[a:b].cpu().numpy()

            st = O.SmaState(1, R, b - a, 0.1, 0.9, [host(z0)], [host(l0)], [host(t) for t in s], [host(t) for t in w0])
            O.sma_step(st)
            assert_bitexact(host(z), st.z[0], f"z[{a}:{b}]")
            assert_bitexact(host(last), st.last[0], f"last[{a}:{b}]")
            for i in range(R):
                assert_bitexact(host(w[i]), st.w[i], f"w[{i}][{a}:{b}]")
            compared += (2 + R) * (b - a)
        assert compared == (2 + R) * n
        print(f"max size ({'split' if split else 'fused'}): {compared} elements compared bit for bit (n = {n})")
    finally:
        g.free()
