"""GPU parity of the fused replica optimiser step.

``cbx_replica_optimise`` restates crossbowKernelOptimiserSMA
(clib-multigpu/kernels/optimisers/sma.cu:3-100): weight decay, learning-rate
scale, momentum, the snapshot ``diff <- data`` and the update, in one pass.
Checked bit for bit against the oracle (which is itself pinned to the
reference's saxpy/sscal/memcpy sequence on OpenBLAS, tests/test_oracle.py),
alone and inside a whole clock loop (local steps, then synchronise).
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import assert_bitexact

pytestmark = pytest.mark.gpu


def _gpu(n, R, momentum, wd, alpha=0.1, policy=None):
    from crossbow_amd import TheGPU
    g = TheGPU()
    g.init([0])
    g.setModel(1, 4 * n)
    g.setModelVariable(0, 1, [n], 4 * n)
    g.setUpdateModelType(7)
    g.setEamsgdAlpha(alpha)
    g.setMomentum(momentum, 0)
    g.setWeightDecay(wd)
    if policy is None:
        g.setLearningRateDecayPolicyFixed(0.05)
    else:
        policy(g)
    g.setModelManager(R, 0)
    return g


AUX_CONFIGS = [None, (64, 2, 2), (256, 1, 0), (512, 1, 8)]


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("wd", [0.0, 5e-4])
@pytest.mark.parametrize("on_torch_stream", [False, True])
@pytest.mark.parametrize("aux", AUX_CONFIGS)
def test_optimise_bitexact(momentum, wd, on_torch_stream, aux):
    import torch
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_GRADIENT, BUF_LAST
    n, R = 70_001, 2
    g = _gpu(n, R, momentum, wd)
    try:
        if aux:
            g.set_aux_kernel_config(*aux)
        stream = torch.cuda.Stream() if on_torch_stream else None
        for i in range(R):
            w = O.fill_normal(n, 300 + i, 0.05)
            gr = O.fill_normal(n, 310 + i, 0.01)
            last = O.fill_normal(n, 320 + i, 0.001) if momentum > 0 else None
            s = np.zeros(n, np.float32)
            g.replica_write(i, BUF_DATA, w)
            g.replica_write(i, BUF_GRADIENT, gr)
            if last is not None:
                g.replica_write(i, BUF_LAST, last)
            g.replica_optimise(i, task=i, stream=stream.cuda_stream if stream else None)
            g.wait()
            O.sma_optimise(np.float32(-0.05), momentum, wd, w, gr, last, s)
            assert_bitexact(g.replica_read(i, BUF_DATA), w, f"w[{i}]")
            assert_bitexact(g.replica_read(i, BUF_DIFF), s, f"s[{i}]")
            assert_bitexact(g.replica_read(i, BUF_GRADIENT), gr, f"g[{i}]")
            if last is not None:
                assert_bitexact(g.replica_read(i, BUF_LAST), last, f"last[{i}]")
    finally:
        g.free()


def test_multistep_learning_rate_raises_copy():
    # solverconfiguration.c:128-136: crossing a step divides the rate by 1/gamma
    # and raises _copy, which the next synchronise turns into Phase D.
    from crossbow_amd import BUF_DATA, BUF_GRADIENT
    n, R = 8192, 2
    g = _gpu(n, R, 0.0, 0.0, policy=lambda h: h.setLearningRateDecayPolicyMultiStep(0.1, 0.5, 0, [3]))
    try:
        assert g.replica_learning_rate(1, 0) == pytest.approx(0.1)
        w = O.fill_normal(n, 400, 0.05)
        gr = O.fill_normal(n, 401, 0.01)
        g.replica_write(0, BUF_DATA, w)
        g.replica_write(0, BUF_GRADIENT, gr)
        g.replica_optimise(0, task=1)  # task+1 = 2 < 3
        assert g.replica_copy(0) == 0
        g.replica_optimise(0, task=2)  # task+1 = 3 >= 3: step, rate 0.05, copy
        assert g.replica_copy(0) == 1
        g.wait()
        s = np.zeros(n, np.float32)
        O.sma_optimise(np.float32(-0.1), 0.0, 0.0, w, gr, None, s)
        O.sma_optimise(np.float32(-0.1) * np.float32(0.5), 0.0, 0.0, w, gr, None, s)
        assert_bitexact(g.replica_read(0, BUF_DATA), w, "w after two steps")
        # the next barrier copies the base model to every replica and resets _copy
        g.lockAny()
        g.synchronise(0, 1, 0, False)
        g.unlockAny()
        g.wait()
        z = g.base_read(0, BUF_DATA)
        for i in range(R):
            assert_bitexact(g.replica_read(i, BUF_DATA), z, f"w[{i}] == z after Phase D")
        assert g.replica_copy(0) == 0
    finally:
        g.free()


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_clock_loop_bitexact(momentum):
    # The whole per-clock loop of the SMA model on one GPU: every replica runs
    # `wpc` local steps (a fresh gradient per task), then the barrier averages.
    from crossbow_amd import BUF_DATA, BUF_GRADIENT, BUF_LAST
    from tests.helpers import compare_states, download, upload
    n, R, clocks, wpc, alpha = 33_333, 3, 3, 2, 0.1
    g = _gpu(n, R, momentum, 1e-4, alpha=alpha)
    try:
        st = O.make_state(n, 1, R, alpha, momentum)
        upload(g, st)
        lasts = [np.zeros(n, np.float32) if momentum > 0 else None for _ in range(R)]
        task = 0
        for clock in range(1, clocks + 1):
            for i in range(R):
                for _ in range(wpc):
                    gr = O.fill_normal(n, 1000 + task, 0.01)
                    g.replica_write(i, BUF_GRADIENT, gr)
                    g.replica_optimise(i, task)
                    O.sma_optimise(np.float32(-0.05), momentum, 1e-4, st.w[i], gr, lasts[i], st.s[i])
                    task += 1
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
            O.sma_step(st)
        g.wait()
        compare_states(download(g, st), st)
        if momentum > 0:
            for i in range(R):
                assert_bitexact(g.replica_read(i, BUF_LAST), lasts[i], f"replica last[{i}]")
        assert_bitexact(g.replica_read(0, BUF_DATA), st.w[0], "w[0]")
    finally:
        g.free()


def _busy(torch, stream, ms=2.0):
    """Hold `stream` for about `ms` milliseconds before whatever is queued next."""
    with torch.cuda.stream(stream):
        try:
            torch.cuda._sleep(int(ms * 2.1e6))  # ~2.1 GHz shader clock
        except (AttributeError, RuntimeError):
            a = torch.randn(2048, 2048, device="cuda")
            for _ in range(8):
                a = a @ a * 1e-3


def _busy_task_main(momentum, fault, q):
    import os
    # 16 hardware queues give every task stream a queue of its own: at HIP's
    # default 4 a later stream can share the sync stream's queue, whose
    # in-order execution would hide a missing wait
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
    if fault:
        os.environ["CBX_FAULT_SKIP_TASK_WAIT"] = "1"  # read at context creation
    try:
        q.put((_busy_task_loop(momentum), None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((None, traceback.format_exc()))


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("fault", [False, True])
def test_clock_loop_on_busy_task_streams_bitexact(momentum, fault):
    # Each replica's optimiser step on a task stream of its own that is busy
    # for ~2 ms before it, and the barrier enqueued at once behind them: the
    # sync stream's wait for every task stream is deferred to the barrier's
    # entry (flush_task_waits), so the averaging still reads the
    # updated w and s, bit for bit.  With the waits dropped
    # ($CBX_FAULT_SKIP_TASK_WAIT) the same loop must come out wrong: the
    # check is sensitive to the ordering it relies on.  A fresh process each.
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_busy_task_main, args=(momentum, fault, q))
    p.start()
    bad, err = q.get(timeout=240)
    p.join(60)
    assert err is None, err
    if fault:
        assert bad, "the race went unseen: the fault switch did nothing"
    else:
        assert not bad, bad


def _busy_task_loop(momentum):
    import torch

    from tests.helpers import compare_states, download, upload
    n, R, clocks, alpha = 1 << 20, 3, 2, 0.1
    g = _gpu(n, R, momentum, 1e-4, alpha=alpha)
    streams = [torch.cuda.Stream() for _ in range(R)]
    try:
        st = O.make_state(n, 1, R, alpha, momentum)
        upload(g, st)
        lasts = [np.zeros(n, np.float32) if momentum > 0 else None for _ in range(R)]
        grads = [O.fill_normal(n, 7000 + i, 0.01) for i in range(R)]
        from crossbow_amd import BUF_GRADIENT
        task = 0
        for clock in range(1, clocks + 1):
            for i in range(R):
                g.replica_write(i, BUF_GRADIENT, grads[i])
            torch.cuda.synchronize()
            for i in range(R):
                _busy(torch, streams[i])
                g.replica_optimise(i, task, streams[i].cuda_stream)
                task += 1
            g.lockAny()
            g.synchronise(0, clock, 0, False)  # right behind the launches: no host wait, no host work
            g.unlockAny()
            for i in range(R):  # the oracle after the enqueue, so the host takes no time in between
                O.sma_optimise(np.float32(-0.05), momentum, 1e-4, st.w[i], grads[i], lasts[i], st.s[i])
            O.sma_step(st)
        g.wait()
        torch.cuda.synchronize()
        try:
            compare_states(download(g, st), st)
        except AssertionError as e:
            return str(e)[:300]
        return None
    finally:
        torch.cuda.synchronize()
        g.free()


def test_nesterov_is_unsupported():
    from crossbow_amd import CbxError, TheGPU, _lib
    n = 4096
    g = TheGPU()
    g.init([0])
    try:
        g.setModel(1, 4 * n)
        g.setModelVariable(0, 1, [n], 4 * n)
        g.setUpdateModelType(7)
        g.setMomentum(0.9, 1)  # NESTEROV (utils.h:101)
        g.setLearningRateDecayPolicyFixed(0.1)
        g.setModelManager(1, 0)
        with pytest.raises(CbxError) as e:
            g.replica_optimise(0, 0)
        assert e.value.code == _lib.CBX_ERR_UNSUPPORTED
    finally:
        g.free()


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("split", [False, True, 4096, 16_384])
@pytest.mark.parametrize("aux", AUX_CONFIGS)
def test_ssgd_clock_loop_bitexact(momentum, split, aux):
    # Synchronous SGD (update model WORKER): task steps add
    # lr-scaled gradients into the base gradient; the barrier all-reduces it,
    # scales by 1/wpc, applies base momentum and copies z to every replica.
    from crossbow_amd import BUF_DATA, BUF_GRADIENT, BUF_LAST, TheGPU
    from tests.helpers import upload
    n, R, wpc, clocks = 50_001, 3, 6, 2
    g = TheGPU()
    g.init([0])
    try:
        g.setModel(1, 4 * n)
        g.setModelVariable(0, 1, [n], 4 * n)
        g.setModelWorkPerClock(wpc)
        g.setUpdateModelType(1)
        g.setMomentum(momentum, 0)
        g.setWeightDecay(1e-4)
        g.setLearningRateDecayPolicyFixed(0.05)
        g.setModelManager(R, 1)  # SSP: the barrier may skip a busy replica
        if aux:
            g.set_aux_kernel_config(*aux)
            g.set_barrier_kernel_config(*aux)
        if split:
            g.set_force_split(True)
            if split is not True:  # bucketed barrier: all-reduce of bucket k+1 beside the apply of bucket k
                g.set_bucket_elements(split)
        st = O.make_state(n, 1, R, 0.1, momentum)
        st.locked[2] = 0  # hold replica 2 (SSP): not copied at the barrier
        upload(g, st)
        acc = [np.zeros(n, np.float32)]
        task = 0
        for clock in range(1, clocks + 1):
            for k in range(wpc):
                i = k % R
                gr = O.fill_normal(n, 2000 + task, 0.01)
                g.replica_write(i, BUF_GRADIENT, gr)
                g.replica_optimise(i, task)
                O.ssgd_worker(np.float32(-0.05), 1e-4, st.w[i], gr, acc[0])
                task += 1
            g.replica_lock(2)
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
            g.replica_unlock(2)
            O.ssgd_sync(st, acc, wpc)
        g.wait()
        assert_bitexact(g.base_read(0, BUF_DATA), st.z[0], "z")
        assert_bitexact(g.base_read(0, BUF_GRADIENT), acc[0], "base gradient reset")
        if momentum > 0:
            assert_bitexact(g.base_read(0, BUF_LAST), st.last[0], "last")
        for i in range(R):
            assert_bitexact(g.replica_read(i, BUF_DATA), st.w[i], f"w[{i}]")
    finally:
        g.free()


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("on_torch_stream", [False, True])
@pytest.mark.parametrize("aux", [None, (64, 2, 2)])
def test_default_clock_loop_bitexact(momentum, on_torch_stream, aux):
    # Update model DEFAULT (0), the reference apps' default: every task step
    # moves the replica and the base model by the same gradient
    # (kernels/optimisers/default.cu:3-131), the barrier copies the base model
    # to the locked replicas (synch/default.c:5-43).  SSP holds replica 2.
    import torch
    from crossbow_amd import BUF_DATA, BUF_GRADIENT, BUF_LAST, UPDATE_DEFAULT, TheGPU
    from tests.helpers import upload
    n, R, tasks, clocks = 50_001, 3, 5, 2
    g = TheGPU()
    g.init([0])
    try:
        g.setModel(1, 4 * n)
        g.setModelVariable(0, 1, [n], 4 * n)
        g.setUpdateModelType(UPDATE_DEFAULT)
        g.setMomentum(momentum, 0)
        g.setWeightDecay(1e-4)
        g.setLearningRateDecayPolicyFixed(0.05)
        g.setModelManager(R, 1)
        if aux:
            g.set_aux_kernel_config(*aux)
            g.set_barrier_kernel_config(*aux)
        st = O.make_state(n, 1, R, 0.1, momentum)
        st.locked[2] = 0
        upload(g, st)
        lasts = [O.fill_normal(n, 700 + i, 0.001) if momentum > 0 else None for i in range(R)]
        for i in range(R):
            if lasts[i] is not None:
                g.replica_write(i, BUF_LAST, lasts[i])
        stream = torch.cuda.Stream() if on_torch_stream else None
        task = 0
        for clock in range(1, clocks + 1):
            for k in range(tasks):
                i = k % R
                gr = O.fill_normal(n, 3000 + task, 0.01)
                g.replica_write(i, BUF_GRADIENT, gr)
                g.replica_optimise(i, task, stream.cuda_stream if stream else None)
                O.default_task(np.float32(-0.05), momentum, 1e-4, st.w[i], gr, lasts[i], st.z[0])
                if stream is not None:
                    stream.synchronize()
                g.wait()
                assert_bitexact(g.replica_read(i, BUF_GRADIENT), gr, f"g[{i}] task {task}")
                task += 1
            g.replica_lock(2)
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
            g.replica_unlock(2)
            O.default_sync(st)
        g.wait()
        assert_bitexact(g.base_read(0, BUF_DATA), st.z[0], "z")
        for i in range(R):
            assert_bitexact(g.replica_read(i, BUF_DATA), st.w[i], f"w[{i}]")
            if lasts[i] is not None:
                assert_bitexact(g.replica_read(i, BUF_LAST), lasts[i], f"last[{i}]")
        assert not np.array_equal(st.w[2], st.z[0]), "the held replica is not copied"
    finally:
        g.free()


@pytest.mark.parametrize("pipeline", ["fused", "cross-step", "cross-step-stride"])
def test_threaded_clock_loop_bitexact(pipeline):
    # The clock loop with the reference's threading: one task thread per
    # replica, each on its own task (torch) stream, locking its replica,
    # running its optimiser steps and releasing it; the result-collector
    # thread runs the barrier once every task of the clock is done.  The
    # optimiser kernels of different replicas interleave on the sync stream
    # in whatever order the threads enqueue them, but touch disjoint
    # replicas, so the result is deterministic: bit-exact vs the oracle.
    import threading

    import torch

    from crossbow_amd import BUF_GRADIENT
    from tests.helpers import compare_states, download, upload
    n, R, clocks, wpc, alpha, momentum = 65_537, 4, 4, 3, 0.1, 0.9
    g = _gpu(n, R, momentum, 1e-4, alpha=alpha)
    try:
        if pipeline.startswith("cross-step"):
            g.set_force_split(True)
            g.set_bucket_elements(8192)
            g.set_pipeline_mode(1)
            g.set_cross_wait_stride(2 if pipeline.endswith("stride") else 1)
        st = O.make_state(n, 1, R, alpha, momentum)
        upload(g, st)
        lasts = [np.zeros(n, np.float32) for _ in range(R)]
        grads = {(c, i, k): O.fill_normal(n, 20_000 + 100 * c + 10 * i + k, 0.01)
                 for c in range(clocks) for i in range(R) for k in range(wpc)}
        streams = [torch.cuda.Stream() for _ in range(R)]
        errors = []

        def worker(i, clock):
            try:
                with torch.cuda.stream(streams[i]):
                    for k in range(wpc):
                        g.replica_lock(i)
                        g.replica_write(i, BUF_GRADIENT, grads[(clock, i, k)])
                        g.replica_optimise(i, (clock * R + i) * wpc + k, streams[i].cuda_stream)
                        g.replica_task_done(i)
                        g.replica_unlock(i)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        for clock in range(clocks):
            threads = [threading.Thread(target=worker, args=(i, clock)) for i in range(R)]
            for t in threads:
                t.start()
            for t in threads:
                t.join(timeout=60)
            assert not errors, errors
            for i in range(R):
                for k in range(wpc):
                    O.sma_optimise(np.float32(-0.05), momentum, 1e-4, st.w[i], grads[(clock, i, k)], lasts[i],
                                   st.s[i])
            assert g.lockAny() == R
            g.synchronise(0, clock + 1, 0, False)
            g.unlockAny()
            O.sma_step(st)
        g.wait()
        torch.cuda.synchronize()
        compare_states(download(g, st), st)
    finally:
        g.free()


def _hip():
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    for name, args in (("hipStreamCreateWithFlags", [ctypes.c_void_p, ctypes.c_uint]),
                       ("hipStreamDestroy", [ctypes.c_void_p]), ("hipStreamSynchronize", [ctypes.c_void_p]),
                       ("hipEventCreateWithFlags", [ctypes.c_void_p, ctypes.c_uint]),
                       ("hipEventRecord", [ctypes.c_void_p, ctypes.c_void_p]),
                       ("hipStreamWaitEvent", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]),
                       ("hipEventDestroy", [ctypes.c_void_p])):
        getattr(hip, name).argtypes = args
        getattr(hip, name).restype = ctypes.c_int
    return hip


def test_task_wait_table_stays_bounded_over_1000_task_streams():
    # VERDICT r05 Weak #6: one deferred-wait entry per caller stream, never
    # pruned.  1,000 task streams, each created, given one replica update
    # (cbx_replica_optimise) and destroyed: first each drained and destroyed
    # before the next (the table must not grow at all), then chained by
    # events behind a ~1 s head and destroyed only after the barrier (HIP's
    # hipStreamDestroy drains the stream): every entry stays incomplete, so
    # the table must stop at its cap of 64, by queuing the waits on the sync
    # stream.  The whole sequence, and the barrier after it, bit for bit
    # against the oracle.
    import ctypes

    import torch

    from crossbow_amd import BUF_DATA, BUF_GRADIENT, BUF_LAST
    from tests.helpers import compare_states, download, upload
    hip = _hip()
    n, R, momentum, wd, alpha = 65_536, 2, 0.9, 1e-4, 0.1
    g = _gpu(n, R, momentum, wd, alpha=alpha)
    try:
        st = O.make_state(n, 1, R, alpha, momentum)
        upload(g, st)
        grads = [O.fill_normal(n, 9100 + i, 0.01) for i in range(R)]
        lasts = [np.zeros(n, np.float32) for _ in range(R)]
        for i in range(R):
            g.replica_write(i, BUF_GRADIENT, grads[i])
            g.replica_write(i, BUF_LAST, lasts[i])
        g.wait()
        counts, prev, live = [], None, []
        for k in range(1000):
            chained = k >= 500
            s, e = ctypes.c_void_p(), ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
            if chained and prev is not None:
                assert hip.hipStreamWaitEvent(s, prev, 0) == 0
            elif chained:  # the chain's head holds every later update back ~1 s: entries pile up to the cap
                _busy(torch, torch.cuda.ExternalStream(s.value), ms=1000.0)
            i = k % R
            g.replica_optimise(i, k, s.value)
            O.sma_optimise(np.float32(-0.05), momentum, wd, st.w[i], grads[i], lasts[i], st.s[i])
            if chained:
                assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0
                assert hip.hipEventRecord(e, s) == 0
                if prev is not None:
                    assert hip.hipEventDestroy(prev) == 0
                prev = e
                live.append(s)  # hipStreamDestroy would drain it: these go after the barrier
            else:
                assert hip.hipStreamSynchronize(s) == 0
                assert hip.hipStreamDestroy(s) == 0
            counts.append(g.task_wait_count(0))
        g.lockAny()
        g.synchronise(0, 1, 0, False)  # waits for every update (flush_task_waits)
        g.unlockAny()
        O.sma_step(st)
        g.wait()
        if prev is not None:
            assert hip.hipEventDestroy(prev) == 0
        for s in live:
            assert hip.hipStreamDestroy(s) == 0
        print(f"task-wait table: max {max(counts[:500])} entries unchained, max {max(counts[500:])} chained")
        assert max(counts[:500]) <= 2, counts[:500]
        assert max(counts[500:]) == 64, max(counts[500:])
        compare_states(download(g, st), st)
        for i in range(R):
            assert_bitexact(g.replica_read(i, BUF_LAST), lasts[i], f"replica last[{i}]")
            assert_bitexact(g.replica_read(i, BUF_GRADIENT), grads[i], f"g[{i}]")
        assert_bitexact(g.replica_read(0, BUF_DATA), st.w[0], "w[0]")
    finally:
        g.free()
