"""HIP SMA path vs the CPU oracle, through the C-ABI (run with -m gpu).

Bar: at G = 1 the HIP kernels use the reference's fp32
operation order (cuBLAS saxpy = fma), so results must be BIT-EXACT with the
oracle (oracle/sma_oracle.c, restating clib-multigpu/synch/sma.c:13-231).
"""
from __future__ import annotations

import os
import tempfile

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import assert_bitexact, compare_states, download, make_gpu, upload

pytestmark = pytest.mark.gpu


def _run(n, R, alpha, momentum, copy_ids=(), first=0, held=(), sync=0, config=None, split=False,
         bucket=0, steps=1, apply=None, algo=0):
    st = O.make_state(n, 1, R, alpha, momentum)
    g = make_gpu(n, R, alpha, momentum, sync=sync)
    try:
        if config:
            config = dict(config)
            occ = config.pop("occupancy", 0)
            g.set_kernel_config(**config)
            g.set_kernel_occupancy(occ)
        if split:
            g.set_force_split(True)
        if algo:
            g.set_allreduce_algorithm(algo)
        if apply:
            g.set_apply_kernel_config(*apply)
        if bucket:
            g.set_bucket_elements(bucket)
        upload(g, st)
        want = st.clone()
        for _ in range(steps):
            for i in copy_ids:
                g.set_replica_copy(i, True)
                want.copy[i] = 1
            for i in held:
                g.replica_lock(i)
            locked = g.lockAny()
            want.locked[:] = 1
            for i in held:
                want.locked[i] = 0
            if sync == 0:
                assert locked == R
            else:
                assert locked == R - len(held)
            want.first = first
            g.synchronise(first, 1, 0, False)
            assert g.unlockAny() == R - len(held)
            for i in held:
                g.replica_unlock(i)
            O.sma_step(want)
        g.wait()
        got = download(g, st)
        compare_states(got, want)
        for i in copy_ids:
            assert g.replica_copy(i) == 0, "Phase D must reset _copy (sma.c:220)"
    finally:
        g.free()


@pytest.mark.parametrize("R", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fused_bitexact(R, momentum):
    _run(4099, R, 0.1, momentum)


@pytest.mark.parametrize("R", [9, 16])
def test_fused_generic_replica_count(R):
    # > 8 replicas per GPU takes the chunked (register-resident groups of 8) kernel.
    _run(1031, R, 0.1, 0.9)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 63, 64, 65, 255, 257, 4096 * 16 + 1])
@pytest.mark.parametrize("split", [False, True])
def test_tiny_and_ragged_sizes(n, split):
    # Sub-float4 and wave-boundary sizes: the float4 tail lives in the arena's
    # padding, which the step must never let leak into the n real elements.
    _run(n, 3, 0.1, 0.9, split=split, copy_ids=(0,) if n % 2 else (), steps=2)


@pytest.mark.parametrize("R", [9, 17, 64])
def test_chunked_replicas_split_path(R):
    # > 8 replicas per GPU in kernel A (chunks of 8) and the maximum, 64, fused.
    _run(2053, R, 0.1, 0.9, split=True, steps=2)
    if R == 64:
        _run(2053, R, 0.1, 0.9, steps=2)


@pytest.mark.parametrize("alpha", [0.0, 1.0, 1e-30])
def test_alpha_extremes(alpha):
    # alpha 0: replicas and acc unchanged, z moves by momentum only;
    # alpha 1: replicas jump by their whole elastic difference; denormal-range alpha.
    _run(4099, 4, alpha, 0.9)
    _run(4099, 4, alpha, 0.9, split=True)


def test_lenet_size_alpha_half():
    # C2: LeNet, 4 replicas on 1 GPU, alpha = 0.5 (SolverConf default).
    _run(1_111_946, 4, 0.5, 0.0)


def test_copy_flag_phase_d():
    # A learning-rate drop on one replica copies the new base model into all.
    _run(4099, 4, 0.1, 0.9, copy_ids=(2,))


def test_first_offset():
    _run(4099, 6, 0.1, 0.9, first=2)


def test_ssp_partial_lock():
    # A replica busy on the task side is skipped by lockAny under SSP.
    _run(4099, 4, 0.1, 0.9, held=(1,), sync=1)


@pytest.mark.parametrize("split", [False, True])
def test_disabled_replica_counted_but_excluded(split):
    # modelmanager.c:217-222: a theta-queue-disabled replica counts toward the
    # BSP barrier but is not locked, so the step, unlockAny and the clock skip it.
    n, R = 4099, 4
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9, sync=0)
    try:
        if split:
            g.set_force_split(True)
        upload(g, st)
        g.set_replica_disabled(2, True)
        assert g.lockAny() == R, "BSP holds: the disabled replica is counted"
        g.synchronise(0, 5, 0, False)
        assert g.unlockAny() == R - 1
        want = st.clone()
        want.locked[2] = 0
        O.sma_step(want)
        g.wait()
        compare_states(download(g, st), want)
        assert g.replica_clock(2) == 0 and g.replica_clock(1) == 5
        # re-enabled, it takes part again
        g.set_replica_disabled(2, False)
        assert g.lockAny() == R
        g.synchronise(0, 6, 0, False)
        assert g.unlockAny() == R
        want.locked[2] = 1
        O.sma_step(want)
        g.wait()
        compare_states(download(g, st), want)
    finally:
        g.free()


def test_bsp_barrier_failure():
    from crossbow_amd import CbxError
    n, R = 1031, 2
    g = make_gpu(n, R, 0.1, 0.0, sync=0)
    try:
        g.replica_lock(1)
        with pytest.raises(CbxError) as e:
            g.lockAny()
        assert "failed to lock all" in str(e.value)
        g.replica_unlock(1)
        assert g.lockAny() == R
        g.unlockAny()
    finally:
        g.free()


@pytest.mark.parametrize("config", [
    dict(block=256, blocks_per_cu=0, policy=0, unroll=1),
    dict(block=256, blocks_per_cu=8, policy=1, unroll=1),
    dict(block=256, blocks_per_cu=4, policy=1, unroll=2),
    dict(block=64, blocks_per_cu=0, policy=1, unroll=4, occupancy=4),
    dict(block=128, blocks_per_cu=0, policy=1, unroll=4, occupancy=0),
    dict(block=64, blocks_per_cu=0, policy=1, unroll=1, occupancy=2),
    dict(block=128, blocks_per_cu=0, policy=1, unroll=1, occupancy=4),
    dict(block=128, blocks_per_cu=0, policy=1, unroll=2),
])
def test_launch_configs_identical(config):
    _run(70_001, 8, 0.1, 0.9, config=config)


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_split_pipeline_one_rank(momentum):
    # Kernel A + RCCL all-reduce (one-rank communicator) + kernel B.
    _run(4099, 4, 0.1, momentum, split=True)


@pytest.mark.parametrize("apply", [(64, 1, -1), (64, 1, 2), (64, 4, 0), (128, 2, 4), (256, 1, 8), (256, 2, -1)])
def test_split_apply_launch_shapes_identical(apply):
    # Kernel B's own launch geometry (cbx_set_apply_kernel_config): ragged n,
    # one bucket and 5 buckets, Phase D on the second step.
    _run(300_001, 3, 0.1, 0.9, split=True, apply=apply, copy_ids=(1,), steps=2)
    _run(300_001, 3, 0.1, 0.9, split=True, apply=apply, bucket=65_536, steps=2)


def test_split_pipeline_buckets_and_copy():
    _run(300_001, 3, 0.1, 0.9, split=True, bucket=65_536, copy_ids=(0,), steps=2)


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("bucket", [0, 65_536, 4096])
def test_split_pipeline_reduce_scatter_one_rank(momentum, bucket):
    # cbx_set_allreduce_algorithm(RSAG): reduce-scatter of acc + the control
    # block's all-reduce, the base momentum on the rank's shard, all-gather,
    # kernel B without momentum.  One rank: the shard is the whole bucket.
    from crossbow_amd._lib import ALLREDUCE_RSAG
    _run(300_001, 3, 0.1, momentum, split=True, bucket=bucket, copy_ids=(1,), steps=3, algo=ALLREDUCE_RSAG)
    _run(4099, 2, 0.5, momentum, split=True, bucket=bucket, held=(0,), sync=1, steps=2, algo=ALLREDUCE_RSAG)


@pytest.mark.parametrize("bucket", [4096, 1_000_000])
def test_split_pipeline_many_buckets_two_streams(bucket):
    # 4096-element buckets -> ~245 buckets per step on two streams with
    # per-bucket events reused across steps; 1e6 > n -> one in-order bucket.
    _run(1_000_003, 2, 0.5, 0.9, split=True, bucket=bucket, steps=3)


@pytest.mark.parametrize("mode", [0, 1])
def test_pipelined_timing_spans(mode):
    """Pipelined steps time their kernels A, collectives and kernels B as
    summed busy spans (each dispatch: its stop minus the latest event that
    bounded its start), so N > 1 benches report the kernels as they ran in
    the timed region; beyond 64 buckets the step keeps no spans (-1)."""
    from crossbow_amd import _lib
    n, R = 300_000, 2
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        g.set_force_split(True)
        g.set_bucket_elements(16_384)  # 19 buckets
        g.set_pipeline_mode(mode)
        g.fill_synthetic(7)
        g.set_timing(True)
        for c in range(6):
            g.lockAny()
            g.synchronise(0, c, 0, False)
            g.unlockAny()
        g.wait()
        t = g.last_timing(0)
        assert t[_lib.T_KERNEL] > 0 and t[_lib.T_ALLREDUCE] > 0 and t[_lib.T_APPLY] > 0 and t[_lib.T_STEP] > 0
        hk = g.timing_history(_lib.T_KERNEL)
        hb = g.timing_history(_lib.T_APPLY)
        hs = g.timing_history(_lib.T_STEP)
        assert len(hk) == 6 and all(x > 0 for x in hk) and all(x > 0 for x in hb) and all(x > 0 for x in hs)
        if mode == 0:  # one stream: A and B never overlap, so their busy time fits in the step
            assert all(k + b <= s * 1.001 + 0.002 for k, b, s in zip(hk, hb, hs)), (hk, hb, hs)
        g.set_bucket_elements(4096)  # 74 buckets (4,096 floats, the smallest): more than the span records keep
        for c in range(6, 8):
            g.lockAny()
            g.synchronise(0, c, 0, False)
            g.unlockAny()
        g.wait()
        t = g.last_timing(0)
        assert t[_lib.T_KERNEL] == -1 and t[_lib.T_APPLY] == -1 and t[_lib.T_STEP] > 0
        g.set_bucket_elements(1 << 40)
        g.lockAny()
        g.synchronise(0, 4, 0, False)
        g.unlockAny()
        t = g.last_timing(0)
        assert t[_lib.T_KERNEL] > 0 and t[_lib.T_ALLREDUCE] > 0 and t[_lib.T_APPLY] > 0
    finally:
        g.free()


def test_hip_event_elapsed_time_is_signed():
    """The kernel-span union (context_internal.h span_sum) takes every event's
    time relative to one reference, so events before it must read negative."""
    import torch
    s = torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    with torch.cuda.stream(s):
        torch.cuda._sleep(2_000_000)
    e1.record(s)
    e1.synchronize()
    assert e0.elapsed_time(e1) > 0 and e1.elapsed_time(e0) < 0
    assert abs(e0.elapsed_time(e1) + e1.elapsed_time(e0)) < 1e-3


def test_timing_history_after_the_ring_wraps():
    """More back-to-back fused steps than the timing ring holds (1024): a step
    queued behind a busy GPU borrows the previous slot's stop as its start, and
    once the ring wraps the oldest slot's stand-in belongs to the newest step.
    That slot must read -1 (no start), never a negative or garbage span."""
    from crossbow_amd import _lib
    g = make_gpu(4_000_000, 2, 0.1, 0.9)
    try:
        g.fill_synthetic(3)
        g.set_timing(True)
        for c in range(1100):
            g.lockAny()
            g.synchronise(0, c, 0, False)
            g.unlockAny()
        g.wait()
        for which in (_lib.T_KERNEL, _lib.T_STEP):
            h = g.timing_history(which, max_steps=1024)
            assert len(h) == 1024
            assert h[0] > 0 or h[0] == -1, h[0]
            assert all(x > 0 for x in h[1:]), min(h[1:])
    finally:
        g.free()


def test_multiple_steps_drift():
    _run(50_000, 4, 0.1, 0.9, steps=3)


def test_update_type_routing():
    from crossbow_amd import CbxError
    # SYNCHRONOUSEAMSGD (3) routes to SMA (executioncontext.c:2287-2295).
    n, R = 1031, 2
    st = O.make_state(n, 1, R, 0.1, 0.0)
    g = make_gpu(n, R, 0.1, 0.0, update_type=3)
    try:
        upload(g, st)
        g.lockAny()
        g.synchronise(0, 1, 0, False)
        g.unlockAny()
        want = st.clone()
        O.sma_step(want)
        compare_states(download(g, st), want)
    finally:
        g.free()
    from crossbow_amd import _lib
    g = make_gpu(n, R, 0.1, 0.0, update_type=5)  # HOGWILD: not this library's path
    try:
        g.lockAny()
        with pytest.raises(CbxError) as e:
            g.synchronise(0, 1, 0, False)
        assert e.value.code == _lib.CBX_ERR_UNSUPPORTED
    finally:
        g.free()
    g = make_gpu(n, R, 0.1, 0.0, update_type=1)  # WORKER (S-SGD) needs the work per clock
    try:
        g.lockAny()
        with pytest.raises(CbxError) as e:
            g.synchronise(0, 1, 0, False)
        assert e.value.code == _lib.CBX_ERR_STATE
    finally:
        g.free()


def test_register_variables_and_replication():
    from crossbow_amd import BUF_DATA, TheGPU
    from crossbow_amd.variables import lenet_variables, register
    n = 1_111_946
    init = O.fill_normal(n, 99, 0.05)
    g = TheGPU()
    g.init([0])
    try:
        assert register(g, lenet_variables(), init) == n
        g.setUpdateModelType(7)
        g.setMomentum(0.9, 0)
        g.setModelManager(3, 0)
        assert g.num_replicas() == 3 and g.elements() == n
        assert_bitexact(g.base_read(0, BUF_DATA), init, "theModel pushed")
        for i in range(3):
            assert_bitexact(g.replica_read(i, BUF_DATA), init, f"replica {i}")
    finally:
        g.free()


def test_checkpoint_roundtrip_file_format():
    from crossbow_amd import BUF_DATA, BUF_LAST
    n, R = 4099, 2
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        upload(g, st)
        with tempfile.TemporaryDirectory() as d:
            g.checkpointModel(d)
            ck = os.path.join(d, "000001")
            names = sorted(os.listdir(ck))
            assert names == ["gpu-00-replica-000-data.dat", "gpu-00-replica-000-last.dat",
                             "gpu-00-replica-001-data.dat", "gpu-00-replica-001-last.dat",
                             "gpu-00-theModel-data.dat", "gpu-00-theModel-last.dat"]
            raw = np.fromfile(os.path.join(ck, "gpu-00-theModel-data.dat"), dtype="<f4")
            assert_bitexact(raw, st.z[0], "raw little-endian fp32 file")
            g.base_write(0, BUF_DATA, np.zeros(n, np.float32))
            g.replica_write(1, BUF_DATA, np.zeros(n, np.float32))
            g.overrideModelData(ck)
            assert_bitexact(g.base_read(0, BUF_DATA), st.z[0], "z restored")
            assert_bitexact(g.base_read(0, BUF_LAST), st.last[0], "last restored")
            assert_bitexact(g.replica_read(1, BUF_DATA), st.w[1], "w restored")
            g.checkpointModel(d)
            assert os.path.isdir(os.path.join(d, "000002"))
    finally:
        g.free()


def test_checkpoint_batchnorm_stats():
    # executioncontext.c:2352-2386 -> cudnnbatchnormparams.c:102-143: each BN
    # operator's running mean / variance beside the model files, per device, by op id.
    import torch
    n, R = 4099, 2
    st = O.make_state(n, 1, R, 0.1, 0.0)
    g = make_gpu(n, R, 0.1, 0.0)
    try:
        upload(g, st)
        ops = {3: 64, 17: 1001}
        mean = {op: torch.from_numpy(O.fill_normal(e, 900 + op, 0.5)).cuda() for op, e in ops.items()}
        var = {op: torch.from_numpy(O.fill_normal(e, 800 + op, 0.5)).cuda() for op, e in ops.items()}
        want = {op: (mean[op].cpu().numpy(), var[op].cpu().numpy()) for op in ops}
        for op, e in ops.items():
            g.register_batchnorm_stats(op, e, [mean[op].data_ptr()], [var[op].data_ptr()])
        g.register_batchnorm_stats(5, 8, [0], [0])  # no copy on this device: no files
        with pytest.raises(ValueError):
            g.register_batchnorm_stats(6, 8, [], [])
        with tempfile.TemporaryDirectory() as d:
            g.checkpointModel(d)
            ck = os.path.join(d, "000001")
            names = sorted(x for x in os.listdir(ck) if "-bn-" in x)
            assert names == ["gpu-00-bn-avg-003.dat", "gpu-00-bn-avg-017.dat",
                             "gpu-00-bn-var-003.dat", "gpu-00-bn-var-017.dat"]
            for op in ops:
                assert_bitexact(np.fromfile(os.path.join(ck, f"gpu-00-bn-avg-{op:03d}.dat"), "<f4"),
                                want[op][0], f"op {op} mean file")
                assert_bitexact(np.fromfile(os.path.join(ck, f"gpu-00-bn-var-{op:03d}.dat"), "<f4"),
                                want[op][1], f"op {op} variance file")
                mean[op].zero_()
                var[op].fill_(-1.0)
            torch.cuda.synchronize()
            g.overrideModelData(ck)
            for op in ops:
                assert_bitexact(mean[op].cpu().numpy(), want[op][0], f"op {op} mean restored")
                assert_bitexact(var[op].cpu().numpy(), want[op][1], f"op {op} variance restored")
            # Unregistered: the next checkpoint has no BN files for it.
            g.register_batchnorm_stats(17, 0, [0], [0])
            g.checkpointModel(d)
            assert sorted(x for x in os.listdir(os.path.join(d, "000002")) if "-bn-" in x) == \
                ["gpu-00-bn-avg-003.dat", "gpu-00-bn-var-003.dat"]
            # A missing file is an I/O error, as crossbowDataBufferLoad's err() (databuffer.c:242-244).
            os.remove(os.path.join(ck, "gpu-00-bn-var-003.dat"))
            with pytest.raises(Exception, match="bn-var-003"):
                g.overrideModelData(ck)
    finally:
        g.free()


def test_staged_roundtrip():
    # Pinned-host staging: stage_in -> step -> stage_out equals the oracle.
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_LAST
    n, R = 65_536, 4
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        g.base_host_view(0, BUF_DATA)[:] = st.z[0]
        g.base_host_view(0, BUF_LAST)[:] = st.last[0]
        for i in range(R):
            g.replica_host_view(i, BUF_DIFF)[:] = st.s[i]
            g.replica_host_view(i, BUF_DATA)[:] = st.w[i]
        g.set_timing(True)
        g.stage_in()
        g.lockAny()
        g.synchronise(0, 1, 0, False)
        g.unlockAny()
        g.stage_out()
        g.wait()
        t = g.last_timing(0)
        assert t[4] > 0 and t[5] > 0 and t[0] > 0
        want = st.clone()
        O.sma_step(want)
        assert_bitexact(g.base_host_view(0, BUF_DATA), want.z[0], "z staged out")
        assert_bitexact(g.base_host_view(0, BUF_LAST), want.last[0], "last staged out")
        for i in range(R):
            assert_bitexact(g.replica_host_view(i, BUF_DATA), want.w[i], f"w[{i}] staged out")
    finally:
        g.free()


@pytest.mark.parametrize("staging", ["zerocopy", "dma"])
@pytest.mark.parametrize("n,buckets,split,copy_step,held,momentum", [
    (4099, 1, False, None, None, 0.9), (4099, 7, False, 1, None, 0.9), (300_001, 16, False, None, 2, 0.9),
    (300_001, 4096, False, 0, None, 0.9), (300_001, 5, True, None, None, 0.9), (300_001, 16, True, 1, 3, 0.9),
    (1_111_946, 16, False, None, None, 0.9), (65_537, 3, True, 0, None, 0.0), (65_537, 1, False, None, 1, 0.0),
])
def test_staged_pipelined(staging, n, buckets, split, copy_step, held, momentum):
    # cbx_synchronise_staged: host mirrors in, host mirrors out.  zerocopy: the
    # kernels read / write the pinned mirror over PCIe themselves; dma: uploads /
    # kernels / downloads overlapped per bucket.  Three steps back to back: each
    # reads what the last wrote; a replica held by a task (SSP) stays out of
    # one step but is still staged in.  Bit-exact with the oracle, host and device.
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_LAST
    from crossbow_amd._lib import STAGING_DMA, STAGING_ZEROCOPY
    R = 4
    st = O.make_state(n, 1, R, 0.1, momentum)
    g = make_gpu(n, R, 0.1, momentum, sync=1 if held is not None else 0)
    try:
        g.set_staging_mode(STAGING_ZEROCOPY if staging == "zerocopy" else STAGING_DMA)
        if split:
            g.set_force_split(True)
        g.base_host_view(0, BUF_DATA)[:] = st.z[0]
        if momentum > 0:
            g.base_host_view(0, BUF_LAST)[:] = st.last[0]
        for i in range(R):
            g.replica_host_view(i, BUF_DIFF)[:] = st.s[i]
            g.replica_host_view(i, BUF_DATA)[:] = st.w[i]
        g.set_timing(True)
        want = st.clone()
        for step in range(3):
            want.locked[:] = 1
            if copy_step == step:
                g.set_replica_copy(1, True)
                want.copy[1] = 1
            if held is not None and step == 1:
                g.replica_lock(held)  # busy on the task side: lockAny (SSP) skips it
                want.locked[held] = 0
            g.lockAny()
            g.synchronise_staged(0, step + 1, 0, buckets)
            g.unlockAny()
            if held is not None and step == 1:
                g.replica_unlock(held)
            O.sma_step(want)
        g.wait()
        t = g.last_timing(0)
        assert t[3] > 0, t
        if staging == "dma":
            assert t[4] > 0 and t[5] > 0, t
            assert t[3] >= max(t[4], t[5]) * 0.99, "the step span covers uploads and downloads"
        assert_bitexact(g.base_host_view(0, BUF_DATA), want.z[0], "z staged out")
        if momentum > 0:
            assert_bitexact(g.base_host_view(0, BUF_LAST), want.last[0], "last staged out")
            assert_bitexact(g.base_read(0, BUF_LAST), want.last[0], "last on device")
        for i in range(R):
            assert_bitexact(g.replica_host_view(i, BUF_DATA), want.w[i], f"w[{i}] staged out")
            assert_bitexact(g.replica_host_view(i, BUF_DIFF), st.s[i], f"s[{i}] host mirror untouched")
            # the device holds what stage_in + synchronise + stage_out leave there
            assert_bitexact(g.replica_read(i, BUF_DATA), want.w[i], f"w[{i}] on device")
            assert_bitexact(g.replica_read(i, BUF_DIFF), st.s[i], f"s[{i}] on device")
        assert_bitexact(g.base_read(0, BUF_DATA), want.z[0], "z on device")
        if copy_step is not None:
            assert g.replica_copy(1) == 0
    finally:
        g.free()


def test_resnet50_full_size_parity_every_element_and_conservation():
    """C3 at full size (n = 25,557,032, R = 8, mu = 0.9): the oracle run on the
    whole downloaded state must match the GPU bit for bit in EVERY element of
    z, last and all 8 w (no sample); plus a size-independent
    conservation checksum:
    z' + sum_i w_i' = z + sum_i w_i + 0.9 last  (exact in real arithmetic)."""
    from crossbow_amd import BUF_DATA, BUF_DIFF, BUF_LAST
    n, R = 25_557_032, 8
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        g.fill_synthetic(O.SEED)
        z0 = g.base_read(0, BUF_DATA)
        l0 = g.base_read(0, BUF_LAST)
        s0 = [g.replica_read(i, BUF_DIFF) for i in range(R)]
        w0 = [g.replica_read(i, BUF_DATA) for i in range(R)]
        before = float(np.sum(z0, dtype=np.float64) + sum(np.sum(w, dtype=np.float64) for w in w0)
                       + 0.9 * np.sum(l0, dtype=np.float64))
        g.lockAny()
        g.synchronise(0, 1, 0, False)
        g.unlockAny()
        g.wait()
        z1 = g.base_read(0, BUF_DATA)
        l1 = g.base_read(0, BUF_LAST)
        w1 = [g.replica_read(i, BUF_DATA) for i in range(R)]
        after = float(np.sum(z1, dtype=np.float64) + sum(np.sum(w, dtype=np.float64) for w in w1))
        assert abs(after - before) <= 1e-6 * max(1.0, abs(before)) + 1e-3, (after, before)
        st = O.SmaState(1, R, n, 0.1, 0.9, [z0], [l0], s0, w0)  # in place: the inputs are not needed again
        O.sma_step(st)
        compared = 0
        assert_bitexact(z1, st.z[0], "z")
        assert_bitexact(l1, st.last[0], "last")
        compared += z1.size + l1.size
        for i in range(R):
            assert_bitexact(w1[i], st.w[i], f"w[{i}]")
            compared += w1[i].size
        assert compared == (R + 2) * n
        print(f"C3 full-size parity: {compared} elements compared bit for bit (z, last, {R} w; n = {n})")
    finally:
        g.free()


def test_golden_fixtures_on_gpu():
    from tests.test_oracle import GOLDEN_DIR, load_golden_cases
    cases = load_golden_cases()
    assert cases, f"no fixtures in {GOLDEN_DIR}"
    for case in cases:
        if case["G"] != 1:
            continue
        st = case["state"]
        held = [int(i) for i in np.nonzero(st.locked == 0)[0]]
        g = make_gpu(st.n, st.size, st.alpha, st.momentum, sync=1 if held else 0)
        try:
            upload(g, st)
            for i in np.nonzero(st.copy)[0]:
                g.set_replica_copy(int(i), True)
            for i in held:  # busy on the task side: lockAny (SSP) skips it
                g.replica_lock(i)
            assert g.lockAny() == st.size - len(held)
            g.synchronise(st.first, 1, 0, False)
            g.unlockAny()
            for i in held:
                g.replica_unlock(i)
            got = download(g, st)
            for k in range(st.size):
                assert_bitexact(got.w[k], case["w_out"][k], f"{case['name']} w[{k}]")
            assert_bitexact(got.z[0], case["z_out"][0], f"{case['name']} z")
        finally:
            g.free()


def test_batchnorm_stats_single_device():
    # One device: the reference returns at once (cudnnbatchnormparams.c:165-166).
    # With the split pipeline forced, the pack / one-rank all-reduce / unpack
    # path runs with count 1 on every layer and must be the identity.
    import torch
    n, R = 4096, 1
    g = make_gpu(n, R, 0.1, 0.0)
    try:
        elements = [64, 256, 2048, 3]
        mean = [torch.from_numpy(O.fill_normal(e, 950 + l, 0.5)).cuda() for l, e in enumerate(elements)]
        var = [torch.from_numpy(O.fill_normal(e, 960 + l, 0.5)).cuda() for l, e in enumerate(elements)]
        before = [t.cpu().numpy().copy() for t in mean + var]
        args = (elements, [t.data_ptr() for t in mean], [t.data_ptr() for t in var], [0] * len(elements))
        torch.cuda.synchronize()
        g.average_batchnorm_stats(*args)
        g.set_force_split(True)
        g.average_batchnorm_stats(*args)
        torch.cuda.synchronize()
        for t, b in zip(mean + var, before):
            assert_bitexact(t.cpu().numpy(), b, "batch-norm statistics with one device")
    finally:
        g.free()


def test_autotune_add_and_del_model():
    # modelmanager.c:362-557 via synchronise(autotune = +1 / -1): the new
    # replica (id R on the single device) copies replica 0's buffers, is
    # locked through the barrier, and takes part in the next SMA step.
    from crossbow_amd import BUF_DATA, BUF_DIFF
    n, R = 20_011, 2
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        upload(g, st)
        ptr0 = g.replica_buffer(0, BUF_DATA)
        g.lockAny()
        g.synchronise(0, 1, 1, False)  # autotune > 0: step, then add one replica per GPU
        assert g.unlockAny() == R + 1
        assert g.num_replicas() == R + 1
        O.sma_step(st)
        # the new replica is a copy of replica 0 after the step
        st2 = O.SmaState(1, R + 1, n, 0.1, 0.9, st.z, st.last, st.s + [st.s[0].copy()], st.w + [st.w[0].copy()])
        g.wait()
        assert_bitexact(g.replica_read(R, BUF_DATA), st2.w[R], "new replica data")
        assert_bitexact(g.replica_read(R, BUF_DIFF), st2.s[R], "new replica snapshot")
        assert g.replica_buffer(0, BUF_DATA) == ptr0, "existing buffers must not move"
        g.lockAny()
        g.synchronise(0, 2, 0, False)
        g.unlockAny()
        O.sma_step(st2)
        compare_states(download(g, st2), st2)
        g.lockAny()
        g.synchronise(0, 3, -1, False)  # autotune < 0: step, then drop the last replica
        g.unlockAny()
        O.sma_step(st2)
        assert g.num_replicas() == R
        g.wait()
        for i in range(R):
            assert_bitexact(g.replica_read(i, BUF_DATA), st2.w[i], f"w[{i}] after del")
    finally:
        g.free()


def test_randomised_configurations_bitexact():
    # 40 random configurations of everything the barrier path takes as input:
    # n (ragged), replicas (1-12, i.e. unrolled and chunked kernels), alpha,
    # momentum, SSP partial locks, `first`, Phase-D copy flags, launch shape,
    # fused vs split pipeline, bucket size, several steps.  Bit-exact.
    import random
    rng = random.Random(20190701)
    for case in range(40):
        n = rng.choice([1, 3, 1023, 4096, 65_537, 131_071, 300_007])
        R = rng.randint(1, 12)
        alpha = rng.choice([0.1, 0.5, 0.25, 1.0])
        momentum = rng.choice([0.0, 0.9])
        held = tuple(sorted(rng.sample(range(R), rng.randint(0, R - 1)))) if R > 1 else ()
        first = rng.randint(0, R - 1) if rng.random() < 0.2 else 0
        copy_ids = tuple(i for i in range(first, R) if i not in held and rng.random() < 0.15)
        split = rng.random() < 0.4
        bucket = rng.choice([0, 4096, 65_536]) if split else 0
        config = rng.choice([None, dict(block=64, blocks_per_cu=0, policy=1, unroll=2),
                             dict(block=64, blocks_per_cu=0, policy=1, unroll=1, occupancy=4),
                             dict(block=256, blocks_per_cu=4, policy=0, unroll=1)])
        try:
            _run(n, R, alpha, momentum, copy_ids=copy_ids, first=first, held=held,
                 sync=1 if held else 0, config=config, split=split, bucket=bucket, steps=rng.randint(1, 3))
        except AssertionError as e:
            raise AssertionError(f"case {case}: n={n} R={R} alpha={alpha} mu={momentum} held={held} "
                                 f"copy={copy_ids} first={first} split={split} bucket={bucket} "
                                 f"config={config}: {e}") from e


@pytest.mark.parametrize("mode", ["fused", "split", "default"])
@pytest.mark.parametrize("timing", [False, True])
def test_step_event_covers_the_step(mode, timing):
    # cbx_step_event stands for base->updated / replica->updated (sma.c:177,204,
    # default.c:32): once it has completed, the step's results are in memory.
    # Checked from the host with hipEventSynchronize and a null-stream copy
    # (the sync stream is non-blocking, so only the event orders the read).
    import ctypes
    from crossbow_amd import BUF_DATA, UPDATE_DEFAULT
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    n, R = 1 << 22, 8
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9, update_type=UPDATE_DEFAULT if mode == "default" else 7)
    try:
        if mode == "split":
            g.set_force_split(True)
            g.set_bucket_elements(n // 3)
        g.set_timing(timing)
        upload(g, st)
        g.wait()
        want = st.clone()
        for clock in (1, 2):
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
            O.default_sync(want) if mode == "default" else O.sma_step(want)
        ev = g.step_event(0)
        assert hip.hipEventSynchronize(ev) == 0
        out = np.empty(n, np.float32)
        for i in (0, R - 1):
            assert hip.hipMemcpy(out.ctypes.data, g.replica_buffer(i, BUF_DATA), 4 * n, 2) == 0
            assert_bitexact(out, want.w[i], f"w[{i}] after the step event")
        assert hip.hipMemcpy(out.ctypes.data, g.base_buffer(0, BUF_DATA), 4 * n, 2) == 0
        assert_bitexact(out, want.z[0], "z after the step event")
    finally:
        g.free()


@pytest.mark.parametrize("pipeline", ["fused", "cross-step", "cross-step-stride"])
def test_concurrent_task_threads_and_barrier(pipeline):
    # The reference's threading: task threads lock a replica,
    # run its optimiser step and release it, while the result-collector
    # thread runs lockAny / synchronise / unlockAny.  Under SSP the barrier
    # skips replicas a task holds.  Stress that interleaving through the
    # C-ABI from Python threads (ctypes releases the GIL) and check the
    # invariants: no error, every replica unlocked at the end, all values
    # finite, clocks never ahead of the barrier.
    import threading

    from crossbow_amd import BUF_DATA, TheGPU
    n, R, workers, iters, barriers = 65_536, 6, 3, 40, 30
    g = TheGPU()
    g.init([0])
    errors = []
    try:
        g.setModel(1, 4 * n)
        g.setModelVariable(0, 1, [n], 4 * n)
        g.setUpdateModelType(7)
        g.setEamsgdAlpha(0.1)
        g.setMomentum(0.9, 0)
        g.setWeightDecay(1e-4)
        g.setLearningRateDecayPolicyFixed(0.01)
        g.setModelManager(R, 1)  # SSP
        if pipeline.startswith("cross-step"):  # kernels A across steps, racing the task threads' optimiser steps
            g.set_force_split(True)
            g.set_bucket_elements(16_384)
            g.set_pipeline_mode(1)
            g.set_cross_wait_stride(2 if pipeline.endswith("stride") else 1)
        g.fill_synthetic(3)

        def worker(k):
            try:
                task = k * 1000
                for it in range(iters):
                    i = (k + it * workers) % R
                    g.replica_lock(i)
                    try:
                        g.replica_optimise(i, task)
                        g.replica_task_done(i)
                    finally:
                        g.replica_unlock(i)
                    task += 1
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))

        threads = [threading.Thread(target=worker, args=(k,)) for k in range(workers)]
        for t in threads:
            t.start()
        for clock in range(1, barriers + 1):
            locked = g.lockAny()
            assert 0 <= locked <= R
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
        for t in threads:
            t.join(timeout=60)
        assert not errors, errors
        g.wait()
        assert g.lockAny() == R, "every replica is free again"
        g.synchronise(0, barriers + 1, 0, False)
        g.unlockAny()
        g.wait()
        for i in range(R):
            assert np.isfinite(g.replica_read(i, BUF_DATA)).all()
            assert g.replica_clock(i) == barriers + 1
    finally:
        g.free()


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("bucket", [65_536, 4096])
@pytest.mark.parametrize("stride,group", [(1, 1), (2, 1), (3, 1), (2, 3), (1, 2), (3, 4)])
@pytest.mark.parametrize("algo", [0, 2])  # all-reduce, reduce-scatter + all-gather
def test_cross_step_pipeline(momentum, bucket, stride, group, algo):
    # cbx_set_pipeline_mode(1): kernels A on their own stream, each waiting
    # only for B of the same bucket in the previous step.  Eight steps with
    # Phase D requests, SSP holds, a host write between two steps (which
    # must make the next step join the whole sync stream) and a switch to the
    # in-step mode and back; bit-exact with the oracle throughout.
    _cross_step_run(momentum, bucket, stride, group, algo)


def _cross_step_child(hw_queues, q):
    # a fresh process: ROCclr reads GPU_MAX_HW_QUEUES once, at HIP's start
    os.environ["GPU_MAX_HW_QUEUES"] = hw_queues
    try:
        _cross_step_run(0.9, 65_536, 2, 2, 0)
        _cross_step_run(0.9, 16_384, 1, 1, 2)
        q.put(None)
    except BaseException:  # pragma: no cover - reported to the parent
        import traceback
        q.put(traceback.format_exc())


@pytest.mark.timeout(240)
def test_cross_step_pipeline_live_at_hip_default_hw_queues():
    # The library's four streams per device share ROCclr's hardware queues
    # when GPU_MAX_HW_QUEUES is HIP's default 4 (with RCCL's and torch's
    # streams beside them), so a stream wait can hold back another stream's
    # work queued behind it: slower, but it must stay
    # live and bit-exact.  The cross-step pipeline with two A streams, wait
    # stride 2 and all-reduce groups of 2, and 19 buckets in the reduce-scatter
    # form, in a process started with GPU_MAX_HW_QUEUES=4.
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_cross_step_child, args=("4", q))
    p.start()
    try:
        err = q.get(timeout=200)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert err is None, err


def _cross_step_run(momentum, bucket, stride, group, algo):
    from crossbow_amd import BUF_DATA
    n, R = 300_001, 3
    st = O.make_state(n, 1, R, 0.1, momentum)
    g = make_gpu(n, R, 0.1, momentum, sync=1)
    try:
        g.set_force_split(True)
        g.set_bucket_elements(bucket)
        g.set_pipeline_mode(1)
        g.set_cross_wait_stride(stride)
        g.set_allreduce_group(group)  # all-reduces per comm-stream wait; mode 0 steps use it too
        g.set_allreduce_algorithm(algo)
        upload(g, st)
        want = st.clone()
        # "timing": cbx_set_timing calls before the step (timing on restarts
        # the span records a continuing step starts from: the step joins)
        plan = [{}, {"copy": 1}, {"hold": 2}, {}, {"write": 0}, {"mode": 0}, {"mode": 1, "copy": 2, "hold": 0},
                {"mode": 0}, {"mode": 1}, {"timing": [True]}, {}, {"timing": [True]}, {"timing": [False, True]},
                {"copy": 0}, {"timing": [False]}, {}]
        for step, p in enumerate(plan):
            want.locked[:] = 1
            for on in p.get("timing", []):
                g.set_timing(on)
            if "mode" in p:
                g.set_pipeline_mode(p["mode"])
            if "write" in p:
                i = p["write"]
                new = O.fill_normal(n, 900 + step, 0.05)
                g.replica_write(i, BUF_DATA, new)
                want.w[i] = new.copy()
            if "copy" in p:
                g.set_replica_copy(p["copy"], True)
                want.copy[p["copy"]] = 1
            if "hold" in p:
                g.replica_lock(p["hold"])
                want.locked[p["hold"]] = 0
            g.lockAny()
            g.synchronise(0, step + 1, 0, False)
            g.unlockAny()
            if "hold" in p:
                g.replica_unlock(p["hold"])
            O.sma_step(want)
        g.wait()
        compare_states(download(g, st), want)
    finally:
        g.free()


def test_cross_step_pipeline_randomised_long_run():
    # 60 steps in pipeline mode 1 with a random mix of Phase-D requests, SSP
    # holds, host writes between steps, bucket-size changes (a new bucket
    # count forces a full join) and mode switches, checked bit for bit
    # against the oracle every 20 steps and at the end.
    import random

    from crossbow_amd import BUF_DATA
    rng = random.Random(4242)
    n, R = 200_003, 4
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9, sync=1)
    try:
        g.set_force_split(True)
        g.set_bucket_elements(16_384)
        g.set_pipeline_mode(1)
        upload(g, st)
        want = st.clone()
        for step in range(60):
            want.locked[:] = 1
            u = rng.random()
            held = None
            if u < 0.08:
                i = rng.randrange(R)
                g.set_replica_copy(i, True)
                want.copy[i] = 1
            elif u < 0.16:
                held = rng.randrange(R)
                g.replica_lock(held)
                want.locked[held] = 0
            elif u < 0.21:
                i = rng.randrange(R)
                new = O.fill_normal(n, 7000 + step, 0.05)
                g.replica_write(i, BUF_DATA, new)
                want.w[i] = new.copy()
            elif u < 0.26:
                g.set_bucket_elements(rng.choice([4096, 16_384, 65_536, 1 << 40]))
            elif u < 0.30:
                g.set_pipeline_mode(rng.choice([0, 1]))
                g.set_cross_wait_stride(rng.choice([1, 2, 3, 8]))
                g.set_allreduce_group(rng.choice([1, 1, 2, 5]))
            elif u < 0.34:
                g.set_allreduce_algorithm(rng.choice([0, 2]))  # all-reduce / reduce-scatter + all-gather
            g.lockAny()
            g.synchronise(0, step + 1, 0, False)
            g.unlockAny()
            if held is not None:
                g.replica_unlock(held)
            O.sma_step(want)
            if step % 20 == 19:
                g.wait()
                compare_states(download(g, st), want)
        g.wait()
        compare_states(download(g, st), want)
    finally:
        g.free()


@pytest.mark.parametrize("mode,stride,group,algo", [(0, 1, 1, 0), (1, 1, 1, 0), (1, 2, 2, 0), (0, 1, 3, 2),
                                                    (1, 2, 1, 2)])
def test_stream_order_check(mode, stride, group, algo):
    # cbx_set_order_check: every split step records per-bucket timestamps
    # (kernel A, the collective, kernel B); cbx_check_order after every two
    # back-to-back steps verifies the bucket pipeline's ordering and, in
    # mode 1, that each A(k) of the second step began after B(k) of the first.
    n, R = 300_001, 3
    st = O.make_state(n, 1, R, 0.1, 0.9)
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        g.set_force_split(True)
        g.set_bucket_elements(65_536)
        g.set_pipeline_mode(mode)
        g.set_cross_wait_stride(stride)
        g.set_allreduce_group(group)
        g.set_allreduce_algorithm(algo)
        g.set_order_check(True)
        upload(g, st)
        want = st.clone()
        for step in range(8):
            want.locked[:] = 1
            g.lockAny()
            g.synchronise(0, step + 1, 0, False)
            g.unlockAny()
            O.sma_step(want)
            if step % 2 == 1:
                assert g.check_order() == 2
        g.wait()
        compare_states(download(g, st), want)
        assert g.check_order() == 0  # nothing new since the last check
    finally:
        g.free()


def test_stream_order_check_detects_a_race(monkeypatch):
    # Fault injection ($CBX_FAULT_SKIP_COMM_WAIT at context creation): the
    # comm stream no longer waits for kernel A, so each bucket's collective
    # reads acc while kernel A is still writing it.  The order check must
    # name that race.
    from crossbow_amd import CbxError
    monkeypatch.setenv("CBX_FAULT_SKIP_COMM_WAIT", "1")
    n = 25_557_032
    g = make_gpu(n, 8, 0.1, 0.9)
    monkeypatch.delenv("CBX_FAULT_SKIP_COMM_WAIT")
    try:
        g.set_force_split(True)
        g.set_bucket_elements(-(-n // 4))
        g.fill_synthetic(7)
        g.set_order_check(True)
        for step in range(2):
            g.lockAny()
            g.synchronise(0, step + 1, 0, False)
            g.unlockAny()
        with pytest.raises(CbxError, match="the collective started before kernel A ended"):
            g.check_order()
        g.wait()
    finally:
        g.free()


@pytest.mark.parametrize("fault", [True, False])
def test_two_a_stream_group_wait_race_is_caught(monkeypatch, fault):
    # Pins round 3's fix (the comm stream waits for the last kernel A on EACH
    # of the two A streams of a cross-step all-reduce group).
    # $CBX_FAULT_ONE_STREAM_COMM_WAIT restores the earlier wait (the group's
    # last kernel A only) and holds back, by 0.5 ms, every kernel A that wait
    # skips: with groups of 2 the even buckets' A on the first A stream, so
    # the group's collective certainly reads acc before it is written.  The
    # order check must name the race; without the switch the same pipeline
    # passes the check and stays bit-exact.
    from crossbow_amd import CbxError
    n, R = 300_001, 3
    st = O.make_state(n, 1, R, 0.1, 0.9)
    if fault:
        monkeypatch.setenv("CBX_FAULT_ONE_STREAM_COMM_WAIT", "1")
    g = make_gpu(n, R, 0.1, 0.9)
    monkeypatch.delenv("CBX_FAULT_ONE_STREAM_COMM_WAIT", raising=False)
    try:
        g.set_force_split(True)
        g.set_bucket_elements(65_536)  # 5 buckets
        g.set_pipeline_mode(1)
        g.set_cross_wait_stride(1)
        g.set_allreduce_group(2)
        g.set_order_check(True)
        upload(g, st)
        want = st.clone()
        for step in range(2):
            want.locked[:] = 1
            g.lockAny()
            g.synchronise(0, step + 1, 0, False)
            g.unlockAny()
            O.sma_step(want)
        if fault:
            with pytest.raises(CbxError, match="the collective started before kernel A ended"):
                g.check_order()
            g.wait()
        else:
            assert g.check_order() == 2
            g.wait()
            compare_states(download(g, st), want)
    finally:
        g.free()


def test_fused_timing_excludes_work_enqueued_between_steps():
    # Back-to-back fused steps reuse the previous step's stop event as their
    # start (no start marker).  When a task's optimiser step was enqueued on
    # the sync stream in between, the next step records its own start, so
    # its kernel span never includes the optimiser kernels.
    import statistics

    from crossbow_amd import _lib
    n, R = 4_000_003, 4
    g = make_gpu(n, R, 0.1, 0.9)
    try:
        g.setLearningRateDecayPolicyFixed(0.01)
        g.fill_synthetic(3)
        g.set_timing(True)
        clock = 0

        def step():
            nonlocal clock
            clock += 1
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()

        for _ in range(12):
            step()
        g.wait()
        plain = g.timing_history(_lib.T_KERNEL)[-10:]
        for _ in range(6):
            for i in range(R):
                g.replica_optimise(i, clock, None)  # on the sync stream
            step()
        g.wait()
        mixed = g.timing_history(_lib.T_KERNEL)[-6:]
        assert min(plain) > 0 and min(mixed) > 0
        assert statistics.median(mixed) < 1.3 * statistics.median(plain), (plain, mixed)
    finally:
        g.free()


def test_short_variable_buffer_is_refused():
    # setModelVariableBuffer copies the variable's whole capacity: a shorter
    # host buffer is refused before the library would over-read it.
    import numpy as np

    from crossbow_amd import CbxError, TheGPU
    g = TheGPU()
    g.init([0])
    try:
        g.setModel(1, 4 * 100)
        g.setModelVariable(0, 1, [100], 4 * 100)
        with pytest.raises(CbxError, match="shorter than its capacity"):
            g.setModelVariableBuffer(0, 1, np.zeros(99, np.float32))
        g.setModelVariableBuffer(0, 1, np.zeros(100, np.float32))
    finally:
        g.free()
