"""The library's multi-rank path (cbx_init_rank, G = 2 and 4) on ONE GPU, bit for
bit against the oracle with the same G.

Two processes each drive the real library sources as rank 0 / rank 1 of a
two-GPU job, both on device 0.  Real RCCL refuses two ranks on one device,
so this build of the library (tests/native/libcrossbow_sma_fakerccl.so,
scripts/build_fake_rccl.sh) is linked against a loopback stand-in for the
RCCL calls it makes (tests/native/fake_rccl.cpp): a stream-ordered,
rank-order fp32 sum over files.  Everything else is the product path: the
round-robin placement, per-rank locks, kernel A / all-reduce / kernel B with
the control block in bucket 0, the bucketed two-stream pipeline, Phase D
decided on any rank, S-SGD, the pipelined host-staged step and BN averaging.
Rank-order summation is the oracle's, so the comparison is bit-exact (with
real RCCL on 2+ GPUs the sum order is RCCL's: rtol 1e-5).

The rank processes never import torch (they bind the ABI through the
torch-free crossbow_amd/_abi.py), so the loopback library is the only
librccl-like object in them.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(ROOT, "tests", "native", "libcrossbow_sma_fakerccl.so")

pytestmark = pytest.mark.gpu

# (name, n, R per rank, momentum, steps, buckets (0 = one), copy {step: replica}, held {step: replica},
#  staged buckets (0 = device-resident), update model)
CASES = [
    ("sma", 50_001, 2, 0.9, 3, 0, {}, {}, 0, 7),
    ("sma-copy-ssp", 50_001, 2, 0.9, 3, 0, {1: 3}, {0: 1}, 0, 7),
    ("sma-5-buckets", 300_007, 3, 0.9, 2, 65_536, {1: 0}, {}, 0, 7),
    ("sma-5-buckets-cross", 300_007, 2, 0.9, 5, 65_536, {2: 1}, {3: 0}, 0, 7),
    ("sma-5-buckets-cross-bcomm", 300_007, 2, 0.9, 5, 65_536, {2: 1}, {3: 0}, 0, 7),
    ("sma-no-momentum", 20_011, 1, 0.0, 2, 4096, {}, {}, 0, 3),
    ("sma-staged", 100_003, 2, 0.9, 2, 0, {1: 2}, {}, 3, 7),
    ("ssgd", 40_009, 2, 0.9, 2, 0, {}, {}, 0, 1),
    ("ssgd-buckets", 40_009, 2, 0.9, 2, 4096, {}, {}, 0, 1),
]


def _abi():
    spec = importlib.util.spec_from_file_location("cbx_abi_standalone", os.path.join(ROOT, "crossbow_amd", "_abi.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _Rank:
    def __init__(self, L, A, ctx):
        self.L, self.A, self.c = L, A, ctx

    def __call__(self, name, *args):
        rc = getattr(self.L, name)(self.c, *args)
        if rc < 0:
            raise RuntimeError(f"{name}{args}: {rc} {self.L.cbx_last_error().decode()}")
        return rc

    def write(self, fn, idx, kind, arr):
        a = np.ascontiguousarray(arr, np.float32)
        self(fn, idx, kind, a.ctypes.data_as(ctypes.c_void_p), a.nbytes)

    def read(self, fn, idx, kind, n):
        out = np.empty(n, np.float32)
        self(fn, idx, kind, out.ctypes.data_as(ctypes.c_void_p), out.nbytes)
        return out

    def host(self, fn, idx, kind, n):
        p = ctypes.c_void_p()
        self(fn, idx, kind, ctypes.byref(p))
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(n,))


def _case(L, A, rank, world, uid, case):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    name, n, R, mom, steps, bucket, copy_at, held_at, staged, utype = case
    c = ctypes.c_void_p()
    ub = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
    if L.cbx_init_rank(ctypes.byref(c), 0, world, rank, ub) < 0:
        raise RuntimeError(L.cbx_last_error().decode())
    g = _Rank(L, A, c)
    try:
        shape = (ctypes.c_int * 1)(n)
        g("cbx_set_model", 1, 4 * n)
        g("cbx_set_model_variable", 0, 1, 1, shape, 4 * n)
        g("cbx_set_update_model_type", utype)
        g("cbx_set_eamsgd_alpha", ctypes.c_float(0.1))
        g("cbx_set_momentum", ctypes.c_float(mom), 0)
        g("cbx_set_weight_decay", ctypes.c_float(1e-4))
        g("cbx_set_learning_rate_decay_policy_fixed", ctypes.c_float(0.05))
        wpc = 2 * world * R
        g("cbx_set_model_work_per_clock", wpc)
        g("cbx_set_model_manager", R, A.SYNC_SSP if held_at else A.SYNC_BSP)
        if bucket:
            g("cbx_set_bucket_elements", ctypes.c_longlong(bucket))
        if name.endswith("-cross"):
            g("cbx_set_pipeline_mode", 1)  # kernels A of the next step overlap this step's tail
        elif name.endswith("-cross-bcomm"):
            g("cbx_set_pipeline_mode", 2)  # and kernels B run behind their all-reduce on its stream
            g("cbx_set_cross_wait_stride", 2)  # one cross-step wait per two buckets
            g("cbx_set_allreduce_group", 3)  # all-reduces 0-2 behind one wait, then 3-4
        elif name == "sma-5-buckets":
            g("cbx_set_allreduce_group", 2)  # mode 0: all-reduces in pairs, B of the previous pair beside them
        size = world * R
        assert g("cbx_num_replicas") == size and g("cbx_num_devices") == world
        mine = [i for i in range(size) if i % world == rank]
        # The theta queue hands out this rank's replicas only, round robin (modelmanager.c:180-190).
        clk = ctypes.c_int(-1)
        got = [g("cbx_acquire_access", ctypes.byref(clk)) for _ in mine]
        assert got == mine and clk.value == 0, got
        for i in got:
            g("cbx_replica_lock", i)
            g("cbx_replica_release", i)
        st = O.make_state(n, world, R, 0.1, mom)
        if staged:
            g.host("cbx_base_host_buffer", rank, A.BUF_DATA, n)[:] = st.z[rank]
            g.host("cbx_base_host_buffer", rank, A.BUF_LAST, n)[:] = st.last[rank]
            for i in mine:
                g.host("cbx_replica_host_buffer", i, A.BUF_DIFF, n)[:] = st.s[i]
                g.host("cbx_replica_host_buffer", i, A.BUF_DATA, n)[:] = st.w[i]
        else:
            g.write("cbx_base_write", rank, A.BUF_DATA, st.z[rank])
            if mom > 0:
                g.write("cbx_base_write", rank, A.BUF_LAST, st.last[rank])
            for i in mine:
                g.write("cbx_replica_write", i, A.BUF_DIFF, st.s[i])
                g.write("cbx_replica_write", i, A.BUF_DATA, st.w[i])
        acc = [np.zeros(n, np.float32) for _ in range(world)]
        task = 0
        for step in range(steps):
            if utype == 1:  # S-SGD task steps: the global task list, each rank runs its replicas' tasks
                for k in range(wpc):
                    i = k % size
                    gr = O.fill_normal(n, 5000 + task, 0.01)
                    if i % world == rank:
                        g.write("cbx_replica_write", i, A.BUF_GRADIENT, gr)
                        g("cbx_replica_optimise", i, task, None)
                    O.ssgd_worker(np.float32(-0.05), 1e-4, st.w[i], gr, acc[i % world])
                    task += 1
            st.locked[:] = 1
            if step in copy_at:
                i = copy_at[step]
                st.copy[i] = 1
                if i % world == rank:
                    g("cbx_replica_set_copy", i, 1)
            hold = held_at.get(step)
            if hold is not None:
                st.locked[hold] = 0
                if hold % world == rank:
                    g("cbx_replica_lock", hold)
            g("cbx_lock_any")
            if staged:
                g("cbx_synchronise_staged", 0, step + 1, 0, staged)
            else:
                g("cbx_synchronise", 0, step + 1, 0, 0)
            g("cbx_unlock_any")
            if hold is not None and hold % world == rank:
                g("cbx_replica_unlock", hold)
            if utype == 1:
                O.ssgd_sync(st, acc, wpc)
            else:
                O.sma_step(st)
        g("cbx_wait")
        bad = []

        def check(what, got, want):
            if not np.array_equal(np.asarray(got).view(np.uint32), np.asarray(want).view(np.uint32)):
                bad.append(f"{what}: {int(np.sum(np.asarray(got).view(np.uint32) != np.asarray(want).view(np.uint32)))} differ")

        if staged:
            check("z (host)", g.host("cbx_base_host_buffer", rank, A.BUF_DATA, n), st.z[rank])
            check("last (host)", g.host("cbx_base_host_buffer", rank, A.BUF_LAST, n), st.last[rank])
            for i in mine:
                check(f"w[{i}] (host)", g.host("cbx_replica_host_buffer", i, A.BUF_DATA, n), st.w[i])
        check("z", g.read("cbx_base_read", rank, A.BUF_DATA, n), st.z[rank])
        if mom > 0:
            check("last", g.read("cbx_base_read", rank, A.BUF_LAST, n), st.last[rank])
        for i in mine:
            check(f"w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
        for i in mine:
            if g("cbx_replica_get_copy", i) != 0:
                bad.append(f"copy flag of replica {i} not reset")
        return bad
    finally:
        L.cbx_free(c)


def _bn_case(L, A, rank, world, uid):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    c = ctypes.c_void_p()
    ub = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
    if L.cbx_init_rank(ctypes.byref(c), 0, world, rank, ub) < 0:
        raise RuntimeError(L.cbx_last_error().decode())
    g = _Rank(L, A, c)
    try:
        n = 4096
        shape = (ctypes.c_int * 1)(n)
        g("cbx_set_model", 1, 4 * n)
        g("cbx_set_model_variable", 0, 1, 1, shape, 4 * n)
        g("cbx_set_update_model_type", 7)
        g("cbx_set_model_manager", 1, A.SYNC_BSP)
        elements = [16, 40, 7]
        updated = [[1, 1, 1]] + [[1, 0, 1] if d % 2 else [0, 1, 1] for d in range(1, world)]
        mean = [[O.fill_normal(e, 50 + 10 * d + l, 0.5) for l, e in enumerate(elements)] for d in range(world)]
        var = [[O.fill_normal(e, 90 + 10 * d + l, 0.5) for l, e in enumerate(elements)] for d in range(world)]
        ref_m = [[a.copy() for a in r] for r in mean]
        ref_v = [[a.copy() for a in r] for r in var]
        O.bn_average(ref_m, ref_v, updated)
        # device scratch for the statistics: this rank's base-model gradient buffer
        p = ctypes.c_void_p()
        g("cbx_base_buffer", rank, A.BUF_GRADIENT, ctypes.byref(p))
        base = p.value
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        ptrs_m, ptrs_v, off = [], [], 0
        for l, e in enumerate(elements):
            for arr, lst in ((mean[rank][l], ptrs_m), (var[rank][l], ptrs_v)):
                dst = base + 4 * off
                assert hip.hipMemcpy(dst, arr.ctypes.data, 4 * e, 1) == 0
                lst.append(dst)
                off += e
        L3 = len(elements)
        el = (ctypes.c_int * L3)(*elements)
        pm = (ctypes.c_void_p * L3)(*ptrs_m)
        pv = (ctypes.c_void_p * L3)(*ptrs_v)
        up = (ctypes.c_int * L3)(*updated[rank])
        g("cbx_average_batchnorm_stats", L3, el, ctypes.cast(pm, ctypes.POINTER(ctypes.c_void_p)),
          ctypes.cast(pv, ctypes.POINTER(ctypes.c_void_p)), up)
        bad = []
        for l, e in enumerate(elements):
            for ptr, want, what in ((ptrs_m[l], ref_m[rank][l], "mean"), (ptrs_v[l], ref_v[rank][l], "var")):
                got = np.empty(e, np.float32)
                assert hip.hipMemcpy(got.ctypes.data, ptr, 4 * e, 2) == 0
                if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                    bad.append(f"bn {what}[{l}] differs")
        return bad
    finally:
        L.cbx_free(c)


def _autotune_case(L, A, rank, world, uid, ckdir):
    # synchronise(autotune = +1 / -1) adds / deletes one replica per device
    # after the step (executioncontext.c:2321-2328, modelmanager.c:362-557):
    # a new replica copies its device's first replica and joins the next step.
    # Then every rank checkpoints into one shared directory (each writes its
    # own device's files, with one BN operator's statistics) and reads it back.
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    n, R, mom = 30_011, 2, 0.9
    c = ctypes.c_void_p()
    ub = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
    if L.cbx_init_rank(ctypes.byref(c), 0, world, rank, ub) < 0:
        raise RuntimeError(L.cbx_last_error().decode())
    g = _Rank(L, A, c)
    try:
        shape = (ctypes.c_int * 1)(n)
        g("cbx_set_model", 1, 4 * n)
        g("cbx_set_model_variable", 0, 1, 1, shape, 4 * n)
        g("cbx_set_update_model_type", 7)
        g("cbx_set_eamsgd_alpha", ctypes.c_float(0.1))
        g("cbx_set_momentum", ctypes.c_float(mom), 0)
        g("cbx_set_model_manager", R, A.SYNC_BSP)
        st = O.make_state(n, world, R, 0.1, mom)
        g.write("cbx_base_write", rank, A.BUF_DATA, st.z[rank])
        g.write("cbx_base_write", rank, A.BUF_LAST, st.last[rank])
        for i in range(st.size):
            if i % world == rank:
                g.write("cbx_replica_write", i, A.BUF_DIFF, st.s[i])
                g.write("cbx_replica_write", i, A.BUF_DATA, st.w[i])
        for step, tune in enumerate((1, 0, -1, 0)):
            g("cbx_lock_any")
            g("cbx_synchronise", 0, step + 1, tune, 0)
            g("cbx_unlock_any")
            O.sma_step(st)
            s, w = list(st.s), list(st.w)
            if tune > 0:
                s += [st.s[d].copy() for d in range(world)]
                w += [st.w[d].copy() for d in range(world)]
            elif tune < 0:
                s, w = s[:-world], w[:-world]
            st = O.SmaState(world, len(s), n, 0.1, mom, st.z, st.last, s, w)
            assert g("cbx_num_replicas") == st.size
        g("cbx_wait")
        bad = []
        for what, got, want in [("z", g.read("cbx_base_read", rank, A.BUF_DATA, n), st.z[rank]),
                                ("last", g.read("cbx_base_read", rank, A.BUF_LAST, n), st.last[rank])] + \
                [(f"w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
                 for i in range(st.size) if i % world == rank]:
            if not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                bad.append(f"autotune {what} differs")
        # checkpoint (executioncontext.c:2340-2364) into the shared directory
        os.makedirs(ckdir, exist_ok=True)
        p = ctypes.c_void_p()
        g("cbx_base_buffer", rank, A.BUF_GRADIENT, ctypes.byref(p))  # scratch for BN statistics
        bn = O.fill_normal(2 * 33, 300 + rank, 0.5)
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMemcpy(p.value, bn.ctypes.data, bn.nbytes, 1) == 0
        pm = (ctypes.c_void_p * 1)(p.value)
        pv = (ctypes.c_void_p * 1)(p.value + 4 * 33)
        g("cbx_register_batchnorm_stats", 7, 33, ctypes.cast(pm, ctypes.POINTER(ctypes.c_void_p)),
          ctypes.cast(pv, ctypes.POINTER(ctypes.c_void_p)))
        ckb = ckdir.encode()
        g("cbx_checkpoint_model", ckb)
        ver = os.path.join(ckdir, "000001")
        files = {f"gpu-{rank:02d}-theModel-data.dat": st.z[rank], f"gpu-{rank:02d}-theModel-last.dat": st.last[rank],
                 f"gpu-{rank:02d}-bn-avg-007.dat": bn[:33], f"gpu-{rank:02d}-bn-var-007.dat": bn[33:]}
        files.update({f"gpu-{rank:02d}-replica-{i:03d}-data.dat": st.w[i] for i in range(st.size) if i % world == rank})
        for name, want in files.items():
            path = os.path.join(ver, name)
            if not os.path.exists(path):
                bad.append(f"checkpoint: {name} missing")
            elif not np.array_equal(np.fromfile(path, "<f4").view(np.uint32), want.view(np.uint32)):
                bad.append(f"checkpoint: {name} differs")
        g.write("cbx_base_write", rank, A.BUF_DATA, np.zeros(n, np.float32))
        g("cbx_override_model_data", ver.encode())
        if not np.array_equal(g.read("cbx_base_read", rank, A.BUF_DATA, n).view(np.uint32), st.z[rank].view(np.uint32)):
            bad.append("override: z not restored")
        return bad
    finally:
        L.cbx_free(c)


def _rank_main(rank, world, uids, fake_dir, q):
    os.environ["FAKE_RCCL_DIR"] = fake_dir
    try:
        A = _abi()
        L = A.bind(ctypes.CDLL(VARIANT))
        out = []
        for case, uid in zip(_cases(world), uids):
            out.append((case[0], _case(L, A, rank, world, uid, case)))
        out.append(("bn", _bn_case(L, A, rank, world, uids[-2])))
        out.append(("autotune", _autotune_case(L, A, rank, world, uids[-1], os.path.join(fake_dir, "ckpt"))))
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _cases(world):
    # four ranks: the SMA cases (placement i % 4, Phase D from rank 3, buckets, both cross-step modes);
    # eight ranks (the driver's full-node G): the plain step and the mode-2 pipeline
    if world == 2:
        return CASES
    if world == 4:
        return [c for c in CASES if c[0] in ("sma", "sma-copy-ssp", "sma-5-buckets", "sma-5-buckets-cross",
                                             "sma-5-buckets-cross-bcomm")]
    return [c for c in CASES if c[0] in ("sma-copy-ssp", "sma-5-buckets-cross-bcomm", "ssgd-buckets")]


@pytest.mark.skipif(not os.path.exists(VARIANT), reason="run scripts/build_fake_rccl.sh first")
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_on_one_gpu_bitexact_vs_oracle(world):
    import multiprocessing as mp
    uids = [os.urandom(16) + bytes(112) for _ in range(len(CASES) + 2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as fake_dir:
        procs = [ctx.Process(target=_rank_main, args=(r, world, uids, fake_dir, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = {}
        try:
            for _ in range(world):
                rank, res, err = q.get(timeout=100)
                got[rank] = (res, err)
        finally:
            for p in procs:
                p.join(timeout=30)
                if p.is_alive():
                    p.kill()
    for rank in range(world):
        res, err = got[rank]
        assert err is None, f"rank {rank}:\n{err}"
        failures = [(name, bad) for name, bad in res if bad]
        assert not failures, f"rank {rank}: {failures}"
        assert [name for name, _ in res] == [c[0] for c in _cases(world)] + ["bn", "autotune"]
