"""The sma.c seam: cbx_sma_plan_step / cbx_sma_optimise_buffers over buffers
the CALLER owns (include/crossbow_sma.h, crossbow_amd/csrc/sma_seam.hip).

A Crossbow build that keeps its own model manager replaces only the bodies of
crossbowSynchronisationSMA (clib-multigpu/synch/sma.c:233-248 -> :13-231) and
crossbowKernelOptimiserSMA (kernels/optimisers/sma.cu:3-100).  Its buffers hold
exactly `elements` floats, so these cases use ragged sizes (the float4 bulk
plus the scalar tail), buffers allocated by the test itself (torch, or raw
hipMalloc in the torch-free workers), and the caller's own streams and
communicators:

* one GPU (the product library): the fused step, bit for bit against the
  oracle, over sizes 1 .. LeNet, 1 .. 9 replicas, momentum 0 / 0.9, `first`,
  unlocked replicas, Phase D, several steps back to back;
* the optimiser step, bit for bit against the oracle's sma.cu restatement;
* G devices in one process (the loopback clique, scripts/build_fake_rccl.sh):
  communicators created by the plan (ncclCommInitAll) or handed over by the
  caller, bit for bit in rank order, within the G > 1 tolerance in ring order;
* G ranks with the REAL librccl (one process per rank, NCCL_HOSTID per rank,
  as tests/test_gpu_realrccl.py): the caller's ncclCommInitRank communicator
  spans the processes; bit for bit at G = 2, within the tolerance at G = 4,
  z / last bitwise identical on every rank.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import tempfile

import numpy as np
import pytest

from tests import multidev_common as C

pytestmark = pytest.mark.gpu

ALPHA = 0.1


def _bits_equal(got, want):
    return np.array_equal(np.asarray(got, np.float32).view(np.uint32), np.asarray(want, np.float32).view(np.uint32))


# (name, n, R, momentum, steps, first, held replica ids, {step: replica asking for Phase D})
ONE_GPU = [
    ("one-element", 1, 1, 0.9, 2, 0, (), {}),
    ("three-elements-no-momentum", 3, 2, 0.0, 2, 0, (), {}),
    ("ragged-4099", 4099, 4, 0.9, 3, 0, (), {1: 2}),
    ("whole-trips", 4096 * 3, 8, 0.9, 2, 0, (), {}),
    ("quarter-chunk-bulk", 4096 + 1024 + 7, 3, 0.9, 2, 0, (), {1: 1}),  # bulk 1,280 float4s: not whole kPadFloat4s
    ("chunked-9-replicas", 65_541, 9, 0.9, 2, 0, (), {0: 3}),
    ("first-and-held", 300_007, 8, 0.9, 2, 2, (5,), {1: 6}),
    ("lenet-c2", 1_111_946, 4, 0.0, 2, 0, (), {}),
    ("no-replica-locked", 10_001, 2, 0.9, 1, 0, (0, 1), {}),
]


@pytest.mark.parametrize("name,n,R,mom,steps,first,held,copy_at", ONE_GPU, ids=[c[0] for c in ONE_GPU])
def test_seam_one_gpu_bitexact(name, n, R, mom, steps, first, held, copy_at):
    import torch

    from crossbow_amd.seam import SmaPlan
    from oracle import oracle as O
    st = O.make_state(n, 1, R, ALPHA, mom)
    st.first = first
    dev = torch.device("cuda:0")
    z = torch.from_numpy(st.z[0].copy()).to(dev)
    last = torch.from_numpy(st.last[0].copy()).to(dev) if mom > 0 else None
    s = [torch.from_numpy(a.copy()).to(dev) for a in st.s]
    w = [torch.from_numpy(a.copy()).to(dev) for a in st.w]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with SmaPlan([0], n) as plan:
        for step in range(steps):
            st.locked[:] = 1
            for i in held:
                st.locked[i] = 0
            if step in copy_at:
                st.copy[copy_at[step]] = 1
            reps = [(0, w[i].data_ptr(), s[i].data_ptr(), int(st.locked[i]), int(st.copy[i])) for i in range(R)]
            ran = plan.step([stream.cuda_stream], [z.data_ptr()], [last.data_ptr()] if last is not None else None,
                            reps, ALPHA, mom, first)
            copies = O.sma_step(st)  # resets the copy flags of the locked replicas it copied (sma.c:220)
            assert ran == (1 if copies > 0 else 0), (step, ran, copies)
        stream.synchronize()
    assert _bits_equal(z.cpu().numpy(), st.z[0]), "z"
    if last is not None:
        assert _bits_equal(last.cpu().numpy(), st.last[0]), "last"
    for i in range(R):
        assert _bits_equal(w[i].cpu().numpy(), st.w[i]), f"w[{i}]"
        assert _bits_equal(s[i].cpu().numpy(), st.s[i]), f"s[{i}] must be untouched"


def _random_cases(count=16, seed=20261017):
    """Seeded sizes log-uniform in [1, 2^18) (every bulk/tail split the seam can
    make: no bulk, bulk at any multiple of 1,024 floats, tails of 0..1,023),
    1..10 replicas (above 8 the kernel walks them in register chunks), momentum 0 / 0.9,
    a Phase-D request at step 1 half of the time."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        n = int(np.exp(rng.uniform(0.0, np.log(1 << 18))))
        R = int(rng.integers(1, 11))
        mom = float(rng.choice([0.0, 0.9]))
        copy_at = {1: int(rng.integers(0, R))} if rng.random() < 0.5 else {}
        out.append((f"random-{k}-n{n}-r{R}", n, R, mom, 2, 0, (), copy_at))
    return out


RANDOM = _random_cases()


@pytest.mark.parametrize("name,n,R,mom,steps,first,held,copy_at", RANDOM, ids=[c[0] for c in RANDOM])
def test_seam_random_sizes_bitexact(name, n, R, mom, steps, first, held, copy_at):
    test_seam_one_gpu_bitexact(name, n, R, mom, steps, first, held, copy_at)


def _golden(G):
    from tests.test_oracle import load_golden_cases
    return [c for c in load_golden_cases() if c["G"] == G]


@pytest.mark.parametrize("gcase", _golden(1), ids=lambda c: c["name"])
def test_seam_golden_fixtures_one_gpu(gcase):
    """The committed fixtures (tests/golden/, the oracle's outputs) through the
    seam on caller-owned buffers: one step, bit for bit."""
    import torch

    from crossbow_amd.seam import SmaPlan
    st = gcase["state"]
    n = st.n
    dev = torch.device("cuda:0")
    z = torch.from_numpy(st.z[0].copy()).to(dev)
    last = torch.from_numpy(st.last[0].copy()).to(dev) if st.last is not None else None
    s_ = [torch.from_numpy(a.copy()).to(dev) for a in st.s]
    w = [torch.from_numpy(a.copy()).to(dev) for a in st.w]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with SmaPlan([0], n) as plan:
        reps = [(0, w[i].data_ptr(), s_[i].data_ptr(), int(st.locked[i]), int(st.copy[i])) for i in range(st.size)]
        plan.step([stream.cuda_stream], [z.data_ptr()], [last.data_ptr()] if last is not None else None, reps,
                  st.alpha, st.momentum, st.first)
        stream.synchronize()
    assert _bits_equal(z.cpu().numpy(), gcase["z_out"][0]), "z"
    if gcase["last_out"] is not None:
        assert _bits_equal(last.cpu().numpy(), gcase["last_out"][0]), "last"
    for i in range(st.size):
        assert _bits_equal(w[i].cpu().numpy(), gcase["w_out"][i]), f"w[{i}]"


def test_seam_resnet50_full_size_bitexact():
    """C3's buffers through the seam: n = 25,557,032 (not a multiple of the
    seam's 1,024-float bulk granularity: a 40-element tail), 8 replicas, mu 0.9."""
    import torch

    from crossbow_amd.seam import SmaPlan
    from oracle import oracle as O
    n, R = 25_557_032, 8
    st = O.make_state(n, 1, R, ALPHA, 0.9, threads=8)
    dev = torch.device("cuda:0")
    z = torch.from_numpy(st.z[0]).to(dev)
    last = torch.from_numpy(st.last[0]).to(dev)
    s = [torch.from_numpy(a).to(dev) for a in st.s]
    w = [torch.from_numpy(a).to(dev) for a in st.w]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with SmaPlan([0], n) as plan:
        reps = [(0, w[i].data_ptr(), s[i].data_ptr(), 1, 0) for i in range(R)]
        assert plan.step([stream.cuda_stream], [z.data_ptr()], [last.data_ptr()], reps, ALPHA, 0.9) == 0
        stream.synchronize()
    O.sma_step(st)
    assert _bits_equal(z.cpu().numpy(), st.z[0])
    assert _bits_equal(last.cpu().numpy(), st.last[0])
    for i in range(R):
        assert _bits_equal(w[i].cpu().numpy(), st.w[i]), f"w[{i}]"


@pytest.mark.parametrize("n", [1, 4099, 4096 * 2, 300_007])
@pytest.mark.parametrize("mom,wd", [(0.9, 1e-4), (0.9, 0.0), (0.0, 1e-4), (0.0, 0.0)])
def test_seam_optimise_bitexact(n, mom, wd):
    import torch

    from crossbow_amd.seam import optimise_buffers
    from oracle import oracle as O
    lr = 0.05
    w0 = O.fill_normal(n, 11, 0.05)
    g0 = O.fill_normal(n, 12, 0.01)
    l0 = O.fill_normal(n, 13, 0.001)
    s0 = O.fill_normal(n, 14, 1.0)
    dev = torch.device("cuda:0")
    w, g, last, s = (torch.from_numpy(a.copy()).to(dev) for a in (w0, g0, l0, s0))
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(2):  # two tasks back to back
        optimise_buffers(stream.cuda_stream, w.data_ptr(), g.data_ptr(), last.data_ptr() if mom > 0 else None,
                         s.data_ptr(), n, lr, mom, wd)
        O.sma_optimise(-lr, mom, wd, w0, g0, l0 if mom > 0 else None, s0)
    stream.synchronize()
    assert _bits_equal(w.cpu().numpy(), w0), "w"
    assert _bits_equal(g.cpu().numpy(), g0), "g"
    assert _bits_equal(s.cpu().numpy(), s0), "s"
    assert _bits_equal(last.cpu().numpy(), l0), "last"


@pytest.mark.parametrize("n,R,mom,wd,buckets", [(4099, 3, 0.9, 1e-4, 0), (300_007, 2, 0.0, 0.0, 0),
                                                 (1, 1, 0.9, 1e-4, 0)])
def test_seam_ssgd_one_gpu_bitexact(n, R, mom, wd, buckets):
    """Synchronous SGD through the seam: task steps (cbx_ssgd_accumulate_buffers)
    into the caller's base gradient, then the barrier (cbx_ssgd_plan_step),
    two clocks, against the oracle's synchronoussgd.cu / .c restatement.
    One rank always runs one apply pass (include/crossbow_sma.h): `buckets`
    must have no effect, which the bit-exact result at every setting shows;
    bucketing itself is covered by the multi-rank seam tests."""
    import torch

    from crossbow_amd.seam import SmaPlan, ssgd_accumulate_buffers
    from oracle import oracle as O
    lr, wpc = 0.05, 2 * R
    st = O.make_state(n, 1, R, ALPHA, mom)
    acc0 = np.zeros(n, np.float32)
    dev = torch.device("cuda:0")
    z = torch.from_numpy(st.z[0].copy()).to(dev)
    last = torch.from_numpy(st.last[0].copy()).to(dev) if mom > 0 else None
    w = [torch.from_numpy(a.copy()).to(dev) for a in st.w]
    acc = torch.zeros(n, device=dev)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    task = 0
    with SmaPlan([0], n, buckets=buckets) as plan:
        for clock in range(2):
            for k in range(wpc):
                i = k % R
                g0 = O.fill_normal(n, 9000 + task, 0.01)
                g = torch.from_numpy(g0.copy()).to(dev)
                torch.cuda.synchronize()
                ssgd_accumulate_buffers(stream.cuda_stream, w[i].data_ptr(), g.data_ptr(), acc.data_ptr(), n, lr, wd)
                O.ssgd_worker(np.float32(-lr), wd, st.w[i], g0, acc0)
                stream.synchronize()
                assert _bits_equal(g.cpu().numpy(), g0), f"task {task}: g"
                task += 1
            st.locked[:] = 1
            if clock == 1:
                st.locked[0] = 0  # a held replica keeps its weights (common.c:208)
            plan.ssgd_step([stream.cuda_stream], [z.data_ptr()], [last.data_ptr()] if last is not None else None,
                           [acc.data_ptr()], [(0, w[i].data_ptr(), int(st.locked[i])) for i in range(R)], mom, wpc)
            O.ssgd_sync(st, [acc0], wpc)
        stream.synchronize()
    assert _bits_equal(z.cpu().numpy(), st.z[0]), "z"
    if last is not None:
        assert _bits_equal(last.cpu().numpy(), st.last[0]), "last"
    assert _bits_equal(acc.cpu().numpy(), acc0), "acc must be reset"
    for i in range(R):
        assert _bits_equal(w[i].cpu().numpy(), st.w[i]), f"w[{i}]"


def test_seam_refuses_bad_arguments():
    import torch

    from crossbow_amd import CbxError
    from crossbow_amd._lib import CBX_ERR_INVALID
    from crossbow_amd.seam import SmaPlan, optimise_buffers
    n = 4099
    buf = torch.zeros(4 * n + 8, device="cuda:0")
    p = buf.data_ptr()
    stream = torch.cuda.Stream()
    with SmaPlan([0], n) as plan:
        with pytest.raises(CbxError) as e:  # misaligned replica buffer
            plan.step([stream.cuda_stream], [p], None, [(0, p + 4, p, 1, 0)], ALPHA, 0.0)
        assert e.value.code == CBX_ERR_INVALID and "aligned" in str(e.value)
        with pytest.raises(CbxError):  # momentum without last buffers
            plan.step([stream.cuda_stream], [p], None, [], ALPHA, 0.9)
        with pytest.raises(CbxError):  # replica on a device the plan does not have
            plan.step([stream.cuda_stream], [p], None, [(1, p, p, 1, 0)], ALPHA, 0.0)
        with pytest.raises(CbxError):  # first out of range
            plan.step([stream.cuda_stream], [p], None, [], ALPHA, 0.0, first=1)
    with pytest.raises(CbxError):
        SmaPlan([0], 0)
    with pytest.raises(CbxError):
        optimise_buffers(stream.cuda_stream, p + 4, p, None, p, 16, 0.1, 0.0, 0.0)


# ---- G devices in one process: the loopback clique --------------------------

class _Dev:
    """Raw device buffers and streams through the HIP runtime (torch-free)."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        self.hip.hipFree.argtypes = [ctypes.c_void_p]
        self.hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        self.hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        self.ptrs, self.streams = [], []

    def upload(self, arr):
        a = np.ascontiguousarray(arr, np.float32)
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), max(16, a.nbytes)) == 0
        assert self.hip.hipMemcpy(p, a.ctypes.data, a.nbytes, 1) == 0
        self.ptrs.append(p.value)
        return p.value

    def download(self, p, n):
        out = np.empty(n, np.float32)
        assert self.hip.hipMemcpy(out.ctypes.data, p, out.nbytes, 2) == 0
        return out

    def stream(self):
        s = ctypes.c_void_p()
        assert self.hip.hipStreamCreate(ctypes.byref(s)) == 0
        self.streams.append(s.value)
        return s.value

    def sync(self):
        for s in self.streams:
            assert self.hip.hipStreamSynchronize(s) == 0

    def free(self):
        self.sync()
        for s in self.streams:
            self.hip.hipStreamDestroy(s)
        for p in self.ptrs:
            self.hip.hipFree(p)


def _seam_standalone():
    """crossbow_amd/seam.py without the package (whose __init__ loads torch)."""
    spec = importlib.util.spec_from_file_location("cbx_seam_standalone",
                                                  os.path.join(C.ROOT, "crossbow_amd", "seam.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _run_devices(L, world, local, n, R, mom, steps, copy_at, held, exact, comms=None, first=0, buckets=0):
    """The seam over `local` devices (positions of this process's devices in
    a G = world job; replica i on device i % world).  Returns (bad, digest of
    z / last per device, differing elements)."""
    SmaPlan = _seam_standalone().SmaPlan
    O = C.oracle()
    st = O.make_state(n, world, R, ALPHA, mom)
    st.first = first
    size = world * R
    mem = _Dev()
    z = {d: mem.upload(st.z[d]) for d in local}
    last = {d: mem.upload(st.last[d]) for d in local} if mom > 0 else None
    w = {i: mem.upload(st.w[i]) for i in range(size) if i % world in local}
    s = {i: mem.upload(st.s[i]) for i in range(size) if i % world in local}
    streams = [mem.stream() for _ in local]
    pos = {d: k for k, d in enumerate(local)}
    plan = SmaPlan([0] * len(local), n, comms=comms, lib=L, buckets=buckets)
    try:
        for step in range(steps):
            st.locked[:] = 1
            for i in held.get(step, ()):
                st.locked[i] = 0
            if step in copy_at:
                st.copy[copy_at[step]] = 1
            reps = [(pos[i % world], w[i], s[i], int(st.locked[i]), int(st.copy[i])) if i in w else (0, 0, 0, 0, 0)
                    for i in range(size)]
            local_copies = sum(int(st.copy[i]) for i in w if st.locked[i] and i >= first)
            ran = plan.step(streams, [z[d] for d in local], [last[d] for d in local] if last else None, reps,
                            ALPHA, mom, first)
            O.sma_step(st)
            assert ran == (1 if local_copies else 0), (step, ran, local_copies)
        mem.sync()
        check = C.Checker(exact=exact)
        dig = {}
        for d in local:
            zd = mem.download(z[d], n)
            ld = mem.download(last[d], n) if last else np.zeros(0, np.float32)
            dig[d] = C.digest(zd, ld)
            check(f"z[{d}]", zd, st.z[d])
            if last:
                check(f"last[{d}]", ld, st.last[d])
        for i in w:
            check(f"w[{i}]", mem.download(w[i], n), st.w[i])
        return check.bad, dig, check.differs
    finally:
        plan.free()
        mem.free()


def _run_ssgd_devices(L, world, local, n, R, mom, steps, exact, comms=None, buckets=0):
    """S-SGD through the seam over `local` devices of a G = world job: each
    process runs its replicas' tasks into its devices' accumulators, then the
    barrier.  Returns (bad, digest of z / last per device, differing elements)."""
    seam = _seam_standalone()
    O = C.oracle()
    lr, wd, wpc = 0.05, 1e-4, 2 * world * R
    st = O.make_state(n, world, R, ALPHA, mom)
    size = world * R
    mem = _Dev()
    z = {d: mem.upload(st.z[d]) for d in local}
    last = {d: mem.upload(st.last[d]) for d in local} if mom > 0 else None
    w = {i: mem.upload(st.w[i]) for i in range(size) if i % world in local}
    zeros = np.zeros(n, np.float32)
    acc = {d: mem.upload(zeros) for d in local}
    acc_ref = [zeros.copy() for _ in range(world)]
    gbuf = mem.upload(zeros)
    streams = [mem.stream() for _ in local]
    pos = {d: k for k, d in enumerate(local)}
    plan = seam.SmaPlan([0] * len(local), n, comms=comms, lib=L, buckets=buckets)
    try:
        task = 0
        for step in range(steps):
            for k in range(wpc):  # the global task list; each process runs its replicas' tasks
                i = k % size
                g0 = O.fill_normal(n, 5000 + task, 0.01)
                if i in w:
                    mem.sync()
                    assert mem.hip.hipMemcpy(gbuf, g0.ctypes.data, g0.nbytes, 1) == 0
                    seam.ssgd_accumulate_buffers(streams[pos[i % world]], w[i], gbuf, acc[i % world], n, lr, wd, lib=L)
                    mem.sync()
                O.ssgd_worker(np.float32(-lr), wd, st.w[i], g0, acc_ref[i % world])
                task += 1
            st.locked[:] = 1
            reps = [(pos[i % world], w[i], 1) if i in w else (0, 0, 0) for i in range(size)]
            plan.ssgd_step(streams, [z[d] for d in local], [last[d] for d in local] if last else None,
                           [acc[d] for d in local], reps, mom, wpc)
            O.ssgd_sync(st, acc_ref, wpc)
        mem.sync()
        check = C.Checker(exact=exact)
        dig = {}
        for d in local:
            zd = mem.download(z[d], n)
            ld = mem.download(last[d], n) if last else np.zeros(0, np.float32)
            dig[d] = C.digest(zd, ld)
            check(f"ssgd z[{d}]", zd, st.z[d])
            if last:
                check(f"ssgd last[{d}]", ld, st.last[d])
            check(f"ssgd acc[{d}] reset", mem.download(acc[d], n), zeros)
        for i in w:
            check(f"ssgd w[{i}]", mem.download(w[i], n), st.w[i])
        return check.bad, dig, check.differs
    finally:
        plan.free()
        mem.free()


def _run_bn_plan(L, world, local, exact, comms=None):
    """BN running-statistics averaging through the plan
    (cbx_sma_plan_average_batchnorm) over the caller's buffers: three layers,
    non-counting devices poisoned with NaN / +-Inf (the reference never reads
    them, cudnnbatchnormparams.c:177-184).  Returns the list of mismatches."""
    seam = _seam_standalone()
    O = C.oracle()
    elements = [16, 40, 7]
    updated = [[1, 1, 1]] + [[1, 0, 1] if d % 2 else [0, 1, 1] for d in range(1, world)]
    mean = [[O.fill_normal(e, 50 + 10 * d + l, 0.5) for l, e in enumerate(elements)] for d in range(world)]
    var = [[O.fill_normal(e, 90 + 10 * d + l, 0.5) for l, e in enumerate(elements)] for d in range(world)]
    for d in range(1, world):
        for l in range(len(elements)):
            if not updated[d][l]:
                mean[d][l][:] = np.nan
                var[d][l][::2] = np.inf
                var[d][l][1::2] = -np.inf
    ref_m = [[a.copy() for a in r] for r in mean]
    ref_v = [[a.copy() for a in r] for r in var]
    O.bn_average(ref_m, ref_v, updated)
    mem = _Dev()
    pm = {(d, l): mem.upload(mean[d][l]) for d in local for l in range(len(elements))}
    pv = {(d, l): mem.upload(var[d][l]) for d in local for l in range(len(elements))}
    plan = seam.SmaPlan([0] * len(local), 4096, comms=comms, lib=L)
    try:
        L3 = len(elements)
        plan.average_batchnorm(elements, [pm[(d, l)] for d in local for l in range(L3)],
                               [pv[(d, l)] for d in local for l in range(L3)],
                               [updated[d][l] for d in local for l in range(L3)])
        check = C.Checker(exact=exact)
        for d in local:
            for l, e in enumerate(elements):
                check(f"bn mean[{l}] on device {d}", mem.download(pm[(d, l)], e), ref_m[d][l])
                check(f"bn var[{l}] on device {d}", mem.download(pv[(d, l)], e), ref_v[d][l])
        return check.bad
    finally:
        plan.free()
        mem.free()


def _run_golden_devices(L, world, local, gcase, comms=None):
    """One committed G > 1 fixture through the seam over `local` devices, bit
    for bit (rank-order loopback or G = 2).  Returns the list of mismatches."""
    seam = _seam_standalone()
    st = gcase["state"]
    n, size = st.n, st.size
    mem = _Dev()
    z = {d: mem.upload(st.z[d]) for d in local}
    last = {d: mem.upload(st.last[d]) for d in local} if st.last is not None else None
    mine = [i for i in range(size) if i % world in local]
    w = {i: mem.upload(st.w[i]) for i in mine}
    s_ = {i: mem.upload(st.s[i]) for i in mine}
    streams = [mem.stream() for _ in local]
    pos = {d: k for k, d in enumerate(local)}
    plan = seam.SmaPlan([0] * len(local), n, comms=comms, lib=L)
    try:
        reps = [(pos[i % world], w[i], s_[i], int(st.locked[i]), int(st.copy[i])) if i in w else (0, 0, 0, 0, 0)
                for i in range(size)]
        plan.step(streams, [z[d] for d in local], [last[d] for d in local] if last else None, reps, st.alpha,
                  st.momentum, st.first)
        mem.sync()
        check = C.Checker(exact=True)
        for d in local:
            check(f"{gcase['name']} z[{d}]", mem.download(z[d], n), gcase["z_out"][d])
            if last:
                check(f"{gcase['name']} last[{d}]", mem.download(last[d], n), gcase["last_out"][d])
        for i in mine:
            check(f"{gcase['name']} w[{i}]", mem.download(w[i], n), gcase["w_out"][i])
        return check.bad
    finally:
        plan.free()
        mem.free()


DEVICE_CASES = [
    # (name, n, R, momentum, steps, {step: copy replica}, {step: held replicas}, first, order, caller comms,
    #  buckets: 0 = the default pipeline of 8, 1 = in order on the caller's stream)
    ("plan-comms", 50_001, 2, 0.9, 3, {1: 3}, {0: (1,)}, 0, "rank", False, 0),
    ("plan-comms-in-order", 50_001, 2, 0.9, 3, {1: 3}, {0: (1,)}, 0, "rank", False, 1),
    ("caller-comms", 50_001, 2, 0.9, 2, {}, {}, 1, "rank", True, 0),
    ("tail-only", 1021, 3, 0.9, 2, {1: 0}, {}, 0, "rank", False, 0),  # below one kernel trip: no bulk launch
    ("no-momentum", 20_011, 1, 0.0, 2, {}, {}, 0, "rank", False, 3),
    ("many-buckets", 300_007, 2, 0.9, 4, {2: 1}, {1: (0,)}, 0, "rank", False, 37),  # more buckets than trips allow
    ("ring-order", 300_007, 2, 0.9, 3, {2: 1}, {}, 0, "ring", False, 0),
]


def _device_worker(G, q):
    try:
        L, A = C.load_variant()
        F = ctypes.CDLL(os.path.join(C.ROOT, "tests", "native", "libfakerccl.so"))
        out = []
        for name, n, R, mom, steps, copy_at, held, first, order, caller, buckets in DEVICE_CASES:
            if order == "ring" and G < 3:
                continue
            os.environ["FAKE_RCCL_ORDER"] = order
            comms = None
            if caller:  # the caller's communicators, as executioncontext.c:185-201 creates them
                arr = (ctypes.c_void_p * G)()
                devs = (ctypes.c_int * G)(*([0] * G))
                assert F.ncclCommInitAll(arr, G, devs) == 0
                comms = [arr[k] for k in range(G)]
            try:
                bad, dig, differs = _run_devices(L, G, list(range(G)), n, R, mom, steps, copy_at, held,
                                                 exact=order == "rank", comms=comms, first=first,
                                                 buckets=buckets)
            finally:
                for c in comms or ():
                    F.ncclCommDestroy(ctypes.c_void_p(c))
            out.append((name, order, bad, len(set(dig.values())), differs))
        for name, buckets in (("ssgd", 0), ("ssgd-in-order", 1)):
            os.environ["FAKE_RCCL_ORDER"] = "rank"
            bad, dig, differs = _run_ssgd_devices(L, G, list(range(G)), 40_009, 2, 0.9, 2, exact=True,
                                                  buckets=buckets)
            out.append((name, "rank", bad, len(set(dig.values())), differs))
        out.append(("bn", "rank", _run_bn_plan(L, G, list(range(G)), exact=True), 1, 0))
        for gcase in C.golden_cases(G):
            os.environ["FAKE_RCCL_ORDER"] = "rank"
            out.append((f"golden {gcase['name']}", "rank", _run_golden_devices(L, G, list(range(G)), gcase), 1, 0))
        q.put((out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((None, traceback.format_exc()))


def _spawn(target, args, timeout=110):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=args + (q,))
    p.start()
    try:
        return q.get(timeout=timeout)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()


@pytest.mark.skipif(not os.path.exists(C.VARIANT), reason="run scripts/build_fake_rccl.sh first")
@pytest.mark.parametrize("G", [2, 4, 8])
def test_seam_devices_one_process(G):
    res, err = _spawn(_device_worker, (G,))
    assert err is None, err
    assert res, "no case ran"
    for name, order, bad, distinct, differs in res:
        assert not bad, (name, bad)
        assert distinct == 1, f"{name}: z / last differ across devices"
        if order == "ring":
            assert differs > 0, f"{name}: ring order never left the oracle's order"


# ---- G ranks with the real librccl ------------------------------------------

class _Uid(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def _rank_worker(world, rank, d, buckets, kind, q):
    try:
        from tests.test_gpu_realrccl import load_real, rank_env
        rank_env(rank)
        L, A = load_real()
        R = ctypes.CDLL("librccl.so.1")
        path = os.path.join(d, "uid")
        if rank == 0:
            uid = _Uid()
            assert R.ncclGetUniqueId(ctypes.byref(uid)) == 0
            with open(path + ".tmp", "wb") as f:
                f.write(bytes(uid))
            os.replace(path + ".tmp", path)
        C.wait_files([path])
        uid = _Uid.from_buffer_copy(open(path, "rb").read())
        comm = ctypes.c_void_p()
        R.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _Uid, ctypes.c_int]
        assert R.ncclCommInitRank(ctypes.byref(comm), world, uid, rank) == 0
        try:
            if kind == "bn":
                bad, dig, differs = _run_bn_plan(L, world, [rank], exact=world == 2, comms=[comm.value]), "bn", 0
            elif kind == "ssgd":
                bad, dig, differs = _run_ssgd_devices(L, world, [rank], 100_003, 2, 0.9, 2, exact=world == 2,
                                                      comms=[comm.value], buckets=buckets)
            else:
                bad, dig, differs = _run_devices(L, world, [rank], 200_003, 2, 0.9, 3, {1: (world - 1) * 2 + 1},
                                                 {2: (0,)}, exact=world == 2, comms=[comm.value], buckets=buckets)
        finally:
            R.ncclCommDestroy(comm)
        q.put(((bad, dig if kind == "bn" else dig[rank], differs), None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((None, traceback.format_exc()))


@pytest.mark.parametrize("world,buckets,kind", [(2, 0, "sma"), (2, 1, "sma"), (4, 0, "sma"), (4, 5, "sma"),
                                                (2, 0, "ssgd"), (4, 0, "ssgd"), (4, 0, "bn")])
def test_seam_real_rccl_ranks(world, buckets, kind):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        qs, ps = [], []
        for rank in range(world):
            q = ctx.Queue()
            p = ctx.Process(target=_rank_worker, args=(world, rank, d, buckets, kind, q))
            p.start()
            qs.append(q)
            ps.append(p)
        try:
            res = [q.get(timeout=110) for q in qs]
        finally:
            for p in ps:
                p.join(timeout=30)
                if p.is_alive():
                    p.kill()
    errs = [e for _, e in res if e]
    assert not errs, errs[0]
    outs = [r for r, _ in res]
    for rank, (bad, _, _) in enumerate(outs):
        assert not bad, (rank, bad)
    assert len({dg for _, dg, _ in outs}) == 1, "z / last differ across ranks"


def test_seam_largest_model_windows_bitexact():
    """The largest model the reference's `int bytes` allows (model.h:35):
    n = 536,870,911 floats per caller-owned buffer, the tail's byte offsets
    just below 2^31.  The step is elementwise, so dense windows (head, around
    byte 2^30, the last whole trip and the tail) are checked against the
    oracle run on the same windows, bit for bit."""
    import torch

    from crossbow_amd.seam import SmaPlan
    from oracle import oracle as O
    n, R, mom = (2**31 - 1) // 4, 2, 0.9
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    z = torch.randn(n, device=dev, generator=gen) * 0.05
    last = torch.randn(n, device=dev, generator=gen) * 0.001
    s = [z + 0.01 * torch.randn(n, device=dev, generator=gen) for _ in range(R)]
    w = [si + 0.001 * torch.randn(n, device=dev, generator=gen) for si in s]
    bulk = (n // 4) // 256 * 256 * 4  # the seam's bulk/tail boundary (kTailQuantum4)
    windows = [(0, 70_000), ((1 << 28) - 35_000, (1 << 28) + 35_000), (bulk - 40_000, n)]
    before = [[t[a:b].cpu().numpy().copy() for t in [z, last] + s + w] for a, b in windows]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with SmaPlan([0], n) as plan:
        plan.step([stream.cuda_stream], [z.data_ptr()], [last.data_ptr()],
                  [(0, w[i].data_ptr(), s[i].data_ptr(), 1, 0) for i in range(R)], ALPHA, mom)
        stream.synchronize()
    for (a, b), arrs in zip(windows, before):
        st = O.SmaState(1, R, b - a, ALPHA, mom, [arrs[0]], [arrs[1]], arrs[2:2 + R], arrs[2 + R:])
        O.sma_step(st)
        assert _bits_equal(z[a:b].cpu().numpy(), st.z[0]), f"z[{a}:{b}]"
        assert _bits_equal(last[a:b].cpu().numpy(), st.last[0]), f"last[{a}:{b}]"
        for i in range(R):
            assert _bits_equal(w[i][a:b].cpu().numpy(), st.w[i]), f"w[{i}][{a}:{b}]"
    del z, last, s, w
    torch.cuda.empty_cache()
