"""Shared by the G > 1 GPU tests that run on ONE GPU through the loopback
collective (tests/native/fake_rccl.cpp):

* tests/test_gpu_multirank.py   -- G processes, each one rank of a G-GPU job
  (cbx_init_rank, the one-process-per-GPU form bench.py uses);
* tests/test_gpu_multidevice.py -- one process driving G devices
  (cbx_init over G devices: the reference's own single-process form,
  ncclCommInitAll + grouped ncclAllReduce, executioncontext.c:185-201,
  synch/common.c:14-54).

Both load tests/native/libcrossbow_sma_fakerccl.so (the library's own sources
linked against the loopback, scripts/build_fake_rccl.sh) through the
torch-free crossbow_amd/_abi.py, so no real RCCL sits beside the loopback one.

Every device is device 0 of the box.  Each check compares the library with
the oracle run with the same G on the same inputs:
* loopback order "rank" (the default): rank-order sums, bit for bit;
* loopback order "ring": the ring all-reduce's order, which is not the
  oracle's for G >= 3, so the check is the stated G > 1 tolerance
  (rtol 1e-5, atol 1e-6) plus the property the design rests
  on: z and last are bitwise identical on every device (sma.c:168-174, every
  device applies the same D).

Test infrastructure only; imported by the two test modules and run inside
their spawned worker processes.
"""
from __future__ import annotations

import ctypes
import hashlib
import importlib.util
import os
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(ROOT, "tests", "native", "libcrossbow_sma_fakerccl.so")
RTOL, ATOL = 1e-5, 1e-6  # the G > 1 tolerance (RCCL's sum order is not rank order)


def abi():
    spec = importlib.util.spec_from_file_location("cbx_abi_standalone", os.path.join(ROOT, "crossbow_amd", "_abi.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def oracle():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from oracle import oracle as O
    return O


def load_variant():
    A = abi()
    return A.bind(ctypes.CDLL(VARIANT)), A


def loopback_dir(need_bytes: int = 1 << 30) -> str:
    """/dev/shm when it has room (fast), else the system temp directory."""
    try:
        st = os.statvfs("/dev/shm")
        if st.f_bavail * st.f_frsize >= need_bytes and os.access("/dev/shm", os.W_OK):
            return "/dev/shm"
    except OSError:
        pass
    import tempfile
    return tempfile.gettempdir()


class Ctx:
    """One library context bound through ctypes; calls raise on a negative code."""

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

    def free(self):
        self.L.cbx_free(self.c)


def init_local(L, A, G: int) -> Ctx:
    """cbx_init over G devices, all of them device 0 (the loopback's clique)."""
    c = ctypes.c_void_p()
    devs = (ctypes.c_int * G)(*([0] * G))
    if L.cbx_init(ctypes.byref(c), devs, G) < 0:
        raise RuntimeError(L.cbx_last_error().decode())
    return Ctx(L, A, c)


def init_rank(L, A, rank: int, world: int, uid: bytes) -> Ctx:
    c = ctypes.c_void_p()
    ub = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
    if L.cbx_init_rank(ctypes.byref(c), 0, world, rank, ub) < 0:
        raise RuntimeError(L.cbx_last_error().decode())
    return Ctx(L, A, c)


@dataclass
class Case:
    name: str
    n: int
    R: int                     # replicas per device
    mom: float
    steps: int
    bucket: int = 0            # elements per bucket (0: library default)
    copy: Dict[int, int] = field(default_factory=dict)   # step -> replica asking for Phase D
    held: Dict[int, int] = field(default_factory=dict)   # step -> replica busy on the task side (SSP)
    staged: int = 0            # > 0: cbx_synchronise_staged over that many buckets
    staging: int = 0           # cbx_set_staging_mode: 0 zero-copy kernels, 1 DMA copies
    utype: int = 7             # update model: 7 SMA, 3 SYNCHRONOUSEAMSGD, 1 WORKER (S-SGD)
    mode: int = 0              # cbx_set_pipeline_mode
    stride: int = 1            # cbx_set_cross_wait_stride
    group: int = 1             # cbx_set_allreduce_group
    order: str = "rank"        # loopback summation order ("rank" or "ring")
    algo: int = 0              # cbx_set_allreduce_algorithm: 0 RCCL, 1 peer reads (one process only)
    algo_at: Dict[int, int] = field(default_factory=dict)  # step -> algorithm switched to before it


def digest(*arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a, np.float32).tobytes())
    return h.hexdigest()


class Checker:
    """Bit-exact in rank order; the G > 1 tolerance otherwise, counting how
    many elements actually differ (so a tolerance case that never left the
    oracle's order is visible)."""

    def __init__(self, exact: bool):
        self.exact = exact
        self.bad: List[str] = []
        self.differs = 0

    def __call__(self, what, got, want):
        got = np.asarray(got, np.float32)
        want = np.asarray(want, np.float32)
        ne = int(np.sum(got.view(np.uint32) != want.view(np.uint32)))
        self.differs += ne
        if self.exact:
            if ne:
                self.bad.append(f"{what}: {ne} differ")
        elif not np.allclose(got, want, rtol=RTOL, atol=ATOL, equal_nan=False):
            err = float(np.max(np.abs(got.astype(np.float64) - want)))
            self.bad.append(f"{what}: outside rtol {RTOL} / atol {ATOL} (max abs err {err:.3g})")


def setup_model(g: Ctx, A, n: int, R: int, mom: float, utype: int, sync: int, wpc: int, alpha: float = 0.1):
    shape = (ctypes.c_int * 1)(n)
    g("cbx_set_model", 1, 4 * n)
    g("cbx_set_model_variable", 0, 1, 1, shape, 4 * n)
    g("cbx_set_update_model_type", utype)
    g("cbx_set_eamsgd_alpha", ctypes.c_float(alpha))
    g("cbx_set_momentum", ctypes.c_float(mom), 0)
    g("cbx_set_weight_decay", ctypes.c_float(1e-4))
    g("cbx_set_learning_rate_decay_policy_fixed", ctypes.c_float(0.05))
    g("cbx_set_model_work_per_clock", wpc)
    g("cbx_set_model_manager", R, sync)


def run_case(g: Ctx, world: int, local: List[int], case: Case, after_setup=None) -> dict:
    """One case on the devices `local` of a G = `world` job.  Returns
    {"bad": [...], "digest": {device: sha of z and last}, "differs": n}.
    `after_setup(g)` runs once the model manager exists (the per-rank
    peer-read form maps the other ranks' buffers there)."""
    O = oracle()
    A = g.A
    n, R, mom = case.n, case.R, case.mom
    wpc = 2 * world * R
    setup_model(g, A, n, R, mom, case.utype, A.SYNC_SSP if case.held else A.SYNC_BSP, wpc)
    if after_setup:
        after_setup(g)
    if case.bucket:
        g("cbx_set_bucket_elements", ctypes.c_longlong(case.bucket))
    g("cbx_set_pipeline_mode", case.mode)
    g("cbx_set_cross_wait_stride", case.stride)
    g("cbx_set_allreduce_group", case.group)
    if case.algo:
        g("cbx_set_allreduce_algorithm", case.algo)
    g("cbx_set_staging_mode", case.staging)
    size = world * R
    assert g("cbx_num_replicas") == size and g("cbx_num_devices") == world
    mine = [i for i in range(size) if i % world in local]
    # The theta queue hands out this process's replicas only, round robin (modelmanager.c:180-190).
    clk = ctypes.c_int(-1)
    got = [g("cbx_acquire_access", ctypes.byref(clk)) for _ in mine]
    assert got == mine and clk.value == 0, got
    for i in got:
        g("cbx_replica_lock", i)
        g("cbx_replica_release", i)
    st = O.make_state(n, world, R, 0.1, mom)
    for d in local:
        if case.staged:
            g.host("cbx_base_host_buffer", d, A.BUF_DATA, n)[:] = st.z[d]
            g.host("cbx_base_host_buffer", d, A.BUF_LAST, n)[:] = st.last[d]
        else:
            g.write("cbx_base_write", d, A.BUF_DATA, st.z[d])
            if mom > 0:
                g.write("cbx_base_write", d, A.BUF_LAST, st.last[d])
    for i in mine:
        if case.staged:
            g.host("cbx_replica_host_buffer", i, A.BUF_DIFF, n)[:] = st.s[i]
            g.host("cbx_replica_host_buffer", i, A.BUF_DATA, n)[:] = st.w[i]
        else:
            g.write("cbx_replica_write", i, A.BUF_DIFF, st.s[i])
            g.write("cbx_replica_write", i, A.BUF_DATA, st.w[i])
    acc = [np.zeros(n, np.float32) for _ in range(world)]
    task = 0
    for step in range(case.steps):
        if step in case.algo_at:
            g("cbx_set_allreduce_algorithm", case.algo_at[step])
        if case.utype == 1:  # S-SGD task steps: the global task list, each process runs its replicas' tasks
            for k in range(wpc):
                i = k % size
                gr = O.fill_normal(n, 5000 + task, 0.01)
                if i % world in local:
                    g.write("cbx_replica_write", i, A.BUF_GRADIENT, gr)
                    g("cbx_replica_optimise", i, task, None)
                O.ssgd_worker(np.float32(-0.05), 1e-4, st.w[i], gr, acc[i % world])
                task += 1
        st.locked[:] = 1
        if step in case.copy:
            i = case.copy[step]
            st.copy[i] = 1
            if i % world in local:
                g("cbx_replica_set_copy", i, 1)
        hold = case.held.get(step)
        if hold is not None:
            st.locked[hold] = 0
            if hold % world in local:
                g("cbx_replica_lock", hold)
        g("cbx_lock_any")
        if case.staged:
            g("cbx_synchronise_staged", 0, step + 1, 0, case.staged)
        else:
            g("cbx_synchronise", 0, step + 1, 0, 0)
        g("cbx_unlock_any")
        if hold is not None and hold % world in local:
            g("cbx_replica_unlock", hold)
        if case.utype == 1:
            O.ssgd_sync(st, acc, wpc)
        else:
            O.sma_step(st)
    g("cbx_wait")
    check = Checker(exact=case.order == "rank" or world < 3)
    dig = {}
    for d in local:
        z = g.read("cbx_base_read", d, A.BUF_DATA, n)
        last = g.read("cbx_base_read", d, A.BUF_LAST, n) if mom > 0 else np.zeros(0, np.float32)
        dig[d] = digest(z, last)
        if case.staged:
            check(f"z[{d}] (host)", g.host("cbx_base_host_buffer", d, A.BUF_DATA, n), st.z[d])
            check(f"last[{d}] (host)", g.host("cbx_base_host_buffer", d, A.BUF_LAST, n), st.last[d])
        check(f"z[{d}]", z, st.z[d])
        if mom > 0:
            check(f"last[{d}]", last, st.last[d])
    for i in mine:
        if case.staged:
            check(f"w[{i}] (host)", g.host("cbx_replica_host_buffer", i, A.BUF_DATA, n), st.w[i])
        check(f"w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
        if g("cbx_replica_get_copy", i) != 0:
            check.bad.append(f"copy flag of replica {i} not reset")
    return {"bad": check.bad, "digest": dig, "differs": check.differs}


def run_golden(g: Ctx, world: int, local: List[int], gcase: dict, algo: int = 0, exact: bool = True,
               after_setup=None) -> List[str]:
    """One committed fixture (tests/golden/, G = world): one step, bit for bit
    (or, with `exact` False, within the G > 1 tolerance: real RCCL's order)."""
    A = g.A
    st = gcase["state"]
    n = st.n
    R = st.size // st.G
    held = [int(i) for i in np.nonzero(st.locked == 0)[0]]
    setup_model(g, A, n, R, st.momentum, 7, A.SYNC_SSP if held else A.SYNC_BSP, 2 * st.size, alpha=st.alpha)
    if after_setup:
        after_setup(g)
    if algo:
        g("cbx_set_allreduce_algorithm", algo)
    mine = [i for i in range(st.size) if i % world in local]
    for d in local:
        g.write("cbx_base_write", d, A.BUF_DATA, st.z[d])
        if st.last is not None:
            g.write("cbx_base_write", d, A.BUF_LAST, st.last[d])
    for i in mine:
        g.write("cbx_replica_write", i, A.BUF_DIFF, st.s[i])
        g.write("cbx_replica_write", i, A.BUF_DATA, st.w[i])
        if st.copy[i]:
            g("cbx_replica_set_copy", i, 1)
    for i in held:
        if i in mine:
            g("cbx_replica_lock", i)
    g("cbx_lock_any")
    g("cbx_synchronise", st.first, 1, 0, 0)
    g("cbx_unlock_any")
    for i in held:
        if i in mine:
            g("cbx_replica_unlock", i)
    g("cbx_wait")
    check = Checker(exact=exact)
    for d in local:
        check(f"{gcase['name']} z[{d}]", g.read("cbx_base_read", d, A.BUF_DATA, n), gcase["z_out"][d])
        if gcase["last_out"] is not None:
            check(f"{gcase['name']} last[{d}]", g.read("cbx_base_read", d, A.BUF_LAST, n), gcase["last_out"][d])
    for i in mine:
        check(f"{gcase['name']} w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), gcase["w_out"][i])
    return check.bad


def golden_cases(world: int):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from tests.test_oracle import load_golden_cases
    return [c for c in load_golden_cases() if c["G"] == world]


def _hip():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return hip


def run_bn(g: Ctx, world: int, local: List[int], poison: bool, exact: bool = True) -> List[str]:
    """BN running-statistics averaging (cudnnbatchnormparams.c:157-222) of
    three layers.  With `poison`, a device whose layer does not count holds
    NaN / Inf there: the reference never reads it (:177-184), so the average
    must be the oracle's, finite, on every device.  `exact` False: within the
    G > 1 tolerance (real RCCL's summation order)."""
    O = oracle()
    A = g.A
    n = 4096
    setup_model(g, A, n, 1, 0.0, 7, A.SYNC_BSP, 2)
    elements = [16, 40, 7]
    updated = [[1, 1, 1]] + [[1, 0, 1] if d % 2 else [0, 1, 1] for d in range(1, world)]
    mean = [[O.fill_normal(e, 50 + 10 * d + l, 0.5) for l, e in enumerate(elements)] for d in range(world)]
    var = [[O.fill_normal(e, 90 + 10 * d + l, 0.5) for l, e in enumerate(elements)] for d in range(world)]
    if poison:
        for d in range(1, world):
            for l in range(len(elements)):
                if not updated[d][l]:
                    mean[d][l][:] = np.nan
                    var[d][l][::2] = np.inf
                    var[d][l][1::2] = -np.inf
    ref_m = [[a.copy() for a in r] for r in mean]
    ref_v = [[a.copy() for a in r] for r in var]
    O.bn_average(ref_m, ref_v, updated)
    hip = _hip()
    L3 = len(elements)
    ptrs = {}
    for d in local:
        # device scratch for the statistics: that device's base-model gradient buffer
        p = ctypes.c_void_p()
        g("cbx_base_buffer", d, A.BUF_GRADIENT, ctypes.byref(p))
        off = 0
        pm, pv = [], []
        for l, e in enumerate(elements):
            for arr, lst in ((mean[d][l], pm), (var[d][l], pv)):
                dst = p.value + 4 * off
                assert hip.hipMemcpy(dst, arr.ctypes.data, 4 * e, 1) == 0
                lst.append(dst)
                off += e
        ptrs[d] = (pm, pv)
    # argument layout: [local device k][layer l] at k * layers + l (include/crossbow_sma.h)
    el = (ctypes.c_int * L3)(*elements)
    pm = (ctypes.c_void_p * (L3 * len(local)))(*[x for d in local for x in ptrs[d][0]])
    pv = (ctypes.c_void_p * (L3 * len(local)))(*[x for d in local for x in ptrs[d][1]])
    up = (ctypes.c_int * (L3 * len(local)))(*[u for d in local for u in updated[d]])
    g("cbx_average_batchnorm_stats", L3, el, ctypes.cast(pm, ctypes.POINTER(ctypes.c_void_p)),
      ctypes.cast(pv, ctypes.POINTER(ctypes.c_void_p)), up)
    bad = []
    for d in local:
        for l, e in enumerate(elements):
            for ptr, want, what in ((ptrs[d][0][l], ref_m[d][l], "mean"), (ptrs[d][1][l], ref_v[d][l], "var")):
                got = np.empty(e, np.float32)
                assert hip.hipMemcpy(got.ctypes.data, ptr, 4 * e, 2) == 0
                if not np.all(np.isfinite(want)):
                    bad.append(f"oracle bn {what}[{l}] on device {d} is not finite")
                check = Checker(exact=exact)
                check(f"bn {what}[{l}] on device {d}", got, want)
                bad += check.bad
    return bad


def run_autotune_checkpoint(g: Ctx, world: int, local: List[int], ckdir: str, exact: bool = True) -> List[str]:
    """synchronise(autotune = +1 / -1) adds / deletes one replica per device
    after the step (executioncontext.c:2321-2328, modelmanager.c:362-557): a
    new replica copies its device's first replica and joins the next step.
    Then checkpoint (one BN operator's statistics per device included) into
    `ckdir` in the reference's file format and override from it."""
    O = oracle()
    A = g.A
    n, R, mom = 30_011, 2, 0.9
    setup_model(g, A, n, R, mom, 7, A.SYNC_BSP, 2 * world * R)
    st = O.make_state(n, world, R, 0.1, mom)
    for d in local:
        g.write("cbx_base_write", d, A.BUF_DATA, st.z[d])
        g.write("cbx_base_write", d, A.BUF_LAST, st.last[d])
    for i in range(st.size):
        if i % world in local:
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
    check = Checker(exact=exact)
    for d in local:
        check(f"autotune z[{d}]", g.read("cbx_base_read", d, A.BUF_DATA, n), st.z[d])
        check(f"autotune last[{d}]", g.read("cbx_base_read", d, A.BUF_LAST, n), st.last[d])
    for i in range(st.size):
        if i % world in local:
            check(f"autotune w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
    bad = check.bad
    if not exact:  # the files must hold the device's own values, byte for byte
        st.z = {d: g.read("cbx_base_read", d, A.BUF_DATA, n) for d in local}
        st.last = {d: g.read("cbx_base_read", d, A.BUF_LAST, n) for d in local}
        st.w = {i: g.read("cbx_replica_read", i, A.BUF_DATA, n) for i in range(st.size) if i % world in local}
    # checkpoint (executioncontext.c:2340-2364) into the shared directory
    os.makedirs(ckdir, exist_ok=True)
    hip = _hip()
    bn = {}
    pm, pv = [], []
    for d in local:
        p = ctypes.c_void_p()
        g("cbx_base_buffer", d, A.BUF_GRADIENT, ctypes.byref(p))  # scratch for BN statistics
        bn[d] = O.fill_normal(2 * 33, 300 + d, 0.5)
        assert hip.hipMemcpy(p.value, bn[d].ctypes.data, bn[d].nbytes, 1) == 0
        pm.append(p.value)
        pv.append(p.value + 4 * 33)
    am = (ctypes.c_void_p * len(local))(*pm)
    av = (ctypes.c_void_p * len(local))(*pv)
    g("cbx_register_batchnorm_stats", 7, 33, ctypes.cast(am, ctypes.POINTER(ctypes.c_void_p)),
      ctypes.cast(av, ctypes.POINTER(ctypes.c_void_p)))
    g("cbx_checkpoint_model", ckdir.encode())
    ver = os.path.join(ckdir, "000001")
    for d in local:
        files = {f"gpu-{d:02d}-theModel-data.dat": st.z[d], f"gpu-{d:02d}-theModel-last.dat": st.last[d],
                 f"gpu-{d:02d}-bn-avg-007.dat": bn[d][:33], f"gpu-{d:02d}-bn-var-007.dat": bn[d][33:]}
        files.update({f"gpu-{d:02d}-replica-{i:03d}-data.dat": st.w[i] for i in range(st.size) if i % world == d})
        for name, want in files.items():
            path = os.path.join(ver, name)
            if not os.path.exists(path):
                bad.append(f"checkpoint: {name} missing")
            elif not np.array_equal(np.fromfile(path, "<f4").view(np.uint32), want.view(np.uint32)):
                bad.append(f"checkpoint: {name} differs")
    for d in local:
        g.write("cbx_base_write", d, A.BUF_DATA, np.zeros(n, np.float32))
    g("cbx_override_model_data", ver.encode())
    for d in local:
        if not np.array_equal(g.read("cbx_base_read", d, A.BUF_DATA, n).view(np.uint32), st.z[d].view(np.uint32)):
            bad.append(f"override: z[{d}] not restored")
    return bad


def run_resync(g: Ctx, world: int, local: List[int], root: int) -> List[str]:
    """cbx_resync_base (ADVICE / VERDICT r05 item 1): base models that differ
    across the devices (as after a failed step) become the root's, bit for
    bit, on every device; then one step runs and matches the oracle from the
    resynchronised state (every device's z / last the root's)."""
    O = oracle()
    A = g.A
    n, R, mom = 30_011, 2, 0.9
    setup_model(g, A, n, R, mom, 7, A.SYNC_BSP, 2 * world * R)
    st = O.make_state(n, world, R, 0.1, mom)
    zs = [O.fill_normal(n, 700 + d, 0.05) for d in range(world)]
    ls = [O.fill_normal(n, 720 + d, 0.001) for d in range(world)]
    for d in local:
        g.write("cbx_base_write", d, A.BUF_DATA, zs[d])
        g.write("cbx_base_write", d, A.BUF_LAST, ls[d])
    mine = [i for i in range(st.size) if i % world in local]
    for i in mine:
        g.write("cbx_replica_write", i, A.BUF_DIFF, st.s[i])
        g.write("cbx_replica_write", i, A.BUF_DATA, st.w[i])
    g("cbx_resync_base", root)
    bad = []
    check = Checker(exact=True)
    for d in local:
        check(f"resync z[{d}]", g.read("cbx_base_read", d, A.BUF_DATA, n), zs[root])
        check(f"resync last[{d}]", g.read("cbx_base_read", d, A.BUF_LAST, n), ls[root])
    st.z = [zs[root].copy() for _ in range(world)]
    st.last = [ls[root].copy() for _ in range(world)]
    g("cbx_lock_any")
    g("cbx_synchronise", 0, 1, 0, 0)
    g("cbx_unlock_any")
    g("cbx_wait")
    O.sma_step(st)
    for d in local:
        check(f"step z[{d}]", g.read("cbx_base_read", d, A.BUF_DATA, n), st.z[d])
        check(f"step last[{d}]", g.read("cbx_base_read", d, A.BUF_LAST, n), st.last[d])
    for i in mine:
        check(f"step w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
    if g.L.cbx_resync_base(g.c, world) != A.CBX_ERR_INVALID:
        bad.append("a root out of range was not refused")
    return bad + check.bad


def _save_npy(d: str, name: str, arr) -> None:
    tmp = os.path.join(d, name + ".tmp")
    with open(tmp, "wb") as f:
        np.save(f, arr)
    os.replace(tmp, os.path.join(d, name + ".npy"))


def save_full_state(g: Ctx, d: str, rank: int, mine: List[int], n: int) -> None:
    """One rank's whole initial state (z, last, s and w of its replicas) as
    .npy files under `d`, then its `in_<rank>.ok` marker: the input of
    full_size_check on every rank."""
    A = g.A
    _save_npy(d, f"z_{rank}", g.read("cbx_base_read", rank, A.BUF_DATA, n))
    _save_npy(d, f"last_{rank}", g.read("cbx_base_read", rank, A.BUF_LAST, n))
    for i in mine:
        _save_npy(d, f"s_{i}", g.read("cbx_replica_read", i, A.BUF_DIFF, n))
        _save_npy(d, f"w_{i}", g.read("cbx_replica_read", i, A.BUF_DATA, n))
    with open(os.path.join(d, f"in_{rank}.ok"), "w"):
        pass


CHUNK = 1 << 20  # elements per oracle chunk


def full_size_check(d: str, world: int, R: int, steps: int, rank: int, z1, l1, w1: Dict[int, np.ndarray],
                    exact: bool, alpha: float = 0.1, mom: float = 0.9):
    """Rank `rank`'s z, last and w after `steps` SMA steps against the oracle
    in EVERY element (no sample).  The oracle runs chunk by chunk
    over every rank's memory-mapped saved inputs: the step is elementwise
    (no Phase-D copy in these runs), so a chunk's result is the whole run's.
    Returns (bad, differs, compared elements)."""
    O = oracle()
    n = z1.size
    size = world * R
    wait_files([os.path.join(d, f"in_{r}.ok") for r in range(world)], seconds=180)
    mm = lambda name: np.load(os.path.join(d, name + ".npy"), mmap_mode="r")  # noqa: E731
    zs = [mm(f"z_{r}") for r in range(world)]
    ls = [mm(f"last_{r}") for r in range(world)]
    S = [mm(f"s_{i}") for i in range(size)]
    W = [mm(f"w_{i}") for i in range(size)]
    bad = []
    if any(not np.array_equal(np.asarray(z).view(np.uint32), np.asarray(zs[0]).view(np.uint32)) for z in zs):
        bad.append("initial z differs across ranks")
    check = Checker(exact=exact)
    compared = 0
    for a in range(0, n, CHUNK):
        b = min(n, a + CHUNK)
        cut = lambda arrs: [np.array(x[a:b]) for x in arrs]  # noqa: E731
        st = O.SmaState(world, size, b - a, alpha, mom, cut(zs), cut(ls), cut(S), cut(W))
        for _ in range(steps):
            O.sma_step(st)
        check(f"z[{a}:{b}]", z1[a:b], st.z[rank])
        check(f"last[{a}:{b}]", l1[a:b], st.last[rank])
        for i, w in w1.items():
            check(f"w[{i}][{a}:{b}]", w[a:b], st.w[i])
        compared += (2 + len(w1)) * (b - a)
    return bad + check.bad[:20], check.differs, compared


def wait_files(paths, seconds=90.0):
    t0 = time.time()
    while not all(os.path.exists(p) for p in paths):
        if time.time() - t0 > seconds:
            raise TimeoutError(f"peers never wrote {[p for p in paths if not os.path.exists(p)]}")
        time.sleep(0.05)
