"""The product library with the REAL librccl, G = 2, 4, 8 ranks on ONE GPU.

RCCL refuses two ranks of one host on one device ("Duplicate GPU detected").
Each rank process here gets its own NCCL_HOSTID, so RCCL takes every rank for
a host of its own and connects them through its network transport (sockets
over the loopback interface) instead of xGMI.  What this runs for real, which
the loopback tests (test_gpu_multirank.py) only stand in for:

* crossbow_amd/libcrossbow_sma.so itself, as built, in G processes
  (cbx_init_rank: the one-process-per-GPU form bench.py uses);
* RCCL's own ncclAllReduce with nranks > 1: its kernels run asynchronously
  on the comm stream beside kernels A and B, with its proxy threads, and sum
  in its own order, not rank order;
* the stream-order check (cbx_check_order) of the bucketed pipeline while
  RCCL's kernels run beside kernels A and B;
* so the G > 1 tolerance (rtol 1e-5 / atol 1e-6) is checked
  against the oracle wherever RCCL's order differs from it (G >= 3), z and
  last must come out bitwise identical on every rank (sma.c:168-174), and at
  G = 2 (a + b is order-free) everything is bit for bit.

Not measured here: xGMI.  The bytes cross sockets on one host, so nothing in
these runs says anything about link bandwidth; they are a correctness run.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import tempfile

import numpy as np
import pytest

from tests import multidev_common as C
from tests.test_gpu_multirank import CASES, N_RESNET50

pytestmark = pytest.mark.gpu

REAL = os.path.join(C.ROOT, "crossbow_amd", "libcrossbow_sma.so")


def rank_env(rank: int) -> None:
    """Every rank a host of its own: RCCL's network transport over loopback."""
    os.environ["NCCL_HOSTID"] = f"cbx-test-rank-{rank}"
    os.environ["NCCL_SOCKET_IFNAME"] = "lo"
    os.environ["NCCL_IB_DISABLE"] = "1"
    os.environ["NCCL_NET"] = "Socket"
    os.environ.setdefault("NCCL_DEBUG", "ERROR")


def load_real():
    A = C.abi()
    return A.bind(ctypes.CDLL(REAL)), A


def share_uid(L, rank: int, path: str) -> bytes:
    """Rank 0's ncclGetUniqueId, handed to the others through a file."""
    if rank == 0:
        ub = (ctypes.c_ubyte * 128)()
        assert L.cbx_get_unique_id(ub) == 0
        with open(path + ".tmp", "wb") as f:
            f.write(bytes(ub))
        os.replace(path + ".tmp", path)
    C.wait_files([path])
    with open(path, "rb") as f:
        return f.read()


def _jobs(world):
    names = {2: ["sma", "sma-copy-ssp", "sma-5-buckets", "sma-5-buckets-cross", "sma-no-momentum", "sma-staged",
                 "sma-staged-dma", "ssgd", "ssgd-buckets", "sma-rsag", "sma-rsag-buckets-cross",
                 "sma-rsag-no-momentum"],
             4: ["sma", "sma-copy-ssp", "sma-5-buckets", "sma-5-buckets-cross-stride", "sma-staged", "ssgd-buckets",
                 "sma-rsag", "sma-rsag-buckets-cross"],
             8: ["sma-copy-ssp", "sma-5-buckets-cross-stride", "ssgd-buckets", "sma-rsag-buckets-cross"]}[world]
    jobs = [("case", n) for n in names]
    jobs += [("golden", gc["name"]) for gc in C.golden_cases(world)]
    jobs += [("golden-rsag", gc["name"]) for gc in C.golden_cases(world)]
    jobs += [("order", "order-all-reduce"), ("order", "order-rsag")]
    if world == 4:
        jobs += [("random", "random-long-run")]
    return jobs + [("bn", "bn"), ("autotune", "autotune")]


def run_random(g, world, rank, steps=40, algos=(0, 2), after_setup=None):
    """A long randomised run under real RCCL: every few steps the bucket size,
    pipeline mode, wait stride, all-reduce group or the collective's form
    changes (the same choice on every rank, from a shared seed), replicas
    ask for Phase D, are held by a task (SSP) or are rewritten by the host,
    and the stream order is checked every two steps.  Against the oracle
    within the G > 1 tolerance at the end; returns (bad, digest, differs)."""
    import random
    O = C.oracle()
    A = g.A
    n, R = 200_003, 2
    C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_SSP, 4 * world)
    if after_setup:
        after_setup(g)
    g("cbx_set_order_check", 1)
    size = world * R
    mine = [i for i in range(size) if i % world == rank]
    st = O.make_state(n, world, R, 0.1, 0.9)
    g.write("cbx_base_write", rank, A.BUF_DATA, st.z[rank])
    g.write("cbx_base_write", rank, A.BUF_LAST, st.last[rank])
    for i in mine:
        g.write("cbx_replica_write", i, A.BUF_DIFF, st.s[i])
        g.write("cbx_replica_write", i, A.BUF_DATA, st.w[i])
    rng = random.Random(9001)  # the same sequence on every rank: collective choices must match
    bad = []
    for step in range(steps):
        st.locked[:] = 1
        u = rng.random()
        hold = None
        if u < 0.1:
            i = rng.randrange(size)
            st.copy[i] = 1
            if i in mine:
                g("cbx_replica_set_copy", i, 1)
        elif u < 0.2:
            hold = rng.randrange(size)
            st.locked[hold] = 0
            if hold in mine:
                g("cbx_replica_lock", hold)
        elif u < 0.3:
            g("cbx_set_bucket_elements", ctypes.c_longlong(rng.choice([16_384, 65_536, 1 << 40])))
        elif u < 0.4:
            g("cbx_set_pipeline_mode", rng.choice([0, 1]))
            g("cbx_set_cross_wait_stride", rng.choice([1, 2, 3]))
            g("cbx_set_allreduce_group", rng.choice([1, 2, 4]))
        elif u < 0.5:
            g("cbx_set_allreduce_algorithm", rng.choice(list(algos)))
        elif u < 0.55:
            i = rng.randrange(size)
            new = O.fill_normal(n, 7000 + step, 0.05)
            st.w[i] = new.copy()
            if i in mine:
                g.write("cbx_replica_write", i, A.BUF_DATA, new)
        g("cbx_lock_any")
        g("cbx_synchronise", 0, step + 1, 0, 0)
        g("cbx_unlock_any")
        if hold is not None and hold in mine:
            g("cbx_replica_unlock", hold)
        O.sma_step(st)
        if step % 2 == 1:
            g("cbx_check_order")  # raises on a violation
    g("cbx_wait")
    check = C.Checker(exact=world < 3)
    z = g.read("cbx_base_read", rank, A.BUF_DATA, n)
    last = g.read("cbx_base_read", rank, A.BUF_LAST, n)
    check(f"z[{rank}]", z, st.z[rank])
    check(f"last[{rank}]", last, st.last[rank])
    for i in mine:
        check(f"w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
    return bad + check.bad, C.digest(z, last), check.differs


def run_order(g, world, algo, after_setup=None):
    """The stream-order check (cbx_set_order_check) under real RCCL, whose
    collective runs asynchronously beside kernels A and B: bucketed, cross-step
    pipeline with wait stride 2 and all-reduce groups of 2, checked after every
    two back-to-back steps."""
    A = g.A
    C.setup_model(g, A, 300_007, 2, 0.9, 7, A.SYNC_BSP, 4 * world)
    if after_setup:
        after_setup(g)
    g("cbx_set_bucket_elements", ctypes.c_longlong(65_536))
    g("cbx_set_pipeline_mode", 1)
    g("cbx_set_cross_wait_stride", 2)
    g("cbx_set_allreduce_group", 2)
    g("cbx_set_allreduce_algorithm", algo)
    g("cbx_fill_synthetic", 5)
    g("cbx_set_order_check", 1)
    bad = []
    progress = os.environ.get("CBX_TEST_PROGRESS_DIR")
    for step in range(6):
        if progress:
            with open(os.path.join(progress, f"order_w{world}_pid{os.getpid()}.log"), "a") as f:
                f.write(f"algo {algo} step {step}\n")
        g("cbx_lock_any")
        g("cbx_synchronise", 0, step + 1, 0, 0)
        g("cbx_unlock_any")
        if step % 2 == 1:
            n = g("cbx_check_order")
            if n != 2:
                bad.append(f"order check after step {step} covered {n} steps, not 2")
    g("cbx_wait")
    return bad


def _rank_main(rank, world, jobs, d, q):
    rank_env(rank)
    try:
        L, A = load_real()
        exact = world < 3  # RCCL's order is rank order only up to commutativity
        cases = {c.name: c for c in CASES}
        goldens = {gc["name"]: gc for gc in C.golden_cases(world)}
        out = []
        progress = os.environ.get("CBX_TEST_PROGRESS_DIR")  # a diagnosis aid: one line per job start / end
        if progress:  # and every rank's Python stacks after 100 s (where a hang sits on the host)
            import faulthandler
            tb = open(os.path.join(progress, f"realrccl_w{world}_r{rank}.stacks"), "w")
            faulthandler.dump_traceback_later(100, repeat=False, file=tb)
        for j, (kind, name) in enumerate(jobs):
            if progress:
                with open(os.path.join(progress, f"realrccl_w{world}_r{rank}.log"), "a") as f:
                    f.write(f"start {j} {kind} {name}\n")
            g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, f"uid_{j}")))
            try:
                if kind == "case":
                    # "ring": the checker's tolerance mode (the loopback order is not used here)
                    res = C.run_case(g, world, [rank], dataclasses.replace(cases[name], order="rank" if exact else "ring"))
                elif kind.startswith("golden"):
                    res = {"bad": C.run_golden(g, world, [rank], goldens[name], exact=exact,
                                               algo=2 if kind == "golden-rsag" else 0)}
                elif kind == "order":
                    res = {"bad": run_order(g, world, 2 if name == "order-rsag" else 0)}
                elif kind == "random":
                    bad, dig, differs = run_random(g, world, rank)
                    res = {"bad": bad, "digest": {rank: dig}, "differs": differs}
                elif kind == "bn":
                    res = {"bad": C.run_bn(g, world, [rank], poison=True, exact=exact)}
                else:
                    res = {"bad": C.run_autotune_checkpoint(g, world, [rank], os.path.join(d, "ckpt"), exact=exact)}
            finally:
                g.free()
            out.append((name, res))
            if progress:
                with open(os.path.join(progress, f"realrccl_w{world}_r{rank}.log"), "a") as f:
                    f.write(f"end {j} {kind} {name} bad={bool(res['bad'])}\n")
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _rank_main_hw_queues(rank, world, jobs, d, hw_queues, q):
    # a fresh process: ROCclr reads GPU_MAX_HW_QUEUES once, at HIP's start
    os.environ["GPU_MAX_HW_QUEUES"] = hw_queues
    _rank_main(rank, world, jobs, d, q)


def _spawn(world, target, args_of_rank, timeout):
    from tests.test_gpu_multirank import _spawn as spawn
    return spawn(world, target, args_of_rank, timeout)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_real_rccl_ranks_on_one_gpu_vs_oracle(world):
    jobs = _jobs(world)
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _rank_main, lambda r: (r, world, jobs, d), timeout=280)
    for rank in range(world):
        assert [name for name, _ in res[rank]] == [name for _, name in jobs]
        failures = [(name, r["bad"]) for name, r in res[rank] if r["bad"]]
        assert not failures, f"rank {rank}: {failures}"
    differs = 0
    for j, (kind, name) in enumerate(jobs):
        if kind not in ("case", "random"):
            continue
        # every rank applied the same D: z and last bitwise identical across ranks (sma.c:168-174)
        digests = {res[r][j][1]["digest"][r] for r in range(world)}
        assert len(digests) == 1, f"{name}: z / last differ across ranks"
        differs += sum(res[r][j][1]["differs"] for r in range(world))
    if world >= 3:
        # the tolerance path was really taken: RCCL summed outside the oracle's order
        assert differs > 0, "RCCL's sums never left the oracle's order"


@pytest.mark.timeout(300)
def test_real_rccl_random_run_live_at_hip_default_hw_queues():
    # The 4-rank randomised run (bucket sizes, pipeline modes, wait strides,
    # all-reduce groups and collective forms switched between steps, Phase D,
    # SSP holds, host writes, the stream order checked every two steps) with
    # GPU_MAX_HW_QUEUES=4, HIP's default: the library's four streams per
    # device then share hardware queues with RCCL's and each other, so a
    # stream wait can hold back work queued behind it.  Slower, but it must
    # stay live and correct.
    world, jobs = 4, [("random", "random-long-run")]
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _rank_main_hw_queues, lambda r: (r, world, jobs, d, "4"), timeout=280)
    for rank in range(world):
        (name, r), = res[rank]
        assert name == "random-long-run" and not r["bad"], f"rank {rank}: {r['bad']}"
    assert len({res[r][0][1]["digest"][r] for r in range(world)}) == 1, "z / last differ across ranks"
    assert sum(res[r][0][1]["differs"] for r in range(world)) > 0, "RCCL's sums never left the oracle's order"


def _full_size_main(rank, world, R, steps, mode, algo, d, q):
    rank_env(rank)
    try:
        L, A = load_real()
        O = C.oracle()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        try:
            n = N_RESNET50
            C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_BSP, 2 * world * R)
            g("cbx_set_pipeline_mode", mode)
            g("cbx_set_allreduce_algorithm", algo)
            g("cbx_fill_synthetic", O.SEED)
            size = world * R
            mine = [i for i in range(size) if i % world == rank]
            rng = np.random.default_rng(11)
            idx = np.unique(np.concatenate([rng.integers(0, n, 60_000), np.arange(4), np.arange(n - 4, n),
                                            np.arange(3_194_000, 3_196_000)]))
            z0 = g.read("cbx_base_read", rank, A.BUF_DATA, n)[idx]
            l0 = g.read("cbx_base_read", rank, A.BUF_LAST, n)[idx]
            s0 = np.stack([g.read("cbx_replica_read", i, A.BUF_DIFF, n)[idx] for i in mine])
            w0 = np.stack([g.read("cbx_replica_read", i, A.BUF_DATA, n)[idx] for i in mine])
            tmp = os.path.join(d, f"in_{rank}.tmp.npz")
            np.savez(tmp, z=z0, last=l0, s=s0, w=w0, ids=np.array(mine))
            os.replace(tmp, os.path.join(d, f"in_{rank}.npz"))
            for step in range(steps):
                g("cbx_lock_any")
                g("cbx_synchronise", 0, step + 1, 0, 0)
                g("cbx_unlock_any")
            g("cbx_wait")
            z1 = g.read("cbx_base_read", rank, A.BUF_DATA, n)
            l1 = g.read("cbx_base_read", rank, A.BUF_LAST, n)
            dig = C.digest(z1, l1)
            w1 = {i: g.read("cbx_replica_read", i, A.BUF_DATA, n)[idx] for i in mine}
        finally:
            g.free()
        C.wait_files([os.path.join(d, f"in_{r}.npz") for r in range(world)])
        ins = [np.load(os.path.join(d, f"in_{r}.npz")) for r in range(world)]
        s, w = [None] * size, [None] * size
        for f in ins:
            for k, i in enumerate(f["ids"]):
                s[int(i)], w[int(i)] = f["s"][k].copy(), f["w"][k].copy()
        st = O.SmaState(world, size, idx.size, 0.1, 0.9, [f["z"].copy() for f in ins],
                        [f["last"].copy() for f in ins], s, w)
        for _ in range(steps):
            O.sma_step(st)
        check = C.Checker(exact=False)
        check("z sample", z1[idx], st.z[rank])
        check("last sample", l1[idx], st.last[rank])
        for i in mine:
            check(f"w[{i}] sample", w1[i], st.w[i])
        q.put((rank, {"bad": check.bad, "digest": dig, "differs": check.differs}, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,R,mode,algo", [(4, 2, 0, 0),   # C4: 2 replicas/GPU x 4
                                               (8, 4, 1, 0),   # C5: 4 replicas/GPU x 8, cross-step pipeline
                                               (8, 4, 1, 2)])  # C5 through reduce-scatter / all-gather
def test_real_rccl_resnet50_full_size(world, R, mode, algo):
    with tempfile.TemporaryDirectory(dir=C.loopback_dir(1 << 30)) as d:
        res = _spawn(world, _full_size_main, lambda r: (r, world, R, 3, mode, algo, d), timeout=280)
    for r in range(world):
        assert not res[r]["bad"], f"rank {r}: {res[r]['bad']}"
    assert len({res[r]["digest"] for r in range(world)}) == 1, "z / last differ across ranks at full size"
    assert sum(res[r]["differs"] for r in range(world)) > 0, "RCCL's sums never left the oracle's order"
