"""The peer-read all-reduce with ONE PROCESS PER GPU (cbx_peer_export /
cbx_peer_import), G = 2, 3, 4, 8 rank processes on ONE GPU, the real library.

Each rank maps every other rank's acc and D buffers through their IPC handles
(hipIpcOpenMemHandle, dmabuf) and pins rank 0's page of completion flags
(POSIX shared memory); the ranks' streams then order each other through the
flags (hipStreamWriteValue64 after kernel A / the reduction of a bucket,
hipStreamWaitValue64 >= this step's sequence number before reading another
rank's acc or D).  Each rank also holds a real RCCL communicator
(cbx_init_rank, sockets over loopback as in test_gpu_realrccl.py), which the
peer form never uses.

The reduction sums in rank order from +0, the oracle's order, so every case
is bit for bit against the oracle with the same G and the committed G > 1
golden fixtures, and z / last are identical on every rank.  Also: the
stream-order check with the form, a randomised run that switches between it,
the all-reduce and the reduce-scatter form between steps, C4 at the full
ResNet-50 size, and a fault-injection run that drops the flag waits
($CBX_FAULT_SKIP_PEER_WAIT, with every rank but 0 starting its kernels A 2 ms
late) and must then come out WRONG, so the waits are known to be what keeps
it right.  Every "device" is device 0: this pins the algorithm and the
cross-process ordering, not xGMI speed.
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
from tests.test_gpu_realrccl import _spawn, load_real, rank_env, run_order, run_random, share_uid

pytestmark = pytest.mark.gpu

PEER = 1


def exchange(g, rank: int, world: int, d: str, tag: str) -> None:
    """cbx_peer_export on every rank, the blobs through files, cbx_peer_import."""
    buf = ctypes.create_string_buffer(g.A.PEER_BLOB_BYTES)
    n = ctypes.c_size_t(0)
    g("cbx_peer_export", buf, ctypes.byref(n))
    assert n.value == g.A.PEER_BLOB_BYTES
    path = os.path.join(d, f"peer_{tag}_{rank}.bin")
    with open(path + ".tmp", "wb") as f:
        f.write(buf.raw)
    os.replace(path + ".tmp", path)
    paths = [os.path.join(d, f"peer_{tag}_{r}.bin") for r in range(world)]
    C.wait_files(paths)
    blobs = b"".join(open(p, "rb").read() for p in paths)
    g("cbx_peer_import", blobs, world)


def _cases(world):
    names = {2: ("sma", "sma-copy-ssp", "sma-5-buckets", "sma-5-buckets-cross", "sma-5-buckets-cross-stride",
                 "sma-no-momentum"),
             3: ("sma-5-buckets-cross", "sma-no-momentum"),  # shards not a power of two; empty trailing shards
             4: ("sma-copy-ssp", "sma-5-buckets", "sma-5-buckets-cross-stride", "sma-no-momentum"),
             8: ("sma-copy-ssp", "sma-5-buckets-cross-stride")}[world]
    return [dataclasses.replace(c, name=c.name + "-peer", algo=PEER, order="rank") for c in CASES if c.name in names]


def _jobs(world):
    jobs = [("case", c.name) for c in _cases(world)]
    jobs += [("golden", gc["name"]) for gc in C.golden_cases(world)]
    jobs += [("order", "order-peer")]
    if world <= 4:
        jobs += [("random", "random-peer-rccl-rsag")]
    return jobs


def _rank_main(rank, world, jobs, d, q):
    rank_env(rank)
    try:
        L, A = load_real()
        cases = {c.name: c for c in _cases(world)}
        goldens = {gc["name"]: gc for gc in C.golden_cases(world)}
        out = []
        for j, (kind, name) in enumerate(jobs):
            g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, f"uid_{j}")))
            hook = lambda g_, j=j: exchange(g_, rank, world, d, str(j))  # noqa: E731
            try:
                if kind == "case":
                    res = C.run_case(g, world, [rank], cases[name], after_setup=hook)
                elif kind == "golden":
                    res = {"bad": C.run_golden(g, world, [rank], goldens[name], algo=PEER, after_setup=hook)}
                elif kind == "order":
                    res = {"bad": run_order(g, world, PEER, after_setup=hook)}
                else:
                    algos = (0, 1, 1, 2) if 1024 % world == 0 else (0, 1, 1)  # the reduce-scatter form: G | 1024
                    bad, dig, differs = run_random(g, world, rank, steps=30, algos=algos, after_setup=hook)
                    res = {"bad": bad, "digest": {rank: dig}, "differs": differs}
            finally:
                g.free()
            out.append((name, res))
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_peer_read_one_process_per_gpu_vs_oracle(world):
    jobs = _jobs(world)
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _rank_main, lambda r: (r, world, jobs, d), timeout=280)
    for rank in range(world):
        assert [name for name, _ in res[rank]] == [name for _, name in jobs]
        failures = [(name, r["bad"]) for name, r in res[rank] if r["bad"]]
        assert not failures, f"rank {rank}: {failures}"
    for j, (kind, name) in enumerate(jobs):
        if kind not in ("case", "random"):
            continue
        digests = {res[r][j][1]["digest"][r] for r in range(world)}
        assert len(digests) == 1, f"{name}: z / last differ across ranks"
        if kind == "case":  # rank-order sums: the oracle's, bit for bit
            assert all(res[r][j][1]["differs"] == 0 for r in range(world)), name


def _fault_main(rank, world, fault, d, q):
    rank_env(rank)
    if fault:
        os.environ["CBX_FAULT_SKIP_PEER_WAIT"] = "1"  # read at context creation
    try:
        L, A = load_real()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        try:
            case = dataclasses.replace(next(c for c in CASES if c.name == "sma-5-buckets"), algo=PEER)
            res = C.run_case(g, world, [rank], case, after_setup=lambda g_: exchange(g_, rank, world, d, "f"))
        finally:
            g.free()
        q.put((rank, res, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(200)
@pytest.mark.parametrize("fault", [True, False])
def test_peer_read_flag_waits_are_what_orders_the_ranks(fault):
    # With the waits dropped and rank 1's kernels A started 2 ms late, rank 0
    # reduces rank 1's acc before it is written: the result must be wrong.
    # The same run with the waits is bit for bit against the oracle.
    world = 2
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _fault_main, lambda r: (r, world, fault, d), timeout=180)
    if fault:
        assert any(res[r]["bad"] for r in range(world)), "the race went unseen: the fault switch did nothing"
    else:
        assert not any(res[r]["bad"] for r in range(world)), [res[r]["bad"] for r in range(world)]
        assert len({res[r]["digest"][r] for r in range(world)}) == 1


def _full_size_main(rank, world, R, steps, d, q):
    rank_env(rank)
    try:
        L, A = load_real()
        O = C.oracle()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        try:
            n = N_RESNET50
            C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_BSP, 2 * world * R)
            exchange(g, rank, world, d, "full")
            g("cbx_set_pipeline_mode", 1)
            g("cbx_set_allreduce_algorithm", PEER)
            g("cbx_fill_synthetic", O.SEED)
            size = world * R
            mine = [i for i in range(size) if i % world == rank]
            rng = np.random.default_rng(12)
            idx = np.unique(np.concatenate([rng.integers(0, n, 60_000), np.arange(4), np.arange(n - 4, n),
                                            np.arange(6_389_000, 6_391_000)]))  # across the 4 ranks' shards
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
        check = C.Checker(exact=True)
        check("z sample", z1[idx], st.z[rank])
        check("last sample", l1[idx], st.last[rank])
        for i in mine:
            check(f"w[{i}] sample", w1[i], st.w[i])
        q.put((rank, {"bad": check.bad, "digest": dig}, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(300)
def test_peer_read_one_process_per_gpu_resnet50_c4():
    # C4 (2 replicas/GPU x 4) at the full ResNet-50 size, cross-step pipeline,
    # 8 buckets (the library default at G > 1): sampled bit for bit, z and
    # last identical on every rank.
    world, R = 4, 2
    with tempfile.TemporaryDirectory(dir=C.loopback_dir(1 << 30)) as d:
        res = _spawn(world, _full_size_main, lambda r: (r, world, R, 3, d), timeout=280)
    for r in range(world):
        assert not res[r]["bad"], f"rank {r}: {res[r]['bad']}"
    assert len({res[r]["digest"] for r in range(world)}) == 1, "z / last differ across ranks at full size"


# The page of completion flags (context_internal.h): per rank kIpcRankWords
# words, a[] then r[] (kIpcMaxBuckets each), then done / opened / broken.
IPC_MAX_BUCKETS, IPC_RANK_WORDS, IPC_RELEASE = 4096, 2 * 4096 + 64, 1 << 62
BLOB_SHM_OFFSET = 4 + 4 + 4 + 4 + 8 + 8 + 64 + 64  # PeerBlob.shm (sync_steps.hip)


def _flag_words(d: str, rank: int, nb: int):
    """Rank `rank`'s A and R words of buckets 0..nb-1 and its broken word,
    read from the shared page (its name is in rank 0's exported blob)."""
    blob = open(os.path.join(d, "peer_fail_0.bin"), "rb").read()
    name = blob[BLOB_SHM_OFFSET:BLOB_SHM_OFFSET + 64].split(b"\0")[0].decode()
    page = np.fromfile(os.path.join("/dev/shm", name.lstrip("/")), dtype=np.uint64)
    base = rank * IPC_RANK_WORDS
    return (page[base:base + nb].copy(), page[base + IPC_MAX_BUCKETS:base + IPC_MAX_BUCKETS + nb].copy(),
            int(page[base + 2 * IPC_MAX_BUCKETS + 2]))


def _failing_main(rank, world, d, q):
    """Rank 1's third peer-read step fails right after it queued its first
    flag write ($CBX_FAULT_PEER_FAIL="1:3")."""
    import time
    rank_env(rank)
    os.environ["CBX_FAULT_PEER_FAIL"] = "1:3"  # read at context creation

    def mark(what):  # each rank's progress, for the report if a rank never arrives
        with open(os.path.join(d, f"progress_{rank}"), "a") as f:
            f.write(f"{time.monotonic():.3f} {what}\n")

    try:
        L, A = load_real()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        out = {"errors": {}}
        try:
            n, nb = 1 << 22, 5
            C.setup_model(g, A, n, 2, 0.9, 7, A.SYNC_BSP, 2 * world * 2)
            exchange(g, rank, world, d, "fail")
            g("cbx_set_allreduce_algorithm", PEER)
            g("cbx_set_bucket_elements", -(-n // nb))
            g("cbx_fill_synthetic", 5)

            def step(clock):
                g("cbx_lock_any")
                try:
                    g("cbx_synchronise", 0, clock, 0, 0)
                finally:
                    g("cbx_unlock_any")

            for clock in (1, 2, 3):
                if clock == 3:  # every rank has enqueued steps 1 and 2 before any enqueues step 3
                    with open(os.path.join(d, f"before3_{rank}"), "w"):
                        pass
                    C.wait_files([os.path.join(d, f"before3_{r}") for r in range(world)])
                try:
                    step(clock)
                    mark(f"step {clock} enqueued")
                except RuntimeError as e:
                    out["errors"][clock] = str(e)
                    mark(f"step {clock} refused: {e}")
            t0 = time.monotonic()
            g("cbx_wait")  # every rank's streams drain: no wait is left on a flag that never comes
            out["drain_s"] = time.monotonic() - t0
            mark("drained")
            if rank == 1:
                a, r, broken = _flag_words(d, 1, nb)
                out["words"] = {"a_min": int(a.min()), "r_min": int(r.min()), "broken": broken}
            with open(os.path.join(d, f"after3_{rank}"), "w"):
                pass
            try:
                C.wait_files([os.path.join(d, f"after3_{r}") for r in range(world)])
            except TimeoutError as e:
                report = {r: open(os.path.join(d, f"progress_{r}")).read() if os.path.exists(
                    os.path.join(d, f"progress_{r}")) else "(nothing)" for r in range(world)}
                raise TimeoutError(f"{e}; progress: {report}") from None
            try:  # the form is unusable on EVERY rank now, not only on the one that failed
                step(4)
                out["step4"] = None
            except RuntimeError as e:
                out["step4"] = str(e)
            g("cbx_set_allreduce_algorithm", 0)  # the RCCL form still runs
            step(5)
            g("cbx_wait")
        finally:
            t0 = time.monotonic()
            g.free()
            out["free_s"] = time.monotonic() - t0
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(200)
def test_peer_read_failed_step_releases_and_stops_every_rank():
    # a rank whose peer-read step fails after queuing flag writes
    # must leave its words at the release value (the queued writes of the
    # step's sequence number land BEFORE the queued release), and every other
    # rank must refuse its next step in the form instead of reading stale
    # acc / D silently; nobody hangs, the RCCL form still runs, free is bounded.
    world = 3
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _failing_main, lambda r: (r, world, d), timeout=180)
    assert "fault injection" in res[1]["errors"].get(3, "") and set(res[1]["errors"]) == {3}, res[1]["errors"]
    for r in (0, 2):
        # step 3 races rank 1's failure: a rank enqueues it (and its waits on
        # rank 1 are released) or already refuses it; steps 1 and 2 run
        errs = res[r]["errors"]
        assert set(errs) <= {3} and all("failed part-way earlier" in m for m in errs.values()), (r, errs)
    w = res[1]["words"]
    assert w["a_min"] >= IPC_RELEASE and w["r_min"] >= IPC_RELEASE and w["broken"] == 1, w
    for r in range(world):
        assert res[r]["step4"] and "failed part-way earlier" in res[r]["step4"], (r, res[r]["step4"])
        assert res[r]["drain_s"] < 30 and res[r]["free_s"] < 70, (r, res[r]["drain_s"], res[r]["free_s"])
