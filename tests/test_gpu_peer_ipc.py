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
            C.save_full_state(g, d, rank, mine, n)
            for step in range(steps):
                g("cbx_lock_any")
                g("cbx_synchronise", 0, step + 1, 0, 0)
                g("cbx_unlock_any")
            g("cbx_wait")
            z1 = g.read("cbx_base_read", rank, A.BUF_DATA, n)
            l1 = g.read("cbx_base_read", rank, A.BUF_LAST, n)
            dig = C.digest(z1, l1)
            w1 = {i: g.read("cbx_replica_read", i, A.BUF_DATA, n) for i in mine}
        finally:
            g.free()
        bad, _, compared = C.full_size_check(d, world, R, steps, rank, z1, l1, w1, exact=True)
        q.put((rank, {"bad": bad, "digest": dig, "compared": compared}, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(330)
def test_peer_read_one_process_per_gpu_resnet50_c4():
    # C4 (2 replicas/GPU x 4) at the full ResNet-50 size, cross-step pipeline,
    # 8 buckets (the library default at G > 1): every element bit for bit, z
    # and last identical on every rank.
    world, R = 4, 2
    need = (2 * world + 2 * world * R) * N_RESNET50 * 4 + (1 << 30)
    with tempfile.TemporaryDirectory(dir=C.loopback_dir(need)) as d:
        res = _spawn(world, _full_size_main, lambda r: (r, world, R, 3, d), timeout=300)
    for r in range(world):
        assert not res[r]["bad"], f"rank {r}: {res[r]['bad']}"
        assert res[r]["compared"] == (2 + R) * N_RESNET50, res[r]["compared"]
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


def _save(d: str, name: str, **arrs) -> None:
    tmp = os.path.join(d, name + ".tmp.npz")
    np.savez(tmp, **arrs)
    os.replace(tmp, os.path.join(d, name + ".npz"))


def _load_all(d: str, name: str, world: int):
    C.wait_files([os.path.join(d, f"{name}_{r}.npz") for r in range(world)], seconds=120)
    return [np.load(os.path.join(d, f"{name}_{r}.npz")) for r in range(world)]


def _oracle_state(O, world, size, n, ins, z_from=None):
    """The job's state from every rank's saved buffers: z / last per rank (or
    rank `z_from`'s on every rank), s and w per replica."""
    s, w = [None] * size, [None] * size
    for f in ins:
        for k, i in enumerate(f["ids"]):
            s[int(i)], w[int(i)] = f["s"][k].copy(), f["w"][k].copy()
    zs = [ins[r if z_from is None else z_from]["z"].copy() for r in range(world)]
    ls = [ins[r if z_from is None else z_from]["last"].copy() for r in range(world)]
    return O.SmaState(world, size, n, 0.1, 0.9, zs, ls, s, w)


def _failing_main(rank, world, mode, fail_seq, bucket, d, q):
    """Rank 1's peer-read step `fail_seq` fails right after it queued kernel
    A of `bucket` ($CBX_FAULT_PEER_FAIL="1:seq:bucket").  Every rank then
    reports what its steps did, is refused in every form, resynchronises, and
    steps again."""
    import time
    rank_env(rank)
    os.environ["CBX_FAULT_PEER_FAIL"] = f"1:{fail_seq}:{bucket}"  # read at context creation

    def mark(what):  # each rank's progress, for the report if a rank never arrives
        with open(os.path.join(d, f"progress_{rank}"), "a") as f:
            f.write(f"{time.monotonic():.3f} {what}\n")

    def meet(tag):
        with open(os.path.join(d, f"{tag}_{rank}"), "w"):
            pass
        try:
            C.wait_files([os.path.join(d, f"{tag}_{r}") for r in range(world)])
        except TimeoutError as e:
            report = {r: open(os.path.join(d, f"progress_{r}")).read() if os.path.exists(
                os.path.join(d, f"progress_{r}")) else "(nothing)" for r in range(world)}
            raise TimeoutError(f"{e}; progress: {report}") from None

    try:
        L, A = load_real()
        O = C.oracle()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        out = {"errors": {}, "bad": []}
        try:
            n, nb, R = 1 << 22, 5, 2
            size = world * R
            mine = [i for i in range(size) if i % world == rank]
            C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_BSP, 2 * world * R)
            exchange(g, rank, world, d, "fail")
            g("cbx_set_allreduce_algorithm", PEER)
            g("cbx_set_bucket_elements", -(-n // nb))
            g("cbx_set_pipeline_mode", mode)  # 1: kernels A of a step overlap the last one's kernels B
            g("cbx_fill_synthetic", 5)

            def state(tag):  # this rank's whole state, for every rank's oracle
                _save(d, f"{tag}_{rank}", z=g.read("cbx_base_read", rank, A.BUF_DATA, n),
                      last=g.read("cbx_base_read", rank, A.BUF_LAST, n),
                      s=np.stack([g.read("cbx_replica_read", i, A.BUF_DIFF, n) for i in mine]),
                      w=np.stack([g.read("cbx_replica_read", i, A.BUF_DATA, n) for i in mine]), ids=np.array(mine))

            state("in")

            def step(clock):
                g("cbx_lock_any")
                try:
                    g("cbx_synchronise", 0, clock, 0, 0)
                finally:
                    g("cbx_unlock_any")

            ok_steps = 0
            for clock in (1, 2, 3):
                if clock == fail_seq:  # every rank has enqueued the steps before it before any enqueues it
                    meet("before_fail")
                try:
                    step(clock)
                    ok_steps += 1
                    mark(f"step {clock} enqueued")
                except RuntimeError as e:
                    out["errors"][clock] = str(e)
                    mark(f"step {clock} refused: {e}")
            t0 = time.monotonic()
            try:
                g("cbx_wait")  # every rank's streams drain: no wait is left on a flag that never comes
                out["wait"] = None
            except RuntimeError as e:  # a kernel B of this rank ran after a broken word was set
                out["wait"] = str(e)
            out["drain_s"] = time.monotonic() - t0
            out["ok_steps"] = ok_steps
            if out["wait"] is not None:  # an undefined model is not checkpointed
                os.makedirs(os.path.join(d, f"ck_{rank}"), exist_ok=True)
                out["ckpt_rc"] = L.cbx_checkpoint_model(g.c, os.path.join(d, f"ck_{rank}").encode())
            mark(f"drained: {out['wait']}")
            # A step that failed part-way (the injected fault) reported itself
            # when called and left this rank's z / last undefined: its
            # kernels B of the buckets before the fault may have run.
            partial = out["partial"] = any("fault injection" in m for m in out["errors"].values())
            if out["wait"] is None and not partial:
                # Nothing reported: every step this rank enqueued must be the
                # oracle's, bit for bit (rank-order sums), every element.
                ins = _load_all(d, "in", world)
                st = _oracle_state(O, world, size, n, ins)
                for _ in range(ok_steps):
                    O.sma_step(st)
                check = C.Checker(exact=True)
                check(f"z after {ok_steps} steps", g.read("cbx_base_read", rank, A.BUF_DATA, n), st.z[rank])
                check(f"last after {ok_steps} steps", g.read("cbx_base_read", rank, A.BUF_LAST, n), st.last[rank])
                for i in mine:
                    check(f"w[{i}] after {ok_steps} steps", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
                out["bad"] += check.bad
            if rank == 1:
                a, r, broken = _flag_words(d, 1, nb)
                out["words"] = {"a_min": int(a.min()), "r_min": int(r.min()), "broken": broken}
            meet("after3")
            refused = {}
            for clock, algo in ((4, PEER), (5, 0)):  # the failure stops EVERY form on EVERY rank
                g("cbx_set_allreduce_algorithm", algo)
                try:
                    step(clock)
                    refused[clock] = None
                except RuntimeError as e:
                    refused[clock] = str(e)
            out["refused"] = refused
            meet("before_resync")
            g("cbx_resync_base", 0)
            mark("resynced")
            z = g.read("cbx_base_read", rank, A.BUF_DATA, n)
            last = g.read("cbx_base_read", rank, A.BUF_LAST, n)
            out["resync_digest"] = C.digest(z, last)
            step(5)  # the RCCL form runs again
            g("cbx_wait")
            out["rccl_digest"] = C.digest(g.read("cbx_base_read", rank, A.BUF_DATA, n),
                                          g.read("cbx_base_read", rank, A.BUF_LAST, n))
            state("mid")
            g("cbx_set_allreduce_algorithm", PEER)  # and so does the peer-read form, from sequence 1
            step(6)
            g("cbx_wait")
            mids = _load_all(d, "mid", world)
            st = _oracle_state(O, world, size, n, mids)
            O.sma_step(st)
            check = C.Checker(exact=True)
            check("z after the peer step", g.read("cbx_base_read", rank, A.BUF_DATA, n), st.z[rank])
            check("last after the peer step", g.read("cbx_base_read", rank, A.BUF_LAST, n), st.last[rank])
            for i in mine:
                check(f"w[{i}] after the peer step", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
            out["bad"] += check.bad
            out["compared"] = n
        finally:
            t0 = time.monotonic()
            g.free()
            out["free_s"] = time.monotonic() - t0
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(280)
@pytest.mark.parametrize("mode,fail_seq,bucket", [(0, 3, 0), (1, 3, 0), (0, 2, 3), (1, 1, 4)])
def test_peer_read_failed_step_releases_and_stops_every_rank(mode, fail_seq, bucket):
    # ADVICE r04 / r05, VERDICT r05: a rank whose peer-read step fails after
    # queuing flag writes leaves its words at the release value (the queued
    # writes of the step's sequence number land BEFORE the queued release).
    # Every step on every rank either equals the oracle (every element) or is
    # reported: refused when called, or named by cbx_wait because its kernel B
    # found a broken word.  Then every form is refused on every rank until
    # cbx_resync_base, after which z / last are identical on every rank and
    # both the RCCL and the peer-read forms run (the latter bit for bit).
    world = 3
    with tempfile.TemporaryDirectory(dir=C.loopback_dir(1 << 30)) as d:
        res = _spawn(world, _failing_main, lambda r: (r, world, mode, fail_seq, bucket, d), timeout=260)
    for r in range(world):  # what each rank saw (pytest -s)
        ok = "OK (its own step failed part-way: state undefined, not compared)" if res[r]["partial"] else \
            "OK (oracle-exact, every element)"
        print(f"rank {r}: failed or refused at call {sorted(res[r]['errors'])}, enqueued {res[r]['ok_steps']}, "
              f"cbx_wait: {(res[r]['wait'] or ok)[:90]}")
    later = set(range(fail_seq, 4))  # the failed step and every step after it
    assert "fault injection" in res[1]["errors"].get(fail_seq, "") and set(res[1]["errors"]) == later, \
        res[1]["errors"]
    for r in range(world):
        errs, wait = res[r]["errors"], res[r]["wait"]
        assert set(errs) <= later and all("failed part-way earlier" in m or "fault injection" in m
                                          for m in errs.values()), (r, errs)
        # rank 1 never reduced its shard of the failed step: a rank that
        # enqueued that step (or a later one) cannot have a correct one, so
        # cbx_wait must report it
        if r != 1 and later - set(errs):
            assert wait and "ran after a rank's step failed" in wait, (r, wait)
        if wait:
            assert res[r]["ckpt_rc"] == -2, (r, res[r]["ckpt_rc"])  # CBX_ERR_STATE
        assert not res[r]["bad"], (r, res[r]["bad"])
        assert res[r]["drain_s"] < 30 and res[r]["free_s"] < 70, (r, res[r]["drain_s"], res[r]["free_s"])
        for clock in (4, 5):
            m = res[r]["refused"][clock]
            assert m and "failed part-way earlier" in m and "cbx_resync_base" in m, (r, clock, m)
        assert res[r]["compared"] == 1 << 22
    w = res[1]["words"]
    assert w["a_min"] >= IPC_RELEASE and w["r_min"] >= IPC_RELEASE and w["broken"] == 1, w
    assert len({res[r]["resync_digest"] for r in range(world)}) == 1, "z / last differ across ranks after the resync"
    assert len({res[r]["rccl_digest"] for r in range(world)}) == 1, "z / last differ across ranks after the RCCL step"


# The per-rank form's export limit (kIpcMaxSlotBytes, context_internal.h):
# ROCm 7.0's IPC keeps an allocation's size in 32 bits, so every exported
# buffer stays below 2 GiB once hipMalloc has rounded it to 2 MiB.  A slot is
# round_up(16 n4 + 256, 2 MiB) + 4 KiB bytes, so the reachable slots nearest
# the limit are 2044 MiB + 4 KiB (accepted: its allocation rounds to 2046 MiB
# = the limit) and 2046 MiB + 4 KiB (refused).  ADVICE r05: the boundary
# itself, not 2042 MiB, and the first size past it.
IPC_MAX_SLOT = (2 << 30) - (2 << 20)


def _slot_bytes(n: int) -> int:
    n4 = -(-(-(-n // 4)) // 1024) * 1024
    return -(-(16 * n4 + 256) // (2 << 20)) * (2 << 20) + 4096


N_SLOT_OK, N_SLOT_REFUSED = 535_818_240, 535_822_336
assert _slot_bytes(N_SLOT_OK) == (2044 << 20) + 4096 <= IPC_MAX_SLOT
assert _slot_bytes(N_SLOT_REFUSED) == (2046 << 20) + 4096 > IPC_MAX_SLOT


def _boundary_main(rank, world, d, q):
    rank_env(rank)
    try:
        # torch first, as in bench.py (crossbow_amd/_lib.py): the library then
        # runs on torch's bundled HIP runtime (7.0), whose IPC keeps the 32-bit
        # size the limit is for, not on the system ROCm's
        import torch
        hip_version = torch.version.hip
        L, A = load_real()
        O = C.oracle()
        out = {"hip": hip_version}
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid_refused")))
        try:
            C.setup_model(g, A, N_SLOT_REFUSED, 1, 0.9, 7, A.SYNC_BSP, 2 * world)
            buf = ctypes.create_string_buffer(A.PEER_BLOB_BYTES)
            nb = ctypes.c_size_t(0)
            rc = L.cbx_peer_export(g.c, buf, ctypes.byref(nb))
            out["refused"] = (rc, L.cbx_last_error().decode())
        finally:
            g.free()
        n = N_SLOT_OK
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid_ok")))
        try:
            C.setup_model(g, A, n, 1, 0.9, 7, A.SYNC_BSP, 2 * world)
            exchange(g, rank, world, d, "edge")  # opens the other rank's 2046 MiB allocations
            g("cbx_set_allreduce_algorithm", PEER)
            g("cbx_set_bucket_elements", ctypes.c_longlong(1 << 26))  # 8 buckets
            g("cbx_fill_synthetic", 3)
            rng = np.random.default_rng(5)
            half = n // 2  # around the two ranks' shards of each bucket and the buffer's ends
            idx = np.unique(np.concatenate([rng.integers(0, n, 100_000), np.arange(4096), np.arange(n - 4096, n),
                                            np.arange(half - 2048, half + 2048)]))
            z0 = g.read("cbx_base_read", rank, A.BUF_DATA, n)
            l0 = g.read("cbx_base_read", rank, A.BUF_LAST, n)
            s0 = g.read("cbx_replica_read", rank, A.BUF_DIFF, n)[idx]
            w0 = g.read("cbx_replica_read", rank, A.BUF_DATA, n)[idx]
            np.savez(os.path.join(d, f"edge_{rank}.tmp.npz"), z=z0[idx], last=l0[idx], s=s0, w=w0)
            os.replace(os.path.join(d, f"edge_{rank}.tmp.npz"), os.path.join(d, f"edge_{rank}.npz"))
            del z0, l0
            g("cbx_lock_any")
            g("cbx_synchronise", 0, 1, 0, 0)
            g("cbx_unlock_any")
            g("cbx_wait")
            z1 = g.read("cbx_base_read", rank, A.BUF_DATA, n)
            l1 = g.read("cbx_base_read", rank, A.BUF_LAST, n)
            out["digest"] = C.digest(z1, l1)
            z1, l1 = z1[idx], l1[idx]
            w1 = g.read("cbx_replica_read", rank, A.BUF_DATA, n)[idx]
        finally:
            g.free()
        C.wait_files([os.path.join(d, f"edge_{r}.npz") for r in range(world)], seconds=120)
        ins = [np.load(os.path.join(d, f"edge_{r}.npz")) for r in range(world)]
        st = O.SmaState(world, world, idx.size, 0.1, 0.9, [f["z"].copy() for f in ins],
                        [f["last"].copy() for f in ins], [f["s"].copy() for f in ins], [f["w"].copy() for f in ins])
        O.sma_step(st)
        check = C.Checker(exact=True)
        check("z sample", z1, st.z[rank])
        check("last sample", l1, st.last[rank])
        check(f"w[{rank}] sample", w1, st.w[rank])
        out["bad"] = check.bad
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(330)
def test_peer_export_slot_boundary():
    world = 2
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _boundary_main, lambda r: (r, world, d), timeout=300)
    for r in range(world):
        rc, msg = res[r]["refused"]
        assert rc == -8 and "at most 2046 MiB" in msg, (r, rc, msg)  # CBX_ERR_UNSUPPORTED
        assert not res[r]["bad"], (r, res[r]["bad"])
    assert res[0]["digest"] == res[1]["digest"], "z / last differ across ranks at the largest exported slot"
    print(f"largest exported slot {_slot_bytes(N_SLOT_OK)} B opened and stepped, {_slot_bytes(N_SLOT_REFUSED)} B "
          f"refused, under torch's HIP {res[0]['hip']}")


def _import_fail_main(rank, world, d, q):
    """Rank 1's opens fail ($CBX_FAULT_IPC_OPEN_FAIL=1): every rank's import
    must fail, no rank may take the form, and the RCCL form must still run on
    every rank (a failed import refuses no collective step)."""
    rank_env(rank)
    os.environ["CBX_FAULT_IPC_OPEN_FAIL"] = "1"  # read at context creation
    try:
        L, A = load_real()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        out = {}
        try:
            n = 1 << 20
            C.setup_model(g, A, n, 2, 0.9, 7, A.SYNC_BSP, 2 * world * 2)
            try:
                exchange(g, rank, world, d, "impfail")
                out["import"] = None
            except RuntimeError as e:
                out["import"] = str(e)
            out["peer"] = L.cbx_set_allreduce_algorithm(g.c, PEER)
            g("cbx_set_allreduce_algorithm", 0)
            g("cbx_set_bucket_elements", ctypes.c_longlong(1 << 18))
            g("cbx_fill_synthetic", 9)
            for clock in (1, 2):
                g("cbx_lock_any")
                g("cbx_synchronise", 0, clock, 0, 0)
                g("cbx_unlock_any")
            g("cbx_wait")
            out["digest"] = C.digest(g.read("cbx_base_read", rank, A.BUF_DATA, n),
                                     g.read("cbx_base_read", rank, A.BUF_LAST, n))
        finally:
            g.free()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(200)
def test_peer_import_fails_on_every_rank_or_none():
    world = 3
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _import_fail_main, lambda r: (r, world, d), timeout=180)
    assert "fault injection" in (res[1]["import"] or ""), res[1]["import"]
    for r in (0, 2):
        assert res[r]["import"] and "rank 1's import failed" in res[r]["import"], (r, res[r]["import"])
    for r in range(world):
        assert res[r]["peer"] == -2, (r, res[r]["peer"])  # CBX_ERR_STATE: the form needs a successful import
    assert len({res[r]["digest"] for r in range(world)}) == 1, "the RCCL form after a failed import"


def _healthy_resync_main(rank, world, d, q):
    """No failure: two peer-read steps, cbx_resync_base (a no-op for z / last,
    which are already identical, but it clears the page and restarts the step
    numbering), two more peer-read steps; every element against the oracle."""
    rank_env(rank)
    try:
        L, A = load_real()
        O = C.oracle()
        g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
        try:
            n, R = 1 << 20, 2
            size = world * R
            mine = [i for i in range(size) if i % world == rank]
            C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_BSP, 2 * world * R)
            exchange(g, rank, world, d, "healthy")
            g("cbx_set_allreduce_algorithm", PEER)
            g("cbx_set_bucket_elements", ctypes.c_longlong(1 << 18))
            g("cbx_set_pipeline_mode", 1)
            g("cbx_fill_synthetic", 4)
            _save(d, f"in_{rank}", z=g.read("cbx_base_read", rank, A.BUF_DATA, n),
                  last=g.read("cbx_base_read", rank, A.BUF_LAST, n),
                  s=np.stack([g.read("cbx_replica_read", i, A.BUF_DIFF, n) for i in mine]),
                  w=np.stack([g.read("cbx_replica_read", i, A.BUF_DATA, n) for i in mine]), ids=np.array(mine))
            for clock in (1, 2, 3, 4):
                if clock == 3:
                    g("cbx_resync_base", 0)
                g("cbx_lock_any")
                g("cbx_synchronise", 0, clock, 0, 0)
                g("cbx_unlock_any")
            g("cbx_wait")
            st = _oracle_state(O, world, size, n, _load_all(d, "in", world))
            for _ in range(4):
                O.sma_step(st)
            check = C.Checker(exact=True)
            check("z", g.read("cbx_base_read", rank, A.BUF_DATA, n), st.z[rank])
            check("last", g.read("cbx_base_read", rank, A.BUF_LAST, n), st.last[rank])
            for i in mine:
                check(f"w[{i}]", g.read("cbx_replica_read", i, A.BUF_DATA, n), st.w[i])
        finally:
            g.free()
        q.put((rank, {"bad": check.bad}, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(200)
def test_peer_resync_without_failure_keeps_the_form_exact():
    world = 2
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as d:
        res = _spawn(world, _healthy_resync_main, lambda r: (r, world, d), timeout=180)
    for r in range(world):
        assert not res[r]["bad"], (r, res[r]["bad"])
