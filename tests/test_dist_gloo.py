"""The G > 1 path, rehearsed on CPU with two gloo ranks (no GPU needed).

Each rank owns the replicas ``i % G == rank`` (clib-multigpu/modelmanager.c:
51-64, ``crossbow_amd.dist.local_replicas``), runs Phase A over its locked
replicas in id order (the oracle's kernel-A restatement), all-reduces
``acc`` together with the Phase-D copy count in a control slot in front of
it (what ``libcrossbow_sma`` sends through RCCL), and applies Phase C / D.
The result on every rank must equal the single-address-space G = 2 oracle
(clib-multigpu/synch/sma.c:13-231): with two ranks the fp32 sum a + b is
order independent, so the comparison is bit for bit.  The synchronous-SGD
barrier and the batch-norm statistics averaging are rehearsed the same way.
The control plane of
``crossbow_amd.dist`` (unique-id broadcast, barrier, max over ranks) runs
over the same gloo group.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CASES = [
    # (n, R per rank, alpha, momentum, copy ids, unlocked ids, first)
    (4099, 2, 0.1, 0.9, [], [], 0),
    (1031, 3, 0.5, 0.0, [3], [], 0),
    (2053, 2, 0.1, 0.9, [], [1], 0),
    (777, 2, 0.1, 0.9, [0], [], 1),
]


def _rank_main(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        import torch
        import torch.distributed as dist

        from crossbow_amd import dist as D
        from oracle import oracle as O

        D.init(world, rank, backend="gloo")
        uid = D.share_unique_id(rank, world, lambda: bytes(range(128)))
        assert uid == bytes(range(128))
        assert D.max_over_ranks(float(rank + 1), world) == float(world)
        D.barrier(world)

        results = []
        for (n, R, alpha, mom, copy_ids, unlocked, first) in CASES:
            ref = O.make_state(n, world, R, alpha, mom)
            for i in copy_ids:
                ref.copy[i] = 1
            for i in unlocked:
                ref.locked[i] = 0
            ref.first = first
            mine = ref.clone()
            O.sma_step(ref)  # single address space, G = world

            ids = [i for i in D.local_replicas(mine.size, world, rank)
                   if i >= first and mine.locked[i]]
            z = mine.z[rank]
            last = mine.last[rank] if mine.last is not None else None
            s = [mine.s[i] for i in ids]
            w = [mine.w[i] for i in ids]
            acc, copies = O.sma_accumulate(alpha, z, s, w, [int(mine.copy[i]) for i in ids])
            # control slot in front of acc, summed with it (sync_steps.hip, sma_internal.h)
            buf = torch.from_numpy(np.concatenate([np.array([copies], np.float32), acc]))
            dist.all_reduce(buf, op=dist.ReduceOp.SUM)
            ctrl, Dsum = float(buf[0]), buf[1:].numpy().copy()
            O.sma_apply(mom, Dsum, z, last, w, ctrl > 0)

            ok = bool(np.array_equal(z.view(np.uint32), ref.z[rank].view(np.uint32)))
            if last is not None:
                ok &= bool(np.array_equal(last.view(np.uint32), ref.last[rank].view(np.uint32)))
            for k, i in enumerate(ids):
                ok &= bool(np.array_equal(w[k].view(np.uint32), ref.w[i].view(np.uint32)))
            # replicas that did not take part are untouched
            for i in D.local_replicas(mine.size, world, rank):
                if i not in ids:
                    ok &= bool(np.array_equal(mine.w[i], ref.w[i]))
            results.append(ok)
        # Synchronous SGD (WORKER, synchronoussgd.c:13-106): task steps add into
        # each rank's base gradient; the barrier all-reduces it and every rank
        # applies it to its own base model and replicas.
        n, R, wpc = 3001, 2, 4
        ref = O.make_state(n, world, R, 0.1, 0.9)
        grads = [O.fill_normal(n, 4000 + i, 0.01) for i in range(ref.size)]
        acc_ref = [np.zeros(n, np.float32) for _ in range(world)]
        mine = ref.clone()
        for i in range(ref.size):
            O.ssgd_worker(np.float32(-0.05), 1e-4, ref.w[i], grads[i].copy(), acc_ref[i % world])
        O.ssgd_sync(ref, acc_ref, wpc)
        ids = D.local_replicas(mine.size, world, rank)
        acc = np.zeros(n, np.float32)
        for i in ids:
            O.ssgd_worker(np.float32(-0.05), 1e-4, mine.w[i], grads[i].copy(), acc)
        buf = torch.from_numpy(acc.copy())
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        local = O.SmaState(1, len(ids), n, 0.1, 0.9, [mine.z[rank]], [mine.last[rank]],
                           [mine.s[i] for i in ids], [mine.w[i] for i in ids])
        O.ssgd_sync(local, [buf.numpy().copy()], wpc)
        ok = bool(np.array_equal(local.z[0].view(np.uint32), ref.z[rank].view(np.uint32)))
        ok &= bool(np.array_equal(local.last[0].view(np.uint32), ref.last[rank].view(np.uint32)))
        for k, i in enumerate(ids):
            ok &= bool(np.array_equal(local.w[k].view(np.uint32), ref.w[i].view(np.uint32)))
        results.append(ok)

        # Batch-norm statistics (cudnnbatchnormparams.c:157-222) the way the
        # library packs them: [count slots | scale*mean | scale*var] per layer,
        # one all-reduce, then * 1/count.  Rank 1 has updates on layer 0 only.
        elements = [16, 40]
        mean = [[O.fill_normal(e, 50 + 10 * g + l, 0.5) for l, e in enumerate(elements)] for g in range(world)]
        var = [[O.fill_normal(e, 90 + 10 * g + l, 0.5) for l, e in enumerate(elements)] for g in range(world)]
        updated = [[1, 1], [1, 0]]
        ref_m = [[a.copy() for a in r] for r in mean]
        ref_v = [[a.copy() for a in r] for r in var]
        O.bn_average(ref_m, ref_v, updated)
        L = len(elements)
        scale = [1.0 if (rank == 0 or updated[rank][l]) else 0.0 for l in range(L)]
        parts = [np.array(scale, np.float32)]
        for l in range(L):
            parts += [np.float32(scale[l]) * mean[rank][l], np.float32(scale[l]) * var[rank][l]]
        buf = torch.from_numpy(np.concatenate(parts))
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        b = buf.numpy()
        off = L
        ok = True
        for l, e in enumerate(elements):
            count = float(b[l])
            r = np.float32(1.0 / count) if count > 1 else np.float32(1.0)
            m, v = r * b[off:off + e], r * b[off + e:off + 2 * e]
            off += 2 * e
            ok &= bool(np.array_equal(m.view(np.uint32), ref_m[rank][l].view(np.uint32)))
            ok &= bool(np.array_equal(v.view(np.uint32), ref_v[rank][l].view(np.uint32)))
        results.append(ok)
        D.barrier(world)
        D.finalize(world)
        q.put((rank, results, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_two_rank_sharded_sma_equals_single_process_oracle():
    import torch.multiprocessing as mp
    from oracle import oracle as O
    O.lib()  # build the oracle before forking ranks
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            out[rank] = (res, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        res, err = out[rank]
        assert err is None, f"rank {rank} failed:\n{err}"
        assert all(res), f"rank {rank}: per-case parity {res} (cases {CASES})"


def test_local_replicas_round_robin():
    from crossbow_amd import dist as D
    assert D.local_replicas(8, 4, 1) == [1, 5]
    assert D.local_replicas(32, 8, 7) == [7, 15, 23, 31]
    assert sorted(sum((D.local_replicas(12, 3, r) for r in range(3)), [])) == list(range(12))


def test_env_rank_defaults(monkeypatch):
    from crossbow_amd import dist as D
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert D.env_rank() == (0, 1, 0)
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert D.env_rank() == (3, 8, 3)


class _FakeGpu:
    """Stands in for TheGPU in tune_buckets: a step 'costs' a rank-dependent
    time per bucket count (sleep), so the ranks disagree locally."""

    def __init__(self, rank, n, fail_on=None):
        self.rank, self.n, self.elems, self.mode, self.stride, self.group = rank, n, 0, 0, 1, 1
        self.algo = 0
        self.threads = -1
        self.fail_on = fail_on  # (buckets, mode) whose steps raise CbxError on this rank

    def set_enqueue_threads(self, t):
        self.threads = t

    def set_allreduce_algorithm(self, a):
        self.algo = a

    def set_bucket_elements(self, e):
        self.elems = e

    def set_pipeline_mode(self, m):
        self.mode = m

    def set_cross_wait_stride(self, s):
        self.stride = s

    def set_allreduce_group(self, g):
        self.group = g

    def wait(self):
        pass

    def step(self):
        import time
        nb = 1 if self.elems >= self.n else -(-self.n // self.elems)
        if self.fail_on == (nb, self.mode):
            from crossbow_amd._abi import CbxError
            raise CbxError(-5, f"injected failure at {nb} buckets, mode {self.mode}")
        # rank 0 is fastest at 8 buckets, rank 1 at 2; the max over ranks is lowest at 4
        cost = {0: {1: 9, 2: 7, 4: 4, 8: 1}, 1: {1: 9, 2: 1, 4: 4, 8: 7}}[self.rank][nb]
        cost += 2 if (self.mode >= 1 and self.rank == 1) else 0  # cross-step modes slower on rank 1
        cost += self.stride - 1  # and fewer cross-step waits slower everywhere
        cost += {0: -1, 1: 2}[self.rank] if self.group > 1 else 0  # grouping helps rank 0 only: max says no
        cost -= 1 if self.algo == 2 else 0  # the reduce-scatter form is faster on both ranks
        time.sleep(cost * 2e-3)


def _tune_main(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        from crossbow_amd import dist as D
        D.init(world, rank, backend="gloo")
        g = _FakeGpu(rank, 1000)
        g.group = 3  # a group left over from an earlier setting must not skew the sweep
        g.algo = 2   # nor an algorithm left over: the sweep runs on the all-reduce
        refreshed = []  # bench.py's fresh-state hook: once per candidate, before its warm-up
        t = D.tune_buckets(g, 1000, world, g.step, steps=2, warmup=1,
                           refresh=lambda: refreshed.append((g.elems, g.mode, g.stride, g.group, g.algo)))
        q.put((rank, (t.bucket_elements, g.elems, t.mode, g.mode, t.stride, g.stride, t.group, g.group, t.algorithm,
                      g.algo, sorted(t.table), refreshed), None))
        D.finalize(world)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_bucket_tuning_agrees_across_ranks():
    # dist.tune_buckets: every rank must end on the same bucket count (else
    # the ranks' RCCL call sequences differ and the all-reduce hangs), chosen
    # by the max-over-ranks step time: 4 buckets here.
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tune_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            out[rank] = (res, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        assert out[rank][1] is None, out[rank][1]
    (e0, set0, m0, setm0, s0, sets0, g0, setg0, a0, seta0, cands, refreshed), \
        (e1, set1, m1, setm1, s1, sets1, g1, setg1, a1, seta1, _, _) = out[0][0], out[1][0]
    assert e0 == e1 == set0 == set1 == 250, (out[0][0], out[1][0])
    assert m0 == m1 == setm0 == setm1 == 0
    assert s0 == s1 == sets0 == sets1 == 1
    assert g0 == g1 == setg0 == setg1 == 1  # the all-reduce group of the winner, by the max over ranks
    want = ["1/0"] + [f"{nb}/{m}" for nb in (2, 4, 8) for m in (0, 1)]
    want += [f"{nb}/1/s{s}" for nb in (4, 8) for s in (2, 4) if s < nb]
    want += [k + "/rsag" for k in want]  # every candidate in the reduce-scatter form too
    want += ["4/0/rsag/g2"]  # groups 1 < g < buckets, timed for the winner only
    assert cands == sorted(want)
    # one fresh state per timed candidate and pass (2 passes), each already in that candidate's setting
    assert len(refreshed) == 2 * len(want), (len(refreshed), len(want))
    assert len(set(refreshed)) == len(want)
    assert a0 == a1 == seta0 == seta1 == 2  # faster on both ranks: chosen


def _tune_fail_main(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        from crossbow_amd import dist as D
        D.init(world, rank, backend="gloo")
        # 4 buckets (the max-over-ranks winner of test_bucket_tuning_agrees_across_ranks)
        # fail in mode 0 on rank 1 only; one process over 2 "devices" also times the
        # peer-read form and the threaded enqueue
        g = _FakeGpu(rank, 1000, fail_on=(4, 0) if rank == 1 else None)
        t = D.tune_buckets(g, 1000, world, g.step, steps=2, warmup=1, threads=True)
        q.put((rank, (t.buckets, t.mode, t.algorithm, t.enqueue_threads, g.threads, sorted(t.table), t.errors), None))
        D.finalize(world)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_bucket_tuning_drops_a_failing_candidate_on_every_rank():
    # A candidate whose step raises CbxError on ONE rank is dropped on every
    # rank (else the ranks would disagree on the winner and their RCCL call
    # sequences diverge), recorded in Tuning.errors, and the sweep goes on.
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tune_fail_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            out[rank] = (res, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        assert out[rank][1] is None, out[rank][1]
    r0, r1 = out[0][0], out[1][0]
    assert r0[:6] == r1[:6], (r0, r1)
    nb, mode, algo, threads, set_threads, table, errors = r0
    assert "4/0" not in table and "4/0/rsag" not in table, table
    assert "4/1" in table  # the same bucket count in mode 1 still runs
    assert sorted(errors) == ["4/0", "4/0/rsag"], errors
    assert "injected failure" in r1[6]["4/0"] and r0[6]["4/0"] == "failed on another rank"
    assert threads in (0, 1) and set_threads == threads
    assert (nb, mode) != (4, 0)


class _FakePeerGpu:
    """Stands in for TheGPU in dist.setup_peer: export returns a rank-stamped
    blob (or fails), import records what it was handed (or fails)."""

    def __init__(self, rank, fail=None):
        self.rank, self.fail, self.imported = rank, fail, None

    def peer_export(self):
        from crossbow_amd._abi import PEER_BLOB_BYTES, CbxError
        if self.fail == "export":
            raise CbxError(-8, f"injected export failure on rank {self.rank}")
        return bytes([self.rank + 1]) * PEER_BLOB_BYTES

    def peer_import(self, blobs):
        from crossbow_amd._abi import CbxError
        if self.fail == "import":
            raise CbxError(-3, f"injected import failure on rank {self.rank}")
        self.imported = [b[0] for b in blobs]


def _peer_main(rank, world, port, fail_rank, fail, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        from crossbow_amd import dist as D
        D.init(world, rank, backend="gloo")
        g = _FakePeerGpu(rank, fail if rank == fail_rank else None)
        why = D.setup_peer(g, world)
        q.put((rank, (why, g.imported), None))
        D.finalize(world)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("fail_rank,fail", [(None, None), (1, "export"), (0, "import")])
def test_peer_ipc_setup_gathers_in_rank_order_and_agrees(fail_rank, fail):
    # dist.setup_peer: every rank imports every rank's blob in rank order;
    # a failure on ONE rank (its export or its import) makes every rank
    # report it, so no rank ever runs the peer-read form alone.
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_peer_main, args=(r, world, port, fail_rank, fail, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            out[rank] = (res, err)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        assert out[rank][1] is None, out[rank][1]
    (why0, imp0), (why1, imp1) = out[0][0], out[1][0]
    if fail is None:
        assert why0 is None and why1 is None
        assert imp0 == imp1 == [1, 2]  # rank order
    else:
        assert why0 and why1, (why0, why1)
        assert f"injected {fail} failure" in (why0 if fail_rank == 0 else why1)
