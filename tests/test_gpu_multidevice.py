"""The reference's own multi-GPU form on ONE GPU: one process drives G devices.

Crossbow runs one JVM over all selected GPUs: ncclCommInitAll over the G
devices (clib-multigpu/executioncontext.c:185-201) and, per step, grouped
ncclAllReduce calls issued from one thread (synch/common.c:14-54).  The JNI
drop-in reaches it through cbx_init(devices, G) (TheGPU_jni.c -> context.hip, sync_steps.hip).

Here cbx_init gets G copies of device 0 and the library build linked
against the loopback collective (tests/native/fake_rccl.cpp), whose
ncclCommInitAll(ndev > 1) forms an in-process clique and runs the grouped
all-reduces at ncclGroupEnd.  So the per-device hipSetDevice loops, the
grouped all-reduce across local communicators, the bucketed pipeline over G
local devices, Phase D, S-SGD, the pipelined host-staged step, BN averaging,
autotune and checkpoint / override over several local devices all run the
product code.  Rank-order loopback: bit for bit against the oracle with the
same G and against the committed golden fixtures; ring-order loopback: the
G > 1 tolerance plus z / last bitwise identical on every device.

The peer-read all-reduce (cbx_set_allreduce_algorithm PEER: two-shot over
direct peer reads, no RCCL pass, bucketed and pipelined like the all-reduce)
runs only in this form; its cases (1 to 25 buckets, both pipeline modes,
groups, wait strides), and the
golden fixtures run through it, are bit for bit against the oracle (device
order from +0 is the oracle's order).  On one GPU every "peer" is device 0
itself, so this pins the algorithm, not its xGMI speed.

The reduce-scatter form (cbx_set_allreduce_algorithm RSAG: reduce-scatter,
base momentum on each device's shard, all-gather) runs here and in the
one-process-per-GPU tests: bit for bit in rank order (the loopback's
reduce-scatter sums in rank order), within the tolerance in ring order, and
through the G > 1 golden fixtures.

The worker runs in a spawned, torch-free process (crossbow_amd/_abi.py), so
no real RCCL is loaded beside the loopback one.  Shared machinery:
tests/multidev_common.py.
"""
from __future__ import annotations

import os
import tempfile

import pytest

from tests import multidev_common as C
from tests.multidev_common import Case

pytestmark = pytest.mark.gpu

CASES = [
    Case("sma", 50_001, 2, 0.9, 3),
    Case("sma-copy-ssp", 50_001, 2, 0.9, 3, copy={1: 3}, held={0: 1}),
    Case("sma-buckets-group", 300_007, 3, 0.9, 2, bucket=65_536, copy={1: 0}, group=2),
    Case("sma-buckets-cross", 300_007, 2, 0.9, 5, bucket=65_536, copy={2: 1}, held={3: 0}, mode=1, stride=2),
    Case("sma-no-momentum", 20_011, 1, 0.0, 2, bucket=4096, utype=3),
    Case("sma-staged", 100_003, 2, 0.9, 3, copy={1: 2}, held={0: 3}, staged=3),  # zero-copy staging kernels
    Case("sma-staged-dma", 100_003, 2, 0.9, 2, copy={0: 1}, held={1: 2}, staged=3, staging=1),
    Case("ssgd", 40_009, 2, 0.9, 2, utype=1),
    Case("ssgd-buckets", 40_009, 2, 0.9, 2, bucket=4096, utype=1),
    Case("sma-ring", 50_001, 2, 0.9, 4, copy={2: 1}, order="ring"),
    Case("sma-ring-buckets-cross", 300_007, 2, 0.9, 4, bucket=65_536, mode=1, order="ring"),
    # the peer-read two-shot all-reduce (cbx_set_allreduce_algorithm PEER): no RCCL pass
    Case("sma-peer", 50_001, 2, 0.9, 3, copy={1: 3}, held={0: 1}, algo=1),
    Case("sma-peer-no-momentum", 20_011, 1, 0.0, 2, utype=3, algo=1),
    Case("sma-peer-empty-shards", 1031, 2, 0.9, 3, copy={2: 0}, algo=1),  # n4 = one pad: trailing shards empty
    Case("sma-peer-big", 300_007, 3, 0.9, 2, algo=1),
    # the peer-read form bucketed and pipelined like the all-reduce (the cases
    # above run the library default, 8 buckets): one bucket in order, groups,
    # the cross-step pipeline with a wait stride, many small buckets
    Case("sma-peer-one-bucket", 300_007, 2, 0.9, 3, bucket=1 << 40, copy={1: 0}, held={2: 1}, algo=1),
    Case("sma-peer-buckets-group", 300_007, 3, 0.9, 3, bucket=65_536, group=3, copy={1: 2}, algo=1),
    Case("sma-peer-buckets-cross", 300_007, 2, 0.9, 5, bucket=65_536, copy={2: 1}, held={3: 0}, mode=1, stride=2,
         group=2, algo=1),
    Case("sma-peer-many-buckets", 100_003, 2, 0.0, 3, bucket=4096, utype=3, mode=1, copy={1: 1}, algo=1),
    # switching between the algorithms, and from the cross-step pipeline, between steps
    Case("sma-peer-switch", 300_007, 2, 0.9, 5, bucket=65_536, mode=1, copy={3: 1}, algo_at={1: 1, 2: 0, 4: 1}),
    # the reduce-scatter form (RSAG: reduce-scatter, momentum on the shard, all-gather)
    Case("sma-rsag", 50_001, 2, 0.9, 3, copy={1: 3}, held={0: 1}, algo=2),
    Case("sma-rsag-no-momentum", 20_011, 1, 0.0, 2, bucket=4096, utype=3, algo=2),
    Case("sma-rsag-buckets-cross", 300_007, 2, 0.9, 5, bucket=65_536, copy={2: 1}, held={3: 0}, mode=1, stride=2,
         group=2, algo=2),
    Case("sma-rsag-ring", 300_007, 2, 0.9, 4, bucket=65_536, mode=1, order="ring", algo=2),
    Case("sma-rsag-switch", 300_007, 2, 0.9, 5, bucket=65_536, mode=1, copy={3: 1}, algo_at={1: 2, 2: 0, 3: 1, 4: 2}),
]


def _jobs(G):
    if G == 3:  # a non-power-of-two clique: the plain step in both orders, and the peer path (RSAG is refused)
        names = ("sma", "sma-ring", "sma-peer", "sma-peer-empty-shards", "sma-peer-buckets-cross")
    elif G == 16:  # the most devices one process takes (kMaxDevices): plain, ring order, peer, reduce-scatter
        names = ("sma-copy-ssp", "sma-ring", "sma-peer", "sma-peer-empty-shards", "sma-peer-buckets-cross", "sma-rsag",
                 "sma-rsag-ring")
    elif G == 8:
        names = ("sma-copy-ssp", "sma-buckets-cross", "ssgd-buckets", "sma-ring", "sma-ring-buckets-cross",
                 "sma-peer", "sma-peer-empty-shards", "sma-peer-switch", "sma-peer-one-bucket", "sma-peer-buckets-cross",
                 "sma-peer-many-buckets", "sma-rsag", "sma-rsag-buckets-cross",
                 "sma-rsag-ring", "sma-rsag-switch")
    else:
        names = [c.name for c in CASES]
    jobs = [("case", n) for n in names if G >= 3 or "-ring" not in n]
    jobs += [("golden", gc["name"]) for gc in C.golden_cases(G)]
    jobs += [("golden-peer", gc["name"]) for gc in C.golden_cases(G)]
    jobs += [("golden-rsag", gc["name"]) for gc in C.golden_cases(G)]
    return jobs + [("bn", "bn"), ("autotune", "autotune"), ("resync", "resync")]


def _worker(G, jobs, ckdir, q, threads=-1):
    try:
        L, A = C.load_variant()
        cases = {c.name: c for c in CASES}
        goldens = {gc["name"]: gc for gc in C.golden_cases(G)}
        local = list(range(G))
        out = []
        for kind, name in jobs:
            os.environ["FAKE_RCCL_ORDER"] = cases[name].order if kind == "case" else "rank"
            g = C.init_local(L, A, G)
            try:
                assert L.cbx_set_enqueue_threads(g.c, threads) == 0
                if G == 3:  # the reduce-scatter form needs G dividing the bucket padding
                    assert L.cbx_set_allreduce_algorithm(g.c, A.ALLREDUCE_RSAG) == A.CBX_ERR_UNSUPPORTED
                if kind == "case":
                    res = C.run_case(g, G, local, cases[name])
                elif kind.startswith("golden"):
                    algo = {"golden": 0, "golden-peer": 1, "golden-rsag": 2}[kind]
                    res = {"bad": C.run_golden(g, G, local, goldens[name], algo=algo)}
                elif kind == "bn":
                    res = {"bad": C.run_bn(g, G, local, poison=True)}
                elif kind == "resync":
                    res = {"bad": C.run_resync(g, G, local, root=G - 1)}
                else:
                    res = {"bad": C.run_autotune_checkpoint(g, G, local, ckdir)}
            finally:
                g.free()
            out.append((name, res))
        q.put((out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((None, traceback.format_exc()))


@pytest.mark.skipif(not os.path.exists(C.VARIANT), reason="run scripts/build_fake_rccl.sh first")
@pytest.mark.parametrize("G,threads", [(2, 1), (3, 1), (4, 1), (8, 1), (16, 1), (2, 0), (4, -1), (8, 0)])
def test_one_process_many_devices_vs_oracle(G, threads):
    """threads 1: one enqueue thread per device, each issuing its own
    communicator's collectives (the loopback meets them at a rendezvous) and,
    in the peer-read form, waiting on the other devices' events only once
    their threads recorded them; 0 and -1 (the default): the reference's
    single thread, collectives grouped across the devices."""
    import multiprocessing as mp
    jobs = _jobs(G)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as ckdir:
        p = ctx.Process(target=_worker, args=(G, jobs, os.path.join(ckdir, "ckpt"), q, threads))
        p.start()
        try:
            res, err = q.get(timeout=110)
        finally:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert err is None, err
    assert [name for name, _ in res] == [name for _, name in jobs]
    failures = [(name, r["bad"]) for name, r in res if r["bad"]]
    assert not failures, failures
    cases = {c.name: c for c in CASES}
    for (kind, name), (_, r) in zip(jobs, res):
        if kind != "case":
            continue
        assert len(set(r["digest"].values())) == 1, f"{name}: z / last differ across devices"
        if cases[name].order == "ring":
            assert r["differs"] > 0, f"{name}: ring order never left the oracle's order"
