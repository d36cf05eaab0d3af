"""The library's one-process-per-GPU path (cbx_init_rank, G = 2, 4, 8) on ONE
GPU, against the oracle with the same G.

G processes each drive the real library sources as one rank of a G-GPU job,
all on device 0.  Real RCCL refuses two ranks on one device, so this build of
the library (tests/native/libcrossbow_sma_fakerccl.so,
scripts/build_fake_rccl.sh) is linked against a loopback stand-in for the
RCCL calls it makes (tests/native/fake_rccl.cpp).  Everything else is the
product path: the round-robin placement, per-rank locks, kernel A /
all-reduce / kernel B with the control block in bucket 0, the bucketed
pipeline in both modes, Phase D decided on any rank, S-SGD, the pipelined
host-staged step, BN averaging, autotune and a shared checkpoint directory.

* Rank-order loopback: bit for bit against the oracle, plus the committed
  G > 1 golden fixtures (tests/golden/g2_*, g4_*, g8_*).
* Ring-order loopback (RCCL's order, not the oracle's, for G >= 3): within
  rtol 1e-5 / atol 1e-6, and z / last bitwise identical on
  every rank after several steps (sma.c:168-174).
* C4 (2 replicas/GPU x 4) and C5 (4 replicas/GPU x 8) at the full ResNet-50
  size, through sampled parity and the cross-rank identity of z and last.

The rank processes never import torch (they bind the ABI through the
torch-free crossbow_amd/_abi.py), so the loopback library is the only
librccl-like object in them.  Shared machinery: tests/multidev_common.py.
"""
from __future__ import annotations

import os
import tempfile

import numpy as np
import pytest

from tests import multidev_common as C
from tests.multidev_common import Case

pytestmark = pytest.mark.gpu

CASES = [
    Case("sma", 50_001, 2, 0.9, 3),
    Case("sma-copy-ssp", 50_001, 2, 0.9, 3, copy={1: 3}, held={0: 1}),
    Case("sma-5-buckets", 300_007, 3, 0.9, 2, bucket=65_536, copy={1: 0}, group=2),
    Case("sma-5-buckets-cross", 300_007, 2, 0.9, 5, bucket=65_536, copy={2: 1}, held={3: 0}, mode=1),
    Case("sma-5-buckets-cross-stride", 300_007, 2, 0.9, 5, bucket=65_536, copy={2: 1}, held={3: 0}, mode=1,
         stride=2, group=3),
    Case("sma-no-momentum", 20_011, 1, 0.0, 2, bucket=4096, utype=3),
    Case("sma-staged", 100_003, 2, 0.9, 3, copy={1: 2}, held={0: 3}, staged=3),  # zero-copy staging kernels
    Case("sma-staged-dma", 100_003, 2, 0.9, 2, copy={0: 1}, held={1: 2}, staged=3, staging=1),
    Case("ssgd", 40_009, 2, 0.9, 2, utype=1),
    Case("ssgd-buckets", 40_009, 2, 0.9, 2, bucket=4096, utype=1),
    # RCCL's (ring) summation order: the stated tolerance and cross-rank identity
    Case("sma-ring", 50_001, 2, 0.9, 4, copy={2: 1}, order="ring"),
    Case("sma-ring-cross", 300_007, 2, 0.9, 4, bucket=65_536, mode=1, stride=2, order="ring"),
    # the reduce-scatter form (cbx_set_allreduce_algorithm RSAG)
    Case("sma-rsag", 50_001, 2, 0.9, 3, copy={1: 3}, held={0: 1}, algo=2),
    Case("sma-rsag-buckets-cross", 300_007, 2, 0.9, 5, bucket=65_536, copy={2: 1}, held={3: 0}, mode=1, stride=2,
         group=2, algo=2),
    Case("sma-rsag-no-momentum", 20_011, 1, 0.0, 2, bucket=4096, utype=3, algo=2),
    Case("sma-rsag-ring", 300_007, 2, 0.9, 4, bucket=65_536, mode=1, order="ring", algo=2),
]


def _cases(world):
    if world == 2:
        return [c for c in CASES if c.order == "rank"]  # a + b is order-free: ring cases add nothing
    if world == 4:
        return [c for c in CASES if c.name in ("sma", "sma-copy-ssp", "sma-5-buckets", "sma-5-buckets-cross",
                                               "sma-5-buckets-cross-stride", "sma-ring", "sma-ring-cross", "sma-rsag",
                                               "sma-rsag-buckets-cross", "sma-rsag-ring")]
    return [c for c in CASES if c.name in ("sma-copy-ssp", "sma-5-buckets-cross-stride", "ssgd-buckets",
                                           "sma-ring", "sma-rsag-buckets-cross", "sma-rsag-ring")]


def _jobs(world):
    jobs = [("case", c.name) for c in _cases(world)]
    jobs += [("golden", gc["name"]) for gc in C.golden_cases(world)]
    jobs += [("golden-rsag", gc["name"]) for gc in C.golden_cases(world)]
    return jobs + [("bn", "bn"), ("autotune", "autotune"), ("resync", "resync")]


def _rank_main(rank, world, jobs, uids, fake_dir, q):
    os.environ["FAKE_RCCL_DIR"] = fake_dir
    try:
        L, A = C.load_variant()
        cases = {c.name: c for c in CASES}
        goldens = {gc["name"]: gc for gc in C.golden_cases(world)}
        out = []
        for (kind, name), uid in zip(jobs, uids):
            case = cases.get(name)
            os.environ["FAKE_RCCL_ORDER"] = case.order if (kind == "case") else "rank"
            g = C.init_rank(L, A, rank, world, uid)
            try:
                # one process per GPU: the peer-read all-reduce needs the other
                # ranks' buffers mapped first (cbx_peer_import, test_gpu_peer_ipc.py)
                assert L.cbx_set_allreduce_algorithm(g.c, A.ALLREDUCE_PEER) == A.CBX_ERR_STATE
                if kind == "case":
                    res = C.run_case(g, world, [rank], case)
                elif kind.startswith("golden"):
                    res = {"bad": C.run_golden(g, world, [rank], goldens[name], algo=2 if kind == "golden-rsag" else 0)}
                elif kind == "bn":
                    res = {"bad": C.run_bn(g, world, [rank], poison=True)}
                elif kind == "resync":
                    res = {"bad": C.run_resync(g, world, [rank], root=world - 1)}
                else:
                    res = {"bad": C.run_autotune_checkpoint(g, world, [rank], os.path.join(fake_dir, "ckpt"))}
            finally:
                g.free()
            out.append((name, res))
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _spawn(world, target, args_of_rank, timeout):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=args_of_rank(r) + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=timeout)
            got[rank] = (res, err)
            # A rank that failed leaves the others waiting in a collective it
            # will never join: report it now instead of hanging to the timeout.
            assert err is None, f"rank {rank}:\n{err}"
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == world else 1)
            if p.is_alive():
                p.kill()
    return {r: got[r][0] for r in range(world)}


@pytest.mark.skipif(not os.path.exists(C.VARIANT), reason="run scripts/build_fake_rccl.sh first")
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_on_one_gpu_vs_oracle(world):
    jobs = _jobs(world)
    uids = [os.urandom(16) + bytes(112) for _ in jobs]
    with tempfile.TemporaryDirectory(dir=C.loopback_dir()) as fake_dir:
        res = _spawn(world, _rank_main, lambda r: (r, world, jobs, uids, fake_dir), timeout=110)
    cases = {c.name: c for c in CASES}
    for rank in range(world):
        assert [name for name, _ in res[rank]] == [name for _, name in jobs]
        failures = [(name, r["bad"]) for name, r in res[rank] if r["bad"]]
        assert not failures, f"rank {rank}: {failures}"
    for j, (kind, name) in enumerate(jobs):
        if kind != "case":
            continue
        # every rank applied the same D: z and last bitwise identical across ranks (sma.c:168-174)
        digests = {res[r][j][1]["digest"][r] for r in range(world)}
        assert len(digests) == 1, f"{name}: z / last differ across ranks"
        if cases[name].order == "ring" and world >= 3:
            # the tolerance path was really taken: some element left the oracle's order
            assert sum(res[r][j][1]["differs"] for r in range(world)) > 0, f"{name}: ring order never differed"


# ---- C4 / C5 at the full ResNet-50 size -------------------------------------
N_RESNET50 = 25_557_032


def _full_size_main(rank, world, R, steps, mode, order, uid, fake_dir, q):
    """Every rank saves its whole initial state, steps, and then checks its
    own z, last and w against the oracle over EVERY element (no
    sample), the oracle run chunk by chunk over every rank's memory-mapped
    inputs."""
    os.environ["FAKE_RCCL_DIR"] = fake_dir
    os.environ["FAKE_RCCL_ORDER"] = order
    try:
        L, A = C.load_variant()
        O = C.oracle()
        g = C.init_rank(L, A, rank, world, uid)
        try:
            n = N_RESNET50
            C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_BSP, 2 * world * R)
            g("cbx_set_pipeline_mode", mode)
            g("cbx_fill_synthetic", O.SEED)  # the same generator on every rank
            size = world * R
            mine = [i for i in range(size) if i % world == rank]
            C.save_full_state(g, fake_dir, rank, mine, n)
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
        bad, differs, compared = C.full_size_check(fake_dir, world, R, steps, rank, z1, l1, w1, exact=order == "rank")
        q.put((rank, {"bad": bad, "digest": dig, "differs": differs, "compared": compared}, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(330)
@pytest.mark.skipif(not os.path.exists(C.VARIANT), reason="run scripts/build_fake_rccl.sh first")
@pytest.mark.parametrize("world,R,mode,order", [(2, 2, 0, "rank"),   # C4's form at 2 ranks, bit for bit
                                                (4, 2, 0, "rank"),   # C4: 2 replicas/GPU x 4, bit for bit
                                                (8, 4, 1, "rank"),   # C5: 4 replicas/GPU x 8, bit for bit
                                                (8, 4, 1, "ring")])  # C5 in RCCL's order: the tolerance
def test_resnet50_full_size_multirank(world, R, mode, order):
    uid = os.urandom(16) + bytes(112)
    steps = 3
    need = (2 * world + 2 * world * R) * N_RESNET50 * 4 + (1 << 30)
    with tempfile.TemporaryDirectory(dir=C.loopback_dir(need)) as fake_dir:
        res = _spawn(world, _full_size_main, lambda r: (r, world, R, steps, mode, order, uid, fake_dir),
                     timeout=300)
    for r in range(world):
        assert not res[r]["bad"], f"rank {r}: {res[r]['bad']}"
        assert res[r]["compared"] == (2 + R) * N_RESNET50, res[r]["compared"]
    print(f"C{'4' if R == 2 else '5'} full size, {world} ranks x R {R}, order {order}: every rank compared "
          f"{res[0]['compared']} elements (z, last, {R} w; n = {N_RESNET50} each)")
    assert len({res[r]["digest"] for r in range(world)}) == 1, "z / last differ across ranks at full size"
    if order == "ring":
        assert sum(res[r]["differs"] for r in range(world)) > 0, "ring order never left the oracle's order"
