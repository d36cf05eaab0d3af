#!/usr/bin/env python3
"""Probe: the REAL librccl with G ranks on ONE GPU.

RCCL refuses two ranks of one host on the same device ("Duplicate GPU
detected").  Giving every rank its own NCCL_HOSTID makes each rank a host of
its own, so the ranks connect through RCCL's network transport (sockets over
the loopback interface) instead of xGMI / shared memory.  The library's
ncclAllReduce calls then run through RCCL's real kernels, proxy threads and
summation order, asynchronously on the comm stream, beside kernels A and B.

Usage: real_rccl_probe.py [world] [n] [steps]
"""
from __future__ import annotations

import ctypes
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_env(rank: int) -> None:
    os.environ["NCCL_HOSTID"] = f"cbx-rank-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.setdefault("NCCL_NET", "Socket")


def main_rank(rank, world, n, steps, d, q):
    rank_env(rank)
    try:
        from tests import multidev_common as C
        A = C.abi()
        L = A.bind(ctypes.CDLL(os.path.join(ROOT, "crossbow_amd", "libcrossbow_sma.so")))
        uid_path = os.path.join(d, "uid")
        if rank == 0:
            ub = (ctypes.c_ubyte * 128)()
            assert L.cbx_get_unique_id(ub) == 0
            with open(uid_path + ".tmp", "wb") as f:
                f.write(bytes(ub))
            os.replace(uid_path + ".tmp", uid_path)
        C.wait_files([uid_path])
        uid = open(uid_path, "rb").read()
        t0 = time.time()
        g = C.init_rank(L, A, rank, world, uid)
        t_init = time.time() - t0
        try:
            case = C.Case("probe", n, 2, 0.9, steps, bucket=n // 3 + 1, copy={1: 1}, order="ring")
            t0 = time.time()
            res = C.run_case(g, world, [rank], case)
            res["t_init"] = t_init
            res["t_case"] = time.time() - t0
        finally:
            g.free()
        q.put((rank, res, None))
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50_001
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        procs = [ctx.Process(target=main_rank, args=(r, world, n, steps, d, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = {}
        for _ in range(world):
            r, res, err = q.get(timeout=120)
            got[r] = (res, err)
        for p in procs:
            p.join(timeout=30)
    ok = True
    for r in range(world):
        res, err = got[r]
        if err:
            print(f"rank {r} error:\n{err}")
            ok = False
        else:
            print(f"rank {r}: bad={res['bad']} differs={res['differs']} digest={list(res['digest'].values())[0][:16]} "
                  f"init {res['t_init']:.2f}s case {res['t_case']:.2f}s")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
