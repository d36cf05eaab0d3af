#!/usr/bin/env python3
"""One rank of a G-rank SMA job on ONE GPU with the real RCCL (socket
transport, NCCL_HOSTID per rank), for a kernel trace of the bucketed
pipeline with an asynchronous collective beside kernels A and B.

Launched once per rank by scripts/trace_real_rccl.sh, each under its own
rocprofv3 (the profiler wraps this program directly).  algo 1: the per-rank
peer-read form (cbx_peer_export / _import through files in $TRACE_DIR).  Ranks meet through
files in $TRACE_DIR.  Usage: trace_rank.py RANK WORLD [buckets] [mode] [algo]
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    buckets = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    mode = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    algo = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    d = os.environ.get("TRACE_DIR", "/tmp")
    from crossbow_amd.dist import rehearsal_env
    rehearsal_env(rank)
    from tests import multidev_common as C
    from tests.test_gpu_realrccl import share_uid
    A = C.abi()
    L = A.bind(ctypes.CDLL(os.path.join(ROOT, "crossbow_amd", "libcrossbow_sma.so")))
    g = C.init_rank(L, A, rank, world, share_uid(L, rank, os.path.join(d, "uid")))
    try:
        n, R = 25_557_032, 8
        C.setup_model(g, A, n, R, 0.9, 7, A.SYNC_BSP, 2 * world * R)
        if algo == 1:  # the per-rank peer-read form: map the other ranks' acc / D first
            from tests.test_gpu_peer_ipc import exchange
            exchange(g, rank, world, d, "trace")
        g("cbx_fill_synthetic", 20190701)
        g("cbx_set_bucket_elements", ctypes.c_longlong(-(-n // buckets)))
        g("cbx_set_pipeline_mode", mode)
        g("cbx_set_allreduce_algorithm", algo)
        t0 = time.time()
        for step in range(6):
            g("cbx_lock_any")
            g("cbx_synchronise", 0, step + 1, 0, 0)
            g("cbx_unlock_any")
        g("cbx_wait")
        print(f"rank {rank}: 6 steps in {time.time() - t0:.3f} s", flush=True)
    finally:
        g.free()


if __name__ == "__main__":
    main()
