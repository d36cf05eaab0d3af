#!/usr/bin/env python3
"""Host side of the single-process multi-device step (Crossbow's own form:
one thread enqueues every device's kernels and collectives, executioncontext.c
:185-201, synch/common.c:14-54) against its device time, on a ONE-GPU box where
every "device" is device 0 (cbx_init([0] * G)).

Two library builds, one per process (pass one):
  --variant peer       the product library, peer-read all-reduce (no RCCL: it
                       refuses a repeated device); G = 2, 4, 8.
  --variant fake-noop  the library linked against the test loopback collective
                       with FAKE_RCCL_NOOP=1: every ncclAllReduce returns at
                       once and moves nothing, so the numbers are the host
                       cost of everything BUT RCCL's own enqueue (which the
                       per-rank real-RCCL rehearsal measures); G = 1 (forced
                       split), 2, 4, 8 at 1 and 8 buckets, pipeline modes 0/1.
Each at enqueue_threads 0 (one thread, the reference's) and 1 (one thread per
device, cbx_set_enqueue_threads).  Per configuration: the median host time of one step (lockAny + synchronise +
unlockAny) enqueued on an idle GPU, the same back to back over the timed
steps, and the device's step (HIP events; on one GPU every device's work
shares the card, so it is G x a real GPU's).  JSON lines on stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(G, buckets, mode, peer, threads, steps=20, warmup=5, force_split=False):
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0] * G)
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setModelManager(8, SYNC_BSP)
    if force_split:
        g.set_force_split(True)
    if peer:
        g.set_allreduce_algorithm(_lib.ALLREDUCE_PEER)
    g.set_bucket_elements((1 << 62) if buckets == 1 else -(-n // buckets))
    g.set_enqueue_threads(threads)
    g.set_pipeline_mode(mode)
    g.fill_synthetic(1)
    g.set_timing(True)
    clock = 0

    def step():
        nonlocal clock
        clock += 1
        g.lockAny()
        g.synchronise(0, clock, 0, False)
        g.unlockAny()

    for _ in range(warmup):
        step()
    g.wait()
    idle = []
    for _ in range(10):
        g.wait()
        t0 = time.perf_counter()
        step()
        idle.append((time.perf_counter() - t0) * 1e3)
    g.wait()
    timed = []
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        step()
        timed.append((time.perf_counter() - h0) * 1e3)
    g.wait()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    dev = statistics.median(g.timing_history(_lib.T_STEP)[-steps:])
    kern = [x for x in g.timing_history(_lib.T_KERNEL)[-steps:] if x > 0]
    g.free()
    return {"G": G, "enqueue_threads": threads, "buckets": buckets if not peer else None, "pipeline_mode": mode if not peer else None,
            "form": "peer" if peer else "rccl-noop", "host_enqueue_ms_idle_gpu": round(statistics.median(idle), 4),
            "host_enqueue_ms_back_to_back": round(statistics.median(timed), 4),
            "device_step_ms_one_gpu": round(dev, 4), "wall_ms_per_step": round(wall, 4),
            "kernel_a_ms_per_step_device0": round(statistics.mean(kern), 4) if kern else None}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", choices=["peer", "fake-noop"], required=True)
    p.add_argument("--gs", default="1,2,4,8")
    a = p.parse_args()
    if a.variant == "fake-noop":
        os.environ["FAKE_RCCL_NOOP"] = "1"
        from crossbow_amd import _lib
        _lib.load(os.path.join(ROOT, "tests", "native", "libcrossbow_sma_fakerccl.so"))
    for G in (int(x) for x in a.gs.split(",")):
        for threads in ((0,) if G == 1 else (0, 1)):
            if a.variant == "peer":
                if G > 1:
                    print(json.dumps(run(G, 1, 0, True, threads)), flush=True)
                continue
            for buckets in (1, 8):
                for mode in ((0,) if buckets == 1 else (0, 1)):
                    print(json.dumps(run(G, buckets, mode, False, threads, force_split=G == 1)), flush=True)


if __name__ == "__main__":
    main()
