#!/usr/bin/env python3
"""The G > 1 bucket pipeline forced at G = 1 (one-rank RCCL) on one MI355X:
ms per step by bucket count, pipeline mode and cross-step wait stride,
ResNet-50, R = 8, momentum 0.9 (wall clock over back-to-back steps,
interleaved passes, best pass kept), with timing on ("spans": the bench's
setting, per-dispatch span events) and off ("notiming").  A repeated variant
gets a context of its own (a placement check).  JSON lines on stdout.

Round 3 ran it with experiment toggles (kernels A on one or two streams;
library streams from the shared hardware-queue pool, on CU-mask queues of
their own, or at high priority): profiles/r03/pipeline_streams_ab.json (as scripts/two_a_ab.py).  The
library now runs kernels A on two streams; its four streams are plain
non-blocking streams created together, each on a hardware queue of its own
(GPU_MAX_HW_QUEUES 16; CU-mask streams synchronise with the null stream, so
they were not kept), and the toggles are gone."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make(variant):
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setModelManager(8, SYNC_BSP)
    g.set_force_split(True)
    g.fill_synthetic(1)
    g.set_timing(True)
    return g, n


def timed(g, steps=30, warmup=5):
    clock = [0]

    def step():
        clock[0] += 1
        g.lockAny()
        g.synchronise(0, clock[0], 0, False)
        g.unlockAny()
    for _ in range(warmup):
        step()
    g.wait()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    g.wait()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="spans,notiming")
    ap.add_argument("--configs", default="1/0/1,4/1/1,8/1/1,8/1/2,8/1/4,8/0/1")
    ap.add_argument("--passes", type=int, default=3)
    a = ap.parse_args()
    variants = a.variants.split(",")  # a repeated variant gets a context of its own (placement check)
    ctx = {}
    for i, v in enumerate(variants):
        name = v if v not in ctx else f"{v}#{i}"
        variants[i] = name
        ctx[name] = make(v)
        if "notiming" in v:
            ctx[name][0].set_timing(False)
    configs = [tuple(int(x) for x in c.split("/")) for c in a.configs.split(",")]
    best = {}
    for _ in range(a.passes):
        for nb, mode, stride in configs:
            for two in variants:
                g, n = ctx[two]
                g.set_bucket_elements((1 << 62) if nb == 1 else -(-n // nb))
                g.set_pipeline_mode(mode)
                g.set_cross_wait_stride(stride)
                ms = timed(g)
                key = (nb, mode, stride, two)
                best[key] = min(ms, best.get(key, ms))
    for (nb, mode, stride, two), ms in sorted(best.items()):
        print(json.dumps({"buckets": nb, "mode": mode, "stride": stride, "variant": two,
                          "ms_per_step": round(ms, 4)}), flush=True)
    for g, _ in ctx.values():
        g.free()


if __name__ == "__main__":
    main()
