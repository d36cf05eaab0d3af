#!/usr/bin/env python3
"""Host-side cost of enqueuing one synchronise() (lockAny + synchronise +
unlockAny) against its device time, for the fused step and the bucketed split
pipeline (one-rank RCCL at G = 1).  If the host needs longer per step than the
device, the device idles between kernels and the step is host-bound.
Writes one JSON line per configuration."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(split, bucket_elems, steps=40):
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setModelManager(8, SYNC_BSP)
    if split:
        g.set_force_split(True)
    g.set_bucket_elements(bucket_elems)
    g.fill_synthetic(1)
    g.set_timing(True)
    clock = 0
    host = []
    for k in range(steps + 5):
        clock += 1
        t0 = time.perf_counter()
        g.lockAny()
        g.synchronise(0, clock, 0, False)
        g.unlockAny()
        if k >= 5:
            host.append((time.perf_counter() - t0) * 1e3)
    g.wait()
    t0 = time.perf_counter()
    for _ in range(steps):
        clock += 1
        g.lockAny()
        g.synchronise(0, clock, 0, False)
        g.unlockAny()
    g.wait()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    dev = statistics.median(g.timing_history(_lib.T_STEP)[-steps:])
    g.free()
    return {"split": split, "bucket_elems": bucket_elems, "host_enqueue_ms": round(statistics.median(host), 4),
            "device_step_ms": round(dev, 4), "wall_ms_per_step": round(wall, 4)}


def main():
    for split, be in ((False, 0), (True, 0), (True, 3_200_000), (True, 6_400_000), (True, 1_600_000)):
        print(json.dumps(run(split, be)), flush=True)


if __name__ == "__main__":
    main()
