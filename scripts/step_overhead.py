#!/usr/bin/env python3
"""Wall time per synchronise() of the fused C3 step (ResNet-50, R = 8, mu 0.9)
with timing off and on, against the kernel time, over 200 back-to-back steps:
what a step costs the stream beyond its kernel."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0])
    register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setModelManager(8, SYNC_BSP)
    g.fill_synthetic(1)
    clock = 0
    res = {}
    for rnd in range(3):
        for timing in (False, True):
            g.set_timing(timing)
            for _ in range(10):
                clock += 1
                g.lockAny(); g.synchronise(0, clock, 0, False); g.unlockAny()
            g.wait()
            steps = 200
            t0 = time.perf_counter()
            for _ in range(steps):
                clock += 1
                g.lockAny(); g.synchronise(0, clock, 0, False); g.unlockAny()
            g.wait()
            res.setdefault(timing, []).append((time.perf_counter() - t0) * 1e3 / steps)
            if timing:
                res.setdefault("kernel", []).append(statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
    print(json.dumps({"timing_off_ms_per_step": [round(x, 4) for x in res[False]],
                      "timing_on_ms_per_step": [round(x, 4) for x in res[True]],
                      "kernel_ms": [round(x, 4) for x in res["kernel"]]}), flush=True)
    g.free()


if __name__ == "__main__":
    main()
