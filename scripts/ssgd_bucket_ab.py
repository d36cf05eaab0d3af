#!/usr/bin/env python3
"""S-SGD (update model WORKER) barrier on the split path, one bucket vs
4/8/16 buckets (all-reduce of bucket k+1 on its own stream beside the apply
kernel of bucket k): ResNet-50, R = 8, momentum 0.9, one GPU, one-rank
all-reduce (force split), interleaved over 5 rounds, wall ms per barrier.
Writes gpurun_out/ssgd_bucket_ab.json."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_WORKER, TheGPU
    from crossbow_amd.variables import MODELS, register
    R, steps, rounds = 8, 30, 5
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_WORKER)
    g.setMomentum(0.9, 0)
    g.setModelWorkPerClock(R)
    g.setModelManager(R, SYNC_BSP)
    g.set_force_split(True)
    g.fill_synthetic(1)
    clock = 0

    def step():
        nonlocal clock
        clock += 1
        g.lockAny()
        g.synchronise(0, clock, 0, False)
        g.unlockAny()

    res = {}
    for _ in range(rounds):
        for nb in (1, 4, 8, 16):
            g.set_bucket_elements(1 << 62 if nb == 1 else -(-n // nb))
            for _ in range(3):
                step()
            g.wait()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            g.wait()
            res.setdefault(nb, []).append((time.perf_counter() - t0) * 1e3 / steps)
    g.free()
    out = [dict(buckets=nb, wall_ms=round(statistics.median(v), 4), rounds=[round(x, 4) for x in v])
           for nb, v in sorted(res.items())]
    for row in out:
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ssgd_bucket_ab.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
