#!/usr/bin/env python3
"""Occupancy-cap sweep per SMA kernel and replica count, on one MI355X.

For every (kernel, R) the library can run -- the fused step, kernel A and
kernel B of the split pipeline -- time each waves-per-CU cap, interleaved over
rounds (box-to-box variance is several percent, so only within-run
comparisons count).  ResNet-50 parameters, momentum 0.9.  Writes
gpurun_out/occupancy.json with the best cap per (kernel, R).
"""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CAPS = [-1, 0, 2, 3, 4, 6, 8, 12]


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    steps, rounds = 12, 3
    n = 25_557_032
    res = {}
    for R in (1, 2, 4, 8):
        for split in (False, True):
            g = TheGPU()
            g.init([0])
            register(g, MODELS["resnet50"]())
            g.setUpdateModelType(UPDATE_SMA)
            g.setEamsgdAlpha(0.1)
            g.setMomentum(0.9, 0)
            g.setModelManager(R, SYNC_BSP)
            if split:
                g.set_force_split(True)
                g.set_bucket_elements(1 << 62)
            g.fill_synthetic(20190701)
            g.set_timing(True)
            clock = 0
            for _ in range(rounds):
                for cap in CAPS:
                    g.set_kernel_occupancy(cap)
                    for _ in range(3 + steps):
                        clock += 1
                        g.lockAny()
                        g.synchronise(0, clock, 0, False)
                        g.unlockAny()
                    g.wait()
                    if split:
                        res.setdefault(("A", R, cap), []).append(
                            statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
                        res.setdefault(("B", R, cap), []).append(
                            statistics.median(g.timing_history(_lib.T_APPLY)[-steps:]))
                    else:
                        res.setdefault(("fused", R, cap), []).append(
                            statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
            g.free()
    nbytes = {"fused": lambda R: (12 * R + 16) * n, "A": lambda R: (12 * R + 8) * n, "B": lambda R: 20 * n}
    out = {"rows": [], "best": {}}
    for (k, R, cap), ms in sorted(res.items()):
        med = statistics.median(ms)
        row = dict(kernel=k, R=R, cap=cap, ms=round(med, 4), GBs=round(nbytes[k](R) / (med * 1e-3) / 1e9, 1))
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    for k in ("fused", "A", "B"):
        for R in (1, 2, 4, 8):
            rows = [r for r in out["rows"] if r["kernel"] == k and r["R"] == R]
            best = min(rows, key=lambda r: r["ms"])
            out["best"][f"{k}/R{R}"] = best
            print("BEST", json.dumps(best), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "occupancy.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
