#!/usr/bin/env python3
"""Bucket count of the pipelined host-staged step (cbx_synchronise_staged) on
C3 (ResNet-50, R = 8, mu 0.9): HIP-event step time, uploads and downloads per
bucket count, beside the unpipelined stage_in + synchronise + stage_out.
Writes gpurun_out/staged_sweep.jsonl."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    R = 8
    g.setModelManager(R, SYNC_BSP)
    g.fill_synthetic(20190701)
    g.set_timing(True)
    step_bytes = (12 * R + 16) * n
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", "staged_sweep.jsonl"), "w")
    clock = 0

    def emit(rec):
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")

    ser = []
    for _ in range(4):
        clock += 1
        g.stage_in()
        g.lockAny()
        g.synchronise(0, clock, 0, False)
        g.unlockAny()
        g.stage_out()
        g.wait()
        t = g.last_timing(0)
        ser.append(t[_lib.T_H2D] + t[_lib.T_KERNEL] + t[_lib.T_D2H])
    ms = statistics.median(ser[1:])
    emit({"mode": "serial", "ms": round(ms, 3), "GBs": round(step_bytes / ms / 1e6, 2)})
    for b in (1, 2, 4, 8, 16, 32, 64, 128):
        ts = []
        for _ in range(4):
            clock += 1
            g.lockAny()
            g.synchronise_staged(0, clock, 0, b)
            g.unlockAny()
            g.wait()
            ts.append(g.last_timing(0))
        ts = ts[1:]
        ms = statistics.median(t[_lib.T_STEP] for t in ts)
        emit({"mode": "pipelined", "buckets": b, "ms": round(ms, 3), "GBs": round(step_bytes / ms / 1e6, 2),
              "h2d_ms": round(statistics.median(t[_lib.T_H2D] for t in ts), 3),
              "d2h_ms": round(statistics.median(t[_lib.T_D2H] for t in ts), 3)})
    g.free()


if __name__ == "__main__":
    main()
