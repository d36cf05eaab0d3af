#!/usr/bin/env python3
"""Where C2's time goes: the fused SMA kernel (R = 4, mu = 0, LeNet's shape)
timed over a range of model sizes, HBM-resident (contexts used in rotation so
the working set never fits the 256 MB Infinity Cache), then fitted to

    t(n) = t0 + bytes(n) / BW        bytes(n) = (12 R + 8) n = 56 n

BW is the steady-state streaming rate and t0 the fixed cost of a launch
(the ramp of the first waves' loads plus the drain of the last stores; the
dispatch gap between launches is outside the HIP-event span).  If BW is at the
big kernels' HBM rate, C2 (n = 1,111,946: 62 MB) is latency-bound and its
0.44 fraction is t0, not a bandwidth problem.

Contexts run one at a time (a host wait after each step): each context has
its own stream, and overlapping launches would share HBM and inflate every
HIP-event span.  Writes gpurun_out/c2_latency.json; run it under rocprofv3 --kernel-trace to
see the dispatch gaps as well.
"""
from __future__ import annotations

import json
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_LENET = 1_111_946
R = 4


def make(n):
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU
    g = TheGPU()
    g.init([0])
    g.setModel(1, 4 * n)
    g.setModelVariable(0, 1, [n], 4 * n)
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.0, 0)
    g.setModelManager(R, SYNC_BSP)
    g.fill_synthetic(20190701)
    g.set_timing(True)
    return g


def main():
    from crossbow_amd import _lib
    steps = 20
    rows = []
    for scale in (0.25, 0.5, 1, 2, 4, 8, 16):
        n = int(N_LENET * scale)
        nbytes = (12 * R + 8) * n
        k = max(2, math.ceil(720e6 / nbytes))  # rotate past the 256 MB Infinity Cache
        gs = [make(n) for _ in range(k)]
        clock = 0
        for rep in range(steps + 3):
            for g in gs:
                clock += 1
                g.lockAny()
                g.synchronise(0, clock, 0, False)
                g.unlockAny()
                g.wait()  # one context at a time: the contexts' streams would otherwise overlap in HBM
        for g in gs:
            g.wait()
        ms = [t for g in gs for t in g.timing_history(_lib.T_KERNEL)[-steps:]]
        med = statistics.median(ms)
        rows.append({"scale": scale, "n": n, "bytes": nbytes, "contexts": k, "kernel_ms_median": round(med, 5),
                     "GBs": round(nbytes / (med * 1e-3) / 1e9, 1)})
        print(json.dumps(rows[-1]), flush=True)
        for g in gs:
            g.free()
    # least-squares fit t = t0 + bytes / BW over every size
    xs = [r["bytes"] for r in rows]
    ys = [r["kernel_ms_median"] * 1e-3 for r in rows]
    mx, my = statistics.mean(xs), statistics.mean(ys)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    t0 = my - slope * mx
    c2 = next(r for r in rows if r["scale"] == 1)
    fit = {"t0_us": round(t0 * 1e6, 2), "steady_GBs": round(1 / slope / 1e9, 1),
           "c2_kernel_us": round(c2["kernel_ms_median"] * 1e3, 2),
           "c2_streaming_us_at_steady_rate": round(c2["bytes"] * slope * 1e6, 2),
           "c2_fixed_share": round(t0 / (c2["kernel_ms_median"] * 1e-3), 3)}
    print(json.dumps({"fit": fit}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "c2_latency.json"), "w") as f:
        json.dump({"rows": rows, "fit": fit}, f, indent=1)


if __name__ == "__main__":
    main()
