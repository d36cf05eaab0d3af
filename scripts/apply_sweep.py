#!/usr/bin/env python3
"""Launch shapes for kernel B of the split SMA path (sma_apply_kernel: reads
D, z, last; writes z, last; 20n bytes) on ResNet-50 (n = 25,557,032, R = 8,
mu 0.9), one bucket in order on the sync stream so that HIP events time
kernel B alone (CBX_T_APPLY), interleaved over rounds.  Kernel A is timed in
the same steps as a control.  Writes gpurun_out/apply_sweep.json."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [(64, 2, -1), (64, 1, -1), (64, 1, 2), (64, 1, 4), (64, 1, 8), (64, 2, 2), (64, 2, 3), (64, 2, 4),
          (64, 2, 6), (64, 4, -1), (128, 2, 4), (128, 2, 8), (256, 1, 8), (256, 1, 16), (256, 2, 8), (256, 1, 0)]


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    R, steps, rounds = 8, 10, 3
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setModelManager(R, SYNC_BSP)
    g.set_force_split(True)
    g.set_bucket_elements(1 << 62)
    g.fill_synthetic(1)
    g.set_timing(True)
    clock = 0
    res = {s: [] for s in SHAPES}
    ctl = {s: [] for s in SHAPES}
    for _ in range(rounds):
        for shape in SHAPES:
            g.set_apply_kernel_config(*shape)
            for _ in range(2 + steps):
                clock += 1
                g.lockAny()
                g.synchronise(0, clock, 0, False)
                g.unlockAny()
            g.wait()
            res[shape].append(statistics.median(g.timing_history(_lib.T_APPLY)[-steps:]))
            ctl[shape].append(statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
    g.free()
    nbytes = 20 * n
    out = []
    for (b, u, c), ms in res.items():
        med = statistics.median(ms)
        row = dict(kernel="sma_apply", block=b, unroll=u, cap=c, us=round(med * 1e3, 1),
                   GBs=round(nbytes / med / 1e6, 1), rounds_us=[round(x * 1e3, 1) for x in ms],
                   kernel_a_us=round(statistics.median(ctl[(b, u, c)]) * 1e3, 1))
        out.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "apply_sweep.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
