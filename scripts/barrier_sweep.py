#!/usr/bin/env python3
"""Launch shapes for the write-heavy barrier kernels of the DEFAULT and S-SGD
update models (ResNet-50, R = 8): broadcast_kernel (1 read + 8 writes) and
ssgd_apply_kernel (3 reads + 11 writes), HIP-event kernel time, interleaved
over rounds.  Writes gpurun_out/barrier_sweep.json."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [(64, 1, -1), (64, 1, 2), (64, 1, 3), (64, 1, 4), (64, 2, -1), (64, 2, 2), (64, 2, 3), (64, 2, 4),
          (128, 2, 4), (256, 1, 8)]


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_DEFAULT, UPDATE_WORKER, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    R, steps, rounds = 8, 10, 3
    n = 25_557_032
    out = {}
    for utype, name, nbytes in ((UPDATE_DEFAULT, "broadcast", (4 + 4 * R) * n),
                                (UPDATE_WORKER, "ssgd_apply", (12 + 4 + 4 + 4 + 4 * R) * n)):
        g = TheGPU()
        g.init([0])
        register(g, MODELS["resnet50"]())
        g.setUpdateModelType(utype)
        g.setMomentum(0.9, 0)
        g.setModelWorkPerClock(R)
        g.setModelManager(R, SYNC_BSP)
        g.fill_synthetic(1)
        g.set_timing(True)
        clock = 0
        res = {s: [] for s in SHAPES}
        for _ in range(rounds):
            for shape in SHAPES:
                g.set_barrier_kernel_config(*shape)
                for _ in range(2 + steps):
                    clock += 1
                    g.lockAny()
                    g.synchronise(0, clock, 0, False)
                    g.unlockAny()
                g.wait()
                res[shape].append(statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
        g.free()
        for (b, u, c), ms in res.items():
            med = statistics.median(ms)
            row = dict(kernel=name, block=b, unroll=u, cap=c, us=round(med * 1e3, 1), GBs=round(nbytes / med / 1e6, 1))
            out.setdefault(name, []).append(row)
            print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "barrier_sweep.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
