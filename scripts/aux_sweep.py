#!/usr/bin/env python3
"""Launch-geometry sweep of the per-task kernels on one MI355X (ResNet-50
parameters): the fused SMA replica optimiser step (kernels/optimisers/sma.cu,
reads w, g, last; writes s, w, g, last: 28n B with momentum and weight decay)
and the synchronous-SGD task step + barrier (synchronoussgd.cu / .c).

Every (block, unroll, waves-per-CU cap) is timed interleaved over rounds on
the same buffers (box-to-box variance is several percent; only within-run
comparisons count).  Optimiser: torch events around 8 back-to-back launches
on one stream.  S-SGD: host wall time of 8 task steps + one barrier, drained.
Writes gpurun_out/aux_sweep.json.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [(64, 1, -1), (128, 1, -1), (128, 1, 0), (64, 1, 4), (64, 1, 8), (64, 1, 12), (64, 2, 2), (64, 2, 3), (64, 2, 4),
           (64, 2, 6), (128, 2, 4), (128, 2, 8), (256, 1, 0), (256, 1, 8), (512, 1, 0)]


def make(update, R):
    from crossbow_amd import SYNC_BSP, TheGPU
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(update)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setWeightDecay(1e-4)
    g.setLearningRateDecayPolicyMultiStep(0.1, 0.1, 0, [1 << 30])
    g.setModelWorkPerClock(R)
    g.setModelManager(R, SYNC_BSP)
    g.fill_synthetic(20190701)
    return g, n


def main():
    import torch
    from crossbow_amd import UPDATE_SMA, UPDATE_WORKER
    rounds, R = 3, 8
    res = {}
    g, n = make(UPDATE_SMA, R)
    stream = torch.cuda.Stream()
    task = 0
    for _ in range(rounds):
        for cfg in CONFIGS:
            g.set_aux_kernel_config(*cfg)
            with torch.cuda.stream(stream):
                for i in range(R):
                    g.replica_optimise(i, task, stream.cuda_stream)
                    task += 1
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(2):
                    for i in range(R):
                        g.replica_optimise(i, task, stream.cuda_stream)
                        task += 1
                e1.record(stream)
            e1.synchronize()
            g.wait()
            res.setdefault(("optimise",) + cfg, []).append(e0.elapsed_time(e1) / (2 * R))
    g.free()

    g, n = make(UPDATE_WORKER, R)
    clock = 0
    for _ in range(rounds):
        for cfg in CONFIGS:
            g.set_aux_kernel_config(*cfg)
            samples = []
            for rep in range(4):
                g.wait()
                t0 = time.perf_counter()
                for i in range(R):
                    g.replica_optimise(i, task, None)
                    task += 1
                clock += 1
                g.lockAny()
                g.synchronise(0, clock, 0, False)
                g.unlockAny()
                g.wait()
                if rep:
                    samples.append((time.perf_counter() - t0) * 1e3)
            res.setdefault(("ssgd_clock",) + cfg, []).append(statistics.median(samples))
    g.free()

    nbytes = {"optimise": 28 * n, "ssgd_clock": R * 20 * n + (16 + 4 * R) * n}
    rows = []
    for key, ms in res.items():
        med = statistics.median(ms)
        row = dict(kernel=key[0], block=key[1], unroll=key[2], cap=key[3], ms=round(med, 4),
                   per_round=[round(x, 4) for x in ms], GBs=round(nbytes[key[0]] / (med * 1e-3) / 1e9, 1))
        rows.append(row)
        print(json.dumps(row), flush=True)
    best = {k: min((r for r in rows if r["kernel"] == k), key=lambda r: r["ms"]) for k in nbytes}
    for b in best.values():
        print("BEST", json.dumps(b), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "aux_sweep.json"), "w") as f:
        json.dump(dict(rows=rows, best=best), f, indent=1)


if __name__ == "__main__":
    main()
