#!/usr/bin/env python3
"""Kernel rates of every BASELINE.json configuration on one MI355X.

The bench line is C3 only.  This script times the SMA kernels of the other
configurations on one GPU, with HIP events (the library's timing ring), so
DESIGN.md can quote absolute GB/s and the HBM fraction for each:

  C2  LeNet (n = 1,111,946), R = 4, alpha 0.1, mu 0   fused.  Its working set
      (62 MB) fits the 256 MB Infinity Cache, so it is timed twice: one
      context (cache-resident, labelled so) and 8 contexts used in rotation
      (720 MB, HBM), as BASELINE.md 2.2 asks.
  C3  ResNet-50 (n = 25,557,032), R = 8, mu 0.9       fused (the bench line)
  C4  ResNet-50, R = 2 per GPU, mu 0.9                fused (G = 1) and the
      G > 1 kernels A and B (one-rank all-reduce)
  C5  ResNet-50, R = 4 per GPU, mu 0.9                kernels A and B
Writes gpurun_out/configs.json.
"""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def make(model, R, mom, split):
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU
    from crossbow_amd.variables import MODELS, register
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS[model]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(mom, 0)
    g.setModelManager(R, SYNC_BSP)
    if split:
        g.set_force_split(True)
        g.set_bucket_elements(1 << 62)  # one bucket, in order: kernels timed apart
    g.fill_synthetic(20190701)
    g.set_timing(True)
    return g, n


def run(gs, steps):
    """`steps` barrier steps on every context in rotation.  Each context has
    its own sync stream, so with several contexts each step is waited for
    before the next context's starts: otherwise two contexts' kernels run at
    once, share HBM, and each launch's HIP-event span is inflated (the
    round-1 C2 "rotated" figure, 3.5 TB/s, was that artefact)."""
    clock = 0
    for _ in range(steps):
        for g in gs:
            clock += 1
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
            if len(gs) > 1:
                g.wait()
    for g in gs:
        g.wait()


def rate(nbytes, ms):
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"ms_median": round(ms, 4), "GBs": round(gbs, 1), "frac_of_8TBs": round(gbs / PEAK, 4)}


def main():
    from crossbow_amd import _lib
    out = {}
    steps = 30

    # C2: LeNet, fused, cache-resident (one context) and rotated (8 contexts).
    n_l = 1_111_946
    b2 = (12 * 4 + 8) * n_l
    g, _ = make("lenet", 4, 0.0, False)
    run([g], 5)
    run([g], steps)
    out["C2_lenet_R4_fused_cache_resident"] = rate(b2, statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
    g.free()
    gs = [make("lenet", 4, 0.0, False)[0] for _ in range(8)]
    run(gs, 3)
    run(gs, steps)
    ks = [statistics.median(x.timing_history(_lib.T_KERNEL)[-steps:]) for x in gs]
    out["C2_lenet_R4_fused_8_rotated_contexts"] = rate(b2, statistics.median(ks))
    for x in gs:
        x.free()

    n = 25_557_032
    for R, label in ((8, "C3"), (2, "C4"), (4, "C5")):
        if R in (8, 2):
            g, _ = make("resnet50", R, 0.9, False)
            run([g], 5)
            run([g], steps)
            out[f"{label}_resnet50_R{R}_fused"] = rate((12 * R + 16) * n,
                                                       statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]))
            g.free()
        if R in (2, 4, 8):
            g, _ = make("resnet50", R, 0.9, True)
            run([g], 5)
            run([g], steps)
            ka = statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:])
            kb = statistics.median(g.timing_history(_lib.T_APPLY)[-steps:])
            ar = statistics.median(g.timing_history(_lib.T_ALLREDUCE)[-steps:])
            out[f"{label}_resnet50_R{R}_kernelA"] = rate((12 * R + 8) * n, ka)
            out[f"{label}_resnet50_R{R}_kernelB"] = rate(20 * n, kb)
            out[f"{label}_resnet50_R{R}_one_rank_allreduce_ms"] = round(ar, 4)
            g.free()
    for k, v in out.items():
        print(k, json.dumps(v), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "configs.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
