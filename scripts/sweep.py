#!/usr/bin/env python3
"""Launch-geometry sweep of the fused SMA kernel on one MI355X (C3 workload).

Runs every (block, blocks_per_cu, policy, unroll) combination in one process
on the same device-resident ResNet-50 buckets and prints the median kernel
time from HIP events; results go to gpurun_out/sweep.json.
"""
from __future__ import annotations

import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def interleaved(g, args, nbytes, m, rounds=3):
    from crossbow_amd import _lib
    # (block, unroll, waves-per-CU cap, workgroups per CU for a grid-stride launch; 0 = one trip)
    configs = [(64, 2, 2, 0), (64, 2, 3, 0), (64, 4, 2, 0), (64, 4, 3, 0), (64, 4, 4, 0), (128, 2, 4, 0),
               (128, 2, 6, 0), (64, 1, 3, 0), (128, 1, 6, 0), (64, 2, 2, 2), (64, 2, 3, 3), (64, 4, 2, 2),
               (128, 2, 4, 2)]
    res = {c: [] for c in configs}
    clock = 0
    for _ in range(rounds):
        for (block, unroll, occ, bpc) in configs:
            g.set_kernel_config(block, bpc, 1, unroll)
            g.set_kernel_occupancy(occ)
            for _ in range(5 + args.steps):
                clock += 1
                g.lockAny()
                g.synchronise(0, clock, 0, False)
                g.unlockAny()
            g.wait()
            res[(block, unroll, occ, bpc)].append(statistics.median(g.timing_history(_lib.T_KERNEL)[-args.steps:]))
    rows = []
    for (block, unroll, occ, bpc), ms in res.items():
        med = statistics.median(ms)
        row = dict(block=block, unroll=unroll, waves_per_cu_cap=occ, blocks_per_cu=bpc, kernel_ms=round(med, 4),
                   per_round=[round(x, 4) for x in ms],
                   GBs=round(nbytes / (med * 1e-3) / 1e9, 1))
        rows.append(row)
        print(json.dumps(row), flush=True)
    best = min(rows, key=lambda r: r["kernel_ms"])
    print("BEST", json.dumps(best), flush=True)
    tag = f"{args.model}_R{args.replicas}_m{m}_interleaved"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"sweep_{tag}.json"), "w") as f:
        json.dump(dict(rows=rows, best=best), f, indent=1)
    g.free()


def main():
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("--replicas", type=int, default=8)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--model", default="resnet50")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--split", action="store_true")
    p.add_argument("--quick", action="store_true")
    p.add_argument("--interleave", action="store_true",
                   help="a few promising configs, interleaved over several rounds (cancels drift)")
    args = p.parse_args()

    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register

    g = TheGPU()
    g.init([0])
    n = register(g, MODELS[args.model]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(args.momentum, 0)
    g.setModelManager(args.replicas, SYNC_BSP)
    if args.split:
        g.set_force_split(True)
    g.fill_synthetic(20190701)
    g.set_timing(True)
    m = 1 if args.momentum > 0 else 0
    nbytes = (12 * args.replicas + 8 + 8 * m) * n if not args.split else (12 * args.replicas + 8) * n

    if args.interleave:
        return interleaved(g, args, nbytes, m)
    blocks = [64, 128, 256] if not args.quick else [128]
    bpcs = [0, 4] if not args.quick else [0]
    policies = [0, 1]
    unrolls = [1] if args.quick else [1, 2]
    rows = []
    clock = 0
    for block, bpc, pol, un in itertools.product(blocks, bpcs, policies, unrolls):
        if block * un > 1024:
            continue
        g.set_kernel_config(block, bpc, pol, un)
        for _ in range(5 + args.steps):
            clock += 1
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
        g.wait()
        k = g.timing_history(_lib.T_KERNEL)[-args.steps:]
        med = statistics.median(k)
        row = dict(block=block, blocks_per_cu=bpc, policy=pol, unroll=un, kernel_ms=round(med, 4),
                   min_ms=round(min(k), 4), GBs=round(nbytes / (med * 1e-3) / 1e9, 1))
        rows.append(row)
        print(json.dumps(row), flush=True)
    best = min(rows, key=lambda r: r["kernel_ms"])
    print("BEST", json.dumps(best), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    tag = f"{args.model}_R{args.replicas}_m{m}{'_split' if args.split else ''}"
    with open(os.path.join(ROOT, "gpurun_out", f"sweep_{tag}.json"), "w") as f:
        json.dump(dict(n=n, bytes=nbytes, rows=rows, best=best), f, indent=1)
    g.free()


if __name__ == "__main__":
    main()
