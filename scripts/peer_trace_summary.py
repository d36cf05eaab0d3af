#!/usr/bin/env python3
"""Where the time of a bucketed peer-read step goes, from a rocprofv3 kernel
trace of scripts/peer_sweep.py --passes 1 --gap-ms 50: the trace is split at
idle gaps longer than 20 ms into one segment per configuration (in the order
peer_sweep.py printed), and per segment, over its timed steps (the last
`steps` of warmup + steps), per step: the wall time (first kernel start to
last kernel end), the GPU's busy time (union of every kernel's interval),
idle = wall - busy, and per kernel kind (A = sma_accumulate, R =
sma_peer_reduce, B = sma_peer_apply) the summed durations and launches.
Usage: python scripts/peer_trace_summary.py <kernel_trace.csv> <peer_sweep stdout>"""
from __future__ import annotations

import csv
import json
import statistics
import sys


def union(iv):
    iv = sorted(iv)
    tot, (lo, hi) = 0, iv[0]
    for a, b in iv[1:]:
        if a > hi:
            tot += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    return tot + hi - lo


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sma_" in r["Kernel_Name"]]
    meta = [json.loads(ln) for ln in open(sys.argv[2]) if ln.startswith('{"order"')][0]
    order, steps, warm = meta["order"], meta["steps"], meta["warmup"]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 "A" if "accumulate" in r["Kernel_Name"] else "R" if "peer_reduce" in r["Kernel_Name"]
                 else "B" if "peer_apply" in r["Kernel_Name"] else "other") for r in rows)
    segs, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[0] - max(x[1] for x in cur[-64:]) > 20_000_000:
            segs.append(cur)
            cur = []
        cur.append(e)
    segs.append(cur)
    segs = segs[-len(order):]  # the setup's kernels (fill) come first
    for key, seg in zip(order, segs):
        nb = key[0]
        na = sum(1 for e in seg if e[2] == "A")
        per_step = max(1, na // (warm + steps))  # kernel-A launches per step (G devices x buckets)
        a_idx = [i for i, e in enumerate(seg) if e[2] == "A"]
        # the timed steps: from the first A of step `warm` on
        start_i = a_idx[warm * per_step] if len(a_idx) > warm * per_step else 0
        timed = seg[start_i:]
        wall = (max(e[1] for e in timed) - timed[0][0]) / 1e3 / steps
        busy = union([(e[0], e[1]) for e in timed]) / 1e3 / steps
        kinds = {}
        for k in ("A", "R", "B"):
            d = [e[1] - e[0] for e in timed if e[2] == k]
            kinds[k] = {"sum_us_per_step": round(sum(d) / 1e3 / steps, 1), "launches_per_step": len(d) // steps,
                        "median_us": round(statistics.median(d) / 1e3, 1) if d else None}
        print(json.dumps({"config": dict(zip(("buckets", "mode", "stride", "group", "threads", "variant"), key)),
                          "wall_us_per_step": round(wall, 1), "busy_us_per_step": round(busy, 1),
                          "idle_us_per_step": round(wall - busy, 1), "kernels": kinds}), flush=True)


if __name__ == "__main__":
    main()
