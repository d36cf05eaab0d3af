#!/usr/bin/env python3
"""Read the per-rank kernel traces of scripts/trace_real_rccl.sh (every rank on
one GPU, so one clock) and report how the collective overlapped the SMA
kernels: per rank, the time kernels A and B ran, the time RCCL kernels ran,
and how much of the RCCL time ran while a kernel A or B of the same rank was
running (the pipeline's overlap); plus the per-step span of the last steps.

Usage: pipeline_overlap.py TRACE_DIR  (prints JSON)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys


def kind(name: str) -> str:
    if "sma_accumulate_kernel" in name:
        return "A"
    if "sma_apply_kernel" in name:
        return "B"
    if "sma_shard_momentum_kernel" in name:
        return "M"
    low = name.lower()
    if "nccl" in low or "rccl" in low:
        return "rccl"
    return "other"


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    """Total length of the intersection of two interval unions."""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d = sys.argv[1]
    ranks = {}
    for path in sorted(glob.glob(os.path.join(d, "rank*", "**", "*kernel_trace.csv"), recursive=True)):
        r = int(path.split(os.sep + "rank")[1].split(os.sep)[0])
        rows = []
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                rows.append((kind(row["Kernel_Name"]), int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
        ranks[r] = rows
    out = {}
    for r, rows in sorted(ranks.items()):
        sma = [(s, e) for k, s, e in rows if k in ("A", "B", "M")]
        a_starts = sorted(s for k, s, e in rows if k == "A")
        # the last three steps: from the first kernel A of step 4 to the end
        nb = max(1, sum(1 for k, _, _ in rows if k == "A") // 6)
        t_from = a_starts[3 * nb] if len(a_starts) > 3 * nb else a_starts[0]
        win = [(k, max(s, t_from), e) for k, s, e in rows if e > t_from]
        by = {}
        for k, s, e in win:
            by.setdefault(k, []).append((s, e))
        u = {k: union(v) for k, v in by.items()}
        busy = {k: sum(e - s for s, e in v) / 1e3 for k, v in u.items()}
        sma_u = union([(s, e) for k, s, e in win if k in ("A", "B", "M")])
        rccl_u = u.get("rccl", [])
        span = (max(e for _, _, e in win) - t_from) / 1e3 if win else 0.0
        out[f"rank{r}"] = {
            "buckets_per_step": nb,
            "kernels": {k: len(v) for k, v in by.items()},
            "busy_us_last3": {k: round(v, 1) for k, v in busy.items()},
            "rccl_us_beside_A_or_B": round(overlap(sma_u, rccl_u) / 1e3, 1),
            "span_us_last3": round(span, 1),
            "total_sma_kernels": len(sma),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
