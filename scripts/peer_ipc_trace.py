#!/usr/bin/env python3
"""Where the per-rank peer-read step's time goes, from the per-rank kernel
traces of scripts/trace_real_rccl.sh with ALGO=1 (every rank on one GPU, so
one clock).  Per bucket k of the last three steps:

  a_to_r: from the LAST rank's kernel A(k) end to this rank's R(k) start
          (the cross-process hand-off through the flag page, plus any queue
          wait), and
  r_to_b: from the last rank's R(k) end to this rank's B(k) start,

and per step the wall time, the GPU's busy time (union of every rank's
kernels) and the idle rest.  Kernels are matched by name (A sma_accumulate,
R sma_peer_reduce, B sma_peer_apply) and by their order within a rank.
Usage: peer_ipc_trace.py TRACE_DIR BUCKETS  (prints JSON)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys


def kind(name: str) -> str | None:
    if "sma_accumulate" in name:
        return "A"
    if "sma_peer_reduce" in name:
        return "R"
    if "sma_peer_apply" in name:
        return "B"
    return None


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
    d, nb = sys.argv[1], int(sys.argv[2])
    ranks = {}
    for path in sorted(glob.glob(os.path.join(d, "rank*", "**", "*kernel_trace.csv"), recursive=True)):
        r = int(path.split(os.sep + "rank")[1].split(os.sep)[0])
        ev = {"A": [], "R": [], "B": []}
        for row in csv.DictReader(open(path, newline="")):
            k = kind(row["Kernel_Name"])
            if k:
                ev[k].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
        for k in ev:
            ev[k].sort()
        ranks[r] = ev
    steps = min(len(ev["B"]) for ev in ranks.values()) // nb
    out = {"buckets": nb, "ranks": len(ranks), "steps_traced": steps, "per_step": [], "handoff_us": {}}
    a_to_r, r_to_b = [], []
    for st in range(max(0, steps - 3), steps):
        sl = slice(st * nb, (st + 1) * nb)
        allk = [iv for ev in ranks.values() for k in ev for iv in ev[k][sl]]
        wall = max(e for _, e in allk) - min(s for s, _ in allk)
        busy = union(allk)
        out["per_step"].append({"step": st, "wall_us": round(wall / 1e3, 1), "busy_us": round(busy / 1e3, 1),
                                "idle_us": round((wall - busy) / 1e3, 1)})
        for b in range(nb):
            i = st * nb + b
            last_a = max(ev["A"][i][1] for ev in ranks.values())
            last_r = max(ev["R"][i][1] for ev in ranks.values())
            for ev in ranks.values():
                a_to_r.append((ev["R"][i][0] - last_a) / 1e3)
                r_to_b.append((ev["B"][i][0] - last_r) / 1e3)
    for name, v in (("a_to_r", a_to_r), ("r_to_b", r_to_b)):
        if v:
            out["handoff_us"][name] = {"median": round(statistics.median(v), 1), "min": round(min(v), 1),
                                       "max": round(max(v), 1)}
    dur = {k: statistics.median((e - s) / 1e3 for ev in ranks.values() for s, e in ev[k]) for k in ("A", "R", "B")}
    out["kernel_median_us"] = {k: round(v, 1) for k, v in dur.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
