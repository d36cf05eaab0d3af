#!/usr/bin/env python3
"""Per-step kernel busy time of the G > 1 bucket pipeline forced at G = 1,
from a rocprofv3 kernel trace of scripts/pipeline_sweep.py (one bucket, then
8 buckets in cross-step mode): dispatch durations summed and as the union of
their intervals (kernels A on two streams overlap).  Usage:
  python scripts/split_trace_summary.py <trace_kernel_trace.csv>"""
import csv, json, statistics as st, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sma_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(("A" if "accumulate" in r["Kernel_Name"] else "B"), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       int(r["Grid_Size_X"]), r["Queue_Id"]) for r in rows]
full = max(e[3] for e in ev if e[0] == "A")
def union(iv):
    iv = sorted(iv); tot = 0; lo, hi = iv[0]
    for a, b in iv[1:]:
        if a > hi: tot += hi - lo; lo, hi = a, b
        else: hi = max(hi, b)
    return tot + hi - lo
# one-bucket steps: full-grid A followed by full-grid B
A1 = [e[2]-e[1] for e in ev if e[0] == "A" and e[3] == full]
Bfull = max(e[3] for e in ev if e[0] == "B")
B1 = [e[2]-e[1] for e in ev if e[0] == "B" and e[3] == Bfull]
# eight-bucket steps: group consecutive 8 A's / 8 B's of the small grids
small = [e for e in ev if (e[0] == "A" and e[3] < full) or (e[0] == "B" and e[3] < Bfull)]
As = [e for e in small if e[0] == "A"]; Bs = [e for e in small if e[0] == "B"]
steps = []
for s in range(min(len(As), len(Bs)) // 8):
    a = As[8*s:8*s+8]; b = Bs[8*s:8*s+8]
    steps.append({"A_sum": sum(x[2]-x[1] for x in a), "A_union": union([(x[1], x[2]) for x in a]),
                  "B_sum": sum(x[2]-x[1] for x in b), "AB_union": union([(x[1], x[2]) for x in a + b]),
                  "A_queues": sorted({x[4] for x in a})})
k = steps[len(steps)//4:]  # past warm-up
med = lambda key: round(st.median(s[key] for s in k) / 1000, 1)
out = {"source": "rocprofv3 --kernel-trace of scripts/pipeline_sweep.py --variants spans --configs 1/0/1,8/1/1 (G > 1 pipeline forced at G = 1, ResNet-50, R = 8)",
       "one_bucket": {"steps": len(A1), "A_us_median": round(st.median(A1)/1000, 1), "B_us_median": round(st.median(B1)/1000, 1),
                      "A_plus_B_us": round((st.median(A1) + st.median(B1))/1000, 1)},
       "eight_buckets_mode1": {"steps_kept": len(k), "A_sum_us_median": med("A_sum"), "A_busy_union_us_median": med("A_union"),
                               "B_sum_us_median": med("B_sum"), "A_and_B_busy_union_us_median": med("AB_union"),
                               "A_queues": k[0]["A_queues"]}}
print(json.dumps(out, indent=1))
