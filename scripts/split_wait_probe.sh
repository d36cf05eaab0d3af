#!/bin/bash
# Kernel A / kernel B durations of the G > 1 pipeline forced at G = 1, one
# bucket (everything in order on the sync stream: no cross-queue wait) against
# 8 buckets (the comm stream waits on each kernel A while it runs), at
# GPU_MAX_HW_QUEUES 4 and 16; rocprofv3 --kernel-trace --stats per case.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/splitwait
mkdir -p "$out"
: > "$out/summary.jsonl"
n4=$(( (25557032 + 3) / 4 ))
for q in 4 16; do
  for cfg in "1b:-1:0" "8b_m0:3194629:0" "8b_m1:3194629:1"; do
    IFS=: read tag elems mode <<< "$cfg"
    t="q${q}_${tag}"
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/$t" -o run --output-format csv -- \
      python3 bench.py --force-split --bucket-elements $( [ "$elems" = -1 ] && echo 4611686018427387904 || echo $elems ) \
      --pipeline-mode $mode --hw-queues $q --steps 30 --warmup 5 --calib-steps 2 --no-cpu-baseline --no-staged \
      --no-copy-ceiling --no-seam --no-optimiser > "$out/$t.json" 2> "$out/$t.err" || { echo "FAILED $t" >&2; tail -5 "$out/$t.err" >&2; exit 1; }
    python3 - "$out/$t" "$out/$t.json" "$t" >> "$out/summary.jsonl" <<'PY'
import csv, glob, json, sys
d, j, tag = sys.argv[1:4]
r = json.load(open(j))
f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)[0]
k = {}
for row in csv.DictReader(open(f)):
    for name in ("sma_accumulate_kernel", "sma_apply_kernel"):
        if name in row["Name"]:
            k[name] = {"calls": int(row["Calls"]), "total_ms": round(float(row["TotalDurationNs"]) / 1e6, 3),
                       "avg_us": round(float(row["AverageNs"]) / 1e3, 2)}
print(json.dumps({"tag": tag, "ms_per_step": r["ms_per_step"], "buckets": r["config"]["buckets"],
                  "roofline_frac": r["roofline"]["frac"], "kernels": k}))
PY
    rm -rf "$out/$t"
    tail -1 "$out/summary.jsonl"
  done
done
