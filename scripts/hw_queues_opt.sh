#!/bin/bash
# The replica optimiser kernel's duration against GPU_MAX_HW_QUEUES and the
# stream it runs on (scripts/hw_queues_opt.py), each case in a fresh process
# under rocprofv3 --kernel-trace --stats; summary in gpurun_out/hwq/summary.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/hwq
mkdir -p "$out"
: > "$out/summary.jsonl"
for pass in 1 2; do
  for q in 4 8 16; do
    for s in torch lib; do
      for x in 0 4; do
        tag="q${q}_${s}_x${x}_p${pass}"
        GPU_MAX_HW_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/$tag" -o run \
          --output-format csv -- python3 scripts/hw_queues_opt.py --stream $s --extra-streams $x \
          > "$out/$tag.json" 2> "$out/$tag.err" || { echo "FAILED $tag" >&2; tail -5 "$out/$tag.err" >&2; exit 1; }
        python3 - "$out/$tag" "$out/$tag.json" "$tag" >> "$out/summary.jsonl" <<'EOF'
import csv, glob, json, sys
d, j, tag = sys.argv[1:4]
r = json.load(open(j))
f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    if "sma_optimise_kernel" in row["Name"]:
        r.update(tag=tag, kernel_avg_us=round(float(row["AverageNs"]) / 1e3, 2),
                 kernel_min_us=round(float(row["MinNs"]) / 1e3, 2), calls=int(row["Calls"]))
print(json.dumps(r))
EOF
        tail -1 "$out/summary.jsonl"
      done
    done
  done
done
