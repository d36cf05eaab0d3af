#!/bin/bash
# The replica optimiser kernel's duration by the kind of stream it is
# launched on, at GPU_MAX_HW_QUEUES 4 and 16 (scripts/hw_queues_opt.py under
# rocprofv3 --kernel-trace --stats, a fresh process per case).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/streamkind
mkdir -p "$out"
: > "$out/summary.jsonl"
for q in 16 4 8; do
  for s in torch torch-hi hip hip-nb hip-prio0 hip-prio-1 hip-prio1 lib; do
    tag="q${q}_${s}"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/$tag" -o run \
      --output-format csv -- python3 scripts/hw_queues_opt.py --stream $s \
      > "$out/$tag.json" 2> "$out/$tag.err" || { echo "FAILED $tag" >&2; tail -5 "$out/$tag.err" >&2; continue; }
    python3 - "$out/$tag" "$out/$tag.json" "$tag" >> "$out/summary.jsonl" <<'PY'
import csv, glob, json, sys
d, j, tag = sys.argv[1:4]
r = json.load(open(j))
f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    if "sma_optimise_kernel" in row["Name"]:
        r.update(tag=tag, kernel_avg_us=round(float(row["AverageNs"]) / 1e3, 2),
                 kernel_min_us=round(float(row["MinNs"]) / 1e3, 2), calls=int(row["Calls"]))
print(json.dumps(r))
PY
    rm -rf "$out/$tag"
    tail -1 "$out/summary.jsonl"
  done
done
