#!/bin/bash
# The replica optimiser's launch shape (block, unroll, occupancy cap) against
# the hardware-queue count and the stream it runs on: a launch of ~100k
# one-wave workgroups is bound by the workgroup dispatch rate of the queue
# it lands on (scripts/hw_queues_opt.sh).  Each case a fresh process under
# rocprofv3 --kernel-trace --stats; summary in gpurun_out/auxq/summary.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/auxq
mkdir -p "$out"
: > "$out/summary.jsonl"
for pass in 1; do
  for aux in 64,1,-1 64,2,-1 128,2,-1 256,1,-1 256,2,-1 64,2,4; do
    for q in 4 16; do
      for s in torch lib; do
        tag="a${aux//,/_}_q${q}_${s}_p${pass}"
        GPU_MAX_HW_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/$tag" -o run \
          --output-format csv -- python3 scripts/hw_queues_opt.py --stream $s --aux "$aux" \
          > "$out/$tag.json" 2> "$out/$tag.err" || { echo "FAILED $tag" >&2; tail -5 "$out/$tag.err" >&2; exit 1; }
        python3 - "$out/$tag" "$out/$tag.json" "$tag" >> "$out/summary.jsonl" <<'PY'
import csv, glob, json, sys
d, j, tag = sys.argv[1:4]
r = json.load(open(j))
f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    if "sma_optimise_kernel" in row["Name"]:
        r.update(tag=tag, kernel=row["Name"][:90], kernel_avg_us=round(float(row["AverageNs"]) / 1e3, 2),
                 kernel_min_us=round(float(row["MinNs"]) / 1e3, 2), calls=int(row["Calls"]))
print(json.dumps(r))
PY
        rm -rf "$out/$tag"
        tail -1 "$out/summary.jsonl"
      done
    done
  done
done
