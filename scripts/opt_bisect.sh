#!/bin/bash
# Replica optimiser regression (VERDICT r04 Weak #2): the same N = 1 bench
# (optimiser leg only kept beside the SMA step) on the HEAD tree and on an
# older worktree under _bisect/, interleaved, at 16 and at 4 hardware queues,
# then one rocprofv3 --kernel-trace --stats pass of each tree.
# Usage (GPU box): bash scripts/opt_bisect.sh [old-tree-dir ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/bisect
mkdir -p "$out"
trees=(. "$@")
COMMON=(--steps 20 --warmup 5 --no-cpu-baseline --no-staged --no-seam --no-copy-ceiling --watchdog-scale 0)
run() {  # tag tree extra...
  local tag=$1 tree=$2; shift 2
  echo "== $tag" >&2
  (cd "$tree" && timeout -k 10 180 python3 bench.py "${COMMON[@]}" "$@") > "$out/$tag.json" 2> "$out/$tag.err" || {
    echo "FAILED $tag rc=$?" >&2; tail -5 "$out/$tag.err" >&2; return 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); o=r['replica_optimiser']; print(sys.argv[2], o['launch_ms_mean'], o['frac'], r['roofline']['launch_ms_mean'], r['config']['hw_queues']['GPU_MAX_HW_QUEUES'])" "$out/$tag.json" "$tag" | tee -a "$out/summary.txt"
}
for pass in 1 2; do
  for i in "${!trees[@]}"; do
    run "t${i}_q16_p$pass" "${trees[$i]}" || exit 1
    GPU_MAX_HW_QUEUES=4 run "t${i}_q4_p$pass" "${trees[$i]}" --keep-hw-queues || exit 1
  done
done
for i in "${!trees[@]}"; do
  echo "== rocprof t$i" >&2
  (cd "${trees[$i]}" && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_t$i" -o run \
     --output-format csv -- python3 bench.py "${COMMON[@]}") > "$out/prof_t$i.json" 2> "$out/prof_t$i.err" || {
    echo "FAILED rocprof t$i" >&2; tail -5 "$out/prof_t$i.err" >&2; exit 1; }
done
echo done >&2
