#!/bin/bash
# Kernel trace of the G > 1 bucketed pipeline with the REAL RCCL on one GPU:
# WORLD rank processes, each under its own rocprofv3 --kernel-trace (bash,
# which never touches the GPU, starts them), linked by RCCL's socket
# transport (scripts/trace_rank.py).  Then scripts/pipeline_overlap.py reads
# both traces on the one GPU's clock and reports how the RCCL kernels overlap
# kernels A and B.  Output under gpurun_out/trace_rccl/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
WORLD=${WORLD:-2}
OUT=gpurun_out/trace_rccl
rm -rf "$OUT"; mkdir -p "$OUT"
export TRACE_DIR=$(mktemp -d)
pids=()
for r in $(seq 0 $((WORLD - 1))); do
  timeout -k 10 ${SECS:-150} rocprofv3 --kernel-trace -d "$OUT/rank$r" -o run --output-format csv -- \
    python3 scripts/trace_rank.py $r $WORLD ${BUCKETS:-8} ${MODE:-1} ${ALGO:-0} > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
rm -rf "$TRACE_DIR"
tail -n 2 "$OUT"/rank*.log
[ $rc -eq 0 ] || exit $rc
python3 scripts/pipeline_overlap.py "$OUT" > "$OUT/overlap.json" && cat "$OUT/overlap.json"
