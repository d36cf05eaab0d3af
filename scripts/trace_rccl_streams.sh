#!/bin/bash
# Which streams and hardware queues RCCL's work lands on beside the library's
# four (sync, comm, two kernel-A streams): two rank processes on one GPU with
# the real RCCL (scripts/trace_rank.py), each under rocprofv3 with the kernel
# trace and the HIP runtime API trace, at GPU_MAX_HW_QUEUES=$Q.  Then
# scripts/rccl_stream_summary.py counts the streams created and lists the
# Stream_Id / Queue_Id of every kernel kind.  Output: gpurun_out/rccl_streams_q$Q/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
Q=${Q:-4}
export GPU_MAX_HW_QUEUES=$Q
OUT=gpurun_out/rccl_streams_q$Q
rm -rf "$OUT"; mkdir -p "$OUT"
export TRACE_DIR=$(mktemp -d)
pids=()
for r in 0 1; do
  timeout -k 10 150 rocprofv3 --kernel-trace --hip-runtime-trace -d "$OUT/rank$r" -o run --output-format csv -- \
    python3 scripts/trace_rank.py $r 2 8 1 0 > "$OUT/rank$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
rm -rf "$TRACE_DIR"
[ $rc -eq 0 ] || { tail -n 5 "$OUT"/rank*.log; exit $rc; }
python3 scripts/rccl_stream_summary.py "$OUT" | tee "$OUT/summary.json"
