set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
: > gpurun_out/r5/queue_wait_probe5.jsonl
for q in 16 8 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 60 scripts/queue_wait_probe >> gpurun_out/r5/queue_wait_probe5.jsonl || { echo "probe failed q=$q rc=$?"; exit 1; }
done
cat gpurun_out/r5/queue_wait_probe5.jsonl
