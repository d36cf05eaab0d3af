cd $GRAFT_REPO_ROOT
for g in 2 4 8; do
  timeout -k 10 300 python bench.py --gpus $g --single-process --rehearse-one-gpu --steps 20 --warmup 3 --no-staged --no-cpu-baseline > gpurun_out/single_n$g.log 2>&1 || { echo "single n$g failed rc=$?"; tail -20 gpurun_out/single_n$g.log; exit 1; }
  grep '^{"metric' gpurun_out/single_n$g.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print($g, d['value'], c['allreduce_algorithm'], c['buckets'], c['pipeline_mode'], c['enqueue_threads'], d['identity']['z_last_identical_on_every_gpu'], d['identity']['trusted'])"
done
