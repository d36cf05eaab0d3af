# The N = 1 bench line five times in a row on one box (fresh process each):
# the spread of `value`, the fused kernel's fraction and the optimiser's.
cd $GRAFT_REPO_ROOT
: > gpurun_out/bench_spread.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-staged --no-seam --no-copy-ceiling > gpurun_out/spread_$i.json 2> gpurun_out/spread_$i.err || { echo "run $i failed"; tail -5 gpurun_out/spread_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/spread_$i.json'))
print(json.dumps({'run': $i, 'value': d['value'], 'frac': d['roofline']['frac'], 'launch_ms': d['roofline']['launch_ms_mean'], 'opt_ms': d['replica_optimiser']['launch_ms_mean'], 'opt_frac': d['replica_optimiser']['frac']}))" | tee -a gpurun_out/bench_spread.jsonl
done
