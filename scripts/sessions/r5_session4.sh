set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
: > gpurun_out/r5/deferred_wait.jsonl
for q in 16 4; do
  for s in torch lib; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5/dw_${q}_$s -o run --output-format csv -- python3 scripts/hw_queues_opt.py --stream $s > gpurun_out/r5/dw_${q}_$s.json 2> gpurun_out/r5/dw_${q}_$s.err || { echo "hwq run failed"; tail -5 gpurun_out/r5/dw_${q}_$s.err; exit 1; }
    python3 -c "
import csv,glob,json,sys
r=json.load(open('gpurun_out/r5/dw_${q}_$s.json'))
f=glob.glob('gpurun_out/r5/dw_${q}_$s/**/run_kernel_stats.csv',recursive=True)[0]
for row in csv.DictReader(open(f)):
    if 'sma_optimise_kernel' in row['Name']: r.update(kernel_avg_us=round(float(row['AverageNs'])/1e3,2), kernel_min_us=round(float(row['MinNs'])/1e3,2))
print(json.dumps(r))" >> gpurun_out/r5/deferred_wait.jsonl
  done
done
cat gpurun_out/r5/deferred_wait.jsonl
timeout -k 10 900 python -u -m pytest -v -x --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_optimiser.py > gpurun_out/r5/pytest_optimiser.log 2>&1 || { echo "optimiser tests failed rc=$?"; tail -30 gpurun_out/r5/pytest_optimiser.log; exit 1; }
tail -2 gpurun_out/r5/pytest_optimiser.log
timeout -k 10 300 python bench.py > gpurun_out/r5/bench_n1.json 2> gpurun_out/r5/bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/r5/bench_n1.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5/bench_n1.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'opt', d['replica_optimiser'], 'hwq', d['config']['hw_queues'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5/bench_rocprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-staged --no-copy-ceiling > gpurun_out/r5/bench_rocprof.json 2> gpurun_out/r5/bench_rocprof.err || { echo "rocprof bench failed"; tail -20 gpurun_out/r5/bench_rocprof.err; exit 1; }
cut -c1-160 $(find gpurun_out/r5/bench_rocprof -name "*kernel_stats.csv") | head -8
