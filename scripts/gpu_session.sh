#!/bin/bash
# A GPU-box session of named steps (the first argument, comma-separated):
#   tests      the whole -m gpu suite
#   tests:K    only the tests matching -k K
#   bench      python bench.py $BENCH_ARGS
#   smoke      __graft_entry__.smoke()
#   rehearse   bench.py at N = 2 / 4 / 8 in both process forms on one GPU
#   rehearse-perrank  the same, one process per rank only
#   enqueue    scripts/host_enqueue_multidev.py (single-process host cost)
#   rocprof    rocprofv3 --kernel-trace --stats of bench.py $BENCH_ARGS
#   markers    rocprofv3 --marker-trace --kernel-trace of the single-process rehearsal
#   script:P   python P (a measurement script under scripts/)
# Every GPU step has its own time limit; a fault / abort / timeout ends the
# script (no later GPU step runs); a plain test failure does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 4 "gpurun_out/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
PYTEST="python -u -m pytest -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider"
IFS=',' read -ra STEPS <<< "${1:-tests,bench}"
for s in "${STEPS[@]}"; do
  case "$s" in
    tests) run pytest_gpu 1100 $PYTEST tests ;;
    tests:*) run "pytest_${s#tests:}" 600 $PYTEST tests -k "${s#tests:}" ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as e; e.smoke()" ;;
    rehearse-perrank)
      for g in 2 4 8; do
        run "perrank_n$g" 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $g --master-addr 127.0.0.1 \
          --master-port $((29600 + g)) bench.py --gpus $g --rehearse-one-gpu --steps 20 --warmup 3 --no-staged --tune-steps 3 --tune-passes 1 --calib-steps 3
      done ;;
    rehearse)
      for g in 2 4 8; do
        run "single_n$g" 300 python bench.py --gpus $g --single-process --rehearse-one-gpu --steps 20 --warmup 3 \
          --no-staged --no-cpu-baseline
      done
      for g in 2 4 8; do
        run "perrank_n$g" 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $g --master-addr 127.0.0.1 \
          --master-port $((29600 + g)) bench.py --gpus $g --rehearse-one-gpu --steps 20 --warmup 3 --no-staged --tune-steps 3 --tune-passes 1 --calib-steps 3
      done ;;
    enqueue)
      run enqueue_peer 400 python scripts/host_enqueue_multidev.py --variant peer
      run enqueue_noop 600 python scripts/host_enqueue_multidev.py --variant fake-noop ;;
    script:*) run "$(basename "${s#script:}" .py)" 600 python ${s#script:} ${SCRIPT_ARGS:-} ;;
    rocprof) run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-staged --no-copy-ceiling --no-seam ${BENCH_ARGS:-} ;;
    markers) run markers 600 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/markers -o run \
      --output-format csv -- python3 bench.py --gpus 8 --single-process --rehearse-one-gpu --steps 20 --warmup 3 \
      --no-staged --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
