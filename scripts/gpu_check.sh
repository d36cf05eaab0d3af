#!/bin/bash
# One GPU-box session: smoke, GPU tests, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
# A plain test failure (pytest exit 1) does not stop the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-smoke,tests,bench,rocprof}
[[ $STEPS == *smoke* ]] && { run smoke 300 python -c "import __graft_entry__ as e; e.smoke()" || true; }
[[ $STEPS == *tests* ]] && { run pytest_gpu 900 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider || true; }
[[ $STEPS == *bench* ]] && { run bench 600 python bench.py ${BENCH_ARGS:-} || true; }
[[ $STEPS == *launcher* ]] && { run launcher 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline || true; }
[[ $STEPS == *sweep* ]] && { run sweep 600 python scripts/sweep.py ${SWEEP_ARGS:-} || true; }
[[ $STEPS == *pcie* ]] && { run pcie_bench 300 ./scripts/pcie_bench || true; }
[[ $STEPS == *c2* ]] && { run c2_latency 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o run --output-format csv -- python3 scripts/c2_latency.py || true; }
[[ $STEPS == *rocprof* ]] && { run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-staged --no-copy-ceiling --no-seam ${BENCH_ARGS:-} || true; }
exit 0
