#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes) over a short bench run,
# then per-launch HBM bytes -> gpurun_out/traffic.json (copy to profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-}
SUFFIX=${KEY_SUFFIX:-resnet50/R8/m1}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-staged --no-copy-ceiling $ARGS \
    > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 gpurun_out/pmc_$c.log; exit 1; }
done
python3 scripts/pmc_traffic.py --out gpurun_out/traffic.json --key-suffix "$SUFFIX" --alg-bytes sma_fused_kernel=${ALG_FUSED:-2862387584} --alg-bytes sma_optimise_kernel=${ALG_OPT:-715596896} \
  gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_traffic.log 2>&1
tail -40 gpurun_out/pmc_traffic.log
