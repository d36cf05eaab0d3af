#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes) over short bench runs,
# then per-launch HBM bytes -> gpurun_out/traffic.json (copy to profiles/).
# Two runs: the fused G = 1 step, and the split pipeline at one bucket (kernels
# A and B over the whole model, as bench.py's N > 1 roofline prices them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
N=25557032  # ResNet-50 elements; bytes per element: fused 112, A 104, B 20, optimiser 28
SUFFIX=${KEY_SUFFIX:-resnet50/R8/m1}
pass() {  # pass <tag> <bench args...>
  local tag=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-staged --no-copy-ceiling --no-seam "$@" \
      > gpurun_out/pmc_${tag}_$c.log 2>&1 || { echo "pmc $tag $c failed rc=$?"; tail -20 gpurun_out/pmc_${tag}_$c.log; exit 1; }
  done
}
pass fused
pass split --force-split --bucket-mb -1
rm -f gpurun_out/traffic.json
python3 scripts/pmc_traffic.py --out gpurun_out/traffic.json --key-suffix "$SUFFIX" \
  --only sma_fused_kernel --only sma_optimise_kernel \
  --alg-bytes sma_fused_kernel=$((112 * N)) --alg-bytes sma_optimise_kernel=$((28 * N)) \
  gpurun_out/pmc_fused_FETCH_SIZE gpurun_out/pmc_fused_WRITE_SIZE > gpurun_out/pmc_traffic.log 2>&1 &&
python3 scripts/pmc_traffic.py --out gpurun_out/traffic.json --key-suffix "$SUFFIX" \
  --only sma_accumulate_kernel --only sma_apply_kernel \
  --alg-bytes sma_accumulate_kernel=$((104 * N)) --alg-bytes sma_apply_kernel=$((20 * N)) \
  gpurun_out/pmc_split_FETCH_SIZE gpurun_out/pmc_split_WRITE_SIZE >> gpurun_out/pmc_traffic.log 2>&1
rc=$?
tail -40 gpurun_out/pmc_traffic.log
exit $rc
