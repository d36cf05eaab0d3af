#!/bin/bash
# Round 6: the GPU tests this round changed or added, one pytest process per
# file group, each under its own time limit; a fault / abort / timeout ends
# the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
PYTEST="python -u -m pytest -m gpu -v --timeout 330 --timeout-method thread -p no:cacheprovider"
step() {  # step <name> <seconds> <pytest args...>
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a gpurun_out/r6/steps.log
  timeout -k 10 "$secs" $PYTEST "$@" > "gpurun_out/r6/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/r6/steps.log
  tail -n 6 "gpurun_out/r6/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc: stopping"; exit $rc;; esac
  return 0
}
case "${1:-a}" in
  a)
    step peer_fail 360 tests/test_gpu_peer_ipc.py -k failed_step -s
    step optimiser_taskwait 200 tests/test_gpu_optimiser.py -k task_wait -s
    step parity_c3_full 300 tests/test_gpu_parity.py -k full_size -s ;;
  a2)
    step peer_fail 360 tests/test_gpu_peer_ipc.py -k failed_step -s
    step optimiser_taskwait 200 tests/test_gpu_optimiser.py -k task_wait -s
    step peer_ipc 900 tests/test_gpu_peer_ipc.py -k "not failed_step" ;;
  b)
    step peer_ipc 900 tests/test_gpu_peer_ipc.py -k "not failed_step" ;;
  c)
    step multirank_full 1100 tests/test_gpu_multirank.py -k full_size -s ;;
  e)
    step peer_fail 360 tests/test_gpu_peer_ipc.py -k failed_step -s
    step peer_ipc 900 tests/test_gpu_peer_ipc.py -k "not failed_step and not slot_boundary" ;;
  d)
    step maxsize_full 700 tests/test_gpu_maxsize.py -s
    step ipc_slot_boundary 360 tests/test_gpu_peer_ipc.py -k slot_boundary -s ;;
esac
