set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
timeout -k 10 300 bash scripts/stream_kind_sweep.sh > gpurun_out/r5/streamkind.log 2>&1 || { echo "stream sweep failed rc=$?"; exit 1; }
timeout -k 10 400 python -u -m pytest -v -x --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_peer_ipc.py -k failed_step > gpurun_out/r5/pytest_peer_fail.log 2>&1 || { echo "peer fail test failed rc=$?"; tail -30 gpurun_out/r5/pytest_peer_fail.log; exit 1; }
tail -3 gpurun_out/r5/pytest_peer_fail.log
timeout -k 10 900 python -u -m pytest -v -x --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_bench_contract.py > gpurun_out/r5/pytest_bench_contract.log 2>&1 || { echo "bench contract failed rc=$?"; tail -40 gpurun_out/r5/pytest_bench_contract.log; exit 1; }
tail -3 gpurun_out/r5/pytest_bench_contract.log
