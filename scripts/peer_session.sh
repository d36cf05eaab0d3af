set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_peer_ipc.py > gpurun_out/pytest_peer_ipc3.log 2>&1 || exit 1
WORLD=2 BUCKETS=4 MODE=1 ALGO=1 SECS=150 bash scripts/trace_real_rccl.sh > gpurun_out/tr4.log 2>&1 || exit 1
mv gpurun_out/trace_rccl gpurun_out/trace_peer4
WORLD=2 BUCKETS=1 MODE=0 ALGO=1 SECS=150 bash scripts/trace_real_rccl.sh > gpurun_out/tr1.log 2>&1 || exit 1
mv gpurun_out/trace_rccl gpurun_out/trace_peer1
WORLD=2 BUCKETS=8 MODE=1 ALGO=1 SECS=150 bash scripts/trace_real_rccl.sh > gpurun_out/tr8.log 2>&1 || exit 1
mv gpurun_out/trace_rccl gpurun_out/trace_peer8
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 3 --no-staged --calib-steps 3 > gpurun_out/perrank_n2_full_tuner.log 2>&1
