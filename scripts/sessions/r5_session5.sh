cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/launcher_n1.json 2> gpurun_out/launcher_n1.err || { echo "launcher n1 failed"; tail -5 gpurun_out/launcher_n1.err; exit 1; }
tail -c 300 gpurun_out/launcher_n1.json; echo
Q=4 timeout -k 10 400 bash scripts/trace_rccl_streams.sh > gpurun_out/rccl_streams_q4.log 2>&1 || { echo "trace q4 failed"; tail -20 gpurun_out/rccl_streams_q4.log; exit 1; }
Q=16 timeout -k 10 400 bash scripts/trace_rccl_streams.sh > gpurun_out/rccl_streams_q16.log 2>&1 || { echo "trace q16 failed"; tail -20 gpurun_out/rccl_streams_q16.log; exit 1; }
cat gpurun_out/rccl_streams_q4.log | tail -60
