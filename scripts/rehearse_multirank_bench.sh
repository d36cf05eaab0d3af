#!/bin/bash
# N > 1 rehearsal of bench.py on a one-GPU box: the driver's own launcher
# (torch.distributed.run, one process per rank) with every rank on device 0
# and the real RCCL linking the ranks over loopback sockets (--rehearse-one-gpu).
# Checks the N > 1 path end to end (calibration, the warm-up tuner, the timed
# region, max over ranks, the JSON line); its numbers are not xGMI numbers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in ${RANKS:-2 4 8}; do
  timeout -k 10 ${SECS:-240} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --steps ${STEPS:-10} --warmup 3 --rehearse-one-gpu ${BENCH_ARGS:-} \
    > gpurun_out/rehearse_n$N.log 2>&1
  rc=$?
  echo "== N=$N rc=$rc"
  grep '^{' gpurun_out/rehearse_n$N.log | tail -1 | cut -c1-600
  [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearse_n$N.log; exit $rc; }
done
