# The IPC size boundary from below, under torch's HIP 7.0: two rank processes
# export and open acc / D slots of 2,141,196,288 B (2042 MiB + 4 KiB, the
# allocation just under 2^31 bytes once rounded to 2 MiB), then run 3
# peer-read steps.  DESIGN.md 6: ROCr 7.0 keeps the size in an int, so this
# opens, while 2 GiB and more never returned (profiles/r04/ipc/).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 \
  scripts/ipc_torch_probe.py --elements 535000000 --replicas 1 > gpurun_out/ipc_boundary_2042MiB.txt 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/ipc_boundary_2042MiB.txt
cat gpurun_out/ipc_boundary_2042MiB.txt | grep -v "^\[rank.*Warning" | tail -20
exit $rc
