#!/bin/bash
# Test infrastructure for the two-rank-on-one-GPU tests (tests/test_gpu_multirank.py):
#   tests/native/libfakerccl.so             loopback stand-in for the RCCL calls the library makes
#   tests/native/libcrossbow_sma_fakerccl.so the library's own sources linked against it
# Both git-ignored; they travel to the GPU box with the tree.  Run here, on the CPU.
set -euo pipefail
cd "$(dirname "$0")/.."
N=tests/native
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -fPIC -shared -Wall \
  -Wl,-soname,libfakerccl.so -o "$N/libfakerccl.so.tmp" "$N/fake_rccl.cpp"
mv "$N/libfakerccl.so.tmp" "$N/libfakerccl.so"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -ffp-contract=off \
  -I include -o "$N/libcrossbow_sma_fakerccl.so.tmp" \
  crossbow_amd/csrc/context.hip crossbow_amd/csrc/sma_kernels.hip \
  -L "$N" -lfakerccl -Wl,-rpath,'$ORIGIN' -lrocprofiler-sdk-roctx -lpthread
mv "$N/libcrossbow_sma_fakerccl.so.tmp" "$N/libcrossbow_sma_fakerccl.so"
echo "built $N/libfakerccl.so $N/libcrossbow_sma_fakerccl.so"
