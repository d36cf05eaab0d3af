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
  crossbow_amd/csrc/context.hip crossbow_amd/csrc/sync_steps.hip crossbow_amd/csrc/sma_kernels.hip crossbow_amd/csrc/sma_seam.hip \
  -L "$N" -lfakerccl -Wl,-rpath,'$ORIGIN' -lrocprofiler-sdk-roctx -lpthread
mv "$N/libcrossbow_sma_fakerccl.so.tmp" "$N/libcrossbow_sma_fakerccl.so"
echo "built $N/libfakerccl.so $N/libcrossbow_sma_fakerccl.so"
# The JNI shim and its driver over the loopback build: tests/test_gpu_jni.py
# runs `jni_driver_fakerccl G`, one process over G copies of device 0.
gcc -O2 -fPIC -shared -Wall -Wextra -std=c11 -I tests/jni_stub -I include \
  -o "$N/libGPU_stubjni_fakerccl.so.tmp" crossbow_amd/csrc/jni/TheGPU_jni.c \
  -L "$N" -l:libcrossbow_sma_fakerccl.so -Wl,-rpath,'$ORIGIN'
mv "$N/libGPU_stubjni_fakerccl.so.tmp" "$N/libGPU_stubjni_fakerccl.so"
gcc -O2 -Wall -Wextra -std=c11 -I tests/jni_stub -I include -I oracle \
  -o "$N/jni_driver_fakerccl.tmp" "$N/jni_driver.c" oracle/sma_oracle.c \
  -L "$N" -l:libGPU_stubjni_fakerccl.so -l:libcrossbow_sma_fakerccl.so \
  -Wl,-rpath,'$ORIGIN' -lm -ldl -lpthread
mv "$N/jni_driver_fakerccl.tmp" "$N/jni_driver_fakerccl"
echo "built $N/libGPU_stubjni_fakerccl.so $N/jni_driver_fakerccl"
