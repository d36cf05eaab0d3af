#!/bin/bash
# Test infrastructure for tests/test_gpu_jni.py: the JNI shim
# (crossbow_amd/csrc/jni/TheGPU_jni.c) compiled against the test-only jni.h
# stand-in (tests/jni_stub/jni.h; no JDK in this image), and a plain-C driver
# that calls its natives through a hand-made JNIEnv (tests/native/jni_driver.c)
# and checks the results with the oracle.
#   tests/native/libGPU_stubjni.so   the shim, linked against crossbow_amd/libcrossbow_sma.so
#   tests/native/jni_driver          the driver
# Both git-ignored; they travel to the GPU box with the tree.  Run here, on the CPU,
# after the library is built.
set -euo pipefail
cd "$(dirname "$0")/.."
N=tests/native
gcc -O2 -fPIC -shared -Wall -Wextra -std=c11 -I tests/jni_stub -I include \
  -o "$N/libGPU_stubjni.so.tmp" crossbow_amd/csrc/jni/TheGPU_jni.c \
  -L crossbow_amd -lcrossbow_sma -Wl,-rpath,'$ORIGIN/../../crossbow_amd'
mv "$N/libGPU_stubjni.so.tmp" "$N/libGPU_stubjni.so"
gcc -O2 -Wall -Wextra -std=c11 -I tests/jni_stub -I include -I oracle \
  -o "$N/jni_driver.tmp" "$N/jni_driver.c" oracle/sma_oracle.c \
  -L "$N" -lGPU_stubjni -L crossbow_amd -lcrossbow_sma \
  -Wl,-rpath,'$ORIGIN' -Wl,-rpath,'$ORIGIN/../../crossbow_amd' -lm -ldl -lpthread
mv "$N/jni_driver.tmp" "$N/jni_driver"
echo "built $N/libGPU_stubjni.so $N/jni_driver"
