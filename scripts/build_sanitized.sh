#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the C-ABI
# library sources linked into a plain-C driver (tests/native/abi_driver.c).
# Every -fsanitize= on the hipcc line sits right after -Xarch_host: device
# code is not instrumented (no GPU ASan on this pool).  Output:
# tests/native/abi_driver_asan (git-ignored; it travels to the GPU box with
# the tree).  Run here, on the CPU.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=tests/native/abi_driver_asan
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
/opt/rocm/lib/llvm/bin/clang -c -O1 -g -std=c11 -fno-omit-frame-pointer -fsanitize=address,undefined \
  -I include -o "$TMP/abi_driver.o" tests/native/abi_driver.c
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -Xarch_host -gline-tables-only -std=c++17 -ffp-contract=off -fno-omit-frame-pointer \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -I include -o "$OUT.tmp" \
  crossbow_amd/csrc/context.hip crossbow_amd/csrc/sync_steps.hip crossbow_amd/csrc/sma_kernels.hip crossbow_amd/csrc/sma_seam.hip -x none "$TMP/abi_driver.o" \
  -lrccl -lrocprofiler-sdk-roctx -lpthread
mv "$OUT.tmp" "$OUT"
echo "built $OUT"
