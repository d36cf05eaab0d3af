#!/bin/bash
# Test infrastructure for tests/test_gpu_host.py: the C++ ModelManager
# (crossbow_amd/host/ModelManager.hpp) linked into a driver with the oracle.
#   tests/native/modelmanager_driver  (git-ignored; travels to the GPU box)
# Run here, on the CPU, after the library is built.
set -euo pipefail
cd "$(dirname "$0")/.."
N=tests/native
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
gcc -O2 -std=c11 -fPIC -I oracle -c -o "$TMP/sma_oracle.o" oracle/sma_oracle.c
g++ -O2 -std=c++17 -Wall -Wextra -I crossbow_amd/host -I include -I oracle \
  -o "$N/modelmanager_driver.tmp" "$N/modelmanager_driver.cpp" "$TMP/sma_oracle.o" \
  -L crossbow_amd -lcrossbow_sma -Wl,-rpath,'$ORIGIN/../../crossbow_amd' -lm -ldl -lpthread
mv "$N/modelmanager_driver.tmp" "$N/modelmanager_driver"
echo "built $N/modelmanager_driver"
