// enqueue_pool_test.cpp -- TEST INFRASTRUCTURE: the per-device enqueue
// thread pool (cbx::host::EnqueuePool, crossbow_amd/csrc/context_internal.h)
// on the CPU, built with ThreadSanitizer by tests/test_enqueue_pool.py.  No
// HIP call is made: the pool only runs host functions.
//   * every run(n, fn) calls fn(k) exactly once for each k < n and returns
//     only after all of them (a counter per device, read right after run);
//   * n changes between runs (8, 2, 5, 1, 16): idle workers stay idle;
//   * failures: the first failing device in device order wins, with its
//     message copied to the calling thread's cbx_last_error text;
//   * back-to-back runs (the per-step use) and the pool's destruction.
// Prints "ok <runs> <mean us per run>" and exits 0, or names the failure.
#include "../../crossbow_amd/csrc/context_internal.h"

#include <chrono>
#include <cstdio>

using cbx::host::EnqueuePool;
using cbx::host::fail;
using cbx::host::g_last_error;

int main() {
  int runs = 0;
  double total_us = 0.0;
  {
    EnqueuePool pool;
    std::vector<std::atomic<int>> hits(16);
    const int sizes[] = {8, 2, 5, 1, 16, 8};
    for (int rep = 0; rep < 500; ++rep) {
      for (int n : sizes) {
        for (auto &h : hits) h.store(0);
        std::vector<int> owner(n, -1);  // written by device k's job only
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = pool.run(n, [&](int k) -> int {
          hits[k].fetch_add(1);
          owner[k] = k;
          return CBX_OK;
        });
        total_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ++runs;
        if (rc != CBX_OK) {
          std::printf("run(%d) failed: %d\n", n, rc);
          return 1;
        }
        for (int k = 0; k < 16; ++k)
          if (hits[k].load() != (k < n ? 1 : 0)) {
            std::printf("run(%d): device %d ran %d times\n", n, k, hits[k].load());
            return 1;
          }
        for (int k = 0; k < n; ++k)
          if (owner[k] != k) {
            std::printf("run(%d): device %d's result missing after run returned\n", n, k);
            return 1;
          }
      }
    }
    // failures: devices 5 and 3 fail; 3 is reported (device order), with its message
    const int rc = pool.run(8, [&](int k) -> int {
      if (k == 5 || k == 3) return fail(CBX_ERR_STATE, "device %d failed", k);
      return CBX_OK;
    });
    if (rc != CBX_ERR_STATE || g_last_error != "device 3 failed") {
      std::printf("failure not propagated: rc %d, message '%s'\n", rc, g_last_error.c_str());
      return 1;
    }
    // and the pool still works afterwards
    std::atomic<int> sum{0};
    if (pool.run(8, [&](int k) -> int { sum += k; return CBX_OK; }) != CBX_OK || sum.load() != 28) {
      std::printf("pool broken after a failure\n");
      return 1;
    }
  }  // destruction joins the workers
  std::printf("ok %d %.2f\n", runs, total_us / runs);
  return 0;
}
