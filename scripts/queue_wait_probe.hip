// Why the replica optimiser kernel runs 108 us on some streams and 144 us on
// others (profiles/r05/stream_kind.jsonl): one HBM-bound kernel (3 reads +
// 4 writes of float4, the optimiser's traffic shape, 28 B per element) timed
// by its own dispatch events, on the first stream a process creates or on a
// later one, with or without the first stream waiting on an event recorded
// after each launch (what cbx_replica_optimise does on a caller's stream:
// the sync stream waits for the updated replica, sma.cu:79-81).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/queue_wait_probe scripts/queue_wait_probe.hip
// Run:   GPU_MAX_HW_QUEUES=16 scripts/queue_wait_probe   (one JSON line per case)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef float v4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void shape_kernel(const v4 *__restrict__ w, v4 *__restrict__ g, v4 *__restrict__ last,
                                                   v4 *__restrict__ s, v4 *__restrict__ wo, long n4) {
  const long i = (long)blockIdx.x * 64 + threadIdx.x;
  if (i >= n4) return;
  v4 a = __builtin_nontemporal_load(&w[i]), b = __builtin_nontemporal_load(&g[i]),
     c = __builtin_nontemporal_load(&last[i]);
  v4 gg = b + 1e-4f * a, l = 0.9f * c + 0.1f * gg;
  __builtin_nontemporal_store(a, &s[i]);
  __builtin_nontemporal_store(a - l, &wo[i]);
  __builtin_nontemporal_store(gg, &g[i]);
  __builtin_nontemporal_store(l, &last[i]);
}

// The same traffic from few, fat workgroups: 256 threads, a grid-stride loop
// over a grid of `blocks` workgroups (one dispatch of 2,048 workgroups
// instead of ~100,000 one-wave ones).
__global__ __launch_bounds__(256) void fat_kernel(const v4 *__restrict__ w, v4 *__restrict__ g, v4 *__restrict__ last,
                                                  v4 *__restrict__ s, v4 *__restrict__ wo, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    v4 a = __builtin_nontemporal_load(&w[i]), b = __builtin_nontemporal_load(&g[i]),
       c = __builtin_nontemporal_load(&last[i]);
    v4 gg = b + 1e-4f * a, l = 0.9f * c + 0.1f * gg;
    __builtin_nontemporal_store(a, &s[i]);
    __builtin_nontemporal_store(a - l, &wo[i]);
    __builtin_nontemporal_store(gg, &g[i]);
    __builtin_nontemporal_store(l, &last[i]);
  }
}

int main(int argc, char **argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 25557032L, n4 = (n + 3) / 4;
  const int launches = 40;
  v4 *buf[5];
  for (auto &b : buf) {
    CK(hipMalloc(&b, n4 * sizeof(v4)));
    CK(hipMemset(b, 0, n4 * sizeof(v4)));
  }
  // the library's four streams are created first (context_internal.h), then a caller's
  hipStream_t lib[4], late, late2;
  for (auto &s : lib) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&late, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&late2, hipStreamNonBlocking));  // the sixth stream
  hipEvent_t t0[launches], t1[launches], client;
  for (int i = 0; i < launches; ++i) {
    CK(hipEventCreate(&t0[i]));
    CK(hipEventCreate(&t1[i]));
  }
  CK(hipEventCreateWithFlags(&client, hipEventDisableTiming));
  const char *env = std::getenv("GPU_MAX_HW_QUEUES");
  // wait: 0 none; 1 an event recorded after each launch (hipEventRecord: a
  // marker packet), which the first stream waits on; 2 the first stream
  // waits on the launch's own dispatch stop event; 3 the marker alone
  // on_late: 0 the first stream, 1 the fifth (a caller's), 2 the second, 3 the sixth;
  // waiter: the stream that waits (0 the first, 2 the second)
  struct Case { const char *name; int on_late; int wait; bool fat; int waiter = 0; };
  for (Case cs : {Case{"sixth stream + second stream waits on a recorded event", 3, 1, false, 1},
                  Case{"sixth stream + third stream waits on a recorded event", 3, 1, false, 2},
                  Case{"second stream + first stream waits on a recorded event", 2, 1, false},
                  Case{"later stream + second stream waits on a recorded event", 1, 1, false, 1},
                  Case{"first stream", 0, 0, false}, Case{"later stream", 1, 0, false},
                  Case{"later stream + first stream waits on a recorded event", 1, 1, false},
                  Case{"later stream + first stream waits on the dispatch's stop event", 1, 2, false},
                  Case{"later stream + recorded event, no wait", 1, 3, false},
                  Case{"first stream", 0, 0, false},
                  Case{"fat: later stream", 1, 0, true},
                  Case{"fat: later stream + first stream waits on a recorded event", 1, 1, true}}) {
    hipStream_t st = cs.on_late == 1 ? late : cs.on_late == 2 ? lib[1] : cs.on_late == 3 ? late2 : lib[0];
    hipStream_t waiter = lib[cs.waiter];
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms
      for (int i = 0; i < launches; ++i) {
        if (cs.fat)
          hipExtLaunchKernelGGL(fat_kernel, dim3(2048), dim3(256), 0, st, t0[i], t1[i], 0,
                                buf[0], buf[1], buf[2], buf[3], buf[4], n4);
        else
          hipExtLaunchKernelGGL(shape_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(64), 0, st, t0[i], t1[i], 0,
                                buf[0], buf[1], buf[2], buf[3], buf[4], n4);
        CK(hipGetLastError());
        if (cs.wait == 1 || cs.wait == 3) CK(hipEventRecord(client, st));
        if (cs.wait == 1) CK(hipStreamWaitEvent(waiter, client, 0));
        if (cs.wait == 2) CK(hipStreamWaitEvent(waiter, t1[i], 0));
      }
      CK(hipDeviceSynchronize());
    }
    std::vector<float> ms(launches);
    for (int i = 0; i < launches; ++i) CK(hipEventElapsedTime(&ms[i], t0[i], t1[i]));
    std::sort(ms.begin(), ms.end());
    double mean = 0;
    for (float x : ms) mean += x;
    mean /= launches;
    std::printf("{\"case\": \"%s\", \"GPU_MAX_HW_QUEUES\": \"%s\", \"launch_us_mean\": %.2f, \"launch_us_median\": %.2f, "
                "\"GBs\": %.1f}\n", cs.name, env ? env : "unset", mean * 1e3, ms[launches / 2] * 1e3,
                28.0 * n / (mean * 1e-3) / 1e9);
  }
  return 0;
}
