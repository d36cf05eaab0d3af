// syncbench.hip -- cost of cross-stream dependencies on one MI355X (not part
// of the product library).  A producer stream runs N streaming kernels (each
// a 12.8 MB-per-stream slice like one bucket of kernel A); after each, a
// consumer stream runs a small kernel that must wait for it.  Modes:
//   0 none     : producer kernels back to back, no consumer
//   1 event    : producer hipEventRecord(e_k) after kernel k; consumer hipStreamWaitEvent(e_k)
//   2 writeval : producer hipStreamWriteValue32(flag, k+1); consumer hipStreamWaitValue32(flag >= k+1)
//   3 kernel   : the producer kernel's last workgroup publishes k+1 itself (release atomic);
//                consumer hipStreamWaitValue32(flag >= k+1); no packet on the producer stream
//   4 kernel-signal : as 3, the flag in hipMallocSignalMemory memory (what
//                hipStreamWaitValue32 documents) and a system-scope release
//   5 kernel-nowait : the producer publishes as in 3, nobody waits (the
//                publish's own cost); 6 kernel-signal-nowait likewise for 4
// Prints producer-stream time per kernel and total time (JSON lines).
// Build: hipcc --offload-arch=gfx950 -O3 -o syncbench syncbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                             \
    }                                                                                           \
  } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

// 8 read streams + 4 write streams per element, one float4 per lane.
__global__ __launch_bounds__(256) void produce(const v4f *__restrict__ in, v4f *__restrict__ out, uint32_t n4,
                                               uint32_t *flag, uint32_t value, uint32_t *ticket, int system_scope) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) {
    v4f t = 0.0f;
#pragma unroll
    for (int s = 0; s < 8; ++s) t += __builtin_nontemporal_load(in + (size_t)s * n4 + i);
#pragma unroll
    for (int s = 0; s < 4; ++s) __builtin_nontemporal_store(t, out + (size_t)s * n4 + i);
  }
  if (flag) {
    // last workgroup to finish publishes `value` (release at agent scope)
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const uint32_t done = atomicAdd(ticket, 1u) + 1u;
      if (done == gridDim.x) {
        *ticket = 0;
        __threadfence();
        if (system_scope) {
          __threadfence_system();
          __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
          __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

__global__ void consume(v4f *out, uint32_t k) {
  if (threadIdx.x == 0) out[k] = (float)k;
}

int main(int argc, char **argv) {
  const int nk = argc > 1 ? std::atoi(argv[1]) : 8;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const uint32_t n4 = (uint32_t)(12800000 / 16);  // 12.8 MB per stream
  CK(hipSetDevice(0));
  v4f *in, *out, *small;
  uint32_t *flag, *ticket;
  CK(hipMalloc(&in, (size_t)8 * n4 * 16));
  CK(hipMalloc(&out, (size_t)4 * n4 * 16));
  CK(hipMalloc(&small, 4096));
  CK(hipMalloc(&flag, 256));
  uint32_t *sflag = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&sflag), 8, hipMallocSignalMemory));  // a signal: 8 bytes
  CK(hipMemset(sflag, 0, 8));
  CK(hipMalloc(&ticket, 256));
  CK(hipMemset(in, 0, (size_t)8 * n4 * 16));
  CK(hipMemset(flag, 0, 256));
  CK(hipMemset(ticket, 0, 256));
  hipStream_t p, c;
  CK(hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(nk);
  for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipEvent_t t0, t1, t2;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  CK(hipEventCreate(&t2));
  const unsigned grid = (n4 + 255) / 256;
  uint32_t counter = 0;
  // mode 4: modes 1's pattern captured once into a hipGraph and replayed.
  hipGraphExec_t gexec = nullptr;
  {
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    CK(hipStreamBeginCapture(p, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(fork, p));
    CK(hipStreamWaitEvent(c, fork, 0));
    for (int k = 0; k < nk; ++k) {
      hipLaunchKernelGGL(produce, dim3(grid), dim3(256), 0, p, in, out, n4, nullptr, 0u, ticket, 0);
      CK(hipEventRecord(ev[k], p));
      CK(hipStreamWaitEvent(c, ev[k], 0));
      hipLaunchKernelGGL(consume, dim3(1), dim3(64), 0, c, small, (uint32_t)k);
    }
    CK(hipEventRecord(join, c));
    CK(hipStreamWaitEvent(p, join, 0));
    hipGraph_t graph;
    CK(hipStreamEndCapture(p, &graph));
    CK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
  }
  for (int round = 0; round < 3; ++round) {
    float tot = 0;
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, p));
      CK(hipGraphLaunch(gexec, p));
      CK(hipEventRecord(t1, p));
      CK(hipEventSynchronize(t1));
      float a;
      CK(hipEventElapsedTime(&a, t0, t1));
      if (r >= 2) tot += a;
    }
    std::printf("{\"round\":%d,\"mode\":\"graph-event\",\"kernels\":%d,\"total_us_per_kernel\":%.2f}\n", round, nk,
                tot * 1e3 / reps / nk);
  }
  for (int round = 0; round < 3; ++round)
    for (int mode = 0; mode < 7; ++mode) {
      float prod_ms = 0, tot_ms = 0;
      for (int r = 0; r < reps + 2; ++r) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(t0, p));
        CK(hipStreamWaitEvent(c, t0, 0));
        for (int k = 0; k < nk; ++k) {
          const uint32_t v = ++counter;
          uint32_t *f = (mode == 3 || mode == 5) ? flag : (mode == 4 || mode == 6) ? sflag : nullptr;
          hipLaunchKernelGGL(produce, dim3(grid), dim3(256), 0, p, in, out, n4, f, v, ticket,
                             (mode == 4 || mode == 6) ? 1 : 0);
          if (mode == 1) {
            CK(hipEventRecord(ev[k], p));
            CK(hipStreamWaitEvent(c, ev[k], 0));
          } else if (mode == 2) {
            CK(hipStreamWriteValue32(p, flag, v, 0));
            CK(hipStreamWaitValue32(c, flag, v, hipStreamWaitValueGte, 0xffffffffu));
          } else if (mode == 3 || mode == 4) {
            CK(hipStreamWaitValue32(c, mode == 3 ? flag : sflag, v, hipStreamWaitValueGte, 0xffffffffu));
          }
          if (mode >= 1 && mode <= 4) hipLaunchKernelGGL(consume, dim3(1), dim3(64), 0, c, small, (uint32_t)k);
        }
        CK(hipEventRecord(t1, p));
        CK(hipEventRecord(t2, c));
        CK(hipEventSynchronize(t1));
        CK(hipEventSynchronize(t2));
        float a, b;
        CK(hipEventElapsedTime(&a, t0, t1));
        CK(hipEventElapsedTime(&b, t0, t2));
        if (r >= 2) {
          prod_ms += a;
          tot_ms += (mode == 0 || mode >= 5 ? a : (b > a ? b : a));
        }
      }
      const char *names[] = {"none", "event", "writeval", "kernel-flag", "kernel-flag-signal", "kernel-flag-nowait",
                             "kernel-flag-signal-nowait"};
      std::printf("{\"round\":%d,\"mode\":\"%s\",\"kernels\":%d,\"producer_us_per_kernel\":%.2f,\"total_us_per_kernel\":%.2f}\n",
                  round, names[mode], nk, prod_ms * 1e3 / reps / nk, tot_ms * 1e3 / reps / nk);
      std::fflush(stdout);
    }
  return 0;
}
