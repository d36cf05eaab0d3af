// waitbench.hip -- what one hipStreamWaitEvent costs the waiting queue on one
// MI355X when the event it waits for has long completed (not part of the
// product library).  A consumer stream runs a one-wave kernel that idles
// ~300 us and stamps the wall clock as it ends, then K waits on events that
// K producer streams recorded after short kernels (long complete by then),
// then a kernel that stamps the wall clock as it starts: gap = start - end.
// Swept over K and the events' flags (default = system-scope acquire /
// release fences; hipEventDisableSystemFence; hipEventReleaseToDevice), with
// the producers' kernels writing 12.8 MB each (dirty L2 lines a system-scope
// release must write back) or nothing.  Also the same dependency through
// hipStreamWriteValue32 / hipStreamWaitValue32.  JSON lines on stdout.
// Run with GPU_MAX_HW_QUEUES >= 17 so every stream has a hardware queue of its own.
// Build: hipcc --offload-arch=gfx950 -O3 -o waitbench waitbench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
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

// One wave idling `ticks` of the wall clock (bounded), lane 0 then stamps its end.
__global__ void idle_then_stamp(uint64_t ticks, unsigned long long *out) {
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < (1 << 20) && wall_clock64() - t0 < ticks; ++i) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) out[0] = wall_clock64();
}

__global__ void stamp(unsigned long long *out) {
  if (threadIdx.x == 0) out[0] = wall_clock64();
}

// A producer's bucket-sized write: 12.8 MB of nontemporal float4 stores.
__global__ __launch_bounds__(256) void produce(v4f *out, uint32_t n4) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) __builtin_nontemporal_store((v4f)1.0f, out + i);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 25;
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const double us_per_tick = 1e3 / (double)khz;
  const int kMax = 16;
  const uint32_t n4 = 800000;  // 12.8 MB
  std::vector<hipStream_t> prod(kMax);
  for (auto &s : prod) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipStream_t cons;
  CK(hipStreamCreateWithFlags(&cons, hipStreamNonBlocking));
  std::vector<v4f *> buf(kMax);
  for (auto &b : buf) CK(hipMalloc(&b, (size_t)n4 * 16));
  unsigned long long *stamps;
  CK(hipMalloc(&stamps, 3 * sizeof(unsigned long long)));
  uint32_t *flags;
  CK(hipMalloc(&flags, kMax * 64));
  CK(hipMemset(flags, 0, kMax * 64));
  struct Mode {
    const char *name;
    unsigned ev_flags;
    bool writeval;
  };
  const Mode modes[] = {{"event-default", hipEventDisableTiming, false},
                        {"event-disable-system-fence", hipEventDisableTiming | hipEventDisableSystemFence, false},
                        {"event-release-to-device", hipEventDisableTiming | hipEventReleaseToDevice, false},
                        {"writeval-waitval", 0, true}};
  const uint64_t idle = (uint64_t)khz * 3 / 10;  // 0.3 ms
  uint32_t value = 0;
  for (const Mode &m : modes) {
    std::vector<hipEvent_t> ev(kMax);
    if (!m.writeval)
      for (auto &e : ev) CK(hipEventCreateWithFlags(&e, m.ev_flags));
    for (int dirty = 0; dirty < 2; ++dirty) {
      for (int K : {0, 1, 2, 4, 8, 16}) {
        std::vector<double> gaps;
        for (int r = 0; r < reps + 3; ++r) {
          ++value;
          hipLaunchKernelGGL(idle_then_stamp, dim3(1), dim3(64), 0, cons, idle, stamps);
          for (int k = 0; k < K; ++k) {
            if (dirty) hipLaunchKernelGGL(produce, dim3((n4 + 255) / 256), dim3(256), 0, prod[k], buf[k], n4);
            else hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, prod[k], stamps + 2);
            if (m.writeval) CK(hipStreamWriteValue32(prod[k], flags + 16 * k, value, 0));
            else CK(hipEventRecord(ev[k], prod[k]));
          }
          for (int k = 0; k < K; ++k) {
            if (m.writeval) CK(hipStreamWaitValue32(cons, flags + 16 * k, value, hipStreamWaitValueGte, 0xffffffffu));
            else CK(hipStreamWaitEvent(cons, ev[k], 0));
          }
          hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, cons, stamps + 1);
          CK(hipGetLastError());
          CK(hipStreamSynchronize(cons));
          for (auto &s : prod) CK(hipStreamSynchronize(s));
          unsigned long long h[2];
          CK(hipMemcpy(h, stamps, sizeof(h), hipMemcpyDeviceToHost));
          if (r >= 3) gaps.push_back((double)(long long)(h[1] - h[0]) * us_per_tick);
        }
        std::sort(gaps.begin(), gaps.end());
        std::printf("{\"mode\":\"%s\",\"dirty_producers\":%d,\"waits\":%d,\"gap_us_median\":%.2f,\"gap_us_p10\":%.2f,"
                    "\"gap_us_p90\":%.2f}\n",
                    m.name, dirty, K, gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10]);
        std::fflush(stdout);
      }
    }
    if (!m.writeval)
      for (auto &e : ev) CK(hipEventDestroy(e));
  }
  return 0;
}
