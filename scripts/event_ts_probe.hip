// event_ts_probe.hip -- which HIP event timestamps are exact across streams?
// (for the stream-order check, cbx_set_order_check).  Stream s1 runs a long
// streaming kernel K whose dispatch stops event EK; stream s2 waits on EK
// and then runs an empty probe P.  If timestamps are exact, P's stop is at or
// after K's stop.  Variants: the probe's stop via hipExtLaunchKernelGGL, via
// hipEventRecord after it, and K's stop via hipEventRecord after K.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/event_ts_probe scripts/event_ts_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void stream_kernel(float4 *dst, const float4 *src, long n) {
  long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}
__global__ void probe_kernel() {}

int main() {
  const long n = 1L << 26;  // 1 GiB per buffer
  float4 *a, *b;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ek, ep, er, ek2, ref;
  CK(hipEventCreate(&ek));
  CK(hipEventCreate(&ep));
  CK(hipEventCreate(&er));
  CK(hipEventCreate(&ek2));
  CK(hipEventCreate(&ref));
  for (int round = 0; round < 4; ++round) {
    CK(hipEventRecord(ref, s1));
    hipExtLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, s1, nullptr, ek, 0, b, a, n);
    CK(hipEventRecord(ek2, s1));                       // K's stop as a plain record
    CK(hipStreamWaitEvent(s2, ek, 0));
    hipExtLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, s2, nullptr, ep, 0);  // probe's dispatch stop
    CK(hipEventRecord(er, s2));                        // a plain record after the probe
    CK(hipDeviceSynchronize());
    float k, k2, p, r;
    CK(hipEventElapsedTime(&k, ref, ek));
    CK(hipEventElapsedTime(&k2, ref, ek2));
    CK(hipEventElapsedTime(&p, ref, ep));
    CK(hipEventElapsedTime(&r, ref, er));
    std::printf("{\"round\":%d,\"K_stop_dispatch_ms\":%.4f,\"K_stop_record_ms\":%.4f,\"probe_stop_dispatch_ms\":%.4f,"
                "\"probe_then_record_ms\":%.4f}\n", round, k, k2, p, r);
  }
  // Start events: exact, or a marker carrying the previous command's end?
  // And what does a per-launch (start, stop) pair cost back to back?
  hipEvent_t e1, es2, e2, t0, t1;
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&es2));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int round = 0; round < 3; ++round) {
    hipExtLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, s1, nullptr, e1, 0, b, a, n);
    hipExtLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, s1, es2, e2, 0, a, b, n);
    CK(hipDeviceSynchronize());
    float gap, dur;
    CK(hipEventElapsedTime(&gap, e1, es2));
    CK(hipEventElapsedTime(&dur, es2, e2));
    std::printf("{\"round\":%d,\"start_after_prev_stop_us\":%.2f,\"k2_start_to_stop_ms\":%.4f}\n", round, gap * 1e3,
                dur);
  }
  std::vector<hipEvent_t> ev(100);
  for (auto &e : ev) CK(hipEventCreate(&e));
  const long m = 1L << 22;  // 64 MiB per buffer: ~20 us kernels, so per-launch costs show
  for (int round = 0; round < 3; ++round) {
    for (int mode = 0; mode < 3; ++mode) {  // 0 no events, 1 stop only, 2 start + stop
      CK(hipEventRecord(t0, s1));
      for (int i = 0; i < 50; ++i)
        hipExtLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, s1, mode == 2 ? ev[2 * i] : nullptr,
                              mode >= 1 ? ev[2 * i + 1] : nullptr, 0, b, a, m);
      CK(hipEventRecord(t1, s1));
      CK(hipDeviceSynchronize());
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      std::printf("{\"round\":%d,\"events\":\"%s\",\"us_per_launch\":%.2f}\n", round,
                  mode == 0 ? "none" : mode == 1 ? "stop" : "start+stop", ms * 1e3 / 50);
    }
  }
  return 0;
}
