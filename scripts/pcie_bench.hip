// pcie_bench.hip -- exploration microbenchmark for the host-staged SMA step
// (cbx_synchronise_staged) on one MI355X; not part of the product library.
//
// C3's staging moves H = (2R+1+m)*4n = 1.84 GB host -> device (z, last, s_i,
// w_i) and D = (R+1+m)*4n = 1.02 GB device -> host (z, last, w_i).  This
// measures how fast the PCIe link carries them, one direction and both at
// once, through the DMA engines (hipMemcpyAsync on one or several streams)
// and through kernels that read / write pinned host memory directly
// (zero-copy), so the staged pipeline can be built on the faster mechanism.
// One JSON line per variant.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o scripts/pcie_bench scripts/pcie_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
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

// Grid-stride float4 copy: host <-> device through the kernel's own loads and
// stores (zero-copy when one side is pinned host memory).
__global__ __launch_bounds__(256) void zc_copy(v4f *dst, const v4f *src, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
}

// Unrolled variant: each lane keeps U loads in flight before its stores.
template <int U>
__global__ __launch_bounds__(256) void zc_copy_u(v4f *dst, const v4f *src, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t b = ((size_t)blockIdx.x * blockDim.x) * U + threadIdx.x; b < n4; b += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n4) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = b + (size_t)u * blockDim.x;
      if (i < n4) dst[i] = v[u];
    }
  }
}

struct Bufs {
  char *hin = nullptr, *din = nullptr;    // H bytes: host source, device destination
  char *dout = nullptr, *hout = nullptr;  // D bytes: device source, host destination
};

static size_t H_BYTES = 1840000000ull, D_BYTES = 1022000000ull;

// Run `enqueue` (which enqueues on the given streams) `reps` times; median
// milliseconds from a common start event to every stream's end.
static double timed(const std::vector<hipStream_t> &st, const std::function<void()> &enqueue, int reps = 3) {
  std::vector<double> ms;
  hipEvent_t start, stop;
  CK(hipEventCreate(&start));
  CK(hipEventCreate(&stop));
  std::vector<hipEvent_t> ends(st.size());
  for (auto &e : ends) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(start, st[0]));
    for (size_t k = 1; k < st.size(); ++k) CK(hipStreamWaitEvent(st[k], start, 0));
    enqueue();
    for (size_t k = 1; k < st.size(); ++k) {
      CK(hipEventRecord(ends[k], st[k]));
      CK(hipStreamWaitEvent(st[0], ends[k], 0));
    }
    CK(hipEventRecord(stop, st[0]));
    CK(hipEventSynchronize(stop));
    float t = 0;
    CK(hipEventElapsedTime(&t, start, stop));
    if (r > 0) ms.push_back(t);  // first pass warms up
  }
  std::sort(ms.begin(), ms.end());
  CK(hipEventDestroy(start));
  CK(hipEventDestroy(stop));
  for (auto &e : ends) CK(hipEventDestroy(e));
  return ms[ms.size() / 2];
}

static void report(const char *name, const char *detail, double ms, double h, double d) {
  std::printf("{\"variant\": \"%s\", \"detail\": \"%s\", \"ms\": %.3f, \"h2d_GB\": %.3f, \"d2h_GB\": %.3f, "
              "\"GBs_total\": %.2f, \"staged_end_to_end_GBs_C3\": %.2f}\n",
              name, detail, ms, h / 1e9, d / 1e9, (h + d) / (ms * 1e-3) / 1e9,
              2862387584.0 / (ms * 1e-3) / 1e9);
  std::fflush(stdout);
}

static void memcpy_split(char *dst, const char *src, size_t bytes, hipMemcpyKind kind,
                         const std::vector<hipStream_t> &st, size_t first, size_t ways, size_t chunk) {
  // `ways` streams, round-robin over chunks of `chunk` bytes
  size_t k = 0;
  for (size_t off = 0; off < bytes; off += chunk, ++k) {
    const size_t len = std::min(chunk, bytes - off);
    CK(hipMemcpyAsync(dst + off, src + off, len, kind, st[first + k % ways]));
  }
}

int main(int argc, char **argv) {
  if (argc > 1) H_BYTES = std::strtoull(argv[1], nullptr, 10);
  if (argc > 2) D_BYTES = std::strtoull(argv[2], nullptr, 10);
  const unsigned flags[3] = {hipHostMallocDefault, hipHostMallocNonCoherent, hipHostMallocCoherent};
  const char *flag_names[3] = {"default", "noncoherent", "coherent"};
  std::vector<hipStream_t> st(4);
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Bufs b;
  CK(hipMalloc(&b.din, H_BYTES));
  CK(hipMalloc(&b.dout, D_BYTES));
  CK(hipMemset(b.dout, 1, D_BYTES));
  const int nflags = argc > 3 ? std::atoi(argv[3]) : 3;
  for (int f = 3 - nflags; f < 3; ++f) {
    CK(hipHostMalloc(&b.hin, H_BYTES, flags[f]));
    CK(hipHostMalloc(&b.hout, D_BYTES, flags[f]));
    std::memset(b.hin, 2, H_BYTES);
    std::memset(b.hout, 0, D_BYTES);
    const char *fl = flag_names[f];
    const double H = (double)H_BYTES, D = (double)D_BYTES;
    char det[160];
    // --- DMA engines -------------------------------------------------------
    report("sdma_h2d", fl, timed({st[0]}, [&] { CK(hipMemcpyAsync(b.din, b.hin, H_BYTES, hipMemcpyHostToDevice, st[0])); }), H, 0);
    report("sdma_d2h", fl, timed({st[0]}, [&] { CK(hipMemcpyAsync(b.hout, b.dout, D_BYTES, hipMemcpyDeviceToHost, st[0])); }), 0, D);
    report("sdma_both", fl, timed({st[0], st[1]}, [&] {
             CK(hipMemcpyAsync(b.din, b.hin, H_BYTES, hipMemcpyHostToDevice, st[0]));
             CK(hipMemcpyAsync(b.hout, b.dout, D_BYTES, hipMemcpyDeviceToHost, st[1]));
           }), H, D);
    for (size_t ways : {2, 3}) {
      std::snprintf(det, sizeof det, "%s, h2d over %zu streams, 64 MiB chunks", fl, ways);
      report("sdma_h2d_split", det, timed(std::vector<hipStream_t>(st.begin(), st.begin() + ways), [&] {
               memcpy_split(b.din, b.hin, H_BYTES, hipMemcpyHostToDevice, st, 0, ways, 64ull << 20);
             }), H, 0);
      std::snprintf(det, sizeof det, "%s, h2d over %zu streams + d2h on one", fl, ways);
      report("sdma_both_split", det, timed(std::vector<hipStream_t>(st.begin(), st.begin() + ways + 1), [&] {
               memcpy_split(b.din, b.hin, H_BYTES, hipMemcpyHostToDevice, st, 0, ways, 64ull << 20);
               CK(hipMemcpyAsync(b.hout, b.dout, D_BYTES, hipMemcpyDeviceToHost, st[ways]));
             }), H, D);
    }
    // --- zero-copy kernels ---------------------------------------------------
    for (unsigned blocks : {256u, 1024u, 4096u, 16384u}) {
      std::snprintf(det, sizeof det, "%s, %u x 256 threads", fl, blocks);
      report("zc_read", det, timed({st[0]}, [&] {
               hipLaunchKernelGGL(zc_copy, dim3(blocks), dim3(256), 0, st[0], (v4f *)b.din, (const v4f *)b.hin, H_BYTES / 16);
             }), H, 0);
      report("zc_write", det, timed({st[0]}, [&] {
               hipLaunchKernelGGL(zc_copy, dim3(blocks), dim3(256), 0, st[0], (v4f *)b.hout, (const v4f *)b.dout, D_BYTES / 16);
             }), 0, D);
      report("zc_both", det, timed({st[0], st[1]}, [&] {
               hipLaunchKernelGGL(zc_copy, dim3(blocks), dim3(256), 0, st[0], (v4f *)b.din, (const v4f *)b.hin, H_BYTES / 16);
               hipLaunchKernelGGL(zc_copy, dim3(blocks), dim3(256), 0, st[1], (v4f *)b.hout, (const v4f *)b.dout, D_BYTES / 16);
             }), H, D);
      report("zc_read_u4", det, timed({st[0]}, [&] {
               hipLaunchKernelGGL(zc_copy_u<4>, dim3(blocks), dim3(256), 0, st[0], (v4f *)b.din, (const v4f *)b.hin, H_BYTES / 16);
             }), H, 0);
    }
    // --- mixed: DMA one way, kernel the other ---------------------------------
    report("sdma_h2d+zc_write", fl, timed({st[0], st[1]}, [&] {
             CK(hipMemcpyAsync(b.din, b.hin, H_BYTES, hipMemcpyHostToDevice, st[0]));
             hipLaunchKernelGGL(zc_copy, dim3(1024), dim3(256), 0, st[1], (v4f *)b.hout, (const v4f *)b.dout, D_BYTES / 16);
           }), H, D);
    report("zc_read+sdma_d2h", fl, timed({st[0], st[1]}, [&] {
             hipLaunchKernelGGL(zc_copy, dim3(1024), dim3(256), 0, st[0], (v4f *)b.din, (const v4f *)b.hin, H_BYTES / 16);
             CK(hipMemcpyAsync(b.hout, b.dout, D_BYTES, hipMemcpyDeviceToHost, st[1]));
           }), H, D);
    CK(hipHostFree(b.hin));
    CK(hipHostFree(b.hout));
  }
  CK(hipFree(b.din));
  CK(hipFree(b.dout));
  for (auto &s : st) CK(hipStreamDestroy(s));
  return 0;
}
