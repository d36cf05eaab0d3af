// ipcprobe.hip -- can two processes on one node order GPU work on each
// other's buffers without a host round trip per step?  (Feasibility probe for
// the per-rank peer-read all-reduce; not part of the product library.)
//
// The producer process owns a 64 MiB device buffer (exported with
// hipIpcGetMemHandle; HSA_ENABLE_IPC_MODE_LEGACY=0, dmabuf) and a page of
// flags in POSIX shared memory that both processes pin with hipHostRegister.
// Per iteration i:
//   producer: idle ~`idle_us` (one wave), fill(buf, i), WriteValue64(flagA, i),
//             WaitValue64(flagB >= i)   (the consumer is done reading buf)
//   consumer: WaitValue64(flagA >= i), check(buf == i) -> mismatch counter,
//             WriteValue64(flagB, i)
// mode 0 keeps both waits; mode 1 drops the consumer's wait (the race must
// then show up as mismatches, so the check is known to be sensitive); modes
// 2 / 3 are 0 / 1 with the two flags in device memory instead (each side's
// flag in its own hipMalloc, exported to the other with hipIpcGetMemHandle).
// Arguments: mode iters idle_us floats (floats 0: no kernels, a pure
// write/wait ping-pong between the two processes' streams).
// On any failure either side writes ~0 into both flags from the host, which
// releases a stream waiting on the other.  One JSON line per process.
// Build: hipcc --offload-arch=gfx950 -O3 -o ipcprobe ipcprobe.hip -lrt
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static volatile uint64_t *g_flags = nullptr;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      if (g_flags) g_flags[0] = g_flags[8] = ~0ull;                                             \
      std::exit(2);                                                                             \
    }                                                                                           \
  } while (0)

__global__ void idle(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < (1 << 20) && wall_clock64() - t0 < ticks; ++i) __builtin_amdgcn_s_sleep(8);
}

__global__ __launch_bounds__(256) void fill(float *buf, uint32_t n, float v) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] = v;
}

__global__ __launch_bounds__(256) void check(const float *buf, uint32_t n, float v, unsigned *bad) {
  unsigned mine = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) mine += buf[i] != v;
  if (mine) atomicAdd(bad + (threadIdx.x & 63), mine);  // lane-varying address: a vector atomic
}

int main(int argc, char **argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
  const int idle_us = argc > 3 ? std::atoi(argv[3]) : 50;
  const uint32_t n = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 16u << 20;  // floats: 64 MiB
  const bool devflags = mode >= 2;
  char name[64];
  std::snprintf(name, sizeof(name), "/cbx_ipcprobe_%d", (int)getpid());
  int fd = shm_open(name, O_CREAT | O_RDWR | O_EXCL, 0600);
  if (fd < 0 || ftruncate(fd, 4096) != 0) return std::perror("shm"), 2;
  void *page = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (page == MAP_FAILED) return std::perror("mmap"), 2;
  std::memset(page, 0, 4096);
  g_flags = static_cast<volatile uint64_t *>(page);  // [0] flagA, [8] flagB, [16..] handle
  int pfd[2];
  if (pipe(pfd) != 0) return 2;
  const pid_t child = fork();  // before any HIP call in either process
  const bool producer = child != 0;
  CK(hipSetDevice(0));
  CK(hipHostRegister(page, 4096, hipHostRegisterMapped | hipHostRegisterPortable));
  uint64_t *dflags = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dflags), page, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int khz = 0;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  float *buf = nullptr;
  unsigned *bad = nullptr;
  uint64_t *myflag = nullptr, *peerflag = nullptr;  // device-memory flags (modes 2, 3)
  int pfd2[2];
  if (pipe(pfd2) != 0) return 2;
  if (devflags) {  // each side exports its own flag (device memory) to the other
    CK(hipMalloc(reinterpret_cast<void **>(&myflag), 4096));
    CK(hipMemset(myflag, 0, 4096));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t fh;
    CK(hipIpcGetMemHandle(&fh, myflag));
    int wfd = producer ? pfd[1] : pfd2[1], rfd = producer ? pfd2[0] : pfd[0];
    if (write(wfd, &fh, sizeof(fh)) != (ssize_t)sizeof(fh)) return 2;
    if (read(rfd, &fh, sizeof(fh)) != (ssize_t)sizeof(fh)) return 2;
    CK(hipIpcOpenMemHandle(reinterpret_cast<void **>(&peerflag), fh, hipIpcMemLazyEnablePeerAccess));
    std::fprintf(stderr, "%s: opened the peer's flag\n", producer ? "producer" : "consumer");
  }
  if (producer) {
    CK(hipMalloc(reinterpret_cast<void **>(&buf), (size_t)(n ? n : 1) * 4));
    CK(hipMemset(buf, 0, (size_t)(n ? n : 1) * 4));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, buf));
    if (write(pfd[1], &h, sizeof(h)) != (ssize_t)sizeof(h)) return 2;
  } else {
    hipIpcMemHandle_t h;
    if (read(pfd[0], &h, sizeof(h)) != (ssize_t)sizeof(h)) return 2;
    CK(hipIpcOpenMemHandle(reinterpret_cast<void **>(&buf), h, hipIpcMemLazyEnablePeerAccess));
    std::fprintf(stderr, "consumer: opened the buffer\n");
    CK(hipMalloc(reinterpret_cast<void **>(&bad), 64 * sizeof(unsigned)));
    CK(hipMemset(bad, 0, 64 * sizeof(unsigned)));
  }
  // producer writes A, waits B; consumer waits A, writes B
  uint64_t *flagA_w = devflags ? myflag : dflags + 0, *flagB_w = devflags ? myflag : dflags + 8;
  uint64_t *flagA_r = devflags ? peerflag : dflags + 0, *flagB_r = devflags ? peerflag : dflags + 8;
  CK(hipDeviceSynchronize());
  int rtv = 0;
  CK(hipRuntimeGetVersion(&rtv));
  std::fprintf(stderr, "%s: loop starts (HIP runtime %d)\n", producer ? "producer" : "consumer", rtv);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 1; i <= iters; ++i) {
    if (producer) {
      if (idle_us > 0) idle<<<1, 64, 0, s>>>((uint64_t)khz * idle_us / 1000);
      if (n) fill<<<1024, 256, 0, s>>>(buf, n, (float)i);
      CK(hipStreamWriteValue64(s, flagA_w, (uint64_t)i, 0));
      CK(hipStreamWaitValue64(s, flagB_r, (uint64_t)i, hipStreamWaitValueGte, ~0ull));
    } else {
      if (mode == 0 || mode == 2) CK(hipStreamWaitValue64(s, flagA_r, (uint64_t)i, hipStreamWaitValueGte, ~0ull));
      if (n) check<<<1024, 256, 0, s>>>(buf, n, (float)i, bad);
      CK(hipStreamWriteValue64(s, flagB_w, (uint64_t)i, 0));
    }
  }
  CK(hipStreamSynchronize(s));
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (producer) {
    int st = 0;
    waitpid(child, &st, 0);
    std::printf("{\"side\":\"producer\",\"mode\":%d,\"iters\":%d,\"idle_us\":%d,\"floats\":%u,\"ms_per_iter\":%.4f,"
                "\"child_rc\":%d}\n", mode, iters, idle_us, n, ms / iters, WIFEXITED(st) ? WEXITSTATUS(st) : -1);
    CK(hipFree(buf));
    shm_unlink(name);
  } else {
    unsigned hb[64];
    CK(hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
    unsigned long long tot = 0;
    for (unsigned v : hb) tot += v;
    std::printf("{\"side\":\"consumer\",\"mode\":%d,\"iters\":%d,\"ms_per_iter\":%.4f,\"mismatches\":%llu}\n", mode,
                iters, ms / iters, tot);
    std::fflush(stdout);
    CK(hipIpcCloseMemHandle(buf));
  }
  if (devflags) {
    CK(hipIpcCloseMemHandle(peerflag));
    CK(hipFree(myflag));
  }
  CK(hipHostUnregister(page));
  return 0;
}
