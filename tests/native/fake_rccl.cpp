// fake_rccl.cpp -- TEST INFRASTRUCTURE: a loopback stand-in for the subset of
// RCCL that libcrossbow_sma calls, so that several processes sharing ONE GPU
// can run the library's multi-rank path (cbx_init_rank, G > 1) against the
// oracle.  Real RCCL refuses two ranks on one device ("Duplicate GPU
// detected"), and the GPU box has one GPU.
//
// ncclAllReduce(float, sum) synchronises the stream it is given (so every
// kernel the library ordered before it has finished), copies the send
// buffer to a file under $FAKE_RCCL_DIR (default /tmp), waits for every
// rank's file of the same sequence number, sums them IN RANK ORDER starting
// from +0 (the oracle's order, oracle/sma_oracle.c; real RCCL's order is its
// own, hence the rtol of the real G > 1 runs), writes the result to the
// receive buffer with a blocking copy and returns.  Stream order is thereby
// preserved: everything the library enqueues afterwards sees the result.
// Every wait times out (ncclSystemError) instead of hanging.
//
// Built by scripts/build_fake_rccl.sh as tests/native/libfakerccl.so; a
// variant of the library linked against it (libcrossbow_sma_fakerccl.so) is
// what tests/test_gpu_multirank.py loads.  Never linked into the product.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

struct ncclComm {
  int nranks = 1;
  int rank = 0;
  int device = 0;
  std::string tag;  // hex of the unique id
  unsigned long long seq = 0;
};

namespace {

std::string dir() {
  const char *d = std::getenv("FAKE_RCCL_DIR");
  return d ? d : "/tmp";
}

std::string path(const ncclComm *c, unsigned long long seq, int rank, const char *kind) {
  char b[96];
  std::snprintf(b, sizeof b, "/fakerccl_%s_%llu_%d.%s", c->tag.c_str(), seq, rank, kind);
  return dir() + b;
}

bool wait_for(const std::string &p, double seconds = 60.0) {
  const auto t0 = std::chrono::steady_clock::now();
  struct stat st;
  while (::stat(p.c_str(), &st) != 0) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return true;
}

bool write_file(const std::string &p, const void *data, size_t bytes) {
  const std::string tmp = p + ".tmp";
  FILE *f = std::fopen(tmp.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(data, 1, bytes, f) == bytes;
  std::fclose(f);
  return ok && std::rename(tmp.c_str(), p.c_str()) == 0;
}

bool read_file(const std::string &p, void *data, size_t bytes) {
  FILE *f = std::fopen(p.c_str(), "rb");
  if (!f) return false;
  const bool ok = std::fread(data, 1, bytes, f) == bytes;
  std::fclose(f);
  return ok;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
  std::random_device rd;
  std::memset(id, 0, sizeof(*id));
  for (int k = 0; k < 16; ++k) id->internal[k] = (char)(rd() & 0xff);
  return ncclSuccess;
}

static std::string hex_tag(const ncclUniqueId &id) {
  char b[40];
  for (int k = 0; k < 16; ++k) std::snprintf(b + 2 * k, 3, "%02x", (unsigned char)id.internal[k]);
  return b;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  ncclComm *c = new ncclComm();
  c->nranks = nranks;
  c->rank = rank;
  (void)hipGetDevice(&c->device);
  c->tag = hex_tag(id);
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comm, int ndev, const int *devlist) {
  if (!comm || ndev != 1) return ncclInvalidArgument;  // one device: the all-reduce is a copy
  ncclComm *c = new ncclComm();
  c->device = devlist ? devlist[0] : 0;
  c->tag = "local";
  comm[0] = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

const char *ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "fake rccl: success";
    case ncclInvalidArgument: return "fake rccl: invalid argument (float sum only)";
    case ncclSystemError: return "fake rccl: a peer never arrived (timeout) or file I/O failed";
    default: return "fake rccl: error";
  }
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t type, ncclRedOp_t op,
                           ncclComm_t c, hipStream_t stream) {
  if (!c || type != ncclFloat || op != ncclSum) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclSystemError;
  const size_t bytes = count * sizeof(float);
  std::vector<float> mine(count), sum(count, 0.0f), peer(count);
  if (hipMemcpy(mine.data(), send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return ncclSystemError;
  const unsigned long long seq = c->seq++;
  if (c->nranks > 1 && !write_file(path(c, seq, c->rank, "bin"), mine.data(), bytes)) return ncclSystemError;
  for (int r = 0; r < c->nranks; ++r) {
    const float *src = mine.data();
    if (r != c->rank) {
      const std::string p = path(c, seq, r, "bin");
      if (!wait_for(p) || !read_file(p, peer.data(), bytes)) return ncclSystemError;
      src = peer.data();
    }
    for (size_t k = 0; k < count; ++k) sum[k] = sum[k] + src[k];  // rank order, from +0
  }
  if (hipMemcpy(recv, sum.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return ncclSystemError;
  if (c->nranks > 1) {
    // Every rank acknowledges; a rank removes its data file once all have read it.
    const char one = 1;
    if (!write_file(path(c, seq, c->rank, "ack"), &one, 1)) return ncclSystemError;
    for (int r = 0; r < c->nranks; ++r)
      if (!wait_for(path(c, seq, r, "ack"))) return ncclSystemError;
    std::remove(path(c, seq, c->rank, "bin").c_str());
    if (seq > 0) std::remove(path(c, seq - 1, c->rank, "ack").c_str());  // every rank is past seq - 1
  }
  return ncclSuccess;
}

}  // extern "C"
