// fake_rccl.cpp -- TEST INFRASTRUCTURE: a loopback stand-in for the subset of
// RCCL that libcrossbow_sma calls, so that the library's multi-GPU paths run
// against the oracle on a box with ONE GPU.  Real RCCL refuses two ranks or
// two communicators on one device ("Duplicate GPU detected").  Two forms:
//
//  * one process per rank (cbx_init_rank, ncclCommInitRank): the send buffer
//    of every rank goes through a file under $FAKE_RCCL_DIR (default /tmp);
//  * one process, G communicators (cbx_init with G devices,
//    ncclCommInitAll(ndev > 1), the reference's own form,
//    executioncontext.c:185-201): the all-reduces issued between
//    ncclGroupStart and ncclGroupEnd are matched by their order on each
//    communicator, as in NCCL, and run at ncclGroupEnd.  An ungrouped call on
//    such a communicator is an error (real NCCL would deadlock on it).  A
//    group that holds only some ranks' calls (one thread per device, each
//    issuing its own communicator's collectives: cbx_set_enqueue_threads)
//    meets the other ranks' k-th calls at a rendezvous; the last to arrive
//    runs the collective for all, the others wait for it (60 s, then
//    ncclSystemError).
//
// Calls: ncclAllReduce, ncclReduceScatter, ncclAllGather (fp32; sum) and
// ncclBroadcast (fp32; cbx_resync_base).
// Each collective synchronises the stream it was given (so every kernel the
// library ordered before it has finished), sums the ranks' send buffers on
// the host, writes the result to every receive buffer with a blocking copy
// and returns.  Stream order is thereby preserved: everything the library
// enqueues afterwards sees the result.  Every file wait times out
// (ncclSystemError) instead of hanging.
//
// Summation order ($FAKE_RCCL_ORDER, read when the communicator is created):
//   "rank" (default): in rank order from +0, the oracle's order
//                     (oracle/sma_oracle.c), so results are bit-exact;
//   "ring":           as a ring all-reduce does it: the buffer is cut into
//                     chunks, the reduction of chunk c starts at rank
//                     (c + 1) mod G and walks the ring, and every rank then
//                     receives the same reduced chunk (the all-gather).  For
//                     G >= 3 this is NOT the oracle's order, so it exercises
//                     the stated G > 1 tolerance and the
//                     cross-rank identity of z (sma.c:168-174).
//
// $FAKE_RCCL_NOOP=1 (read when the communicator is created): every
// collective returns at once and moves nothing -- results are wrong.  Only
// for timing the host side of the library's enqueue without a collective's
// own cost (scripts/host_enqueue_multidev.py); no parity test sets it.
//
// Built by scripts/build_fake_rccl.sh as tests/native/libfakerccl.so; a
// variant of the library linked against it (libcrossbow_sma_fakerccl.so) is
// what tests/test_gpu_multirank.py and tests/test_gpu_multidevice.py load.
// Never linked into the product.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

struct Clique;

struct ncclComm {
  int nranks = 1;
  int rank = 0;
  int device = 0;
  bool ring = false;
  bool noop = false;  // $FAKE_RCCL_NOOP: collectives move nothing (host-side timing only)
  std::string tag;  // hex of the unique id
  unsigned long long seq = 0;
  unsigned long long rv_seq = 0;  // rendezvous calls on this communicator
  Clique *clique = nullptr;  // single-process communicators (ncclCommInitAll, ndev > 1)
};

struct Clique {
  std::vector<ncclComm *> comms;
  int live = 0;
  // Rendezvous of per-thread groups: the k-th call of every rank.
  struct Slot {
    std::vector<const void *> ops;  // PendingOp of each rank
    int have = 0, left = 0;
    bool done = false;
    int rc = 0;
  };
  std::mutex m;
  std::condition_variable cv;
  std::map<unsigned long long, Slot> rv;
};

namespace {

// Elements per ring chunk: small enough that a few-thousand-element test
// buffer spans several chunks, so every start rank occurs.
constexpr size_t kRingChunk = 1024;

bool noop_from_env() {
  const char *o = std::getenv("FAKE_RCCL_NOOP");
  return o && std::strcmp(o, "1") == 0;
}

bool ring_order_from_env() {
  const char *o = std::getenv("FAKE_RCCL_ORDER");
  return o && std::strcmp(o, "ring") == 0;
}

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

// sum[k] over the ranks' buffers src[0..G-1], in rank order from +0 or in
// the ring's order (see the header).
void reduce(const std::vector<const float *> &src, size_t count, bool ring, float *sum) {
  const int G = (int)src.size();
  if (!ring || G < 3) {
    for (size_t k = 0; k < count; ++k) sum[k] = 0.0f;
    for (int r = 0; r < G; ++r)
      for (size_t k = 0; k < count; ++k) sum[k] = sum[k] + src[r][k];
    return;
  }
  for (size_t c0 = 0, c = 0; c0 < count; c0 += kRingChunk, ++c) {
    const size_t c1 = std::min(count, c0 + kRingChunk);
    const int start = (int)((c + 1) % (size_t)G);
    for (size_t k = c0; k < c1; ++k) sum[k] = src[start][k];
    for (int j = 1; j < G; ++j) {
      const float *x = src[(start + j) % G];
      for (size_t k = c0; k < c1; ++k) sum[k] = sum[k] + x[k];
    }
  }
}

enum OpKind { kAllReduce = 0, kReduceScatter = 1, kAllGather = 2, kBroadcast = 3 };

// Floats of one rank's send buffer / receive buffer for a call with `count`
// (the NCCL argument: recvcount for reduce-scatter, sendcount for all-gather).
size_t send_elems(int kind, size_t count, int G) { return kind == kReduceScatter ? count * (size_t)G : count; }
size_t recv_elems(int kind, size_t count, int G) { return kind == kAllGather ? count * (size_t)G : count; }

// The collective over the ranks' host copies src[0..G-1] of their send
// buffers: what rank `rank` receives, into out (recv_elems floats).
//   all-reduce: the sum;  reduce-scatter: rank's slice of the sum (the ring
//   order, if on, is that of a ring all-reduce's reduce phase);  all-gather:
//   the concatenation in rank order;  broadcast: root's buffer.
void collective(int kind, const std::vector<const float *> &src, size_t count, bool ring, int rank, float *out,
                int root) {
  const int G = (int)src.size();
  if (kind == kBroadcast) {
    std::memcpy(out, src[root], count * sizeof(float));
    return;
  }
  if (kind == kAllGather) {
    for (int r = 0; r < G; ++r) std::memcpy(out + (size_t)r * count, src[r], count * sizeof(float));
    return;
  }
  const size_t n = send_elems(kind, count, G);
  std::vector<float> sum(n);
  reduce(src, n, ring, sum.data());
  const size_t off = kind == kReduceScatter ? (size_t)rank * count : 0;
  std::memcpy(out, sum.data() + off, count * sizeof(float));
}

struct PendingOp {
  int kind;
  const void *send;
  void *recv;
  size_t count;
  ncclComm *comm;
  hipStream_t stream;
  int root;
};

thread_local int g_depth = 0;
thread_local std::vector<PendingOp> g_ops;

// One grouped collective of a single-process clique: ops[r] is rank r's.
ncclResult_t run_clique(const std::vector<PendingOp *> &ops) {
  const int G = (int)ops.size();
  const int kind = ops[0]->kind;
  const size_t count = ops[0]->count;
  const size_t ns = send_elems(kind, count, G), nr = recv_elems(kind, count, G);
  std::vector<std::vector<float>> host(G, std::vector<float>(ns));
  std::vector<const float *> src(G);
  for (int r = 0; r < G; ++r) {
    if (ops[r]->count != count || ops[r]->kind != kind || ops[r]->root != ops[0]->root) return ncclInvalidArgument;
    if (hipSetDevice(ops[r]->comm->device) != hipSuccess) return ncclSystemError;
    if (hipStreamSynchronize(ops[r]->stream) != hipSuccess) return ncclSystemError;
    if (hipMemcpy(host[r].data(), ops[r]->send, ns * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
      return ncclSystemError;
    src[r] = host[r].data();
  }
  std::vector<float> out(nr);
  for (int r = 0; r < G; ++r) {
    collective(kind, src, count, ops[0]->comm->ring, r, out.data(), ops[0]->root);
    if (hipSetDevice(ops[r]->comm->device) != hipSuccess) return ncclSystemError;
    if (hipMemcpy(ops[r]->recv, out.data(), nr * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      return ncclSystemError;
  }
  return ncclSuccess;
}

// One rank's call of a clique collective whose other ranks' calls come from
// other threads: wait for all of them, the last one runs it.
ncclResult_t rendezvous(const PendingOp &op) {
  Clique *q = op.comm->clique;
  const int G = (int)q->comms.size();
  std::unique_lock<std::mutex> l(q->m);
  const unsigned long long key = op.comm->rv_seq++;
  Clique::Slot &s = q->rv[key];
  if (s.ops.empty()) s.ops.assign(G, nullptr);
  s.ops[op.comm->rank] = &op;
  if (++s.have == G) {
    std::vector<PendingOp *> coll(G);
    for (int r = 0; r < G; ++r) coll[r] = const_cast<PendingOp *>(static_cast<const PendingOp *>(s.ops[r]));
    l.unlock();
    const ncclResult_t rc = run_clique(coll);
    l.lock();
    s.rc = (int)rc;
    s.done = true;
    q->cv.notify_all();
  } else if (!q->cv.wait_for(l, std::chrono::seconds(60), [&] { return s.done; })) {
    return ncclSystemError;  // a rank never arrived
  }
  const ncclResult_t rc = (ncclResult_t)s.rc;
  if (++s.left == G) q->rv.erase(key);
  return rc;
}

// The per-rank (multi-process) collective through files.
ncclResult_t run_ranked(int kind, const void *send, void *recv, size_t count, ncclComm *c, hipStream_t stream,
                        int root) {
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclSystemError;
  const size_t ns = send_elems(kind, count, c->nranks), nr = recv_elems(kind, count, c->nranks);
  const size_t bytes = ns * sizeof(float);
  std::vector<std::vector<float>> host(c->nranks);
  std::vector<const float *> src(c->nranks);
  host[c->rank].resize(ns);
  if (hipMemcpy(host[c->rank].data(), send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return ncclSystemError;
  const unsigned long long seq = c->seq++;
  if (c->nranks > 1 && !write_file(path(c, seq, c->rank, "bin"), host[c->rank].data(), bytes)) return ncclSystemError;
  for (int r = 0; r < c->nranks; ++r) {
    if (r != c->rank) {
      host[r].resize(ns);
      const std::string p = path(c, seq, r, "bin");
      if (!wait_for(p) || !read_file(p, host[r].data(), bytes)) return ncclSystemError;
    }
    src[r] = host[r].data();
  }
  std::vector<float> out(nr);
  collective(kind, src, count, c->ring, c->rank, out.data(), root);
  if (hipMemcpy(recv, out.data(), nr * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return ncclSystemError;
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

ncclResult_t enqueue(int kind, const void *send, void *recv, size_t count, ncclDataType_t type, ncclComm_t c,
                     hipStream_t stream, int root = 0) {
  if (!c || type != ncclFloat || root < 0 || root >= c->nranks) return ncclInvalidArgument;
  if (c->noop) return ncclSuccess;
  if (c->clique) {
    if (g_depth == 0) return ncclInvalidUsage;
    g_ops.push_back(PendingOp{kind, send, recv, count, c, stream, root});
    return ncclSuccess;
  }
  return run_ranked(kind, send, recv, count, c, stream, root);
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
  c->ring = ring_order_from_env();
  c->noop = noop_from_env();
  (void)hipGetDevice(&c->device);
  c->tag = hex_tag(id);
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comm, int ndev, const int *devlist) {
  if (!comm || ndev < 1) return ncclInvalidArgument;
  Clique *q = ndev > 1 ? new Clique() : nullptr;
  for (int r = 0; r < ndev; ++r) {
    ncclComm *c = new ncclComm();
    c->nranks = ndev;
    c->rank = r;
    c->device = devlist ? devlist[r] : r;
    c->ring = ring_order_from_env();
    c->noop = noop_from_env();
    c->tag = "local";
    c->clique = q;
    if (q) q->comms.push_back(c);
    comm[r] = c;
  }
  if (q) q->live = ndev;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int *count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = comm->nranks;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int *rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  Clique *q = comm->clique;
  delete comm;
  if (q && --q->live == 0) delete q;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++g_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (g_depth <= 0) return ncclInvalidUsage;
  if (--g_depth > 0) return ncclSuccess;
  std::vector<PendingOp> ops;
  ops.swap(g_ops);
  // NCCL matches the grouped calls of a clique by their order on each
  // communicator: the k-th call on every rank forms the k-th collective.
  std::vector<bool> done(ops.size(), false);
  // A clique only some of whose ranks are in this group: per-thread groups,
  // every call goes to the rendezvous in order.
  std::map<Clique *, std::vector<bool>> ranks;
  for (const PendingOp &op : ops) {
    auto &v = ranks[op.comm->clique];
    v.resize(op.comm->clique->comms.size(), false);
    v[op.comm->rank] = true;
  }
  for (size_t a = 0; a < ops.size(); ++a) {
    const auto &v = ranks[ops[a].comm->clique];
    if (std::find(v.begin(), v.end(), false) == v.end()) continue;
    const ncclResult_t r = rendezvous(ops[a]);
    if (r != ncclSuccess) return r;
    done[a] = true;
  }
  for (size_t a = 0; a < ops.size(); ++a) {
    if (done[a]) continue;
    Clique *q = ops[a].comm->clique;
    const int G = (int)q->comms.size();
    std::vector<PendingOp *> coll(G, nullptr);
    int have = 0;
    for (size_t b = a; b < ops.size() && have < G; ++b) {
      if (done[b] || ops[b].comm->clique != q || coll[ops[b].comm->rank]) continue;
      coll[ops[b].comm->rank] = &ops[b];
      done[b] = true;
      ++have;
    }
    if (have != G) return ncclInvalidUsage;  // a rank of the clique did not take part
    const ncclResult_t r = run_clique(coll);
    if (r != ncclSuccess) return r;
  }
  return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "fake rccl: success";
    case ncclInvalidArgument: return "fake rccl: invalid argument (float sum only)";
    case ncclInvalidUsage: return "fake rccl: invalid usage (ungrouped call on a multi-device clique, or a rank missing)";
    case ncclSystemError: return "fake rccl: a peer never arrived (timeout) or file I/O failed";
    default: return "fake rccl: error";
  }
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t type, ncclRedOp_t op,
                           ncclComm_t c, hipStream_t stream) {
  if (op != ncclSum) return ncclInvalidArgument;
  return enqueue(kAllReduce, send, recv, count, type, c, stream);
}

ncclResult_t ncclReduceScatter(const void *send, void *recv, size_t recvcount, ncclDataType_t type, ncclRedOp_t op,
                               ncclComm_t c, hipStream_t stream) {
  if (op != ncclSum) return ncclInvalidArgument;
  return enqueue(kReduceScatter, send, recv, recvcount, type, c, stream);
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t sendcount, ncclDataType_t type, ncclComm_t c,
                           hipStream_t stream) {
  return enqueue(kAllGather, send, recv, sendcount, type, c, stream);
}

ncclResult_t ncclBroadcast(const void *send, void *recv, size_t count, ncclDataType_t type, int root, ncclComm_t c,
                           hipStream_t stream) {
  return enqueue(kBroadcast, send, recv, count, type, c, stream, root);
}

}  // extern "C"
