// sync_steps.hip -- the barrier steps behind cbx_synchronise and
// cbx_synchronise_staged: the SMA step (clib-multigpu/synch/sma.c:13-231,
// synch/common.c:3-57) fused at G = 1 and as kernel A / collective / kernel B
// per bucket at G > 1, its peer-read and reduce-scatter forms, the pipelined
// host-staged step, synchronous SGD (synch/synchronoussgd.c:13-106), and the
// stream-order check that verifies the bucket pipeline's ordering.
#include "context_internal.h"

namespace cbx::host {

// ---------------------------------------------------------------------------
// SMA step, clib-multigpu/synch/sma.c:13-231
// ---------------------------------------------------------------------------
int build_args(cbx_context *c, Device &d, int first, cbx::SmaArgs &a, int *copies) {
  std::memset(&a, 0, sizeof(a));
  int k = 0;
  int cp = 0;
  for (int id : d.replicas) {  // increasing id order, sma.c:69
    if (id < first || !c->locked[id]) continue;
    if (k >= cbx::kMaxReplicas)
      return fail(CBX_ERR_UNSUPPORTED, "more than %d locked replicas on one device", cbx::kMaxReplicas);
    Replica &r = *c->replicas[id];
    a.s[k] = reinterpret_cast<const cbx::v4f *>(replica_dev(d, r, CBX_BUF_DIFF));
    a.w[k] = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_DATA));
    if (r.conf.copy) cp++;  // sma.c:113-120
    ++k;
  }
  a.nrep = k;
  a.z = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_DATA));
  a.last = c->has_last ? reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_LAST)) : nullptr;
  a.acc = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_GRADIENT));
  a.D = reinterpret_cast<const cbx::v4f *>(base_dev(c, d, CBX_BUF_DIFF));
  a.ctrl_out = base_ctrl(d, CBX_BUF_GRADIENT);
  a.ctrl_in = base_ctrl(d, CBX_BUF_DIFF);
  a.n4 = c->n4;
  a.alpha = c->model.conf.alpha;  // sma.c:33, theModel's conf
  a.copies = (float)cp;
  *copies = cp;
  return CBX_OK;
}

cbx::SmaArgs offset_args(const cbx::SmaArgs &a, int64_t start4, int64_t len4) {
  cbx::SmaArgs b = a;
  for (int r = 0; r < a.nrep; ++r) {
    b.s[r] = a.s[r] + start4;
    b.w[r] = a.w[r] + start4;
  }
  b.z = a.z + start4;
  if (a.last) b.last = a.last + start4;
  b.acc = a.acc + start4;
  b.D = a.D + start4;
  b.n4 = len4;
  return b;
}

// The reference records synched / base->updated (sma.c:177,204) and one
// replica->updated per replica (sma.c:115,222) at points that, in this
// pipeline, are all the same: the end of the step on the sync stream.  One
// event per device stands for all of them (cbx_step_event); each extra
// record is a marker packet costing GPU time between steps.  With timing
// on, the step's last dispatch already timestamps a ring event at its end;
// that event is the step event and no marker is added.
int finish_step(cbx_context *c) {
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    if (c->timing && !d.ring.empty()) {
      const int prev = (d.ring_pos + Device::kRing - 1) % Device::kRing;
      d.step_event = d.ring[(size_t)prev * 4 + (d.ring_split[prev] == 0 ? EV_A : EV_B)];
    } else {
      if (!d.synched_by_dispatch) HIP_TRY(hipEventRecord(d.synched, d.stream));
      d.step_event = d.synched;
    }
    d.synched_by_dispatch = false;
  }
  return CBX_OK;
}

// The stop event for a step's LAST dispatch: the ring event `ev` when timing,
// else `synched`, which the dispatch then completes itself: no marker packet
// between steps (a marker cost ~3 us per fused step, scripts/step_overhead.py).
hipEvent_t step_stop_event(cbx_context *c, Device &d, int ev) {
  if (c->timing && !d.ring.empty()) return d.ring[(size_t)d.ring_pos * 4 + ev];
  d.synched_by_dispatch = true;
  return d.synched;
}

// The communicators, created on first use where cbx_init did not create them:
// a one-rank communicator at G = 1 (cbx_set_force_split, S-SGD's split path,
// BN averaging), so a single-GPU host exercises kernel A + RCCL + kernel B;
// and the ncclCommInitAll clique of a device selection that repeats a device
// (a one-GPU rehearsal of the single-process form), which real RCCL refuses:
// there only the peer-read form (no communicator) runs.
int ensure_comms(cbx_context *c) {
  if (c->devs[0].comm != nullptr || (c->per_rank && c->G > 1)) return CBX_OK;
  std::vector<ncclComm_t> comms(c->devs.size());
  std::vector<int> ids;
  for (Device &d : c->devs) ids.push_back(d.hip_id);
  HIP_TRY(hipSetDevice(ids[0]));
  ncclResult_t r = ncclCommInitAll(comms.data(), (int)ids.size(), ids.data());
  if (r != ncclSuccess)
    return fail(CBX_ERR_RCCL, "ncclCommInitAll over %d device(s): %s%s", (int)ids.size(), ncclGetErrorString(r),
                ids.size() > 1 ? " (RCCL takes each device once; the peer-read all-reduce needs no communicator)" : "");
  for (size_t k = 0; k < comms.size(); ++k) c->devs[k].comm = comms[k];
  return CBX_OK;
}

// ---------------------------------------------------------------------------
// Peer-read all-reduce, single process over G devices (sma_internal.h,
// PeerArgs): the collective of SplitStep below becomes R, a kernel on every
// device g that sums shard g of the bucket from every device's acc into g's
// own D (device order from +0), and kernel B reads each shard of D from its
// owner.  Per bucket k, on device g:
//   A_g(k)  ->  R_g(k) waits A_h(k) of EVERY device h  ->  B_g(k) waits R_h(k) of every h
// One bucket: all three in order on the sync stream.  Buckets: A on the
// A streams, R on the comm stream, B on the sync stream, exactly as the
// RCCL all-reduce's pipeline (modes 0 and 1, wait strides, groups), so R(k)
// and B(k) overlap A(k+1).  Cross-step safety, the RCCL form's plus the
// peers': A_h(k) of the next step overwrites acc_h(k), which R_g(k) of this
// step reads, and follows B_h(k) (stream order, or its cross-step wait),
// which waited for every R_g(k); R_g(k) of the next step overwrites D_g(k),
// which B_h(k) of this step reads, and waits for every A_h(k) of the next
// step, which follow B_h(k).
// ---------------------------------------------------------------------------
int ensure_peer_access(cbx_context *c) {
  if (c->peer_ready) return CBX_OK;
  for (Device &a : c->devs)
    for (Device &b : c->devs) {
      if (a.hip_id == b.hip_id) continue;  // one device reads itself directly
      int can = 0;
      HIP_TRY(hipDeviceCanAccessPeer(&can, a.hip_id, b.hip_id));
      if (!can) return fail(CBX_ERR_UNSUPPORTED, "device %d cannot access device %d's memory", a.hip_id, b.hip_id);
      HIP_TRY(hipSetDevice(a.hip_id));
      hipError_t e = hipDeviceEnablePeerAccess(b.hip_id, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      else if (e != hipSuccess) return fail(CBX_ERR_HIP, "hipDeviceEnablePeerAccess(%d -> %d): %s", a.hip_id, b.hip_id, hipGetErrorString(e));
    }
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    if (!d.peer_a) HIP_TRY(hipEventCreateWithFlags(&d.peer_a, hipEventDisableTiming));
    if (!d.peer_r) HIP_TRY(hipEventCreateWithFlags(&d.peer_r, hipEventDisableTiming));
  }
  c->peer_ready = true;
  return CBX_OK;
}

// ---------------------------------------------------------------------------
// The same form with one process per GPU (cbx_init_rank): the other ranks'
// arenas through IPC handles (dmabuf), and the cross-process order through
// flags in a shared host page instead of events (cbx_context::PeerIpc in
// context_internal.h).  The pipeline is SplitStep's, unchanged: where the
// single-process form waits on device h's event of bucket b, a rank waits
// for rank h's flag of bucket b to reach this step's sequence number.
// ---------------------------------------------------------------------------
namespace {

struct PeerBlob {
  uint32_t magic;
  int32_t rank, G, pad;
  int64_t n4;
  uint64_t slot_bytes;
  hipIpcMemHandle_t acc, D;  // the base model's acc and D slots (control block first)
  char shm[64];              // rank 0's: the flag page
};
static_assert(sizeof(PeerBlob) <= CBX_PEER_BLOB_BYTES, "peer blob size");
constexpr uint32_t kPeerMagic = 0x50584243u;  // "CBXP"

int map_flag_page(cbx_context *c, bool create) {
  auto &p = c->ipc;
  p.page_bytes = ((size_t)c->G * kIpcRankWords * sizeof(uint64_t) + 4095) / 4096 * 4096;
  const int fd = shm_open(p.shm_name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return fail(CBX_ERR_IO, "shm_open(%s): %s", p.shm_name, strerror(errno));
  p.owner = create;
  if (create && ftruncate(fd, (off_t)p.page_bytes) != 0) {
    close(fd);
    return fail(CBX_ERR_IO, "ftruncate(%s): %s", p.shm_name, strerror(errno));
  }
  void *m = mmap(nullptr, p.page_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return fail(CBX_ERR_IO, "mmap(%s): %s", p.shm_name, strerror(errno));
  p.page = m;  // a new object reads zero: no flag set yet
  HIP_TRY(hipSetDevice(c->devs[0].hip_id));
  HIP_TRY(hipHostRegister(p.page, p.page_bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&p.dpage), p.page, 0));
  return CBX_OK;
}

std::string fmt_msg(const char *f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

volatile uint64_t *host_word(cbx_context *c, int rank, int kind, int64_t b) {
  return static_cast<volatile uint64_t *>(c->ipc.page) + ipc_word(rank, kind, b);
}

// A step that failed part-way, or one refused because another rank's failed:
// no other rank may wait on this one's flags forever, and none may run
// another step against it.  The host raises the rank's broken word (every
// rank checks the page before its next collective step, peer_guard, and each
// step's poison check after its last kernel B reads it, kIpcPoison), and only
// then writes the release value into every flag word of this rank (a peer
// stream waiting on one goes on: whatever such a wait lets a kernel read, the
// broken word was set before it).  The
// failed step may have queued writes of its sequence number that land later
// and would overwrite the release (the GPU runs behind the host), so the
// release is also queued behind them, on every stream that carries flag
// writes, for the words of the `nb` buckets in use: on each stream the
// release lands last.  No stream is synchronised here: one may wait on a
// peer's flag that never comes (then its own earlier writes never land either).
// `broken` false: teardown (every rank is done with every step) or a failed
// import (no step ran); the flags go, no rank's steps are refused for it.
void release_flags(cbx_context *c, int64_t nb, bool broken = true) {
  auto &p = c->ipc;
  if (!p.page) return;
  if (broken) {
    *host_word(c, p.me, kIpcBroken, 0) = 1;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  for (int64_t b = 0; b < kIpcMaxBuckets; ++b) {
    *host_word(c, p.me, kIpcA, b) = kIpcRelease;
    *host_word(c, p.me, kIpcR, b) = kIpcRelease;
  }
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  p.released = true;
  if (nb <= 0 || !p.dpage) return;
  Device &d = c->devs[0];
  (void)hipSetDevice(d.hip_id);
  for (hipStream_t s : {d.stream, d.comm_stream, d.a_stream, d.a_stream2})
    for (int64_t b = 0; s && b < std::min(nb, kIpcMaxBuckets); ++b)
      for (int kind : {kIpcA, kIpcR})
        (void)hipStreamWriteValue64(s, p.dpage + ipc_word(p.me, kind, b), kIpcRelease, 0);
}

// The first rank whose broken word is set (a step of it failed part-way or
// was refused), or -1.
int first_broken_rank(cbx_context *c) {
  for (int h = 0; h < c->G; ++h)
    if (*host_word(c, h, kIpcBroken, 0) != 0) return h;
  return -1;
}

bool any_rank_broken(cbx_context *c) { return first_broken_rank(c) >= 0; }

// Polls every stream of every local device until it drains or `seconds`
// pass (a stream may wait on a flag of a rank that never arrives).
bool drain_polled(cbx_context *c, int seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  for (Device &d : c->devs) {
    (void)hipSetDevice(d.hip_id);
    for (hipStream_t s : {d.stream, d.comm_stream, d.a_stream, d.a_stream2}) {
      hipError_t e = hipErrorNotReady;
      while (s && (e = hipStreamQuery(s)) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - t0 < std::chrono::seconds(seconds))
        sched_yield();
      if (s && e == hipErrorNotReady) return false;
    }
  }
  return true;
}

}  // namespace

int peer_guard(cbx_context *c, const char *what) {
  auto &p = c->ipc;
  if (!p.ready) return CBX_OK;
  const int h = first_broken_rank(c);
  if (h < 0 && !p.broken) return CBX_OK;
  // A rank already waiting on this one's flags of a step this rank will now
  // never run must go on: release them, whatever this call was.
  if (!p.released) release_flags(c, p.max_nb);
  p.broken = true;
  const uint64_t poisoned = *host_word(c, p.me, kIpcPoison, 0);
  return fail(CBX_ERR_STATE, "%s refused: a per-rank peer-read step failed part-way earlier on this or another rank "
              "(rank %d's broken word is set; flags released)%s; z / last may differ across ranks, so every "
              "collective step is refused until cbx_resync_base", what, h < 0 ? p.me : h,
              poisoned ? fmt_msg(", and this rank's step %llu read released flags",
                                 (unsigned long long)poisoned).c_str() : "");
}

int peer_wait_check(cbx_context *c) {
  auto &p = c->ipc;
  if (!p.ready) return CBX_OK;
  const uint64_t poisoned = *host_word(c, p.me, kIpcPoison, 0);
  if (poisoned == 0) return CBX_OK;
  if (!p.released) release_flags(c, p.max_nb);
  p.broken = true;
  return fail(CBX_ERR_STATE, "peer-read step %llu on rank %d ran after a rank's step failed part-way (the check "
              "after its last kernel B found a broken word): this rank's z / last are undefined from that step on, "
              "and every collective step is refused until cbx_resync_base", (unsigned long long)poisoned, p.me);
}

// Every rank calls it (the broadcast and both barriers are collectives).  A
// rank that knows of a failure releases its flags first, so every rank's
// queued steps drain; the page is cleared only once every rank has drained
// (barrier 1), and no rank starts a step before every rank has cleared its
// words (barrier 2): a step's first wait must not pass on a stale release.
int resync_base(cbx_context *c, int root) {
  if (root < 0 || root >= c->G) return fail(CBX_ERR_INVALID, "cbx_resync_base: root %d out of range (G %d)", root, c->G);
  if (c->G == 1) return CBX_OK;
  TRY(flush_task_waits(c));
  auto &p = c->ipc;
  if (p.ready && !p.released) {
    bool known = p.broken || any_rank_broken(c);
    for (int h = 0; h < c->G && !known; ++h) known = *host_word(c, h, kIpcPoison, 0) != 0;
    if (known) release_flags(c, p.max_nb);
  }
  if (!drain_polled(c, 60))
    return fail(CBX_ERR_STATE, "cbx_resync_base: this rank's streams are still busy after 60 s (a rank that never "
                "called cbx_resync_base?)");
  TRY(ensure_comms(c));
  auto barrier = [&]() -> int {
    NCCL_TRY(ncclGroupStart());
    for (Device &d : c->devs) {
      HIP_TRY(hipSetDevice(d.hip_id));
      float *x = base_ctrl(d, CBX_BUF_DIFF);  // scratch: every step rewrites D's control block
      NCCL_TRY(ncclAllReduce(x, x, 1, ncclFloat, ncclSum, d.comm, d.stream));
    }
    NCCL_TRY(ncclGroupEnd());
    if (!drain_polled(c, 60))
      return fail(CBX_ERR_STATE, "cbx_resync_base: a rank never reached the barrier (60 s)");
    return CBX_OK;
  };
  NCCL_TRY(ncclGroupStart());
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    const size_t count = (size_t)c->n4 * 4;
    float *z = base_dev(c, d, CBX_BUF_DATA);
    NCCL_TRY(ncclBroadcast(z, z, count, ncclFloat, root, d.comm, d.stream));
    if (c->has_last) {
      float *l = base_dev(c, d, CBX_BUF_LAST);
      NCCL_TRY(ncclBroadcast(l, l, count, ncclFloat, root, d.comm, d.stream));
    }
  }
  NCCL_TRY(ncclGroupEnd());
  TRY(barrier());
  if (p.ready) {
    for (int64_t b = 0; b < kIpcMaxBuckets; ++b) {
      *host_word(c, p.me, kIpcA, b) = 0;
      *host_word(c, p.me, kIpcR, b) = 0;
    }
    *host_word(c, p.me, kIpcPoison, 0) = 0;
    *host_word(c, p.me, kIpcBroken, 0) = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    TRY(barrier());
    p.seq = 0;  // every rank's next step in the form is number 1 again
    p.broken = false;
    p.released = false;
  }
  for (Device &d : c->devs) {
    d.cross_valid = false;
    d.span_last = -1;
  }
  c->foreign_ops.fetch_add(1, std::memory_order_acq_rel);
  return CBX_OK;
}

int peer_export(cbx_context *c, void *blob, size_t *bytes) {
  if (!c->manager) return fail(CBX_ERR_STATE, "cbx_peer_export: set the model manager first");
  if (!c->per_rank || c->G < 2)
    return fail(CBX_ERR_UNSUPPORTED, "cbx_peer_export: one process per GPU with G > 1 only (one process over "
                "every device reaches its peers directly)");
  if (c->G > cbx::kMaxDevices) return fail(CBX_ERR_UNSUPPORTED, "the peer-read all-reduce takes at most %d ranks",
                                           cbx::kMaxDevices);
  if (!blob || !bytes) return fail(CBX_ERR_INVALID, "cbx_peer_export: null blob");
  Device &d = c->devs[0];
  if (d.stride > kIpcMaxSlotBytes)
    return fail(CBX_ERR_UNSUPPORTED, "the per-rank peer-read form maps at most %zu MiB per buffer (%zu asked): ROCm "
                "7.0's IPC keeps an allocation's size in 32 bits, and an open of 2 GiB or more never returns",
                kIpcMaxSlotBytes >> 20, d.stride >> 20);
  HIP_TRY(hipSetDevice(d.hip_id));
  if (!d.xslot[0]) {
    // acc and D move out of the arena into allocations of their own, which
    // is all the other ranks map (contents kept: the step may be mid-run)
    for (hipStream_t s : {d.stream, d.comm_stream, d.a_stream, d.a_stream2})
      if (s) HIP_TRY(hipStreamSynchronize(s));
    char *x[2] = {nullptr, nullptr};
    for (int k = 0; k < 2; ++k) {
      hipError_t e = hipMalloc(reinterpret_cast<void **>(&x[k]), d.stride);
      if (e == hipSuccess) e = hipMemcpy(x[k], d.arena + (size_t)(k + 1) * d.stride, d.stride, hipMemcpyDeviceToDevice);
      if (e != hipSuccess) {
        for (char *p : x)
          if (p) (void)hipFree(p);
        return fail(CBX_ERR_HIP, "cbx_peer_export: the acc / D slots: %s", hipGetErrorString(e));
      }
    }
    d.xslot[0] = x[0];
    d.xslot[1] = x[1];
    c->foreign_ops.fetch_add(1, std::memory_order_acq_rel);  // a cross-step pipeline rejoins
  }
  PeerBlob pb;
  std::memset(&pb, 0, sizeof(pb));
  pb.magic = kPeerMagic;
  pb.rank = d.g;
  pb.G = c->G;
  pb.n4 = c->n4;
  pb.slot_bytes = d.stride;
  HIP_TRY(hipIpcGetMemHandle(&pb.acc, d.xslot[0]));
  HIP_TRY(hipIpcGetMemHandle(&pb.D, d.xslot[1]));
  if (d.g == 0 && !c->ipc.page) {
    std::snprintf(c->ipc.shm_name, sizeof(c->ipc.shm_name), "/cbx_peer_%d_%llx", (int)getpid(),
                  (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
    TRY(map_flag_page(c, true));
  }
  if (d.g == 0) std::memcpy(pb.shm, c->ipc.shm_name, sizeof(pb.shm));
  std::memset(blob, 0, CBX_PEER_BLOB_BYTES);
  std::memcpy(blob, &pb, sizeof(pb));
  *bytes = CBX_PEER_BLOB_BYTES;
  return CBX_OK;
}

int peer_import(cbx_context *c, const void *blobs, int nranks) {
  auto &p = c->ipc;
  if (p.ready) return fail(CBX_ERR_STATE, "cbx_peer_import: already imported");
  if (!c->manager || !c->per_rank || c->G < 2) return fail(CBX_ERR_STATE, "cbx_peer_import: call cbx_peer_export first");
  if (!blobs || nranks != c->G) return fail(CBX_ERR_INVALID, "cbx_peer_import: need the blobs of all %d ranks", c->G);
  Device &d = c->devs[0];
  std::vector<PeerBlob> pb(nranks);
  for (int h = 0; h < nranks; ++h) {
    std::memcpy(&pb[h], static_cast<const char *>(blobs) + (size_t)h * CBX_PEER_BLOB_BYTES, sizeof(PeerBlob));
    if (pb[h].magic != kPeerMagic || pb[h].rank != h || pb[h].G != c->G || pb[h].n4 != c->n4 ||
        pb[h].slot_bytes != d.stride)
      return fail(CBX_ERR_INVALID, "cbx_peer_import: blob %d is not rank %d's of this job (rank %d, G %d, %lld "
                  "float4s)", h, h, pb[h].rank, pb[h].G, (long long)pb[h].n4);
  }
  p.me = d.g;
  if (p.me != 0) {
    std::memcpy(p.shm_name, pb[0].shm, sizeof(p.shm_name));
    p.shm_name[sizeof(p.shm_name) - 1] = 0;
    TRY(map_flag_page(c, false));
  }
  if (!p.page) return fail(CBX_ERR_STATE, "cbx_peer_import: rank 0 exported no flag page");
  p.mapped.assign(2 * (size_t)nranks, nullptr);
  p.acc.assign(nranks, nullptr);
  p.acc_ctrl.assign(nranks, nullptr);
  p.D.assign(nranks, nullptr);
  HIP_TRY(hipSetDevice(d.hip_id));
  // The ranks open the others' handles one rank at a time; the others wait
  // for the opener's "opened" word (a stream wait on the page, then
  // hipStreamSynchronize).  The exporter's side of an open is served by a
  // thread of the exporter's runtime (its IPC socket server), whatever the
  // exporter's own threads do, so this order is not what makes an open
  // complete: opens of a buffer of 2 GiB or more never complete under ROCm
  // 7.0 (kIpcMaxSlotBytes), and export refuses those.  The
  // order is kept because it was what the round-4 probes and tests ran, and
  // it costs the import a few milliseconds per rank.
  // A rank that never takes its turn (it failed before, or died) must not
  // park the others forever: 120 s after the import began (it takes
  // seconds) a timer thread writes every awaited word itself, and the
  // import fails.
  hipStream_t park = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&park, hipStreamNonBlocking));
  std::string err;
  std::atomic<int> waiting_for{-1};
  std::atomic<bool> finished{false}, timed_out{false};
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
  std::thread timer([&] {
    while (!finished.load(std::memory_order_acquire)) {
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      const int w = waiting_for.load(std::memory_order_acquire);
      if (w >= 0 && std::chrono::steady_clock::now() > deadline) {
        timed_out.store(true, std::memory_order_release);
        *host_word(c, w, kIpcOpened, 0) = kIpcRelease;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
      }
    }
  });
  for (int r = 0; r < nranks; ++r) {
    if (r != p.me) {
      waiting_for.store(r, std::memory_order_release);
      hipError_t e = hipStreamWaitValue64(park, p.dpage + ipc_word(r, kIpcOpened, 0), 1, hipStreamWaitValueGte, ~0ull);
      if (e == hipSuccess) e = hipStreamSynchronize(park);
      waiting_for.store(-1, std::memory_order_release);
      if (e != hipSuccess && err.empty()) err = fmt_msg("waiting for rank %d's turn: %s", r, hipGetErrorString(e));
      if (timed_out.load(std::memory_order_acquire) && err.empty())
        err = fmt_msg("rank %d had not opened its handles 120 s into the import", r);
      continue;
    }
    if (p.me == 0 && c->fault_ipc_stall_s > 0) {
      // Fault injection: stuck where the opens run, as a thread inside
      // hipIpcOpenMemHandle would be (bounded, in 1 s sleeps).
      for (int s = 0; s < c->fault_ipc_stall_s; ++s) std::this_thread::sleep_for(std::chrono::seconds(1));
    }
    if (c->fault_ipc_open_fail == p.me && err.empty())
      err = fmt_msg("fault injection: rank %d's opens fail ($CBX_FAULT_IPC_OPEN_FAIL)", p.me);
    for (int h = 0; h < nranks && err.empty(); ++h) {
      char *slot[2] = {d.xslot[0], d.xslot[1]};
      for (int k = 0; k < 2 && h != p.me; ++k) {
        void *m = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&m, k == 0 ? pb[h].acc : pb[h].D, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
          err = fmt_msg("hipIpcOpenMemHandle(rank %d's %s): %s", h, k == 0 ? "acc" : "D", hipGetErrorString(e));
          break;
        }
        p.mapped[2 * (size_t)h + k] = slot[k] = static_cast<char *>(m);
      }
      if (!err.empty()) break;
      const size_t data = (size_t)cbx::kCtrlFloats * sizeof(float);  // the control block comes first
      p.acc[h] = reinterpret_cast<const cbx::v4f *>(slot[0] + data);
      p.acc_ctrl[h] = reinterpret_cast<const float *>(slot[0]);
      p.D[h] = reinterpret_cast<const cbx::v4f *>(slot[1] + data);
    }
    // The next rank's turn, success (1) or not (2): either satisfies its wait.
    *host_word(c, p.me, kIpcOpened, 0) = err.empty() ? 1 : 2;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  finished.store(true, std::memory_order_release);
  timer.join();
  (void)hipStreamDestroy(park);
  // Every rank's word is final here (this rank waited for each one's turn):
  // the import succeeds on every rank or on none, so no rank steps in the
  // form, or has its collective steps refused, because of another's failed
  // import (cbx_peer_import's contract; dist.setup_peer also agrees).
  for (int h = 0; h < nranks && err.empty(); ++h)
    if (*host_word(c, h, kIpcOpened, 0) != 1)
      err = fmt_msg("rank %d's import failed or timed out", h);
  if (!err.empty()) {
    peer_close(c);
    return fail(CBX_ERR_HIP, "cbx_peer_import: %s", err.c_str());
  }
  p.ready = true;
  return CBX_OK;
}

void peer_close(cbx_context *c) {
  auto &p = c->ipc;
  if (!p.page && p.mapped.empty()) return;
  Device &d = c->devs[0];
  (void)hipSetDevice(d.hip_id);
  // At most 60 s in all: a peer that died mid-step leaves this rank's streams
  // waiting on its flags, and a rank that died never arrives on the page.
  auto t0 = std::chrono::steady_clock::now();
  auto in_time = [&] { return std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60); };
  auto drain = [&] {  // polled, not synchronised, so the deadline holds
    bool ok = true;
    for (hipStream_t s : {d.stream, d.comm_stream, d.a_stream, d.a_stream2}) {
      hipError_t e = hipErrorNotReady;
      while (s && (e = hipStreamQuery(s)) == hipErrorNotReady && in_time()) sched_yield();
      if (s && e == hipErrorNotReady) ok = false;
    }
    return ok;
  };
  bool drained = true;
  if (p.page) {
    // done with the others' memory (also when this rank's import failed, so
    // a rank whose import succeeded does not wait for it in vain)
    drained = drain();
    if (!drained) {
      // This rank's streams wait on flags a peer will never write (it died
      // mid-step): write the release into every rank's words on its behalf
      // (the page is shared), so the waits end and the streams drain; the
      // broken word first, so a step that the release lets run is reported
      // by its poison check.
      *host_word(c, p.me, kIpcBroken, 0) = 1;
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      for (int h = 0; h < c->G; ++h)
        for (int64_t b = 0; b < kIpcMaxBuckets; ++b) {
          *host_word(c, h, kIpcA, b) = kIpcRelease;
          *host_word(c, h, kIpcR, b) = kIpcRelease;
        }
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      t0 = std::chrono::steady_clock::now() - std::chrono::seconds(50);  // 10 s more
      drained = drain();
    }
    if (drained) *host_word(c, p.me, kIpcDone, 0) = 1;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  bool met = true;  // every rank said it is done with every step
  if (p.ready && drained) {
    // Every rank's streams must be done with this rank's memory (and this
    // rank with theirs) before any buffer goes: drained above, then meet the
    // others on the page.
    for (int h = 0; h < c->G; ++h) {
      while (*host_word(c, h, kIpcDone, 0) == 0 && in_time()) sched_yield();
      met = met && *host_word(c, h, kIpcDone, 0) != 0;
    }
  }
  if (!drained) {
    // Streams still queued against the others' memory: unmapping it (or the
    // pinned page their waits read) under them would fault the device.  Leak
    // the mappings and the page instead; the process is going down anyway.
    // The name goes all the same: unlinking a mapped, pinned
    // object only removes /dev/shm's entry, so no run leaves one behind.
    release_flags(c, 0);
    if (p.owner) shm_unlink(p.shm_name);
    p.mapped.clear();
    p.page = nullptr;
    p.dpage = nullptr;
    p.ready = false;
    return;
  }
  for (char *m : p.mapped)
    if (m) (void)hipIpcCloseMemHandle(m);
  p.mapped.clear();
  if (p.page) {
    // A rank still stepping when the meeting gave up must not take what it
    // reads next for a step's data: then the release marks this rank broken.
    release_flags(c, 0, !met);
    (void)hipHostUnregister(p.page);
    munmap(p.page, p.page_bytes);
    if (p.owner) shm_unlink(p.shm_name);
  }
  p.page = nullptr;
  p.dpage = nullptr;
  p.ready = false;
}

// Float4s per device shard of a peer-read bucket of `len4` float4s: whole
// kPadFloat4 units, so a wave's float4s never straddle two owners.
inline int64_t peer_shard4(int64_t len4, int G) {
  const int64_t pad = cbx::kPadFloat4;
  return ((len4 + G - 1) / G + pad - 1) / pad * pad;
}

// ---------------------------------------------------------------------------
// The split SMA step (G > 1, or forced at G = 1): kernel A, the collective of
// acc (+ control block), kernel B.  With one bucket everything runs in order
// on the sync stream.  With nb > 1 buckets the collective runs on a second
// stream:
//   stream      : A(0) A(1) [wait red(0)] B(0) A(2) [wait red(1)] B(1) ...
//   comm_stream :      [wait acc(0)] AR(0) [wait acc(1)] AR(1) ...
// so kernel A of bucket k+1 overlaps the xGMI collective of bucket k.
// Cross-step mode (cbx_set_pipeline_mode 1): kernels A on a_stream, B on the
// sync stream.  A(k) waits only for B(k) of the previous step, so the next
// step's first buckets run while this step's last collectives are still on
// the link:
//   a_stream    : [wait b(0)'] A(0) [wait b(1)'] A(1) ...
//   comm_stream : [wait acc(0)] AR(0) [wait acc(1)] AR(1) ...
//   stream      : [wait red(0)] B(0) [wait red(1)] B(1) ...
// A step joins the whole sync stream instead when anything else was enqueued
// since the last cross-pipelined step (foreign_ops).
// Per-bucket events ride on the kernels' own dispatch packets (stop event)
// instead of a separate hipEventRecord marker, which left a ~10 us gap on the
// sync stream per bucket: -2 to -8 % per step (round 1, dispatch_event_ab:
// profiles/r01/dispatch_event_ab.json).  Mode 1: A(k) waits for
// B(k + stride - 1) of the last step once per `stride` buckets (it implies
// B(k..): same stream).  Each satisfied cross-queue wait still costs the
// waiting queue ~10 us; fewer waits trade that for less cross-step overlap
// (cbx_set_cross_wait_stride).
// ---------------------------------------------------------------------------
struct SplitStep {
  cbx_context *c;
  std::vector<cbx::SmaArgs> &args;
  bool mom;
  int64_t b4 = 0, nb = 0, wait_stride = 1;
  bool pipelined = false, cross = false, rsag = false, peer = false, ocheck = false, spans = false;
  // The peer-read form with one process per GPU: the other ranks are
  // reached through cbx_context::PeerIpc, ordered by its flag page at this
  // step's sequence number `seq` (ipc_started: flags of this step may have
  // been enqueued, so a failure must release the other ranks).
  bool ipc = false, ipc_started = false;
  uint64_t seq = 0;
  unsigned long long foreign = 0;
  std::vector<char> join;
  // Peer-read steps enqueued by one thread per device: device k's count of
  // this step's kernels A (a_seq) and reductions R (r_seq) enqueued with
  // their events recorded.  A device enqueues a wait on another device's
  // event only once that device's count covers it (a wait on an event not
  // yet recorded would wait on its previous step's record instead).
  std::unique_ptr<std::atomic<int64_t>[]> a_seq, r_seq;
  std::atomic<bool> failed{false};
  // Kernel spans (Device::SpanSlot), per device: the step's slot, the
  // previous pipelined step's, the last stop event on each stream the step
  // uses (0 sync stream, 1 a_stream, 2 comm_stream, 3 a_stream2) and the
  // events each of those streams waited on since.
  struct Track {
    Device::SpanSlot *slot = nullptr, *prev = nullptr;
    hipEvent_t last[4] = {};
    std::vector<hipEvent_t> pending[4];
  };
  std::vector<Track> tr;

  SplitStep(cbx_context *ctx, std::vector<cbx::SmaArgs> &a, bool momentum) : c(ctx), args(a), mom(momentum) {}

  int64_t start_of(int64_t b) const { return b * b4; }
  int64_t len_of(int64_t b) const { return std::min(b4, c->n4 - b * b4); }

  // The event kernel A(b) of this step stops (the collective of b waits on it).
  hipEvent_t ev_a(size_t k, int64_t b) {
    Device &d = c->devs[k];
    if (peer && !pipelined) return d.peer_a;  // one bucket: recorded after A on the sync stream
    return ocheck ? d.ord[d.ord_cur].a1[b] : spans ? tr[k].slot->a[b] : d.bucket_acc[b];
  }
  // The event recorded on the comm stream after the collective of bucket b.
  hipEvent_t ev_red(size_t k, int64_t b) {
    if (peer && !pipelined) return c->devs[k].peer_r;
    return spans ? tr[k].slot->red[b] : c->devs[k].bucket_red[b];
  }

  // The peer-read form's participants: the local devices (one process,
  // ordered by events) or every rank (one process per GPU, ordered by the
  // flag page); pg(k) is local device k's index among them.
  int pn() const { return ipc ? c->G : (int)c->devs.size(); }
  int pg(size_t k) const { return ipc ? c->ipc.me : (int)k; }
  const cbx::v4f *p_acc(int h) const {
    return ipc ? c->ipc.acc[h] : reinterpret_cast<const cbx::v4f *>(base_dev(c, c->devs[h], CBX_BUF_GRADIENT));
  }
  const float *p_acc_ctrl(int h) const { return ipc ? c->ipc.acc_ctrl[h] : base_ctrl(c->devs[h], CBX_BUF_GRADIENT); }
  const cbx::v4f *p_D(int h) const {
    return ipc ? c->ipc.D[h] : reinterpret_cast<const cbx::v4f *>(base_dev(c, c->devs[h], CBX_BUF_DIFF));
  }
  // One process per GPU: this rank's flag of bucket b says "done" once the
  // work queued before it on `st` is; a wait holds `st` until rank h's flag
  // has reached this step.
  int put_flag(hipStream_t st, int kind, int64_t b) {
    if (ipc) HIP_TRY(hipStreamWriteValue64(st, c->ipc.dpage + ipc_word(c->ipc.me, kind, b), seq, 0));
    return CBX_OK;
  }
  int wait_flags(hipStream_t st, int kind, int64_t b) {
    for (int h = 0; ipc && !c->fault_skip_peer_wait && h < c->G; ++h)
      if (h != c->ipc.me)
        HIP_TRY(hipStreamWaitValue64(st, c->ipc.dpage + ipc_word(h, kind, b), seq, hipStreamWaitValueGte, ~0ull));
    return CBX_OK;
  }

  // Peer-read, threaded: publish that device k's event of bucket b is
  // recorded / wait until every device's is.
  void publish(std::unique_ptr<std::atomic<int64_t>[]> &seq, size_t k, int64_t b) {
    if (seq) seq[k].store(b + 1, std::memory_order_release);
  }
  int await_all(std::unique_ptr<std::atomic<int64_t>[]> &seq, int64_t b) {
    if (!seq) return CBX_OK;
    for (size_t h = 0; h < c->devs.size(); ++h)
      while (seq[h].load(std::memory_order_acquire) <= b) {
        if (failed.load(std::memory_order_acquire))
          return fail(CBX_ERR_STATE, "peer-read step: the enqueue of another device failed");
        sched_yield();
      }
    return CBX_OK;
  }

  void note_wait(size_t k, int s, hipEvent_t e) {
    if (spans) tr[k].pending[s].push_back(e);
  }
  // A dispatch on stream s stopping `stop`: its start is bounded by the last
  // stop on s and by every event s waited on since (or known exactly).
  void note_dispatch(size_t k, int s, int kind, hipEvent_t stop, hipEvent_t exact_start) {
    if (!spans) return;
    Track &t = tr[k];
    Device::SpanRec r;
    r.stop = stop;
    r.kind = kind;
    if (exact_start) {
      r.pred[r.npred++] = exact_start;
    } else {
      if (t.last[s]) r.pred[r.npred++] = t.last[s];
      for (hipEvent_t e : t.pending[s]) {
        if (r.npred == Device::kSpanPreds) {
          r.npred = 0;  // more than it keeps: start unknown
          break;
        }
        r.pred[r.npred++] = e;
      }
    }
    t.slot->recs.push_back(r);
    t.last[s] = stop;
    t.pending[s].clear();
  }

  // This step's span slot on device k, and where each stream left off.
  int prepare_spans(size_t k) {
    Device &d = c->devs[k];
    Track &t = tr[k];
    const int p = d.span_pos;
    Device::SpanSlot &sl = d.spans[p];
    if (sl.ring_slot >= 0 && d.ring_span[sl.ring_slot] == p) d.ring_span[sl.ring_slot] = -1;
    d.spans[(p + 1) % Device::kSpanRing].preds_valid = false;  // its records may point into this slot
    sl.ring_slot = d.ring_pos;
    sl.preds_valid = true;
    sl.nb = nb;
    sl.recs.clear();
    for (auto *v : {&sl.a, &sl.red, &sl.b})
      while ((int64_t)v->size() < nb) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        v->push_back(e);
      }
    if (!sl.entry) HIP_TRY(hipEventCreate(&sl.entry));
    sl.a_used.assign(nb, nullptr);
    sl.b_used.assign(nb, nullptr);
    t.slot = &sl;
    const int prev_ring = (d.ring_pos + Device::kRing - 1) % Device::kRing;
    t.prev = nullptr;
    if (d.span_last >= 0 && d.spans[d.span_last].ring_slot == prev_ring && d.ring_count > 0)
      t.prev = &d.spans[d.span_last];
    if (t.prev) t.last[2] = t.prev->red[t.prev->nb - 1];
    if (!cross) {
      if (d.ring_count > 0) t.last[0] = ring_stop(d, prev_ring);
    } else if (!join[k] && !t.prev) {
      join[k] = 1;  // the previous step's span records are gone (timing reset): join the whole sync stream
    } else if (!join[k]) {  // continues the previous cross step bucket by bucket (same nb, spans on)
      const int64_t last_odd = (nb - 1) & 1 ? nb - 1 : nb - 2, last_even = (nb - 1) & 1 ? nb - 2 : nb - 1;
      t.last[1] = t.prev->a_used[last_even];
      t.last[3] = t.prev->a_used[last_odd];
      t.last[0] = t.prev->b_used[nb - 1];
    }
    return CBX_OK;
  }

  // Bucket geometry and the step's modes, for every device.
  int prepare_common() {
    const int64_t pad = cbx::kPadFloat4;
    b4 = c->n4;
    if (c->bucket_elems > 0) {
      b4 = ((c->bucket_elems / 4 + pad - 1) / pad) * pad;
    } else if (c->G > 1) {
      b4 = ((c->n4 / kDefaultBuckets + pad - 1) / pad) * pad;  // auto: kDefaultBuckets buckets
    }
    if (b4 <= 0 || b4 > c->n4) b4 = c->n4;
    nb = (c->n4 + b4 - 1) / b4;
    pipelined = nb > 1;
    cross = pipelined && c->pipeline_mode == 1;
    rsag = c->allreduce_algo == CBX_ALLREDUCE_RSAG;
    peer = c->allreduce_algo == CBX_ALLREDUCE_PEER && c->G > 1;
    ipc = peer && c->per_rank;
    // Any form: refused once a rank is broken (synchronise_impl checked
    // already; a step that reaches here another way is checked all the same).
    TRY(peer_guard(c, "the split step"));
    if (ipc) {
      if (!c->ipc.ready) return fail(CBX_ERR_STATE, "the per-rank peer-read form needs cbx_peer_import");
      if (nb > kIpcMaxBuckets)
        return fail(CBX_ERR_UNSUPPORTED, "the per-rank peer-read form takes at most %lld buckets (%lld asked)",
                    (long long)kIpcMaxBuckets, (long long)nb);
      seq = ++c->ipc.seq;
      c->ipc.max_nb = std::max(c->ipc.max_nb, nb);
      ipc_started = true;
    }
    // After the sequence number: a per-rank peer-read step that fails here
    // releases its flags like any other failed step.
    if (c->fault_fail_buckets > 0 && nb == c->fault_fail_buckets)
      return fail(CBX_ERR_STATE, "fault injection: a split step over %lld buckets fails ($CBX_FAULT_FAIL_STEP_BUCKETS)",
                  (long long)nb);
    if (peer && threaded(c)) {
      a_seq.reset(new std::atomic<int64_t>[c->devs.size()]);
      r_seq.reset(new std::atomic<int64_t>[c->devs.size()]);
      for (size_t k = 0; k < c->devs.size(); ++k) {
        a_seq[k].store(0, std::memory_order_relaxed);
        r_seq[k].store(0, std::memory_order_relaxed);
      }
    }
    ocheck = c->order_check && c->timing;
    spans = c->timing && !ocheck && pipelined && nb <= Device::kSpanMaxBuckets;
    for (Device &d : c->devs) spans = spans && !d.spans.empty();
    wait_stride = std::max(1, c->cross_wait_stride);
    foreign = c->foreign_ops.load(std::memory_order_acquire);
    join.assign(c->devs.size(), 1);
    tr.assign(c->devs.size(), Track());
    return CBX_OK;
  }

  // Device k's per-bucket events, its cross-step join decision, its span
  // slot, and a fresh set of stream-order timestamps when the check is on.
  int prepare_device(size_t k) {
    {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      if (pipelined) {
        while ((int64_t)d.bucket_acc.size() < nb) {
          hipEvent_t ea, er, eb;
          // ea / eb are also handed to kernel dispatches as their stop events.
          HIP_TRY(hipEventCreate(&ea));
          HIP_TRY(hipEventCreateWithFlags(&er, hipEventDisableTiming));
          HIP_TRY(hipEventCreate(&eb));
          d.bucket_acc.push_back(ea);
          d.bucket_red.push_back(er);
          d.bucket_b.push_back(eb);
        }
      }
      if (cross) {
        if (!d.cross_entry) {
          HIP_TRY(hipEventCreateWithFlags(&d.cross_entry, hipEventDisableTiming));
          HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d.decision), 256));
          HIP_TRY(hipMemsetAsync(d.decision, 0, 256, d.stream));
          d.cross_valid = false;
        }
        join[k] = !d.cross_valid || d.cross_nb != nb || d.cross_foreign != foreign || d.cross_spans != spans;
      }
      if (spans) TRY(prepare_spans(k));
      if (cross && join[k]) {
        hipEvent_t e = spans ? tr[k].slot->entry : d.cross_entry;
        HIP_TRY(hipEventRecord(e, d.stream));
        HIP_TRY(hipStreamWaitEvent(d.a_stream, e, 0));
        HIP_TRY(hipStreamWaitEvent(d.a_stream2, e, 0));
        note_wait(k, 1, e);
        note_wait(k, 3, e);
        if (spans) tr[k].last[0] = e;  // everything before it on the sync stream
      }
      if (ocheck) {
        d.ord_cur ^= 1u;
        std::vector<hipEvent_t> &pool = d.ord_pool[d.ord_cur];
        while ((int64_t)pool.size() < 6 * nb) {
          hipEvent_t e;
          HIP_TRY(hipEventCreate(&e));
          pool.push_back(e);
        }
        Device::OrderStep &o = d.ord[d.ord_cur];
        o.valid = true;
        o.cont = cross && !join[k];
        o.nb = nb;
        o.pa.assign(pool.begin(), pool.begin() + nb);
        o.c0.assign(pool.begin() + nb, pool.begin() + 2 * nb);
        o.c1.assign(pool.begin() + 2 * nb, pool.begin() + 3 * nb);
        o.pb.assign(pool.begin() + 3 * nb, pool.begin() + 4 * nb);
        o.b1.assign(pool.begin() + 4 * nb, pool.begin() + 5 * nb);
        o.a1.assign(pool.begin() + 5 * nb, pool.begin() + 6 * nb);
      }
    }
    return CBX_OK;
  }

  // Kernel A (Phase A) of bucket b on devices [k0, k1).
  int accumulate(int64_t b, size_t k0, size_t k1) {
    for (size_t k = k0; k < k1; ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      cbx::LaunchConfig cfg = c->cfg;
      cfg.num_cus = d.num_cus;
      cbx::Timing t;
      if (b == 0) t.start = pipelined ? step_start_event(c, d, 2) : ring_event(c, d, EV_START);
      if (!pipelined) t.stop = ring_event(c, d, EV_A);
      // Cross-step mode: even buckets on a_stream, odd ones on a_stream2.
      hipStream_t st = cross ? ((b & 1) ? d.a_stream2 : d.a_stream) : d.stream;
      const int si = cross ? ((b & 1) ? 3 : 1) : 0;
      // The wait goes by the position on the kernel's own stream; waiting on
      // a later B implies every earlier one (the B's run in order).
      const int64_t pos = cross ? b / 2 : b;
      if (cross && !join[k] && pos % wait_stride == 0) {  // B(b), B(b+2) .. of the last step
        const int64_t w = std::min<int64_t>(b + 2 * (wait_stride - 1), nb - 1);
        hipEvent_t e = ocheck ? d.ord[d.ord_cur ^ 1u].b1[w] : spans ? tr[k].prev->b_used[w] : d.bucket_b[w];
        HIP_TRY(hipStreamWaitEvent(st, e, 0));
        note_wait(k, si, e);
      }
      if (pipelined) t.stop = ev_a(k, b);
      if (cross && c->fault_one_stream_comm_wait) {
        // Fault injection: a kernel A the faulted comm wait skips (not the
        // last of its all-reduce group) starts 0.5 ms late.
        const int64_t ar_group = std::max(1, c->allreduce_group);
        if ((b + 1) % ar_group != 0 && b != nb - 1) {
          int khz = 0;
          HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d.hip_id));
          HIP_TRY(cbx::launch_delay(st, (uint64_t)khz / 2));
        }
      }
      if (ipc && c->fault_skip_peer_wait && c->ipc.me != 0) {
        // Fault injection: this rank's kernel A starts 2 ms late, so a rank
        // that skips its flag waits reads acc before it is written.
        int khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d.hip_id));
        HIP_TRY(cbx::launch_delay(st, (uint64_t)khz * 2));
      }
      if (ocheck) {
        Device::OrderStep &o = d.ord[d.ord_cur];
        HIP_TRY(cbx::launch_order_probe(st, {nullptr, o.pa[b]}));
        o.a1[b] = t.stop;  // with timing on, A always carries a stop event (the pool's or the ring's)
      }
      HIP_TRY(cbx::launch_sma_accumulate(offset_args(args[k], start_of(b), len_of(b)), b == 0, cfg, st, t));
      if (peer && !pipelined && !ipc) HIP_TRY(hipEventRecord(d.peer_a, st));  // the other devices' R waits on it
      TRY(put_flag(st, kIpcA, b));  // one process per GPU: the other ranks' R waits on it
      if (ipc && b == std::min<int64_t>(c->fault_peer_fail_bucket, nb - 1) && c->fault_peer_fail_rank == c->ipc.me &&
          (int64_t)c->fault_peer_fail_seq == (int64_t)seq) {
        c->fault_peer_fail_seq = -1;  // once: numbering restarts after cbx_resync_base
        return fail(CBX_ERR_STATE, "fault injection: rank %d's peer-read step %llu fails after kernel A of bucket "
                    "%lld ($CBX_FAULT_PEER_FAIL)", c->ipc.me, (unsigned long long)seq, (long long)b);
      }
      if (spans) tr[k].slot->a_used[b] = t.stop;
      note_dispatch(k, si, Device::SPAN_A, t.stop, b == 0 ? t.start : nullptr);
      publish(a_seq, k, b);
    }
    return CBX_OK;
  }

  // The collective of bucket b (common.c:14-54: grouped, fp32 sum; bucket 0
  // also carries the control block right in front of the data).  `wait_acc`:
  // the comm stream first waits for kernels A up to that bucket, from bucket
  // `wait_from` on (-1: no wait; an earlier collective of the same group
  // already waited).  Kernels A run in order on their stream, so the last
  // one implies the earlier ones; in cross-step mode they alternate over two
  // streams, and the last one on each stream is waited for.
  int collective(int64_t b, bool on_comm, int64_t wait_from, int64_t wait_acc, size_t k0, size_t k1) {
    const int64_t start = start_of(b), len = len_of(b);
    if (on_comm && wait_acc >= 0 && !c->fault_skip_comm_wait) {
      // the last kernel A on each A stream (two in cross-step mode); the
      // peer-read reduction reads every device's acc, so it waits for every
      // device's kernels A
      const int64_t streams = cross && !c->fault_one_stream_comm_wait ? 2 : 1;
      TRY(await_all(a_seq, wait_acc));
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        for (int64_t a = wait_acc; a >= wait_from && a > wait_acc - streams; --a) {
          for (size_t h = peer ? 0 : k; h < (peer ? c->devs.size() : k + 1); ++h) {
            hipEvent_t e = ev_a(h, a);
            HIP_TRY(hipStreamWaitEvent(d.comm_stream, e, 0));
            note_wait(k, 2, e);
          }
          TRY(wait_flags(d.comm_stream, kIpcA, a));  // one process per GPU: every other rank's
        }
      }
    } else if (peer && !on_comm) {
      // one bucket, in order on the sync stream: its own kernel A by stream
      // order, the other devices' by their events
      TRY(await_all(a_seq, b));
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        for (size_t h = 0; h < c->devs.size(); ++h)
          if (h != k) HIP_TRY(hipStreamWaitEvent(d.stream, ev_a(h, b), 0));
        TRY(wait_flags(d.stream, kIpcA, b));
      }
    }
    for (size_t k = k0; ocheck && k < k1; ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      HIP_TRY(cbx::launch_order_probe(on_comm ? d.comm_stream : d.stream, {nullptr, d.ord[d.ord_cur].c0[b]}));
    }
    if (peer) {
      // Peer-read reduction R: device k sums shard k of the bucket from every
      // device's acc into its own D (device order from +0: the oracle's);
      // bucket 0 also sums the control blocks.
      const int G = pn();
      const int64_t sh4 = peer_shard4(len, G);
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        const int64_t s0 = std::min<int64_t>((int64_t)pg(k) * sh4, len);
        cbx::PeerArgs r;
        std::memset(&r, 0, sizeof(r));
        r.G = G;
        r.shard4 = sh4;
        for (int h = 0; h < G; ++h) {
          r.acc[h] = p_acc(h) + start + s0;
          r.ctrl_in[h] = p_acc_ctrl(h);
        }
        r.out = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_DIFF)) + start + s0;
        r.ctrl_out = b == 0 ? base_ctrl(d, CBX_BUF_DIFF) : nullptr;
        r.n4 = std::min(sh4, len - s0);  // 0 for a trailing empty shard (one block runs, and sums the control block)
        cbx::LaunchConfig cfg = c->apply_cfg;
        cfg.num_cus = d.num_cus;
        HIP_TRY(cbx::launch_sma_peer_reduce(r, cfg, on_comm ? d.comm_stream : d.stream));
      }
    } else if (rsag) {
      // Reduce-scatter form: shard g of the bucket (len / G float4s) is
      // reduced on rank g, which applies the base momentum to its shard of
      // last; the all-gather of last (or of D without momentum) then hands
      // every rank the whole bucket of D' for kernel B.  The control block
      // rides a 64-float all-reduce grouped with bucket 0's reduce-scatter.
      const int64_t sh4 = len / c->G;
      NCCL_TRY(ncclGroupStart());
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        hipStream_t st = on_comm ? d.comm_stream : d.stream;
        if (b == 0)
          NCCL_TRY(ncclAllReduce(base_ctrl(d, CBX_BUF_GRADIENT), base_ctrl(d, CBX_BUF_DIFF), cbx::kCtrlFloats,
                                 ncclFloat, ncclSum, d.comm, st));
        NCCL_TRY(ncclReduceScatter(base_dev(c, d, CBX_BUF_GRADIENT) + start * 4,
                                   base_dev(c, d, CBX_BUF_DIFF) + (start + d.g * sh4) * 4, (size_t)sh4 * 4,
                                   ncclFloat, ncclSum, d.comm, st));
      }
      NCCL_TRY(ncclGroupEnd());
      const int gather = mom ? CBX_BUF_LAST : CBX_BUF_DIFF;
      for (size_t k = k0; mom && k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        cbx::SmaArgs a = offset_args(args[k], start + d.g * sh4, sh4);
        cbx::LaunchConfig cfg = c->apply_cfg;
        cfg.num_cus = d.num_cus;
        HIP_TRY(cbx::launch_sma_shard_momentum(a, cfg, on_comm ? d.comm_stream : d.stream));
      }
      NCCL_TRY(ncclGroupStart());
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        float *buf = base_dev(c, d, gather) + start * 4;
        NCCL_TRY(ncclAllGather(buf + d.g * sh4 * 4, buf, (size_t)sh4 * 4, ncclFloat, d.comm,
                               on_comm ? d.comm_stream : d.stream));
      }
      NCCL_TRY(ncclGroupEnd());
    } else {
      NCCL_TRY(ncclGroupStart());
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        const float *src = base_dev(c, d, CBX_BUF_GRADIENT) + start * 4;
        float *dst = base_dev(c, d, CBX_BUF_DIFF) + start * 4;
        size_t count = (size_t)len * 4;
        if (b == 0) {
          src -= cbx::kCtrlFloats;
          dst -= cbx::kCtrlFloats;
          count += cbx::kCtrlFloats;
        }
        NCCL_TRY(ncclAllReduce(src, dst, count, ncclFloat, ncclSum, d.comm, on_comm ? d.comm_stream : d.stream));
      }
      NCCL_TRY(ncclGroupEnd());
    }
    for (size_t k = k0; ocheck && k < k1; ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      HIP_TRY(cbx::launch_order_probe(on_comm ? d.comm_stream : d.stream, {nullptr, d.ord[d.ord_cur].c1[b]}));
    }
    if (on_comm) {
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        HIP_TRY(hipEventRecord(ev_red(k, b), d.comm_stream));
        note_dispatch(k, 2, Device::SPAN_COLL, ev_red(k, b), nullptr);
        TRY(put_flag(d.comm_stream, kIpcR, b));
      }
    } else if (peer) {
      for (size_t k = k0; k < k1; ++k) {  // the other devices' kernels B wait on it
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        if (ipc) TRY(put_flag(d.stream, kIpcR, b));
        else HIP_TRY(hipEventRecord(ev_red(k, b), d.stream));
      }
    }
    for (size_t k = k0; k < k1; ++k) publish(r_seq, k, b);
    return CBX_OK;
  }

  // Kernel B (Phase C, + D on copy) of bucket b on devices [k0, k1).
  int apply(int64_t b, size_t k0, size_t k1) {
    const int64_t ar_group = std::max(1, c->allreduce_group);
    if (peer) TRY(await_all(r_seq, b));
    for (size_t k = k0; k < k1; ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      // its bucket's collective; the peer-read kernel B reads D from every
      // shard's owner, so it waits for every device's reduction.  (Relaying
      // them through the comm stream, one wait here instead of G, measured
      // slower in both modes: profiles/r04/peer_ab.jsonl.)
      for (size_t h = peer ? 0 : k; h < (peer ? c->devs.size() : k + 1); ++h) {
        if (!pipelined && h == k) continue;  // in order on this stream
        HIP_TRY(hipStreamWaitEvent(d.stream, ev_red(h, b), 0));
        note_wait(k, 0, ev_red(h, b));
      }
      // One process per GPU: every other rank's reduction.  With all-reduce
      // groups, once per group, on the group's last bucket: each rank's
      // reductions run in order on its comm stream, so that flag implies the
      // group's earlier ones, and every R of the group is enqueued before
      // its first B (fewer cross-process hand-offs, ~19 us each when the
      // wait blocks: profiles/r04/ipc/).
      if (!pipelined || b % ar_group == 0)
        TRY(wait_flags(d.stream, kIpcR, pipelined ? std::min<int64_t>(b + ar_group - 1, nb - 1) : b));
      cbx::LaunchConfig cfg = c->apply_cfg;
      cfg.num_cus = d.num_cus;
      cbx::Timing t;
      if (b == nb - 1) t.stop = step_stop_event(c, d, EV_B);
      cbx::SmaArgs a = offset_args(args[k], start_of(b), len_of(b));
      if (rsag && mom) a.D = a.last;  // the gathered D' (kernel B then adds it without momentum)
      if (cross) {
        // The next step's AR(0) may overwrite D's control block before this
        // step's later buckets run: B(0) publishes the Phase-D decision to a
        // per-parity slot that B(1..) read.
        a.decision_mode = b == 0 ? 1 : 2;
        a.decision = d.decision + (d.cross_parity & 1u);
      }
      const bool in_dispatch = cross && !t.stop;
      if (in_dispatch) t.stop = ocheck ? d.ord[d.ord_cur].b1[b] : spans ? tr[k].slot->b[b] : d.bucket_b[b];
      if (spans && !t.stop) t.stop = tr[k].slot->b[b];  // every B stops an event of its own for its span
      if (ocheck) {
        Device::OrderStep &o = d.ord[d.ord_cur];
        HIP_TRY(cbx::launch_order_probe(d.stream, {nullptr, o.pb[b]}));
        if (!t.stop) t.stop = o.b1[b];
        o.b1[b] = t.stop;
      }
      if (peer) {
        cbx::PeerArgs p;
        std::memset(&p, 0, sizeof(p));
        p.G = pn();
        p.shard4 = peer_shard4(len_of(b), p.G);
        for (int h = 0; h < p.G; ++h) p.D[h] = p_D(h) + start_of(b);
        HIP_TRY(cbx::launch_sma_peer_apply(a, p, mom, cfg, d.stream, t));
        if (ipc && b == nb - 1)  // every kernel B of the step is done before it (same stream)
          HIP_TRY(cbx::launch_peer_poison_check(c->ipc.dpage + ipc_word(0, kIpcBroken, 0), (int64_t)kIpcRankWords,
                                                c->G, c->ipc.dpage + ipc_word(c->ipc.me, kIpcPoison, 0), seq,
                                                d.stream));
      } else {
        HIP_TRY(cbx::launch_sma_apply(a, mom && !rsag, cfg, d.stream, t));
      }
      if (cross && !in_dispatch && !spans) HIP_TRY(hipEventRecord(d.bucket_b[b], d.stream));
      if (spans) tr[k].slot->b_used[b] = t.stop;  // the last B's is the ring's stop event
      note_dispatch(k, 0, Device::SPAN_B, t.stop, nullptr);
    }
    return CBX_OK;
  }

  // The whole step on devices [k0, k1): every device at once from one
  // thread (the reference's order, each collective grouped over the range),
  // or one device per enqueue thread.
  int run_devices(size_t k0, size_t k1) {
    for (size_t k = k0; k < k1; ++k) TRY(prepare_device(k));
    if (!pipelined) {
      TRY(accumulate(0, k0, k1));
      TRY(collective(0, false, -1, -1, k0, k1));
      for (size_t k = k0; k < k1; ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        TRY(mark(c, d, EV_AR));
      }
      TRY(apply(0, k0, k1));
    } else {
      // Collectives go out in groups of `ar_group` buckets behind a single
      // comm-stream wait on the group's last kernel A (cbx_set_allreduce_group).
      // Every event is recorded before the wait on it is enqueued: a group's
      // collectives follow its last A, and B(j) follows AR(j).  Mode 0 applies
      // the previous group while this one is on the link; mode 1 applies a
      // group right behind its collectives.  ar_group 1 is the per-bucket
      // order A(b) AR(b) B(b-1) (mode 0) / A(b) AR(b) B(b) (mode 1).
      const int64_t ar_group = std::max(1, c->allreduce_group);
      int64_t applied = 0;
      for (int64_t b = 0; b < nb; ++b) {
        TRY(accumulate(b, k0, k1));
        if ((b + 1) % ar_group != 0 && b != nb - 1) continue;
        const int64_t g0 = b - b % ar_group;
        for (int64_t j = g0; j <= b; ++j) TRY(collective(j, true, g0, j == g0 ? b : -1, k0, k1));
        const int64_t upto = cross ? b + 1 : g0;
        for (; applied < upto; ++applied) TRY(apply(applied, k0, k1));
      }
      // The wait inside apply(nb-1) also joins every earlier collective
      // (comm_stream is in order) back into the sync stream.
      for (; applied < nb; ++applied) TRY(apply(applied, k0, k1));
    }
    for (size_t k = k0; k < k1; ++k) {
      Device &d = c->devs[k];
      if (spans) {
        d.pending_span = d.span_pos;
        d.span_last = d.span_pos;
        d.span_pos = (d.span_pos + 1) % Device::kSpanRing;
      } else {
        d.span_last = -1;
      }
      ring_advance(c, d, pipelined ? 2 : 1);
      d.cross_valid = cross;
      if (cross) {
        d.cross_nb = nb;
        d.cross_foreign = foreign;
        d.cross_parity ^= 1u;
        d.cross_spans = spans;
      }
    }
    return CBX_OK;
  }

  int run() {
    TRY(prepare_common());
    if (threaded(c)) {
      TRY(for_devices(c, [this](int k) {
        const int rc = run_devices((size_t)k, (size_t)k + 1);
        if (rc < 0) failed.store(true, std::memory_order_release);  // releases the others' peer waits
        return rc;
      }));
    } else {
      TRY(run_devices(0, c->devs.size()));
    }
    c->last_step_split = true;
    return CBX_OK;
  }
};

int sma_step(cbx_context *c, int first) {
  const bool mom = c->has_last && c->model.conf.momentum > 0;  // sma.c:150 (base conf)
  std::vector<cbx::SmaArgs> args(c->devs.size());
  int copies_total = 0;
  for (size_t k = 0; k < c->devs.size(); ++k) {
    int cp = 0;
    TRY(build_args(c, c->devs[k], first, args[k], &cp));
    copies_total += cp;
  }

  if (c->G > 1 ? c->allreduce_algo != CBX_ALLREDUCE_PEER : c->force_split) TRY(ensure_comms(c));
  if (c->allreduce_algo == CBX_ALLREDUCE_PEER && c->G > 1 && !c->per_rank) TRY(ensure_peer_access(c));
  if (c->G == 1 && !c->force_split) {
    // Single GPU: Phase B is the identity, so A + C (+ D) fuse into one pass.
    // (sma.c:63 waits on base->updated; every producer of z is this stream,
    // so stream order already gives that dependency.)
    Device &d = c->devs[0];
    HIP_TRY(hipSetDevice(d.hip_id));
    cbx::LaunchConfig cfg = c->cfg;
    cfg.num_cus = d.num_cus;
    // The dispatch timestamps its own stop (and, on an idle GPU, start) ring
    // events: no marker packets between back-to-back steps.
    HIP_TRY(cbx::launch_sma_fused(args[0], mom, copies_total > 0, cfg, d.stream,
                                  {step_start_event(c, d, 0), step_stop_event(c, d, EV_A)}));
    ring_advance(c, d, 0);
    d.cross_valid = false;
    c->last_step_split = false;
  } else {
    SplitStep split(c, args, mom);
    const int rc = split.run();
    if (rc < 0) {
      // A step that failed part-way left its per-bucket and span events
      // half-recorded: the next step must not continue from it.
      for (Device &d : c->devs) {
        d.cross_valid = false;
        d.span_last = -1;
      }
      if (split.ipc_started) {
        // and the other ranks may already wait on flags it will never write
        const std::string msg = g_last_error;
        release_flags(c, c->ipc.max_nb);
        c->ipc.broken = true;
        g_last_error = msg;
      }
      return rc;
    }
  }

  TRY(finish_step(c));
  for (Device &d : c->devs)
    for (int id : d.replicas) {
      if (id < first || !c->locked[id]) continue;
      c->replicas[id]->conf.copy = 0;  // sma.c:220 (a no-op unless a copy happened)
    }
  return CBX_OK;
}

// ---------------------------------------------------------------------------
// Host-staged SMA step, pipelined (cbx_synchronise_staged).  Same result as
// cbx_stage_in + cbx_synchronise + cbx_stage_out, bit for bit (every phase is
// elementwise, and the all-reduce of a bucket sums the same elements), but the
// flat buffers are cut into `nb` buckets and, per device,
//   h2d_stream : H2D(0) H2D(1) H2D(2) ...
//   stream     :   [h2d 0] K(0) [h2d 1] K(1) ...
//   d2h_stream :            [k 0] D2H(0)   [k 1] D2H(1) ...
// so the PCIe uploads of bucket k+1 and the downloads of bucket k-1 run at
// the same time (PCIe is full duplex; separate DMA engines) and the step
// costs about max(H2D, D2H) instead of their sum.  K(b) is the fused kernel
// at G = 1, else kernel A + RCCL all-reduce + kernel B of the bucket, in
// order on the sync stream (bucket 0 carries the control block, so every
// later kernel B sees the Phase-D decision).
// ---------------------------------------------------------------------------
int alloc_host_mirror(cbx_context *c);

int ensure_stage_streams(Device &d, int64_t nb) {
  if (!d.h2d_stream) {
    HIP_TRY(hipStreamCreateWithFlags(&d.h2d_stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&d.d2h_stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&d.stage_entry, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.stage_done, hipEventDisableTiming));
  }
  while ((int64_t)d.stage_h2d.size() < nb) {
    hipEvent_t a, b;
    HIP_TRY(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    d.stage_h2d.push_back(a);
    d.stage_k.push_back(b);
  }
  return CBX_OK;
}

// Copy floats [start4*4, start4*4 + len4*4) of one buffer, clipped to the
// model's n elements (the device pad beyond n stays zero and never travels).
int stage_range(cbx_context *c, void *dst, const void *src, int64_t start4, int64_t len4, hipMemcpyKind kind,
                hipStream_t st) {
  const int64_t lo = start4 * 4, hi = std::min<int64_t>((start4 + len4) * 4, c->n);
  if (hi <= lo) return CBX_OK;
  HIP_TRY(hipMemcpyAsync(static_cast<float *>(dst) + lo, static_cast<const float *>(src) + lo,
                         (size_t)(hi - lo) * sizeof(float), kind, st));
  return CBX_OK;
}

// The same staged step through zero-copy kernels (staging mode ZEROCOPY,
// sma_internal.h StagedArgs): the kernels read z, last, s_i, w_i from the
// pinned host mirror and write w_i, z, last to it and to the device, so the
// link carries each byte once and both directions at once, with no copy
// engine and no copy call per buffer and bucket.  G = 1: one fused launch.
// G > 1 (or forced split), per bucket k:
//   stream      : A(k) A(k+1) ...                         (reads the host)
//   comm_stream : [wait A(k)] AR(k) B(k) [wait A(k+1)] ... (writes the host)
// so kernel B of bucket k writes back over PCIe while kernel A of bucket k+1
// reads.  Replicas outside the step (not locked, or below `first`) are
// staged in by copy, as cbx_stage_in would.
int sma_step_staged_zerocopy(cbx_context *c, int first, int buckets, std::vector<cbx::SmaArgs> &args,
                             int copies_total, bool mom) {
  const bool fused = c->G == 1 && !c->force_split;
  const int64_t pad = cbx::kPadFloat4;
  int64_t b4 = c->n4;
  if (!fused) {
    b4 = ((c->n4 / buckets + pad - 1) / pad) * pad;
    if (b4 <= 0 || b4 > c->n4) b4 = c->n4;
  }
  const int64_t nb = (c->n4 + b4 - 1) / b4;
  std::vector<cbx::StagedArgs> sa(c->devs.size());
  for (size_t k = 0; k < c->devs.size(); ++k) {
    Device &d = c->devs[k];
    const cbx::SmaArgs &a = args[k];
    cbx::StagedArgs &x = sa[k];
    std::memset(&x, 0, sizeof(x));
    int r = 0;
    HIP_TRY(hipSetDevice(d.hip_id));
    for (int id : d.replicas) {
      Replica &rep = *c->replicas[id];
      if (id < first || !c->locked[id]) {
        // not in the step: its inputs still reach the device (cbx_stage_in)
        const size_t bytes = (size_t)c->n * 4;
        HIP_TRY(hipMemcpyAsync(replica_dev(d, rep, CBX_BUF_DIFF), replica_host(d, rep, CBX_BUF_DIFF), bytes,
                               hipMemcpyHostToDevice, d.stream));
        HIP_TRY(hipMemcpyAsync(replica_dev(d, rep, CBX_BUF_DATA), replica_host(d, rep, CBX_BUF_DATA), bytes,
                               hipMemcpyHostToDevice, d.stream));
        continue;
      }
      x.sh[r] = reinterpret_cast<const cbx::v4f *>(replica_host(d, rep, CBX_BUF_DIFF));
      x.wh[r] = reinterpret_cast<cbx::v4f *>(replica_host(d, rep, CBX_BUF_DATA));
      x.sd[r] = const_cast<cbx::v4f *>(a.s[r]);
      x.wd[r] = a.w[r];
      ++r;
    }
    x.nrep = a.nrep;
    x.zh = reinterpret_cast<cbx::v4f *>(base_host(d, CBX_BUF_DATA));
    x.zd = a.z;
    if (c->has_last) {
      x.lh = reinterpret_cast<cbx::v4f *>(base_host(d, CBX_BUF_LAST));
      x.ld = a.last;
      if (!mom) {  // `last` exists but is not part of the step: staged in by copy
        HIP_TRY(hipMemcpyAsync(x.ld, x.lh, (size_t)c->n * 4, hipMemcpyHostToDevice, d.stream));
      }
    }
    x.acc = a.acc;
    x.D = a.D;
    x.ctrl_out = a.ctrl_out;
    x.ctrl_in = a.ctrl_in;
    x.alpha = a.alpha;
    x.copies = a.copies;
  }
  auto at = [&](const cbx::StagedArgs &x, int64_t s4, int64_t l4) {
    cbx::StagedArgs y = x;
    for (int r = 0; r < x.nrep; ++r) {
      y.sh[r] = x.sh[r] + s4;
      y.sd[r] = x.sd[r] + s4;
      y.wh[r] = x.wh[r] + s4;
      y.wd[r] = x.wd[r] + s4;
    }
    y.zh = x.zh + s4;
    y.zd = x.zd + s4;
    if (x.lh) {
      y.lh = x.lh + s4;
      y.ld = x.ld + s4;
    }
    y.acc = x.acc + s4;
    y.D = x.D + s4;
    y.n4 = l4;
    return y;
  };
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    d.ev_valid[EV_H2D0] = d.ev_valid[EV_H2D1] = d.ev_valid[EV_D2H0] = d.ev_valid[EV_D2H1] = false;
    if (!fused) {
      while ((int64_t)d.bucket_acc.size() < nb) {
        hipEvent_t ea, er, eb;
        HIP_TRY(hipEventCreate(&ea));
        HIP_TRY(hipEventCreateWithFlags(&er, hipEventDisableTiming));
        HIP_TRY(hipEventCreate(&eb));
        d.bucket_acc.push_back(ea);
        d.bucket_red.push_back(er);
        d.bucket_b.push_back(eb);
      }
    }
  }
  if (fused) {
    Device &d = c->devs[0];
    HIP_TRY(hipSetDevice(d.hip_id));
    cbx::LaunchConfig cfg = c->staged_cfg;
    cfg.num_cus = d.num_cus;
    sa[0].n4 = c->n4;
    HIP_TRY(cbx::launch_sma_fused_staged(sa[0], mom, copies_total > 0, cfg, d.stream,
                                         {ring_event(c, d, EV_START), step_stop_event(c, d, EV_B)}));
    ring_advance(c, d, 2);
    c->last_step_split = false;
    return CBX_OK;
  }
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t s4 = b * b4, l4 = std::min(b4, c->n4 - s4);
    for (size_t k = 0; k < c->devs.size(); ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      cbx::LaunchConfig cfg = c->staged_cfg;
      cfg.num_cus = d.num_cus;
      cbx::Timing t;
      if (b == 0) t.start = ring_event(c, d, EV_START);
      t.stop = d.bucket_acc[b];
      HIP_TRY(cbx::launch_sma_accumulate_staged(at(sa[k], s4, l4), b == 0, cfg, d.stream, t));
      HIP_TRY(hipStreamWaitEvent(d.comm_stream, d.bucket_acc[b], 0));
    }
    NCCL_TRY(ncclGroupStart());
    for (Device &d : c->devs) {
      HIP_TRY(hipSetDevice(d.hip_id));
      const float *src = base_dev(c, d, CBX_BUF_GRADIENT) + s4 * 4;
      float *dst = base_dev(c, d, CBX_BUF_DIFF) + s4 * 4;
      size_t count = (size_t)l4 * 4;
      if (b == 0) {  // the control block rides with bucket 0 (common.c:45-52 + sma.c:113-120)
        src -= cbx::kCtrlFloats;
        dst -= cbx::kCtrlFloats;
        count += cbx::kCtrlFloats;
      }
      NCCL_TRY(ncclAllReduce(src, dst, count, ncclFloat, ncclSum, d.comm, d.comm_stream));
    }
    NCCL_TRY(ncclGroupEnd());
    for (size_t k = 0; k < c->devs.size(); ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      cbx::LaunchConfig cfg = c->staged_cfg;
      cfg.num_cus = d.num_cus;
      cbx::Timing t;
      if (b == nb - 1) t.stop = d.bucket_b[b];
      HIP_TRY(cbx::launch_sma_apply_staged(at(sa[k], s4, l4), mom, cfg, d.comm_stream, t));
    }
  }
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipStreamWaitEvent(d.stream, d.bucket_b[nb - 1], 0));  // the step ends on the sync stream
    TRY(mark(c, d, EV_B));
    ring_advance(c, d, 2);
    d.cross_valid = false;
  }
  c->last_step_split = true;
  return CBX_OK;
}

int sma_step_staged(cbx_context *c, int first, int buckets) {
  const bool mom = c->has_last && c->model.conf.momentum > 0;  // sma.c:150
  std::vector<cbx::SmaArgs> args(c->devs.size());
  int copies_total = 0;
  for (size_t k = 0; k < c->devs.size(); ++k) {
    int cp = 0;
    TRY(build_args(c, c->devs[k], first, args[k], &cp));
    copies_total += cp;
  }
  if (c->G > 1 || c->force_split) TRY(ensure_comms(c));
  TRY(alloc_host_mirror(c));
  if (c->staging_mode == CBX_STAGING_ZEROCOPY) {
    TRY(sma_step_staged_zerocopy(c, first, buckets, args, copies_total, mom));
    TRY(finish_step(c));
    for (Device &d : c->devs)
      for (int id : d.replicas) {
        if (id < first || !c->locked[id]) continue;
        c->replicas[id]->conf.copy = 0;  // sma.c:220
      }
    return CBX_OK;
  }
  const bool fused = c->G == 1 && !c->force_split;
  const int64_t pad = cbx::kPadFloat4;
  int64_t b4 = ((c->n4 / buckets + pad - 1) / pad) * pad;
  if (b4 <= 0 || b4 > c->n4) b4 = c->n4;
  const int64_t nb = (c->n4 + b4 - 1) / b4;

  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    TRY(ensure_stage_streams(d, nb));
    TRY(mark(c, d, EV_START));
    HIP_TRY(hipEventRecord(d.stage_entry, d.stream));  // everything enqueued before this call
    HIP_TRY(hipStreamWaitEvent(d.h2d_stream, d.stage_entry, 0));
    if (c->timing) {
      HIP_TRY(hipEventRecord(d.ev[EV_H2D0], d.h2d_stream));
      d.ev_valid[EV_H2D0] = true;
    }
  }
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t s4 = b * b4, l4 = std::min(b4, c->n4 - s4);
    // inputs: z, last, s_i, w_i (cbx_stage_in's set)
    for (Device &d : c->devs) {
      HIP_TRY(hipSetDevice(d.hip_id));
      const auto H2D = hipMemcpyHostToDevice;
      TRY(stage_range(c, base_dev(c, d, CBX_BUF_DATA), base_host(d, CBX_BUF_DATA), s4, l4, H2D, d.h2d_stream));
      if (c->has_last)
        TRY(stage_range(c, base_dev(c, d, CBX_BUF_LAST), base_host(d, CBX_BUF_LAST), s4, l4, H2D, d.h2d_stream));
      for (int id : d.replicas) {
        Replica &r = *c->replicas[id];
        TRY(stage_range(c, replica_dev(d, r, CBX_BUF_DIFF), replica_host(d, r, CBX_BUF_DIFF), s4, l4, H2D, d.h2d_stream));
        TRY(stage_range(c, replica_dev(d, r, CBX_BUF_DATA), replica_host(d, r, CBX_BUF_DATA), s4, l4, H2D, d.h2d_stream));
      }
      HIP_TRY(hipEventRecord(d.stage_h2d[b], d.h2d_stream));
      HIP_TRY(hipStreamWaitEvent(d.stream, d.stage_h2d[b], 0));
    }
    // compute the bucket on every device's sync stream
    for (size_t k = 0; k < c->devs.size(); ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      cbx::LaunchConfig cfg = c->cfg;
      cfg.num_cus = d.num_cus;
      const cbx::SmaArgs a = offset_args(args[k], s4, l4);
      if (fused) HIP_TRY(cbx::launch_sma_fused(a, mom, copies_total > 0, cfg, d.stream));
      else HIP_TRY(cbx::launch_sma_accumulate(a, b == 0, cfg, d.stream));
    }
    if (!fused) {
      NCCL_TRY(ncclGroupStart());
      for (Device &d : c->devs) {
        HIP_TRY(hipSetDevice(d.hip_id));
        const float *src = base_dev(c, d, CBX_BUF_GRADIENT) + s4 * 4;
        float *dst = base_dev(c, d, CBX_BUF_DIFF) + s4 * 4;
        size_t count = (size_t)l4 * 4;
        if (b == 0) {  // the control block rides with bucket 0 (common.c:45-52 + sma.c:113-120)
          src -= cbx::kCtrlFloats;
          dst -= cbx::kCtrlFloats;
          count += cbx::kCtrlFloats;
        }
        NCCL_TRY(ncclAllReduce(src, dst, count, ncclFloat, ncclSum, d.comm, d.stream));
      }
      NCCL_TRY(ncclGroupEnd());
      for (size_t k = 0; k < c->devs.size(); ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        cbx::LaunchConfig cfg = c->apply_cfg;
        cfg.num_cus = d.num_cus;
        HIP_TRY(cbx::launch_sma_apply(offset_args(args[k], s4, l4), mom, cfg, d.stream));
      }
    }
    // outputs: z, last, w_i (cbx_stage_out's set)
    for (Device &d : c->devs) {
      HIP_TRY(hipSetDevice(d.hip_id));
      HIP_TRY(hipEventRecord(d.stage_k[b], d.stream));
      HIP_TRY(hipStreamWaitEvent(d.d2h_stream, d.stage_k[b], 0));
      if (b == 0 && c->timing) {
        HIP_TRY(hipEventRecord(d.ev[EV_D2H0], d.d2h_stream));
        d.ev_valid[EV_D2H0] = true;
      }
      const auto D2H = hipMemcpyDeviceToHost;
      TRY(stage_range(c, base_host(d, CBX_BUF_DATA), base_dev(c, d, CBX_BUF_DATA), s4, l4, D2H, d.d2h_stream));
      if (c->has_last)
        TRY(stage_range(c, base_host(d, CBX_BUF_LAST), base_dev(c, d, CBX_BUF_LAST), s4, l4, D2H, d.d2h_stream));
      for (int id : d.replicas) {
        Replica &r = *c->replicas[id];
        TRY(stage_range(c, replica_host(d, r, CBX_BUF_DATA), replica_dev(d, r, CBX_BUF_DATA), s4, l4, D2H, d.d2h_stream));
      }
    }
  }
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    if (c->timing) {
      HIP_TRY(hipEventRecord(d.ev[EV_H2D1], d.h2d_stream));
      HIP_TRY(hipEventRecord(d.ev[EV_D2H1], d.d2h_stream));
      d.ev_valid[EV_H2D1] = d.ev_valid[EV_D2H1] = true;
    }
    HIP_TRY(hipEventRecord(d.stage_done, d.d2h_stream));
    HIP_TRY(hipStreamWaitEvent(d.stream, d.stage_done, 0));
    TRY(mark(c, d, EV_B));
    ring_advance(c, d, 2);
  }
  c->last_step_split = !fused;
  TRY(finish_step(c));
  for (Device &d : c->devs)
    for (int id : d.replicas) {
      if (id < first || !c->locked[id]) continue;
      c->replicas[id]->conf.copy = 0;  // sma.c:220
    }
  return CBX_OK;
}

// ---------------------------------------------------------------------------
// Synchronous SGD barrier (update model WORKER), synch/synchronoussgd.c:13-106
// with common.c:3-57 (all-reduce) and :198-220 (base -> replicas).  The
// reference's SINGLE_GPU variant is disabled like SMA's (:5-11); G = 1 runs
// the multi-GPU algorithm with an identity all-reduce, in one kernel.
// ---------------------------------------------------------------------------
int ssgd_step(cbx_context *c, int first) {
  if (c->model.wpc <= 0) return fail(CBX_ERR_STATE, "S-SGD needs the work per clock (setModelWorkPerClock)");
  const float ratio = (float)(1.0 / (double)(float)c->model.wpc);  // synchronoussgd.c:55
  const bool mom = c->has_last && c->model.conf.momentum > 0;        // :64
  const bool split = c->G > 1 || c->force_split;
  if (split) TRY(ensure_comms(c));
  std::vector<cbx::SsgdArgs> args(c->devs.size());
  for (size_t k = 0; k < c->devs.size(); ++k) {
    Device &d = c->devs[k];
    cbx::SsgdArgs &a = args[k];
    std::memset(&a, 0, sizeof(a));
    int r = 0;
    for (int id : d.replicas) {
      if (id < first || !c->locked[id]) continue;  // common.c:208
      if (r >= cbx::kMaxReplicas) return fail(CBX_ERR_UNSUPPORTED, "too many replicas on one device");
      a.w[r++] = reinterpret_cast<cbx::v4f *>(replica_dev(d, *c->replicas[id], CBX_BUF_DATA));
    }
    a.nrep = r;
    a.z = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_DATA));
    a.last = mom ? reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_LAST)) : nullptr;
    a.acc = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_GRADIENT));
    a.D = split ? reinterpret_cast<const cbx::v4f *>(base_dev(c, d, CBX_BUF_DIFF)) : a.acc;
    a.n4 = c->n4;
    a.ratio = ratio;
    a.momentum = mom ? c->model.conf.momentum : 0.0f;
  }
  // Buckets as in the SMA split pipeline (cbx_set_bucket_elements; 8 by
  // default at G > 1).  With more than one, the all-reduce of bucket k+1
  // runs on comm_stream beside the apply kernel of bucket k:
  //   stream      : [entry] [wait red(0)] K(0) [wait red(1)] K(1) ...
  //   comm_stream : [wait entry] AR(0) AR(1) ...
  int64_t b4 = c->n4, nb = 1;
  if (split) {
    const int64_t pad = cbx::kPadFloat4;
    if (c->bucket_elems > 0) b4 = ((c->bucket_elems / 4 + pad - 1) / pad) * pad;
    else if (c->G > 1) b4 = ((c->n4 / kDefaultBuckets + pad - 1) / pad) * pad;
    if (b4 <= 0 || b4 > c->n4) b4 = c->n4;
    nb = (c->n4 + b4 - 1) / b4;
  }
  const bool pipelined = nb > 1;
  if (split) {
    for (Device &d : c->devs) {
      HIP_TRY(hipSetDevice(d.hip_id));
      TRY(mark(c, d, EV_START));
      if (!pipelined) continue;
      while ((int64_t)d.bucket_red.size() < nb) {
        hipEvent_t ea, er, eb;
        HIP_TRY(hipEventCreate(&ea));
        HIP_TRY(hipEventCreateWithFlags(&er, hipEventDisableTiming));
        HIP_TRY(hipEventCreate(&eb));
        d.bucket_acc.push_back(ea);
        d.bucket_red.push_back(er);
        d.bucket_b.push_back(eb);
      }
      // everything the task steps accumulated into acc, in sync-stream order
      HIP_TRY(hipEventRecord(d.bucket_acc[0], d.stream));
      HIP_TRY(hipStreamWaitEvent(d.comm_stream, d.bucket_acc[0], 0));
    }
  }
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t start = b * b4, len = std::min(b4, c->n4 - start);
    if (split) {
      NCCL_TRY(ncclGroupStart());
      for (Device &d : c->devs) {
        HIP_TRY(hipSetDevice(d.hip_id));
        NCCL_TRY(ncclAllReduce(base_dev(c, d, CBX_BUF_GRADIENT) + start * 4, base_dev(c, d, CBX_BUF_DIFF) + start * 4,
                               (size_t)len * 4, ncclFloat, ncclSum, d.comm, pipelined ? d.comm_stream : d.stream));
      }
      NCCL_TRY(ncclGroupEnd());
    }
    for (size_t k = 0; k < c->devs.size(); ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      if (pipelined) {
        HIP_TRY(hipEventRecord(d.bucket_red[b], d.comm_stream));
        HIP_TRY(hipStreamWaitEvent(d.stream, d.bucket_red[b], 0));
      }
      cbx::LaunchConfig cfg = c->ssgd_apply_cfg;
      cfg.num_cus = d.num_cus;
      cbx::Timing t;
      if (!split) t.start = ring_event(c, d, EV_START);
      if (b == nb - 1) t.stop = step_stop_event(c, d, split ? EV_B : EV_A);
      cbx::SsgdArgs a = args[k];
      for (int r = 0; r < a.nrep; ++r) a.w[r] += start;
      a.z += start;
      if (a.last) a.last += start;
      a.acc += start;
      a.D += start;
      a.n4 = len;
      HIP_TRY(cbx::launch_ssgd_apply(a, cfg, d.stream, t));
      if (b == nb - 1) ring_advance(c, d, split ? 2 : 0);
    }
  }
  c->last_step_split = split;
  return finish_step(c);
}

// ---------------------------------------------------------------------------
// Stream-order check (cbx_set_order_check / cbx_check_order).  From the
// timestamps a split step recorded, per bucket k on every device:
//   the collective of k started after kernel A(k) ended;
//   kernel B(k) started after the collective of k ended, and after B(k-1);
// and between two consecutive split steps: kernel A(k) of the later step
// started after B(k) of the earlier one (continued bucket by bucket), or
// A(0) after the earlier step's last B (joined).  "Started after X ended"
// is checked as "the probe dispatched right after the wait ended after X
// ended": both are exact dispatch-completion timestamps, and the probe
// cannot run before its stream's wait is satisfied (slack: kOrderSlackMs).
// ---------------------------------------------------------------------------
constexpr float kOrderSlackMs = 0.0005f;

int order_fail(int64_t k, const char *what, float gap_ms) {
  return fail(CBX_ERR_STATE, "stream order violated at bucket %lld: %s (%.2f us early)", (long long)k, what,
              -gap_ms * 1e3f);
}

int check_order_step(const Device::OrderStep &o) {
  HIP_TRY(hipEventSynchronize(o.b1[o.nb - 1]));
  auto at = [&](hipEvent_t e, float *ms) { return hipEventElapsedTime(ms, o.pa[0], e); };
  float prev_b1 = -1e30f;
  for (int64_t k = 0; k < o.nb; ++k) {
    float a1, c0, c1, pb, b1;
    HIP_TRY(at(o.a1[k], &a1));
    HIP_TRY(at(o.c0[k], &c0));
    HIP_TRY(at(o.c1[k], &c1));
    HIP_TRY(at(o.pb[k], &pb));
    HIP_TRY(at(o.b1[k], &b1));
    if (c0 - a1 < -kOrderSlackMs) return order_fail(k, "the collective started before kernel A ended", c0 - a1);
    if (pb - c1 < -kOrderSlackMs) return order_fail(k, "kernel B started before its collective ended", pb - c1);
    if (pb - prev_b1 < -kOrderSlackMs) return order_fail(k, "kernel B started before the previous B ended", pb - prev_b1);
    prev_b1 = b1;
  }
  return CBX_OK;
}

int check_order_pair(const Device::OrderStep &p, const Device::OrderStep &q) {
  HIP_TRY(hipEventSynchronize(q.b1[q.nb - 1]));
  auto at = [&](hipEvent_t e, float *ms) { return hipEventElapsedTime(ms, p.pa[0], e); };
  if (q.cont && q.nb == p.nb) {
    for (int64_t k = 0; k < q.nb; ++k) {
      float pa, b1;
      HIP_TRY(at(q.pa[k], &pa));
      HIP_TRY(at(p.b1[k], &b1));
      if (pa - b1 < -kOrderSlackMs)
        return order_fail(k, "kernel A of the next step started before this step's kernel B ended", pa - b1);
    }
    return CBX_OK;
  }
  float pa, b1;
  HIP_TRY(at(q.pa[0], &pa));
  HIP_TRY(at(p.b1[p.nb - 1], &b1));
  if (pa - b1 < -kOrderSlackMs) return order_fail(0, "the next step started before this step ended", pa - b1);
  return CBX_OK;
}

int alloc_host_mirror(cbx_context *c) {
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    // Coherent (fine-grained) pinned memory: the zero-copy staged kernels
    // read and write it over PCIe, and the host reads / writes it between
    // steps, so no GPU cache may hold a stale line of it.
    if (!d.host) {
      HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&d.host), d.arena_bytes, hipHostMallocCoherent));
      std::memset(d.host, 0, d.arena_bytes);
    }
    d.extra_host.resize(d.extra.size(), nullptr);
    for (size_t k = 0; k < d.extra.size(); ++k) {
      if (!d.extra[k] || d.extra_host[k]) continue;
      const size_t bytes = d.stride * kReplicaSlots;
      HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&d.extra_host[k]), bytes, hipHostMallocCoherent));
      std::memset(d.extra_host[k], 0, bytes);
    }
  }
  return CBX_OK;
}

}  // namespace cbx::host
