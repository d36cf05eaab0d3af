// sma_seam.hip -- the synchronisation steps over buffers the CALLER owns, for
// a Crossbow build that keeps its own model manager, model buffers and task
// side (modelmanager.c, model.c, executioncontext.c) and replaces only these
// function bodies:
//   crossbowSynchronisationSMA (clib-multigpu/synch/sma.c:233-248 -> :13-231)
//   crossbowKernelOptimiserSMA (kernels/optimisers/sma.cu:3-100)
//   crossbowSynchronisationSynchronousSGD (synch/synchronoussgd.c:13-106)
//   crossbowKernelOptimiserSynchronousSGD (kernels/optimisers/synchronoussgd.cu:3-56)
//   crossbowCudnnBatchNormParamsSynchroniseEstimatedMeanAndVariable
//     (cudnn/cudnnbatchnormparams.c:157-222)
//
// The context API (context.hip) owns an arena whose buffers are padded to
// whole kernel trips; the reference's buffers hold exactly `elements` floats.
// So every launch here runs the bulk of the buffers through the same float4
// kernels (n4b float4s, a multiple of kTailQuantum4) and the last < 4 *
// kTailQuantum4 elements on extra workgroups of the same launch, one float per
// lane (the kernels' TAIL instantiations, sma_kernels.hip), with the same fma
// sequence per element: the results equal the context path's and the
// oracle's bit for bit.
//
// The plan owns what the step needs beyond the caller's buffers: the
// accumulator and the all-reduced difference (base->gradient and base->diff
// in the reference, sma.c:66,82) with the 256-byte control block that carries
// the Phase-D request count through the all-reduce, and -- unless the caller
// hands over its own (executioncontext.c:185-201) -- the RCCL communicators.
#include "context_internal.h"

using namespace cbx::host;

namespace {

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int cus_of_current_device(int *cus) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  static std::atomic<int> cache[cbx::kMaxDevices * 4] = {};
  if (dev >= 0 && dev < (int)(sizeof(cache) / sizeof(cache[0])) && cache[dev].load(std::memory_order_relaxed) > 0) {
    *cus = cache[dev].load(std::memory_order_relaxed);
    return CBX_OK;
  }
  int n = 0;
  HIP_TRY(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  if (dev >= 0 && dev < (int)(sizeof(cache) / sizeof(cache[0]))) cache[dev].store(n, std::memory_order_relaxed);
  *cus = n;
  return CBX_OK;
}

// Largest prefix of an n-float buffer that the float4 kernels cover without
// bounds checks, in float4s.  Their loops need whole waves' chunks (64 lanes
// x unroll float4s, every launch shape here has unroll <= 4); bucket starts
// stay on kPadFloat4.  A smaller tail is fewer scalar workgroups: ResNet-50's
// n = 25,557,032 leaves 40 elements (2,088 at kPadFloat4 granularity, whose
// tail workgroups cost ~7 us per fused step on separately allocated buffers:
// scripts/seam_layout_ab.py, profiles/r02/seam_layout_trace/).
constexpr int64_t kTailQuantum4 = 256;
static_assert(cbx::kPadFloat4 % kTailQuantum4 == 0, "bucket starts must stay on whole chunks");
int64_t bulk_float4s(int64_t n) { return (n / 4) / kTailQuantum4 * kTailQuantum4; }

}  // namespace

struct cbx_sma_plan {
  struct Dev {
    int hip_id = 0;
    int num_cus = 256;
    ncclComm_t comm = nullptr;
    bool own_comm = false;
    char *scratch = nullptr;  // [ctrl | acc (padded)] [ctrl | D (padded)]
    float *acc_ctrl = nullptr;
    float *D_ctrl = nullptr;
    // Bucketed pipeline (G > 1): the all-reduces run on this stream beside
    // kernel A of the next bucket; per bucket, kernel A done / all-reduce done.
    hipStream_t comm_stream = nullptr;
    std::vector<hipEvent_t> ev_a, ev_r;
    int global = 0;  // rank in the communicator (0: the default device)
    // Batch-norm statistics averaging: segment table and packed scratch.
    cbx::BnSegment *bn_table = nullptr;
    size_t bn_table_bytes = 0;
    float *bn_scratch = nullptr;
    size_t bn_scratch_bytes = 0;
  };
  std::vector<Dev> devs;
  int64_t n = 0;
  int64_t n4b = 0;  // bulk float4s
  int ranks = 1;    // ranks of the communicator (1: no collective)
  int buckets = 0;  // G > 1: 0 = kDefaultBuckets, 1 = in order on the caller's stream
  cbx::LaunchConfig cfg;
  cbx::LaunchConfig apply_cfg = cbx::sma_apply_launch_config();
  cbx::LaunchConfig ssgd_apply_cfg = cbx::ssgd_apply_launch_config();
};

namespace {

int ensure_pipeline(cbx_sma_plan *p, int64_t nb) {
  for (auto &d : p->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    if (!d.comm_stream) HIP_TRY(hipStreamCreateWithFlags(&d.comm_stream, hipStreamNonBlocking));
    while ((int64_t)d.ev_a.size() < nb) {
      hipEvent_t a, r;
      HIP_TRY(hipEventCreateWithFlags(&a, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&r, hipEventDisableTiming));
      d.ev_a.push_back(a);
      d.ev_r.push_back(r);
    }
  }
  return CBX_OK;
}

}  // namespace

extern "C" {

int cbx_sma_plan_free(cbx_sma_plan *p) {
  if (!p) return CBX_OK;
  for (auto &d : p->devs) {
    (void)hipSetDevice(d.hip_id);
    (void)hipDeviceSynchronize();
    if (d.own_comm && d.comm) (void)ncclCommDestroy(d.comm);
    if (d.scratch) (void)hipFree(d.scratch);
    if (d.bn_table) (void)hipFree(d.bn_table);
    if (d.bn_scratch) (void)hipFree(d.bn_scratch);
    for (hipEvent_t e : d.ev_a) (void)hipEventDestroy(e);
    for (hipEvent_t e : d.ev_r) (void)hipEventDestroy(e);
    if (d.comm_stream) (void)hipStreamDestroy(d.comm_stream);
  }
  delete p;
  return CBX_OK;
}

int cbx_sma_plan_create(cbx_sma_plan **out, const int *devices, int ndevices, long long elements,
                        void *const *comms) {
  if (!out || !devices || ndevices <= 0 || ndevices > cbx::kMaxDevices)
    return fail(CBX_ERR_INVALID, "cbx_sma_plan_create: need 1..%d devices", cbx::kMaxDevices);
  *out = nullptr;
  // model.h:35 `int bytes`; the kernels address a buffer with 32-bit byte offsets.
  if (elements <= 0 || elements * 4 + 4096 >= (1ll << 32))
    return fail(CBX_ERR_INVALID, "cbx_sma_plan_create: %lld elements out of range", elements);
  cbx_sma_plan *p = new cbx_sma_plan();
  p->n = elements;
  p->n4b = bulk_float4s(elements);
  p->devs.resize(ndevices);
  const int64_t pad = cbx::kPadFloat4;
  const int64_t n4 = ((elements + 3) / 4 + pad - 1) / pad * pad;
  const size_t half = ((size_t)cbx::kCtrlFloats * 4 + (size_t)n4 * 16 + 255) / 256 * 256;
  for (int k = 0; k < ndevices; ++k) {
    auto &d = p->devs[k];
    int rc = probe_device(devices[k], &d.num_cus);
    if (rc < 0) {
      std::string msg = g_last_error;
      cbx_sma_plan_free(p);
      return fail(rc, "%s", msg.c_str());
    }
    d.hip_id = devices[k];
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&d.scratch), 2 * half);
    if (e == hipSuccess) e = hipMemset(d.scratch, 0, 2 * half);
    if (e != hipSuccess) {
      cbx_sma_plan_free(p);
      return fail(CBX_ERR_HIP, "plan scratch of %zu bytes: %s", 2 * half, hipGetErrorString(e));
    }
    d.acc_ctrl = reinterpret_cast<float *>(d.scratch);
    d.D_ctrl = reinterpret_cast<float *>(d.scratch + half);
  }
  if (comms) {
    for (int k = 0; k < ndevices; ++k) {
      p->devs[k].comm = static_cast<ncclComm_t>(comms[k]);
      if (!p->devs[k].comm) {
        cbx_sma_plan_free(p);
        return fail(CBX_ERR_INVALID, "cbx_sma_plan_create: null communicator for device %d", k);
      }
    }
    int count = 0;
    ncclResult_t r = ncclCommCount(p->devs[0].comm, &count);
    for (int k = 0; r == ncclSuccess && k < ndevices; ++k) r = ncclCommUserRank(p->devs[k].comm, &p->devs[k].global);
    if (r != ncclSuccess) {
      cbx_sma_plan_free(p);
      return fail(CBX_ERR_RCCL, "ncclCommCount / ncclCommUserRank: %s", ncclGetErrorString(r));
    }
    p->ranks = count;
  } else if (ndevices > 1) {
    // executioncontext.c:185-201
    std::vector<ncclComm_t> cs(ndevices);
    ncclResult_t r = ncclCommInitAll(cs.data(), ndevices, devices);
    if (r != ncclSuccess) {
      cbx_sma_plan_free(p);
      return fail(CBX_ERR_RCCL, "ncclCommInitAll: %s", ncclGetErrorString(r));
    }
    for (int k = 0; k < ndevices; ++k) {
      p->devs[k].comm = cs[k];
      p->devs[k].own_comm = true;
      p->devs[k].global = k;
    }
    p->ranks = ndevices;
  }
  if (p->ranks < ndevices) {
    cbx_sma_plan_free(p);
    return fail(CBX_ERR_INVALID, "communicator of %d ranks for %d local devices", p->ranks, ndevices);
  }
  *out = p;
  return CBX_OK;
}

int cbx_sma_plan_step(cbx_sma_plan *p, void *const *streams, float *const *z, float *const *last, int nreplicas,
                      const int *replica_device, float *const *w, const float *const *s, const int *locked,
                      const int *copy, float alpha, float momentum, int first) {
  TraceRange trace("cbx_sma_plan_step");
  if (!p) return fail(CBX_ERR_INVALID, "null plan");
  const int G = (int)p->devs.size();
  if (!streams || !z || nreplicas < 0 || (nreplicas > 0 && (!replica_device || !w || !s || !locked || !copy)))
    return fail(CBX_ERR_INVALID, "cbx_sma_plan_step: missing arguments");
  if (first < 0 || first > nreplicas) return fail(CBX_ERR_INVALID, "first replica %d out of range", first);
  const bool mom = momentum > 0.0f;  // sma.c:150: base momentum forced to 0.9 when > 0
  if (mom && !last) return fail(CBX_ERR_INVALID, "base momentum > 0 needs the base models' last buffers");
  // Per device: its locked replicas from `first` on, in id order (sma.c:69-73).
  std::vector<cbx::SmaArgs> args(G);
  int copies_total = 0;
  for (int k = 0; k < G; ++k) {
    std::memset(&args[k], 0, sizeof(cbx::SmaArgs));
    if (!z[k] || !aligned16(z[k]) || (mom && (!last[k] || !aligned16(last[k]))))
      return fail(CBX_ERR_INVALID, "device %d: base buffers must be non-null and 16-byte aligned", k);
  }
  for (int id = first; id < nreplicas; ++id) {
    if (!locked[id]) continue;
    const int k = replica_device[id];
    if (k < 0 || k >= G) return fail(CBX_ERR_INVALID, "replica %d on device %d of %d", id, k, G);
    if (!w[id] || !s[id] || !aligned16(w[id]) || !aligned16(s[id]))
      return fail(CBX_ERR_INVALID, "replica %d: buffers must be non-null and 16-byte aligned", id);
    cbx::SmaArgs &a = args[k];
    if (a.nrep >= cbx::kMaxReplicas)
      return fail(CBX_ERR_UNSUPPORTED, "more than %d locked replicas on one device", cbx::kMaxReplicas);
    a.s[a.nrep] = reinterpret_cast<const cbx::v4f *>(s[id]);
    a.w[a.nrep] = reinterpret_cast<cbx::v4f *>(w[id]);
    if (copy[id]) {
      a.copies += 1.0f;  // sma.c:113-120
      ++copies_total;
    }
    ++a.nrep;
  }
  for (int k = 0; k < G; ++k) {
    auto &d = p->devs[k];
    cbx::SmaArgs &a = args[k];
    a.z = reinterpret_cast<cbx::v4f *>(z[k]);
    a.last = mom ? reinterpret_cast<cbx::v4f *>(last[k]) : nullptr;
    a.acc = reinterpret_cast<cbx::v4f *>(d.acc_ctrl + cbx::kCtrlFloats);
    a.D = reinterpret_cast<const cbx::v4f *>(d.D_ctrl + cbx::kCtrlFloats);
    a.ctrl_out = d.acc_ctrl;
    a.ctrl_in = d.D_ctrl;
    a.n4 = p->n4b;
    a.alpha = alpha;  // sma.c:33
  }
  // The elements past the last whole trip, done by extra workgroups of the
  // launch that covers the buffers' end; float indices relative to the
  // launch's pointers (offset by start4 float4s).
  auto with_tail = [&](cbx::SmaArgs a, int64_t start4) {
    a.tail_lo = (p->n4b - start4) * 4;
    a.tail_hi = p->n - start4 * 4;
    return a;
  };
  if (p->ranks == 1) {
    // One GPU: the all-reduce of one buffer is the identity, so Phases A + C
    // (+ D) fuse into one pass, as in the context's G = 1 step.
    auto &d = p->devs[0];
    hipStream_t st = static_cast<hipStream_t>(streams[0]);
    HIP_TRY(hipSetDevice(d.hip_id));
    cbx::LaunchConfig cfg = p->cfg;
    cfg.num_cus = d.num_cus;
    HIP_TRY(cbx::launch_sma_fused(with_tail(args[0], 0), mom, copies_total > 0, cfg, st));
    return copies_total > 0 ? 1 : 0;
  }
  // G > 1: kernel A, the grouped all-reduce of the control block + acc
  // (common.c:14-54), kernel B.  One bucket: everything in order on each
  // device's stream, the reference's structure.  nb > 1 buckets (the
  // default): the all-reduce of bucket k runs on a stream of the plan's,
  // beside kernel A of bucket k+1, as in the context's pipeline:
  //   stream      : A(0) A(1) [wait r(0)] B(0) A(2) [wait r(1)] B(1) ...
  //   comm_stream : [wait a(0)] AR(0) [wait a(1)] AR(1) ...
  // The control block rides bucket 0; the tail rides the last bucket (its
  // kernel A / B launches take the tail too, its all-reduce extends to n).  The next step's AR(k) waits for its A(k), which follows this
  // step's last B on the caller's stream, so no buffer is overwritten early.
  const int64_t pad = cbx::kPadFloat4;
  int64_t nb = p->buckets > 0 ? p->buckets : kDefaultBuckets;
  int64_t b4 = p->n4b;
  if (nb > 1 && p->n4b > 0) b4 = ((p->n4b + nb - 1) / nb + pad - 1) / pad * pad;
  nb = b4 > 0 ? (p->n4b + b4 - 1) / b4 : 1;
  const bool piped = nb > 1;
  if (piped) TRY(ensure_pipeline(p, nb));
  auto start_of = [&](int64_t b) { return b * b4; };
  auto len_of = [&](int64_t b) { return std::min(b4, p->n4b - b * b4); };
  auto apply = [&](int64_t b) -> int {
    for (int k = 0; k < G; ++k) {
      auto &d = p->devs[k];
      hipStream_t st = static_cast<hipStream_t>(streams[k]);
      HIP_TRY(hipSetDevice(d.hip_id));
      if (piped) HIP_TRY(hipStreamWaitEvent(st, d.ev_r[b], 0));
      cbx::LaunchConfig cfg = p->apply_cfg;
      cfg.num_cus = d.num_cus;
      cbx::SmaArgs a = offset_args(args[k], start_of(b), len_of(b));
      if (b == nb - 1) a = with_tail(a, start_of(b));
      HIP_TRY(cbx::launch_sma_apply(a, mom, cfg, st));
    }
    return CBX_OK;
  };
  for (int64_t b = 0; b < nb; ++b) {
    for (int k = 0; k < G; ++k) {
      auto &d = p->devs[k];
      hipStream_t st = static_cast<hipStream_t>(streams[k]);
      HIP_TRY(hipSetDevice(d.hip_id));
      cbx::LaunchConfig cfg = p->cfg;
      cfg.num_cus = d.num_cus;
      cbx::SmaArgs a = offset_args(args[k], start_of(b), len_of(b));
      if (b == nb - 1) a = with_tail(a, start_of(b));
      HIP_TRY(cbx::launch_sma_accumulate(a, b == 0, cfg, st));
      if (piped) {
        HIP_TRY(hipEventRecord(d.ev_a[b], st));
        HIP_TRY(hipStreamWaitEvent(d.comm_stream, d.ev_a[b], 0));
      }
    }
    NCCL_TRY(ncclGroupStart());
    for (int k = 0; k < G; ++k) {
      auto &d = p->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      const int64_t lo_f = start_of(b) * 4;
      const int64_t hi_f = b == nb - 1 ? p->n : (start_of(b) + len_of(b)) * 4;
      float *src = d.acc_ctrl + cbx::kCtrlFloats + lo_f, *dst = d.D_ctrl + cbx::kCtrlFloats + lo_f;
      size_t count = (size_t)(hi_f - lo_f);
      if (b == 0) {
        src -= cbx::kCtrlFloats;
        dst -= cbx::kCtrlFloats;
        count += cbx::kCtrlFloats;
      }
      NCCL_TRY(ncclAllReduce(src, dst, count, ncclFloat, ncclSum, d.comm,
                             piped ? d.comm_stream : static_cast<hipStream_t>(streams[k])));
    }
    NCCL_TRY(ncclGroupEnd());
    if (piped) {
      for (int k = 0; k < G; ++k) {
        auto &d = p->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        HIP_TRY(hipEventRecord(d.ev_r[b], d.comm_stream));
      }
      if (b >= 1) TRY(apply(b - 1));
    }
  }
  TRY(apply(nb - 1));
  return copies_total > 0 ? 1 : 0;
}

// crossbowSynchronisationSynchronousSGD (synch/synchronoussgd.c:13-106) over
// the caller's buffers: the all-reduce of every device's accumulated,
// lr-scaled gradient, the 1/wpc scale, the base momentum (the configured one,
// not forced to 0.9), z += D, the reset of the accumulator and base ->
// replica copies (common.c:198-220), in one apply pass per bucket.  G = 1 runs
// the multi-GPU algorithm with the identity all-reduce (the reference's
// single-GPU variant is err(), :5-11), as the context does.
int cbx_ssgd_plan_step(cbx_sma_plan *p, void *const *streams, float *const *z, float *const *last, float *const *acc,
                       int nreplicas, const int *replica_device, float *const *w, const int *locked, float momentum,
                       int wpc, int first) {
  TraceRange trace("cbx_ssgd_plan_step");
  if (!p) return fail(CBX_ERR_INVALID, "null plan");
  const int G = (int)p->devs.size();
  if (!streams || !z || !acc || nreplicas < 0 || (nreplicas > 0 && (!replica_device || !w || !locked)))
    return fail(CBX_ERR_INVALID, "cbx_ssgd_plan_step: missing arguments");
  if (wpc <= 0) return fail(CBX_ERR_INVALID, "S-SGD needs the work per clock (wpc %d)", wpc);
  if (first < 0 || first > nreplicas) return fail(CBX_ERR_INVALID, "first replica %d out of range", first);
  const bool mom = momentum > 0.0f;  // synchronoussgd.c:64
  if (mom && !last) return fail(CBX_ERR_INVALID, "momentum > 0 needs the base models' last buffers");
  std::vector<cbx::SsgdArgs> args(G);
  for (int k = 0; k < G; ++k) {
    cbx::SsgdArgs &a = args[k];
    std::memset(&a, 0, sizeof(a));
    if (!z[k] || !acc[k] || !aligned16(z[k]) || !aligned16(acc[k]) || (mom && (!last[k] || !aligned16(last[k]))))
      return fail(CBX_ERR_INVALID, "device %d: base buffers must be non-null and 16-byte aligned", k);
    a.z = reinterpret_cast<cbx::v4f *>(z[k]);
    a.last = mom ? reinterpret_cast<cbx::v4f *>(last[k]) : nullptr;
    a.acc = reinterpret_cast<cbx::v4f *>(acc[k]);
    a.D = p->ranks == 1 ? a.acc : reinterpret_cast<const cbx::v4f *>(p->devs[k].D_ctrl + cbx::kCtrlFloats);
    a.n4 = p->n4b;
    a.ratio = (float)(1.0 / (double)(float)wpc);  // :55
    a.momentum = mom ? momentum : 0.0f;
  }
  for (int id = first; id < nreplicas; ++id) {  // common.c:208: locked replicas from `first` on
    if (!locked[id]) continue;
    const int k = replica_device[id];
    if (k < 0 || k >= G) return fail(CBX_ERR_INVALID, "replica %d on device %d of %d", id, k, G);
    if (!w[id] || !aligned16(w[id])) return fail(CBX_ERR_INVALID, "replica %d: buffer must be 16-byte aligned", id);
    if (args[k].nrep >= cbx::kMaxReplicas)
      return fail(CBX_ERR_UNSUPPORTED, "more than %d locked replicas on one device", cbx::kMaxReplicas);
    args[k].w[args[k].nrep++] = reinterpret_cast<cbx::v4f *>(w[id]);
  }
  // Buckets as in the SMA step; at G > 1 with more than one, the all-reduce
  // of bucket k+1 runs on the plan's stream beside the apply of bucket k:
  //   stream      : [entry] [wait r(0)] K(0) [wait r(1)] K(1) ...
  //   comm_stream : [wait entry] AR(0) AR(1) ...
  const int64_t pad = cbx::kPadFloat4;
  int64_t nb = p->ranks == 1 ? 1 : (p->buckets > 0 ? p->buckets : kDefaultBuckets);
  int64_t b4 = p->n4b;
  if (nb > 1 && p->n4b > 0) b4 = ((p->n4b + nb - 1) / nb + pad - 1) / pad * pad;
  nb = b4 > 0 ? (p->n4b + b4 - 1) / b4 : 1;
  const bool piped = p->ranks > 1 && nb > 1;
  if (piped) {
    TRY(ensure_pipeline(p, nb));
    for (int k = 0; k < G; ++k) {  // everything the task steps accumulated, in stream order
      auto &d = p->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
      HIP_TRY(hipEventRecord(d.ev_a[0], static_cast<hipStream_t>(streams[k])));
      HIP_TRY(hipStreamWaitEvent(d.comm_stream, d.ev_a[0], 0));
    }
  }
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t s4 = b * b4, l4 = std::min(b4, p->n4b - s4);
    if (p->ranks > 1) {
      NCCL_TRY(ncclGroupStart());
      for (int k = 0; k < G; ++k) {
        auto &d = p->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        const int64_t hi_f = b == nb - 1 ? p->n : (s4 + l4) * 4;
        NCCL_TRY(ncclAllReduce(acc[k] + s4 * 4, d.D_ctrl + cbx::kCtrlFloats + s4 * 4, (size_t)(hi_f - s4 * 4),
                               ncclFloat, ncclSum, d.comm,
                               piped ? d.comm_stream : static_cast<hipStream_t>(streams[k])));
      }
      NCCL_TRY(ncclGroupEnd());
    }
    for (int k = 0; k < G; ++k) {
      auto &d = p->devs[k];
      hipStream_t st = static_cast<hipStream_t>(streams[k]);
      HIP_TRY(hipSetDevice(d.hip_id));
      if (piped) {
        HIP_TRY(hipEventRecord(d.ev_r[b], d.comm_stream));
        HIP_TRY(hipStreamWaitEvent(st, d.ev_r[b], 0));
      }
      cbx::SsgdArgs a = args[k];
      for (int r = 0; r < a.nrep; ++r) a.w[r] += s4;
      a.z += s4;
      if (a.last) a.last += s4;
      a.acc += s4;
      a.D += s4;
      a.n4 = l4;
      if (b == nb - 1) {  // the elements past the last whole trip ride this launch
        a.tail_lo = (p->n4b - s4) * 4;
        a.tail_hi = p->n - s4 * 4;
      }
      cbx::LaunchConfig cfg = p->ssgd_apply_cfg;
      cfg.num_cus = d.num_cus;
      HIP_TRY(cbx::launch_ssgd_apply(a, cfg, st));
    }
  }
  return CBX_OK;
}

// crossbowKernelOptimiserSynchronousSGD (kernels/optimisers/synchronoussgd.cu:
// 3-56) over the caller's buffers, one pass: weight decay into the replica's
// gradient, then the lr-scaled gradient added into the device's base-model
// gradient.  On `stream` = the device's model-synchronisation stream, after
// it waits for the task's gradient (:37-40), so the tasks of a clock add in
// stream order.
int cbx_ssgd_accumulate_buffers(void *stream, const float *w, float *g, float *acc, long long elements,
                                float learning_rate, float weight_decay) {
  TraceRange trace("cbx_ssgd_accumulate_buffers");
  if (elements <= 0 || elements * 4 + 4096 >= (1ll << 32))
    return fail(CBX_ERR_INVALID, "cbx_ssgd_accumulate_buffers: %lld elements out of range", elements);
  if (!g || !acc || (weight_decay > 0.0f && !w)) return fail(CBX_ERR_INVALID, "cbx_ssgd_accumulate_buffers: missing buffers");
  if (!aligned16(g) || !aligned16(acc) || (weight_decay > 0.0f && !aligned16(w)))
    return fail(CBX_ERR_INVALID, "cbx_ssgd_accumulate_buffers: buffers must be 16-byte aligned");
  int cus = 256;
  TRY(cus_of_current_device(&cus));
  cbx::SsgdArgs a;
  std::memset(&a, 0, sizeof(a));
  a.wsrc = reinterpret_cast<const cbx::v4f *>(w);
  a.g = reinterpret_cast<cbx::v4f *>(g);
  a.acc = reinterpret_cast<cbx::v4f *>(acc);
  a.n4 = bulk_float4s(elements);
  a.rate = -1.0f * learning_rate;  // :46
  a.wd = weight_decay;
  a.tail_lo = a.n4 * 4;
  a.tail_hi = elements;
  cbx::LaunchConfig cfg = cbx::aux_launch_config();
  cfg.num_cus = cus;
  HIP_TRY(cbx::launch_ssgd_accumulate(a, cfg, static_cast<hipStream_t>(stream)));
  return CBX_OK;
}

// crossbowCudnnBatchNormParamsSynchroniseEstimatedMeanAndVariable
// (cudnn/cudnnbatchnormparams.c:157-222) over the caller's statistics buffers,
// the same packed all-reduce as cbx_average_batchnorm_stats, on the plan's
// stream; device-synchronises before and after, as the reference does.
int cbx_sma_plan_average_batchnorm(cbx_sma_plan *p, int layers, const int *elements, float *const *mean,
                                   float *const *variance, const int *updated) {
  TraceRange trace("cbx_sma_plan_average_batchnorm");
  if (!p) return fail(CBX_ERR_INVALID, "null plan");
  if (layers < 0 || (layers > 0 && (!elements || !mean || !variance || !updated)))
    return fail(CBX_ERR_INVALID, "bad batch-norm statistics arguments");
  if (layers == 0 || p->ranks == 1) return CBX_OK;  // :165-166: nothing to average with one device
  TRY(ensure_pipeline(p, 1));
  std::vector<BnDevice> devs;
  for (auto &d : p->devs)
    devs.push_back({d.hip_id, d.global, d.comm, d.comm_stream, &d.bn_table, &d.bn_table_bytes, &d.bn_scratch,
                    &d.bn_scratch_bytes});
  return bn_average(devs, layers, elements, mean, variance, updated);
}

int cbx_sma_plan_set_buckets(cbx_sma_plan *p, int buckets) {
  if (!p) return fail(CBX_ERR_INVALID, "null plan");
  if (buckets < 0 || buckets > 4096) return fail(CBX_ERR_INVALID, "plan buckets must be 0..4096, got %d", buckets);
  p->buckets = buckets;
  return CBX_OK;
}

int cbx_sma_optimise_buffers(void *stream, float *w, float *g, float *last, float *s, long long elements,
                             float learning_rate, float momentum, float weight_decay) {
  TraceRange trace("cbx_sma_optimise_buffers");
  if (elements <= 0 || elements * 4 + 4096 >= (1ll << 32))
    return fail(CBX_ERR_INVALID, "cbx_sma_optimise_buffers: %lld elements out of range", elements);
  if (!w || !g || !s || (momentum > 0.0f && !last))
    return fail(CBX_ERR_INVALID, "cbx_sma_optimise_buffers: missing buffers");
  if (!aligned16(w) || !aligned16(g) || !aligned16(s) || (momentum > 0.0f && !aligned16(last)))
    return fail(CBX_ERR_INVALID, "cbx_sma_optimise_buffers: buffers must be 16-byte aligned");
  hipStream_t st = static_cast<hipStream_t>(stream);
  int cus = 256;
  TRY(cus_of_current_device(&cus));
  cbx::OptArgs a;
  std::memset(&a, 0, sizeof(a));
  a.w = reinterpret_cast<cbx::v4f *>(w);
  a.g = reinterpret_cast<cbx::v4f *>(g);
  a.last = momentum > 0.0f ? reinterpret_cast<cbx::v4f *>(last) : nullptr;
  a.s = reinterpret_cast<cbx::v4f *>(s);
  a.n4 = bulk_float4s(elements);
  a.rate = -1.0f * learning_rate;  // sma.cu:43
  a.momentum = momentum;
  a.wd = weight_decay;
  cbx::LaunchConfig cfg = cbx::aux_launch_config();
  cfg.num_cus = cus;
  a.tail_lo = a.n4 * 4;  // the elements past the last whole trip ride the same launch
  a.tail_hi = elements;
  HIP_TRY(cbx::launch_sma_optimise(a, cfg, st));
  return CBX_OK;
}

}  // extern "C"
