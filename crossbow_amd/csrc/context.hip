// context.hip -- execution context, model manager and SMA orchestration
// behind the C-ABI of include/crossbow_sma.h.
//
// MI355X-first restatement of the reference's native runtime for the model
// path: crossbowExecutionContext (clib-multigpu/executioncontext.c), the model
// manager (modelmanager.c), the model buffers (model.c, databuffer.c), solver
// configuration (solverconfiguration.c) and the SMA synchronisation
// (synch/sma.c, synch/common.c).  Differences by design:
//   * one device arena per GPU (one hipMalloc) holding the base model and every
//     replica buffer, instead of ~5 cudaMallocs per model;
//   * the SMA step is one fused kernel at G = 1 and kernel A + RCCL all-reduce
//     + kernel B at G > 1 (optionally bucketed and pipelined), instead of
//     3R+3 cuBLAS saxpys, R+4 copies and three cudaDeviceSynchronize;
//   * the Phase-D "copy base to replicas" decision travels with the all-reduce
//     (control block) instead of a host-side count;
//   * errors return codes; the JNI shim turns them back into exit(1).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <pthread.h>
#include <sched.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <fcntl.h>
#include <unistd.h>
#include <errno.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/crossbow_sma.h"
#include "sma_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(call)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return fail(CBX_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(call)                                                                             \
  do {                                                                                             \
    ncclResult_t r_ = (call);                                                                      \
    if (r_ != ncclSuccess)                                                                         \
      return fail(CBX_ERR_RCCL, "%s:%d %s: %s", __FILE__, __LINE__, #call, ncclGetErrorString(r_)); \
  } while (0)

// ROCTx range over one C-ABI call (tracing): rocprofv3
// --marker-trace shows each barrier step, staging pass, checkpoint and task
// step as a host range beside its kernels.  Without a tool attached a push /
// pop is a call through an empty dispatch table.
struct TraceRange {
  explicit TraceRange(const char *name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange &) = delete;
  TraceRange &operator=(const TraceRange &) = delete;
};

#define TRY(expr)            \
  do {                       \
    int rc_ = (expr);        \
    if (rc_ < 0) return rc_; \
  } while (0)

// ---------------------------------------------------------------------------
// Solver configuration, clib-multigpu/solverconfiguration.{h,c}
// ---------------------------------------------------------------------------
enum LrPolicy { LR_FIXED = 0, LR_INV, LR_STEP, LR_MULTISTEP, LR_EXP, LR_CLR, LR_LSR };

struct SolverConf {
  float alpha = 0.5f;  // solverconfiguration.c:17
  int tau = 1;
  LrPolicy policy = LR_FIXED;
  float learningRate = 0.0f;
  double gamma = 0.0;
  double power = 0.0;
  int size = 0;
  std::vector<int> steps;
  int step = 0;
  int warmuptasks = 0;
  float momentum = 0.0f;
  int momentumMethod = 0;
  float weightDecay = 0.0f;
  float baseModelMomentum = 0.0f;
  unsigned copy = 0;  // `_copy`, solverconfiguration.h:41-52
  int irregular = 0;  // variables with a learning-rate multiplier != 1 (executioncontext.c:1602)
  float circularLearningRate[3] = {0, 0, 0};  // CLR (executioncontext.c:1701-1718)
  float circularMomentum[3] = {0, 0, 0};
  int superConvergence = 0;

  // crossbowSolverConfGetLearningRate, solverconfiguration.c:116-162.
  int learning_rate(int task, float *out) {
    float rate = 0.0f;
    switch (policy) {
      case LR_FIXED: rate = learningRate; break;
      case LR_INV: rate = learningRate * (float)std::pow(1.0 + gamma * (double)(task + 1), -power); break;
      case LR_STEP:
        if (size <= 0) return fail(CBX_ERR_STATE, "step learning-rate policy with size 0");
        rate = learningRate * (float)std::pow(gamma, std::floor((double)((task + 1) / size)));
        break;
      case LR_MULTISTEP:
        if (step < (int)steps.size() && (task + 1) >= steps[step]) {
          step++;
          copy = 1;  // signal Phase D (solverconfiguration.c:133)
        }
        rate = learningRate * (float)std::pow(gamma, (double)step);
        break;
      case LR_LSR:
        if (warmuptasks <= 0) return fail(CBX_ERR_STATE, "LSR policy without warm-up tasks");
        if (task < warmuptasks) {
          rate = (learningRate * (float)task) / (float)warmuptasks;
        } else {
          if (step < (int)steps.size() && (task + 1) >= steps[step]) {
            step++;
            copy = 1;  // solverconfiguration.c:147
          }
          rate = learningRate * (float)std::pow(gamma, (double)step);
        }
        break;
      case LR_EXP: rate = learningRate * (float)std::pow(gamma, (double)(task + 1)); break;
      case LR_CLR: return fail(CBX_ERR_UNSUPPORTED, "circular learning rate is unsupported");  // :155-157
      default: return fail(CBX_ERR_UNSUPPORTED, "learning-rate policy %d unsupported", (int)policy);
    }
    *out = rate;
    return CBX_OK;
  }
};

// ---------------------------------------------------------------------------
// Model definition (theModel before the manager exists), model.c:8-200
// ---------------------------------------------------------------------------
struct Variable {
  int64_t offset_bytes;
  int64_t bytes;
  int64_t elements;
  float lr_multiplier = 1.0f;  // variable.c; read only by per-variable optimisers, not by SMA's
};

struct ModelDef {
  bool defined = false;
  int ops = 0;
  int64_t bytes = 0;       // setModel size (sum of capacities)
  int64_t offset = 0;      // model.c:151 running offset
  int64_t elements = 0;    // model.c:153
  int wpc = 0;
  int type = 0;            // update model type
  SolverConf conf;
  std::map<std::pair<int, int>, Variable> vars;  // (op id, order) -> variable
  std::vector<int> count_per_op;
  std::vector<float> host;  // initial values (PIN host buffer of theModel->data)
};

// The model manager's theta queue (thetaqueue.c, modelmanager.c:121-132): one
// cache-line slot per replica id.  FREE; BUSY = reserved by a task from
// acquireAccess until its release; SKIP = disabled.
enum ThetaState { kThetaFree = 0, kThetaBusy = 1, kThetaSkip = 2 };  // thetaqueue.c:6-8
struct alignas(64) ThetaSlot {
  std::atomic<int> state{kThetaFree};
};

struct Replica {
  int id = 0;
  int g = 0;          // global device index (id % G)
  int local = -1;     // local device slot, -1 if in another process
  int slot = 0;       // replica slot within its device
  int clock = 0;
  int updates = 0;
  SolverConf conf;
  pthread_mutex_t lock;
  hipEvent_t client = nullptr;  // end of the last optimiser step on a task stream (sma.cu:79)
};

enum TimingEv { EV_START = 0, EV_A, EV_AR, EV_B, EV_H2D0, EV_H2D1, EV_D2H0, EV_D2H1, EV_COUNT };

struct Device {
  int hip_id = 0;
  int g = 0;  // global device index
  // The device number in checkpoint file names, `model->dev` in the
  // reference (modelmanager.c:285,324,337): the selected HIP device id, or
  // the rank in the one-process-per-GPU form.
  int file_id = 0;
  hipStream_t stream = nullptr;       // model synchronisation stream (kernels)
  hipStream_t comm_stream = nullptr;  // RCCL all-reduce of the bucketed pipeline (G > 1)
  // Pipelined host-staged step (cbx_synchronise_staged): pinned H2D and D2H
  // run on their own streams (separate DMA engines, both PCIe directions at
  // once) beside the kernels on `stream`.  Created on first use.
  hipStream_t h2d_stream = nullptr;
  hipStream_t d2h_stream = nullptr;
  hipEvent_t stage_entry = nullptr;       // sync stream -> h2d stream at entry
  hipEvent_t stage_done = nullptr;        // d2h stream -> sync stream at exit
  std::vector<hipEvent_t> stage_h2d;      // per bucket: inputs landed
  std::vector<hipEvent_t> stage_k;        // per bucket: outputs computed
  std::vector<hipEvent_t> bucket_acc;  // per bucket: kernel A done (stream -> comm_stream)
  std::vector<hipEvent_t> bucket_red;  // per bucket: all-reduce done (comm_stream -> stream)
  // Cross-step pipeline (cbx_set_pipeline_mode 1): kernels A run on a_stream,
  // kernels B stay on `stream`; bucket_b[k] marks B(k) done, which A(k) of
  // the next step waits for instead of the whole previous step.
  hipStream_t a_stream = nullptr;
  std::vector<hipEvent_t> bucket_b;
  hipEvent_t cross_entry = nullptr;
  float *decision = nullptr;           // 2 floats: the Phase-D decision, by step parity
  bool cross_valid = false;            // the last step was cross-pipelined ...
  int64_t cross_nb = 0;                // ... over this many buckets ...
  unsigned long long cross_foreign = 0;  // ... and nothing else was enqueued since
  unsigned cross_parity = 0;
  ncclComm_t comm = nullptr;
  // Peer-read all-reduce (cbx_set_allreduce_algorithm PEER): kernel A done /
  // this device's shard of D reduced; the other devices' streams wait on them.
  hipEvent_t peer_a = nullptr;
  hipEvent_t peer_r = nullptr;
  // Stream-order check (cbx_set_order_check): timestamps of the last two
  // split steps, by step parity, per bucket.  Every point is the stop
  // timestamp of a dispatch (a start event is a marker packet of its own):
  // an empty probe dispatch right after each wait (before kernel A, before
  // the collective, before kernel B), one right after the collective, and
  // kernels A and B themselves.
  struct OrderStep {
    bool valid = false;
    bool cont = false;  // continued the previous step bucket by bucket (mode 1, no join)
    int64_t nb = 0;
    std::vector<hipEvent_t> pa, a1, c0, c1, pb, b1;  // probe<A, A, probe<coll, probe>coll, probe<B, B
  };
  OrderStep ord[2];
  // Owned timing events, 6 per bucket (pa, a1, c0, c1, pb, b1).  While the
  // check is on, kernel A's and B's dispatches stop these instead of the
  // reused bucket_acc / bucket_b, and the cross-stream waits use them too,
  // so the two recorded steps keep their own timestamps.
  std::vector<hipEvent_t> ord_pool[2];
  unsigned ord_cur = 0;
  cbx::BnSegment *bn_table = nullptr;  // batch-norm averaging: segment table (device)
  size_t bn_table_bytes = 0;
  float *bn_scratch = nullptr;         // packed statistics, all-reduced
  size_t bn_scratch_bytes = 0;
  int num_cus = 256;
  // Arena: [base data][base gradient(ctrl+acc)][base diff(ctrl+D)][base last]
  //        then per replica [data][diff][last][gradient].
  char *arena = nullptr;
  char *host = nullptr;  // pinned mirror, same layout (lazy)
  size_t arena_bytes = 0;
  size_t stride = 0;  // bytes per buffer slot
  int base_slots = 0;  // replica slots inside the arena (replicas per device at creation)
  // Replica slots added by autotune (modelmanager.c:362-470) beyond the arena:
  // one block of kReplicaSlots buffers each, so existing pointers stay valid.
  std::vector<char *> extra;
  std::vector<char *> extra_host;
  std::vector<int> replicas;  // global ids, increasing
  hipEvent_t synched = nullptr;     // end-of-step event when timing is off
  bool synched_by_dispatch = false;  // the step's last dispatch completes `synched` itself
  hipEvent_t step_event = nullptr;  // end of the last step (cbx_step_event)
  hipEvent_t ev[EV_COUNT] = {};
  bool ev_valid[EV_COUNT] = {};
  // Per-step timing ring: events {START, A, AR, B} of the last kRing steps,
  // so a benchmark reads every launch of its timed region afterwards without
  // a host synchronisation between steps.
  static constexpr int kRing = 1024;
  std::vector<hipEvent_t> ring;
  std::vector<char> ring_split;
  // 1: this slot recorded no START; its step queued right behind the previous
  // slot's fused step, whose stop event stands in as its start (ring_start).
  std::vector<char> ring_from_prev;
  bool start_chosen = false;  // step_start_event decided this slot's ring_from_prev
  int ring_pos = 0;
  int ring_count = 0;
};

}  // namespace

struct cbx_context {
  std::vector<Device> devs;
  int G = 1;           // global device count (ranks)
  bool per_rank = false;
  ModelDef model;
  bool manager = false;
  int R = 0;           // replicas per device
  // R * G.  Task threads read it (the theta queue) while the barrier thread
  // may add or delete replicas (autotune), hence atomic.
  std::atomic<int> size{0};
  int sync_type = CBX_SYNC_BSP;
  std::vector<Replica *> replicas;  // global id -> replica (all ids; remote ones have local = -1)
  // Replicas removed by cbx_del_model.  A task thread may still be spinning
  // on one's clock or blocked on its lock (cbx_get_next_or_wait), so the
  // objects live until cbx_free instead of being deleted at once.
  std::vector<Replica *> retired;
  std::vector<int> locked;
  std::unique_ptr<ThetaSlot[]> theta;  // kMaxReplicas * G slots, index = replica id
  std::atomic<unsigned> theta_iter{0};  // round-robin cursor (thetaqueue.c:95-104)
  int64_t n = 0;       // model elements
  int64_t n4 = 0;      // padded float4 count
  bool has_last = false;
  unsigned long long version = 0;
  // BN operators whose running statistics travel with the checkpoint
  // (executioncontext.c:2352-2364): op id -> per-local-device buffers.
  struct BnStats {
    int elements = 0;
    std::vector<float *> mean, variance;
  };
  std::map<int, BnStats> bn_stats;
  bool timing = false;
  cbx::LaunchConfig cfg;
  // Optimiser step and S-SGD kernels (one float4 stream per buffer, few reads).
  cbx::LaunchConfig aux_cfg = cbx::aux_launch_config();
  // Write-heavy barrier kernels of DEFAULT and S-SGD (scripts/barrier_sweep.py).
  cbx::LaunchConfig broadcast_cfg = cbx::broadcast_launch_config();
  cbx::LaunchConfig ssgd_apply_cfg = cbx::ssgd_apply_launch_config();
  // Kernel B of the split SMA path (scripts/apply_sweep.py).
  cbx::LaunchConfig apply_cfg = cbx::sma_apply_launch_config();
  int64_t bucket_elems = 0;
  bool force_split = false;
  bool last_step_split = false;
  int pipeline_mode = 0;  // 0 bucketed within a step, 1 across steps (G > 1 split path)
  int cross_wait_stride = 1;  // mode 1: buckets per cross-step wait
  int allreduce_group = 1;     // pipelined split path: buckets per comm-stream wait
  int allreduce_algo = CBX_ALLREDUCE_RCCL;
  int staging_mode = CBX_STAGING_ZEROCOPY;  // cbx_synchronise_staged: zero-copy kernels or DMA copies
  cbx::LaunchConfig staged_cfg = cbx::staged_launch_config();
  bool peer_ready = false;     // hipDeviceEnablePeerAccess done between every pair of devices
  bool order_check = false;    // record per-bucket timestamps of split steps (cbx_set_order_check)
  // Fault injection for the order check's own test: $CBX_FAULT_SKIP_COMM_WAIT
  // at context creation drops the comm stream's wait on kernel A, so the
  // collective races its input (results are then wrong; tests only).
  bool fault_skip_comm_wait = std::getenv("CBX_FAULT_SKIP_COMM_WAIT") != nullptr;
  // Bumped by every C-ABI call that may enqueue work on a sync stream other
  // than the barrier path itself: a cross-step pipelined step then joins the
  // whole sync stream instead of waiting bucket by bucket.
  std::atomic<unsigned long long> foreign_ops{0};
};

namespace {

// ---------------------------------------------------------------------------
// Arena layout helpers
// ---------------------------------------------------------------------------
constexpr int kBaseSlots = 4;     // data, gradient, diff, last
constexpr int kReplicaSlots = 4;  // data, diff, last, gradient
constexpr size_t kAlign = 2u << 20;
// Extra bytes between consecutive buffer slots, so the 2R+2 streams of one
// element index do not all start on the same 2 MiB boundary (measured +1-2 %
// on the fused kernel, scripts/membench.hip, profiles/r01).
constexpr size_t kSlotStagger = 4096;
// Buckets of the G > 1 pipeline when cbx_set_bucket_elements was not called.
constexpr int64_t kDefaultBuckets = 8;

size_t slot_index_base(int kind) {
  switch (kind) {
    case CBX_BUF_DATA: return 0;
    case CBX_BUF_GRADIENT: return 1;
    case CBX_BUF_DIFF: return 2;
    default: return 3;
  }
}

size_t slot_index_replica(int slot, int kind) {
  size_t k;
  switch (kind) {
    case CBX_BUF_DATA: k = 0; break;
    case CBX_BUF_DIFF: k = 1; break;
    case CBX_BUF_LAST: k = 2; break;
    default: k = 3; break;
  }
  return kBaseSlots + (size_t)slot * kReplicaSlots + k;
}

// Byte offset of the model data inside a slot: acc and D carry a 256-byte
// control block in front (sma_internal.h).
size_t data_offset(bool ctrl) { return ctrl ? (size_t)cbx::kCtrlFloats * sizeof(float) : 0; }

float *slot_ptr(char *arena, const Device &d, size_t slot, bool ctrl) {
  return reinterpret_cast<float *>(arena + slot * d.stride + data_offset(ctrl));
}

bool base_has(const cbx_context *c, int kind) { return kind != CBX_BUF_LAST || c->has_last; }

float *base_dev(const cbx_context *c, const Device &d, int kind) {
  const bool ctrl = (kind == CBX_BUF_GRADIENT || kind == CBX_BUF_DIFF);
  return slot_ptr(d.arena, d, slot_index_base(kind), ctrl);
}

float *base_ctrl(const Device &d, int kind) {
  return reinterpret_cast<float *>(d.arena + slot_index_base(kind) * d.stride);
}

size_t replica_kind_index(int kind) { return slot_index_replica(0, kind) - kBaseSlots; }

float *replica_dev(const Device &d, const Replica &r, int kind) {
  if (r.slot >= d.base_slots)
    return reinterpret_cast<float *>(d.extra[r.slot - d.base_slots] + replica_kind_index(kind) * d.stride);
  return slot_ptr(d.arena, d, slot_index_replica(r.slot, kind), false);
}

float *base_host(const Device &d, int kind) {
  const bool ctrl = (kind == CBX_BUF_GRADIENT || kind == CBX_BUF_DIFF);
  return slot_ptr(d.host, d, slot_index_base(kind), ctrl);
}

float *replica_host(const Device &d, const Replica &r, int kind) {
  if (r.slot >= d.base_slots)
    return reinterpret_cast<float *>(d.extra_host[r.slot - d.base_slots] + replica_kind_index(kind) * d.stride);
  return slot_ptr(d.host, d, slot_index_replica(r.slot, kind), false);
}

// The *_q checks are for calls that enqueue no device work (the barrier path,
// replica locks, queries); the others also count a possible foreign op.
int check_ctx_q(cbx_context *c) {
  if (!c) return fail(CBX_ERR_INVALID, "null context");
  return CBX_OK;
}

int check_ctx(cbx_context *c) {
  TRY(check_ctx_q(c));
  c->foreign_ops.fetch_add(1, std::memory_order_relaxed);
  return CBX_OK;
}

int check_manager_q(cbx_context *c) {
  TRY(check_ctx_q(c));
  if (!c->manager) return fail(CBX_ERR_STATE, "model manager not created (call cbx_set_model_manager)");
  return CBX_OK;
}

int check_manager(cbx_context *c) {
  TRY(check_manager_q(c));
  c->foreign_ops.fetch_add(1, std::memory_order_relaxed);
  return CBX_OK;
}

int check_replica_q(cbx_context *c, int id, bool need_local) {
  TRY(check_manager_q(c));
  if (id < 0 || id >= c->size) return fail(CBX_ERR_INVALID, "replica id %d out of range [0, %d)", id, c->size.load());
  if (need_local && c->replicas[id]->local < 0)
    return fail(CBX_ERR_INVALID, "replica %d lives in another process (device %d)", id, c->replicas[id]->g);
  return CBX_OK;
}

int check_replica(cbx_context *c, int id, bool need_local) {
  TRY(check_manager(c));
  if (id < 0 || id >= c->size) return fail(CBX_ERR_INVALID, "replica id %d out of range [0, %d)", id, c->size.load());
  if (need_local && c->replicas[id]->local < 0)
    return fail(CBX_ERR_INVALID, "replica %d lives in another process (device %d)", id, c->replicas[id]->g);
  return CBX_OK;
}

int local_of(cbx_context *c, int g) {
  for (size_t k = 0; k < c->devs.size(); ++k)
    if (c->devs[k].g == g) return (int)k;
  return -1;
}

int gfx950_device_count(int *count) {
  int n = 0;
  *count = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return CBX_OK;
  }
  int k = 0;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) != hipSuccess) continue;
    if (std::strncmp(p.gcnArchName, "gfx950", 6) == 0) ++k;
  }
  *count = k;
  return CBX_OK;
}

int open_device(Device &d, int hip_id, int g) {
  int total = 0;
  hipError_t ce = hipGetDeviceCount(&total);
  if (ce != hipSuccess) {
    (void)hipGetLastError();
    return fail(CBX_ERR_NO_DEVICE, "no MI355X visible: %s", hipGetErrorString(ce));
  }
  if (hip_id < 0 || hip_id >= total) return fail(CBX_ERR_NO_DEVICE, "device %d not visible (%d devices)", hip_id, total);
  hipDeviceProp_t p;
  HIP_TRY(hipGetDeviceProperties(&p, hip_id));
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    return fail(CBX_ERR_NO_DEVICE, "device %d is %s, this library is built for gfx950 (MI355X) only", hip_id,
                p.gcnArchName);
  d.hip_id = hip_id;
  d.g = g;
  d.file_id = g;
  d.num_cus = p.multiProcessorCount;
  HIP_TRY(hipSetDevice(hip_id));
  // executioncontext.c:324: one non-blocking model-synchronisation stream.
  HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&d.comm_stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&d.synched, hipEventDisableTiming));
  for (int k = 0; k < EV_COUNT; ++k) HIP_TRY(hipEventCreate(&d.ev[k]));
  return CBX_OK;
}

void close_device(Device &d) {
  if (d.stream == nullptr && d.arena == nullptr) return;
  (void)hipSetDevice(d.hip_id);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  if (d.comm_stream) (void)hipStreamSynchronize(d.comm_stream);
  if (d.comm) (void)ncclCommDestroy(d.comm);
  if (d.arena) (void)hipFree(d.arena);
  for (char *p : d.extra)
    if (p) (void)hipFree(p);
  for (char *p : d.extra_host)
    if (p) (void)hipHostFree(p);
  if (d.bn_table) (void)hipFree(d.bn_table);
  if (d.bn_scratch) (void)hipFree(d.bn_scratch);
  if (d.host) (void)hipHostFree(d.host);
  if (d.synched) (void)hipEventDestroy(d.synched);
  for (int k = 0; k < EV_COUNT; ++k)
    if (d.ev[k]) (void)hipEventDestroy(d.ev[k]);
  for (hipEvent_t e : d.ring) (void)hipEventDestroy(e);
  for (hipEvent_t e : d.bucket_acc) (void)hipEventDestroy(e);
  for (hipEvent_t e : d.bucket_red) (void)hipEventDestroy(e);
  if (d.a_stream) (void)hipStreamSynchronize(d.a_stream);
  for (hipEvent_t e : d.bucket_b) (void)hipEventDestroy(e);
  if (d.cross_entry) (void)hipEventDestroy(d.cross_entry);
  for (auto &pool : d.ord_pool)
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  if (d.peer_a) (void)hipEventDestroy(d.peer_a);
  if (d.peer_r) (void)hipEventDestroy(d.peer_r);
  if (d.decision) (void)hipFree(d.decision);
  if (d.a_stream) (void)hipStreamDestroy(d.a_stream);
  for (hipStream_t st : {d.h2d_stream, d.d2h_stream})
    if (st) (void)hipStreamSynchronize(st);
  for (hipEvent_t e : d.stage_h2d) (void)hipEventDestroy(e);
  for (hipEvent_t e : d.stage_k) (void)hipEventDestroy(e);
  if (d.stage_entry) (void)hipEventDestroy(d.stage_entry);
  if (d.stage_done) (void)hipEventDestroy(d.stage_done);
  if (d.h2d_stream) (void)hipStreamDestroy(d.h2d_stream);
  if (d.d2h_stream) (void)hipStreamDestroy(d.d2h_stream);
  if (d.stream) (void)hipStreamDestroy(d.stream);
  if (d.comm_stream) (void)hipStreamDestroy(d.comm_stream);
  d = Device();
}

// The current ring slot's event `ev` (START..B) when timing is enabled, for
// a dispatch to timestamp itself (hipExtLaunchKernelGGL); else nullptr.
hipEvent_t ring_event(cbx_context *c, Device &d, int ev) {
  if (!c->timing || d.ring.empty()) return nullptr;
  return d.ring[(size_t)d.ring_pos * 4 + ev];
}

// The stop event of ring slot `slot`'s step: EV_A for a fused step (kind 0),
// EV_B for a split one.
hipEvent_t ring_stop(Device &d, int slot) {
  return d.ring[(size_t)slot * 4 + (d.ring_split[slot] == 0 ? EV_A : EV_B)];
}

// The START event for the first dispatch of a fused (kind 0) or pipelined
// split (kind 2) step.  A dispatch start event is a marker packet that costs
// the stream ~4.5 us per launch, while a stop event costs nothing
// (scripts/event_ts_probe.hip: 20.8 vs 16.4 us per back-to-back launch).
// When the previous slot is a step of the same kind whose stop has not
// completed yet, this step is enqueued behind a busy GPU: that stop stands in
// as this step's start (a fused step queues right behind it on the same
// stream; a pipelined step's span becomes its stop-to-stop share of the
// pipeline) and no marker is added.  Otherwise (an idle GPU, another kind of
// step) START is recorded.
hipEvent_t step_start_event(cbx_context *c, Device &d, int kind) {
  if (!c->timing || d.ring.empty()) return nullptr;
  const int slot = d.ring_pos;
  d.ring_from_prev[slot] = 0;
  if (d.ring_count > 0) {
    const int prev = (slot + Device::kRing - 1) % Device::kRing;
    const bool busy = d.ring_split[prev] == kind && hipEventQuery(ring_stop(d, prev)) == hipErrorNotReady;
    (void)hipGetLastError();  // hipEventQuery leaves NotReady as the thread's last error
    if (busy) {
      d.ring_from_prev[slot] = 1;
      d.start_chosen = true;
      return nullptr;
    }
  }
  d.start_chosen = true;
  return d.ring[(size_t)slot * 4 + EV_START];
}

// The event that opens ring slot `slot`: its START, or the previous slot's
// stop when the step was enqueued behind it (step_start_event).
hipEvent_t ring_start(Device &d, int slot) {
  if (!d.ring_from_prev.empty() && d.ring_from_prev[slot])
    return ring_stop(d, (slot + Device::kRing - 1) % Device::kRing);
  return d.ring[(size_t)slot * 4 + EV_START];
}

// Record a timing marker when timing is enabled.  Step events (START..B) go
// to the current ring slot, staging events to the fixed ones.
int mark(cbx_context *c, Device &d, int ev) {
  if (!c->timing) return CBX_OK;
  if (ev <= EV_B && !d.ring.empty()) {
    HIP_TRY(hipEventRecord(d.ring[(size_t)d.ring_pos * 4 + ev], d.stream));
    return CBX_OK;
  }
  HIP_TRY(hipEventRecord(d.ev[ev], d.stream));
  d.ev_valid[ev] = true;
  return CBX_OK;
}

// kind: 0 fused (START, A=B), 1 split in order (START, A, AR, B),
// 2 split pipelined (START, B only: per-kernel spans are not separable).
void ring_advance(cbx_context *c, Device &d, int kind) {
  if (!c->timing || d.ring.empty()) return;
  d.ring_split[d.ring_pos] = (char)kind;
  if (!d.start_chosen) d.ring_from_prev[d.ring_pos] = 0;  // a path that records START itself
  d.start_chosen = false;
  d.ring_pos = (d.ring_pos + 1) % Device::kRing;
  if (d.ring_count < Device::kRing) d.ring_count++;
}

// Elapsed ms between events a and b of ring slot `slot` (-1 if absent).
int ring_span(Device &d, int slot, int a, int b, float *out) {
  *out = -1.0f;
  HIP_TRY(hipEventSynchronize(d.ring[(size_t)slot * 4 + b]));
  hipEvent_t from = a == EV_START ? ring_start(d, slot) : d.ring[(size_t)slot * 4 + a];
  HIP_TRY(hipEventElapsedTime(out, from, d.ring[(size_t)slot * 4 + b]));
  return CBX_OK;
}

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

// cbx_set_force_split at G = 1: the split pipeline runs over a one-rank
// communicator so a single-GPU host exercises kernel A + RCCL + kernel B.
int ensure_one_rank_comm(cbx_context *c) {
  if (c->G != 1 || !c->force_split || c->devs[0].comm != nullptr) return CBX_OK;
  Device &d = c->devs[0];
  HIP_TRY(hipSetDevice(d.hip_id));
  int dev = d.hip_id;
  NCCL_TRY(ncclCommInitAll(&d.comm, 1, &dev));
  return CBX_OK;
}

// ---------------------------------------------------------------------------
// Peer-read all-reduce, single process over G devices (sma_internal.h,
// PeerArgs).  Per device, all on its sync stream:
//   A(g)  [wait A(h) of every other device]  R(g)  [wait R(h) ...]  B(g)
// R(g) sums shard g of every device's acc into this device's D (device
// order from +0), B(g) reads each shard of D from its owner.  The next
// step's A(h) follows B(h) on h's stream, and B(h) waited for every R, so
// no device overwrites an acc another device is still reading; R of the
// next step waits for every A of it, which follow every B of this one.
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

int sma_step_peer(cbx_context *c, std::vector<cbx::SmaArgs> &args, bool mom) {
  TRY(ensure_peer_access(c));
  const int G = (int)c->devs.size();
  const int64_t pad = cbx::kPadFloat4;
  const int64_t s4 = ((c->n4 + G - 1) / G + pad - 1) / pad * pad;  // float4s per shard
  cbx::PeerArgs p;
  std::memset(&p, 0, sizeof(p));
  p.G = G;
  p.shard4 = s4;
  for (int h = 0; h < G; ++h) {
    p.ctrl_in[h] = base_ctrl(c->devs[h], CBX_BUF_GRADIENT);
    p.D[h] = reinterpret_cast<const cbx::v4f *>(base_dev(c, c->devs[h], CBX_BUF_DIFF));
  }
  for (int k = 0; k < G; ++k) {
    Device &d = c->devs[k];
    HIP_TRY(hipSetDevice(d.hip_id));
    cbx::LaunchConfig cfg = c->cfg;
    cfg.num_cus = d.num_cus;
    HIP_TRY(cbx::launch_sma_accumulate(args[k], true, cfg, d.stream, {ring_event(c, d, EV_START), ring_event(c, d, EV_A)}));
    HIP_TRY(hipEventRecord(d.peer_a, d.stream));
  }
  for (int k = 0; k < G; ++k) {
    Device &d = c->devs[k];
    HIP_TRY(hipSetDevice(d.hip_id));
    for (int h = 0; h < G; ++h)
      if (h != k) HIP_TRY(hipStreamWaitEvent(d.stream, c->devs[h].peer_a, 0));
    const int64_t start = std::min<int64_t>((int64_t)k * s4, c->n4);
    cbx::PeerArgs r = p;
    for (int h = 0; h < G; ++h)
      r.acc[h] = reinterpret_cast<const cbx::v4f *>(base_dev(c, c->devs[h], CBX_BUF_GRADIENT)) + start;
    r.out = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_DIFF)) + start;
    r.ctrl_out = base_ctrl(d, CBX_BUF_DIFF);
    r.n4 = std::min(s4, c->n4 - start);  // 0 for a trailing empty shard: block 0 still sums the control block
    cbx::LaunchConfig cfg = c->apply_cfg;
    cfg.num_cus = d.num_cus;
    HIP_TRY(cbx::launch_sma_peer_reduce(r, cfg, d.stream, {nullptr, ring_event(c, d, EV_AR)}));
    HIP_TRY(hipEventRecord(d.peer_r, d.stream));
  }
  for (int k = 0; k < G; ++k) {
    Device &d = c->devs[k];
    HIP_TRY(hipSetDevice(d.hip_id));
    for (int h = 0; h < G; ++h)
      if (h != k) HIP_TRY(hipStreamWaitEvent(d.stream, c->devs[h].peer_r, 0));
    cbx::LaunchConfig cfg = c->apply_cfg;
    cfg.num_cus = d.num_cus;
    HIP_TRY(cbx::launch_sma_peer_apply(args[k], p, mom, cfg, d.stream, {nullptr, step_stop_event(c, d, EV_B)}));
    ring_advance(c, d, 1);
    d.cross_valid = false;
  }
  c->last_step_split = true;
  return CBX_OK;
}

int sma_step(cbx_context *c, int first) {
  const bool mom = c->has_last && c->model.conf.momentum > 0;  // sma.c:150 (base conf)
  std::vector<cbx::SmaArgs> args(c->devs.size());
  int copies_total = 0;
  for (size_t k = 0; k < c->devs.size(); ++k) {
    int cp = 0;
    TRY(build_args(c, c->devs[k], first, args[k], &cp));
    copies_total += cp;
  }

  TRY(ensure_one_rank_comm(c));
  if (c->allreduce_algo == CBX_ALLREDUCE_PEER && c->G > 1) {
    TRY(sma_step_peer(c, args, mom));
  } else if (c->G == 1 && !c->force_split) {
    // Single GPU: Phase B is the identity, so A + C (+ D) fuse into one pass.
    // (sma.c:63 waits on base->updated; every producer of z is this stream,
    // so stream order already gives that dependency.)
    Device &d = c->devs[0];
    HIP_TRY(hipSetDevice(d.hip_id));
    cbx::LaunchConfig cfg = c->cfg;
    cfg.num_cus = d.num_cus;
    // The dispatch timestamps its own (start, stop) ring events: no marker
    // packets between steps (each costs ~3 us of stream time, membench v4).
    HIP_TRY(cbx::launch_sma_fused(args[0], mom, copies_total > 0, cfg, d.stream,
                                  {step_start_event(c, d, 0), step_stop_event(c, d, EV_A)}));
    ring_advance(c, d, 0);
    d.cross_valid = false;
    c->last_step_split = false;
  } else {
    // G > 1: kernel A, grouped RCCL all-reduce of acc (+ control block),
    // kernel B.  With one bucket everything runs in order on the sync
    // stream.  With nb > 1 buckets the all-reduce runs on a second stream:
    //   stream      : A(0) A(1) [wait red(0)] B(0) A(2) [wait red(1)] B(1) ...
    //   comm_stream :      [wait acc(0)] AR(0) [wait acc(1)] AR(1) ...
    // so kernel A of bucket k+1 overlaps the xGMI all-reduce of bucket k.
    const int64_t pad = cbx::kPadFloat4;
    int64_t b4 = c->n4;
    if (c->bucket_elems > 0) {
      b4 = ((c->bucket_elems / 4 + pad - 1) / pad) * pad;
    } else if (c->G > 1) {
      b4 = ((c->n4 / kDefaultBuckets + pad - 1) / pad) * pad;  // auto: kDefaultBuckets buckets
    }
    if (b4 <= 0 || b4 > c->n4) b4 = c->n4;
    const int64_t nb = (c->n4 + b4 - 1) / b4;
    const bool pipelined = nb > 1;
    // Cross-step mode (cbx_set_pipeline_mode 1): kernels A on a_stream, B on
    // the sync stream.  A(k) waits only for B(k) of the previous step, so the
    // next step's first buckets run while this step's last all-reduces are
    // still on the link:
    //   a_stream    : [wait b(0)'] A(0) [wait b(1)'] A(1) ...
    //   comm_stream : [wait acc(0)] AR(0) [wait acc(1)] AR(1) ...
    //   stream      : [wait red(0)] B(0) [wait red(1)] B(1) ...
    // A step joins the whole sync stream instead when anything else was
    // enqueued since the last cross-pipelined step (foreign_ops).
    const bool cross = pipelined && c->pipeline_mode == 1;
    const bool rsag = c->allreduce_algo == CBX_ALLREDUCE_RSAG;
    // Per-bucket events ride on the kernels' own dispatch packets (stop
    // event) instead of a separate hipEventRecord marker, which left a
    // ~10 us gap on the sync stream per bucket: -2 to -8 % per step
    // (scripts/dispatch_event_ab.py, profiles/r01/dispatch_event_ab.json).
    // Mode 1: A(k) waits for B(k + stride - 1) of the last step once per
    // `stride` buckets (it implies B(k..): same stream).  Each satisfied
    // cross-queue wait still costs the waiting queue ~10 us; fewer waits
    // trade that for less cross-step overlap (cbx_set_cross_wait_stride).
    const int64_t wait_stride = std::max(1, c->cross_wait_stride);
    const unsigned long long foreign = c->foreign_ops.load(std::memory_order_acquire);
    std::vector<char> join(c->devs.size(), 1);
    for (size_t k = 0; k < c->devs.size(); ++k) {
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
        if (!d.a_stream) {
          HIP_TRY(hipStreamCreateWithFlags(&d.a_stream, hipStreamNonBlocking));
          HIP_TRY(hipEventCreateWithFlags(&d.cross_entry, hipEventDisableTiming));
          HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d.decision), 256));
          HIP_TRY(hipMemsetAsync(d.decision, 0, 256, d.stream));
          d.cross_valid = false;
        }
        join[k] = !d.cross_valid || d.cross_nb != nb || d.cross_foreign != foreign;
        if (join[k]) {
          HIP_TRY(hipEventRecord(d.cross_entry, d.stream));
          HIP_TRY(hipStreamWaitEvent(d.a_stream, d.cross_entry, 0));
        }
      }
    }
    // Stream-order check: a fresh set of per-bucket timestamps for this step.
    const bool ocheck = c->order_check && c->timing;
    for (size_t k = 0; ocheck && k < c->devs.size(); ++k) {
      Device &d = c->devs[k];
      HIP_TRY(hipSetDevice(d.hip_id));
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
    // `wait_acc`: the comm stream first waits for kernel A of that bucket
    // (-1: no wait; an earlier all-reduce of the same group already waited
    // on a later bucket, which implies this one: A runs in order).
    auto allreduce = [&](int64_t b, bool on_comm, int64_t wait_acc) -> int {
      const int64_t start = b * b4;
      const int64_t len = std::min(b4, c->n4 - start);
      // common.c:14-54: grouped all-reduce, fp32 sum.  Bucket 0 also carries
      // the control block that sits right in front of the data.
      if (on_comm && wait_acc >= 0 && !c->fault_skip_comm_wait) {
        for (size_t k = 0; k < c->devs.size(); ++k) {
          Device &d = c->devs[k];
          HIP_TRY(hipSetDevice(d.hip_id));
          HIP_TRY(hipStreamWaitEvent(d.comm_stream, ocheck ? d.ord[d.ord_cur].a1[wait_acc] : d.bucket_acc[wait_acc], 0));
        }
      }
      for (size_t k = 0; ocheck && k < c->devs.size(); ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        HIP_TRY(cbx::launch_order_probe(on_comm ? d.comm_stream : d.stream, {nullptr, d.ord[d.ord_cur].c0[b]}));
      }
      if (rsag) {
        // Reduce-scatter form: shard g of the bucket (len / G float4s) is
        // reduced on rank g, which applies the base momentum to its shard of
        // last; the all-gather of last (or of D without momentum) then hands
        // every rank the whole bucket of D' for kernel B.  The control block
        // rides a 64-float all-reduce grouped with bucket 0's reduce-scatter.
        const int64_t sh4 = len / c->G;
        NCCL_TRY(ncclGroupStart());
        for (size_t k = 0; k < c->devs.size(); ++k) {
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
        for (size_t k = 0; k < c->devs.size(); ++k) {
          if (!mom) break;
          Device &d = c->devs[k];
          HIP_TRY(hipSetDevice(d.hip_id));
          cbx::SmaArgs a = offset_args(args[k], start + d.g * sh4, sh4);
          cbx::LaunchConfig cfg = c->apply_cfg;
          cfg.num_cus = d.num_cus;
          HIP_TRY(cbx::launch_sma_shard_momentum(a, cfg, on_comm ? d.comm_stream : d.stream));
        }
        NCCL_TRY(ncclGroupStart());
        for (size_t k = 0; k < c->devs.size(); ++k) {
          Device &d = c->devs[k];
          HIP_TRY(hipSetDevice(d.hip_id));
          float *buf = base_dev(c, d, gather) + start * 4;
          NCCL_TRY(ncclAllGather(buf + d.g * sh4 * 4, buf, (size_t)sh4 * 4, ncclFloat, d.comm,
                                 on_comm ? d.comm_stream : d.stream));
        }
        NCCL_TRY(ncclGroupEnd());
      } else {
        NCCL_TRY(ncclGroupStart());
        for (size_t k = 0; k < c->devs.size(); ++k) {
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
      for (size_t k = 0; ocheck && k < c->devs.size(); ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        HIP_TRY(cbx::launch_order_probe(on_comm ? d.comm_stream : d.stream, {nullptr, d.ord[d.ord_cur].c1[b]}));
      }
      if (on_comm) {
        for (size_t k = 0; k < c->devs.size(); ++k) {
          Device &d = c->devs[k];
          HIP_TRY(hipSetDevice(d.hip_id));
          HIP_TRY(hipEventRecord(d.bucket_red[b], d.comm_stream));
        }
      }
      return CBX_OK;
    };
    auto accumulate = [&](int64_t b) -> int {
      const int64_t start = b * b4;
      const int64_t len = std::min(b4, c->n4 - start);
      for (size_t k = 0; k < c->devs.size(); ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        cbx::LaunchConfig cfg = c->cfg;
        cfg.num_cus = d.num_cus;
        cbx::Timing t;
        if (b == 0) t.start = pipelined ? step_start_event(c, d, 2) : ring_event(c, d, EV_START);
        if (!pipelined) t.stop = ring_event(c, d, EV_A);
        hipStream_t st = cross ? d.a_stream : d.stream;
        if (cross && !join[k] && b % wait_stride == 0) {  // B(b .. b+stride-1) of the last step
          const int64_t w = std::min<int64_t>(b + wait_stride - 1, nb - 1);
          HIP_TRY(hipStreamWaitEvent(st, ocheck ? d.ord[d.ord_cur ^ 1u].b1[w] : d.bucket_b[w], 0));
        }
        if (pipelined) t.stop = ocheck ? d.ord[d.ord_cur].a1[b] : d.bucket_acc[b];
        if (ocheck) {
          Device::OrderStep &o = d.ord[d.ord_cur];
          HIP_TRY(cbx::launch_order_probe(st, {nullptr, o.pa[b]}));
          o.a1[b] = t.stop;  // with timing on, A always carries a stop event (the pool's or the ring's)
        }
        HIP_TRY(cbx::launch_sma_accumulate(offset_args(args[k], start, len), b == 0, cfg, st, t));
      }
      return CBX_OK;
    };
    auto apply = [&](int64_t b) -> int {
      const int64_t start = b * b4;
      const int64_t len = std::min(b4, c->n4 - start);
      for (size_t k = 0; k < c->devs.size(); ++k) {
        Device &d = c->devs[k];
        HIP_TRY(hipSetDevice(d.hip_id));
        if (pipelined) HIP_TRY(hipStreamWaitEvent(d.stream, d.bucket_red[b], 0));
        cbx::LaunchConfig cfg = c->apply_cfg;
        cfg.num_cus = d.num_cus;
        cbx::Timing t;
        if (b == nb - 1) t.stop = step_stop_event(c, d, EV_B);
        cbx::SmaArgs a = offset_args(args[k], start, len);
        if (rsag && mom) a.D = a.last;  // the gathered D' (kernel B then adds it without momentum)
        if (cross) {
          // The next step's AR(0) may overwrite D's control block before this
          // step's later buckets run: B(0) publishes the Phase-D decision to a
          // per-parity slot that B(1..) read.
          a.decision_mode = b == 0 ? 1 : 2;
          a.decision = d.decision + (d.cross_parity & 1u);
        }
        const bool in_dispatch = cross && !t.stop;
        if (in_dispatch) t.stop = ocheck ? d.ord[d.ord_cur].b1[b] : d.bucket_b[b];
        if (ocheck) {
          Device::OrderStep &o = d.ord[d.ord_cur];
          HIP_TRY(cbx::launch_order_probe(d.stream, {nullptr, o.pb[b]}));
          if (!t.stop) t.stop = o.b1[b];
          o.b1[b] = t.stop;
        }
        HIP_TRY(cbx::launch_sma_apply(a, mom && !rsag, cfg, d.stream, t));
        if (cross && !in_dispatch) HIP_TRY(hipEventRecord(d.bucket_b[b], d.stream));
      }
      return CBX_OK;
    };
    if (!pipelined) {
      TRY(accumulate(0));
      TRY(allreduce(0, false, -1));
      for (Device &d : c->devs) {
        HIP_TRY(hipSetDevice(d.hip_id));
        TRY(mark(c, d, EV_AR));
      }
      TRY(apply(0));
    } else {
      // All-reduces go out in groups of `ar_group` buckets behind a single
      // comm-stream wait on the group's last kernel A (cbx_set_allreduce_group).
      // Every event is recorded before the wait on it is enqueued: a group's
      // all-reduces follow its last A, and B(j) follows AR(j).  Mode 0 applies
      // the previous group while this one is on the link; mode 1 applies a
      // group right behind its all-reduces.  ar_group 1 is the per-bucket order
      // A(b) AR(b) B(b-1) (mode 0) / A(b) AR(b) B(b) (mode 1).
      const int64_t ar_group = std::max(1, c->allreduce_group);
      int64_t applied = 0;
      for (int64_t b = 0; b < nb; ++b) {
        TRY(accumulate(b));
        if ((b + 1) % ar_group != 0 && b != nb - 1) continue;
        const int64_t g0 = b - b % ar_group;
        for (int64_t j = g0; j <= b; ++j) TRY(allreduce(j, true, j == g0 ? b : -1));
        const int64_t upto = cross ? b + 1 : g0;
        for (; applied < upto; ++applied) TRY(apply(applied));
      }
      // The wait inside apply(nb-1) also joins every earlier all-reduce
      // (comm_stream is in order) back into the sync stream.
      for (; applied < nb; ++applied) TRY(apply(applied));
    }
    for (Device &d : c->devs) {
      ring_advance(c, d, pipelined ? 2 : 1);
      d.cross_valid = cross;
      if (cross) {
        d.cross_nb = nb;
        d.cross_foreign = foreign;
        d.cross_parity ^= 1u;
      }
    }
    c->last_step_split = true;
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
  TRY(ensure_one_rank_comm(c));
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
  if (split && c->G == 1 && c->devs[0].comm == nullptr) {
    Device &d = c->devs[0];
    HIP_TRY(hipSetDevice(d.hip_id));
    int dev = d.hip_id;
    NCCL_TRY(ncclCommInitAll(&d.comm, 1, &dev));
  }
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
// Checkpoint helpers, databuffer.c:215-259, model.c:396-416
// ---------------------------------------------------------------------------
int write_file(const std::string &path, const void *data, size_t bytes) {
  int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return fail(CBX_ERR_IO, "failed to open %s: %s", path.c_str(), strerror(errno));
  size_t done = 0;
  while (done < bytes) {
    ssize_t w = write(fd, (const char *)data + done, bytes - done);
    if (w <= 0) {
      close(fd);
      return fail(CBX_ERR_IO, "%zu/%zu bytes written to %s", done, bytes, path.c_str());
    }
    done += (size_t)w;
  }
  close(fd);
  return CBX_OK;
}

int read_file(const std::string &path, void *data, size_t bytes) {
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return fail(CBX_ERR_IO, "failed to open %s: %s", path.c_str(), strerror(errno));
  size_t done = 0;
  while (done < bytes) {
    ssize_t r = read(fd, (char *)data + done, bytes - done);
    if (r <= 0) {
      close(fd);
      return fail(CBX_ERR_IO, "%zu/%zu bytes read from %s", done, bytes, path.c_str());
    }
    done += (size_t)r;
  }
  close(fd);
  return CBX_OK;
}

std::string fmt(const char *f, ...) {
  char buf[4096];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

int store_buffer(const float *dev, size_t bytes, const std::string &path, std::vector<char> &tmp) {
  tmp.resize(bytes);
  HIP_TRY(hipMemcpy(tmp.data(), dev, bytes, hipMemcpyDeviceToHost));
  return write_file(path, tmp.data(), bytes);
}

int load_buffer(float *dev, size_t bytes, const std::string &path, std::vector<char> &tmp) {
  tmp.resize(bytes);
  TRY(read_file(path, tmp.data(), bytes));
  HIP_TRY(hipMemcpy(dev, tmp.data(), bytes, hipMemcpyHostToDevice));
  return CBX_OK;
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

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int cbx_abi_version(void) { return CBX_ABI_VERSION; }

const char *cbx_last_error(void) { return g_last_error.c_str(); }

int cbx_device_count(int *count) {
  if (!count) return fail(CBX_ERR_INVALID, "null count");
  return gfx950_device_count(count);
}

int cbx_init(cbx_context **out, const int *devices, int ndevices) {
  if (!out || !devices || ndevices <= 0) return fail(CBX_ERR_INVALID, "cbx_init: need at least one device");
  *out = nullptr;
  cbx_context *c = new cbx_context();
  c->G = ndevices;
  c->devs.resize(ndevices);
  for (int k = 0; k < ndevices; ++k) {
    int rc = open_device(c->devs[k], devices[k], k);
    if (rc < 0) {
      std::string msg = g_last_error;
      cbx_free(c);
      return fail(rc, "%s", msg.c_str());
    }
  }
  // Checkpoint files carry the selected device id, as the reference's do.  A
  // selection that repeats a device (only the loopback test harness can run
  // one; RCCL refuses it) keeps the position, so the names stay distinct.
  bool repeated = false;
  for (int a = 0; a < ndevices; ++a)
    for (int b = 0; b < a; ++b) repeated = repeated || devices[a] == devices[b];
  if (!repeated)
    for (Device &d : c->devs) d.file_id = d.hip_id;
  if (ndevices > 1) {
    // executioncontext.c:185-201: ncclCommInitAll over the selected devices;
    // communicators are indexed by rank (selected-device order).
    std::vector<ncclComm_t> comms(ndevices);
    std::vector<int> ids(devices, devices + ndevices);
    ncclResult_t r = ncclCommInitAll(comms.data(), ndevices, ids.data());
    if (r != ncclSuccess) {
      cbx_free(c);
      return fail(CBX_ERR_RCCL, "ncclCommInitAll: %s", ncclGetErrorString(r));
    }
    for (int k = 0; k < ndevices; ++k) c->devs[k].comm = comms[k];
  }
  *out = c;
  return CBX_OK;
}

int cbx_get_unique_id(unsigned char unique_id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(unique_id, &id, sizeof(id));
  return CBX_OK;
}

int cbx_init_rank(cbx_context **out, int device, int nranks, int rank, const unsigned char unique_id[128]) {
  if (!out || nranks <= 0 || rank < 0 || rank >= nranks) return fail(CBX_ERR_INVALID, "cbx_init_rank: bad rank");
  *out = nullptr;
  cbx_context *c = new cbx_context();
  c->G = nranks;
  c->per_rank = true;
  c->devs.resize(1);
  int rc = open_device(c->devs[0], device, rank);
  if (rc < 0) {
    std::string msg = g_last_error;
    cbx_free(c);
    return fail(rc, "%s", msg.c_str());
  }
  if (nranks > 1) {
    if (!unique_id) {
      cbx_free(c);
      return fail(CBX_ERR_INVALID, "cbx_init_rank: unique id required for %d ranks", nranks);
    }
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&c->devs[0].comm, nranks, id, rank);
    if (r != ncclSuccess) {
      cbx_free(c);
      return fail(CBX_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
  }
  *out = c;
  return CBX_OK;
}

int cbx_free(cbx_context *c) {
  if (!c) return CBX_OK;
  for (Replica *r : c->replicas) {
    if (r && r->client && r->local >= 0) {
      (void)hipSetDevice(c->devs[r->local].hip_id);
      (void)hipEventDestroy(r->client);
      r->client = nullptr;
    }
  }
  for (Device &d : c->devs) close_device(d);
  for (std::vector<Replica *> *list : {&c->replicas, &c->retired})
    for (Replica *r : *list) {
      if (!r) continue;
      if (r->client) (void)hipEventDestroy(r->client);
      pthread_mutex_destroy(&r->lock);
      delete r;
    }
  delete c;
  return CBX_OK;
}

// ---- model registration ---------------------------------------------------
int cbx_set_model(cbx_context *c, int variables, int bytes) {
  TRY(check_ctx(c));
  if (c->manager) return fail(CBX_ERR_STATE, "model already finalised");
  if (variables <= 0 || bytes <= 0) return fail(CBX_ERR_INVALID, "setModel(%d, %d)", variables, bytes);
  c->model = ModelDef();
  c->model.defined = true;
  c->model.ops = variables;
  c->model.bytes = bytes;
  c->model.count_per_op.assign(variables, 0);
  c->model.host.assign(((size_t)bytes + 3) / 4, 0.0f);
  return CBX_OK;
}

int cbx_set_model_variable(cbx_context *c, int id, int order, int ndims, const int *shape, int capacity) {
  TRY(check_ctx(c));
  ModelDef &m = c->model;
  if (!m.defined) return fail(CBX_ERR_STATE, "setModelVariable before setModel");
  if (c->manager) return fail(CBX_ERR_STATE, "model already finalised");
  if (id < 0 || id >= m.ops) return fail(CBX_ERR_INVALID, "variable op %d out of range [0, %d)", id, m.ops);
  if (ndims < 0 || (ndims > 0 && !shape) || capacity < 0) return fail(CBX_ERR_INVALID, "bad variable shape");
  // model.c:127-157: the next variable of op `id` must have order count+1.
  if (order != m.count_per_op[id] + 1)
    return fail(CBX_ERR_INVALID, "invalid model variable order (ndx=%d, ord=%d)", id, m.count_per_op[id] + 1);
  int64_t elements = 1;
  for (int k = 0; k < ndims; ++k) {
    if (shape[k] < 0) return fail(CBX_ERR_INVALID, "negative dimension %d of variable (%d, %d)", shape[k], id, order);
    elements *= shape[k];
  }
  if (elements * 4 > capacity)
    return fail(CBX_ERR_INVALID, "variable (%d, %d) of %lld floats exceeds its capacity of %d bytes", id, order,
                (long long)elements, capacity);
  if (m.offset + capacity > m.bytes)
    return fail(CBX_ERR_INVALID, "variable overflows the model (%lld + %d > %lld)", (long long)m.offset, capacity,
                (long long)m.bytes);
  m.vars[{id, order}] = Variable{m.offset, capacity, elements};
  m.count_per_op[id]++;
  m.offset += capacity;
  m.elements += elements;
  return CBX_OK;
}

int cbx_set_model_variable_buffer(cbx_context *c, int id, int order, const void *src) {
  TRY(check_ctx(c));
  auto it = c->model.vars.find({id, order});
  if (it == c->model.vars.end()) return fail(CBX_ERR_INVALID, "model variable not found (id %d, order %d)", id, order);
  if (!src) return fail(CBX_ERR_INVALID, "null variable buffer");
  // executioncontext.c:1583-1590 -> databuffer.c:80-84: copy into the pinned
  // host image of theModel; it reaches the device at setModelManager.
  std::memcpy(reinterpret_cast<char *>(c->model.host.data()) + it->second.offset_bytes, src,
              (size_t)it->second.bytes);
  return CBX_OK;
}

int cbx_set_model_variable_learning_rate_multiplier(cbx_context *c, int id, int order, float multiplier) {
  TRY(check_ctx(c));
  auto it = c->model.vars.find({id, order});
  if (it == c->model.vars.end()) return fail(CBX_ERR_INVALID, "model variable not found (id %d, order %d)", id, order);
  it->second.lr_multiplier = multiplier;
  if (multiplier != 1.0f) c->model.conf.irregular++;  // executioncontext.c:1602-1603
  return CBX_OK;
}

int cbx_set_model_work_per_clock(cbx_context *c, int wpc) {
  TRY(check_ctx(c));
  c->model.wpc = wpc;
  return CBX_OK;
}

int cbx_set_update_model_type(cbx_context *c, int type) {
  TRY(check_ctx(c));
  if (type < 0 || type > 7) return fail(CBX_ERR_INVALID, "Invalid update model type");  // executioncontext.c:1623
  c->model.type = type;
  return CBX_OK;
}

// ---- solver ---------------------------------------------------------------
int cbx_set_learning_rate_decay_policy_fixed(cbx_context *c, float rate) {
  TRY(check_ctx(c));
  c->model.conf.policy = LR_FIXED;
  c->model.conf.learningRate = rate;
  return CBX_OK;
}

int cbx_set_learning_rate_decay_policy_inv(cbx_context *c, float rate, double gamma, double power) {
  TRY(check_ctx(c));
  c->model.conf.policy = LR_INV;
  c->model.conf.learningRate = rate;
  c->model.conf.gamma = gamma;
  c->model.conf.power = power;
  return CBX_OK;
}

int cbx_set_learning_rate_decay_policy_step(cbx_context *c, float rate, double gamma, int size) {
  TRY(check_ctx(c));
  c->model.conf.policy = LR_STEP;
  c->model.conf.learningRate = rate;
  c->model.conf.gamma = gamma;
  c->model.conf.size = size;
  return CBX_OK;
}

int cbx_set_learning_rate_decay_policy_multistep(cbx_context *c, float rate, double gamma, int warmuptasks,
                                                  int nsteps, const int *steps) {
  TRY(check_ctx(c));
  if (nsteps < 0 || (nsteps > 0 && !steps)) return fail(CBX_ERR_INVALID, "bad multistep schedule");
  SolverConf &s = c->model.conf;
  s.policy = warmuptasks > 0 ? LR_LSR : LR_MULTISTEP;  // executioncontext.c:1690
  s.learningRate = rate;
  s.gamma = gamma;
  s.warmuptasks = warmuptasks;
  s.steps.assign(steps, steps + nsteps);
  return CBX_OK;
}

int cbx_set_learning_rate_decay_policy_exp(cbx_context *c, float rate, double gamma) {
  TRY(check_ctx(c));
  c->model.conf.policy = LR_EXP;
  c->model.conf.learningRate = rate;
  c->model.conf.gamma = gamma;
  return CBX_OK;
}

int cbx_set_learning_rate_decay_policy_circular(cbx_context *c, const float *rate, int superconvergence,
                                                 const float *momentum, int step) {
  TRY(check_ctx(c));
  if (!rate || !momentum) return fail(CBX_ERR_INVALID, "circular policy needs 3 rates and 3 momenta");
  SolverConf &s = c->model.conf;
  s.policy = LR_CLR;  // executioncontext.c:1701-1718
  s.superConvergence = superconvergence;
  for (int i = 0; i < 3; ++i) {
    s.circularLearningRate[i] = rate[i];
    s.circularMomentum[i] = momentum[i];
  }
  s.size = step;
  return CBX_OK;
}

int cbx_set_base_model_momentum(cbx_context *c, float m) {
  TRY(check_ctx(c));
  c->model.conf.baseModelMomentum = m;  // stored, never used natively (sma.c:152)
  return CBX_OK;
}

int cbx_set_momentum(cbx_context *c, float m, int method) {
  TRY(check_ctx(c));
  if (method != 0 && method != 1) return fail(CBX_ERR_INVALID, "Invalid momentum type");
  c->model.conf.momentum = m;
  c->model.conf.momentumMethod = method;
  return CBX_OK;
}

int cbx_set_weight_decay(cbx_context *c, float decay) {
  TRY(check_ctx(c));
  c->model.conf.weightDecay = decay;
  return CBX_OK;
}

int cbx_set_eamsgd_alpha(cbx_context *c, float alpha) {
  TRY(check_ctx(c));
  c->model.conf.alpha = alpha;
  return CBX_OK;
}

int cbx_set_eamsgd_tau(cbx_context *c, int tau) {
  TRY(check_ctx(c));
  c->model.conf.tau = tau;
  return CBX_OK;
}

// ---- model manager --------------------------------------------------------
int cbx_set_model_manager(cbx_context *c, int replicas, int type) {
  TRY(check_ctx(c));
  if (c->manager) return fail(CBX_ERR_STATE, "model manager already created");
  if (!c->model.defined) return fail(CBX_ERR_STATE, "setModelManager before setModel");
  if (type != CBX_SYNC_BSP && type != CBX_SYNC_SSP && type != CBX_SYNC_ASP)
    return fail(CBX_ERR_INVALID, "illegal synchronisation type %d", type);
  if (replicas <= 0) return fail(CBX_ERR_INVALID, "need at least one replica per device");
  if (replicas > cbx::kMaxReplicas) return fail(CBX_ERR_UNSUPPORTED, "at most %d replicas per device", cbx::kMaxReplicas);
  ModelDef &m = c->model;
  if (m.elements <= 0) {
    // A model registered as raw bytes (no variables): every 4 bytes are a float.
    m.elements = m.bytes / 4;
  }
  if ((int64_t)m.elements * 4 > m.bytes) return fail(CBX_ERR_INVALID, "model elements exceed model bytes");

  c->n = m.elements;
  const int64_t pad = cbx::kPadFloat4;
  c->n4 = ((c->n + 3) / 4 + pad - 1) / pad * pad;
  if (c->n4 * 16 + 4096 >= (int64_t)1 << 32)
    return fail(CBX_ERR_UNSUPPORTED, "model of %lld elements exceeds the 4 GiB per-buffer kernel offset range",
                (long long)c->n);
  // model.c:116-120: `last` exists iff momentum > 0 (theModel's conf).
  c->has_last = m.conf.momentum > 0;
  c->R = replicas;
  c->size = replicas * c->G;
  c->sync_type = type;

  // Replicas round-robin over devices: replica j*G + g on device g.
  c->replicas.assign(c->size, nullptr);
  c->locked.assign(c->size, 0);
  // Capacity for every replica addModel can create, so that the task side's
  // lookups never see these arrays move (add / del only resize them).
  c->replicas.reserve((size_t)cbx::kMaxReplicas * c->G);
  c->locked.reserve((size_t)cbx::kMaxReplicas * c->G);
  c->theta.reset(new ThetaSlot[(size_t)cbx::kMaxReplicas * c->G]);
  for (int i = 0; i < c->size; ++i) {
    Replica *r = new Replica();
    r->id = i;
    r->g = i % c->G;
    r->local = local_of(c, r->g);
    r->slot = i / c->G;
    r->conf = m.conf;  // crossbowSolverConfReplicate (model.c:265)
    pthread_mutex_init(&r->lock, nullptr);
    c->replicas[i] = r;
  }

  const size_t data_bytes = (size_t)c->n4 * 16 + (size_t)cbx::kCtrlFloats * sizeof(float);
  const size_t stride = (data_bytes + kAlign - 1) / kAlign * kAlign + kSlotStagger;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    d.stride = stride;
    d.base_slots = replicas;
    d.arena_bytes = stride * (size_t)(kBaseSlots + kReplicaSlots * replicas);
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&d.arena), d.arena_bytes);
    if (e != hipSuccess)
      return fail(CBX_ERR_HIP, "hipMalloc(%zu) for the model arena: %s", d.arena_bytes, hipGetErrorString(e));
    HIP_TRY(hipMemsetAsync(d.arena, 0, d.arena_bytes, d.stream));
    d.replicas.clear();
    for (int i = 0; i < c->size; ++i)
      if (c->replicas[i]->g == d.g) d.replicas.push_back(i);
    // executioncontext.c:1741: push theModel's initial values, then every
    // base model and replica starts as a copy of it (modelmanager.c:28-64).
    float *z = base_dev(c, d, CBX_BUF_DATA);
    HIP_TRY(hipMemcpyAsync(z, m.host.data(), (size_t)c->n * 4, hipMemcpyHostToDevice, d.stream));
    for (int id : d.replicas) {
      Replica &r = *c->replicas[id];
      HIP_TRY(hipMemcpyAsync(replica_dev(d, r, CBX_BUF_DATA), z, (size_t)c->n * 4, hipMemcpyDeviceToDevice, d.stream));
    }
    HIP_TRY(hipEventRecord(d.synched, d.stream));
    d.step_event = d.synched;
    HIP_TRY(hipStreamSynchronize(d.stream));
  }
  c->manager = true;
  return CBX_OK;
}

// ---- barrier path ---------------------------------------------------------
int cbx_lock_any(cbx_context *c) {
  TRY(check_manager_q(c));
  // modelmanager.c:212-231: trylock every replica this process owns.
  int count = 0, local = 0;
  for (int i = 0; i < c->size; ++i) {
    c->locked[i] = 0;
    Replica *r = c->replicas[i];
    if (r->local < 0) continue;
    ++local;
    if (c->theta[i].state.load(std::memory_order_acquire) == kThetaSkip) {
      // modelmanager.c:217-222: counted, so BSP holds, but not locked and
      // therefore left out of the step, unlockAny and the clock.
      ++count;
      continue;
    }
    if (pthread_mutex_trylock(&r->lock) == 0) {
      c->locked[i] = 1;
      ++count;
    }
  }
  if (c->sync_type == CBX_SYNC_BSP) {
    // executioncontext.c:2199-2205
    if (count != local) {
      for (int i = 0; i < c->size; ++i)
        if (c->locked[i]) {
          pthread_mutex_unlock(&c->replicas[i]->lock);
          c->locked[i] = 0;
        }
      return fail(CBX_ERR_BARRIER, "failed to lock all GPU model replicas at synchronisation barrier");
    }
    return c->size;
  }
  return count;
}

int cbx_merge(cbx_context *c, int pull, int *first_out) {
  (void)pull;
  TRY(check_manager_q(c));
  if (!first_out) return fail(CBX_ERR_INVALID, "null merge result");
  // executioncontext.c:2219-2245
  int N = 0;
  for (int i = 0; i < c->size; ++i)
    if (c->locked[i]) N += c->replicas[i]->updates;
  *first_out = -1;
  if (N == 0) return CBX_OK;
  if (c->size == 1) {
    *first_out = 0;
    return CBX_OK;
  }
  int first = 0;
  for (; first < c->size; ++first)
    if (c->locked[first]) break;
  *first_out = first;
  return CBX_OK;
}

static int default_step(cbx_context *c, int first);

// staged: 0 = device-resident step; > 0 = host-staged step over that many
// buckets (cbx_synchronise_staged).
static int synchronise_impl(cbx_context *c, int first, int clock, int autotune, int staged) {
  TraceRange trace(staged ? "cbx_synchronise_staged" : "cbx_synchronise");
  TRY(check_manager_q(c));
  if (first < 0 || first > c->size) return fail(CBX_ERR_INVALID, "first replica %d out of range", first);
  // executioncontext.c:2287-2315: SYNCHRONOUSEAMSGD (3) routes to SMA because
  // ELASTIC_AVERAGE is #undef'd; SMA is 7.  The other update models are not
  // this library's path.
  // WORKER (1) is synchronous SGD (executioncontext.c:2277-2279), which shares
  // the base-model buffers and the all-reduce.
  const int type = c->model.type;
  if (staged || (type != CBX_UPDATE_SMA && type != CBX_UPDATE_SYNCHRONOUSEAMSGD)) {
    c->foreign_ops.fetch_add(1, std::memory_order_relaxed);
    for (Device &d : c->devs) d.cross_valid = false;
  }
  if (type == CBX_UPDATE_WORKER || type == CBX_UPDATE_DEFAULT) {
    if (staged) TRY(cbx_stage_in(c));
    TRY(type == CBX_UPDATE_WORKER ? ssgd_step(c, first) : default_step(c, first));
    if (staged) TRY(cbx_stage_out(c));
  } else if (type == CBX_UPDATE_SMA || type == CBX_UPDATE_SYNCHRONOUSEAMSGD) {
    TRY(staged ? sma_step_staged(c, first, staged) : sma_step(c, first));
  } else {
    return fail(CBX_ERR_UNSUPPORTED, "update model %d is not on this library's path (SMA, SYNCHRONOUSEAMSGD, WORKER, DEFAULT)", type);
  }
  if (autotune < 0) TRY(cbx_del_model(c));
  if (autotune > 0) TRY(cbx_add_model(c));
  // modelmanager.c:259-265: clock of every locked replica.
  for (int i = 0; i < c->size; ++i)
    if (c->locked[i]) {
      __atomic_store_n(&c->replicas[i]->clock, clock, __ATOMIC_RELEASE);  // read by cbx_get_next_or_wait
      c->replicas[i]->updates = 0;
    }
  return CBX_OK;
}

int cbx_synchronise(cbx_context *c, int first, int clock, int autotune, int push) {
  // push is unused by the reference too (executioncontext.c:2264).
  (void)push;
  return synchronise_impl(c, first, clock, autotune, 0);
}

int cbx_synchronise_staged(cbx_context *c, int first, int clock, int autotune, int buckets) {
  if (buckets < 1 || buckets > 4096) return fail(CBX_ERR_INVALID, "staged buckets must be 1..4096, got %d", buckets);
  return synchronise_impl(c, first, clock, autotune, buckets);
}

int cbx_unlock_any(cbx_context *c) {
  TRY(check_manager_q(c));
  int count = 0;
  for (int i = 0; i < c->size; ++i)
    if (c->locked[i]) {
      pthread_mutex_unlock(&c->replicas[i]->lock);
      c->locked[i] = 0;
      ++count;
    }
  return count;
}

// ---- checkpoint -----------------------------------------------------------
static int batchnorm_checkpoint(cbx_context *c, const std::string &dir, bool store);

int cbx_checkpoint_model(cbx_context *c, const char *dir) {
  TraceRange trace("cbx_checkpoint_model");
  TRY(check_manager(c));
  if (!dir) return fail(CBX_ERR_INVALID, "null checkpoint directory");
  // executioncontext.c:2340-2350: dir/%06llu, a new version per call.
  std::string path = fmt("%s/%06llu", dir, ++c->version);
  if (mkdir(path.c_str(), 0777) < 0 && !(c->per_rank && errno == EEXIST))
    return fail(CBX_ERR_IO, "Failed to create directory %s", path.c_str());
  TRY(cbx_wait(c));
  std::vector<char> tmp;
  const size_t bytes = (size_t)c->n * 4;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    // modelmanager.c:306-343, model.c:396-405
    std::string prefix = fmt("%s/gpu-%02d-theModel", path.c_str(), d.file_id);
    TRY(store_buffer(base_dev(c, d, CBX_BUF_DATA), bytes, prefix + "-data.dat", tmp));
    if (c->has_last) TRY(store_buffer(base_dev(c, d, CBX_BUF_LAST), bytes, prefix + "-last.dat", tmp));
    for (int id : d.replicas) {
      Replica &r = *c->replicas[id];
      std::string rp = fmt("%s/gpu-%02d-replica-%03d", path.c_str(), d.file_id, id);
      TRY(store_buffer(replica_dev(d, r, CBX_BUF_DATA), bytes, rp + "-data.dat", tmp));
      if (c->has_last) TRY(store_buffer(replica_dev(d, r, CBX_BUF_LAST), bytes, rp + "-last.dat", tmp));
    }
  }
  return batchnorm_checkpoint(c, path, true);  // :2352-2364
}

int cbx_override_model_data(cbx_context *c, const char *dir) {
  TraceRange trace("cbx_override_model_data");
  TRY(check_manager(c));
  if (!dir) return CBX_OK;  // GPU.c:1169: a null directory is a no-op
  TRY(cbx_wait(c));
  std::vector<char> tmp;
  const size_t bytes = (size_t)c->n * 4;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    // modelmanager.c:267-304
    std::string prefix = fmt("%s/gpu-%02d-theModel", dir, d.file_id);
    TRY(load_buffer(base_dev(c, d, CBX_BUF_DATA), bytes, prefix + "-data.dat", tmp));
    if (c->has_last) TRY(load_buffer(base_dev(c, d, CBX_BUF_LAST), bytes, prefix + "-last.dat", tmp));
    for (int id : d.replicas) {
      Replica &r = *c->replicas[id];
      std::string rp = fmt("%s/gpu-%02d-replica-%03d", dir, d.file_id, id);
      TRY(load_buffer(replica_dev(d, r, CBX_BUF_DATA), bytes, rp + "-data.dat", tmp));
      if (c->has_last) TRY(load_buffer(replica_dev(d, r, CBX_BUF_LAST), bytes, rp + "-last.dat", tmp));
    }
  }
  return batchnorm_checkpoint(c, dir, false);  // :2375-2386
}

// cudnnbatchnormparams.c:102-143: one BN operator's running mean / variance,
// one pair of files per device that holds it.  `store` selects the direction.
static int batchnorm_stats_files(cbx_context *c, const std::string &dir, int op, int elements,
                                 float *const *mean, float *const *variance, bool store) {
  if (op < 0 || elements <= 0 || !mean || !variance)
    return fail(CBX_ERR_INVALID, "bad batch-norm checkpoint arguments (op %d, %d elements)", op, elements);
  std::vector<char> tmp;
  const size_t bytes = (size_t)elements * 4;
  for (size_t k = 0; k < c->devs.size(); ++k) {
    Device &d = c->devs[k];
    if (!mean[k] && !variance[k]) continue;  // :110-111
    if (!mean[k] || !variance[k])
      return fail(CBX_ERR_INVALID, "device %d holds only one of operator %d's mean / variance", d.g, op);
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipDeviceSynchronize());
    const std::string avg = fmt("%s/gpu-%02d-bn-avg-%03d.dat", dir.c_str(), d.file_id, op);
    const std::string var = fmt("%s/gpu-%02d-bn-var-%03d.dat", dir.c_str(), d.file_id, op);
    if (store) {
      TRY(store_buffer(mean[k], bytes, avg, tmp));
      TRY(store_buffer(variance[k], bytes, var, tmp));
    } else {
      TRY(load_buffer(mean[k], bytes, avg, tmp));
      TRY(load_buffer(variance[k], bytes, var, tmp));
    }
  }
  return CBX_OK;
}

static int batchnorm_checkpoint(cbx_context *c, const std::string &dir, bool store) {
  for (auto &e : c->bn_stats)
    TRY(batchnorm_stats_files(c, dir, e.first, e.second.elements, e.second.mean.data(), e.second.variance.data(),
                              store));
  return CBX_OK;
}

// crossbowCudnnBatchNormParamsSetEstimatedMeanAndVariable (executioncontext.c:
// 1280-1290) hands each device's buffers to the operator's BN params; here the
// dataflow side hands them to the context, once per BN operator.
int cbx_register_batchnorm_stats(cbx_context *c, int op, int elements, float *const *mean, float *const *variance) {
  TRY(check_ctx(c));
  if (op < 0) return fail(CBX_ERR_INVALID, "bad batch-norm operator id %d", op);
  if (elements == 0) {
    c->bn_stats.erase(op);
    return CBX_OK;
  }
  if (elements < 0 || !mean || !variance)
    return fail(CBX_ERR_INVALID, "bad batch-norm statistics (op %d, %d elements)", op, elements);
  cbx_context::BnStats b;
  b.elements = elements;
  for (size_t k = 0; k < c->devs.size(); ++k) {
    if (!mean[k] != !variance[k])
      return fail(CBX_ERR_INVALID, "device %d holds only one of operator %d's mean / variance", c->devs[k].g, op);
    b.mean.push_back(mean[k]);
    b.variance.push_back(variance[k]);
  }
  c->bn_stats[op] = std::move(b);
  return CBX_OK;
}

// crossbowModelManagerAddModel, modelmanager.c:362-470: one new replica per
// device, ids size .. size+G-1 (id size+g on device g, keeping the round-robin
// placement), each a copy of the first replica on its device (data, gradient,
// last, diff and solver state: model.c:202-306), locked so that the barrier's
// unlockAny releases it.
int cbx_add_model(cbx_context *c) {
  TRY(check_manager(c));
  if (c->R + 1 > cbx::kMaxReplicas) return fail(CBX_ERR_UNSUPPORTED, "at most %d replicas per device", cbx::kMaxReplicas);
  const int size_ = c->size + c->G;
  const int slot = c->R;  // id / G of every new replica
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipStreamSynchronize(d.stream));  // :417 cudaDeviceSynchronize
    if (slot >= d.base_slots) {
      const size_t k = (size_t)(slot - d.base_slots);
      if (d.extra.size() <= k) d.extra.resize(k + 1, nullptr);
      if (!d.extra[k]) {
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&d.extra[k]), d.stride * kReplicaSlots);
        if (e != hipSuccess) {
          d.extra[k] = nullptr;
          return fail(CBX_ERR_HIP, "hipMalloc for a new replica: %s", hipGetErrorString(e));
        }
      }
      if (d.host) TRY(alloc_host_mirror(c));
    }
  }
  c->replicas.resize(size_, nullptr);
  c->locked.resize(size_, 0);
  for (int g = 0; g < c->G; ++g) {
    const int id = c->size + g;
    Replica *r = new Replica();
    r->id = id;
    r->g = g;
    r->local = local_of(c, g);
    r->slot = slot;
    // :420-425: the first replica on the device is the template.
    const Replica &src = *c->replicas[g];
    r->conf = src.conf;  // crossbowSolverConfReplicate
    r->clock = src.clock;
    r->updates = src.updates;
    pthread_mutex_init(&r->lock, nullptr);
    c->replicas[id] = r;
    c->theta[id].state.store(kThetaFree, std::memory_order_release);  // crossbowThetaQueueExpand (:442)
    if (r->local >= 0) {
      Device &d = c->devs[r->local];
      HIP_TRY(hipSetDevice(d.hip_id));
      for (int kind : {CBX_BUF_DATA, CBX_BUF_GRADIENT, CBX_BUF_DIFF, CBX_BUF_LAST})
        HIP_TRY(hipMemcpyAsync(replica_dev(d, *r, kind), replica_dev(d, src, kind), d.stride, hipMemcpyDeviceToDevice,
                               d.stream));
      HIP_TRY(hipStreamSynchronize(d.stream));
      pthread_mutex_lock(&r->lock);  // :433-435
      c->locked[id] = 1;
    }
  }
  for (Device &d : c->devs) d.replicas.push_back(c->size + d.g);
  c->size = size_;
  c->R += 1;
  return CBX_OK;
}

// crossbowModelManagerDelModel, modelmanager.c:473-557: drop the last replica
// of every device (ids size-G .. size-1).
int cbx_del_model(cbx_context *c) {
  TRY(check_manager(c));
  if (c->R <= 1) return fail(CBX_ERR_STATE, "cannot delete the last replica of a device");  // :511
  const int size_ = c->size - c->G;
  // crossbowThetaQueueShrink (:537): the slots leave the rotation first, so
  // no task reserves a removed id from now on; a task still holding its
  // reservation gets 0 from cbx_upgrade_access.
  for (int id = size_; id < c->size; ++id) c->theta[id].state.store(kThetaSkip, std::memory_order_release);
  // A task may hold a removed replica (ASP / SSP barriers do not lock busy
  // ones): wait until it releases it (cbx_replica_release still takes the
  // id) before its buffers go.  Then shrink the count, so no lookup sees the
  // removed ids any more.
  for (int id = size_; id < c->size; ++id)
    if (!c->locked[id]) pthread_mutex_lock(&c->replicas[id]->lock);
  const int old_size = c->size;
  c->size = size_;
  for (int id = size_; id < old_size; ++id) {
    Replica *r = c->replicas[id];
    if (r->local >= 0) {
      Device &d = c->devs[r->local];
      HIP_TRY(hipSetDevice(d.hip_id));
      HIP_TRY(hipDeviceSynchronize());  // :530, every stream (task streams included)
      if (r->slot >= d.base_slots) {
        const size_t k = (size_t)(r->slot - d.base_slots);
        HIP_TRY(hipFree(d.extra[k]));
        d.extra[k] = nullptr;
        if (k < d.extra_host.size() && d.extra_host[k]) {
          HIP_TRY(hipHostFree(d.extra_host[k]));
          d.extra_host[k] = nullptr;
        }
      }
      if (r->client) (void)hipEventDestroy(r->client);
      r->client = nullptr;
      d.replicas.erase(std::remove(d.replicas.begin(), d.replicas.end(), id), d.replicas.end());
    }
    pthread_mutex_unlock(&r->lock);
    c->retired.push_back(r);  // freed by cbx_free: a task may still hold a reference
  }
  // The arrays keep their capacity (reserved at creation), so they never
  // move under a reader.
  c->replicas.resize(size_);
  c->locked.resize(size_);
  c->R -= 1;
  return CBX_OK;
}

// ---- replica optimiser step (kernels/optimisers/sma.cu:3-100) -------------
// crossbowKernelOptimiserDefault, kernels/optimisers/default.cu:3-131: the
// replica and its device's base model take the same step.  The reference
// updates the replica on the task stream and the base model on the sync
// stream after the gradient is ready (:84-99, :115-127); base-model updates
// of concurrent tasks are ordered by that one stream.  Here the whole step is
// one pass on the sync stream (it waits for the task stream first), and the
// task stream then waits for it before using the replica again.
static int default_task_step(cbx_context *c, Replica &r, Device &d, int task, hipStream_t st) {
  SolverConf &conf = r.conf;
  if (conf.momentum > 0 && conf.momentumMethod == 1)
    return fail(CBX_ERR_UNSUPPORTED, "Nesterov's momentum has been disabled");  // default.cu:42-44
  if (conf.momentum > 0 && !c->has_last)
    return fail(CBX_ERR_STATE, "replica momentum without a `last` buffer (model.c:116-120)");
  float lr = 0.0f;
  TRY(conf.learning_rate(task, &lr));
  cbx::OptArgs a;
  std::memset(&a, 0, sizeof(a));
  a.w = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_DATA));
  a.g = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_GRADIENT));
  a.last = conf.momentum > 0 ? reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_LAST)) : nullptr;
  a.z = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_DATA));
  a.n4 = c->n4;
  a.rate = -lr;  // default.cu:38
  a.momentum = conf.momentum;
  a.wd = conf.weightDecay;
  HIP_TRY(hipSetDevice(d.hip_id));
  if (!r.client) HIP_TRY(hipEventCreateWithFlags(&r.client, hipEventDisableTiming));
  if (st != d.stream) {
    HIP_TRY(hipEventRecord(r.client, st));  // the gradient is ready (default.cu:64,101)
    HIP_TRY(hipStreamWaitEvent(d.stream, r.client, 0));
  }
  cbx::LaunchConfig cfg = c->aux_cfg;
  cfg.num_cus = d.num_cus;
  cfg.blocks_per_cu = 0;
  HIP_TRY(cbx::launch_default_optimise(a, cfg, d.stream, {}));
  if (st != d.stream) {
    HIP_TRY(hipEventRecord(r.client, d.stream));  // replica->server (:98,:127)
    HIP_TRY(hipStreamWaitEvent(st, r.client, 0));
  }
  return CBX_OK;
}

// DEFAULT barrier, synch/default.c:5-43: copy the base model to every locked
// replica i >= first.  Multi-GPU DEFAULT is err() in the reference (:46-51).
static int default_step(cbx_context *c, int first) {
  if (c->G > 1) return fail(CBX_ERR_UNSUPPORTED, "Multi-GPU default SGD model synchronisation is not supported yet");
  Device &d = c->devs[0];
  cbx::SmaArgs a;
  std::memset(&a, 0, sizeof(a));
  int k = 0;
  for (int id : d.replicas) {
    if (id < first || !c->locked[id]) continue;
    if (k >= cbx::kMaxReplicas) return fail(CBX_ERR_UNSUPPORTED, "too many replicas on one device");
    a.w[k++] = reinterpret_cast<cbx::v4f *>(replica_dev(d, *c->replicas[id], CBX_BUF_DATA));
  }
  a.nrep = k;
  a.z = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_DATA));
  a.n4 = c->n4;
  HIP_TRY(hipSetDevice(d.hip_id));
  cbx::LaunchConfig cfg = c->broadcast_cfg;
  cfg.num_cus = d.num_cus;
  cfg.blocks_per_cu = 0;
  HIP_TRY(cbx::launch_broadcast(a, cfg, d.stream, {step_start_event(c, d, 0), step_stop_event(c, d, EV_A)}));
  ring_advance(c, d, 0);
  c->last_step_split = false;
  return finish_step(c);
}

// crossbowKernelOptimiserSynchronousSGD, kernels/optimisers/synchronoussgd.cu:3-56:
// weight decay on the replica gradient, then the lr-scaled gradient is added
// into the device's base-model gradient on the sync stream (:38-52).
static int ssgd_worker_step(cbx_context *c, Replica &r, Device &d, int task, hipStream_t st) {
  SolverConf &conf = r.conf;
  if (conf.momentumMethod == 1) return fail(CBX_ERR_UNSUPPORTED, "Nesterov's momentum has been disabled");  // :42-44
  float lr = 0.0f;
  TRY(conf.learning_rate(task, &lr));
  cbx::SsgdArgs a;
  std::memset(&a, 0, sizeof(a));
  a.wsrc = reinterpret_cast<const cbx::v4f *>(replica_dev(d, r, CBX_BUF_DATA));
  a.g = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_GRADIENT));
  a.acc = reinterpret_cast<cbx::v4f *>(base_dev(c, d, CBX_BUF_GRADIENT));
  a.n4 = c->n4;
  a.rate = -lr;  // :46
  a.wd = conf.weightDecay;
  HIP_TRY(hipSetDevice(d.hip_id));
  if (st != d.stream) {
    // :38-40: the sync stream waits for the task's gradient.
    if (!r.client) HIP_TRY(hipEventCreateWithFlags(&r.client, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(r.client, st));
    HIP_TRY(hipStreamWaitEvent(d.stream, r.client, 0));
  }
  cbx::LaunchConfig cfg = c->aux_cfg;
  cfg.num_cus = d.num_cus;
  cfg.blocks_per_cu = 0;
  HIP_TRY(cbx::launch_ssgd_accumulate(a, cfg, d.stream, {}));
  return CBX_OK;
}

static int replica_optimise_impl(cbx_context *c, int id, int task, void *stream);

// Task threads call this while the collector thread may be enqueueing a
// barrier.  The foreign-op counter is bumped on entry (check_replica) AND
// after the enqueue: a cross-step pipelined step that read the counter
// between the two then sees it move again, and the next step joins the
// whole sync stream, which by then holds this call's wait.
int cbx_replica_optimise(cbx_context *c, int id, int task, void *stream) {
  TraceRange trace("cbx_replica_optimise");
  const int rc = replica_optimise_impl(c, id, task, stream);
  if (c) c->foreign_ops.fetch_add(1, std::memory_order_release);
  return rc;
}

static int replica_optimise_impl(cbx_context *c, int id, int task, void *stream) {
  TRY(check_replica(c, id, true));
  Replica &r = *c->replicas[id];
  Device &d = c->devs[r.local];
  SolverConf &conf = r.conf;
  const int type = c->model.type;
  if (type == CBX_UPDATE_WORKER)
    return ssgd_worker_step(c, r, d, task, stream ? reinterpret_cast<hipStream_t>(stream) : d.stream);
  if (type == CBX_UPDATE_DEFAULT)
    return default_task_step(c, r, d, task, stream ? reinterpret_cast<hipStream_t>(stream) : d.stream);
  if (type != CBX_UPDATE_SMA && type != CBX_UPDATE_SYNCHRONOUSEAMSGD)
    return fail(CBX_ERR_UNSUPPORTED, "update model %d has no optimiser step in this library", type);
  if (conf.momentum > 0 && conf.momentumMethod == 1)
    return fail(CBX_ERR_UNSUPPORTED, "Nesterov's momentum has been disabled");  // sma.cu:46-48
  if (conf.momentum > 0 && !c->has_last)
    return fail(CBX_ERR_STATE, "replica momentum without a `last` buffer (model.c:116-120)");
  float lr = 0.0f;
  TRY(conf.learning_rate(task, &lr));  // may raise _copy (solverconfiguration.c:133,147)
  cbx::OptArgs a;
  std::memset(&a, 0, sizeof(a));
  a.w = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_DATA));
  a.g = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_GRADIENT));
  a.last = conf.momentum > 0 ? reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_LAST)) : nullptr;
  a.s = reinterpret_cast<cbx::v4f *>(replica_dev(d, r, CBX_BUF_DIFF));
  a.n4 = c->n4;
  a.rate = -lr;  // sma.cu:43
  a.momentum = conf.momentum;
  a.wd = conf.weightDecay;
  HIP_TRY(hipSetDevice(d.hip_id));
  hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : d.stream;
  cbx::LaunchConfig cfg = c->aux_cfg;
  cfg.num_cus = d.num_cus;
  cfg.blocks_per_cu = 0;
  // The replica must not be updated while the last synchronise() still uses
  // it (the reference's forward kernels wait on replica->updated).
  if (st != d.stream && d.step_event) HIP_TRY(hipStreamWaitEvent(st, d.step_event, 0));
  HIP_TRY(cbx::launch_sma_optimise(a, cfg, st, {}));
  if (st != d.stream) {
    // sma.cu:79-81: the synchronisation stream waits for the updated replica.
    if (!r.client) HIP_TRY(hipEventCreateWithFlags(&r.client, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(r.client, st));
    HIP_TRY(hipStreamWaitEvent(d.stream, r.client, 0));
  }
  return CBX_OK;
}

// ---- batch-norm running statistics (cudnn/cudnnbatchnormparams.c:157-222) --
static int grow(void **p, size_t *have, size_t need) {
  if (*have >= need) return CBX_OK;
  if (*p) HIP_TRY(hipFree(*p));
  *p = nullptr;
  *have = 0;
  HIP_TRY(hipMalloc(p, need));
  *have = need;
  return CBX_OK;
}

int cbx_average_batchnorm_stats(cbx_context *c, int layers, const int *elements, float *const *mean,
                                float *const *variance, const int *updated) {
  TraceRange trace("cbx_average_batchnorm_stats");
  TRY(check_ctx(c));
  if (layers < 0 || (layers > 0 && (!elements || !mean || !variance || !updated)))
    return fail(CBX_ERR_INVALID, "bad batch-norm statistics arguments");
  if (layers == 0) return CBX_OK;
  // :165-166: nothing to average with one device.
  const bool run = c->G > 1 || c->force_split;
  if (!run) return CBX_OK;
  if (c->G == 1 && c->devs[0].comm == nullptr) {
    Device &d = c->devs[0];
    HIP_TRY(hipSetDevice(d.hip_id));
    int dev = d.hip_id;
    NCCL_TRY(ncclCommInitAll(&d.comm, 1, &dev));
  }
  uint32_t maxlen = 0;
  size_t total = 0;
  for (int l = 0; l < layers; ++l) {
    if (elements[l] < 0) return fail(CBX_ERR_INVALID, "layer %d has %d elements", l, elements[l]);
    maxlen = std::max(maxlen, (uint32_t)elements[l]);
    total += (size_t)elements[l];
  }
  const size_t head = ((size_t)layers + 63) / 64 * 64;  // count slots, one per layer
  const size_t floats = head + 2 * total;
  const int nseg = 2 * layers;
  std::vector<cbx::BnSegment> segs(nseg);
  for (size_t k = 0; k < c->devs.size(); ++k) {
    Device &d = c->devs[k];
    HIP_TRY(hipSetDevice(d.hip_id));
    size_t off = head;
    for (int l = 0; l < layers; ++l) {
      const size_t j = k * (size_t)layers + l;
      if (!mean[j] || !variance[j]) return fail(CBX_ERR_INVALID, "null statistics buffer (device %zu, layer %d)", k, l);
      // :175: the default device (global 0) always counts, the others iff updated.
      const float scale = (d.g == 0 || updated[j]) ? 1.0f : 0.0f;
      segs[2 * l] = {mean[j], (uint32_t)elements[l], (uint32_t)off, (uint32_t)l, scale};
      segs[2 * l + 1] = {variance[j], (uint32_t)elements[l], (uint32_t)(off + elements[l]), (uint32_t)l, scale};
      off += 2 * (size_t)elements[l];
    }
    TRY(grow(reinterpret_cast<void **>(&d.bn_table), &d.bn_table_bytes, segs.size() * sizeof(cbx::BnSegment)));
    TRY(grow(reinterpret_cast<void **>(&d.bn_scratch), &d.bn_scratch_bytes, floats * sizeof(float)));
    HIP_TRY(hipDeviceSynchronize());  // :171 (producers on any stream are done)
    HIP_TRY(hipMemcpy(d.bn_table, segs.data(), segs.size() * sizeof(cbx::BnSegment), hipMemcpyHostToDevice));
    HIP_TRY(cbx::launch_bn_pack(d.bn_table, nseg, maxlen, d.bn_scratch, d.stream));
  }
  NCCL_TRY(ncclGroupStart());
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    NCCL_TRY(ncclAllReduce(d.bn_scratch, d.bn_scratch, floats, ncclFloat, ncclSum, d.comm, d.stream));
  }
  NCCL_TRY(ncclGroupEnd());
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(cbx::launch_bn_unpack(d.bn_table, nseg, maxlen, d.bn_scratch, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));  // :218
  }
  return CBX_OK;
}

// ---- task-side replica access ---------------------------------------------
int cbx_replica_lock(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, true));
  pthread_mutex_lock(&c->replicas[id]->lock);
  return CBX_OK;
}

int cbx_replica_unlock(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, true));
  pthread_mutex_unlock(&c->replicas[id]->lock);
  return CBX_OK;
}

int cbx_replica_task_done(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, true));
  c->replicas[id]->updates++;
  return CBX_OK;
}

int cbx_replica_clock(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, false));
  return c->replicas[id]->clock;
}

int cbx_replica_learning_rate(cbx_context *c, int id, int task, float *rate) {
  TRY(check_replica_q(c, id, false));
  if (!rate) return fail(CBX_ERR_INVALID, "null rate");
  return c->replicas[id]->conf.learning_rate(task, rate);
}

int cbx_replica_get_copy(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, false));
  return (int)c->replicas[id]->conf.copy;
}

int cbx_replica_set_copy(cbx_context *c, int id, int flag) {
  TRY(check_replica_q(c, id, false));
  c->replicas[id]->conf.copy = flag ? 1u : 0u;
  return CBX_OK;
}

// crossbowThetaQueueDisable / Enable (thetaqueue.c:168-206).
int cbx_replica_set_disabled(cbx_context *c, int id, int flag) {
  TRY(check_replica_q(c, id, false));
  std::atomic<int> &st = c->theta[id].state;
  if (flag) {
    int expect = kThetaFree;
    if (st.compare_exchange_strong(expect, kThetaSkip, std::memory_order_acq_rel)) return 0;
    return expect == kThetaSkip ? 0 : 1;  // :199-201: reserved by a task, still enabled
  }
  int expect = kThetaSkip;
  if (st.compare_exchange_strong(expect, kThetaFree, std::memory_order_acq_rel) || expect == kThetaFree) return CBX_OK;
  return fail(CBX_ERR_STATE, "replica %d is reserved by a task; enable it before acquiring it", id);  // :182-184
}

// ---- the theta queue: task-side reservation (modelmanager.c:147-204) ---------
static inline void spin_pause(unsigned &spins) {
  if (++spins < 4096)
    __builtin_ia32_pause();
  else
    sched_yield();
}

// crossbowThetaQueueGetNextSafely + Reserve (thetaqueue.c:106-128): the next
// enabled slot of this process in round-robin order, then spin until it is
// free and reserve it.  The reference spins forever when every slot is
// disabled; here that is CBX_ERR_STATE.
static int theta_reserve_next(cbx_context *c) {
  for (;;) {
    const int size = c->size;
    int id = -1;
    for (int tries = 0; tries < size && id < 0; ++tries) {
      const int next = (int)(c->theta_iter.fetch_add(1, std::memory_order_relaxed) % (unsigned)size);
      if (c->replicas[next]->local >= 0 && c->theta[next].state.load(std::memory_order_acquire) != kThetaSkip)
        id = next;
    }
    if (id < 0) return fail(CBX_ERR_STATE, "every model replica of this process is disabled");
    std::atomic<int> &st = c->theta[id].state;
    unsigned spins = 0;
    for (;;) {
      int expect = kThetaFree;
      if (st.compare_exchange_weak(expect, kThetaBusy, std::memory_order_acq_rel)) return id;
      if (expect == kThetaSkip) break;  // disabled meanwhile: take the next one
      spin_pause(spins);
    }
  }
}

int cbx_acquire_access(cbx_context *c, int *clock) {
  TRY(check_manager_q(c));
  if (!clock) return fail(CBX_ERR_INVALID, "null clock");
  // modelmanager.c:180-190
  const int id = theta_reserve_next(c);
  if (id < 0) return id;
  *clock = __atomic_load_n(&c->replicas[id]->clock, __ATOMIC_ACQUIRE);
  return id;
}

int cbx_upgrade_access(cbx_context *c, int id, int *clock) {
  TRY(check_manager_q(c));
  if (!clock) return fail(CBX_ERR_INVALID, "null clock");
  // modelmanager.c:192-198; 0 (Java null: the task processor re-acquires,
  // TaskProcessor.java:112-114) once the replica has been deleted.
  if (id < 0 || id >= c->size || c->theta[id].state.load(std::memory_order_acquire) != kThetaBusy) return 0;
  *clock = __atomic_load_n(&c->replicas[id]->clock, __ATOMIC_ACQUIRE);
  return 1;
}

int cbx_get_next_or_wait(cbx_context *c, int bound) {
  TRY(check_manager_q(c));
  // modelmanager.c:147-167: reserve, wait for the replica's clock to reach
  // `bound` (the barrier advances it), lock.
  const int id = theta_reserve_next(c);
  if (id < 0) return id;
  Replica &r = *c->replicas[id];
  unsigned spins = 0;
  while (bound > __atomic_load_n(&r.clock, __ATOMIC_ACQUIRE)) spin_pause(spins);
  pthread_mutex_lock(&r.lock);
  return id;
}

int cbx_replica_release(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, true));
  // modelmanager.c:200-204: unlock, then free the theta slot.  The reference
  // spins until the slot is BUSY; a slot nobody reserved is an error here.
  // A slot cbx_del_model took out of the rotation (SKIP) while the task held
  // it is still released: the delete waits for this unlock.
  std::atomic<int> &st = c->theta[id].state;
  if (st.load(std::memory_order_acquire) == kThetaFree)
    return fail(CBX_ERR_STATE, "replica %d was not reserved (cbx_acquire_access)", id);
  pthread_mutex_unlock(&c->replicas[id]->lock);
  int busy = kThetaBusy;
  st.compare_exchange_strong(busy, kThetaFree, std::memory_order_acq_rel);
  return CBX_OK;
}

int cbx_replica_device(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, false));
  return c->replicas[id]->g;
}

int cbx_replica_is_local(cbx_context *c, int id) {
  TRY(check_replica_q(c, id, false));
  return c->replicas[id]->local >= 0 ? 1 : 0;
}

int cbx_num_replicas(cbx_context *c) {
  TRY(check_manager_q(c));
  return c->size;
}

int cbx_num_devices(cbx_context *c) {
  TRY(check_ctx_q(c));
  return c->G;
}

int cbx_num_local_devices(cbx_context *c) {
  TRY(check_ctx_q(c));
  return (int)c->devs.size();
}

int cbx_local_device_index(cbx_context *c, int local) {
  TRY(check_ctx_q(c));
  if (local < 0 || local >= (int)c->devs.size()) return fail(CBX_ERR_INVALID, "local device %d out of range", local);
  return c->devs[local].g;
}

long long cbx_model_elements(cbx_context *c) {
  if (!c) return fail(CBX_ERR_INVALID, "null context");
  return c->manager ? (long long)c->n : (long long)c->model.elements;
}

// ---- buffers --------------------------------------------------------------
static int replica_ptr(cbx_context *c, int id, int kind, float **p, Device **dev) {
  TRY(check_replica(c, id, true));
  if (kind < CBX_BUF_DATA || kind > CBX_BUF_LAST) return fail(CBX_ERR_INVALID, "bad buffer kind %d", kind);
  if (kind == CBX_BUF_LAST && !c->has_last) return fail(CBX_ERR_INVALID, "no momentum buffer (momentum == 0)");
  Replica &r = *c->replicas[id];
  Device &d = c->devs[r.local];
  *p = replica_dev(d, r, kind);
  if (dev) *dev = &d;
  return CBX_OK;
}

static int base_ptr(cbx_context *c, int g, int kind, float **p, Device **dev) {
  TRY(check_manager(c));
  if (kind < CBX_BUF_DATA || kind > CBX_BUF_LAST) return fail(CBX_ERR_INVALID, "bad buffer kind %d", kind);
  if (!base_has(c, kind)) return fail(CBX_ERR_INVALID, "no momentum buffer (momentum == 0)");
  int k = local_of(c, g);
  if (k < 0) return fail(CBX_ERR_INVALID, "device %d is not driven by this process", g);
  *p = base_dev(c, c->devs[k], kind);
  if (dev) *dev = &c->devs[k];
  return CBX_OK;
}

int cbx_replica_buffer(cbx_context *c, int id, int kind, void **dev_ptr) {
  float *p = nullptr;
  TRY(replica_ptr(c, id, kind, &p, nullptr));
  *dev_ptr = p;
  return CBX_OK;
}

int cbx_base_buffer(cbx_context *c, int g, int kind, void **dev_ptr) {
  float *p = nullptr;
  TRY(base_ptr(c, g, kind, &p, nullptr));
  *dev_ptr = p;
  return CBX_OK;
}

static int copy_io(cbx_context *c, Device *d, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
  if (bytes != (size_t)c->n * 4)
    return fail(CBX_ERR_INVALID, "buffer is %lld bytes, got %zu", (long long)c->n * 4, bytes);
  HIP_TRY(hipSetDevice(d->hip_id));
  HIP_TRY(hipStreamSynchronize(d->stream));
  HIP_TRY(hipMemcpy(dst, src, bytes, kind));
  return CBX_OK;
}

int cbx_replica_write(cbx_context *c, int id, int kind, const void *src, size_t bytes) {
  float *p = nullptr;
  Device *d = nullptr;
  TRY(replica_ptr(c, id, kind, &p, &d));
  return copy_io(c, d, p, src, bytes, hipMemcpyHostToDevice);
}

int cbx_replica_read(cbx_context *c, int id, int kind, void *dst, size_t bytes) {
  float *p = nullptr;
  Device *d = nullptr;
  TRY(replica_ptr(c, id, kind, &p, &d));
  return copy_io(c, d, dst, p, bytes, hipMemcpyDeviceToHost);
}

int cbx_base_write(cbx_context *c, int g, int kind, const void *src, size_t bytes) {
  float *p = nullptr;
  Device *d = nullptr;
  TRY(base_ptr(c, g, kind, &p, &d));
  return copy_io(c, d, p, src, bytes, hipMemcpyHostToDevice);
}

int cbx_base_read(cbx_context *c, int g, int kind, void *dst, size_t bytes) {
  float *p = nullptr;
  Device *d = nullptr;
  TRY(base_ptr(c, g, kind, &p, &d));
  return copy_io(c, d, dst, p, bytes, hipMemcpyDeviceToHost);
}

// ---- staging --------------------------------------------------------------
int cbx_stage_in(cbx_context *c) {
  TraceRange trace("cbx_stage_in");
  TRY(check_manager(c));
  TRY(alloc_host_mirror(c));
  const size_t bytes = (size_t)c->n * 4;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    TRY(mark(c, d, EV_H2D0));
    HIP_TRY(hipMemcpyAsync(base_dev(c, d, CBX_BUF_DATA), base_host(d, CBX_BUF_DATA), bytes, hipMemcpyHostToDevice, d.stream));
    if (c->has_last)
      HIP_TRY(hipMemcpyAsync(base_dev(c, d, CBX_BUF_LAST), base_host(d, CBX_BUF_LAST), bytes, hipMemcpyHostToDevice, d.stream));
    for (int id : d.replicas) {
      Replica &r = *c->replicas[id];
      HIP_TRY(hipMemcpyAsync(replica_dev(d, r, CBX_BUF_DIFF), replica_host(d, r, CBX_BUF_DIFF), bytes, hipMemcpyHostToDevice, d.stream));
      HIP_TRY(hipMemcpyAsync(replica_dev(d, r, CBX_BUF_DATA), replica_host(d, r, CBX_BUF_DATA), bytes, hipMemcpyHostToDevice, d.stream));
    }
    TRY(mark(c, d, EV_H2D1));
  }
  return CBX_OK;
}

int cbx_stage_out(cbx_context *c) {
  TraceRange trace("cbx_stage_out");
  TRY(check_manager(c));
  TRY(alloc_host_mirror(c));
  const size_t bytes = (size_t)c->n * 4;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    TRY(mark(c, d, EV_D2H0));
    HIP_TRY(hipMemcpyAsync(base_host(d, CBX_BUF_DATA), base_dev(c, d, CBX_BUF_DATA), bytes, hipMemcpyDeviceToHost, d.stream));
    if (c->has_last)
      HIP_TRY(hipMemcpyAsync(base_host(d, CBX_BUF_LAST), base_dev(c, d, CBX_BUF_LAST), bytes, hipMemcpyDeviceToHost, d.stream));
    for (int id : d.replicas) {
      Replica &r = *c->replicas[id];
      HIP_TRY(hipMemcpyAsync(replica_host(d, r, CBX_BUF_DATA), replica_dev(d, r, CBX_BUF_DATA), bytes, hipMemcpyDeviceToHost, d.stream));
    }
    TRY(mark(c, d, EV_D2H1));
  }
  return CBX_OK;
}

int cbx_replica_host_buffer(cbx_context *c, int id, int kind, void **host_ptr) {
  float *p = nullptr;
  TRY(replica_ptr(c, id, kind, &p, nullptr));
  TRY(alloc_host_mirror(c));
  Replica &r = *c->replicas[id];
  *host_ptr = replica_host(c->devs[r.local], r, kind);
  return CBX_OK;
}

int cbx_base_host_buffer(cbx_context *c, int g, int kind, void **host_ptr) {
  float *p = nullptr;
  Device *d = nullptr;
  TRY(base_ptr(c, g, kind, &p, &d));
  TRY(alloc_host_mirror(c));
  *host_ptr = base_host(*d, kind);
  return CBX_OK;
}

int cbx_wait(cbx_context *c) {
  TRY(check_ctx_q(c));
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    HIP_TRY(hipStreamSynchronize(d.stream));
  }
  return CBX_OK;
}

int cbx_step_event(cbx_context *c, int local, void **event) {
  TRY(check_ctx_q(c));
  if (local < 0 || local >= (int)c->devs.size() || !event) return fail(CBX_ERR_INVALID, "bad step-event query");
  *event = reinterpret_cast<void *>(c->devs[local].step_event ? c->devs[local].step_event : c->devs[local].synched);
  return CBX_OK;
}

// ---- measurement ----------------------------------------------------------
int cbx_set_timing(cbx_context *c, int enable) {
  TRY(check_ctx(c));
  c->timing = enable != 0;
  for (Device &d : c->devs) {
    for (int k = 0; k < EV_COUNT; ++k) d.ev_valid[k] = false;
    d.ring_pos = 0;
    d.ring_count = 0;
    if (c->timing && d.ring.empty()) {
      HIP_TRY(hipSetDevice(d.hip_id));
      d.ring.resize((size_t)Device::kRing * 4, nullptr);
      d.ring_split.assign(Device::kRing, 0);
      d.ring_from_prev.assign(Device::kRing, 0);
      for (hipEvent_t &e : d.ring) HIP_TRY(hipEventCreate(&e));
    }
  }
  return CBX_OK;
}

int cbx_set_order_check(cbx_context *c, int enable) {
  // check_ctx counts a foreign op: the next step joins the whole stream, so
  // no cross-step wait spans a change of the events the waits use.
  TRY(check_ctx(c));
  if (enable && !c->timing) TRY(cbx_set_timing(c, 1));
  c->order_check = enable != 0;
  for (Device &d : c->devs)
    for (Device::OrderStep &o : d.ord) o.valid = false;
  return CBX_OK;
}

int cbx_check_order(cbx_context *c) {
  TRY(check_ctx_q(c));
  if (!c->order_check) return fail(CBX_ERR_STATE, "stream-order checking is off (cbx_set_order_check)");
  int checked = 0;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    Device::OrderStep &q = d.ord[d.ord_cur];      // the latest split step
    Device::OrderStep &p = d.ord[d.ord_cur ^ 1];  // the one before it
    for (Device::OrderStep *o : {&p, &q})
      if (o->valid) {
        TRY(check_order_step(*o));
        ++checked;
      }
    if (p.valid && q.valid) TRY(check_order_pair(p, q));
    p.valid = q.valid = false;
  }
  return checked;
}

int cbx_last_timing(cbx_context *c, int local, float *ms) {
  TRY(check_ctx_q(c));
  if (local < 0 || local >= (int)c->devs.size() || !ms) return fail(CBX_ERR_INVALID, "bad timing query");
  Device &d = c->devs[local];
  HIP_TRY(hipSetDevice(d.hip_id));
  for (int k = 0; k < CBX_T_COUNT; ++k) ms[k] = -1.0f;
  if (d.ring_count > 0) {
    const int slot = (d.ring_pos + Device::kRing - 1) % Device::kRing;
    const int kind = d.ring_split[slot];
    if (kind != 2) TRY(ring_span(d, slot, EV_START, EV_A, &ms[CBX_T_KERNEL]));
    if (kind == 1) {
      TRY(ring_span(d, slot, EV_A, EV_AR, &ms[CBX_T_ALLREDUCE]));
      TRY(ring_span(d, slot, EV_AR, EV_B, &ms[CBX_T_APPLY]));
    }
    TRY(ring_span(d, slot, EV_START, kind == 0 ? EV_A : EV_B, &ms[CBX_T_STEP]));
  }
  auto span = [&](int a, int b, float *out) -> int {
    if (!d.ev_valid[a] || !d.ev_valid[b]) return CBX_OK;
    HIP_TRY(hipEventSynchronize(d.ev[b]));
    HIP_TRY(hipEventElapsedTime(out, d.ev[a], d.ev[b]));
    return CBX_OK;
  };
  TRY(span(EV_H2D0, EV_H2D1, &ms[CBX_T_H2D]));
  TRY(span(EV_D2H0, EV_D2H1, &ms[CBX_T_D2H]));
  return CBX_OK;
}

int cbx_timing_history(cbx_context *c, int local, int which, float *ms, int max) {
  TRY(check_ctx_q(c));
  if (local < 0 || local >= (int)c->devs.size() || !ms || max < 0) return fail(CBX_ERR_INVALID, "bad history query");
  if (which != CBX_T_KERNEL && which != CBX_T_ALLREDUCE && which != CBX_T_APPLY && which != CBX_T_STEP)
    return fail(CBX_ERR_INVALID, "history covers kernel / all-reduce / apply / step only");
  Device &d = c->devs[local];
  HIP_TRY(hipSetDevice(d.hip_id));
  const int count = std::min(max, d.ring_count);
  for (int k = 0; k < count; ++k) {
    const int slot = (d.ring_pos + Device::kRing - count + k) % Device::kRing;
    int a = EV_START, b = EV_A;
    if (which == CBX_T_ALLREDUCE) { a = EV_A; b = EV_AR; }
    if (which == CBX_T_APPLY) { a = EV_AR; b = EV_B; }
    const int kind = d.ring_split[slot];
    if (which == CBX_T_STEP) { a = EV_START; b = (kind == 0) ? EV_A : EV_B; }
    if ((which == CBX_T_KERNEL && kind == 2) ||
        ((which == CBX_T_ALLREDUCE || which == CBX_T_APPLY) && kind != 1)) {
      ms[k] = -1.0f;
      continue;
    }
    TRY(ring_span(d, slot, a, b, &ms[k]));
  }
  return count;
}

int cbx_set_kernel_config(cbx_context *c, int block, int blocks_per_cu, int policy, int unroll) {
  TRY(check_ctx(c));
  // __launch_bounds__(256): at most one wave per SIMD per workgroup, so an
  // unroll-4 wave may hold its 72 float4s in the 512-entry VGPR+AGPR file.
  if (block < 64 || block > 256 || block % 64 != 0) return fail(CBX_ERR_INVALID, "block must be 64..256, multiple of 64");
  if (unroll != 1 && unroll != 2 && unroll != 4) return fail(CBX_ERR_INVALID, "unroll must be 1, 2 or 4");
  if (policy != 0 && policy != 1) return fail(CBX_ERR_INVALID, "policy must be 0 or 1");
  if (blocks_per_cu < 0) return fail(CBX_ERR_INVALID, "blocks_per_cu must be >= 0");
  if ((int64_t)block * unroll > cbx::kPadFloat4 || cbx::kPadFloat4 % ((int64_t)block * unroll) != 0)
    return fail(CBX_ERR_INVALID, "block*unroll must divide %lld", (long long)cbx::kPadFloat4);
  c->cfg.block = block;
  c->cfg.blocks_per_cu = blocks_per_cu;
  c->cfg.policy = policy;
  c->apply_cfg.policy = policy;  // load/store policy is shared; kernel B keeps its own geometry
  c->cfg.unroll = unroll;
  return CBX_OK;
}

int cbx_set_kernel_occupancy(cbx_context *c, int waves_per_cu) {
  TRY(check_ctx(c));
  if (waves_per_cu < -1 || waves_per_cu > 32) return fail(CBX_ERR_INVALID, "waves per CU must be -1 (auto) or 0..32");
  c->cfg.waves_per_cu = waves_per_cu;
  return CBX_OK;
}

int cbx_set_aux_kernel_config(cbx_context *c, int block, int unroll, int waves_per_cu) {
  TRY(check_ctx(c));
  if (block < 64 || block > 512 || block % 64 != 0) return fail(CBX_ERR_INVALID, "block must be 64..512, multiple of 64");
  if (unroll != 1 && unroll != 2) return fail(CBX_ERR_INVALID, "unroll must be 1 or 2");
  if ((int64_t)block * unroll > cbx::kPadFloat4 || cbx::kPadFloat4 % ((int64_t)block * unroll) != 0)
    return fail(CBX_ERR_INVALID, "block*unroll must divide %lld", (long long)cbx::kPadFloat4);
  if (waves_per_cu < -1 || waves_per_cu > 32) return fail(CBX_ERR_INVALID, "waves per CU must be -1 (auto) or 0..32");
  c->aux_cfg.block = block;
  c->aux_cfg.unroll = unroll;
  c->aux_cfg.waves_per_cu = waves_per_cu;
  return CBX_OK;
}

int cbx_set_barrier_kernel_config(cbx_context *c, int block, int unroll, int waves_per_cu) {
  TRY(check_ctx(c));
  if (block < 64 || block > 512 || block % 64 != 0) return fail(CBX_ERR_INVALID, "block must be 64..512, multiple of 64");
  if (unroll != 1 && unroll != 2) return fail(CBX_ERR_INVALID, "unroll must be 1 or 2");
  if ((int64_t)block * unroll > cbx::kPadFloat4 || cbx::kPadFloat4 % ((int64_t)block * unroll) != 0)
    return fail(CBX_ERR_INVALID, "block*unroll must divide %lld", (long long)cbx::kPadFloat4);
  if (waves_per_cu < -1 || waves_per_cu > 32) return fail(CBX_ERR_INVALID, "waves per CU must be -1 (auto) or 0..32");
  for (cbx::LaunchConfig *cfg : {&c->broadcast_cfg, &c->ssgd_apply_cfg}) {
    cfg->block = block;
    cfg->unroll = unroll;
    cfg->waves_per_cu = waves_per_cu;
  }
  return CBX_OK;
}

int cbx_set_apply_kernel_config(cbx_context *c, int block, int unroll, int waves_per_cu) {
  TRY(check_ctx(c));
  if (block < 64 || block > 256 || block % 64 != 0) return fail(CBX_ERR_INVALID, "block must be 64..256, multiple of 64");
  if (unroll != 1 && unroll != 2 && unroll != 4) return fail(CBX_ERR_INVALID, "unroll must be 1, 2 or 4");
  if ((int64_t)block * unroll > cbx::kPadFloat4 || cbx::kPadFloat4 % ((int64_t)block * unroll) != 0)
    return fail(CBX_ERR_INVALID, "block*unroll must divide %lld", (long long)cbx::kPadFloat4);
  if (waves_per_cu < -1 || waves_per_cu > 32) return fail(CBX_ERR_INVALID, "waves per CU must be -1 (auto) or 0..32");
  c->apply_cfg.block = block;
  c->apply_cfg.unroll = unroll;
  c->apply_cfg.waves_per_cu = waves_per_cu;
  return CBX_OK;
}

int cbx_set_pipeline_mode(cbx_context *c, int mode) {
  TRY(check_ctx(c));
  if (mode < 0 || mode > 1) return fail(CBX_ERR_INVALID, "pipeline mode must be 0 or 1");
  c->pipeline_mode = mode;
  return CBX_OK;
}

int cbx_set_cross_wait_stride(cbx_context *c, int stride) {
  TRY(check_ctx(c));
  if (stride < 1 || stride > 4096) return fail(CBX_ERR_INVALID, "cross-step wait stride must be 1..4096");
  c->cross_wait_stride = stride;
  return CBX_OK;
}

int cbx_set_allreduce_group(cbx_context *c, int group) {
  TRY(check_ctx(c));
  if (group < 1 || group > 4096) return fail(CBX_ERR_INVALID, "all-reduce group must be 1..4096");
  c->allreduce_group = group;
  return CBX_OK;
}

int cbx_set_allreduce_algorithm(cbx_context *c, int algorithm) {
  TRY(check_ctx(c));
  if (algorithm != CBX_ALLREDUCE_RCCL && algorithm != CBX_ALLREDUCE_PEER && algorithm != CBX_ALLREDUCE_RSAG)
    return fail(CBX_ERR_INVALID, "all-reduce algorithm must be CBX_ALLREDUCE_RCCL, _PEER or _RSAG");
  if (algorithm == CBX_ALLREDUCE_RSAG && (c->G > cbx::kMaxDevices || cbx::kPadFloat4 % c->G != 0))
    return fail(CBX_ERR_UNSUPPORTED, "the reduce-scatter form needs G dividing %lld (G = %d)",
                (long long)cbx::kPadFloat4, c->G);
  if (algorithm == CBX_ALLREDUCE_PEER && c->per_rank && c->G > 1)
    return fail(CBX_ERR_UNSUPPORTED, "the peer-read all-reduce needs one process over every device (cbx_init)");
  if (algorithm == CBX_ALLREDUCE_PEER && c->G > cbx::kMaxDevices)
    return fail(CBX_ERR_UNSUPPORTED, "the peer-read all-reduce takes at most %d devices", cbx::kMaxDevices);
  c->allreduce_algo = algorithm;
  return CBX_OK;
}

int cbx_set_staging_mode(cbx_context *c, int mode) {
  TRY(check_ctx(c));
  if (mode != CBX_STAGING_ZEROCOPY && mode != CBX_STAGING_DMA)
    return fail(CBX_ERR_INVALID, "staging mode must be CBX_STAGING_ZEROCOPY or CBX_STAGING_DMA");
  c->staging_mode = mode;
  return CBX_OK;
}

int cbx_set_bucket_elements(cbx_context *c, long long bucket_elements) {
  TRY(check_ctx(c));
  if (bucket_elements < 0) return fail(CBX_ERR_INVALID, "negative bucket size");
  c->bucket_elems = bucket_elements;
  return CBX_OK;
}

int cbx_set_force_split(cbx_context *c, int force) {
  TRY(check_ctx(c));
  c->force_split = force != 0;
  return CBX_OK;
}

int cbx_fill_synthetic(cbx_context *c, unsigned long long seed) {
  TRY(check_manager(c));
  const int64_t n = c->n;
  for (Device &d : c->devs) {
    HIP_TRY(hipSetDevice(d.hip_id));
    // Buffer ids as in oracle/sma_oracle.h: z 0, last 1, s_i 16+2i, w_i 17+2i.
    float *z = base_dev(c, d, CBX_BUF_DATA);
    HIP_TRY(cbx::launch_fill_normal(z, n, seed ^ 0ULL, 0.05f, nullptr, d.stream));
    if (c->has_last) HIP_TRY(cbx::launch_fill_normal(base_dev(c, d, CBX_BUF_LAST), n, seed ^ 1ULL, 0.001f, nullptr, d.stream));
    for (int id : d.replicas) {
      Replica &r = *c->replicas[id];
      float *s = replica_dev(d, r, CBX_BUF_DIFF);
      HIP_TRY(cbx::launch_fill_normal(s, n, seed ^ (unsigned long long)(16 + 2 * id), 0.01f, z, d.stream));
      HIP_TRY(cbx::launch_fill_normal(replica_dev(d, r, CBX_BUF_DATA), n, seed ^ (unsigned long long)(17 + 2 * id),
                                      0.001f, s, d.stream));
    }
    HIP_TRY(hipStreamSynchronize(d.stream));
  }
  return CBX_OK;
}

int cbx_bench_copy(cbx_context *c, size_t bytes, int iters, float *gbps) {
  TRY(check_ctx(c));
  if (!gbps || iters <= 0 || bytes < 16) return fail(CBX_ERR_INVALID, "bad copy benchmark arguments");
  Device &d = c->devs[0];
  HIP_TRY(hipSetDevice(d.hip_id));
  const int64_t n4 = (int64_t)(bytes / 16);
  cbx::v4f *a = nullptr, *b = nullptr;
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(&a), (size_t)n4 * 16));
  hipError_t e = hipMalloc(reinterpret_cast<void **>(&b), (size_t)n4 * 16);
  if (e != hipSuccess) {
    (void)hipFree(a);
    return fail(CBX_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
  }
  cbx::LaunchConfig cfg = c->cfg;
  cfg.num_cus = d.num_cus;
  int rc = CBX_OK;
  float ms = 0.0f;
  do {
    if (hipMemsetAsync(a, 0, (size_t)n4 * 16, d.stream) != hipSuccess) { rc = fail(CBX_ERR_HIP, "memset"); break; }
    for (int k = 0; k < 3 && rc == CBX_OK; ++k)
      if (cbx::launch_copy(b, a, n4, cfg, d.stream) != hipSuccess) rc = fail(CBX_ERR_HIP, "copy launch");
    if (rc != CBX_OK) break;
    if (hipEventRecord(d.ev[EV_H2D0], d.stream) != hipSuccess) { rc = fail(CBX_ERR_HIP, "event"); break; }
    for (int k = 0; k < iters && rc == CBX_OK; ++k) {
      hipError_t le = (k & 1) ? cbx::launch_copy(a, b, n4, cfg, d.stream) : cbx::launch_copy(b, a, n4, cfg, d.stream);
      if (le != hipSuccess) rc = fail(CBX_ERR_HIP, "copy launch: %s", hipGetErrorString(le));
    }
    if (rc != CBX_OK) break;
    if (hipEventRecord(d.ev[EV_H2D1], d.stream) != hipSuccess) { rc = fail(CBX_ERR_HIP, "event"); break; }
    if (hipEventSynchronize(d.ev[EV_H2D1]) != hipSuccess) { rc = fail(CBX_ERR_HIP, "sync"); break; }
    if (hipEventElapsedTime(&ms, d.ev[EV_H2D0], d.ev[EV_H2D1]) != hipSuccess) { rc = fail(CBX_ERR_HIP, "elapsed"); break; }
    *gbps = (float)(2.0 * (double)n4 * 16.0 * iters / (ms * 1e-3) / 1e9);
  } while (0);
  d.ev_valid[EV_H2D0] = d.ev_valid[EV_H2D1] = false;
  (void)hipFree(a);
  (void)hipFree(b);
  return rc;
}

}  // extern "C"
