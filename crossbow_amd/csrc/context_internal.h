// context_internal.h -- the execution context's types and helpers, shared by
// context.hip (the C-ABI, the model manager, checkpoints) and sync_steps.hip
// (the barrier steps: SMA, host-staged SMA, S-SGD, the stream-order check).
// Internal to libcrossbow_sma; the C-ABI is include/crossbow_sma.h.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <fcntl.h>
#include <unistd.h>
#include <errno.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/crossbow_sma.h"
#include "sma_internal.h"

namespace cbx::host {

inline thread_local std::string g_last_error;

inline int fail(int code, const char *fmt, ...) {
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
// One enqueue thread per local device (cbx_set_enqueue_threads).  The
// reference drives every GPU's sync step from its one ResultCollector thread
// (sma.c:42-128, common.c:14-54); at 8 devices and 8 buckets the HIP and RCCL
// calls of a step then take the host longer than the GPUs take to run them
// (profiles/r03/host_enqueue_single_thread.jsonl: 1.1 ms before RCCL's own
// enqueue cost, against ~0.6 ms of device time).  run(n, fn) calls fn(k) for
// every k < n, k = 0 on the calling thread and the others on workers that
// live as long as the context, and returns when all have finished (the first
// failure's code and message, in device order).  NCCL / RCCL take one thread
// per device with ncclCommInitAll's communicators: each thread issues its own
// device's collectives.
// ---------------------------------------------------------------------------
class EnqueuePool {
 public:
  EnqueuePool() = default;
  EnqueuePool(const EnqueuePool &) = delete;
  EnqueuePool &operator=(const EnqueuePool &) = delete;
  ~EnqueuePool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_start_.notify_all();
    for (std::thread &t : threads_) t.join();
  }

  int run(int n, const std::function<int(int)> &fn) {
    while ((int)threads_.size() < n - 1) {
      const int k = (int)threads_.size() + 1;
      try {
        threads_.emplace_back([this, k] { worker(k); });
      } catch (const std::exception &e) {  // no exception crosses the C-ABI
        return fail(CBX_ERR_STATE, "cannot start enqueue thread %d: %s", k, e.what());
      }
    }
    rc_.assign(n, 0);
    err_.assign(n, std::string());
    {
      std::lock_guard<std::mutex> l(m_);
      job_ = &fn;
      n_ = n;
      pending_.store(n - 1, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_start_.notify_all();
    rc_[0] = fn(0);
    if (rc_[0] < 0) err_[0] = g_last_error;
    // Wait for the workers: spin a little (a step's enqueue is ~0.1 ms), then sleep.
    for (int spin = 0; pending_.load(std::memory_order_acquire) != 0; ++spin) {
      if (spin < 4000) {
        sched_yield();
        continue;
      }
      std::unique_lock<std::mutex> l(m_);
      cv_done_.wait(l, [this] { return pending_.load(std::memory_order_acquire) == 0; });
    }
    {
      std::lock_guard<std::mutex> l(m_);  // a worker outside this run may be reading it
      job_ = nullptr;
    }
    for (int k = 0; k < n; ++k)
      if (rc_[k] < 0) {
        g_last_error = err_[k];
        return rc_[k];
      }
    return CBX_OK;
  }

 private:
  void worker(int k) {
    uint64_t seen = 0;
    for (;;) {
      // Spin briefly on the generation (steps come back to back), then sleep.
      uint64_t g = gen_.load(std::memory_order_acquire);
      for (int spin = 0; g == seen && spin < 2000; ++spin) {
        sched_yield();
        g = gen_.load(std::memory_order_acquire);
      }
      const std::function<int(int)> *job;
      int n;
      {
        std::unique_lock<std::mutex> l(m_);
        if (g == seen) cv_start_.wait(l, [&] { return gen_.load(std::memory_order_acquire) != seen; });
        if (stop_) return;
        // generation, job and count change together under the lock
        seen = gen_.load(std::memory_order_acquire);
        job = job_;
        n = n_;
      }
      if (job && k < n) {
        rc_[k] = (*job)(k);
        if (rc_[k] < 0) err_[k] = g_last_error;
        if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
          std::lock_guard<std::mutex> l(m_);
          cv_done_.notify_all();
        }
      }
    }
  }

  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_start_, cv_done_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  bool stop_ = false;
  const std::function<int(int)> *job_ = nullptr;
  int n_ = 0;
  std::vector<int> rc_;
  std::vector<std::string> err_;
};

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
  // Kernels A alternate over two streams, so the waves of bucket k+1 fill
  // the CUs while bucket k's drain instead of after (8 buckets: 0.548 ms per
  // step against 0.586-0.623 on one stream and 0.551 with one bucket,
  // profiles/r03/pipeline_streams_ab.json).
  hipStream_t a_stream = nullptr;
  hipStream_t a_stream2 = nullptr;
  std::vector<hipEvent_t> bucket_b;
  // The sync stream's wait for replica updates made on callers' streams
  // (cbx_replica_optimise with a stream of its own: sma.cu:79-81), deferred
  // to the next operation of the library on this device (flush_task_waits):
  // per caller stream an event recorded after its latest update.  A wait
  // queued at once stays pending on the sync stream's hardware queue while
  // the update runs, and a kernel on a hardware queue of its own runs about a
  // third slower while another queue of the process holds a wait on it
  // (scripts/queue_wait_probe.hip).  Task threads add entries
  // concurrently, hence the lock.
  struct TaskWait {
    hipStream_t stream;
    hipEvent_t event;
    bool pending;
  };
  std::vector<TaskWait> task_waits;
  std::unique_ptr<std::mutex> task_mu = std::make_unique<std::mutex>();
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
  // The base model's acc (gradient) and D (diff) slots in allocations of
  // their own, once cbx_peer_export has run (one process per GPU): the other
  // ranks map exactly these two through IPC handles, not the whole arena (an
  // IPC open of a 2 GB allocation hung under HIP 7.0).  Null:
  // the arena's slots 1 and 2.
  char *xslot[2] = {nullptr, nullptr};
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
  // 2: the same, but the previous slot has since been reused by a newer step
  // (the ring wrapped), so this slot has no start any more (spans read -1).
  std::vector<char> ring_from_prev;
  bool start_chosen = false;  // step_start_event decided this slot's ring_from_prev
  unsigned long long start_foreign = ~0ull;  // foreign_ops at the last step_start_event
  int ring_pos = 0;
  int ring_count = 0;
  // Kernel spans of pipelined split steps (timing on, order check off): in
  // the last kSpanRing such steps every kernel A and B dispatch stops an
  // event of its own, and so does the collective of each bucket (an event
  // recorded on the comm stream after it).  Each record also keeps the events
  // that bound its start: the previous dispatch on its stream and the events
  // its stream waited on since.  A dispatch starts when the last of them has
  // completed, so stop - (latest of them) is its busy span, an upper bound
  // that includes the dispatch latency (SplitStep, cbx_timing_history).
  static constexpr int kSpanRing = 64;
  static constexpr int64_t kSpanMaxBuckets = 64;
  // a peer-read reduction waits for the last kernel A on both A streams of
  // every device, plus its stream's previous dispatch
  static constexpr int kSpanPreds = 2 * cbx::kMaxDevices + 2;
  enum SpanKind { SPAN_A = 0, SPAN_B = 1, SPAN_COLL = 2 };
  struct SpanRec {
    hipEvent_t stop = nullptr;
    hipEvent_t pred[kSpanPreds] = {};
    int npred = 0;  // 0: start unknown
    int kind = SPAN_A;
  };
  struct SpanSlot {
    int ring_slot = -1;       // the timing-ring slot of the step it holds
    bool preds_valid = true;  // false once the slot before it was reused (its records' predecessors are gone)
    int64_t nb = 0;
    std::vector<hipEvent_t> a, red, b;  // owned, timing-enabled, per bucket
    hipEvent_t entry = nullptr;         // owned: the cross-step join point on the sync stream
    std::vector<hipEvent_t> a_used, b_used;  // the stop events kernels A(k) / B(k) really carried
    std::vector<SpanRec> recs;
  };
  std::vector<SpanSlot> spans;  // kSpanRing, created with the timing ring
  std::vector<int> ring_span;   // timing-ring slot -> span slot, or -1
  int span_pos = 0;
  int span_last = -1;        // span slot of the last pipelined step
  int pending_span = -1;     // span slot of the step ring_advance is about to close
  bool cross_spans = false;  // the last cross-pipelined step ran with span events
};

}  // namespace cbx::host

struct cbx_context {
  using Device = cbx::host::Device;
  using ModelDef = cbx::host::ModelDef;
  using Replica = cbx::host::Replica;
  using ThetaSlot = cbx::host::ThetaSlot;
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
  // $CBX_FAULT_ONE_STREAM_COMM_WAIT restores the wait the pipeline had before
  // round 3's fix: with kernels A on two streams (mode 1) and all-reduce
  // groups, the group's comm wait covers only its last kernel A, not the last
  // one on the other A stream; a one-wave delay ahead of every kernel A that
  // wait skips makes the race certain (tests only: results are then wrong).
  bool fault_one_stream_comm_wait = std::getenv("CBX_FAULT_ONE_STREAM_COMM_WAIT") != nullptr;
  // $CBX_FAULT_FAIL_STEP_BUCKETS=N: a split SMA step over exactly N buckets
  // fails before it enqueues anything (the bench tuner's error path, tests only).
  int64_t fault_fail_buckets = std::getenv("CBX_FAULT_FAIL_STEP_BUCKETS")
                                   ? std::atoll(std::getenv("CBX_FAULT_FAIL_STEP_BUCKETS")) : 0;
  // Bumped by every C-ABI call that may enqueue work on a sync stream other
  // than the barrier path itself: a cross-step pipelined step then joins the
  // whole sync stream instead of waiting bucket by bucket.
  std::atomic<unsigned long long> foreign_ops{0};
  // One process over several local devices: 1 = each device's share of a
  // barrier step is enqueued by a thread of its own (cbx_set_enqueue_threads);
  // 0 and -1 (auto, the default) = the reference's one thread, until the
  // threaded form is measured on distinct devices (bench.py's tuner times both).
  int enqueue_threads = -1;
  std::unique_ptr<cbx::host::EnqueuePool> pool;
  // The peer-read all-reduce with one process per GPU (cbx_peer_export /
  // cbx_peer_import, sync_steps.hip): every other rank's acc and D slots
  // (Device::xslot) mapped here through IPC handles, and one page of completion flags in
  // POSIX shared memory that every rank pins (hipHostRegister).  Rank h
  // writes its flags from its streams (hipStreamWriteValue64: the step's
  // sequence number once kernel A / the reduction of a bucket is done); the
  // others' streams wait on them (hipStreamWaitValue64 >=).  The page is
  // host memory: it needs no IPC mapping of its own (scripts/ipcprobe.hip).
  struct PeerIpc {
    bool ready = false;
    bool broken = false;                  // a step failed part-way: the flags were released
    int me = 0;
    std::vector<char *> mapped;           // 2 per rank: its acc and D slots opened here (own: nullptr)
    std::vector<const cbx::v4f *> acc;    // per rank: acc data (own: the local arena's)
    std::vector<const float *> acc_ctrl;  // per rank: acc control block
    std::vector<const cbx::v4f *> D;      // per rank: D data
    void *page = nullptr;                 // the flag page, shared by every rank
    size_t page_bytes = 0;
    uint64_t *dpage = nullptr;            // the same page as the device sees it
    bool owner = false;                   // rank 0 created the shared-memory object
    char shm_name[64] = {};
    uint64_t seq = 0;                     // split steps run in this form
    int64_t max_nb = 0;                   // the most buckets any of them had (flag words in use)
    bool released = false;                // this rank's words hold the release value
  } ipc;
  // $CBX_FAULT_SKIP_PEER_WAIT (tests only): the per-rank peer-read form skips
  // its waits on the other ranks' flags, and every rank but 0 runs a 2 ms
  // idle kernel ahead of each kernel A, so rank 0 reads acc before it is
  // written (results are then wrong: the test proves the waits matter).
  bool fault_skip_peer_wait = std::getenv("CBX_FAULT_SKIP_PEER_WAIT") != nullptr;
  // $CBX_FAULT_PEER_FAIL="rank:seq[:bucket]" (tests only): that rank's
  // per-rank peer-read step with sequence number seq fails right after it
  // queued the flag write of kernel A of `bucket` (default 0; later buckets
  // leave earlier buckets' collectives and kernels B queued too), the
  // failure the release path must survive (queued flag writes vs
  // the host release).
  int fault_peer_fail_rank = fault_pair(std::getenv("CBX_FAULT_PEER_FAIL"), 0);
  int fault_peer_fail_seq = fault_pair(std::getenv("CBX_FAULT_PEER_FAIL"), 1);
  int fault_peer_fail_bucket = std::max(0, fault_pair(std::getenv("CBX_FAULT_PEER_FAIL"), 2));
  // $CBX_FAULT_IPC_STALL=seconds (tests only): rank 0's cbx_peer_import sleeps
  // that long where it would open the others' handles, as a thread stuck
  // inside hipIpcOpenMemHandle would (no timer of the library reaches it):
  // bench.py must still print its line (VERDICT r04 Next #1).
  int fault_ipc_stall_s = std::getenv("CBX_FAULT_IPC_STALL") ? std::atoi(std::getenv("CBX_FAULT_IPC_STALL")) : 0;
  // $CBX_FAULT_IPC_OPEN_FAIL=rank (tests only): that rank's opens in
  // cbx_peer_import fail, so every rank's import must fail with it.
  int fault_ipc_open_fail = std::getenv("CBX_FAULT_IPC_OPEN_FAIL") ? std::atoi(std::getenv("CBX_FAULT_IPC_OPEN_FAIL"))
                                                                    : -1;
  // $CBX_FAULT_SKIP_TASK_WAIT (tests only): cbx_replica_optimise on a
  // caller's stream queues no wait for the sync stream at all, so a barrier
  // right behind a busy task stream reads stale replicas (the test proves the
  // deferred wait is what orders them).
  bool fault_skip_task_wait = std::getenv("CBX_FAULT_SKIP_TASK_WAIT") != nullptr;

  static int fault_pair(const char *s, int which) {
    int v[3] = {-1, -1, -1};
    if (s && std::sscanf(s, "%d:%d:%d", &v[0], &v[1], &v[2]) >= 2) return v[which];
    return -1;
  }
};

namespace cbx::host {

// Whether a barrier step enqueues each local device's work on its own thread.
inline bool threaded(const cbx_context *c) { return c->devs.size() > 1 && c->enqueue_threads == 1; }

// Runs fn(k) for every local device k, on one thread per device when the
// context enqueues threaded, else in device order on this thread.
inline int for_devices(cbx_context *c, const std::function<int(int)> &fn) {
  if (!threaded(c)) {
    for (int k = 0; k < (int)c->devs.size(); ++k) TRY(fn(k));
    return CBX_OK;
  }
  if (!c->pool) c->pool.reset(new EnqueuePool());
  return c->pool->run((int)c->devs.size(), fn);
}

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

inline size_t slot_index_base(int kind) {
  switch (kind) {
    case CBX_BUF_DATA: return 0;
    case CBX_BUF_GRADIENT: return 1;
    case CBX_BUF_DIFF: return 2;
    default: return 3;
  }
}

inline size_t slot_index_replica(int slot, int kind) {
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
inline size_t data_offset(bool ctrl) { return ctrl ? (size_t)cbx::kCtrlFloats * sizeof(float) : 0; }

inline float *slot_ptr(char *arena, const Device &d, size_t slot, bool ctrl) {
  return reinterpret_cast<float *>(arena + slot * d.stride + data_offset(ctrl));
}

inline bool base_has(const cbx_context *c, int kind) { return kind != CBX_BUF_LAST || c->has_last; }

// A base-model slot: in the arena, or (acc / D after cbx_peer_export) in its own allocation.
inline char *base_slot(const Device &d, int kind) {
  const size_t s = slot_index_base(kind);
  if ((s == 1 || s == 2) && d.xslot[s - 1]) return d.xslot[s - 1];
  return d.arena + s * d.stride;
}

inline float *base_dev(const cbx_context *c, const Device &d, int kind) {
  const bool ctrl = (kind == CBX_BUF_GRADIENT || kind == CBX_BUF_DIFF);
  return reinterpret_cast<float *>(base_slot(d, kind) + data_offset(ctrl));
}

inline float *base_ctrl(const Device &d, int kind) {
  return reinterpret_cast<float *>(base_slot(d, kind));
}

inline size_t replica_kind_index(int kind) { return slot_index_replica(0, kind) - kBaseSlots; }

inline float *replica_dev(const Device &d, const Replica &r, int kind) {
  if (r.slot >= d.base_slots)
    return reinterpret_cast<float *>(d.extra[r.slot - d.base_slots] + replica_kind_index(kind) * d.stride);
  return slot_ptr(d.arena, d, slot_index_replica(r.slot, kind), false);
}

inline float *base_host(const Device &d, int kind) {
  const bool ctrl = (kind == CBX_BUF_GRADIENT || kind == CBX_BUF_DIFF);
  return slot_ptr(d.host, d, slot_index_base(kind), ctrl);
}

inline float *replica_host(const Device &d, const Replica &r, int kind) {
  if (r.slot >= d.base_slots)
    return reinterpret_cast<float *>(d.extra_host[r.slot - d.base_slots] + replica_kind_index(kind) * d.stride);
  return slot_ptr(d.host, d, slot_index_replica(r.slot, kind), false);
}

// The *_q checks are for calls that enqueue no device work (the barrier path,
// replica locks, queries); the others also count a possible foreign op.
inline int check_ctx_q(cbx_context *c) {
  if (!c) return fail(CBX_ERR_INVALID, "null context");
  return CBX_OK;
}

inline int check_ctx(cbx_context *c) {
  TRY(check_ctx_q(c));
  c->foreign_ops.fetch_add(1, std::memory_order_relaxed);
  return CBX_OK;
}

inline int check_manager_q(cbx_context *c) {
  TRY(check_ctx_q(c));
  if (!c->manager) return fail(CBX_ERR_STATE, "model manager not created (call cbx_set_model_manager)");
  return CBX_OK;
}

inline int check_manager(cbx_context *c) {
  TRY(check_manager_q(c));
  c->foreign_ops.fetch_add(1, std::memory_order_relaxed);
  return CBX_OK;
}

inline int check_replica_q(cbx_context *c, int id, bool need_local) {
  TRY(check_manager_q(c));
  if (id < 0 || id >= c->size) return fail(CBX_ERR_INVALID, "replica id %d out of range [0, %d)", id, c->size.load());
  if (need_local && c->replicas[id]->local < 0)
    return fail(CBX_ERR_INVALID, "replica %d lives in another process (device %d)", id, c->replicas[id]->g);
  return CBX_OK;
}

inline int check_replica(cbx_context *c, int id, bool need_local) {
  TRY(check_manager(c));
  if (id < 0 || id >= c->size) return fail(CBX_ERR_INVALID, "replica id %d out of range [0, %d)", id, c->size.load());
  if (need_local && c->replicas[id]->local < 0)
    return fail(CBX_ERR_INVALID, "replica %d lives in another process (device %d)", id, c->replicas[id]->g);
  return CBX_OK;
}

inline int local_of(cbx_context *c, int g) {
  for (size_t k = 0; k < c->devs.size(); ++k)
    if (c->devs[k].g == g) return (int)k;
  return -1;
}

inline int gfx950_device_count(int *count) {
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

// A visible gfx950 device: its CU count, and it becomes the current device.
// Anything else fails loudly (no CPU fallback).
inline int probe_device(int hip_id, int *num_cus) {
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
  *num_cus = p.multiProcessorCount;
  HIP_TRY(hipSetDevice(hip_id));
  return CBX_OK;
}

// A non-blocking stream for the library's own work (executioncontext.c:324).
// ROCclr maps streams onto a pool of GPU_MAX_HW_QUEUES (4) hardware queues
// per device, shared by every stream of the process: a new stream takes a
// new queue until the pool is full, then the least-used one.  Two streams on
// one queue serialise at every stream wait, so the bucket pipeline's waits
// on one stream would stall another's kernels: 8-bucket cross-step steps
// measured 0.59-0.62 ms on some contexts and 0.72-1.1 ms on others, by
// creation order (profiles/r03/pipeline_streams_ab.json).  So a device's four
// streams (sync, comm, and the two of kernels A) are created together in
// open_device, before RCCL creates its own, and take the pool's first
// queues: at HIP's default 4 queues the pipeline then measured within 3 % of
// 16 (profiles/r04/hw_queues_ab.jsonl).  HIP's default 4 is the recommended
// deployment setting (beyond 4, a later stream's queue shares
// a pipe with one of these), which the library does not impose.  (CU-mask
// streams get queues of their own too, but they synchronise with the null
// stream; the reference's sync stream is non-blocking.)
inline int create_stream(hipStream_t *s) {
  HIP_TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
  return CBX_OK;
}

inline int open_device(Device &d, int hip_id, int g) {
  TRY(probe_device(hip_id, &d.num_cus));
  d.hip_id = hip_id;
  d.g = g;
  d.file_id = g;
  // executioncontext.c:324: one non-blocking model-synchronisation stream.
  TRY(create_stream(&d.stream));
  TRY(create_stream(&d.comm_stream));
  TRY(create_stream(&d.a_stream));
  TRY(create_stream(&d.a_stream2));
  HIP_TRY(hipEventCreateWithFlags(&d.synched, hipEventDisableTiming));
  for (int k = 0; k < EV_COUNT; ++k) HIP_TRY(hipEventCreate(&d.ev[k]));
  return CBX_OK;
}

inline void close_device(Device &d) {
  if (d.stream == nullptr && d.arena == nullptr) return;
  (void)hipSetDevice(d.hip_id);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  if (d.comm_stream) (void)hipStreamSynchronize(d.comm_stream);
  if (d.comm) (void)ncclCommDestroy(d.comm);
  if (d.arena) (void)hipFree(d.arena);
  for (char *&x : d.xslot)
    if (x) (void)hipFree(x);
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
  for (Device::SpanSlot &s : d.spans) {
    for (auto *v : {&s.a, &s.red, &s.b})
      for (hipEvent_t e : *v) (void)hipEventDestroy(e);
    if (s.entry) (void)hipEventDestroy(s.entry);
  }
  for (hipEvent_t e : d.bucket_acc) (void)hipEventDestroy(e);
  for (hipEvent_t e : d.bucket_red) (void)hipEventDestroy(e);
  if (d.a_stream) (void)hipStreamSynchronize(d.a_stream);
  if (d.a_stream2) (void)hipStreamSynchronize(d.a_stream2);
  for (hipEvent_t e : d.bucket_b) (void)hipEventDestroy(e);
  if (d.cross_entry) (void)hipEventDestroy(d.cross_entry);
  for (Device::TaskWait &w : d.task_waits) (void)hipEventDestroy(w.event);
  d.task_waits.clear();
  for (auto &pool : d.ord_pool)
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  if (d.peer_a) (void)hipEventDestroy(d.peer_a);
  if (d.peer_r) (void)hipEventDestroy(d.peer_r);
  if (d.decision) (void)hipFree(d.decision);
  if (d.a_stream) (void)hipStreamDestroy(d.a_stream);
  if (d.a_stream2) (void)hipStreamDestroy(d.a_stream2);
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
inline hipEvent_t ring_event(cbx_context *c, Device &d, int ev) {
  if (!c->timing || d.ring.empty()) return nullptr;
  return d.ring[(size_t)d.ring_pos * 4 + ev];
}

// The stop event of ring slot `slot`'s step: EV_A for a fused step (kind 0),
// EV_B for a split one.
inline hipEvent_t ring_stop(Device &d, int slot) {
  return d.ring[(size_t)slot * 4 + (d.ring_split[slot] == 0 ? EV_A : EV_B)];
}

// The START event for the first dispatch of a fused (kind 0) or pipelined
// split (kind 2) step.  A dispatch start event is a marker packet that costs
// the stream ~4.5 us per launch, while a stop event costs nothing
// (scripts/event_ts_probe.hip: 20.8 vs 16.4 us per back-to-back launch).
// When the previous slot is a step of the same kind whose stop has not
// completed yet, and no other C-ABI call enqueued work since, this step is
// enqueued behind a busy GPU: that stop stands in
// as this step's start (a fused step queues right behind it on the same
// stream; a pipelined step's span becomes its stop-to-stop share of the
// pipeline) and no marker is added.  Otherwise (an idle GPU, another kind of
// step) START is recorded.
inline hipEvent_t step_start_event(cbx_context *c, Device &d, int kind) {
  if (!c->timing || d.ring.empty()) return nullptr;
  const int slot = d.ring_pos;
  d.ring_from_prev[slot] = 0;
  // Nothing else may have been enqueued since the previous step (a task's
  // optimiser step on the sync stream, a host write): the dispatch must queue
  // directly behind that step's stop.
  const unsigned long long foreign = c->foreign_ops.load(std::memory_order_acquire);
  const bool nothing_between = d.start_foreign == foreign;
  d.start_foreign = foreign;
  if (d.ring_count > 0 && nothing_between) {
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
inline hipEvent_t ring_start(Device &d, int slot) {
  if (!d.ring_from_prev.empty() && d.ring_from_prev[slot] == 2) return nullptr;  // its stand-in was overwritten
  if (!d.ring_from_prev.empty() && d.ring_from_prev[slot])
    return ring_stop(d, (slot + Device::kRing - 1) % Device::kRing);
  return d.ring[(size_t)slot * 4 + EV_START];
}

// Record a timing marker when timing is enabled.  Step events (START..B) go
// to the current ring slot, staging events to the fixed ones.
inline int mark(cbx_context *c, Device &d, int ev) {
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
inline void ring_advance(cbx_context *c, Device &d, int kind) {
  if (!c->timing || d.ring.empty()) return;
  d.ring_split[d.ring_pos] = (char)kind;
  if (!d.ring_span.empty()) d.ring_span[d.ring_pos] = d.pending_span;
  d.pending_span = -1;
  if (!d.start_chosen) d.ring_from_prev[d.ring_pos] = 0;  // a path that records START itself
  d.start_chosen = false;
  // The next slot (the oldest once the ring is full) borrowed the stop of the
  // slot just written as its start: that stop now belongs to the newest step.
  const int next = (d.ring_pos + 1) % Device::kRing;
  if (d.ring_from_prev[next] == 1) d.ring_from_prev[next] = 2;
  d.ring_pos = next;
  if (d.ring_count < Device::kRing) d.ring_count++;
}

// Elapsed ms between events a and b of ring slot `slot` (-1 if absent).
inline int ring_span(Device &d, int slot, int a, int b, float *out) {
  *out = -1.0f;
  HIP_TRY(hipEventSynchronize(d.ring[(size_t)slot * 4 + b]));
  hipEvent_t from = a == EV_START ? ring_start(d, slot) : d.ring[(size_t)slot * 4 + a];
  if (!from) return CBX_OK;  // the slot's start was lost to the ring's wrap
  HIP_TRY(hipEventElapsedTime(out, from, d.ring[(size_t)slot * 4 + b]));
  return CBX_OK;
}

// Busy ms of the `kind` dispatches (Device::SpanKind) of the pipelined step
// in ring slot `slot`: the length of the union of their intervals, each from
// the latest event that bounded its start to its stop (kernels A on two
// streams overlap; a plain sum would count the overlap twice).  Times are
// taken relative to the first such dispatch's stop, so events before it read
// negative (hipEventElapsedTime is signed; tests/test_gpu_parity.py pins it).
// -1 when the step kept no span records (another form, or overwritten).
inline int span_sum(Device &d, int slot, int kind, float *out) {
  *out = -1.0f;
  if (d.ring_span.empty() || d.ring_span[slot] < 0) return CBX_OK;
  Device::SpanSlot &sp = d.spans[d.ring_span[slot]];
  if (sp.ring_slot != slot || !sp.preds_valid) return CBX_OK;
  hipEvent_t ref = nullptr;
  std::vector<std::pair<float, float>> iv;
  for (const Device::SpanRec &r : sp.recs) {
    if (r.kind != kind) continue;
    if (r.npred <= 0) return CBX_OK;
    HIP_TRY(hipEventSynchronize(r.stop));
    if (!ref) ref = r.stop;
    float t1 = 0.0f, t0 = -1e30f;
    HIP_TRY(hipEventElapsedTime(&t1, ref, r.stop));
    for (int i = 0; i < r.npred; ++i) {
      float tp = 0.0f;
      HIP_TRY(hipEventElapsedTime(&tp, ref, r.pred[i]));
      t0 = std::max(t0, tp);
    }
    if (t1 < t0) return CBX_OK;
    iv.emplace_back(t0, t1);
  }
  if (iv.empty()) return CBX_OK;
  std::sort(iv.begin(), iv.end());
  float sum = 0.0f, lo = iv[0].first, hi = iv[0].second;
  for (size_t i = 1; i < iv.size(); ++i) {
    if (iv[i].first > hi) {
      sum += hi - lo;
      lo = iv[i].first;
      hi = iv[i].second;
    } else {
      hi = std::max(hi, iv[i].second);
    }
  }
  *out = sum + (hi - lo);
  return CBX_OK;
}

// ---- batch-norm running-statistics averaging (context.hip) ------------------
// One device of an averaging: its HIP id, global index (0 = the default
// device, which always counts), communicator, stream, and the segment table
// and packed scratch it grows on demand.
struct BnDevice {
  int hip_id;
  int global;
  ncclComm_t comm;
  hipStream_t stream;
  cbx::BnSegment **table;
  size_t *table_bytes;
  float **scratch;
  size_t *scratch_bytes;
};
int bn_average(std::vector<BnDevice> &devs, int layers, const int *elements, float *const *mean,
               float *const *variance, const int *updated);
int grow_device_buffer(void **p, size_t *have, size_t need);

// ---- the barrier steps (sync_steps.hip) ------------------------------------
// The same arguments over float4s [start4, start4 + len4) of every buffer.
cbx::SmaArgs offset_args(const cbx::SmaArgs &a, int64_t start4, int64_t len4);
// SMA (synch/sma.c:13-231): fused at G = 1; kernel A / collective / kernel B
// per bucket at G > 1 (or forced); the peer-read form.
int sma_step(cbx_context *c, int first);
// The same step from and to the pinned host mirror (cbx_synchronise_staged).
int sma_step_staged(cbx_context *c, int first, int buckets);
// Synchronous SGD, update model WORKER (synch/synchronoussgd.c:13-106).
int ssgd_step(cbx_context *c, int first);
// RCCL communicators on first use (one-rank, or a clique that repeats a device).
int ensure_comms(cbx_context *c);
// The step event of every device (cbx_step_event), after a step's last dispatch.
int finish_step(cbx_context *c);
// The stop event for a step's LAST dispatch (see sync_steps.hip).
hipEvent_t step_stop_event(cbx_context *c, Device &d, int ev);
int alloc_host_mirror(cbx_context *c);
// Stream-order check of one recorded step, and of two consecutive ones.
int check_order_step(const Device::OrderStep &o);
int check_order_pair(const Device::OrderStep &p, const Device::OrderStep &q);
// A replica update enqueued on a caller's stream `st`: the sync stream must
// wait for it before the library next uses the replica (defer_task_wait), and
// does so at its next operation on the device (flush_task_waits).
// At most kTaskWaitCap entries per device (defer_task_wait).
constexpr size_t kTaskWaitCap = 64;
int defer_task_wait(Device &d, hipStream_t st);
int flush_task_waits(cbx_context *c);

// The per-rank peer-read form's handles (cbx_peer_export / _import) and its
// teardown (cbx_free: waits until every rank is done with this rank's memory).
int peer_export(cbx_context *c, void *blob, size_t *bytes);
int peer_import(cbx_context *c, const void *blobs, int nranks);
void peer_close(cbx_context *c);

// Completion flags of the per-rank peer-read form, per rank: one word per
// bucket for "kernel A done", one for "reduction done", and one for "done
// with the other ranks' memory" (teardown), each holding a step sequence
// number (monotonic: a waiter waits for >=, so a flag already past it never
// blocks).  A failed step sets its kIpcBroken word, then writes kIpcRelease
// into its rank's words so no other rank's stream waits forever.  A release
// lets a wait pass on a flag whose data may never have been written, so a
// one-wave kernel after each step's last kernel B (same stream: every load
// of the step's kernels B has returned) reads all ranks' kIpcBroken words
// and, if one is set, records the step's sequence number in the rank's
// kIpcPoison word (a consumer may only have read stale data if a release,
// and so a broken word, came first).  Every
// rank checks the words before each collective step and in cbx_wait
// (peer_guard, peer_wait_check); cbx_resync_base clears them.
constexpr int64_t kIpcMaxBuckets = 4096;
constexpr size_t kIpcRankWords = 2 * kIpcMaxBuckets + 64;  // a[], r[], done + padding (512 B)
// kIpcOpened: this rank's imports are done; kIpcBroken: a step of this rank
// failed part-way or was refused; kIpcPoison: the sequence number of a step
// whose kernels B on this rank may have run after some rank's broken word was set
constexpr int kIpcA = 0, kIpcR = 1, kIpcDone = 2, kIpcOpened = 3, kIpcBroken = 4, kIpcPoison = 5;
constexpr uint64_t kIpcRelease = 1ull << 62;
// The largest buffer the per-rank peer-read form exports.  ROCr 1.18 as
// shipped with ROCm 7.0 (torch's bundled runtime, which the library shares
// inside a torch process) keeps each exported allocation's size as a 32-bit
// int (Runtime::IPCCreate stores it in a std::map<unsigned long, int>; its
// socket thread AsyncIPCSockServerConnLoop sign-extends it for the dmabuf
// export): from 2 GiB on the export fails, the thread closes the connection
// without an fd, and the opener's IPCClientImport retries its 0-byte recvmsg
// forever inside hipIpcOpenMemHandle.  ROCm 7.2 keeps the size in 64 bits.
// So every exported buffer stays below 2 GiB, rounded as ROCclr rounds an
// allocation (2 MiB): DESIGN.md 6.  ResNet-50's acc is 102 MB.
constexpr size_t kIpcMaxSlotBytes = (2ull << 30) - (2ull << 20);
inline size_t ipc_word(int rank, int kind, int64_t b) {
  return (size_t)rank * kIpcRankWords +
         (kind >= kIpcDone ? 2 * kIpcMaxBuckets + (size_t)(kind - kIpcDone) : (size_t)kind * kIpcMaxBuckets + b);
}
static_assert(2 * kIpcMaxBuckets + (kIpcPoison - kIpcDone) < (int64_t)kIpcRankWords, "flag words per rank");
// Before a collective step of any form (and the batch-norm all-reduce): once
// any rank's broken or poison word is set, this rank releases its own flags
// (so no rank's stream waits on them) and refuses with CBX_ERR_STATE until
// cbx_resync_base.  `what` names the refused call.
int peer_guard(cbx_context *c, const char *what);
// cbx_wait, after the streams drained: CBX_ERR_STATE if a kernel B of this
// rank recorded a poisoned step (its z / last are undefined).
int peer_wait_check(cbx_context *c);
// cbx_resync_base: broadcast z and last from `root` and clear the flag page.
int resync_base(cbx_context *c, int root);

}  // namespace cbx::host
