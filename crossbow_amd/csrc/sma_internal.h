// sma_internal.h -- kernel arguments and launchers shared by the SMA kernels
// (sma_kernels.hip) and the execution context (context.hip).  Not part of the
// C-ABI; see include/crossbow_sma.h for that.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace cbx {

// Replicas per device handled by one launch (kernarg holds 2 pointers each).
constexpr int kMaxReplicas = 64;
// Unrolled (register-resident) replica chunk inside the kernels.
constexpr int kChunk = 8;
// Base-model momentum, hard-coded at clib-multigpu/synch/sma.c:152.
constexpr float kBaseMomentum = 0.9f;

typedef float v4f __attribute__((ext_vector_type(4)));

// One kernel argument block for every SMA kernel.  All buffers are fp32
// arrays of n4 float4s (the flat model buffer, clib-multigpu/model.c:127-157,
// padded to a multiple of kPadFloat4; the pad is zero and stays zero).  The
// acc / D buffers are preceded by a 256-byte control block whose first float
// counts this device's Phase-D copy requests; it is summed by the all-reduce
// together with the first bucket, so kernel B learns "copy on any device"
// without a host round trip.
struct SmaArgs {
  const v4f *s[kMaxReplicas];  // replica snapshots   (replica->diff)
  v4f *w[kMaxReplicas];        // replica parameters  (replica->data)
  v4f *z;                      // base model          (base->data)
  v4f *last;                   // base momentum       (base->last), may be null
  v4f *acc;                    // Phase A output      (base->gradient)
  const v4f *D;                // Phase B output      (base->diff)
  float *ctrl_out;             // acc control block   (kernel A writes)
  const float *ctrl_in;        // D control block     (kernel B reads)
  int64_t n4;                  // float4s in the launch's range (multiple of kPadFloat4)
  float alpha;                 // conf->alpha (sma.c:33)
  float copies;                // Phase D requests on this device (kernel A)
  int nrep;                    // locked replicas on this device, id order
  // Kernel B's Phase-D decision: 0 read ctrl_in; 1 read ctrl_in and publish
  // it to *decision (bucket 0 of a cross-step pipelined step); 2 read
  // *decision (its later buckets, whose ctrl_in the next step's first
  // all-reduce may already be overwriting).
  int decision_mode;
  float *decision;
  // Caller-owned buffers (the sma.c seam): elements [tail_lo, tail_hi) past
  // the last whole trip, done by the launch's first tail_blocks workgroups
  // (set by the launcher).  Zero for the context's padded buffers.
  int64_t tail_lo, tail_hi;
  int tail_blocks;
};

// Buffers are padded to this many float4s so every trip of every kernel is
// full (block * unroll <= 1024) and no bounds checks sit in the inner loop.
constexpr int64_t kPadFloat4 = 1024;
// Control block in front of acc / D, in floats (256 bytes keeps data aligned).
constexpr int64_t kCtrlFloats = 64;

struct LaunchConfig {
  int block = 64;          // threads per workgroup: 64 x unroll 2 at 2 waves/CU measured best (sweep.py --interleave)
  int blocks_per_cu = 0;   // 0: one trip per thread; >0: grid-stride, this many WGs per CU
  int policy = 1;          // 0 plain, 1 nontemporal global loads/stores
  int unroll = 2;          // float4s per lane per trip (1 or 2), wave-contiguous
  int num_cus = 256;
  // Occupancy cap, in waves per CU: 0 = none, -1 = auto (below).  Enforced
  // by reserving dynamic LDS per workgroup so that only that many waves fit.
  // Fewer concurrent waves keep fewer DRAM pages open: every streaming kernel
  // here runs fastest with about kStreamsPerCU buffer streams (reads plus
  // writes, one float4 per lane each) in flight per CU
  // (scripts/occupancy_sweep.py, scripts/aux_sweep.py, profiles/r01/).
  int waves_per_cu = -1;
};

constexpr int kStreamsPerCU = 56;

// The optimiser-step and S-SGD kernels: one-wave workgroups, one float4 per
// lane, auto occupancy (scripts/aux_sweep.py).
inline LaunchConfig aux_launch_config() {
  LaunchConfig c;
  c.block = 64;
  c.unroll = 1;
  c.waves_per_cu = -1;
  return c;
}

// The write-heavy barrier kernels (scripts/barrier_sweep.py, ResNet-50, R = 8):
// the DEFAULT broadcast (1 read + R writes) is fastest with 256-thread blocks
// at 8 waves per CU (148 us vs 174 us at the per-task shape), the S-SGD apply
// (3 reads + R + 3 writes) with one-wave blocks, two float4 per lane, 3 waves
// per CU (229 us vs 252 us).
inline LaunchConfig broadcast_launch_config() {
  LaunchConfig c;
  c.block = 256;
  c.unroll = 1;
  c.waves_per_cu = 8;
  return c;
}
// Kernel B of the G > 1 split path (sma_apply_kernel: 3 reads + 2 writes);
// cbx_set_apply_kernel_config overrides it.
inline LaunchConfig sma_apply_launch_config() {
  LaunchConfig c;
  c.block = 64;
  c.unroll = 2;
  c.waves_per_cu = -1;
  return c;
}
// The zero-copy staged kernels (PCIe-bound): one-wave blocks, two float4 per
// lane, a grid-stride loop over 4 blocks per CU, uncapped (scripts/pcie_bench.hip:
// the link saturates with a few hundred blocks in flight).
inline LaunchConfig staged_launch_config() {
  LaunchConfig c;
  c.block = 64;
  c.unroll = 2;
  c.blocks_per_cu = 4;
  c.waves_per_cu = 0;
  return c;
}
inline LaunchConfig ssgd_apply_launch_config() {
  LaunchConfig c;
  c.block = 64;
  c.unroll = 2;
  c.waves_per_cu = 3;
  return c;
}

// Waves per CU for a kernel whose lanes stream `reads` + `writes` buffers:
// 2 for the R = 8 SMA step (18 + 10), 8 for the optimiser step (3 + 4),
// 11 for kernel B (3 + 2).
inline int auto_waves_per_cu(int reads, int writes) {
  int streams = reads + writes;
  if (streams < 1) streams = 1;
  int w = (kStreamsPerCU + streams / 2) / streams;
  return w < 2 ? 2 : (w > 12 ? 12 : w);
}

// Dynamic LDS bytes per workgroup that cap a CU at the configured waves
// (160 KiB of LDS per CU, at most 64 KiB per workgroup on gfx950).
// In auto mode a launch too small to fill the chip many times over (under
// 16 waves per CU, e.g. LeNet's 4 MB buffers) is latency-bound and runs
// uncapped.
inline unsigned lds_for_occupancy(const LaunchConfig &cfg, int reads, int writes, unsigned grid) {
  const int waves_per_wg = (cfg.block + 63) / 64;
  if (cfg.waves_per_cu < 0 && (int64_t)grid * waves_per_wg < 16ll * cfg.num_cus) return 0;
  const int cap = cfg.waves_per_cu < 0 ? auto_waves_per_cu(reads, writes) : cfg.waves_per_cu;
  if (cap <= 0) return 0;
  int wgs_per_cu = cap / waves_per_wg;
  if (wgs_per_cu < 1) wgs_per_cu = 1;
  // The least LDS that still keeps a (wgs+1)-th workgroup out: the rest of
  // the CU's LDS stays free for kernels running beside this one (the RCCL
  // all-reduce on the comm stream of the G > 1 pipeline).
  unsigned per = (160u / (unsigned)(wgs_per_cu + 1) + 1u) * 1024u;
  if (per > 64u * 1024u) per = 64u * 1024u;
  return per;
}

// A launch too small to fill the chip 16 waves per CU over (LeNet's 4 MB
// buffers, small G > 1 buckets) is latency-bound: with one element group per
// lane every wave loads, then every wave stores, in lockstep across the chip.
// In auto mode such a launch of one-wave blocks runs one float4 per lane in a
// grid-stride loop over 8 blocks per CU instead, so waves fall out of step and
// one iteration's stores overlap the next one's loads (scripts/lenet_sweep.py,
// profiles/r01/lenet_sweep.jsonl: C2 22.6 -> 20.5 us).
inline LaunchConfig small_launch_shape(const LaunchConfig &cfg, int64_t n4) {
  if (cfg.waves_per_cu >= 0 || cfg.blocks_per_cu != 0 || cfg.block != 64) return cfg;
  const int64_t waves = (n4 + 64ll * cfg.unroll - 1) / (64ll * cfg.unroll);
  if (waves >= 16ll * cfg.num_cus) return cfg;
  LaunchConfig c = cfg;
  c.unroll = 1;
  c.blocks_per_cu = 8;
  return c;
}

// Every SMA launcher takes an optional (start, stop) event pair that the
// dispatch itself timestamps (hipExtLaunchKernelGGL): timing a launch adds no
// marker packets to the stream.  Pass nullptr for untimed launches.
struct Timing {
  hipEvent_t start = nullptr;
  hipEvent_t stop = nullptr;
};
// Fused 1-GPU step: Phase A + (identity) B + C (+ D when copy).
hipError_t launch_sma_fused(const SmaArgs &a, bool momentum, bool copy,
                            const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Multi-GPU kernel A: Phase A only, writes acc and the control slot.
hipError_t launch_sma_accumulate(const SmaArgs &a, bool write_ctrl,
                                 const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Multi-GPU kernel B: Phase C (+ D, gated by the reduced control slot).
hipError_t launch_sma_apply(const SmaArgs &a, bool momentum,
                            const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Reduce-scatter form (cbx_set_allreduce_algorithm RSAG), on this rank's
// shard of a bucket (a.n4 float4s, any count): last = fma(0.9, last, D).
hipError_t launch_sma_shard_momentum(const SmaArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// An empty dispatch whose own timestamps mark a point on `stream` (the
// stream-order check, cbx_set_order_check).
hipError_t launch_order_probe(hipStream_t stream, Timing t);
// One wave idling `ticks` of the wall clock (hipDeviceAttributeWallClockRate,
// kHz), touching no memory: fault injection for the order check's own tests.
hipError_t launch_delay(hipStream_t stream, uint64_t ticks);
// Host-staged step through zero-copy (cbx_synchronise_staged, staging mode
// CBX_STAGING_ZEROCOPY): the kernels read their inputs straight from the
// pinned host mirror over PCIe and write their outputs to the host mirror AND
// the device buffers, so each byte crosses the link once, both directions at
// once, with no DMA-engine copies and no per-bucket copy calls
// (scripts/pcie_bench.hip: 1.84 GB up + 1.02 GB down in 34-35 ms through
// kernels).  The device ends as cbx_stage_in + cbx_synchronise +
// cbx_stage_out leave it: s_i staged in, w_i / z / last updated.
struct StagedArgs {
  const v4f *sh[kMaxReplicas];  // host s_i (read)
  v4f *sd[kMaxReplicas];        // device s_i (written: the staged-in snapshot)
  v4f *wh[kMaxReplicas];        // host w_i (read; written back)
  v4f *wd[kMaxReplicas];        // device w_i (written)
  v4f *zh, *zd;                 // base model: host (read; written back) / device
  v4f *lh, *ld;                 // base momentum: host / device (may be null)
  v4f *acc;                     // kernel A: Phase A output (device)
  const v4f *D;                 // kernel B: all-reduced acc (device)
  float *ctrl_out;              // kernel A: acc control block
  const float *ctrl_in;         // kernel B: D control block
  int64_t n4;
  float alpha;
  float copies;
  int nrep;
  int pad_;
};
// G = 1: Phase A + C (+ D) in one pass, host in, host and device out.
hipError_t launch_sma_fused_staged(const StagedArgs &a, bool momentum, bool copy, const LaunchConfig &cfg,
                                   hipStream_t stream, Timing t = {});
// G > 1 kernel A: reads z, s_i, w_i from the host; writes s_i, w_i, z to the
// device, w_i to the host, acc (and the control block) to the device.
hipError_t launch_sma_accumulate_staged(const StagedArgs &a, bool write_ctrl, const LaunchConfig &cfg,
                                        hipStream_t stream, Timing t = {});
// G > 1 kernel B: reads D, z (device) and last (host); writes z, last to the
// host and the device (and w_i to both on Phase D).
hipError_t launch_sma_apply_staged(const StagedArgs &a, bool momentum, const LaunchConfig &cfg,
                                   hipStream_t stream, Timing t = {});
// Peer-read all-reduce of the single-process multi-device form (one process
// drives every GPU, the reference's own form, executioncontext.c:185-201):
// instead of an RCCL pass, kernels read the peers' buffers directly over
// xGMI (hipDeviceEnablePeerAccess), the way the reference's non-NCCL path
// copies peer buffers (synch/common.c:64-95).  Two-shot: device g reduces
// shard g of every device's acc (peer reads) into its own D, then kernel B
// on every device reads each shard of D from its owner and applies Phase C.
// Per GPU that moves 2 (G-1)/G * 4n bytes over xGMI, as a ring all-reduce
// does, but over all G-1 links at once, with no RCCL kernel and no extra D
// pass.  The sums run in device order from +0: the oracle's order, so the
// result is bit-exact and identical on every device.
constexpr int kMaxDevices = 16;
struct PeerArgs {
  const v4f *acc[kMaxDevices];        // reduce: every device's acc at this device's shard
  const float *ctrl_in[kMaxDevices];  // reduce: every device's acc control block
  const v4f *D[kMaxDevices];          // apply: every device's D (whole buffer; shard h is valid on device h)
  v4f *out;                           // reduce: this device's D at its shard
  float *ctrl_out;                    // reduce: this device's D control block
  int64_t n4;                         // reduce: float4s of the shard (may be 0)
  int64_t shard4;                     // float4s per shard (a multiple of kPadFloat4)
  int G;
  int pad_;
};
// D[shard] = sum over devices of acc[shard] in device order; the control
// blocks are summed the same way (block 0).
hipError_t launch_sma_peer_reduce(const PeerArgs &p, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Kernel B reading D from each shard's owner: Phase C (+ D on copy).
hipError_t launch_sma_peer_apply(const SmaArgs &a, const PeerArgs &p, bool momentum, const LaunchConfig &cfg,
                                 hipStream_t stream, Timing t = {});
// One wave, after a per-rank peer-read step's last kernel B on the same
// stream: if any of the G broken words (rank h's at broken + h * stride) is
// set, store seq into *poison unless it already holds a step
// (context_internal.h, kIpcPoison).
hipError_t launch_peer_poison_check(const uint64_t *broken, int64_t stride, int G, uint64_t *poison, uint64_t seq,
                                    hipStream_t stream);
// The replica's local optimiser step of one task (the producer of s and w,
// clib-multigpu/kernels/optimisers/sma.cu:3-100), fused into one pass.
struct OptArgs {
  v4f *w;          // replica->data
  v4f *g;          // replica->gradient (updated in place, as the reference leaves it)
  v4f *last;       // replica->last (momentum > 0 only)
  v4f *s;          // replica->diff: the snapshot of w before the update
  v4f *z;          // DEFAULT only: the device's base model (base->data), stepped too
  int64_t n4;      // float4s (multiple of kPadFloat4)
  float rate;      // -learning rate (sma.cu:43)
  float momentum;  // replica conf->momentum
  float wd;        // replica conf->weightDecay
  int pad_;
  int64_t tail_lo, tail_hi;  // caller-owned buffers: elements past the last whole trip (see SmaArgs)
  int tail_blocks;
};
hipError_t launch_sma_optimise(const OptArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// DEFAULT update model (0, kernels/optimisers/default.cu:3-131): the task
// step moves the replica and its device's base model by the same gradient.
// Reads w, g (, last), z; writes g (if changed), last, w, z.
hipError_t launch_default_optimise(const OptArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// DEFAULT barrier (synch/default.c:5-43): w_i = z for a.nrep replicas a.w[].
hipError_t launch_broadcast(const SmaArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Synchronous SGD (update model WORKER = 1), the other synchronous model that
// shares the base-model buffers and the all-reduce.
struct SsgdArgs {
  v4f *w[kMaxReplicas];  // locked replicas on this device (barrier copy), id order
  v4f *z;                // base->data
  v4f *last;             // base->last (momentum > 0 only)
  v4f *acc;              // base->gradient: accumulated lr-scaled replica gradients
  const v4f *D;          // base->diff: all-reduced acc (== acc at G = 1)
  const v4f *wsrc;       // task step: replica->data (weight decay input)
  v4f *g;                // task step: replica->gradient
  int64_t n4;
  float rate;            // task step: -learning rate (synchronoussgd.cu:46)
  float wd;              // task step: weight decay
  float ratio;           // barrier: 1 / wpc (synchronoussgd.c:55)
  float momentum;        // barrier: base conf->momentum (synchronoussgd.c:64)
  int nrep;
  int pad_;
  int64_t tail_lo, tail_hi;  // caller-owned buffers: elements past the last whole trip (see SmaArgs)
  int tail_blocks;
};
// Per task (synchronoussgd.cu:3-56): g = fma(wd, w, g); acc = fma(rate, g, acc).
hipError_t launch_ssgd_accumulate(const SsgdArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Barrier (synchronoussgd.c:13-106, common.c:198-220): D *= 1/wpc; momentum;
// z += D; acc = 0; every locked replica := z.
hipError_t launch_ssgd_apply(const SsgdArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t = {});
// Batch-norm running-statistics averaging (cudnn/cudnnbatchnormparams.c:157-222):
// every (layer, mean|variance) buffer of a device is one segment of a packed
// scratch buffer that a single all-reduce sums across devices.
struct BnSegment {
  float *ptr;      // the layer's running mean or variance on this device
  uint32_t len;    // floats
  uint32_t off;    // offset of the segment in the scratch (floats)
  uint32_t layer;  // count slot: scratch[layer] sums the counted devices
  float scale;     // 1 if this device's statistics count, else 0
};
// scratch[seg.off + i] = seg.ptr[i] if seg.scale != 0 else +0 (the buffer is
// then not read); scratch[seg.layer] = seg.scale.
hipError_t launch_bn_pack(const BnSegment *segs, int nseg, uint32_t maxlen, float *scratch, hipStream_t stream);
// seg.ptr[i] = r * scratch[seg.off + i], r = 1/count (count > 1) else 1.
hipError_t launch_bn_unpack(const BnSegment *segs, int nseg, uint32_t maxlen, const float *scratch,
                            hipStream_t stream);
// Synthetic normal fill.
hipError_t launch_fill_normal(float *out, int64_t n, uint64_t seed, float sigma,
                              const float *mean, hipStream_t stream);
// Float4 copy used to measure the HBM ceiling on the box.
hipError_t launch_copy(v4f *dst, const v4f *src, int64_t n4, const LaunchConfig &cfg,
                       hipStream_t stream);

}  // namespace cbx
