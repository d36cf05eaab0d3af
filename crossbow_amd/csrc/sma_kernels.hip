// sma_kernels.hip -- HIP kernels of the SMA step for CDNA4 (gfx950).
//
// The reference runs the step as 3R+3 cuBLAS saxpy calls, R+4 copies/memsets
// and 3 host-blocking syncs per GPU (clib-multigpu/synch/sma.c:13-231), moving
// (44R+48)n bytes.  Here one streaming pass reads every input once and writes
// every output once:
//
//   fused (1 GPU)     reads z, last, s_i, w_i  writes w_i, z, last   (12R+8+8m)n B
//   accumulate (A)    reads z, s_i, w_i        writes w_i, acc       (12R+8)n B
//   apply (B)         reads D, z, last         writes z, last (, w)  (12+8m)n B
//
// The work is an fp32 AXPY/reduce at ~0.1 flop/byte: HBM-bound, no MFMA.  Each
// lane moves 16-byte float4s (1 KiB per wave instruction), every load of a trip
// is issued before the first arithmetic, and the per-replica partial sum stays
// in registers -- no LDS is needed because no element is re-read.
//
// Arithmetic is the reference's, bit for bit: cuBLAS saxpy y := fma(a, x, y)
// in fp32 and the same operation order, so 1-GPU results equal the oracle's.
#include <hip/hip_ext.h>

#include "sma_internal.h"

namespace cbx {
namespace {

template <int P>
__device__ __forceinline__ v4f ld(const v4f *p) {
  if constexpr (P == 1) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

template <int P>
__device__ __forceinline__ void st(v4f *p, v4f v) {
  if constexpr (P == 1) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// Uniform (SGPR) base + 32-bit lane byte offset: lets the compiler use the
// global_load/store "saddr + voffset" form, one VGPR per address instead of a
// 64-bit pair per stream (18+ streams per lane at R = 8).
template <int P>
__device__ __forceinline__ v4f ldo(const v4f *base, uint32_t off) {
  return ld<P>(reinterpret_cast<const v4f *>(reinterpret_cast<const char *>(base) + off));
}

template <int P>
__device__ __forceinline__ void sto(v4f *base, uint32_t off, v4f v) {
  st<P>(reinterpret_cast<v4f *>(reinterpret_cast<char *>(base) + off), v);
}

// Wave-contiguous indexing: with U float4s per lane, wave w of block b owns
// the 64*U consecutive float4s starting at (b * waves_per_block + w) * 64 * U,
// lane l the float4s base + 64 u.  Each wave-instruction still moves one
// contiguous KiB, and a wave's U instructions per stream cover U KiB in a
// row (U = 2 at 64-thread blocks measured best: scripts/sweep.py --interleave).
template <int U>
__device__ __forceinline__ uint32_t first_elem(uint32_t block) {
  return (block * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64u * U + (threadIdx.x & 63u);
}

template <int U>
__device__ __forceinline__ uint32_t first_elem() {
  return first_elem<U>(blockIdx.x);
}

__device__ __forceinline__ v4f vfma(v4f a, v4f b, v4f c) {
  return __builtin_elementwise_fma(a, b, c);
}

// Buffers the caller owns (the sma.c seam, sma_seam.hip) hold exactly n
// floats, not whole kernel trips.  Their last elements [a.tail_lo, a.tail_hi)
// go to the first a.tail_blocks workgroups of the same launch (TAIL
// instantiations), one float per lane, with the float4 path's fma sequence;
// the bulk runs on the remaining workgroups.  One launch per phase instead of
// a second tail launch (a separate tail kernel cost ~20 us per step on
// separately allocated buffers: scripts/seam_layout_ab.py).
// PHASE 0: the fused step; 1: Phase A into acc; 2: Phases C (+ D if `copy`).
template <int PHASE, bool MOM>
__device__ __forceinline__ void sma_tail_elem(const SmaArgs &a, bool copy) {
  const int64_t i = a.tail_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.tail_hi) return;
  float *z = reinterpret_cast<float *>(a.z);
  float *last = reinterpret_cast<float *>(a.last);
  float D;
  float z0 = z[i];
  float l0 = 0.0f;
  if constexpr (MOM) l0 = last[i];
  if constexpr (PHASE == 2) {
    D = reinterpret_cast<const float *>(a.D)[i];
  } else {
    // Replicas in chunks of kTailChunk whose loads are all issued before the
    // chunk's first store (a store to w_r may alias any later load, so a
    // plain loop pays one HBM round trip per replica).
    constexpr int kTailChunk = 8;
    float acc = 0.0f;  // sma.c:66
    for (int c = 0; c < a.nrep; c += kTailChunk) {
      float sv[kTailChunk], wv[kTailChunk];
#pragma unroll
      for (int r = 0; r < kTailChunk; ++r) {
        if (c + r < a.nrep) {
          sv[r] = reinterpret_cast<const float *>(a.s[c + r])[i];
          wv[r] = reinterpret_cast<const float *>(a.w[c + r])[i];
        }
      }
#pragma unroll
      for (int r = 0; r < kTailChunk; ++r) {
        if (c + r < a.nrep) {
          const float d = fmaf(-1.0f, z0, sv[r]);                                     // sma.c:79-90
          reinterpret_cast<float *>(a.w[c + r])[i] = fmaf(-a.alpha, d, wv[r]);       // :93-99
          acc = fmaf(a.alpha, d, acc);                                               // :102-107
        }
      }
    }
    if constexpr (PHASE == 1) {
      reinterpret_cast<float *>(a.acc)[i] = acc;
      return;
    }
    D = acc;
  }
  if constexpr (MOM) {
    D = fmaf(kBaseMomentum, l0, D);  // sma.c:155-164
    last[i] = D;
  }
  z0 = fmaf(1.0f, D, z0);  // sma.c:169-174
  z[i] = z0;
  if (copy)
    for (int r = 0; r < a.nrep; ++r) reinterpret_cast<float *>(a.w[r])[i] = z0;  // sma.c:185-227
}

// ---------------------------------------------------------------------------
// Fused 1-GPU step.  R >= 0 replicas fully unrolled (R <= kChunk); R == -1
// takes a.nrep and walks the replicas in register-resident chunks of kChunk.
// Per element (sma.c):
//   d   = fma(-1, z, s_i)              :79-90
//   w_i = fma(-alpha, d, w_i)          :93-99
//   acc = fma(+alpha, d, acc)          :102-107   (acc starts at +0, :66)
//   D   = acc                          common.c:3-57 with one rank
//   D   = fma(0.9, last, D); last = D  :148-166 (if momentum > 0)
//   z   = fma(1, D, z)                 :168-174
//   w_i = z                            :185-227 (if any replica asked to copy)
// ---------------------------------------------------------------------------
template <int R, bool MOM, bool COPY, int P, bool TAIL, int U>
__global__ __launch_bounds__(256) void sma_fused_kernel(const SmaArgs a) {
  constexpr int RR = (R > 0) ? R : kChunk;
  if constexpr (TAIL) {
    if (blockIdx.x < (uint32_t)a.tail_blocks) {
      sma_tail_elem<0, MOM>(a, COPY);
      return;
    }
  }
  const uint32_t tb = TAIL ? (uint32_t)a.tail_blocks : 0u;
  const uint32_t trip = (gridDim.x - tb) * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f al = a.alpha;
  const v4f nal = -a.alpha;
  const v4f mb = kBaseMomentum;
  const v4f one = 1.0f;
  const v4f mone = -1.0f;
  for (uint32_t base = first_elem<U>(blockIdx.x - tb); base < n4; base += trip) {
    v4f zv[U], lv[U], acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      zv[u] = ldo<P>(a.z, i);
      if constexpr (MOM) lv[u] = ldo<P>(a.last, i);
      acc[u] = 0.0f;
    }
    const int nrep = (R >= 0) ? R : a.nrep;
    for (int c = 0; c < nrep; c += RR) {
      v4f sv[U][RR], wv[U][RR];
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sv[u][r] = ldo<P>(a.s[c + r], i);
          if constexpr (!COPY) wv[u][r] = ldo<P>(a.w[c + r], i);
        }
      }
      // Keep every load of the chunk in flight before the first use: without
      // this fence the scheduler sinks the last load below the first FMAs to
      // save registers, serialising one HBM round trip per wave (measured
      // +1-4 %, scripts/membench.hip v5), and it needs fewer VGPRs, not more.
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const v4f d = vfma(mone, zv[u], sv[u][r]);
          if constexpr (!COPY) wv[u][r] = vfma(nal, d, wv[u][r]);
          acc[u] = vfma(al, d, acc[u]);
        }
      }
      if constexpr (!COPY) {
#pragma unroll
        for (int r = 0; r < RR; ++r) {
          if (R < 0 && c + r >= nrep) break;
#pragma unroll
          for (int u = 0; u < U; ++u) sto<P>(a.w[c + r], (base + u * 64u) * 16u, wv[u][r]);
        }
      }
      if constexpr (R >= 0) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      v4f D = acc[u];
      if constexpr (MOM) {
        D = vfma(mb, lv[u], D);
        sto<P>(a.last, i, D);
      }
      zv[u] = vfma(one, D, zv[u]);
      sto<P>(a.z, i, zv[u]);
    }
    if constexpr (COPY) {
      for (int r = 0; r < nrep; ++r) {
#pragma unroll
        for (int u = 0; u < U; ++u) sto<P>(a.w[r], (base + u * 64u) * 16u, zv[u]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Kernel A (G > 1): Phase A on this device's locked replicas -> acc.
// ---------------------------------------------------------------------------
template <int R, int P, bool TAIL, int U>
__global__ __launch_bounds__(256) void sma_accumulate_kernel(const SmaArgs a) {
  constexpr int RR = (R > 0) ? R : kChunk;
  if (a.ctrl_out != nullptr && blockIdx.x == 0 && threadIdx.x < kCtrlFloats)
    a.ctrl_out[threadIdx.x] = (threadIdx.x == 0) ? a.copies : 0.0f;
  if constexpr (TAIL) {
    if (blockIdx.x < (uint32_t)a.tail_blocks) {
      sma_tail_elem<1, false>(a, false);
      return;
    }
  }
  const uint32_t tb = TAIL ? (uint32_t)a.tail_blocks : 0u;
  const uint32_t trip = (gridDim.x - tb) * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f al = a.alpha;
  const v4f nal = -a.alpha;
  const v4f mone = -1.0f;
  for (uint32_t base = first_elem<U>(blockIdx.x - tb); base < n4; base += trip) {
    v4f zv[U], acc[U];
    const int nrep = (R >= 0) ? R : a.nrep;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc[u] = 0.0f;
      if (nrep > 0) zv[u] = ldo<P>(a.z, (base + u * 64u) * 16u);
    }
    for (int c = 0; c < nrep; c += RR) {
      v4f sv[U][RR], wv[U][RR];
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sv[u][r] = ldo<P>(a.s[c + r], i);
          wv[u][r] = ldo<P>(a.w[c + r], i);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // all loads in flight first (see fused)
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const v4f d = vfma(mone, zv[u], sv[u][r]);
          wv[u][r] = vfma(nal, d, wv[u][r]);
          acc[u] = vfma(al, d, acc[u]);
        }
      }
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) sto<P>(a.w[c + r], (base + u * 64u) * 16u, wv[u][r]);
      }
      if constexpr (R >= 0) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) sto<P>(a.acc, (base + u * 64u) * 16u, acc[u]);
  }
}

// ---------------------------------------------------------------------------
// Kernel B (G > 1): Phase C on the all-reduced D, then Phase D when the
// reduced control block says any device had a copy request.
// ---------------------------------------------------------------------------
template <bool MOM, int P, bool TAIL, int U>
__global__ __launch_bounds__(256) void sma_apply_kernel(const SmaArgs a) {
  const float requests = a.decision_mode == 2 ? *a.decision : a.ctrl_in[0];
  if (a.decision_mode == 1 && blockIdx.x == 0 && threadIdx.x == 0) *a.decision = requests;
  const bool copy = requests > 0.0f;
  if constexpr (TAIL) {
    if (blockIdx.x < (uint32_t)a.tail_blocks) {
      sma_tail_elem<2, MOM>(a, copy);
      return;
    }
  }
  const uint32_t tb = TAIL ? (uint32_t)a.tail_blocks : 0u;
  const uint32_t trip = (gridDim.x - tb) * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f mb = kBaseMomentum;
  const v4f one = 1.0f;
  for (uint32_t base = first_elem<U>(blockIdx.x - tb); base < n4; base += trip) {
    v4f Dv[U], zv[U], lv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      Dv[u] = ldo<P>(a.D, i);
      zv[u] = ldo<P>(a.z, i);
      if constexpr (MOM) lv[u] = ldo<P>(a.last, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      if constexpr (MOM) {
        Dv[u] = vfma(mb, lv[u], Dv[u]);
        sto<P>(a.last, i, Dv[u]);
      }
      zv[u] = vfma(one, Dv[u], zv[u]);
      sto<P>(a.z, i, zv[u]);
    }
    if (copy) {
      for (int r = 0; r < a.nrep; ++r) {
#pragma unroll
        for (int u = 0; u < U; ++u) sto<P>(a.w[r], (base + u * 64u) * 16u, zv[u]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Reduce-scatter form of Phase C (cbx_set_allreduce_algorithm RSAG): on this
// rank's shard of a bucket, D' = fma(0.9, last, D) into last (sma.c:155-164);
// the all-gather of last then gives every rank every shard of D', and kernel B
// (without momentum, D := last) adds it to z.  One float4 per lane, bounds-
// checked: a shard is 1/G of a padded bucket.
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(256) void sma_shard_momentum_kernel(const SmaArgs a) {
  const v4f mb = kBaseMomentum;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n4; i += stride)
    st<P>(a.last + i, vfma(mb, ld<P>(a.last + i), ld<P>(a.D + i)));
}

// ---------------------------------------------------------------------------
// Host-staged step through zero-copy (sma_internal.h, StagedArgs).  Same
// arithmetic, in the same order, as the device-resident kernels above; host
// memory is read and written with plain loads / stores (PCIe-bound: ~55 GB/s
// each way), device memory with the nontemporal ones.
// ---------------------------------------------------------------------------
template <int R, bool MOM, bool COPY, int U>
__global__ __launch_bounds__(256) void sma_fused_staged_kernel(const StagedArgs a) {
  constexpr int RR = (R > 0) ? R : kChunk;
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f al = a.alpha, nal = -a.alpha, mb = kBaseMomentum, one = 1.0f, mone = -1.0f;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    v4f zv[U], lv[U], acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      zv[u] = ldo<0>(a.zh, i);
      if constexpr (MOM) lv[u] = ldo<0>(a.lh, i);
      acc[u] = 0.0f;
    }
    const int nrep = (R >= 0) ? R : a.nrep;
    for (int c = 0; c < nrep; c += RR) {
      v4f sv[U][RR], wv[U][RR];
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sv[u][r] = ldo<0>(a.sh[c + r], i);
          if constexpr (!COPY) wv[u][r] = ldo<0>(a.wh[c + r], i);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sto<1>(a.sd[c + r], i, sv[u][r]);
          const v4f d = vfma(mone, zv[u], sv[u][r]);
          if constexpr (!COPY) {
            wv[u][r] = vfma(nal, d, wv[u][r]);
            sto<0>(a.wh[c + r], i, wv[u][r]);
            sto<1>(a.wd[c + r], i, wv[u][r]);
          }
          acc[u] = vfma(al, d, acc[u]);
        }
      }
      if constexpr (R >= 0) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      v4f D = acc[u];
      if constexpr (MOM) {
        D = vfma(mb, lv[u], D);
        sto<0>(a.lh, i, D);
        sto<1>(a.ld, i, D);
      }
      zv[u] = vfma(one, D, zv[u]);
      sto<0>(a.zh, i, zv[u]);
      sto<1>(a.zd, i, zv[u]);
    }
    if constexpr (COPY) {
      for (int r = 0; r < nrep; ++r) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          sto<0>(a.wh[r], (base + u * 64u) * 16u, zv[u]);
          sto<1>(a.wd[r], (base + u * 64u) * 16u, zv[u]);
        }
      }
    }
  }
}

template <int R, int U>
__global__ __launch_bounds__(256) void sma_accumulate_staged_kernel(const StagedArgs a) {
  constexpr int RR = (R > 0) ? R : kChunk;
  if (a.ctrl_out != nullptr && blockIdx.x == 0 && threadIdx.x < kCtrlFloats)
    a.ctrl_out[threadIdx.x] = (threadIdx.x == 0) ? a.copies : 0.0f;
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f al = a.alpha, nal = -a.alpha, mone = -1.0f;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    v4f zv[U], acc[U];
    const int nrep = (R >= 0) ? R : a.nrep;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      acc[u] = 0.0f;
      zv[u] = ldo<0>(a.zh, i);
      sto<1>(a.zd, i, zv[u]);  // kernel B reads z from the device
    }
    for (int c = 0; c < nrep; c += RR) {
      v4f sv[U][RR], wv[U][RR];
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sv[u][r] = ldo<0>(a.sh[c + r], i);
          wv[u][r] = ldo<0>(a.wh[c + r], i);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sto<1>(a.sd[c + r], i, sv[u][r]);
          const v4f d = vfma(mone, zv[u], sv[u][r]);
          wv[u][r] = vfma(nal, d, wv[u][r]);
          sto<0>(a.wh[c + r], i, wv[u][r]);
          sto<1>(a.wd[c + r], i, wv[u][r]);
          acc[u] = vfma(al, d, acc[u]);
        }
      }
      if constexpr (R >= 0) break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) sto<1>(a.acc, (base + u * 64u) * 16u, acc[u]);
  }
}

template <bool MOM, int U>
__global__ __launch_bounds__(256) void sma_apply_staged_kernel(const StagedArgs a) {
  const bool copy = a.ctrl_in[0] > 0.0f;
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f mb = kBaseMomentum, one = 1.0f;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    v4f Dv[U], zv[U], lv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      Dv[u] = ldo<1>(a.D, i);
      zv[u] = ldo<1>(a.zd, i);
      if constexpr (MOM) lv[u] = ldo<0>(a.lh, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      if constexpr (MOM) {
        Dv[u] = vfma(mb, lv[u], Dv[u]);
        sto<0>(a.lh, i, Dv[u]);
        sto<1>(a.ld, i, Dv[u]);
      }
      zv[u] = vfma(one, Dv[u], zv[u]);
      sto<0>(a.zh, i, zv[u]);
      sto<1>(a.zd, i, zv[u]);
    }
    if (copy) {
      for (int r = 0; r < a.nrep; ++r) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          sto<0>(a.wh[r], (base + u * 64u) * 16u, zv[u]);
          sto<1>(a.wd[r], (base + u * 64u) * 16u, zv[u]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Peer-read two-shot all-reduce (single process, G devices; sma_internal.h).
// Reduce: this device's shard of D = sum over devices of acc, every load of a
// trip (G streams, G-1 of them remote over xGMI) in flight before the adds.
// ---------------------------------------------------------------------------
template <int G_, int P, int U>
__global__ __launch_bounds__(256) void sma_peer_reduce_kernel(const PeerArgs p) {
  constexpr int GG = (G_ > 0) ? G_ : kMaxDevices;
  const int G = (G_ > 0) ? G_ : p.G;
  if (p.ctrl_out != nullptr && blockIdx.x == 0 && threadIdx.x < kCtrlFloats) {
    float s = 0.0f;  // common.c:45-52 sums the control block with the data
    for (int h = 0; h < G; ++h) s = s + p.ctrl_in[h][threadIdx.x];
    p.ctrl_out[threadIdx.x] = s;
  }
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)p.n4;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    v4f x[U][GG];
#pragma unroll
    for (int h = 0; h < GG; ++h) {
      if (G_ <= 0 && h >= G) break;
#pragma unroll
      for (int u = 0; u < U; ++u) x[u][h] = ldo<P>(p.acc[h], (base + u * 64u) * 16u);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v4f sum = 0.0f;  // device order from +0: the oracle's (and the loopback's rank) order
#pragma unroll
      for (int h = 0; h < GG; ++h) {
        if (G_ <= 0 && h >= G) break;
        sum = sum + x[u][h];
      }
      sto<P>(p.out, (base + u * 64u) * 16u, sum);
    }
  }
}

// Kernel B of the peer path: D of element i comes from the owner of its
// shard.  Shards are multiples of kPadFloat4 float4s and a wave's 64*U float4s
// never straddle one, so the owner is wave-uniform (readfirstlane: the
// pointer is fetched with a scalar load).
template <bool MOM, int P, int U>
__global__ __launch_bounds__(256) void sma_peer_apply_kernel(const SmaArgs a, const PeerArgs p) {
  // the Phase-D decision as in sma_apply_kernel (decision_mode: cross-step buckets)
  const float requests = a.decision_mode == 2 ? *a.decision : a.ctrl_in[0];
  if (a.decision_mode == 1 && blockIdx.x == 0 && threadIdx.x == 0) *a.decision = requests;
  const bool copy = requests > 0.0f;
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const uint32_t shard4 = (uint32_t)p.shard4;
  const v4f mb = kBaseMomentum;
  const v4f one = 1.0f;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    int owner = __builtin_amdgcn_readfirstlane((int)(base / shard4));
    if (owner > p.G - 1) owner = p.G - 1;
    const v4f *D = p.D[owner];
    v4f Dv[U], zv[U], lv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      Dv[u] = ldo<P>(D, i);
      zv[u] = ldo<P>(a.z, i);
      if constexpr (MOM) lv[u] = ldo<P>(a.last, i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      if constexpr (MOM) {
        Dv[u] = vfma(mb, lv[u], Dv[u]);
        sto<P>(a.last, i, Dv[u]);
      }
      zv[u] = vfma(one, Dv[u], zv[u]);
      sto<P>(a.z, i, zv[u]);
    }
    if (copy) {
      for (int r = 0; r < a.nrep; ++r) {
#pragma unroll
        for (int u = 0; u < U; ++u) sto<P>(a.w[r], (base + u * 64u) * 16u, zv[u]);
      }
    }
  }
}

// One process per GPU (context_internal.h, kIpcPoison): launched on the sync
// stream right after a peer-read step's last kernel B, so every load of
// every kernel B of the step has returned before it reads each rank's broken
// word, past the caches.  A flag release that let one of those loads see
// another rank's stale acc or D was preceded by a broken word, and shows
// here; lane 0 then records the step's sequence number (the first poisoned
// step's is kept: later steps' checks run after this one on the same stream
// and find the word set).  One wave per step: the check once per wave of
// kernel B cost a PCIe read per wave, ~100 k small reads per step, and made
// kernel B 40x slower (profiles/r06/rehearse_perrank_n2_wave_check.log).
__global__ __launch_bounds__(64) void peer_poison_check_kernel(const uint64_t *broken, int64_t stride, int G,
                                                               uint64_t *poison, uint64_t seq) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t v = 0;
  if (lane < (uint32_t)G)
    v = __hip_atomic_load(const_cast<uint64_t *>(broken) + (int64_t)lane * stride, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_SYSTEM);
  if (__builtin_amdgcn_ballot_w64(v != 0) != 0 && lane == 0 &&
      __hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
    __hip_atomic_store(poison, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Replica optimiser step (clib-multigpu/kernels/optimisers/sma.cu:3-100).  The
// reference issues up to 6 full-model ops per task (saxpy wd, sscal, saxpy mu,
// copy last, copy diff, saxpy); here one pass reads w, g (, last) once and
// writes g, s, w (, last) once:  (20 + 8m) n bytes, or 16n (+4n if wd > 0)
// without momentum.  Per element, in the reference's order and rounding:
//   g = fma(wd, w, g)                    :24-31 (wd > 0)
//   g = rate * g ; g = fma(mu, last, g)  :52-64 ; last = g  :68
//   s = w                                :71 / :87
//   w = fma(1, g, w)  or  fma(rate, g, w) without momentum  :74 / :90
// ---------------------------------------------------------------------------
template <bool MOM, bool WD, int P, bool TAIL, int U>
__global__ __launch_bounds__(512) void sma_optimise_kernel(const OptArgs a) {
  if constexpr (TAIL) {
    if (blockIdx.x < (uint32_t)a.tail_blocks) {  // the caller's last elements (see sma_tail_elem)
      const int64_t i = a.tail_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
      if (i >= a.tail_hi) return;
      float *w = reinterpret_cast<float *>(a.w), *g = reinterpret_cast<float *>(a.g);
      const float wv = w[i];
      float gv = g[i];
      if constexpr (WD) gv = fmaf(a.wd, wv, gv);  // sma.cu:24-31
      reinterpret_cast<float *>(a.s)[i] = wv;     // :71 / :87
      if constexpr (MOM) {
        float *last = reinterpret_cast<float *>(a.last);
        gv = a.rate * gv;                  // :52-56
        gv = fmaf(a.momentum, last[i], gv);  // :59-64
        last[i] = gv;                      // :68
        w[i] = fmaf(1.0f, gv, wv);         // :74
        g[i] = gv;
      } else {
        w[i] = fmaf(a.rate, gv, wv);  // :90
        if constexpr (WD) g[i] = gv;
      }
      return;
    }
  }
  const uint32_t tb = TAIL ? (uint32_t)a.tail_blocks : 0u;
  const uint32_t trip = (gridDim.x - tb) * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f rate = a.rate, mu = a.momentum, wd = a.wd, one = 1.0f;
  for (uint32_t base = first_elem<U>(blockIdx.x - tb); base < n4; base += trip) {
    v4f w[U], g[U], l[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      w[u] = ldo<P>(a.w, i);
      g[u] = ldo<P>(a.g, i);
      if constexpr (MOM) l[u] = ldo<P>(a.last, i);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      if constexpr (WD) g[u] = vfma(wd, w[u], g[u]);
      sto<P>(a.s, i, w[u]);
      if constexpr (MOM) {
        g[u] = rate * g[u];
        g[u] = vfma(mu, l[u], g[u]);
        sto<P>(a.last, i, g[u]);
        sto<P>(a.w, i, vfma(one, g[u], w[u]));
        sto<P>(a.g, i, g[u]);
      } else {
        sto<P>(a.w, i, vfma(rate, g[u], w[u]));
        if constexpr (WD) sto<P>(a.g, i, g[u]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// DEFAULT task step (kernels/optimisers/default.cu:3-131): the reference runs
// up to 5 replica ops on the task stream and one base-model saxpy on the sync
// stream; here one pass reads w, g (, last), z once and writes them once.
//   g = fma(wd, w, g)                            :26-35 (wd > 0)
//   g = rate * g ; g = fma(mu, last, g); last = g :46-73
//   w = fma(1, g, w) ; z = fma(1, g, z)           :75-94
//   without momentum: w = fma(rate, g, w) ; z = fma(rate, g, z)   :102-125
// ---------------------------------------------------------------------------
template <bool MOM, bool WD, int P, int U>
__global__ __launch_bounds__(512) void default_optimise_kernel(const OptArgs a) {
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f rate = a.rate, mu = a.momentum, wd = a.wd, one = 1.0f;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    v4f w[U], g[U], l[U], z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      w[u] = ldo<P>(a.w, i);
      g[u] = ldo<P>(a.g, i);
      if constexpr (MOM) l[u] = ldo<P>(a.last, i);
      z[u] = ldo<P>(a.z, i);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      if constexpr (WD) g[u] = vfma(wd, w[u], g[u]);
      if constexpr (MOM) {
        g[u] = rate * g[u];
        g[u] = vfma(mu, l[u], g[u]);
        sto<P>(a.last, i, g[u]);
        sto<P>(a.w, i, vfma(one, g[u], w[u]));
        sto<P>(a.z, i, vfma(one, g[u], z[u]));
        sto<P>(a.g, i, g[u]);
      } else {
        sto<P>(a.w, i, vfma(rate, g[u], w[u]));
        sto<P>(a.z, i, vfma(rate, g[u], z[u]));
        if constexpr (WD) sto<P>(a.g, i, g[u]);
      }
    }
  }
}

// DEFAULT barrier (synch/default.c:19-37): the reference issues one D2D copy
// per locked replica (8n B each); here z is read once: (4 + 4R) n B.
template <int P, int U>
__global__ __launch_bounds__(512) void broadcast_kernel(const SmaArgs a) {
  const uint32_t trip = gridDim.x * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  for (uint32_t base = first_elem<U>(); base < n4; base += trip) {
    v4f z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) z[u] = ldo<P>(a.z, (base + u * 64u) * 16u);
    for (int r = 0; r < a.nrep; ++r) {
#pragma unroll
      for (int u = 0; u < U; ++u) sto<P>(a.w[r], (base + u * 64u) * 16u, z[u]);
    }
  }
}

// ---------------------------------------------------------------------------
// Synchronous SGD (WORKER).  Task step, on the sync stream so replicas add
// into the device's one accumulator in enqueue order (synchronoussgd.cu:3-56):
//   g = fma(wd, w, g)        :20-26 (wd > 0; g written back)
//   acc = fma(rate, g, acc)  :46-52
// Reads g, acc (, w) and writes acc (, g): 12n B (+8n with weight decay).
// ---------------------------------------------------------------------------
template <bool WD, int P, bool TAIL, int U>
__global__ __launch_bounds__(512) void ssgd_accumulate_kernel(const SsgdArgs a) {
  if constexpr (TAIL) {
    if (blockIdx.x < (uint32_t)a.tail_blocks) {  // the caller's last elements (see sma_tail_elem)
      const int64_t i = a.tail_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
      if (i >= a.tail_hi) return;
      float *g = reinterpret_cast<float *>(a.g), *acc = reinterpret_cast<float *>(a.acc);
      float gv = g[i];
      if constexpr (WD) {
        gv = fmaf(a.wd, reinterpret_cast<const float *>(a.wsrc)[i], gv);  // synchronoussgd.cu:20-26
        g[i] = gv;
      }
      acc[i] = fmaf(a.rate, gv, acc[i]);  // :46-52
      return;
    }
  }
  const uint32_t tb = TAIL ? (uint32_t)a.tail_blocks : 0u;
  const uint32_t trip = (gridDim.x - tb) * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f rate = a.rate, wd = a.wd;
  for (uint32_t base = first_elem<U>(blockIdx.x - tb); base < n4; base += trip) {
    v4f g[U], acc[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      g[u] = ldo<P>(a.g, i);
      acc[u] = ldo<P>(a.acc, i);
      if constexpr (WD) w[u] = ldo<P>(a.wsrc, i);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      if constexpr (WD) {
        g[u] = vfma(wd, w[u], g[u]);
        sto<P>(a.g, i, g[u]);
      }
      sto<P>(a.acc, i, vfma(rate, g[u], acc[u]));
    }
  }
}

// S-SGD barrier, per device after the all-reduce (synchronoussgd.c:13-106):
//   D = ratio * D                     :55-62 (sscal, ratio = 1/wpc)
//   D = fma(mu, last, D); last = D    :64-76 (base momentum, NOT forced to 0.9)
//   z = fma(1, D, z)                  :79-84
//   acc = 0                           :103
//   w_i = z for locked replicas       common.c:198-220
// Reads D, z (, last) and writes z, acc, R x w (, last).
template <bool MOM, int P, bool TAIL, int U>
__global__ __launch_bounds__(512) void ssgd_apply_kernel(const SsgdArgs a) {
  if constexpr (TAIL) {
    if (blockIdx.x < (uint32_t)a.tail_blocks) {  // the caller's last elements (see sma_tail_elem)
      const int64_t i = a.tail_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
      if (i >= a.tail_hi) return;
      float *z = reinterpret_cast<float *>(a.z);
      float D = a.ratio * reinterpret_cast<const float *>(a.D)[i];  // synchronoussgd.c:55-62
      if constexpr (MOM) {
        float *last = reinterpret_cast<float *>(a.last);
        D = fmaf(a.momentum, last[i], D);  // :64-76
        last[i] = D;
      }
      const float zv = fmaf(1.0f, D, z[i]);  // :79-84
      z[i] = zv;
      reinterpret_cast<float *>(a.acc)[i] = 0.0f;  // :103
      for (int r = 0; r < a.nrep; ++r) reinterpret_cast<float *>(a.w[r])[i] = zv;  // common.c:198-220
      return;
    }
  }
  const uint32_t tb = TAIL ? (uint32_t)a.tail_blocks : 0u;
  const uint32_t trip = (gridDim.x - tb) * blockDim.x * U;
  const uint32_t n4 = (uint32_t)a.n4;
  const v4f ratio = a.ratio, mu = a.momentum, one = 1.0f, zero = 0.0f;
  for (uint32_t base = first_elem<U>(blockIdx.x - tb); base < n4; base += trip) {
    v4f D[U], z[U], l[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      D[u] = ldo<P>(a.D, i);
      z[u] = ldo<P>(a.z, i);
      if constexpr (MOM) l[u] = ldo<P>(a.last, i);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = (base + u * 64u) * 16u;
      D[u] = ratio * D[u];
      if constexpr (MOM) {
        D[u] = vfma(mu, l[u], D[u]);
        sto<P>(a.last, i, D[u]);
      }
      z[u] = vfma(one, D[u], z[u]);
      sto<P>(a.z, i, z[u]);
      sto<P>(a.acc, i, zero);
    }
    for (int r = 0; r < a.nrep; ++r) {
#pragma unroll
      for (int u = 0; u < U; ++u) sto<P>(a.w[r], (base + u * 64u) * 16u, z[u]);
    }
  }
}

// ---------------------------------------------------------------------------
// Batch-norm statistics averaging: pack -> (RCCL sum) -> unpack.  Small,
// latency-bound buffers (one block row per segment); blockIdx.y = segment.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_pack_kernel(const BnSegment *segs, float *scratch) {
  const BnSegment sg = segs[blockIdx.y];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // A device that does not count contributes an exact +0 without its
  // statistics being read: the reference never touches a non-updated
  // device's buffers (cudnnbatchnormparams.c:177-184), so a NaN or Inf left
  // in them must not reach the average (0 * Inf would be NaN).
  if (i < sg.len) scratch[sg.off + i] = sg.scale != 0.0f ? sg.ptr[i] : 0.0f;
  // A device's count for the layer, written once (by its mean segment's first thread).
  if (i == 0 && (blockIdx.y & 1u) == 0) scratch[sg.layer] = sg.scale;
}

__global__ __launch_bounds__(256) void bn_unpack_kernel(const BnSegment *segs, const float *scratch) {
  const BnSegment sg = segs[blockIdx.y];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= sg.len) return;
  const float count = scratch[sg.layer];
  // cudnnbatchnormparams.c:192-197: ratio = 1. / (float) count, only if count > 1.
  const float ratio = count > 1.0f ? (float)(1.0 / (double)count) : 1.0f;
  sg.ptr[i] = ratio * scratch[sg.off + i];
}

// ---------------------------------------------------------------------------
// Synthetic inputs: splitmix64 -> Box-Muller in double.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_normal_kernel(float *out, int64_t n, uint64_t seed, float sigma,
                                                          const float *mean) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const uint64_t x = splitmix64(seed + (uint64_t)(2 * k) * 0x9E3779B97F4A7C15ULL);
    const uint64_t y = splitmix64(seed + (uint64_t)(2 * k + 1) * 0x9E3779B97F4A7C15ULL);
    const double u1 = (double)((x >> 11) + 1) * (1.0 / 9007199254740992.0);
    const double u2 = (double)(y >> 11) * (1.0 / 9007199254740992.0);
    const float v = (float)((double)sigma * (sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2)));
    out[k] = mean ? (mean[k] + v) : v;
  }
}

template <int P>
__global__ __launch_bounds__(512) void copy_kernel(v4f *dst, const v4f *src, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) st<P>(dst + i, ld<P>(src + i));
}

// Grid for a range of n4 float4s (a multiple of block*unroll).
inline dim3 grid_for(int64_t n4, const LaunchConfig &cfg) {
  const int64_t per_block = (int64_t)cfg.block * cfg.unroll;
  int64_t blocks = (n4 + per_block - 1) / per_block;
  if (cfg.blocks_per_cu > 0) {
    const int64_t cap = (int64_t)cfg.num_cus * cfg.blocks_per_cu;
    if (blocks > cap) blocks = cap;
  }
  if (blocks < 1) blocks = 1;
  return dim3((unsigned)blocks);
}

// Workgroups for a launch's tail elements (SmaArgs / OptArgs tail_lo..hi).
inline unsigned tail_blocks_for(int64_t lo, int64_t hi, int block) {
  return hi > lo ? (unsigned)((hi - lo + block - 1) / block) : 0u;
}

template <int R, bool MOM, bool COPY, int P>
hipError_t fused_u(const SmaArgs &a0, const LaunchConfig &cfg0, hipStream_t s, Timing t) {
  const LaunchConfig cfg = small_launch_shape(cfg0, a0.n4);
  dim3 g = grid_for(a0.n4, cfg);
  const unsigned lds = lds_for_occupancy(cfg, (COPY ? 1 : 2) * a0.nrep + 1 + (MOM ? 1 : 0), a0.nrep + 1 + (MOM ? 1 : 0), g.x);
  if (a0.tail_hi > a0.tail_lo) {  // caller-owned buffers: the tail rides the same launch
    if constexpr (P != 1) {
      return hipErrorInvalidValue;
    } else {
      SmaArgs a = a0;
      a.tail_blocks = (int)tail_blocks_for(a.tail_lo, a.tail_hi, cfg.block);
      g.x += (unsigned)a.tail_blocks;
      if (cfg.unroll == 2)
        hipExtLaunchKernelGGL((sma_fused_kernel<R, MOM, COPY, P, true, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
      else if (cfg.unroll == 1)
        hipExtLaunchKernelGGL((sma_fused_kernel<R, MOM, COPY, P, true, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
      else
        return hipErrorInvalidValue;
      return hipGetLastError();
    }
  }
  const SmaArgs &a = a0;
  if (cfg.unroll == 4)
    hipExtLaunchKernelGGL((sma_fused_kernel<R, MOM, COPY, P, false, 4>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  else if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_fused_kernel<R, MOM, COPY, P, false, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_fused_kernel<R, MOM, COPY, P, false, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  return hipGetLastError();
}

template <bool MOM, bool COPY, int P>
hipError_t fused_r(const SmaArgs &a, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  switch (a.nrep) {
    case 0: return fused_u<0, MOM, COPY, P>(a, cfg, s, t);
    case 1: return fused_u<1, MOM, COPY, P>(a, cfg, s, t);
    case 2: return fused_u<2, MOM, COPY, P>(a, cfg, s, t);
    case 3: return fused_u<3, MOM, COPY, P>(a, cfg, s, t);
    case 4: return fused_u<4, MOM, COPY, P>(a, cfg, s, t);
    case 5: return fused_u<5, MOM, COPY, P>(a, cfg, s, t);
    case 6: return fused_u<6, MOM, COPY, P>(a, cfg, s, t);
    case 7: return fused_u<7, MOM, COPY, P>(a, cfg, s, t);
    case 8: return fused_u<8, MOM, COPY, P>(a, cfg, s, t);
    default: return fused_u<-1, MOM, COPY, P>(a, cfg, s, t);
  }
}

template <int R, int P>
hipError_t acc_u(const SmaArgs &a0, const LaunchConfig &cfg0, hipStream_t s, Timing t) {
  const LaunchConfig cfg = small_launch_shape(cfg0, a0.n4);
  dim3 g = grid_for(a0.n4, cfg);
  const unsigned lds = lds_for_occupancy(cfg, 2 * a0.nrep + 1, a0.nrep + 1, g.x);
  if (a0.tail_hi > a0.tail_lo) {
    if constexpr (P != 1) {
      return hipErrorInvalidValue;
    } else {
      SmaArgs a = a0;
      a.tail_blocks = (int)tail_blocks_for(a.tail_lo, a.tail_hi, cfg.block);
      g.x += (unsigned)a.tail_blocks;
      if (cfg.unroll == 2)
        hipExtLaunchKernelGGL((sma_accumulate_kernel<R, P, true, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
      else if (cfg.unroll == 1)
        hipExtLaunchKernelGGL((sma_accumulate_kernel<R, P, true, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
      else
        return hipErrorInvalidValue;
      return hipGetLastError();
    }
  }
  const SmaArgs &a = a0;
  if (cfg.unroll == 4)
    hipExtLaunchKernelGGL((sma_accumulate_kernel<R, P, false, 4>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  else if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_accumulate_kernel<R, P, false, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_accumulate_kernel<R, P, false, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  return hipGetLastError();
}

template <int P>
hipError_t acc_r(const SmaArgs &a, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  switch (a.nrep) {
    case 0: return acc_u<0, P>(a, cfg, s, t);
    case 1: return acc_u<1, P>(a, cfg, s, t);
    case 2: return acc_u<2, P>(a, cfg, s, t);
    case 3: return acc_u<3, P>(a, cfg, s, t);
    case 4: return acc_u<4, P>(a, cfg, s, t);
    case 5: return acc_u<5, P>(a, cfg, s, t);
    case 6: return acc_u<6, P>(a, cfg, s, t);
    case 7: return acc_u<7, P>(a, cfg, s, t);
    case 8: return acc_u<8, P>(a, cfg, s, t);
    default: return acc_u<-1, P>(a, cfg, s, t);
  }
}

template <bool MOM, int P>
hipError_t apply_u(const SmaArgs &a0, const LaunchConfig &cfg0, hipStream_t s, Timing t) {
  const LaunchConfig cfg = small_launch_shape(cfg0, a0.n4);
  dim3 g = grid_for(a0.n4, cfg);
  const unsigned lds = lds_for_occupancy(cfg, MOM ? 3 : 2, MOM ? 2 : 1, g.x);
  if (a0.tail_hi > a0.tail_lo) {
    if constexpr (P != 1) {
      return hipErrorInvalidValue;
    } else {
      SmaArgs a = a0;
      a.tail_blocks = (int)tail_blocks_for(a.tail_lo, a.tail_hi, cfg.block);
      g.x += (unsigned)a.tail_blocks;
      if (cfg.unroll == 2)
        hipExtLaunchKernelGGL((sma_apply_kernel<MOM, P, true, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
      else if (cfg.unroll == 1)
        hipExtLaunchKernelGGL((sma_apply_kernel<MOM, P, true, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
      else
        return hipErrorInvalidValue;
      return hipGetLastError();
    }
  }
  const SmaArgs &a = a0;
  if (cfg.unroll == 4)
    hipExtLaunchKernelGGL((sma_apply_kernel<MOM, P, false, 4>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  else if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_apply_kernel<MOM, P, false, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_apply_kernel<MOM, P, false, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a);
  return hipGetLastError();
}

template <int G_, int P>
hipError_t peer_reduce_g(const PeerArgs &p, const LaunchConfig &cfg0, hipStream_t s, Timing t) {
  const LaunchConfig cfg = small_launch_shape(cfg0, p.n4);
  const dim3 g = grid_for(p.n4, cfg);
  const unsigned lds = lds_for_occupancy(cfg, p.G, 1, g.x);
  if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_peer_reduce_kernel<G_, P, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, p);
  else
    hipExtLaunchKernelGGL((sma_peer_reduce_kernel<G_, P, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, p);
  return hipGetLastError();
}

template <int P>
hipError_t peer_reduce_p(const PeerArgs &p, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  switch (p.G) {
    case 2: return peer_reduce_g<2, P>(p, cfg, s, t);
    case 4: return peer_reduce_g<4, P>(p, cfg, s, t);
    case 8: return peer_reduce_g<8, P>(p, cfg, s, t);
    default: return peer_reduce_g<-1, P>(p, cfg, s, t);
  }
}

template <bool MOM, int P>
hipError_t peer_apply_u(const SmaArgs &a, const PeerArgs &p, const LaunchConfig &cfg0, hipStream_t s, Timing t) {
  const LaunchConfig cfg = small_launch_shape(cfg0, a.n4);
  const dim3 g = grid_for(a.n4, cfg);
  const unsigned lds = lds_for_occupancy(cfg, MOM ? 3 : 2, MOM ? 2 : 1, g.x);
  if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_peer_apply_kernel<MOM, P, 2>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a, p);
  else
    hipExtLaunchKernelGGL((sma_peer_apply_kernel<MOM, P, 1>), g, dim3(cfg.block), lds, s, t.start, t.stop, 0, a, p);
  return hipGetLastError();
}

// Zero-copy staged launches: PCIe-bound, so no occupancy cap (the cap keeps
// DRAM pages few for the HBM-bound kernels; here the link is the limit and
// more waves keep more host reads in flight).
template <int R, bool MOM, bool COPY>
hipError_t fused_staged_u(const StagedArgs &a, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  const dim3 g = grid_for(a.n4, cfg);
  if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_fused_staged_kernel<R, MOM, COPY, 2>), g, dim3(cfg.block), 0, s, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_fused_staged_kernel<R, MOM, COPY, 1>), g, dim3(cfg.block), 0, s, t.start, t.stop, 0, a);
  return hipGetLastError();
}

template <bool MOM, bool COPY>
hipError_t fused_staged_r(const StagedArgs &a, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  switch (a.nrep) {
    case 0: return fused_staged_u<0, MOM, COPY>(a, cfg, s, t);
    case 1: return fused_staged_u<1, MOM, COPY>(a, cfg, s, t);
    case 2: return fused_staged_u<2, MOM, COPY>(a, cfg, s, t);
    case 4: return fused_staged_u<4, MOM, COPY>(a, cfg, s, t);
    case 8: return fused_staged_u<8, MOM, COPY>(a, cfg, s, t);
    default: return fused_staged_u<-1, MOM, COPY>(a, cfg, s, t);
  }
}

template <int R>
hipError_t acc_staged_u(const StagedArgs &a, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  const dim3 g = grid_for(a.n4, cfg);
  if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_accumulate_staged_kernel<R, 2>), g, dim3(cfg.block), 0, s, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_accumulate_staged_kernel<R, 1>), g, dim3(cfg.block), 0, s, t.start, t.stop, 0, a);
  return hipGetLastError();
}

template <bool MOM>
hipError_t apply_staged_u(const StagedArgs &a, const LaunchConfig &cfg, hipStream_t s, Timing t) {
  const dim3 g = grid_for(a.n4, cfg);
  if (cfg.unroll == 2)
    hipExtLaunchKernelGGL((sma_apply_staged_kernel<MOM, 2>), g, dim3(cfg.block), 0, s, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_apply_staged_kernel<MOM, 1>), g, dim3(cfg.block), 0, s, t.start, t.stop, 0, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_sma_fused_staged(const StagedArgs &a, bool momentum, bool copy, const LaunchConfig &cfg,
                                   hipStream_t stream, Timing t) {
  if (momentum) return copy ? fused_staged_r<true, true>(a, cfg, stream, t) : fused_staged_r<true, false>(a, cfg, stream, t);
  return copy ? fused_staged_r<false, true>(a, cfg, stream, t) : fused_staged_r<false, false>(a, cfg, stream, t);
}

hipError_t launch_sma_accumulate_staged(const StagedArgs &a, bool write_ctrl, const LaunchConfig &cfg,
                                        hipStream_t stream, Timing t) {
  StagedArgs b = a;
  if (!write_ctrl) b.ctrl_out = nullptr;
  switch (b.nrep) {
    case 0: return acc_staged_u<0>(b, cfg, stream, t);
    case 1: return acc_staged_u<1>(b, cfg, stream, t);
    case 2: return acc_staged_u<2>(b, cfg, stream, t);
    case 4: return acc_staged_u<4>(b, cfg, stream, t);
    case 8: return acc_staged_u<8>(b, cfg, stream, t);
    default: return acc_staged_u<-1>(b, cfg, stream, t);
  }
}

hipError_t launch_sma_apply_staged(const StagedArgs &a, bool momentum, const LaunchConfig &cfg, hipStream_t stream,
                                   Timing t) {
  return momentum ? apply_staged_u<true>(a, cfg, stream, t) : apply_staged_u<false>(a, cfg, stream, t);
}

hipError_t launch_sma_peer_reduce(const PeerArgs &p, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  if (p.G < 1 || p.G > kMaxDevices) return hipErrorInvalidValue;
  return cfg.policy == 1 ? peer_reduce_p<1>(p, cfg, stream, t) : peer_reduce_p<0>(p, cfg, stream, t);
}

hipError_t launch_sma_peer_apply(const SmaArgs &a, const PeerArgs &p, bool momentum, const LaunchConfig &cfg,
                                 hipStream_t stream, Timing t) {
  if (p.G < 1 || p.G > kMaxDevices || p.shard4 <= 0 || p.shard4 % kPadFloat4 != 0) return hipErrorInvalidValue;
  if (cfg.policy == 1)
    return momentum ? peer_apply_u<true, 1>(a, p, cfg, stream, t) : peer_apply_u<false, 1>(a, p, cfg, stream, t);
  return momentum ? peer_apply_u<true, 0>(a, p, cfg, stream, t) : peer_apply_u<false, 0>(a, p, cfg, stream, t);
}

hipError_t launch_peer_poison_check(const uint64_t *broken, int64_t stride, int G, uint64_t *poison, uint64_t seq,
                                    hipStream_t stream) {
  if (!broken || !poison || G < 1 || G > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_poison_check_kernel, dim3(1), dim3(64), 0, stream, broken, stride, G, poison, seq);
  return hipGetLastError();
}

hipError_t launch_sma_fused(const SmaArgs &a, bool momentum, bool copy, const LaunchConfig &cfg,
                            hipStream_t stream, Timing t) {
  if (cfg.policy == 1) {
    if (momentum) return copy ? fused_r<true, true, 1>(a, cfg, stream, t) : fused_r<true, false, 1>(a, cfg, stream, t);
    return copy ? fused_r<false, true, 1>(a, cfg, stream, t) : fused_r<false, false, 1>(a, cfg, stream, t);
  }
  if (momentum) return copy ? fused_r<true, true, 0>(a, cfg, stream, t) : fused_r<true, false, 0>(a, cfg, stream, t);
  return copy ? fused_r<false, true, 0>(a, cfg, stream, t) : fused_r<false, false, 0>(a, cfg, stream, t);
}

hipError_t launch_sma_accumulate(const SmaArgs &a, bool write_ctrl, const LaunchConfig &cfg,
                                 hipStream_t stream, Timing t) {
  SmaArgs b = a;
  if (!write_ctrl) b.ctrl_out = nullptr;
  return cfg.policy == 1 ? acc_r<1>(b, cfg, stream, t) : acc_r<0>(b, cfg, stream, t);
}

hipError_t launch_sma_apply(const SmaArgs &a, bool momentum, const LaunchConfig &cfg, hipStream_t stream,
                            Timing t) {
  if (cfg.policy == 1) return momentum ? apply_u<true, 1>(a, cfg, stream, t) : apply_u<false, 1>(a, cfg, stream, t);
  return momentum ? apply_u<true, 0>(a, cfg, stream, t) : apply_u<false, 0>(a, cfg, stream, t);
}

// An empty one-wave kernel whose dispatch timestamps mark a point on a stream
// (the stream-order check's collective start / end, cbx_set_order_check):
// unlike an event record, a dispatch after a stream wait is timestamped when
// it really runs.
__global__ void order_probe_kernel() {}

hipError_t launch_order_probe(hipStream_t stream, Timing t) {
  hipExtLaunchKernelGGL(order_probe_kernel, dim3(1), dim3(64), 0, stream, t.start, t.stop, 0);
  return hipGetLastError();
}

// One wave that idles for `ticks` of the constant-rate wall clock (fault
// injection only: it holds back the kernel queued behind it on its stream, so
// a race the injected fault opens is certain rather than timing-dependent).
// No memory is touched; the loop is bounded whatever the clock does.
__global__ void delay_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < (1 << 20) && wall_clock64() - t0 < ticks; ++i) __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_delay(hipStream_t stream, uint64_t ticks) {
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, stream, ticks);
  return hipGetLastError();
}

hipError_t launch_sma_shard_momentum(const SmaArgs &a, const LaunchConfig &cfg0, hipStream_t stream, Timing t) {
  LaunchConfig cfg = cfg0;
  cfg.unroll = 1;
  const dim3 g = grid_for(a.n4, cfg);
  const unsigned lds = lds_for_occupancy(cfg, 2, 1, g.x);
  if (cfg.policy == 1)
    hipExtLaunchKernelGGL((sma_shard_momentum_kernel<1>), g, dim3(cfg.block), lds, stream, t.start, t.stop, 0, a);
  else
    hipExtLaunchKernelGGL((sma_shard_momentum_kernel<0>), g, dim3(cfg.block), lds, stream, t.start, t.stop, 0, a);
  return hipGetLastError();
}

// Launch `K<..., U>` for the configured unroll (1 or 2) with the occupancy
// cap for `reads` + `writes` buffer streams.
#define CBX_LAUNCH_U(KERNEL, ...)                                                                        \
  do {                                                                                                   \
    const dim3 g_ = grid_for(a.n4, cfg);                                                                 \
    const unsigned l_ = lds_for_occupancy(cfg, reads, writes, g_.x);                                             \
    if (cfg.unroll == 2)                                                                                 \
      hipExtLaunchKernelGGL((KERNEL<__VA_ARGS__, 2>), g_, dim3(cfg.block), l_, stream, t.start, t.stop, 0, a); \
    else                                                                                                 \
      hipExtLaunchKernelGGL((KERNEL<__VA_ARGS__, 1>), g_, dim3(cfg.block), l_, stream, t.start, t.stop, 0, a); \
  } while (0)

template <bool MOM, bool WD, int P>
hipError_t optimise_p(const OptArgs &a0, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const int reads = 2 + (MOM ? 1 : 0), writes = MOM ? 4 : (WD ? 3 : 2);
  if (a0.tail_hi > a0.tail_lo) {  // caller-owned buffers: the tail rides the same launch
    if constexpr (P != 1) {
      return hipErrorInvalidValue;
    } else {
      OptArgs a = a0;
      dim3 g = grid_for(a.n4, cfg);
      const unsigned l = lds_for_occupancy(cfg, reads, writes, g.x);
      a.tail_blocks = (int)tail_blocks_for(a.tail_lo, a.tail_hi, cfg.block);
      g.x += (unsigned)a.tail_blocks;
      if (cfg.unroll == 2)
        hipExtLaunchKernelGGL((sma_optimise_kernel<MOM, WD, P, true, 2>), g, dim3(cfg.block), l, stream, t.start, t.stop, 0, a);
      else if (cfg.unroll == 1)
        hipExtLaunchKernelGGL((sma_optimise_kernel<MOM, WD, P, true, 1>), g, dim3(cfg.block), l, stream, t.start, t.stop, 0, a);
      else
        return hipErrorInvalidValue;
      return hipGetLastError();
    }
  }
  const OptArgs &a = a0;
  CBX_LAUNCH_U(sma_optimise_kernel, MOM, WD, P, false);
  return hipGetLastError();
}

hipError_t launch_sma_optimise(const OptArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const bool mom = a.momentum > 0.0f, wd = a.wd > 0.0f;
  if (cfg.policy == 1) {
    if (mom) return wd ? optimise_p<true, true, 1>(a, cfg, stream, t) : optimise_p<true, false, 1>(a, cfg, stream, t);
    return wd ? optimise_p<false, true, 1>(a, cfg, stream, t) : optimise_p<false, false, 1>(a, cfg, stream, t);
  }
  if (mom) return wd ? optimise_p<true, true, 0>(a, cfg, stream, t) : optimise_p<true, false, 0>(a, cfg, stream, t);
  return wd ? optimise_p<false, true, 0>(a, cfg, stream, t) : optimise_p<false, false, 0>(a, cfg, stream, t);
}

template <bool MOM, bool WD, int P>
hipError_t default_p(const OptArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const int reads = 3 + (MOM ? 1 : 0), writes = 2 + (MOM ? 2 : (WD ? 1 : 0));
  CBX_LAUNCH_U(default_optimise_kernel, MOM, WD, P);
  return hipGetLastError();
}

hipError_t launch_default_optimise(const OptArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const bool mom = a.momentum > 0.0f, wd = a.wd > 0.0f;
  if (cfg.policy == 1) {
    if (mom) return wd ? default_p<true, true, 1>(a, cfg, stream, t) : default_p<true, false, 1>(a, cfg, stream, t);
    return wd ? default_p<false, true, 1>(a, cfg, stream, t) : default_p<false, false, 1>(a, cfg, stream, t);
  }
  if (mom) return wd ? default_p<true, true, 0>(a, cfg, stream, t) : default_p<true, false, 0>(a, cfg, stream, t);
  return wd ? default_p<false, true, 0>(a, cfg, stream, t) : default_p<false, false, 0>(a, cfg, stream, t);
}

template <int P>
hipError_t broadcast_p(const SmaArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const int reads = 1, writes = a.nrep;
  CBX_LAUNCH_U(broadcast_kernel, P);
  return hipGetLastError();
}

hipError_t launch_broadcast(const SmaArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  return cfg.policy == 1 ? broadcast_p<1>(a, cfg, stream, t) : broadcast_p<0>(a, cfg, stream, t);
}

// Launch KERNEL<..., TAIL = true, U> with the launch's tail workgroups in
// front (caller-owned buffers: a.tail_lo .. a.tail_hi); policy 1, unroll 1 or 2.
#define CBX_LAUNCH_TAIL(KERNEL, ...)                                                                     \
  do {                                                                                                   \
    if constexpr (P != 1) {                                                                              \
      return hipErrorInvalidValue;                                                                       \
    } else {                                                                                             \
      auto a = a0;                                                                                       \
      dim3 g_ = grid_for(a.n4, cfg);                                                                     \
      const unsigned l_ = lds_for_occupancy(cfg, reads, writes, g_.x);                                   \
      a.tail_blocks = (int)tail_blocks_for(a.tail_lo, a.tail_hi, cfg.block);                             \
      g_.x += (unsigned)a.tail_blocks;                                                                   \
      if (cfg.unroll == 2)                                                                               \
        hipExtLaunchKernelGGL((KERNEL<__VA_ARGS__, true, 2>), g_, dim3(cfg.block), l_, stream, t.start, t.stop, 0, a); \
      else if (cfg.unroll == 1)                                                                          \
        hipExtLaunchKernelGGL((KERNEL<__VA_ARGS__, true, 1>), g_, dim3(cfg.block), l_, stream, t.start, t.stop, 0, a); \
      else                                                                                               \
        return hipErrorInvalidValue;                                                                     \
      return hipGetLastError();                                                                          \
    }                                                                                                    \
  } while (0)

template <bool WD, int P>
hipError_t ssgd_acc_p(const SsgdArgs &a0, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const int reads = 2 + (WD ? 1 : 0), writes = 1 + (WD ? 1 : 0);
  if (a0.tail_hi > a0.tail_lo) CBX_LAUNCH_TAIL(ssgd_accumulate_kernel, WD, P);
  const SsgdArgs &a = a0;
  CBX_LAUNCH_U(ssgd_accumulate_kernel, WD, P, false);
  return hipGetLastError();
}

hipError_t launch_ssgd_accumulate(const SsgdArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const bool wd = a.wd > 0.0f;
  if (cfg.policy == 1) return wd ? ssgd_acc_p<true, 1>(a, cfg, stream, t) : ssgd_acc_p<false, 1>(a, cfg, stream, t);
  return wd ? ssgd_acc_p<true, 0>(a, cfg, stream, t) : ssgd_acc_p<false, 0>(a, cfg, stream, t);
}

template <bool MOM, int P>
hipError_t ssgd_apply_p(const SsgdArgs &a0, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const int reads = 2 + (MOM ? 1 : 0), writes = 2 + (MOM ? 1 : 0) + a0.nrep;
  if (a0.tail_hi > a0.tail_lo) CBX_LAUNCH_TAIL(ssgd_apply_kernel, MOM, P);
  const SsgdArgs &a = a0;
  CBX_LAUNCH_U(ssgd_apply_kernel, MOM, P, false);
  return hipGetLastError();
}

hipError_t launch_ssgd_apply(const SsgdArgs &a, const LaunchConfig &cfg, hipStream_t stream, Timing t) {
  const bool mom = a.momentum > 0.0f;
  if (cfg.policy == 1) return mom ? ssgd_apply_p<true, 1>(a, cfg, stream, t) : ssgd_apply_p<false, 1>(a, cfg, stream, t);
  return mom ? ssgd_apply_p<true, 0>(a, cfg, stream, t) : ssgd_apply_p<false, 0>(a, cfg, stream, t);
}

#undef CBX_LAUNCH_U
#undef CBX_LAUNCH_TAIL

hipError_t launch_bn_pack(const BnSegment *segs, int nseg, uint32_t maxlen, float *scratch, hipStream_t stream) {
  if (nseg <= 0 || maxlen == 0) return hipSuccess;
  const dim3 g((maxlen + 255) / 256, (unsigned)nseg);
  hipLaunchKernelGGL(bn_pack_kernel, g, dim3(256), 0, stream, segs, scratch);
  return hipGetLastError();
}

hipError_t launch_bn_unpack(const BnSegment *segs, int nseg, uint32_t maxlen, const float *scratch,
                            hipStream_t stream) {
  if (nseg <= 0 || maxlen == 0) return hipSuccess;
  const dim3 g((maxlen + 255) / 256, (unsigned)nseg);
  hipLaunchKernelGGL(bn_unpack_kernel, g, dim3(256), 0, stream, segs, scratch);
  return hipGetLastError();
}

hipError_t launch_fill_normal(float *out, int64_t n, uint64_t seed, float sigma, const float *mean,
                              hipStream_t stream) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(fill_normal_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, out, n, seed, sigma, mean);
  return hipGetLastError();
}

hipError_t launch_copy(v4f *dst, const v4f *src, int64_t n4, const LaunchConfig &cfg, hipStream_t stream) {
  LaunchConfig c = cfg;
  c.unroll = 1;
  const dim3 g = grid_for(n4, c);
  if (cfg.policy == 1)
    hipLaunchKernelGGL((copy_kernel<1>), g, dim3(c.block), 0, stream, dst, src, n4);
  else
    hipLaunchKernelGGL((copy_kernel<0>), g, dim3(c.block), 0, stream, dst, src, n4);
  return hipGetLastError();
}

}  // namespace cbx
