// membench.hip -- exploration microbenchmark for the fused SMA kernel's
// memory shape on one MI355X (not part of the product library).
//
// Workload C3: n = 25,557,032 fp32, R = 8 replicas, momentum on:
// 18 read streams (z, last, 8 s, 8 w) and 10 write streams (8 w, z, last).
// Measures ceilings (copy, read-only, write-only) and fused-kernel variants
// over buffer layouts (arena stagger) and launch shapes.  Prints one JSON
// line per variant.  Build: hipcc --offload-arch=gfx950 -O3 -o membench membench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr int R = 8;

struct Args {
  const v4f *s[R];
  v4f *w[R];
  v4f *z;
  v4f *last;
  uint32_t n4;
  float alpha;
};

template <int P>
__device__ __forceinline__ v4f ld(const v4f *p) {
  if constexpr (P == 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int P>
__device__ __forceinline__ void st(v4f *p, v4f v) {
  if constexpr (P == 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ v4f vfma(v4f a, v4f b, v4f c) { return __builtin_elementwise_fma(a, b, c); }

// PL / PS: load / store policy (0 plain, 1 nontemporal).
// ORDER 0: all s, all w loads first.  ORDER 1: s_i, w_i interleaved.
// ORDER 2: per replica load-compute-store.
// WC: wave-contiguous (lane l of a wave handles float4s wbase + l + 64u, so a
// wave touches 64*U*16 contiguous bytes per stream) instead of block-strided.
template <int PL, int PS, int ORDER, int U, bool WC>
__global__ __launch_bounds__(1024) void fused(const Args a) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t stride_u = WC ? 64u : blockDim.x;
  const uint32_t first = WC ? (blockIdx.x * blockDim.x * U + wave * 64u * U + lane)
                            : (blockIdx.x * blockDim.x * U + threadIdx.x);
  const v4f al = a.alpha, nal = -a.alpha, mb = 0.9f, one = 1.0f, mone = -1.0f;
  const uint32_t base = first;
  if (base >= a.n4) return;
  v4f zv[U], lv[U], acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t i = base + u * stride_u;
    zv[u] = ld<PL>(a.z + i);
    lv[u] = ld<PL>(a.last + i);
    acc[u] = 0.0f;
  }
  if constexpr (ORDER == 2) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * stride_u;
        v4f s = ld<PL>(a.s[r] + i), w = ld<PL>(a.w[r] + i);
        v4f d = vfma(mone, zv[u], s);
        st<PS>(a.w[r] + i, vfma(nal, d, w));
        acc[u] = vfma(al, d, acc[u]);
      }
    }
  } else {
    v4f sv[U][R], wv[U][R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * stride_u;
        sv[u][r] = ld<PL>(a.s[r] + i);
        if constexpr (ORDER == 1) wv[u][r] = ld<PL>(a.w[r] + i);
      }
    }
    if constexpr (ORDER == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) wv[u][r] = ld<PL>(a.w[r] + base + u * stride_u);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v4f d = vfma(mone, zv[u], sv[u][r]);
        wv[u][r] = vfma(nal, d, wv[u][r]);
        acc[u] = vfma(al, d, acc[u]);
      }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) st<PS>(a.w[r] + base + u * stride_u, wv[u][r]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t i = base + u * stride_u;
    v4f D = vfma(mb, lv[u], acc[u]);
    st<PS>(a.last + i, D);
    st<PS>(a.z + i, vfma(one, D, zv[u]));
  }
}

template <int P>
__global__ __launch_bounds__(1024) void copyk(v4f *dst, const v4f *src, uint32_t n4) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) st<P>(dst + i, ld<P>(src + i));
}

// Read-only: 18 streams, one float4 each per thread (one trip).
template <int P>
__global__ __launch_bounds__(1024) void readk(const Args a, float *sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n4) return;
  v4f t = ld<P>(a.z + i) + ld<P>(a.last + i);
#pragma unroll
  for (int r = 0; r < R; ++r) t += ld<P>(a.s[r] + i) + ld<P>(a.w[r] + i);
  if (t.x == 12345.678f) sink[0] = t.y;
}

// Write-only: 10 streams, one trip.
template <int P>
__global__ __launch_bounds__(1024) void writek(const Args a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n4) return;
  const v4f v = (float)i;
  st<P>(a.z + i, v);
  st<P>(a.last + i, v);
#pragma unroll
  for (int r = 0; r < R; ++r) st<P>(a.w[r] + i, v);
}


// ---- v3: library-style kernel (SGPR base + 32-bit lane offset), min-waves
// hint MW (caps VGPRs), optional XCD-aware block remap, no-dependency mix.
template <int P>
__device__ __forceinline__ v4f ldo(const v4f *b, uint32_t off) {
  return ld<P>(reinterpret_cast<const v4f *>(reinterpret_cast<const char *>(b) + off));
}
template <int P>
__device__ __forceinline__ void sto(v4f *b, uint32_t off, v4f v) {
  st<P>(reinterpret_cast<v4f *>(reinterpret_cast<char *>(b) + off), v);
}
template <int MW, bool XCD, bool SB = false>
__global__ __launch_bounds__(256, MW) void fused3(const Args a) {
  uint32_t blk = blockIdx.x;
  if constexpr (XCD) {
    // blocks b, b+8, ... share an XCD: give each XCD one contiguous range.
    const uint32_t per = gridDim.x / 8, full = per * 8;
    if (blockIdx.x < full) blk = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  }
  const uint32_t e = blk * blockDim.x + threadIdx.x;
  if (e >= a.n4) return;
  const uint32_t i = e * 16u;
  const v4f al = a.alpha, nal = -a.alpha, mb = 0.9f, one = 1.0f, mone = -1.0f;
  v4f zv = ldo<1>(a.z, i), lv = ldo<1>(a.last, i), acc = 0.0f;
  v4f sv[R], wv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) sv[r] = ldo<1>(a.s[r], i);
#pragma unroll
  for (int r = 0; r < R; ++r) wv[r] = ldo<1>(a.w[r], i);
  if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    v4f d = vfma(mone, zv, sv[r]);
    wv[r] = vfma(nal, d, wv[r]);
    acc = vfma(al, d, acc);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) sto<1>(a.w[r], i, wv[r]);
  v4f D = vfma(mb, lv, acc);
  sto<1>(a.last, i, D);
  sto<1>(a.z, i, vfma(one, D, zv));
}

// Same memory shape, stores independent of loads (loads kept alive by a
// never-taken sink store): the DRAM read/write mix without the dependency.
__global__ __launch_bounds__(256) void mixnodep(const Args a, float *sink) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n4) return;
  const uint32_t i = e * 16u;
  const v4f v = (float)e;
  sto<1>(a.z, i, v);
  sto<1>(a.last, i, v);
#pragma unroll
  for (int r = 0; r < R; ++r) sto<1>(a.w[r], i, v);
  v4f t = ldo<1>(a.z, i + 0) ;
  t += ldo<1>(a.last, i);
#pragma unroll
  for (int r = 0; r < R; ++r) t += ldo<1>(a.s[r], i) + ldo<1>(a.w[r], i);
  if (t.x == 12345.678f) sink[0] = t.y;
}


__global__ void fillk(uint32_t *p, size_t nwords, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwords; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    float f = ((float)(x >> 8) * (1.0f / 16777216.0f) - 0.5f) * 0.1f;
    p[i] = __float_as_uint(f);
  }
}


// ---- v6: persistent, software-pipelined: the next element's 18 loads are
// issued before the current element's 10 stores.
__device__ __forceinline__ void load18(const Args &a, uint32_t i, v4f &z, v4f &l, v4f *sv, v4f *wv) {
  z = ldo<1>(a.z, i);
  l = ldo<1>(a.last, i);
#pragma unroll
  for (int r = 0; r < R; ++r) sv[r] = ldo<1>(a.s[r], i);
#pragma unroll
  for (int r = 0; r < R; ++r) wv[r] = ldo<1>(a.w[r], i);
}
__device__ __forceinline__ void comp_store(const Args &a, uint32_t i, v4f z, v4f l, v4f *sv, v4f *wv) {
  const v4f al = a.alpha, nal = -a.alpha, mb = 0.9f, one = 1.0f, mone = -1.0f;
  v4f acc = 0.0f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    v4f d = vfma(mone, z, sv[r]);
    wv[r] = vfma(nal, d, wv[r]);
    acc = vfma(al, d, acc);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) sto<1>(a.w[r], i, wv[r]);
  v4f D = vfma(mb, l, acc);
  sto<1>(a.last, i, D);
  sto<1>(a.z, i, vfma(one, D, z));
}
__global__ __launch_bounds__(256) void fused_pipe(const Args a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n4) return;
  v4f z0, l0, s0[R], w0[R];
  load18(a, e * 16u, z0, l0, s0, w0);
  while (true) {
    const uint32_t en = e + stride;
    if (en < a.n4) {
      v4f z1, l1, s1[R], w1[R];
      load18(a, en * 16u, z1, l1, s1, w1);
      __builtin_amdgcn_sched_barrier(0);
      comp_store(a, e * 16u, z0, l0, s0, w0);
      z0 = z1; l0 = l1;
#pragma unroll
      for (int r = 0; r < R; ++r) { s0[r] = s1[r]; w0[r] = w1[r]; }
      e = en;
    } else {
      comp_store(a, e * 16u, z0, l0, s0, w0);
      break;
    }
  }
}

// ---- v7: buffer_load/store through ONE descriptor over the arena, stream
// base in soffset, with explicit cache-policy bits (aux: sc0=1 nt=2 sc1=16).
typedef unsigned v4u __attribute__((ext_vector_type(4)));
struct BArgs {
  uint32_t off_s[R], off_w[R], off_z, off_last;
  uint32_t n4;
  float alpha;
};
template <int LA, int SA>
__global__ __launch_bounds__(128) void fused_buf(const BArgs a, char *arena, uint32_t bytes) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(arena, 0, bytes, 0x00020000);
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n4) return;
  const uint32_t i = e * 16u;
  auto L = [&](uint32_t so) { v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, i, so, LA); return __builtin_bit_cast(v4f, x); };
  auto S = [&](uint32_t so, v4f v) { __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rs, i, so, SA); };
  const v4f al = a.alpha, nal = -a.alpha, mb = 0.9f, one = 1.0f, mone = -1.0f;
  v4f zv = L(a.off_z), lv = L(a.off_last), acc = 0.0f;
  v4f sv[R], wv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) sv[r] = L(a.off_s[r]);
#pragma unroll
  for (int r = 0; r < R; ++r) wv[r] = L(a.off_w[r]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    v4f d = vfma(mone, zv, sv[r]);
    wv[r] = vfma(nal, d, wv[r]);
    acc = vfma(al, d, acc);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) S(a.off_w[r], wv[r]);
  v4f D = vfma(mb, lv, acc);
  S(a.off_last, D);
  S(a.off_z, vfma(one, D, zv));
}

// ---- v9: wave-contiguous U float4 per lane per stream (a wave covers
// U KiB of each stream), all loads in flight before the first FMA.
template <int U>
__global__ __launch_bounds__(256) void fused_wc(const Args a) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t e0 = (blockIdx.x * (blockDim.x >> 6) + wave) * 64u * U + lane;
  if (e0 >= a.n4) return;
  const v4f al = a.alpha, nal = -a.alpha, mb = 0.9f, one = 1.0f, mone = -1.0f;
  v4f zv[U], lv[U], sv[U][R], wv[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t i = (e0 + 64u * u) * 16u;
    zv[u] = ldo<1>(a.z, i);
    lv[u] = ldo<1>(a.last, i);
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u) sv[u][r] = ldo<1>(a.s[r], (e0 + 64u * u) * 16u);
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u) wv[u][r] = ldo<1>(a.w[r], (e0 + 64u * u) * 16u);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t i = (e0 + 64u * u) * 16u;
    v4f acc = 0.0f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v4f d = vfma(mone, zv[u], sv[u][r]);
      wv[u][r] = vfma(nal, d, wv[u][r]);
      acc = vfma(al, d, acc);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) sto<1>(a.w[r], i, wv[u][r]);
    v4f D = vfma(mb, lv[u], acc);
    sto<1>(a.last, i, D);
    sto<1>(a.z, i, vfma(one, D, zv[u]));
  }
}
static hipEvent_t e0, e1;

template <typename F>
static float time_ms(F launch, int iters) {
  for (int k = 0; k < 3; ++k) launch();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int k = 0; k < iters; ++k) {
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

// ---- v10: ceilings in the library's launch shape (64-thread blocks, U = 2
// wave-contiguous float4s per lane, nt) under the same dynamic-LDS occupancy
// caps, so the fused kernel is compared with ceilings at ITS occupancy.
__device__ __forceinline__ uint32_t wc2(uint32_t u) { return blockIdx.x * 128u + u * 64u + (threadIdx.x & 63u); }
__global__ __launch_bounds__(64) void read18_u2(const Args a, float *sink) {
  v4f t = 0.0f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t i = wc2(u) * 16u;
    t += ldo<1>(a.z, i) + ldo<1>(a.last, i);
#pragma unroll
    for (int r = 0; r < R; ++r) t += ldo<1>(a.s[r], i) + ldo<1>(a.w[r], i);
  }
  if (t.x == 12345.678f) sink[0] = t.y;
}
__global__ __launch_bounds__(64) void write10_u2(const Args a) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t i = wc2(u) * 16u;
    const v4f v = (float)i;
    sto<1>(a.z, i, v);
    sto<1>(a.last, i, v);
#pragma unroll
    for (int r = 0; r < R; ++r) sto<1>(a.w[r], i, v);
  }
}
// 18 reads + 10 writes with no load->store dependency (stores write a constant).
__global__ __launch_bounds__(64) void mix_u2(const Args a, float *sink) {
  v4f t = 0.0f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t i = wc2(u) * 16u;
    t += ldo<1>(a.z, i) + ldo<1>(a.last, i);
#pragma unroll
    for (int r = 0; r < R; ++r) t += ldo<1>(a.s[r], i) + ldo<1>(a.w[r], i);
    const v4f v = (float)i;
#pragma unroll
    for (int r = 0; r < R; ++r) sto<1>(a.w[r], i, v);
    sto<1>(a.z, i, v);
    sto<1>(a.last, i, v);
  }
  if (t.x == 12345.678f) sink[0] = t.y;
}
__global__ __launch_bounds__(64) void copy_u2(v4f *dst, const v4f *src) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t i = wc2(u) * 16u;
    sto<1>(dst, i, ldo<1>(src, i));
  }
}

// ---- v11: load order / store placement variants of the library's fused
// kernel (64-thread blocks, U = 2 wave-contiguous, nt), under the LDS caps.
//   LO 0: z, last, then per replica s_r, w_r (the library's order)
//   LO 1: z, last, all s, all w
//   LO 2: all s, all w, then z, last
//   SO 0: all FMAs, then w stores, then last, z (the library's)
//   SO 1: each w_r stored right after its FMA
template <int LO, int SO>
__global__ __launch_bounds__(64) void fused_v11(const Args a) {
  const uint32_t e0 = blockIdx.x * 128u + (threadIdx.x & 63u);
  const v4f al = a.alpha, nal = -a.alpha, mb = 0.9f, one = 1.0f, mone = -1.0f;
  v4f zv[2], lv[2], sv[2][R], wv[2][R];
  auto ldzl = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t i = (e0 + 64u * u) * 16u;
      zv[u] = ldo<1>(a.z, i);
      lv[u] = ldo<1>(a.last, i);
    }
  };
  if constexpr (LO != 2) ldzl();
  if constexpr (LO == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t i = (e0 + 64u * u) * 16u;
        sv[u][r] = ldo<1>(a.s[r], i);
        wv[u][r] = ldo<1>(a.w[r], i);
      }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < 2; ++u) sv[u][r] = ldo<1>(a.s[r], (e0 + 64u * u) * 16u);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < 2; ++u) wv[u][r] = ldo<1>(a.w[r], (e0 + 64u * u) * 16u);
  }
  if constexpr (LO == 2) ldzl();
  __builtin_amdgcn_sched_barrier(0);
  v4f acc[2] = {0.0f, 0.0f};
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      v4f d = vfma(mone, zv[u], sv[u][r]);
      wv[u][r] = vfma(nal, d, wv[u][r]);
      acc[u] = vfma(al, d, acc[u]);
      if constexpr (SO == 1) sto<1>(a.w[r], (e0 + 64u * u) * 16u, wv[u][r]);
    }
  if constexpr (SO == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < 2; ++u) sto<1>(a.w[r], (e0 + 64u * u) * 16u, wv[u][r]);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t i = (e0 + 64u * u) * 16u;
    v4f D = vfma(mb, lv[u], acc[u]);
    sto<1>(a.last, i, D);
    sto<1>(a.z, i, vfma(one, D, zv[u]));
  }
}

int main(int argc, char **argv) {
  const int64_t n = 25557032;
  const uint32_t n4 = (uint32_t)(((n + 3) / 4 + 1023) / 1024 * 1024);
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20;
  CK(hipSetDevice(0));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 256;
  {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    cus = p.multiProcessorCount;
  }
  const size_t buf = (size_t)n4 * 16;
  const int nbuf = 2 + 2 * R;
  // One big arena; layouts carve it with different strides/staggers.
  const size_t max_stagger = 4u << 20;
  const size_t arena_bytes = std::max((size_t)nbuf * (buf + (2u << 20) + max_stagger) + (64u << 20),
                                      ((size_t)2 << 30) + (8u << 20));
  char *arena;
  CK(hipMalloc(&arena, arena_bytes));
  CK(hipMemset(arena, 0, arena_bytes));
  float *sink;
  CK(hipMalloc(&sink, 64));
  const double alg = (12.0 * R + 16.0) * (double)n;

  struct Layout {
    const char *name;
    size_t stride_align;
    size_t stagger;
  };
  std::vector<Layout> layouts = {
      {"2MiB-aligned", 2u << 20, 0}, {"packed-256B", 256, 0}, {"stagger-4KiB", 2u << 20, 4096},
  };


  if (argc > 2 && std::strcmp(argv[2], "v4") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    hipEvent_t et, en;
    CK(hipEventCreate(&et));
    CK(hipEventCreateWithFlags(&en, hipEventDisableTiming));
    for (int data = 0; data < 2; ++data) {
      if (data == 1) {
        hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
        CK(hipDeviceSynchronize());
      }
      for (int blk : {128, 256}) {
        const unsigned grid = n4 / blk;
        auto launch = [&] { hipLaunchKernelGGL((fused3<1, false>), dim3(grid), dim3(blk), 0, 0, a); };
        float iso = time_ms(launch, iters);
        for (int mode = 0; mode < 3; ++mode) {
          const int K = 50;
          for (int k = 0; k < 3; ++k) launch();
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0, 0));
          for (int k = 0; k < K; ++k) {
            launch();
            if (mode == 1) CK(hipEventRecord(et, 0));
            if (mode == 2) CK(hipEventRecord(en, 0));
          }
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= K;
          std::printf("{\"v4\":1,\"data\":\"%s\",\"block\":%d,\"isolated_ms\":%.4f,\"b2b_mode\":\"%s\",\"b2b_ms\":%.4f,\"iso_GBs\":%.1f,\"b2b_GBs\":%.1f}\n",
                      data ? "random" : "zero", blk, iso, mode == 0 ? "none" : (mode == 1 ? "timing-event" : "notiming-event"),
                      ms, alg / iso / 1e6, alg / ms / 1e6);
        }
      }
    }
    return 0;
  }

  if (argc > 2 && std::strcmp(argv[2], "v5") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 3; ++round)
      for (int blk : {64, 128, 256}) {
        const unsigned grid = n4 / blk;
        float t0 = time_ms([&] { hipLaunchKernelGGL((fused3<1, false, false>), dim3(grid), dim3(blk), 0, 0, a); }, iters);
        float t1 = time_ms([&] { hipLaunchKernelGGL((fused3<1, false, true>), dim3(grid), dim3(blk), 0, 0, a); }, iters);
        std::printf("{\"v5\":%d,\"block\":%d,\"base_GBs\":%.1f,\"schedbar_GBs\":%.1f}\n", round, blk, alg / t0 / 1e6, alg / t1 / 1e6);
      }
    return 0;
  }

  if (argc > 2 && std::strcmp(argv[2], "v6") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 2; ++round) {
      float t = time_ms([&] { hipLaunchKernelGGL((fused3<1, false, true>), dim3(n4 / 128), dim3(128), 0, 0, a); }, iters);
      std::printf("{\"v6\":%d,\"kind\":\"onetrip-128\",\"GBs\":%.1f}\n", round, alg / t / 1e6);
      for (int blk : {128, 256})
        for (int wpc : {1, 2, 3, 4, 6}) {
          const unsigned grid = cus * wpc * (256 / blk);
          float tp = time_ms([&] { hipLaunchKernelGGL(fused_pipe, dim3(grid), dim3(blk), 0, 0, a); }, iters);
          std::printf("{\"v6\":%d,\"kind\":\"pipe\",\"block\":%d,\"wg256_per_cu\":%d,\"GBs\":%.1f}\n", round, blk, wpc, alg / tp / 1e6);
        }
    }
    return 0;
  }

  if (argc > 2 && std::strcmp(argv[2], "v7") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    BArgs b;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    b.off_z = 0;
    b.off_last = (uint32_t)stride;
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
      b.off_s[r] = (uint32_t)((2 + 2 * r) * stride);
      b.off_w[r] = (uint32_t)((3 + 2 * r) * stride);
    }
    a.n4 = b.n4 = n4;
    a.alpha = b.alpha = 0.1f;
    const uint32_t bytes = (uint32_t)std::min<size_t>(nbuf * stride, 0xFFFFFFF0u);
    hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
    CK(hipDeviceSynchronize());
    const unsigned grid = n4 / 128;
    for (int round = 0; round < 2; ++round) {
      float t = time_ms([&] { hipLaunchKernelGGL((fused3<1, false, true>), dim3(grid), dim3(128), 0, 0, a); }, iters);
      std::printf("{\"v7\":%d,\"kind\":\"global-nt\",\"GBs\":%.1f}\n", round, alg / t / 1e6);
#define RUNB(LA, SA) { float tb = time_ms([&] { hipLaunchKernelGGL((fused_buf<LA, SA>), dim3(grid), dim3(128), 0, 0, b, arena, bytes); }, iters); \
      std::printf("{\"v7\":%d,\"kind\":\"buffer\",\"ld_aux\":%d,\"st_aux\":%d,\"GBs\":%.1f}\n", round, LA, SA, alg / tb / 1e6); }
      RUNB(2, 2) RUNB(2, 16) RUNB(2, 18) RUNB(2, 17) RUNB(2, 19) RUNB(2, 0) RUNB(0, 2) RUNB(16, 2) RUNB(18, 18) RUNB(3, 3) RUNB(17, 17) RUNB(0, 0)
#undef RUNB
    }
    return 0;
  }

  if (argc > 2 && std::strcmp(argv[2], "v8") == 0) {
    // Allocation flavour: the default hipMalloc arena vs a physically
    // contiguous one (hipDeviceMallocContiguous): fewer, larger TLB fragments
    // for 28 streams spread over ~2 GB.
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    char *contig = nullptr;
    hipError_t ce = hipExtMallocWithFlags((void **)&contig, nbuf * stride + (4u << 20), hipDeviceMallocContiguous);
    std::printf("{\"v8\":\"contiguous-alloc\",\"ok\":%d}\n", ce == hipSuccess ? 1 : 0);
    for (int round = 0; round < 2; ++round)
      for (int which = 0; which < (ce == hipSuccess ? 2 : 1); ++which) {
        char *base = which ? contig : arena;
        Args a;
        a.z = (v4f *)base;
        a.last = (v4f *)(base + stride);
        for (int r = 0; r < R; ++r) {
          a.s[r] = (const v4f *)(base + (2 + 2 * r) * stride);
          a.w[r] = (v4f *)(base + (3 + 2 * r) * stride);
        }
        a.n4 = n4;
        a.alpha = 0.1f;
        if (round == 0) {
          hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)base, nbuf * stride / 4, 12345u);
          CK(hipDeviceSynchronize());
        }
        float t = time_ms([&] { hipLaunchKernelGGL((fused3<1, false, true>), dim3(n4 / 128), dim3(128), 0, 0, a); }, iters);
        float tr = time_ms([&] { hipLaunchKernelGGL(readk<1>, dim3(n4 / 128), dim3(128), 0, 0, a, sink); }, iters);
        std::printf("{\"v8\":%d,\"alloc\":\"%s\",\"fused_GBs\":%.1f,\"read18_GBs\":%.1f}\n", round,
                    which ? "contiguous" : "default", alg / t / 1e6, 18.0 * n4 * 16 / tr / 1e6);
      }
    if (contig) CK(hipFree(contig));
    return 0;
  }

  if (argc > 2 && std::strcmp(argv[2], "v11") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
    CK(hipDeviceSynchronize());
    const unsigned grid = n4 / 128;
    for (int round = 0; round < 3; ++round)
      for (int cap : {2, 3}) {
        const unsigned lds = (160u / (unsigned)(cap + 1) + 1u) * 1024u;
        auto go = [&](auto kern, int lo, int so) {
          float t = time_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, 0, a); }, iters);
          std::printf("{\"v11\":%d,\"cap\":%d,\"LO\":%d,\"SO\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n", round, cap, lo, so, t,
                      alg / t / 1e6);
        };
        go(fused_v11<0, 0>, 0, 0);
        go(fused_v11<1, 0>, 1, 0);
        go(fused_v11<2, 0>, 2, 0);
        go(fused_v11<0, 1>, 0, 1);
        go(fused_v11<1, 1>, 1, 1);
      }
    return 0;
  }
  if (argc > 2 && std::strcmp(argv[2], "v10") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
    CK(hipDeviceSynchronize());
    const unsigned grid = n4 / 128;
    const double rbytes = 18.0 * n4 * 16, wbytes = 10.0 * n4 * 16;
    // copy over 14 buffers' worth (1.43 GB) so it sees the same working-set size
    const uint32_t cn4 = (uint32_t)(7 * (size_t)stride / 16 / 128 * 128);
    v4f *csrc = (v4f *)arena, *cdst = (v4f *)(arena + 7 * stride + (2u << 20));
    for (int round = 0; round < 3; ++round)
      for (int cap : {0, 2, 3, 4, 6, 8, 12}) {
        // dynamic LDS that admits `cap` one-wave workgroups per CU (160 KiB per CU)
        const unsigned lds = cap ? std::min(64u * 1024u, (160u / (unsigned)(cap + 1) + 1u) * 1024u) : 0u;
        float t;
        t = time_ms([&] { hipLaunchKernelGGL(read18_u2, dim3(grid), dim3(64), lds, 0, a, sink); }, iters);
        std::printf("{\"v10\":%d,\"kind\":\"read18\",\"cap\":%d,\"GBs\":%.1f}\n", round, cap, rbytes / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(write10_u2, dim3(grid), dim3(64), lds, 0, a); }, iters);
        std::printf("{\"v10\":%d,\"kind\":\"write10\",\"cap\":%d,\"GBs\":%.1f}\n", round, cap, wbytes / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(mix_u2, dim3(grid), dim3(64), lds, 0, a, sink); }, iters);
        std::printf("{\"v10\":%d,\"kind\":\"mix18r10w-nodep\",\"cap\":%d,\"GBs\":%.1f}\n", round, cap, (rbytes + wbytes) / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(copy_u2, dim3(cn4 / 128), dim3(64), lds, 0, cdst, csrc); }, iters);
        std::printf("{\"v10\":%d,\"kind\":\"copy\",\"cap\":%d,\"GBs\":%.1f}\n", round, cap, 2.0 * cn4 * 16 / t / 1e6);
      }
    return 0;
  }
  if (argc > 2 && std::strcmp(argv[2], "v9") == 0) {
    const size_t stride = (buf + (2u << 20) - 1) / (2u << 20) * (2u << 20) + 4096;
    Args a;
    a.z = (v4f *)arena;
    a.last = (v4f *)(arena + stride);
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)(arena + (2 + 2 * r) * stride);
      a.w[r] = (v4f *)(arena + (3 + 2 * r) * stride);
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    hipLaunchKernelGGL(fillk, dim3(8192), dim3(256), 0, 0, (uint32_t *)arena, nbuf * stride / 4, 12345u);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 3; ++round)
      for (int blk : {64, 128, 256}) {
        auto go = [&](auto kern, int U) {
          const unsigned grid = (n4 + blk * U - 1) / (blk * U);
          float t = time_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(blk), 0, 0, a); }, iters);
          std::printf("{\"v9\":%d,\"block\":%d,\"U\":%d,\"GBs\":%.1f}\n", round, blk, U, alg / t / 1e6);
        };
        go(fused_wc<1>, 1);
        go(fused_wc<2>, 2);
        go(fused_wc<3>, 3);
        go(fused_wc<4>, 4);
      }
    return 0;
  }
  // Ceilings on the same arena (1 GiB copy).
  {
    const uint32_t cn4 = (uint32_t)((1u << 30) / 16);
    v4f *a = (v4f *)arena, *b = (v4f *)(arena + (1u << 30) + (2u << 20));
    for (int blk : {256, 512}) {
      unsigned g = (cn4 + blk - 1) / blk;
      float ms = time_ms([&] { hipLaunchKernelGGL(copyk<1>, dim3(g), dim3(blk), 0, 0, b, a, cn4); }, iters);
      std::printf("{\"kind\":\"copy-nt\",\"block\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n", blk, ms, 2.0 * cn4 * 16 / ms / 1e6);
      ms = time_ms([&] { hipLaunchKernelGGL(copyk<0>, dim3(g), dim3(blk), 0, 0, b, a, cn4); }, iters);
      std::printf("{\"kind\":\"copy-plain\",\"block\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n", blk, ms, 2.0 * cn4 * 16 / ms / 1e6);
    }
    for (int wpc : {4, 8, 16}) {
      unsigned g = cus * wpc;
      float ms = time_ms([&] { hipLaunchKernelGGL(copyk<1>, dim3(g), dim3(256), 0, 0, b, a, cn4); }, iters);
      std::printf("{\"kind\":\"copy-nt-gridstride\",\"wg_per_cu\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n", wpc, ms,
                  2.0 * cn4 * 16 / ms / 1e6);
    }
  }

  for (int round = 0; round < 2; ++round)
  for (const Layout &L : layouts) {
    const size_t stride = (buf + L.stride_align - 1) / L.stride_align * L.stride_align + L.stagger;
    Args a;
    std::vector<char *> p(nbuf);
    for (int k = 0; k < nbuf; ++k) p[k] = arena + (size_t)k * stride;
    a.z = (v4f *)p[0];
    a.last = (v4f *)p[1];
    for (int r = 0; r < R; ++r) {
      a.s[r] = (const v4f *)p[2 + 2 * r];
      a.w[r] = (v4f *)p[3 + 2 * r];
    }
    a.n4 = n4;
    a.alpha = 0.1f;
    auto run = [&](const char *kind, auto kern, int blk, int U) {
      const unsigned grid = n4 / (blk * U);
      float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(blk), 0, 0, a); }, iters);
      std::printf("{\"round\":%d,\"layout\":\"%s\",\"kind\":\"%s\",\"block\":%d,\"U\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n",
                  round, L.name, kind, blk, U, ms, alg / ms / 1e6);
    };
    for (int blk : {64, 128, 256}) {
      run("lib", fused3<1, false>, blk, 1);
    }
    if (L.stagger != 0) continue;
    for (int blk : {128, 256}) {
      run("lib-xcd", fused3<1, true>, blk, 1);
      run("lib-mw5", fused3<5, false>, blk, 1);
      run("lib-mw6", fused3<6, false>, blk, 1);
      run("lib-mw8", fused3<8, false>, blk, 1);
      run("o2-128", fused<1, 1, 2, 1, false>, blk, 1);
      float ms = time_ms([&] { hipLaunchKernelGGL(mixnodep, dim3(n4 / blk), dim3(blk), 0, 0, a, sink); }, iters);
      std::printf("{\"round\":%d,\"layout\":\"%s\",\"kind\":\"mixnodep\",\"block\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n", round, L.name, blk, ms, alg / ms / 1e6);
    }
  }
  CK(hipFree(arena));
  CK(hipFree(sink));
  return 0;
}
