// _hopsx_comm: collectives over IPC-mapped peer buffers (xGMI point-to-point), gfx950.
//
// for small and mid-size messages on one node a ring all-reduce is latency
// bound (2(N-1) hops).  MI355X links every GPU to its 7 peers directly, so instead
//   * one-shot: each rank copies its data into its own IPC-shared staging buffer, raises a
//     per-(source rank, workgroup) flag in every peer's uncached signal page, waits for every
//     peer's flag, then reads all N staging buffers (N-1 of them over xGMI) and sums them in
//     rank order, so every rank produces bit-identical results.  One launch, one hop.
//   * two-shot: rank r reduces slice r (reduce-scatter), then gathers the other owners' reduced
//     slices: 2(N-1)/N of the bytes per GPU instead of (N-1).
//   * dp_step (the data-parallel training step's tail, one launch): stage + zero the gradient,
//     reduce slice r, apply the optimizer to slice r only, publish the new weights of slice r,
//     gather every other slice's new weights.  Default wire: fp32 gradient + bf16 weights
//     (ZeRO-1: 6 B per parameter instead of a two-shot all-reduce's 8; opt-in bf16 gradients: 4).
//     The optimizer touches 1/N of the parameters and there is no separate optimizer launch.
//     Every replica ends with the owners' bit-identical compute weights.
// Staging is double-buffered by epoch parity; a rank cannot be two epochs ahead of a reader (it
// needs that reader's flag of the epoch in between), so reuse is safe.  The epoch is a
// per-workgroup counter in device memory (not a kernel argument), so the launches can be captured
// in a hipGraph and replayed.
//
// Failure handling: every spin is bounded by the wall clock (`spin` ticks of the 100 MHz
// counter).  A workgroup whose peer never arrives sets *err and returns WITHOUT reducing or
// writing its output (it would read an older epoch's staging) and without advancing its epoch.
// *err is sticky: every later launch on this rank sees it at entry and does nothing, so peers
// time out too and every rank reports the failure (the host polls err and raises) — no rank
// silently trains on stale sums.
//
// Reference parity: the reference's all-reduces are TF-internal NCCL calls under
// MirroredStrategy; these replace them on one node.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../ops/optim_core.h"  // upd<KIND>, OptHP, Prefetch: one definition with optim.hip

namespace py = pybind11;
using u = uintptr_t;

// the DLPack v0 ABI (dlpack.h), the subset alloc_tensor needs to hand device memory to torch.from_dlpack
extern "C" {
enum { kDLFloat = 2 };
enum { kDLROCM = 10 };
struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code, bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
}

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;  // <= one workgroup per CU: every block of every rank is resident
constexpr int kThreads = 256;
constexpr int kParity = 3;  // staging floats per parity, in units of cap: input, reduced fp32, reduced bf16
constexpr int kWireChunk = 64;  // weight-wire mask granularity (= the arena's parameter alignment)

struct Peers {
  float* buf[kMaxRanks];        // staging buffers, [parity][input | reduced | reduced bf16] = 6 * cap floats
  unsigned* flag[kMaxRanks];    // signal pages, [3 rows][kMaxRanks][kMaxBlocks] uint32 each
};

struct GradPeers {
  const float* g[kMaxRanks];  // every rank's zero-copy arena gradient as mapped in this process
};

struct Sync {
  unsigned* epochs;  // int32[kMaxBlocks] device counters (zeroed once)
  int* err;          // sticky device error flag: 1 + the rank that never arrived
  long long spin;    // wall-clock ticks (100 MHz) a workgroup waits for a peer
};

#define HIP_OK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

// workgroup-uniform: has an earlier launch on this rank failed?
__device__ inline bool poisoned(const int* err) {
  __shared__ int s_err;
  if (threadIdx.x == 0) s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return s_err != 0;
}

// Raise flag row `row` for this workgroup in every peer's page, then wait for every peer's.
// Returns false (workgroup-uniform) when a peer did not arrive within the spin bound.
__device__ inline bool flag_round(const Peers& peers, int rank, int world, int row, int b, unsigned e,
                                  const Sync& sy) {
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  // every wave publishes its own stores system-wide before the flags go out
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < world) {
    const int slot = (row * kMaxRanks + rank) * kMaxBlocks + b;
    __hip_atomic_store(peers.flag[t] + slot, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = peers.flag[rank] + (row * kMaxRanks + t) * kMaxBlocks + b;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if ((long long)(wall_clock64() - t0) > sy.spin) {
        atomicExch(sy.err, 1 + t);
        bad = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system-scope acquire for every wave before the peer reads
  return bad == 0;
}

// copy over [lo, hi) with 16-B lanes and a scalar tail
__device__ inline void copy_range(float* dst, const float* src, long lo, long hi) {
  for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(src + i);
    } else {
      for (long j = i; j < hi; ++j) dst[j] = src[j];
    }
  }
}

// s = sum over ranks 0..world-1 (in rank order) of buf[p][off + i .. i+3]
__device__ inline float4 sum4(const Peers& peers, int world, long off) {
  float4 s = *reinterpret_cast<const float4*>(peers.buf[0] + off);
  for (int p = 1; p < world; ++p) {
    const float4 v = *reinterpret_cast<const float4*>(peers.buf[p] + off);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  return s;
}
__device__ inline float sum1(const Peers& peers, int world, long off) {
  float s = peers.buf[0][off];
  for (int p = 1; p < world; ++p) s += peers.buf[p][off];
  return s;
}

// Slice geometry shared by two-shot and dp_step: slice s = [s*L, (s+1)*L) (L a multiple of 4),
// workgroup b owns [s*L + b*per, ...) of every slice, clipped to the slice and to n.
struct Slices {
  long L, per, n;
  __device__ Slices(long n_, int world, int G) : n(n_) {
    L = (n + world - 1) / world;
    L = (L + 3) & ~3L;
    per = (L + G - 1) / G;
    per = (per + 3) & ~3L;
  }
  __device__ void sub(int slice, int b, long& lo, long& hi) const {
    lo = (long)slice * L + (long)b * per;
    hi = lo + per;
    const long send = (long)slice * L + L;
    if (hi > send) hi = send;
    if (hi > n) hi = n;
    if (lo > hi) lo = hi;
  }
};

__global__ __launch_bounds__(kThreads) void oneshot_ar_k(const float* __restrict__ in, float* out, long n,
                                                         long cap, int rank, int world, Peers peers, Sync sy) {
  if (poisoned(sy.err)) return;
  const int b = blockIdx.x, G = gridDim.x;
  const unsigned e = sy.epochs[b] + 1;
  const long off = (long)(e & 1u) * kParity * cap;  // same parity layout as two-shot (modes may mix)
  // 16-B aligned chunk per workgroup
  long per = (n + G - 1) / G;
  per = (per + 3) & ~3L;
  const long lo = (long)b * per, hi = lo + per < n ? lo + per : n;

  copy_range(peers.buf[rank] + off, in, lo, hi);
  if (!flag_round(peers, rank, world, 0, b, e, sy)) return;  // never reduce another epoch's data

  for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      *reinterpret_cast<float4*>(out + i) = sum4(peers, world, off + i);
    } else {
      for (long j = i; j < hi; ++j) out[j] = sum1(peers, world, off + j);
    }
  }
  if (threadIdx.x == 0) sy.epochs[b] = e;
}

// Two-shot (reduce-scatter + all-gather over P2P) for mid-size messages: rank r owns slice r and
// reduces it (reading (N-1)/N of the data from peers), then every rank gathers the other owners'
// reduced slices.  Staging per rank: [parity][input | reduced] of cap floats each; flag rows 1, 2.
__global__ __launch_bounds__(kThreads) void twoshot_ar_k(const float* __restrict__ in, float* out, long n,
                                                         long cap, int rank, int world, Peers peers, Sync sy) {
  if (poisoned(sy.err)) return;
  const int b = blockIdx.x;
  const unsigned e = sy.epochs[b] + 1;
  const long base = (long)(e & 1u) * kParity * cap;
  const Slices S(n, world, gridDim.x);
  long lo, hi;
  for (int sl = 0; sl < world; ++sl) {
    S.sub(sl, b, lo, hi);
    copy_range(peers.buf[rank] + base, in, lo, hi);
  }
  if (!flag_round(peers, rank, world, 1, b, e, sy)) return;
  S.sub(rank, b, lo, hi);
  float* red = peers.buf[rank] + base + cap;
  for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      const float4 s = sum4(peers, world, base + i);
      *reinterpret_cast<float4*>(red + i) = s;
      *reinterpret_cast<float4*>(out + i) = s;
    } else {
      for (long j = i; j < hi; ++j) {
        const float s = sum1(peers, world, base + j);
        red[j] = s;
        out[j] = s;
      }
    }
  }
  if (!flag_round(peers, rank, world, 2, b, e, sy)) return;
  for (int k = 1; k < world; ++k) {
    const int p = (rank + k) % world;  // stagger so the N-1 peers are read over different links at once
    S.sub(p, b, lo, hi);
    copy_range(out, peers.buf[p] + base + cap, lo, hi);
  }
  if (threadIdx.x == 0) sy.epochs[b] = e;
}

// Owner pieces of the fused step: the arena is cut into pieces [c_k, c_{k+1}) — the DP buckets when the
// per-bucket reduce-scatter overlaps the backward, else one piece [0, n) — and rank r owns slice r of
// EVERY piece (L_k = ceil(len_k / world) rounded to 4), so every rank reduces a share of every bucket and
// the tail after the backward is 1/N of the last bucket, not a whole slice of the arena.  Workgroup b
// owns [c_k + s L_k + b per_k, ...) of slice s of piece k.  Cut points are multiples of 4 (the arena
// aligns parameters to 64 elements).
constexpr int kMaxCuts = 32;
struct Cuts {
  long c[kMaxCuts + 1];
  int k;  // pieces
};
struct PieceSlices {
  const Cuts& cu;
  int world, G;
  __device__ PieceSlices(const Cuts& c, int w, int g) : cu(c), world(w), G(g) {}
  __device__ void sub(int piece, int slice, int b, long& lo, long& hi) const {
    const long p0 = cu.c[piece], p1 = cu.c[piece + 1];
    long L = (p1 - p0 + world - 1) / world;
    L = (L + 3) & ~3L;
    long per = (L + G - 1) / G;
    per = (per + 3) & ~3L;
    const long s0 = p0 + (long)slice * L;
    lo = s0 + (long)b * per;
    hi = lo + per;
    if (hi > s0 + L) hi = s0 + L;
    if (hi > p1) hi = p1;
    if (lo > hi) lo = hi;
  }
};

// ------------------------------------------------------------------ fused data-parallel step
// Wire formats (what crosses xGMI per parameter and step; each GPU reads (N-1)/N of it):
//   gradients  GB = 0: fp32 reduce-scatter (4 B)   GB = 1: bf16, accumulated in fp32 (2 B)
//   weights, per 64-element chunk of the arena (wmask; nullptr = every chunk fp32):
//     fp32 (4 B): every replica receives the owner's fp32 master (parameters some kernel reads
//                 in fp32: biases, norm scales, embedding tables);
//     bf16 (2 B): ZeRO-1 for parameters the kernels read only through the bf16 compute copy
//                 (conv / dense weights): only the owner keeps their fp32 master current, the
//                 replicas share the bf16 shadow bit-for-bit, and the host gathers the owners'
//                 fp32 slices at sync points (checkpoint, verification, close).
// Staging per rank and parity: [input: cap floats | reduced fp32: cap floats | reduced bf16: cap].
struct DpArgs {
  float* master;      // fp32 [n] parameters (owner slice always current; fp32-wire chunks everywhere)
  float* grad;        // fp32 [n] local gradient; staged and zeroed here
  float* s1;          // optimizer state (full-size buffers; only this rank's slice is kept current)
  float* s2;
  float* s3;
  bf16_raw* shadow;   // bf16 [n] compute copy, refreshed for every slice
  long n;
  OptHP h;            // by value; overridden by hp_dev when given
  const float* hp_dev;
  float* step_dev;    // completed-step counter (bias correction)
  unsigned* arrive;   // arrival counter of the bookkeeping (kArriveWords, zero at rest)
  unsigned long long* rng;
  const unsigned char* wmask;  // [ceil(n / 64)] 1 = bf16 weight wire for that chunk
  Prefetch pf;
  // zero-copy gradient (fp32 wire): every rank's arena gradient IS IPC-shared memory (alloc_tensor),
  // gpeer[r] = rank r's gradient as mapped here (own at [rank] = grad).  Phase 0 then stages nothing:
  // owners read the peers' gradients in place, and each rank zeroes its own after the peers are done.
  const float* gpeer[kMaxRanks];
  int zc;           // 1: zero-copy gradients (gpeer valid)
  int pre_reduced;  // 1: dp_rs_k already summed this rank's slice into grad (per-bucket reduce-scatter
                    // during the backward): no gather round 1, the owner reads its own slice locally
};

// the 4 elements at i (i % 4 == 0) share one 64-element chunk
__device__ __forceinline__ bool wire16(const DpArgs& a, long i) { return a.wmask && a.wmask[i / kWireChunk]; }

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }
__device__ __forceinline__ uint2 pack4(const float4& w) {
  return make_uint2((uint32_t)f2bf(w.x) | ((uint32_t)f2bf(w.y) << 16),
                    (uint32_t)f2bf(w.z) | ((uint32_t)f2bf(w.w) << 16));
}

// 4 staged values at element index i of a staging region holding fp32 (BF = false) or bf16
template <bool BF>
__device__ __forceinline__ float4 ld4(const float* region, long i) {
  if (BF) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_raw*>(region) + i);
    return make_float4(bf2f(v.x & 0xffffu), bf2f(v.x >> 16), bf2f(v.y & 0xffffu), bf2f(v.y >> 16));
  }
  return *reinterpret_cast<const float4*>(region + i);
}
template <bool BF>
__device__ __forceinline__ float ld1(const float* region, long j) {
  if (BF) return bf2f(reinterpret_cast<const bf16_raw*>(region)[j]);
  return region[j];
}
template <bool BF>
__device__ __forceinline__ void st4(float* region, long i, const float4& v) {
  if (BF) {
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_raw*>(region) + i) = pack4(v);
  } else {
    *reinterpret_cast<float4*>(region + i) = v;
  }
}
template <bool BF>
__device__ __forceinline__ void st1(float* region, long j, float v) {
  if (BF) {
    reinterpret_cast<bf16_raw*>(region)[j] = f2bf(v);
  } else {
    region[j] = v;
  }
}

// rank-ordered sum of the staged gradients (every owner sums in the same order: replicas agree)
template <bool GB>
__device__ __forceinline__ float4 gsum4(const Peers& peers, int world, long base, long i) {
  float4 s = ld4<GB>(peers.buf[0] + base, i);
  for (int p = 1; p < world; ++p) {
    const float4 v = ld4<GB>(peers.buf[p] + base, i);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  return s;
}
template <bool GB>
__device__ __forceinline__ float gsum1(const Peers& peers, int world, long base, long j) {
  float s = ld1<GB>(peers.buf[0] + base, j);
  for (int p = 1; p < world; ++p) s += ld1<GB>(peers.buf[p] + base, j);
  return s;
}

// rank-ordered sum of the peers' gradients read in place (zero-copy); same order as gsum4
__device__ __forceinline__ float4 zsum4(const DpArgs& a, int world, long i) {
  float4 s = *reinterpret_cast<const float4*>(a.gpeer[0] + i);
  for (int p = 1; p < world; ++p) {
    const float4 v = *reinterpret_cast<const float4*>(a.gpeer[p] + i);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  return s;
}
__device__ __forceinline__ float zsum1(const DpArgs& a, int world, long j) {
  float s = a.gpeer[0][j];
  for (int p = 1; p < world; ++p) s += a.gpeer[p][j];
  return s;
}
// the owner's summed gradient at i: staged copies (GB / copy path), the peers' gradients in place
// (zero-copy), or this rank's own gradient already reduced by dp_rs_k (pre_reduced)
template <bool GB>
__device__ __forceinline__ float4 owner_g4(const DpArgs& a, const Peers& peers, int world, long base, long i) {
  if (!GB && a.pre_reduced) return *reinterpret_cast<const float4*>(a.grad + i);
  if (!GB && a.zc) return zsum4(a, world, i);
  return gsum4<GB>(peers, world, base, i);
}
template <bool GB>
__device__ __forceinline__ float owner_g1(const DpArgs& a, const Peers& peers, int world, long base, long j) {
  if (!GB && a.pre_reduced) return a.grad[j];
  if (!GB && a.zc) return zsum1(a, world, j);
  return gsum1<GB>(peers, world, base, j);
}
__device__ inline void zero_range(float* g, long lo, long hi) {
  for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      *reinterpret_cast<float4*>(g + i) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (long j = i; j < hi; ++j) g[j] = 0.f;
    }
  }
}

// red: this rank's reduced-fp32 region; red16: its reduced-bf16 region
template <int KIND, bool GB>
__device__ inline void owner_update(const DpArgs& a, const Peers& peers, int world, long base, float* red,
                                    bf16_raw* red16, long i, const OptHP& h, float bc1, float bc2) {
  constexpr int NS = nstate<KIND>();
  const float4 g = owner_g4<GB>(a, peers, world, base, i);
  float4 w = *reinterpret_cast<const float4*>(a.master + i);
  float4 x = NS >= 1 ? *reinterpret_cast<const float4*>(a.s1 + i) : make_float4(0, 0, 0, 0);
  float4 y = NS >= 2 ? *reinterpret_cast<const float4*>(a.s2 + i) : make_float4(0, 0, 0, 0);
  float4 z = NS >= 3 ? *reinterpret_cast<const float4*>(a.s3 + i) : make_float4(0, 0, 0, 0);
  w.x = upd<KIND>(w.x, g.x * h.gscale, x.x, y.x, z.x, h, bc1, bc2);
  w.y = upd<KIND>(w.y, g.y * h.gscale, x.y, y.y, z.y, h, bc1, bc2);
  w.z = upd<KIND>(w.z, g.z * h.gscale, x.z, y.z, z.z, h, bc1, bc2);
  w.w = upd<KIND>(w.w, g.w * h.gscale, x.w, y.w, z.w, h, bc1, bc2);
  *reinterpret_cast<float4*>(a.master + i) = w;
  if (NS >= 1) *reinterpret_cast<float4*>(a.s1 + i) = x;
  if (NS >= 2) *reinterpret_cast<float4*>(a.s2 + i) = y;
  if (NS >= 3) *reinterpret_cast<float4*>(a.s3 + i) = z;
  const uint2 wb = pack4(w);
  if (wire16(a, i)) {
    *reinterpret_cast<uint2*>(red16 + i) = wb;
  } else {
    *reinterpret_cast<float4*>(red + i) = w;
  }
  *reinterpret_cast<uint2*>(a.shadow + i) = wb;
}

template <int KIND, bool GB>
__device__ inline void owner_update1(const DpArgs& a, const Peers& peers, int world, long base, float* red,
                                     bf16_raw* red16, long j, const OptHP& h, float bc1, float bc2) {
  constexpr int NS = nstate<KIND>();
  const float g = owner_g1<GB>(a, peers, world, base, j);
  float x = NS >= 1 ? a.s1[j] : 0.f, y = NS >= 2 ? a.s2[j] : 0.f, z = NS >= 3 ? a.s3[j] : 0.f;
  const float w = upd<KIND>(a.master[j], g * h.gscale, x, y, z, h, bc1, bc2);
  a.master[j] = w;
  if (NS >= 1) a.s1[j] = x;
  if (NS >= 2) a.s2[j] = y;
  if (NS >= 3) a.s3[j] = z;
  const bf16_raw wb = f2bf(w);
  if (wire16(a, j)) {
    red16[j] = wb;
  } else {
    red[j] = w;
  }
  a.shadow[j] = wb;
}

template <int KIND, bool GB>
__global__ __launch_bounds__(kThreads) void dp_step_k(DpArgs a, long cap, int rank, int world, Peers peers, Sync sy,
                                                      Cuts cuts) {
  if (poisoned(sy.err)) return;
  const int b = blockIdx.x;
  const unsigned e = sy.epochs[b] + 1;
  const long base = (long)(e & 1u) * kParity * cap;
  const PieceSlices S(cuts, world, gridDim.x);
  const OptHP h = load_hp(a.h, a.hp_dev);
  const float t = (a.step_dev ? a.step_dev[0] : 0.f) + 1.f;  // read by every workgroup before the last bumps it
  float bc1, bc2;
  bias_corr<KIND>(h, t, bc1, bc2);
  float* mine = peers.buf[rank] + base;
  long lo, hi;

  const bool zc = !GB && a.zc;
  // phase 0: stage this workgroup's share of every slice (in the gradient wire format) and zero the
  // local gradient for the next step's accumulation; the next batch's prefetch overlaps the wait.
  // Zero-copy: nothing to stage (the peers read the gradient itself); zeroing moves after the reads
  for (int k = 0; k < cuts.k && !zc; ++k)
    for (int sl = 0; sl < world; ++sl) {
      S.sub(k, sl, b, lo, hi);
      for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
        if (i + 3 < hi) {
          st4<GB>(mine, i, *reinterpret_cast<const float4*>(a.grad + i));
          *reinterpret_cast<float4*>(a.grad + i) = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          for (long j = i; j < hi; ++j) {
            st1<GB>(mine, j, a.grad[j]);
            a.grad[j] = 0.f;
          }
        }
      }
    }
  prefetch_copy(a.pf);
  // round 1 (every rank's gradient final) — already held per bucket when dp_rs_k pre-reduced the slice
  if (!(zc && a.pre_reduced) && !flag_round(peers, rank, world, 1, b, e, sy)) return;

  // phase 1: reduce + update this rank's slice; publish the new weights in their wire format
  float* red = mine + cap;
  bf16_raw* red16 = reinterpret_cast<bf16_raw*>(mine + 2 * cap);
  for (int k = 0; k < cuts.k; ++k) {
    S.sub(k, rank, b, lo, hi);
    for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
      if (i + 3 < hi) {
        owner_update<KIND, GB>(a, peers, world, base, red, red16, i, h, bc1, bc2);
      } else {
        for (long j = i; j < hi; ++j) owner_update1<KIND, GB>(a, peers, world, base, red, red16, j, h, bc1, bc2);
      }
    }
    // zero-copy: this rank's own slice of its gradient is read by nobody else — clear it now (the same
    // threads read it above, so no barrier is needed)
    if (zc) zero_range(a.grad, lo, hi);
  }
  if (!flag_round(peers, rank, world, 2, b, e, sy)) return;

  // phase 2: every other owner's new weights -> bf16 shadow (+ fp32 master on fp32-wire chunks)
  for (int q = 0; q < cuts.k * (world - 1); ++q) {
    const int k = q / (world - 1), p = (rank + 1 + q % (world - 1)) % world;
    const float* src = peers.buf[p] + base + cap;
    const bf16_raw* src16 = reinterpret_cast<const bf16_raw*>(peers.buf[p] + base + 2 * cap);
    S.sub(k, p, b, lo, hi);
    // zero-copy: rank p's workgroup b read our gradient over [lo, hi) in its phase 1 (or its dp_rs_k),
    // and round 2 says it is done: clear it for the next step's accumulation
    if (zc) zero_range(a.grad, lo, hi);
    for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
      if (i + 3 < hi) {
        if (wire16(a, i)) {
          *reinterpret_cast<uint2*>(a.shadow + i) = *reinterpret_cast<const uint2*>(src16 + i);
        } else {
          const float4 w = *reinterpret_cast<const float4*>(src + i);
          *reinterpret_cast<float4*>(a.master + i) = w;
          *reinterpret_cast<uint2*>(a.shadow + i) = pack4(w);
        }
      } else {
        for (long j = i; j < hi; ++j) {
          if (wire16(a, j)) {
            a.shadow[j] = src16[j];
          } else {
            const float w = src[j];
            a.master[j] = w;
            a.shadow[j] = f2bf(w);
          }
        }
      }
    }
  }
  if (threadIdx.x == 0) sy.epochs[b] = e;
  step_bookkeeping(a.arrive, a.step_dev, t, a.rng, a.pf);
}

// Per-bucket reduce-scatter during the backward (zero-copy gradients, fp32): launched on a side stream
// once the bucket's last gradient kernel is done, it sums every rank's gradient over the part of THIS
// rank's owner slice that lies in the bucket [blo, bhi) and writes the sum into this rank's own gradient
// in place (no other rank reads this rank's gradient inside its own slice).  One flag round (row 1) per
// launch: a peer's flag says its bucket is final.  The step tail (dp_step_k, pre_reduced) then updates
// the slice from local memory.
__global__ __launch_bounds__(kThreads) void dp_rs_k(float* grad, long n, long blo, long bhi, int rank, int world,
                                                    Peers peers, GradPeers gp, Sync sy) {
  if (poisoned(sy.err)) return;
  const int b = blockIdx.x, G = gridDim.x;
  const unsigned e = sy.epochs[b] + 1;
  if (!flag_round(peers, rank, world, 1, b, e, sy)) return;
  // the bucket is one owner piece of the step tail (PieceSlices): this rank's slice of it
  long L = (bhi - blo + world - 1) / world;
  L = (L + 3) & ~3L;
  long lo = blo + (long)rank * L, hi = lo + L;
  if (hi > bhi) hi = bhi;
  if (hi > n) hi = n;
  if (hi > lo) {
    long per = (hi - lo + G - 1) / G;
    per = (per + 3) & ~3L;
    const long wlo = lo + (long)b * per;
    const long whi = wlo + per < hi ? wlo + per : hi;
    for (long i = wlo + 4L * threadIdx.x; i < whi; i += 4L * kThreads) {
      if (i + 3 < whi && (i & 3) == 0) {
        float4 s = *reinterpret_cast<const float4*>(gp.g[0] + i);
        for (int p = 1; p < world; ++p) {
          const float4 v = *reinterpret_cast<const float4*>(gp.g[p] + i);
          s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        *reinterpret_cast<float4*>(grad + i) = s;
      } else {
        for (long j = i; j < whi && j < i + 4; ++j) {
          float s = gp.g[0][j];
          for (int p = 1; p < world; ++p) s += gp.g[p][j];
          grad[j] = s;
        }
      }
    }
  }
  if (threadIdx.x == 0) sy.epochs[b] = e;
}

// ---- exchange-protocol instruments (runtime/persist_sim.py and the cross-process tests) ----
// A peer rank emulated from another process: push `n` 4-byte words into a (typically IPC-mapped,
// uncached) exchange buffer with system-scope stores, as a producer rank's persistent kernel does.
// The flags go in a SECOND launch on the same stream (xfill_k), so every payload word has completed
// before any flag is visible — the producer side of the persistent step's hand-off.
__global__ __launch_bounds__(kThreads) void xpush_k(unsigned* dst, const unsigned* __restrict__ src, long n) {
  for (long i = blockIdx.x * (long)kThreads + threadIdx.x; i < n; i += (long)gridDim.x * kThreads)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(kThreads) void xfill_k(unsigned* dst, long n, unsigned v) {
  for (long i = blockIdx.x * (long)kThreads + threadIdx.x; i < n; i += (long)gridDim.x * kThreads)
    __hip_atomic_store(dst + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Occupancy hog: `gridDim.x` workgroups that hold `lds` bytes of LDS each (one per CU at > 80 KiB) and
// sleep for `ticks` of the 100 MHz wall clock — a concurrently resident kernel for the persistent
// step's co-residency test.  Bounded: every wave leaves after `ticks`.
__global__ __launch_bounds__(64) void hog_k(long long ticks, unsigned* touch) {
  extern __shared__ unsigned hog_lds[];
  const long long t0 = wall_clock64();
  hog_lds[threadIdx.x] = threadIdx.x;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  if (touch && threadIdx.x == 0 && blockIdx.x == 0) touch[0] = hog_lds[1];
}

py::bytes handle_of(u ptr) {
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

Peers make_peers(int rank, int world, const std::vector<u>& bufs, const std::vector<u>& flags) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) throw std::runtime_error("bad rank/world");
  if ((int)bufs.size() != world || (int)flags.size() != world) throw std::runtime_error("need one ptr per rank");
  Peers pr{};
  for (int i = 0; i < world; ++i) {
    if ((bufs[i] | flags[i]) & 15u) throw std::runtime_error("staging / flag pages must be 16-B aligned");
    pr.buf[i] = reinterpret_cast<float*>(bufs[i]);
    pr.flag[i] = reinterpret_cast<unsigned*>(flags[i]);
  }
  return pr;
}

long long spin_ticks(double seconds) {
  if (!(seconds > 0)) throw std::runtime_error("timeout must be > 0");
  return (long long)(seconds * 1e8);  // s_memrealtime runs at 100 MHz
}

}  // namespace

PYBIND11_MODULE(_hopsx_comm, m) {
  m.doc() = "hopsx P2P collectives over IPC-mapped peer buffers (xGMI, gfx950)";
  m.attr("MAX_RANKS") = kMaxRanks;
  m.attr("MAX_BLOCKS") = kMaxBlocks;
  m.attr("THREADS") = kThreads;
  m.attr("FLAG_ROWS") = 3;
  m.attr("STAGING_FLOATS_PER_CAP") = 2 * kParity;  // staging buffer = this * cap floats
  m.attr("WIRE_CHUNK") = kWireChunk;  // row 0: one-shot, rows 1-2: the two rounds of two-shot / dp_step

  // staging memory (coarse-grained) or an uncached signal page; zeroed; returns (ptr, ipc handle)
  m.def("alloc", [](long bytes, bool uncached) {
    void* p = nullptr;
    if (uncached) {
      HIP_OK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    } else {
      HIP_OK(hipMalloc(&p, bytes));
    }
    HIP_OK(hipMemset(p, 0, bytes));
    HIP_OK(hipDeviceSynchronize());
    return py::make_tuple(reinterpret_cast<u>(p), handle_of(reinterpret_cast<u>(p)));
  });
  m.def("free", [](u p) { HIP_OK(hipFree(reinterpret_cast<void*>(p))); });
  m.def("open", [](py::bytes hb) {
    std::string s = hb;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    return reinterpret_cast<u>(p);
  });
  m.def("close", [](u p) { HIP_OK(hipIpcCloseMemHandle(reinterpret_cast<void*>(p))); });
  m.def("handle_size", []() { return (int)sizeof(hipIpcMemHandle_t); });
  // synchronous device copy between raw pointers (exchange buffers <-> tensors, runtime/persist_sim.py)
  m.def("copy", [](u dst, u src, long bytes) {
    if (bytes <= 0) return;
    HIP_OK(hipMemcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), bytes, hipMemcpyDefault));
  });
  // system-scope payload push / flag fill (4-byte words) on `stream`: the emulated peer's producer side
  m.def("xpush", [](u dst, u src, long bytes, u stream) {
    if (bytes <= 0 || (bytes & 3) || ((dst | src) & 3u)) throw std::runtime_error("xpush: 4-B aligned words");
    const long n = bytes / 4;
    const int blocks = (int)std::min<long>(256, (n + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(xpush_k, dim3(blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<unsigned*>(dst), reinterpret_cast<const unsigned*>(src), n);
    HIP_OK(hipGetLastError());
  });
  m.def("xfill", [](u dst, long nwords, unsigned value, u stream) {
    if (nwords <= 0 || (dst & 3u)) throw std::runtime_error("xfill: 4-B aligned words");
    const int blocks = (int)std::min<long>(64, (nwords + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(xfill_k, dim3(blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<unsigned*>(dst), nwords, value);
    HIP_OK(hipGetLastError());
  });
  m.def("hog", [](double seconds, int blocks, int lds_bytes, u touch, u stream) {
    if (blocks < 1 || blocks > 4096 || lds_bytes < 256 || lds_bytes > 160 * 1024 || !(seconds > 0 && seconds < 10))
      throw std::runtime_error("hog: bad shape");
    HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(hog_k), hipFuncAttributeMaxDynamicSharedMemorySize,
                               lds_bytes));
    hipLaunchKernelGGL(hog_k, dim3(blocks), dim3(64), lds_bytes, reinterpret_cast<hipStream_t>(stream),
                       spin_ticks(seconds), reinterpret_cast<unsigned*>(touch));
    HIP_OK(hipGetLastError());
  });

  // out = sum over ranks of in (fp32, n elements, n <= cap); blocks <= MAX_BLOCKS, identical on all
  // ranks; epochs: int32[MAX_BLOCKS] device counters (zeroed once); err: int32 sticky device flag;
  // timeout: seconds a workgroup waits for a peer before it gives up (sets err, writes nothing)
  // two_shot: reduce-scatter + all-gather variant (staging: STAGING_FLOATS_PER_CAP * cap floats)
  m.def("allreduce_f32", [](u in, u out, long n, long cap, int rank, int world, std::vector<u> bufs,
                            std::vector<u> flags, u epochs, u err, int blocks, u stream, bool two_shot,
                            double timeout) {
    const Peers pr = make_peers(rank, world, bufs, flags);
    if (n < 0 || n > cap) throw std::runtime_error("n exceeds the staging capacity");
    if (blocks < 1 || blocks > kMaxBlocks) throw std::runtime_error("blocks out of range");
    if ((in | out) & 15u) throw std::runtime_error("in/out must be 16-B aligned");
    const Sync sy{reinterpret_cast<unsigned*>(epochs), reinterpret_cast<int*>(err), spin_ticks(timeout)};
    hipLaunchKernelGGL(two_shot ? twoshot_ar_k : oneshot_ar_k, dim3(blocks), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float*>(in),
                       reinterpret_cast<float*>(out), n, cap, rank, world, pr, sy);
    HIP_OK(hipGetLastError());
  });

  // Fused data-parallel step tail: reduce-scatter(grad) -> optimizer on this rank's slice ->
  // all-gather(new fp32 weights) + bf16 shadow refresh + grad zeroing + step bookkeeping, one launch.
  // kind: 0 SGD, 1 Adam, 2 AdamW, 3 Adadelta, 4 RMSprop, 5 Adagrad, 6 FTRL (optim_core.h)
  m.def("dp_step", [](int kind, u master, u grad, u s1, u s2, u s3, u shadow, long n, std::vector<float> hp,
                      u hp_dev, u step_dev, u arrive, u rng, std::vector<u> pf_src, std::vector<u> pf_dst,
                      std::vector<long> pf_bytes, u pf_cursor, int pf_nbatch, long cap, int rank, int world,
                      std::vector<u> bufs, std::vector<u> flags, u epochs, u err, int blocks, u stream,
                      double timeout, bool grad_bf16, u wmask, std::vector<u> gpeers, bool pre_reduced,
                      std::vector<long> cuts) {
    const Peers pr = make_peers(rank, world, bufs, flags);
    // owner pieces: the cut points 0 = c_0 < ... < c_K = n (empty: one piece), multiples of 4
    Cuts cu{};
    if (cuts.empty()) cuts = {0, n};
    if ((int)cuts.size() < 2 || (int)cuts.size() > kMaxCuts + 1 || cuts.front() != 0 || cuts.back() != n)
      throw std::runtime_error("cuts must run 0 .. n with at most 32 pieces");
    for (size_t i = 0; i < cuts.size(); ++i) {
      if ((i && cuts[i] <= cuts[i - 1]) || (cuts[i] & 3)) throw std::runtime_error("cuts: increasing multiples of 4");
      cu.c[i] = cuts[i];
    }
    cu.k = (int)cuts.size() - 1;
    if (n < 0 || n > cap) throw std::runtime_error("arena exceeds the staging capacity");
    if (blocks < 1 || blocks > kMaxBlocks) throw std::runtime_error("blocks out of range");
    if (!master || !grad || !shadow) throw std::runtime_error("dp_step needs master, grad and shadow");
    if ((master | grad | s1 | s2 | s3) & 15u || shadow & 7u) throw std::runtime_error("buffers must be 16-B aligned");
    DpArgs a{};
    a.master = reinterpret_cast<float*>(master);
    a.grad = reinterpret_cast<float*>(grad);
    a.s1 = reinterpret_cast<float*>(s1);
    a.s2 = reinterpret_cast<float*>(s2);
    a.s3 = reinterpret_cast<float*>(s3);
    a.shadow = reinterpret_cast<bf16_raw*>(shadow);
    a.n = n;
    a.h = OptHP{0, 1, 0, 0, 0, 0, 0, 0};
    float* hv = &a.h.lr;
    for (size_t i = 0; i < hp.size() && i < 8; ++i) hv[i] = hp[i];
    a.hp_dev = reinterpret_cast<const float*>(hp_dev);
    a.step_dev = reinterpret_cast<float*>(step_dev);
    a.arrive = reinterpret_cast<unsigned*>(arrive);
    a.rng = reinterpret_cast<unsigned long long*>(rng);
    a.wmask = reinterpret_cast<const unsigned char*>(wmask);
    if (!gpeers.empty()) {
      // zero-copy gradients: one mapped pointer per rank, ours first-class at [rank] (fp32 wire only)
      if ((int)gpeers.size() != world || grad_bf16) throw std::runtime_error("zero-copy needs one fp32 gradient per rank");
      if (gpeers[rank] != grad) throw std::runtime_error("zero-copy: this rank's entry must be its own gradient");
      for (int r = 0; r < world; ++r) {
        if (!gpeers[r] || (gpeers[r] & 15u)) throw std::runtime_error("zero-copy gradients must be 16-B aligned");
        a.gpeer[r] = reinterpret_cast<const float*>(gpeers[r]);
      }
      a.zc = 1;
      a.pre_reduced = pre_reduced ? 1 : 0;
    } else if (pre_reduced) {
      throw std::runtime_error("pre_reduced needs zero-copy gradients");
    }
    a.pf = Prefetch{};
    const size_t nj = std::min<size_t>(2, std::min(pf_src.size(), std::min(pf_dst.size(), pf_bytes.size())));
    if (nj > 0 && pf_cursor && pf_nbatch > 0 && arrive) {
      for (size_t j = 0; j < nj; ++j) {
        if ((pf_src[j] | pf_dst[j] | (u)pf_bytes[j]) % 16 != 0) throw std::runtime_error("prefetch not 16-B aligned");
        a.pf.job[j] = PrefetchJob{reinterpret_cast<const unsigned char*>(pf_src[j]),
                                  reinterpret_cast<unsigned char*>(pf_dst[j]), pf_bytes[j]};
      }
      a.pf.njobs = (int)nj;
      a.pf.cursor = reinterpret_cast<long long*>(pf_cursor);
      a.pf.nbatch = pf_nbatch;
    }
    if ((step_dev || rng || a.pf.njobs) && !arrive) throw std::runtime_error("bookkeeping needs the arrival counter");
    const Sync sy{reinterpret_cast<unsigned*>(epochs), reinterpret_cast<int*>(err), spin_ticks(timeout)};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define DP_CASE(K)                                                                                  \
  case K:                                                                                           \
    if (grad_bf16) {                                                                                \
      hipLaunchKernelGGL((dp_step_k<K, true>), dim3(blocks), dim3(kThreads), 0, st, a, cap, rank, world, pr, sy, cu); \
    } else {                                                                                        \
      hipLaunchKernelGGL((dp_step_k<K, false>), dim3(blocks), dim3(kThreads), 0, st, a, cap, rank, world, pr, sy, cu); \
    }                                                                                               \
    break;
    switch (kind) {
      DP_CASE(0) DP_CASE(1) DP_CASE(2) DP_CASE(3) DP_CASE(4) DP_CASE(5) DP_CASE(6)
      default: throw std::runtime_error("unknown optimizer kind");
    }
#undef DP_CASE
    HIP_OK(hipGetLastError());
  });

  // per-bucket reduce-scatter of zero-copy fp32 gradients (dp_rs_k): sums every rank's gradient over
  // [blo, bhi) ∩ this rank's owner slice into this rank's own gradient; the same `blocks` on every rank
  m.def("dp_rs", [](u grad, long n, long blo, long bhi, long cap, int rank, int world, std::vector<u> bufs,
                    std::vector<u> flags, std::vector<u> gpeers, u epochs, u err, int blocks, u stream, double timeout) {
    const Peers pr = make_peers(rank, world, bufs, flags);
    if (n < 0 || n > cap || blo < 0 || bhi > n || blo > bhi) throw std::runtime_error("bad bucket range");
    if (blocks < 1 || blocks > kMaxBlocks) throw std::runtime_error("blocks out of range");
    if ((int)gpeers.size() != world || gpeers[rank] != grad) throw std::runtime_error("need one gradient per rank");
    GradPeers gp{};
    for (int r = 0; r < world; ++r) {
      if (!gpeers[r] || (gpeers[r] & 15u)) throw std::runtime_error("gradients must be 16-B aligned");
      gp.g[r] = reinterpret_cast<const float*>(gpeers[r]);
    }
    const Sync sy{reinterpret_cast<unsigned*>(epochs), reinterpret_cast<int*>(err), spin_ticks(timeout)};
    hipLaunchKernelGGL(dp_rs_k, dim3(blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<float*>(grad), n, blo, bhi, rank, world, pr, gp, sy);
    HIP_OK(hipGetLastError());
  });

  // Device memory (hipMalloc, zeroed) handed to torch as a tensor through DLPack, plus its IPC handle:
  // the arena gradient of the zero-copy P2P step, which the peers map and read in place.  The memory
  // is freed when the last torch reference goes (peers' mappings keep their own reference).
  m.def("alloc_tensor", [](long nfloats, int device) {
    if (nfloats <= 0) throw std::runtime_error("alloc_tensor: empty");
    void* p = nullptr;
    HIP_OK(hipSetDevice(device));
    HIP_OK(hipMalloc(&p, nfloats * 4));
    HIP_OK(hipMemset(p, 0, nfloats * 4));
    HIP_OK(hipDeviceSynchronize());
    py::bytes h = handle_of(reinterpret_cast<u>(p));
    auto* mt = new DLManagedTensor{};
    auto* shape = new int64_t[1]{nfloats};
    mt->dl_tensor.data = p;
    mt->dl_tensor.device = DLDevice{kDLROCM, device};
    mt->dl_tensor.ndim = 1;
    mt->dl_tensor.dtype = DLDataType{kDLFloat, 32, 1};
    mt->dl_tensor.shape = shape;
    mt->dl_tensor.strides = nullptr;
    mt->dl_tensor.byte_offset = 0;
    mt->manager_ctx = shape;
    mt->deleter = [](DLManagedTensor* self) {
      (void)hipFree(self->dl_tensor.data);
      delete[] static_cast<int64_t*>(self->manager_ctx);
      delete self;
    };
    // an unconsumed capsule frees the tensor itself; torch renames a consumed one "used_dltensor"
    py::capsule cap(mt, "dltensor", [](PyObject* o) {
      if (PyCapsule_IsValid(o, "dltensor")) {
        auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(o, "dltensor"));
        if (t && t->deleter) t->deleter(t);
      }
    });
    return py::make_tuple(cap, reinterpret_cast<u>(p), h);
  });
}
