// hopsx CDNA4 (gfx950) kernel library — shared device helpers.
//
// All kernels in csrc/ops are written for MI355X only: 64-lane waves, MFMA
// bf16 16x16x32 tiles, 160 KiB LDS per CU, 8 XCDs with private L2s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HOPSX_WAVE 64

typedef uint16_t bf16_raw;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Branch-free masking for gathers: load from a clamped (always valid) address, then zero the
// value unless `keep`.  A `cond ? load : 0` makes hipcc branch around each load and wait
// vmcnt(0) per element, serialising what should be independent loads in flight.
__device__ __forceinline__ bf16x8 zero_unless(bf16x8 v, bool keep) {
  const short m = keep ? (short)-1 : (short)0;
  return v & (bf16x8){m, m, m, m, m, m, m, m};
}
typedef __attribute__((address_space(3))) bf16x4* lds_v4_ptr;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even fp32 -> bf16 (NaN preserved)
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// DPP row rotation (lane l of a 16-lane row reads lane (l + R) % 16 of the same row): plain VALU,
// no LDS round trip, unlike __shfl_xor (ds_bpermute)
template <int R>
__device__ __forceinline__ float dpp_ror(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + R, 0xF, 0xF, false));
}
// sum of the lanes of v congruent to this lane mod CW (CW a power of two <= 16) within its 16-lane row
template <int CW>
__device__ __forceinline__ float row_fold(float v) {
  if constexpr (CW <= 1) v += dpp_ror<1>(v);
  if constexpr (CW <= 2) v += dpp_ror<2>(v);
  if constexpr (CW <= 4) v += dpp_ror<4>(v);
  if constexpr (CW <= 8) v += dpp_ror<8>(v);
  return v;
}

// Grid-wide "am I the last workgroup?" for a launch whose workgroups each arrive once (thread 0
// calls it after the workgroup's writes are complete and released).  The counter is 9 x 32 uint32,
// zero at rest: 8 shards on their own 128-B lines (blockIdx % 8 = the XCD under round-robin
// dispatch) and the top word at index 0.  One word taking every arrival serialises at ~12 ns per
// atomic (~3 us for 256 workgroups, MI355X_MICROARCH "fanin"); sharded, each word sees grid/8.
// The counter is back at zero when the last arriver returns true.
constexpr int kArriveWords = 9 * 32;
// replica rows of the zero-at-rest BatchNorm statistics accumulators [HOPSX_BN_NREP][2C]
// (norm.hip; conv epilogues that produce BN statistics add into the same layout)
constexpr int HOPSX_BN_NREP = 8;
__device__ inline bool grid_arrive_last(unsigned* arrive) {
  const unsigned G = gridDim.x;
  const unsigned shard = blockIdx.x & 7u;
  const unsigned members = (G - shard + 7u) / 8u;  // blocks b < G with b % 8 == shard
  unsigned* sw = arrive + 32u * (shard + 1u);
  if (atomicAdd(sw, 1u) != members - 1u) return false;
  atomicExch(sw, 0u);
  const unsigned shards = G < 8u ? G : 8u;
  if (atomicAdd(arrive, 1u) != shards - 1u) return false;
  atomicExch(arrive, 0u);
  return true;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming T1):
// consecutive logical tiles land on the same XCD so neighbouring tiles share L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg <= 8) return bid;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Counter-based RNG: stateless, so dropout masks are regenerated in the backward pass from
// (seed, offset, index) instead of stored.  Two rounds of a 32-bit xorshift-multiply finalizer
// (4 v_mul_lo_u32) with the 64-bit key folded in between: a splitmix64 finalizer costs ~16
// quarter-rate 32-bit multiplies per draw, which made the RNG the bulk of the conv+pool+dropout
// epilogue.  The first round is a bijection of the index, the second mixes in the other key half.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  const uint32_t ka = (uint32_t)seed ^ (uint32_t)(idx >> 32) * 0x9E3779B9u;
  const uint32_t kb = (uint32_t)(seed >> 32);
  return mix32(mix32((uint32_t)idx ^ ka) + kb);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  return (hash_u32(seed, idx) & 0xFFFFFF) * (1.0f / 16777216.0f);
}

// dropout key for (device RNG state, per-layer salt); state = {seed, step counter}
__device__ __forceinline__ uint64_t drop_key(const unsigned long long* rng, unsigned salt) {
  return (uint64_t)rng[0] ^ ((uint64_t)salt * 0xD1B54A32D192ED03ull) ^ ((uint64_t)rng[1] * 0x8CB92BA72F3D8DD7ull);
}

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3 };

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}
// derivative of the activation expressed through its OUTPUT y
__device__ __forceinline__ float act_grad_from_out(float y, int act) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: return y * (1.f - y);
    case ACT_TANH: return 1.f - y * y;
    default: return 1.f;
  }
}

#define HOPSX_CHECK_LAUNCH() (void)hipGetLastError()

#include <cstdlib>
#include <cstring>
// Host-side kill switch for specialised fast paths, for A/B checks:
// HOPSX_DISABLE=direct_conv,pool8,rowreduce,loss_thread,splitk
// (read on every call: a cached getenv pointer dangles once the process changes the variable — the
// A/B tests toggle it between runs — and then decided launches from freed memory)
static inline bool hopsx_disabled(const char* name) {
  const char* env = std::getenv("HOPSX_DISABLE");
  return env && *env && std::strstr(env, name) != nullptr;
}
// integer tuning knob from the environment (read on every call: host-side launch sizing only)
static inline long hopsx_env_int(const char* name, long dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atol(e) : dflt;
}

// ---- deterministic mode (HOPSX_DETERMINISTIC=1) ----
// Every float reduction that crosses workgroups is made order-fixed, so a replay from the same state
// is bit-identical:
//  * host side: no split-K (plan_gemm / want_splitk / the gg engine plan one K slice per tile), so an
//    output element of a GEMM has exactly one producer;
//  * device side: the sites where several workgroups add into the same floats (bias-gradient column
//    sums, weight-gradient partials over pixel chunks, split-K head workspaces, BatchNorm statistics)
//    take turns in workgroup order: workgroup `my` waits until the site's counter reads `my`, adds,
//    drains its atomics and hands the turn on (the last one resets the counter to zero).  Workgroups
//    are dispatched in id order per XCD, so the lowest waiting one's predecessor is always running
//    or done: no deadlock; a wait that still exceeds ~1 s gives up (correct, no longer ordered) and
//    counts in hx_det_lost.  Deterministic mode assumes one stream (concurrent launches of the same
//    site would interleave their turns).
// The flag and the counters are per translation unit (static device symbols, zero at load);
// HOPSX_DET_TU(tag) in a .hip file defines the host setter hopsx_det_set_<tag>.
static inline bool hopsx_deterministic() {
  static const bool on = [] {
    const char* e = std::getenv("HOPSX_DETERMINISTIC");
    return e && *e == '1';
  }();
  return on;
}
constexpr int HX_DET_SITES = 16;
static __device__ int hx_det_on;
static __device__ unsigned hx_det_ctr[HX_DET_SITES * 32];  // one 128-B line per site
static __device__ unsigned hx_det_lost;
// site ids (distinct per kernel that may run in the same launch)
enum HxDetSite : int { DET_GEMM_COLSUM = 0, DET_DGRAD_COLSUM = 1, DET_WGRAD = 2, DET_MLP_WS = 3, DET_BN_FWD = 4,
                       DET_BN_STATS = 5, DET_POOL_COLSUM = 6, DET_GG_COLSUM = 7, DET_COLSUM = 8, DET_BN_BWD = 9 };

__device__ __forceinline__ bool det_on() { return __builtin_amdgcn_readfirstlane(hx_det_on) != 0; }
// workgroup-uniform: wait for this workgroup's turn at `site` (all threads call it)
__device__ inline void det_turn_begin(int site, unsigned my) {
  if (threadIdx.x == 0) {
    unsigned* c = hx_det_ctr + site * 32;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != my) {
      if (wall_clock64() - t0 > 100000000ll) {
        atomicAdd(&hx_det_lost, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}
// hand the turn on once this workgroup's atomics have completed (all threads call it)
__device__ inline void det_turn_end(int site, unsigned my, unsigned total) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(hx_det_ctr + site * 32, my + 1u == total ? 0u : my + 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}
// ---- device-side bound checks.  hx_check(c) compiles to `true` in a release build; in the debug build
// (-DHOPSX_DEBUG=1: module _hopsx_ops_dbg, loaded when HOPSX_DEBUG=1) it evaluates c, and a failure records
// the translation unit's first failing site (source line, workgroup, thread) plus a failure count in
// hx_dbg_err and yields false, so the caller skips the access instead of faulting.  hx_guard(c) is the
// same check kept in release builds too: for user-supplied indices (embedding ids, class labels), where
// an out-of-range value must not become an out-of-bounds access.  kernels.debug_errors() reads and
// clears the records (HOPSX_DBG_TU below); the debug build's kernels.check() raises on one after every
// launch outside graph capture.
#ifndef HOPSX_DEBUG
#define HOPSX_DEBUG 0
#endif
static __device__ unsigned hx_dbg_err[4];  // failures, line of the first, its workgroup, its thread
__device__ __forceinline__ bool hx_fail_at(int line) {
  if (atomicAdd(&hx_dbg_err[0], 1u) == 0u) {
    atomicExch(&hx_dbg_err[1], (unsigned)line);
    atomicExch(&hx_dbg_err[2], blockIdx.x + gridDim.x * blockIdx.y);
    atomicExch(&hx_dbg_err[3], threadIdx.x);
  }
  return false;
}
#define hx_guard(c) ((c) ? true : hx_fail_at(__LINE__))
#if HOPSX_DEBUG
#define hx_check(c) hx_guard(c)
#else
#define hx_check(c) true
#endif
// host reader of the translation unit's records: out[4] as above; clears them
#define HOPSX_DBG_TU(tag)                                                                            \
  extern "C" int hopsx_dbg_read_##tag(unsigned* out) {                                              \
    int e = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(hx_dbg_err), 4 * sizeof(unsigned), 0,          \
                                     hipMemcpyDeviceToHost);                                        \
    const unsigned z[4] = {0u, 0u, 0u, 0u};                                                         \
    if (!e && out[0]) e = (int)hipMemcpyToSymbol(HIP_SYMBOL(hx_dbg_err), z, sizeof(z), 0, hipMemcpyHostToDevice); \
    return e;                                                                                       \
  }
#define HOPSX_DET_TU(tag)                                                                          \
  HOPSX_DBG_TU(tag)                                                                                \
  extern "C" int hopsx_det_set_##tag(int on) {                                                     \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(hx_det_on), &on, sizeof(int), 0, hipMemcpyHostToDevice); \
  }                                                                                                \
  extern "C" unsigned hopsx_det_lost_##tag() {                                                     \
    unsigned v = 0;                                                                                \
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(hx_det_lost), sizeof(unsigned), 0, hipMemcpyDeviceToHost); \
    return v;                                                                                      \
  }
