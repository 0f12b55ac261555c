// _hopsx_comm: one-shot all-reduce over IPC-mapped peer buffers (xGMI point-to-point).
//
// for buffers below ~1 MB on one node a ring all-reduce is latency bound
// (2(N-1) hops).  MI355X links every GPU to its 7 peers directly, so each rank instead
//   1. copies its chunk into its own IPC-shared staging buffer,
//   2. raises a per-(source rank, workgroup) flag in every peer's uncached signal page,
//   3. waits for the same flag from every peer, then
//   4. reads the chunk from all N staging buffers (N-1 of them over xGMI) and sums them in rank
//      order, so every rank produces bit-identical results.
// One launch, one hop.  Staging is double-buffered by epoch parity; a rank cannot be two epochs
// ahead of a reader (it needs that reader's flag of the epoch in between), so reuse is safe.
// The epoch is a per-workgroup counter in device memory (not a kernel argument), so the launch
// can be captured in a hipGraph and replayed.  Every spin is bounded by the wall clock: a peer
// that never arrives sets *err and the wave exits, so the grid always drains.
//
// Reference parity: the reference's all-reduces are TF-internal NCCL calls under
// MirroredStrategy; this replaces the small-message ones.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;
using u = uintptr_t;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 128;  // <= one workgroup per CU: every block of every rank is resident
constexpr int kThreads = 256;
constexpr unsigned long long kSpinTicks = 400000000ull;  // ~4 s at the 100 MHz wall clock

struct Peers {
  float* buf[kMaxRanks];        // staging buffers, [parity][input | reduced] = 4 * cap floats each
  unsigned* flag[kMaxRanks];    // signal pages, [3 rows][kMaxRanks][kMaxBlocks] uint32 each
};

#define HIP_OK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

__global__ __launch_bounds__(kThreads) void oneshot_ar_k(const float* __restrict__ in, float* out, long n,
                                                         long cap, int rank, int world, Peers peers,
                                                         unsigned* epochs, int* err) {
  const int b = blockIdx.x, G = gridDim.x, t = threadIdx.x;
  const unsigned e = epochs[b] + 1;
  const long off = (long)(e & 1u) * 2 * cap;  // same parity layout as two-shot (modes may mix)
  // 16-B aligned chunk per workgroup
  long per = (n + G - 1) / G;
  per = (per + 3) & ~3L;
  const long lo = (long)b * per, hi = lo + per < n ? lo + per : n;

  float* mine = peers.buf[rank] + off;
  for (long i = lo + 4L * t; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      *reinterpret_cast<float4*>(mine + i) = *reinterpret_cast<const float4*>(in + i);
    } else {
      for (long j = i; j < hi; ++j) mine[j] = in[j];
    }
  }
  // every wave publishes its own stores system-wide before the flags go out
  __threadfence_system();
  __syncthreads();
  if (t < world) {
    __hip_atomic_store(peers.flag[t] + rank * kMaxBlocks + b, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = peers.flag[rank] + t * kMaxBlocks + b;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (wall_clock64() - t0 > kSpinTicks) {
        atomicExch(err, 1 + t);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system-scope acquire for every wave before the peer reads

  for (long i = lo + 4L * t; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      float4 s = *reinterpret_cast<const float4*>(peers.buf[0] + off + i);
      for (int p = 1; p < world; ++p) {
        const float4 v = *reinterpret_cast<const float4*>(peers.buf[p] + off + i);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      *reinterpret_cast<float4*>(out + i) = s;
    } else {
      for (long j = i; j < hi; ++j) {
        float s = peers.buf[0][off + j];
        for (int p = 1; p < world; ++p) s += peers.buf[p][off + j];
        out[j] = s;
      }
    }
  }
  if (t == 0) epochs[b] = e;
}

// copy / reduce helpers over [lo, hi) with 16-B lanes and a scalar tail
__device__ inline void copy_range(float* dst, const float* src, long lo, long hi) {
  for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(src + i);
    } else {
      for (long j = i; j < hi; ++j) dst[j] = src[j];
    }
  }
}

// raise flag row `row` for this workgroup in every peer's page, then wait for every peer's
__device__ inline void flag_round(const Peers& peers, int rank, int world, int row, int b, unsigned e, int* err) {
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < world) {
    const int slot = (row * kMaxRanks + rank) * kMaxBlocks + b;
    __hip_atomic_store(peers.flag[t] + slot, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = peers.flag[rank] + (row * kMaxRanks + t) * kMaxBlocks + b;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (wall_clock64() - t0 > kSpinTicks) {
        atomicExch(err, 1 + t);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
}

// Two-shot (reduce-scatter + all-gather over P2P) for mid-size messages: rank r owns slice r and
// reduces it (reading (N-1)/N of the data from peers), then every rank gathers the other owners'
// reduced slices.  Per-GPU xGMI traffic 2(N-1)/N * n instead of (N-1) * n for one-shot.
// Staging per rank: [parity][input | reduced] of cap floats each; flag rows 1 and 2.
__global__ __launch_bounds__(kThreads) void twoshot_ar_k(const float* __restrict__ in, float* out, long n,
                                                         long cap, int rank, int world, Peers peers,
                                                         unsigned* epochs, int* err) {
  const int b = blockIdx.x, G = gridDim.x;
  const unsigned e = epochs[b] + 1;
  const long base = (long)(e & 1u) * 2 * cap;
  long L = (n + world - 1) / world;
  L = (L + 3) & ~3L;
  long per = (L + G - 1) / G;
  per = (per + 3) & ~3L;
  auto sub = [&](int slice, long& lo, long& hi) {
    lo = (long)slice * L + (long)b * per;
    hi = lo + per;
    const long send = (long)slice * L + L;
    if (hi > send) hi = send;
    if (hi > n) hi = n;
    if (lo > hi) lo = hi;
  };
  long lo, hi;
  for (int sl = 0; sl < world; ++sl) {
    sub(sl, lo, hi);
    copy_range(peers.buf[rank] + base, in, lo, hi);
  }
  flag_round(peers, rank, world, 1, b, e, err);
  sub(rank, lo, hi);
  float* red = peers.buf[rank] + base + cap;
  for (long i = lo + 4L * threadIdx.x; i < hi; i += 4L * kThreads) {
    if (i + 3 < hi) {
      float4 s = *reinterpret_cast<const float4*>(peers.buf[0] + base + i);
      for (int p = 1; p < world; ++p) {
        const float4 v = *reinterpret_cast<const float4*>(peers.buf[p] + base + i);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      *reinterpret_cast<float4*>(red + i) = s;
      *reinterpret_cast<float4*>(out + i) = s;
    } else {
      for (long j = i; j < hi; ++j) {
        float s = peers.buf[0][base + j];
        for (int p = 1; p < world; ++p) s += peers.buf[p][base + j];
        red[j] = s;
        out[j] = s;
      }
    }
  }
  flag_round(peers, rank, world, 2, b, e, err);
  for (int k = 1; k < world; ++k) {
    const int p = (rank + k) % world;  // stagger so the N-1 peers are read over different links at once
    sub(p, lo, hi);
    copy_range(out, peers.buf[p] + base + cap, lo, hi);
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

py::bytes handle_of(u ptr) {
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

}  // namespace

PYBIND11_MODULE(_hopsx_comm, m) {
  m.doc() = "hopsx one-shot xGMI all-reduce over IPC-mapped peer buffers (gfx950)";
  m.attr("MAX_RANKS") = kMaxRanks;
  m.attr("MAX_BLOCKS") = kMaxBlocks;
  m.attr("THREADS") = kThreads;
  m.attr("FLAG_ROWS") = 3;  // row 0: one-shot, rows 1-2: the two rounds of two-shot

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

  // out = sum over ranks of in (fp32, n elements, n <= cap); blocks <= MAX_BLOCKS, identical on all
  // ranks; epochs: int32[MAX_BLOCKS] device counters (zeroed once); err: int32 device flag
  // two_shot: reduce-scatter + all-gather variant (staging must hold 4 * cap floats)
  m.def("allreduce_f32", [](u in, u out, long n, long cap, int rank, int world, std::vector<u> bufs,
                            std::vector<u> flags, u epochs, u err, int blocks, u stream, bool two_shot) {
    if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) throw std::runtime_error("bad rank/world");
    if ((int)bufs.size() != world || (int)flags.size() != world) throw std::runtime_error("need one ptr per rank");
    if (n < 0 || n > cap) throw std::runtime_error("n exceeds the staging capacity");
    if (blocks < 1 || blocks > kMaxBlocks) throw std::runtime_error("blocks out of range");
    if ((in | out) & 15u) throw std::runtime_error("in/out must be 16-B aligned");
    Peers pr{};
    for (int i = 0; i < world; ++i) {
      pr.buf[i] = reinterpret_cast<float*>(bufs[i]);
      pr.flag[i] = reinterpret_cast<unsigned*>(flags[i]);
    }
    hipLaunchKernelGGL(two_shot ? twoshot_ar_k : oneshot_ar_k, dim3(blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const float*>(in), reinterpret_cast<float*>(out), n, cap, rank, world, pr,
                       reinterpret_cast<unsigned*>(epochs), reinterpret_cast<int*>(err));
    HIP_OK(hipGetLastError());
  });
}
