// Embedding-bag (sum / mean) for the wide & deep and census models.  The
// forward writes straight into a column slice of the concatenated feature
// matrix (ldo = row stride of that matrix), so "embed + concat" is one pass.
// The backward is a scatter-add into the fp32 gradient of the table.
#include "common.h"
#include "ops_api.h"

HOPSX_DBG_TU(embedding)

// Bag [s, e) of bag `bag`: CSR offsets, or fixed-length bags (bag_len rows each).
__device__ __forceinline__ void bag_range(const long* __restrict__ offs, long bag, int nbags, long nidx, int bag_len,
                                          long& s, long& e) {
  if (offs) {
    s = offs[bag];
    e = bag + 1 < nbags ? offs[bag + 1] : nidx;
    if (!hx_guard(0 <= s && s <= e && e <= nidx)) e = s;  // malformed offsets: an empty bag
  } else {
    s = bag * (long)bag_len;
    e = s + bag_len;
  }
}

__device__ __forceinline__ void store_out(void* out, int of32, long i, float v) {
  if (of32) ((float*)out)[i] = v;
  else ((bf16_raw*)out)[i] = f2bf(v);
}

// dim > 16: one wave per bag, lanes stride over the embedding dim (coalesced row reads)
__global__ __launch_bounds__(256) void embag_fwd_k(const float* __restrict__ table, const long* __restrict__ idx,
                                                   const long* __restrict__ offs, int nbags, int dim, long nidx,
                                                   int bag_len, int mode, void* __restrict__ out, int of32, long ldo,
                                                   long rows) {
  const int lane = threadIdx.x & 63;
  for (long bag = (long)blockIdx.x * 4 + (threadIdx.x >> 6); bag < nbags; bag += (long)gridDim.x * 4) {
    long s, e;
    bag_range(offs, bag, nbags, nidx, bag_len, s, e);
    const float sc = (mode == 1 && e > s) ? 1.f / (float)(e - s) : 1.f;
    for (int d = lane; d < dim; d += 64) {
      float acc = 0.f;
      for (long j = s; j < e; ++j) {
        const long r = idx[j];
        if (hx_guard((unsigned long)r < (unsigned long)rows)) acc += table[r * dim + d];  // an id out of range adds 0
      }
      store_out(out, of32, bag * ldo + d, acc * sc);
    }
  }
}

// dim <= 16 (wide/linear models: dim 1): one thread per (bag, d) so a wave covers
// 64/dim bags instead of idling 64-dim lanes
__global__ __launch_bounds__(256) void embag_fwd_small_k(const float* __restrict__ table, const long* __restrict__ idx,
                                                         const long* __restrict__ offs, int nbags, int dim, long nidx,
                                                         int bag_len, int mode, void* __restrict__ out, int of32,
                                                         long ldo, long rows) {
  const long total = (long)nbags * dim;
  for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const long bag = t / dim;
    const int d = (int)(t - bag * dim);
    long s, e;
    bag_range(offs, bag, nbags, nidx, bag_len, s, e);
    float acc = 0.f;
    for (long j = s; j < e; ++j) {
      const long r = idx[j];
      if (hx_guard((unsigned long)r < (unsigned long)rows)) acc += table[r * dim + d];
    }
    if (mode == 1 && e > s) acc *= 1.f / (float)(e - s);
    store_out(out, of32, bag * ldo + d, acc);
  }
}

__device__ __forceinline__ float load_g(const void* dout, int df32, long i) {
  return df32 ? ((const float*)dout)[i] : bf2f(((const bf16_raw*)dout)[i]);
}

__global__ __launch_bounds__(256) void embag_bwd_k(const void* __restrict__ dout, int df32, long ldo,
                                                   const long* __restrict__ idx, const long* __restrict__ offs,
                                                   int nbags, int dim, long nidx, int bag_len, int mode,
                                                   float* __restrict__ dtable, long rows) {
  const int lane = threadIdx.x & 63;
  for (long bag = (long)blockIdx.x * 4 + (threadIdx.x >> 6); bag < nbags; bag += (long)gridDim.x * 4) {
    long s, e;
    bag_range(offs, bag, nbags, nidx, bag_len, s, e);
    const float sc = (mode == 1 && e > s) ? 1.f / (float)(e - s) : 1.f;
    for (int d = lane; d < dim; d += 64) {
      const float g = load_g(dout, df32, bag * ldo + d) * sc;
      for (long j = s; j < e; ++j) {
        const long r = idx[j];
        if (hx_guard((unsigned long)r < (unsigned long)rows)) atomicAdd(dtable + r * dim + d, g);
      }
    }
  }
}

__global__ __launch_bounds__(256) void embag_bwd_small_k(const void* __restrict__ dout, int df32, long ldo,
                                                         const long* __restrict__ idx, const long* __restrict__ offs,
                                                         int nbags, int dim, long nidx, int bag_len, int mode,
                                                         float* __restrict__ dtable, long rows) {
  const long total = (long)nbags * dim;
  for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const long bag = t / dim;
    const int d = (int)(t - bag * dim);
    long s, e;
    bag_range(offs, bag, nbags, nidx, bag_len, s, e);
    float g = load_g(dout, df32, bag * ldo + d);
    if (mode == 1 && e > s) g *= 1.f / (float)(e - s);
    for (long j = s; j < e; ++j) {
      const long r = idx[j];
      if (hx_guard((unsigned long)r < (unsigned long)rows)) atomicAdd(dtable + r * dim + d, g);
    }
  }
}

static int embag_grid(int nbags, int dim, bool small) {
  long work = small ? ((long)nbags * dim + 255) / 256 : ((long)nbags + 3) / 4;
  return (int)(work < 1 ? 1 : (work > 4096 ? 4096 : work));
}

extern "C" int hopsx_embedding_bag_fwd(const float* table, const long* idx, const long* offsets, int nbags, int dim,
                                       long nidx, int bag_len, int mode, void* out, int out_f32, long ldo,
                                       long rows, hipStream_t st) {
  const bool small = dim <= 16;
  const int g = embag_grid(nbags, dim, small);
  if (small)
    hipLaunchKernelGGL(embag_fwd_small_k, dim3(g), dim3(256), 0, st, table, idx, offsets, nbags, dim, nidx, bag_len,
                       mode, out, out_f32, ldo, rows);
  else
    hipLaunchKernelGGL(embag_fwd_k, dim3(g), dim3(256), 0, st, table, idx, offsets, nbags, dim, nidx, bag_len, mode,
                       out, out_f32, ldo, rows);
  return (int)hipGetLastError();
}

extern "C" int hopsx_embedding_bag_bwd(const void* dout, int dout_f32, long ldo, const long* idx, const long* offsets,
                                       int nbags, int dim, long nidx, int bag_len, int mode, float* dtable,
                                       long rows, hipStream_t st) {
  const bool small = dim <= 16;
  const int g = embag_grid(nbags, dim, small);
  if (small)
    hipLaunchKernelGGL(embag_bwd_small_k, dim3(g), dim3(256), 0, st, dout, dout_f32, ldo, idx, offsets, nbags, dim,
                       nidx, bag_len, mode, dtable, rows);
  else
    hipLaunchKernelGGL(embag_bwd_k, dim3(g), dim3(256), 0, st, dout, dout_f32, ldo, idx, offsets, nbags, dim, nidx,
                       bag_len, mode, dtable, rows);
  return (int)hipGetLastError();
}
