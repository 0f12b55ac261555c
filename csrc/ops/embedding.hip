// Embedding-bag (sum / mean) for the wide & deep and census models.  The
// forward writes straight into a column slice of the concatenated feature
// matrix (ldo = row stride of that matrix), so "embed + concat" is one pass.
// The backward is a scatter-add into the fp32 gradient of the table.
#include "common.h"
#include "ops_api.h"

// one wave per bag, lanes stride over the embedding dim
__global__ __launch_bounds__(256) void embag_fwd_k(const float* __restrict__ table, const long* __restrict__ idx,
                                                   const long* __restrict__ offs, int nbags, int dim, long nidx,
                                                   int mode, void* __restrict__ out, int of32, long ldo) {
  const int lane = threadIdx.x & 63;
  for (long bag = (long)blockIdx.x * 4 + (threadIdx.x >> 6); bag < nbags; bag += (long)gridDim.x * 4) {
    const long s = offs ? offs[bag] : bag;
    const long e = offs ? (bag + 1 < nbags ? offs[bag + 1] : nidx) : bag + 1;
    const float sc = (mode == 1 && e > s) ? 1.f / (float)(e - s) : 1.f;
    for (int d = lane; d < dim; d += 64) {
      float acc = 0.f;
      for (long j = s; j < e; ++j) acc += table[idx[j] * (long)dim + d];
      acc *= sc;
      if (of32) ((float*)out)[bag * ldo + d] = acc;
      else ((bf16_raw*)out)[bag * ldo + d] = f2bf(acc);
    }
  }
}

__global__ __launch_bounds__(256) void embag_bwd_k(const void* __restrict__ dout, int df32, long ldo,
                                                   const long* __restrict__ idx, const long* __restrict__ offs,
                                                   int nbags, int dim, long nidx, int mode,
                                                   float* __restrict__ dtable) {
  const int lane = threadIdx.x & 63;
  for (long bag = (long)blockIdx.x * 4 + (threadIdx.x >> 6); bag < nbags; bag += (long)gridDim.x * 4) {
    const long s = offs ? offs[bag] : bag;
    const long e = offs ? (bag + 1 < nbags ? offs[bag + 1] : nidx) : bag + 1;
    const float sc = (mode == 1 && e > s) ? 1.f / (float)(e - s) : 1.f;
    for (int d = lane; d < dim; d += 64) {
      const float g = (df32 ? ((const float*)dout)[bag * ldo + d] : bf2f(((const bf16_raw*)dout)[bag * ldo + d])) * sc;
      for (long j = s; j < e; ++j) atomicAdd(dtable + idx[j] * (long)dim + d, g);
    }
  }
}

extern "C" int hopsx_embedding_bag_fwd(const float* table, const long* idx, const long* offsets, int nbags, int dim,
                                       long nidx, int mode, void* out, int out_f32, long ldo, hipStream_t st) {
  int g = (nbags + 3) / 4;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(embag_fwd_k, dim3(g), dim3(256), 0, st, table, idx, offsets, nbags, dim, nidx, mode, out, out_f32,
                     ldo);
  return (int)hipGetLastError();
}

extern "C" int hopsx_embedding_bag_bwd(const void* dout, int dout_f32, long ldo, const long* idx, const long* offsets,
                                       int nbags, int dim, long nidx, int mode, float* dtable, hipStream_t st) {
  int g = (nbags + 3) / 4;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(embag_bwd_k, dim3(g), dim3(256), 0, st, dout, dout_f32, ldo, idx, offsets, nbags, dim, nidx, mode,
                     dtable);
  return (int)hipGetLastError();
}
