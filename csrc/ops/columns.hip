// Columnar -> row-major fp32 ingest (io/parquet.py, featurestore to_device): ONE launch per staged
// chunk converts every column of a Parquet row group (int8 .. int64, f16 / f32 / f64, as Arrow
// decoded them into the pinned ring and the H2D copy moved them) and interleaves them into the
// [rows][ld] fp32 matrix the models read.  Replaces one torch copy_ launch per column.
// 256 rows per workgroup: each column is read coalesced (consecutive rows on consecutive lanes),
// the [256][k] tile goes through LDS so the row-major output is written with consecutive
// addresses when ld == k.
#include <hip/hip_fp16.h>

#include "common.h"
#include "ops_api.h"

namespace {

constexpr int kMaxCols = 16;

struct ColSet {
  const void* p[kMaxCols];
  int dt[kMaxCols];  // 0 f32, 1 f64, 2 i64, 3 i32, 4 i16, 5 i8, 6 u8, 7 f16
  int k;
};

__device__ __forceinline__ float col_at(const ColSet& c, int j, long r) {
  switch (c.dt[j]) {
    case 0: return ((const float*)c.p[j])[r];
    case 1: return (float)((const double*)c.p[j])[r];
    case 2: return (float)((const long long*)c.p[j])[r];
    case 3: return (float)((const int*)c.p[j])[r];
    case 4: return (float)((const short*)c.p[j])[r];
    case 5: return (float)((const signed char*)c.p[j])[r];
    case 6: return (float)((const unsigned char*)c.p[j])[r];
    default: return __half2float(((const __half*)c.p[j])[r]);
  }
}

__global__ __launch_bounds__(256) void cols_to_f32_k(ColSet c, float* __restrict__ out, long ld, long rows) {
  __shared__ float tile[256 * (kMaxCols + 1)];
  const long r0 = (long)blockIdx.x * 256;
  const int tid = threadIdx.x, k = c.k, stride = k + 1;  // +1: odd row stride, no bank conflicts
  const long r = r0 + tid;
  for (int j = 0; j < k; ++j) tile[tid * stride + j] = r < rows ? col_at(c, j, r) : 0.f;
  __syncthreads();
  const long nrow = rows - r0 < 256 ? rows - r0 : 256;
  for (long i = tid; i < nrow * k; i += 256) {
    const long rr = i / k;
    const int j = (int)(i - rr * k);
    out[(r0 + rr) * ld + j] = tile[rr * stride + j];
  }
}

}  // namespace

extern "C" int hopsx_cols_to_f32(const void* const* cols, const int* dtypes, int k, long rows, float* out, long ld,
                                 hipStream_t st) {
  if (k < 1 || k > kMaxCols || rows < 0 || ld < k) return -2;
  if (rows == 0) return 0;
  ColSet c{};
  for (int j = 0; j < k; ++j) {
    if (dtypes[j] < 0 || dtypes[j] > 7 || !cols[j]) return -2;
    c.p[j] = cols[j];
    c.dt[j] = dtypes[j];
  }
  c.k = k;
  const long g = (rows + 255) / 256;
  if (g > 0x7fffffffL) return -2;
  hipLaunchKernelGGL(cols_to_f32_k, dim3((unsigned)g), dim3(256), 0, st, c, out, ld, rows);
  return (int)hipGetLastError();
}
