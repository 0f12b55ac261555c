// Feature-store column statistics on the GPU: descriptive stats (count of
// non-NaN, sum, sum of squares, min, max), per-column histograms and the
// centred Gram matrix for Pearson correlations.  These back
// FeatureGroup.statistics and the data-validation rule evaluator
// (reference: statistics_config at notebooks/featurestore/hsfs/basics/feature_engineering.ipynb:182,
//  Deequ rules at notebooks/featurestore/hsfs/data_validation/feature_validation_python.ipynb:218-242).
#include "common.h"
#include "ops_api.h"

__device__ __forceinline__ void atomic_min_f(float* a, float v) {
  if (v >= 0.f) atomicMin((int*)a, __float_as_int(v));
  else atomicMax((unsigned*)a, __float_as_uint(v));
}
__device__ __forceinline__ void atomic_max_f(float* a, float v) {
  if (v >= 0.f) atomicMax((int*)a, __float_as_int(v));
  else atomicMin((unsigned*)a, __float_as_uint(v));
}

// out_stats[c*5 + {0..4}] = {count, sum, sumsq, min, max}; caller initialises min=+inf, max=-inf
__global__ __launch_bounds__(256) void colstats_k(const float* __restrict__ x, int rows, int cols, int rpb,
                                                  float* __restrict__ st) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float n = 0.f, s = 0.f, q = 0.f, mn = INFINITY, mx = -INFINITY;
  if (c < cols)
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) {
      const float v = x[(long)r * cols + c];
      if (v != v) continue;  // NaN = missing
      n += 1.f;
      s += v;
      q += v * v;
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
  __shared__ float red[5][4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  red[0][w][l] = n; red[1][w][l] = s; red[2][w][l] = q; red[3][w][l] = mn; red[4][w][l] = mx;
  __syncthreads();
  if (threadIdx.x < 64 && c < cols) {
    float a = 0.f, b = 0.f, d = 0.f, e = INFINITY, f = -INFINITY;
    for (int k = 0; k < 4; ++k) {
      a += red[0][k][l]; b += red[1][k][l]; d += red[2][k][l];
      e = fminf(e, red[3][k][l]); f = fmaxf(f, red[4][k][l]);
    }
    atomicAdd(st + c * 5 + 0, a);
    atomicAdd(st + c * 5 + 1, b);
    atomicAdd(st + c * 5 + 2, d);
    if (e != INFINITY) atomic_min_f(st + c * 5 + 3, e);
    if (f != -INFINITY) atomic_max_f(st + c * 5 + 4, f);
  }
}

__global__ __launch_bounds__(256) void colhist_k(const float* __restrict__ x, int rows, int cols,
                                                 const float* __restrict__ mins, const float* __restrict__ maxs,
                                                 int bins, unsigned* __restrict__ hist) {
  const long total = (long)rows * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = i % cols;
    const float v = x[i];
    if (v != v) continue;
    const float lo = mins[c], hi = maxs[c];
    int b = (hi > lo) ? (int)((v - lo) / (hi - lo) * bins) : 0;
    b = b < 0 ? 0 : (b >= bins ? bins - 1 : b);
    atomicAdd(hist + (long)c * bins + b, 1u);
  }
}

// gram[i][j] = sum_r (x[r][i]-mean[i]) * (x[r][j]-mean[j]); 16x16 output tile per block, rows split on grid.z
__global__ __launch_bounds__(256) void gram_k(const float* __restrict__ x, const float* __restrict__ mean, int rows,
                                              int cols, int rpb, float* __restrict__ gram) {
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  const int r0 = blockIdx.z * rpb, r1 = min(rows, r0 + rpb);
  __shared__ float ti[64][17], tj[64][17];
  float acc = 0.f;
  for (int rb = r0; rb < r1; rb += 64) {
    for (int t = threadIdx.x; t < 64 * 16; t += 256) {
      const int rr = t >> 4, cc = t & 15;
      const int r = rb + rr;
      const int ci = blockIdx.y * 16 + cc, cj = blockIdx.x * 16 + cc;
      float a = 0.f, b = 0.f;
      if (r < r1) {
        if (ci < cols) { a = x[(long)r * cols + ci]; a = (a != a) ? 0.f : a - mean[ci]; }
        if (cj < cols) { b = x[(long)r * cols + cj]; b = (b != b) ? 0.f : b - mean[cj]; }
      }
      ti[rr][cc] = a;
      tj[rr][cc] = b;
    }
    __syncthreads();
#pragma unroll 8
    for (int rr = 0; rr < 64; ++rr) acc += ti[rr][threadIdx.x >> 4] * tj[rr][threadIdx.x & 15];
    __syncthreads();
  }
  if (i < cols && j < cols) atomicAdd(gram + (long)i * cols + j, acc);
}

// fp64 variant for the data-validation rules (Deequ computes in double): per column
// out[c*7 + {0..6}] = {count, sum, sumsq, min, max, #(v >= 0), #(v > 0)} over non-NaN values.
// One workgroup per (64-column slab, row chunk), fp64 partials combined with fp64 atomics; min/max
// via a CAS loop on the double's bits (caller initialises min = +inf, max = -inf).
__device__ inline void atomic_min_d(double* a, double v) {
  unsigned long long* p = (unsigned long long*)a;
  unsigned long long old = *p;
  while (v < __longlong_as_double((long long)old)) {
    const unsigned long long prev = atomicCAS(p, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}
__device__ inline void atomic_max_d(double* a, double v) {
  unsigned long long* p = (unsigned long long*)a;
  unsigned long long old = *p;
  while (v > __longlong_as_double((long long)old)) {
    const unsigned long long prev = atomicCAS(p, old, (unsigned long long)__double_as_longlong(v));
    if (prev == old) break;
    old = prev;
  }
}

__global__ __launch_bounds__(256) void colstats64_k(const double* __restrict__ x, int rows, int cols, int rpb,
                                                    double* __restrict__ st) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  double n = 0, s = 0, q = 0, mn = INFINITY, mx = -INFINITY, nn = 0, np_ = 0;
  if (c < cols)
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) {
      const double v = x[(long)r * cols + c];
      if (v != v) continue;
      n += 1;
      s += v;
      q += v * v;
      mn = fmin(mn, v);
      mx = fmax(mx, v);
      nn += v >= 0;
      np_ += v > 0;
    }
  __shared__ double red[7][4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  red[0][w][l] = n; red[1][w][l] = s; red[2][w][l] = q; red[3][w][l] = mn; red[4][w][l] = mx;
  red[5][w][l] = nn; red[6][w][l] = np_;
  __syncthreads();
  if (threadIdx.x < 64 && c < cols) {
    double a[7] = {0, 0, 0, INFINITY, -INFINITY, 0, 0};
    for (int k = 0; k < 4; ++k) {
      a[0] += red[0][k][l]; a[1] += red[1][k][l]; a[2] += red[2][k][l];
      a[3] = fmin(a[3], red[3][k][l]); a[4] = fmax(a[4], red[4][k][l]);
      a[5] += red[5][k][l]; a[6] += red[6][k][l];
    }
    double* o = st + (long)c * 7;
    atomicAdd(o + 0, a[0]);
    atomicAdd(o + 1, a[1]);
    atomicAdd(o + 2, a[2]);
    if (a[3] != INFINITY) atomic_min_d(o + 3, a[3]);
    if (a[4] != -INFINITY) atomic_max_d(o + 4, a[4]);
    atomicAdd(o + 5, a[5]);
    atomicAdd(o + 6, a[6]);
  }
}

extern "C" int hopsx_column_stats64(const double* x, int rows, int cols, double* out_stats, hipStream_t st) {
  const int gx = (cols + 63) / 64;
  int gy = (rows + 2047) / 2048;
  const int max_gy = (2048 + gx - 1) / gx;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  const int rpb = (rows + gy - 1) / gy;
  hipLaunchKernelGGL(colstats64_k, dim3(gx, gy), dim3(256), 0, st, x, rows, cols, rpb, out_stats);
  return (int)hipGetLastError();
}

extern "C" int hopsx_column_stats(const float* x, int rows, int cols, float* out_stats, hipStream_t st) {
  const int gx = (cols + 63) / 64;
  int gy = (rows + 1023) / 1024;
  const int max_gy = (2048 + gx - 1) / gx;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  const int rpb = (rows + gy - 1) / gy;
  hipLaunchKernelGGL(colstats_k, dim3(gx, gy), dim3(256), 0, st, x, rows, cols, rpb, out_stats);
  return (int)hipGetLastError();
}

extern "C" int hopsx_column_hist(const float* x, int rows, int cols, const float* mins, const float* maxs, int bins,
                                 unsigned* hist, hipStream_t st) {
  long n = (long)rows * cols;
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(colhist_k, dim3(g), dim3(256), 0, st, x, rows, cols, mins, maxs, bins, hist);
  return (int)hipGetLastError();
}

extern "C" int hopsx_gram(const float* x, const float* mean, int rows, int cols, float* gram, hipStream_t st) {
  const int t = (cols + 15) / 16;
  int gz = (rows + 4095) / 4096;
  const int max_gz = (1024 + t * t - 1) / (t * t);
  if (gz > max_gz) gz = max_gz;
  if (gz < 1) gz = 1;
  const int rpb = (rows + gz - 1) / gz;
  hipLaunchKernelGGL(gram_k, dim3(t, t, gz), dim3(256), 0, st, x, mean, rows, cols, rpb, gram);
  return (int)hipGetLastError();
}
