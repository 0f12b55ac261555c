// Range-window aggregates on the GPU: Spark's
//   F.sum(v).over(Window.partitionBy(keys).orderBy(ts).rangeBetween(lo, hi))
// (notebooks/featurestore/hsfs/basics/feature_engineering.ipynb:229-249: sales over the last
// 30/90/180/365 days per (store, dept) and per store, rangeBetween(days(-N), days(-1))).
//
// The host sorts the rows by (partition, ts) and passes the partition boundaries; the device
//   1. builds the exclusive fp64 prefix sum P of the values (three-pass scan: tile sums, a scan of
//      the tile sums, tile rescans — fp64 so differences of large running sums stay exact enough);
//   2. answers every (row, window) pair with two binary searches inside the row's partition
//      (first ts >= ts_i + lo, last ts <= ts_i + hi) and one difference P[b] - P[a]; an empty range
//      is Spark's null (NaN here, count 0).
// One launch answers all W windows of all rows; O(n log n) work, no per-window passes.
#include "common.h"
#include "ops_api.h"

namespace {

constexpr int kScanThreads = 256;
constexpr int kPer = 16;                      // elements per thread in a scan tile
constexpr int kTile = kScanThreads * kPer;    // 4096

__device__ inline double block_exclusive_scan(double v, double* sh, double& total) {
  // Hillis-Steele over the 256 thread totals in LDS (256 doubles): log2(256) = 8 steps
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < kScanThreads; o <<= 1) {
    const double a = t >= o ? sh[t - o] : 0.0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  total = sh[kScanThreads - 1];
  const double incl = sh[t];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(kScanThreads) void tile_sum_k(const double* __restrict__ v, long n,
                                                           double* __restrict__ tsum) {
  __shared__ double sh[kScanThreads];
  const long base = (long)blockIdx.x * kTile + (long)threadIdx.x * kPer;
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) s += base + j < n ? v[base + j] : 0.0;
  double total;
  block_exclusive_scan(s, sh, total);
  if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

// one workgroup: exclusive scan of the tile sums in place (any count, 256 per chunk)
__global__ __launch_bounds__(kScanThreads) void scan_tiles_k(double* __restrict__ tsum, long ntiles) {
  __shared__ double sh[kScanThreads];
  double carry = 0.0;
  for (long c = 0; c < ntiles; c += kScanThreads) {
    const long i = c + threadIdx.x;
    const double x = i < ntiles ? tsum[i] : 0.0;
    double total;
    const double ex = block_exclusive_scan(x, sh, total);
    if (i < ntiles) tsum[i] = carry + ex;
    carry += total;
  }
}

// P[i] = sum_{j < i} v[j] for i in [0, n]  (P has n + 1 entries)
__global__ __launch_bounds__(kScanThreads) void tile_rescan_k(const double* __restrict__ v, long n,
                                                              const double* __restrict__ toff, double* __restrict__ P) {
  __shared__ double sh[kScanThreads];
  const long base = (long)blockIdx.x * kTile + (long)threadIdx.x * kPer;
  double loc[kPer];
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    loc[j] = base + j < n ? v[base + j] : 0.0;
    s += loc[j];
  }
  double total;
  double run = block_exclusive_scan(s, sh, total) + toff[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (base + j < n) P[base + j] = run;
    run += loc[j];
  }
  if (base < n && base + kPer >= n) P[n] = run;  // the thread holding the last element writes the total
}

// first index in [a, b) with ts >= x   (ts ascending inside [a, b))
__device__ inline long lower_bound_i64(const long* ts, long a, long b, long x) {
  while (a < b) {
    const long m = (a + b) >> 1;
    if (ts[m] < x) a = m + 1;
    else b = m;
  }
  return a;
}
// first index in [a, b) with ts > x
__device__ inline long upper_bound_i64(const long* ts, long a, long b, long x) {
  while (a < b) {
    const long m = (a + b) >> 1;
    if (ts[m] <= x) a = m + 1;
    else b = m;
  }
  return a;
}

__global__ __launch_bounds__(256) void range_window_k(const long* __restrict__ ts, const int* __restrict__ seg,
                                                      const long* __restrict__ seg_off, const double* __restrict__ P,
                                                      long n, const long* __restrict__ lo, const long* __restrict__ hi,
                                                      int W, double* __restrict__ sum, int* __restrict__ cnt) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int s = seg[i];
    const long a = seg_off[s], b = seg_off[s + 1];
    const long t = ts[i];
    for (int w = 0; w < W; ++w) {
      const long f = lower_bound_i64(ts, a, b, t + lo[w]);
      const long l = upper_bound_i64(ts, a, b, t + hi[w]);  // one past the last
      const long c = l > f ? l - f : 0;
      sum[i * W + w] = c ? P[l] - P[f] : __builtin_nan("");
      if (cnt) cnt[i * W + w] = (int)c;
    }
  }
}

}  // namespace

extern "C" int hopsx_prefix_sum_f64(const double* v, long n, double* P, double* work, hipStream_t st) {
  // work: >= ceil(n / 4096) doubles
  if (n < 0) return -2;
  const long nt = n > 0 ? (n + kTile - 1) / kTile : 1;
  if (n == 0) {
    hipMemsetAsync(P, 0, sizeof(double), st);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(tile_sum_k, dim3((unsigned)nt), dim3(kScanThreads), 0, st, v, n, work);
  hipLaunchKernelGGL(scan_tiles_k, dim3(1), dim3(kScanThreads), 0, st, work, nt);
  hipLaunchKernelGGL(tile_rescan_k, dim3((unsigned)nt), dim3(kScanThreads), 0, st, v, n, work, P);
  return (int)hipGetLastError();
}

extern "C" int hopsx_range_window(const long* ts, const int* seg, const long* seg_off, const double* P, long n,
                                  const long* lo, const long* hi, int W, double* sum, int* cnt, hipStream_t st) {
  if (n < 0 || W < 1) return -2;
  if (n == 0) return 0;
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(range_window_k, dim3((unsigned)g), dim3(256), 0, st, ts, seg, seg_off, P, n, lo, hi, W, sum, cnt);
  return (int)hipGetLastError();
}
