// TFX Transform on the GPU: the apply half of the Chicago-taxi preprocessing_fn.
//
// The reference README names a TFX Chicago-taxi pipeline whose Transform stage is absent from the
// snapshot (README.md:99-112).  Its preprocessing_fn (public TFX taxi example) is
//   dense    : tft.scale_to_z_score(fill_in_missing(x))                  trip_miles, fare, trip_seconds
//   bucket   : tft.bucketize(fill_in_missing(x), 10) (quantile bounds)   pickup/dropoff lat/long
//   vocab    : tft.compute_and_apply_vocabulary(top_k 1000, 10 OOV)      payment_type, company
//   identity : fill_in_missing(x), identity column (out of range -> 0)   hour/day/month, tracts, areas
//   label    : fare missing -> 0, else tips > 0.2 * fare
// The analyze half (means/variances, quantile histograms) runs on the stats.hip kernels; the
// vocabulary lookup of the two string columns is a host dictionary (strings never reach the GPU, the
// ids do).  This kernel applies everything else in ONE pass over the raw rows: one thread per row
// reads its raw fp32 columns (NaN = missing) and writes the z-scored dense block, the 13 wide ids
// already offset into the concatenated one-hot space of the wide&deep model, and the label.
#include "common.h"
#include "ops_api.h"

namespace {

constexpr int kMaxCols = 16;     // per role
constexpr int kMaxBounds = 31;   // bucket boundaries per column (<= 32 buckets)

struct TransformSpec {
  int F;                         // raw columns per row
  int nd, nb, ni, nv;            // dense, bucket, identity, vocab (precomputed id) columns
  int dcol[kMaxCols];
  float mean[kMaxCols], inv_std[kMaxCols];
  int bcol[kMaxCols], nbound[kMaxCols];
  float bound[kMaxCols][kMaxBounds];
  int icol[kMaxCols], icard[kMaxCols];
  int vcard[kMaxCols];
  long off[3 * kMaxCols];        // wide-id offset of each cat output column (bucket, vocab, identity order)
  int fare_col, tips_col;        // label inputs (-1: no label)
  float tip_frac;
};

__global__ __launch_bounds__(256) void taxi_transform_k(const float* __restrict__ raw, const int* __restrict__ vids,
                                                        long n, TransformSpec s, float* __restrict__ dense,
                                                        long* __restrict__ cat, float* __restrict__ label) {
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < n; r += (long)gridDim.x * blockDim.x) {
    const float* row = raw + r * s.F;
    for (int j = 0; j < s.nd; ++j) {
      float v = row[s.dcol[j]];
      v = v != v ? 0.f : v;  // fill_in_missing (default 0)
      dense[r * s.nd + j] = (v - s.mean[j]) * s.inv_std[j];
    }
    const int nc = s.nb + s.nv + s.ni;
    long* out = cat + r * nc;
    for (int j = 0; j < s.nb; ++j) {
      float v = row[s.bcol[j]];
      v = v != v ? 0.f : v;
      int id = 0;  // apply_buckets: number of boundaries <= v
      for (int b = 0; b < s.nbound[j]; ++b) id += s.bound[j][b] <= v;
      out[j] = s.off[j] + id;
    }
    for (int j = 0; j < s.nv; ++j) {
      int id = vids[r * s.nv + j];
      id = id < 0 || id >= s.vcard[j] ? 0 : id;
      out[s.nb + j] = s.off[s.nb + j] + id;
    }
    for (int j = 0; j < s.ni; ++j) {
      const float v = row[s.icol[j]];
      int id = v != v ? 0 : (int)v;  // fill_in_missing, then identity column (default 0 out of range)
      id = id < 0 || id >= s.icard[j] ? 0 : id;
      out[s.nb + s.nv + j] = s.off[s.nb + s.nv + j] + id;
    }
    if (s.fare_col >= 0 && label) {
      const float fare = row[s.fare_col], tips = row[s.tips_col];
      label[r] = fare != fare ? 0.f : ((tips != tips ? 0.f : tips) > s.tip_frac * fare ? 1.f : 0.f);
    }
  }
}

}  // namespace

extern "C" int hopsx_taxi_transform(const float* raw, const int* vids, long n, const int* ints, const float* flts,
                                    const long* offs, float* dense, long* cat, float* label, hipStream_t st) {
  // ints: F, nd, nb, ni, nv, fare_col, tips_col, dcol[nd], bcol[nb], nbound[nb], icol[ni], icard[ni], vcard[nv]
  // flts: tip_frac, mean[nd], inv_std[nd], bound[nb][kMaxBounds]
  TransformSpec s{};
  int p = 0;
  s.F = ints[p++]; s.nd = ints[p++]; s.nb = ints[p++]; s.ni = ints[p++]; s.nv = ints[p++];
  s.fare_col = ints[p++]; s.tips_col = ints[p++];
  if (s.nd > kMaxCols || s.nb > kMaxCols || s.ni > kMaxCols || s.nv > kMaxCols || s.F < 1 || n < 0) return -2;
  for (int j = 0; j < s.nd; ++j) s.dcol[j] = ints[p++];
  for (int j = 0; j < s.nb; ++j) s.bcol[j] = ints[p++];
  for (int j = 0; j < s.nb; ++j) {
    s.nbound[j] = ints[p++];
    if (s.nbound[j] < 0 || s.nbound[j] > kMaxBounds) return -2;
  }
  for (int j = 0; j < s.ni; ++j) s.icol[j] = ints[p++];
  for (int j = 0; j < s.ni; ++j) s.icard[j] = ints[p++];
  for (int j = 0; j < s.nv; ++j) s.vcard[j] = ints[p++];
  int q = 0;
  s.tip_frac = flts[q++];
  for (int j = 0; j < s.nd; ++j) s.mean[j] = flts[q++];
  for (int j = 0; j < s.nd; ++j) s.inv_std[j] = flts[q++];
  for (int j = 0; j < s.nb; ++j)
    for (int b = 0; b < kMaxBounds; ++b) s.bound[j][b] = flts[q++];
  const int nc = s.nb + s.nv + s.ni;
  if (nc > 3 * kMaxCols) return -2;
  for (int j = 0; j < nc; ++j) s.off[j] = offs[j];
  for (int j = 0; j < s.nd; ++j)
    if (s.dcol[j] < 0 || s.dcol[j] >= s.F) return -2;
  for (int j = 0; j < s.nb; ++j)
    if (s.bcol[j] < 0 || s.bcol[j] >= s.F) return -2;
  for (int j = 0; j < s.ni; ++j)
    if (s.icol[j] < 0 || s.icol[j] >= s.F) return -2;
  if (s.fare_col >= s.F || s.tips_col >= s.F || (s.fare_col >= 0 && s.tips_col < 0)) return -2;
  if (s.nv > 0 && !vids) return -2;
  if (n == 0) return 0;
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(taxi_transform_k, dim3((unsigned)g), dim3(256), 0, st, raw, vids, n, s, dense, cat, label);
  return (int)hipGetLastError();
}

extern "C" int hopsx_transform_max_bounds() { return kMaxBounds; }
