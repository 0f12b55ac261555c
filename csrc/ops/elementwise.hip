// Memory-bound helpers: dropout (stateless counter RNG whose state lives on the
// device so graph replays draw fresh masks), dtype casts, the uint8 image
// "landing" normaliser, bias-gradient column sums and activation backward.
// bf16 streams are moved 8 elements (16 B) per lane where the layout allows.
#include "common.h"
#include "ops_api.h"

HOPSX_DET_TU(elementwise)

static inline int ew_grid(long n, int per_thread = 1) {
  long g = (n / per_thread + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}


__global__ void dropout_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y, long n, float p,
                          const unsigned long long* __restrict__ rng, unsigned salt) {
  const uint64_t key = drop_key(rng, salt);
  const float scale = 1.f / (1.f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float keep = uniform01(key, i) >= p ? scale : 0.f;
    y[i] = f2bf(bf2f(x[i]) * keep);
  }
}

__global__ void rng_adv_k(unsigned long long* rng) { rng[1] += 1; }

__global__ void cast_f32_bf16_k(const float* __restrict__ x, bf16_raw* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}
__global__ void cast_bf16_f32_k(const bf16_raw* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = bf2f(x[i]);
}

// y = x * scale + shift, uint8 -> bf16, 8 elements per lane when aligned
__global__ void u8_norm_k(const unsigned char* __restrict__ x, bf16_raw* __restrict__ y, long n, float scale,
                          float shift, int vec) {
  const long n8 = vec ? n / 8 : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const uint2 v = ((const uint2*)x)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (short)f2bf(((v.x >> (8 * j)) & 0xff) * scale + shift);
      o[j + 4] = (short)f2bf(((v.y >> (8 * j)) & 0xff) * scale + shift);
    }
    ((bf16x8*)y)[i] = o;
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i] * scale + shift);
}

// Per-channel image normalisation of uint8 NHWC pixels (C <= 4) -> bf16, optionally reversing the
// channel order (RGB -> BGR for caffe-style models): y[p][c] = x[p][rev ? C-1-c : c] * scale[c] + shift[c].
// One launch replaces the torch addcmul + bf16 cast pair (two at::native kernels) on the input path.
struct ChanAffine {
  float scale[4], shift[4];
};
__global__ void u8_norm_chan_k(const unsigned char* __restrict__ x, bf16_raw* __restrict__ y, long pixels, int C,
                               ChanAffine a, int rev) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < pixels; p += (long)gridDim.x * blockDim.x) {
    const unsigned char* px = x + p * C;
    bf16_raw* py = y + p * C;
    for (int c = 0; c < C; ++c) py[c] = f2bf(px[rev ? C - 1 - c : c] * a.scale[c] + a.shift[c]);
  }
}

// C <= 4 channels in, 8 out (channels C..7 zero): the layout of a stem conv whose input channels are
// zero-padded to 8 so it runs on the C % 8 == 0 MFMA conv paths; one 16-B store per pixel
__global__ void u8_norm_chan8_k(const unsigned char* __restrict__ x, bf16_raw* __restrict__ y, long pixels, int C,
                                ChanAffine a, int rev) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < pixels; p += (long)gridDim.x * blockDim.x) {
    const unsigned char* px = x + p * C;
    bf16x8 q = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < C) q[c] = (short)f2bf(px[rev ? C - 1 - c : c] * a.scale[c] + a.shift[c]);
    *(bf16x8*)(y + p * 8) = q;
  }
}

// out[n] += sum_m x[m][n]; one workgroup owns a column strip, rows split over gridDim.y
__global__ __launch_bounds__(256) void colsum_k(const bf16_raw* __restrict__ x, float* __restrict__ out, int M,
                                                int N, int rows_per_block) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float s = 0.f;
  if (n < N)
    for (int m = r0 + (threadIdx.x >> 6); m < r1; m += 4) s += bf2f(x[(long)m * N + n]);
  __shared__ float red[4][64];
  red[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  const bool det = det_on();
  const unsigned dmy = blockIdx.y * gridDim.x + blockIdx.x;
  if (det) det_turn_begin(DET_COLSUM, dmy);
  if (threadIdx.x < 64 && n < N) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(out + n, t);
  }
  if (det) det_turn_end(DET_COLSUM, dmy, gridDim.x * gridDim.y);
}

__global__ void act_bwd_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ y, bf16_raw* __restrict__ dx,
                          long n, int act) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dx[i] = f2bf(bf2f(dy[i]) * act_grad_from_out(bf2f(y[i]), act));
}

// dx = dy * act'(y) and colsum[n] += sum_m dx[m][n] in one pass (bias gradient of
// the layer whose activation output is y); one workgroup per (64-column strip, row slab)
__global__ __launch_bounds__(256) void act_bwd_colsum_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ y,
                                                        bf16_raw* __restrict__ dx, int M, int N, int act,
                                                        float* __restrict__ colsum, int rpb) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  float s = 0.f;
  if (n < N)
    for (int m = r0 + (threadIdx.x >> 6); m < r1; m += 4) {
      const long i = (long)m * N + n;
      float v = bf2f(dy[i]);
      if (y) v *= act_grad_from_out(bf2f(y[i]), act);
      dx[i] = f2bf(v);
      s += v;
    }
  if (!colsum) return;
  __shared__ float red[4][64];
  red[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  const bool det = det_on();
  const unsigned dmy = blockIdx.y * gridDim.x + blockIdx.x;
  if (det) det_turn_begin(DET_COLSUM, dmy);
  if (threadIdx.x < 64 && n < N)
    atomicAdd(colsum + n, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
  if (det) det_turn_end(DET_COLSUM, dmy, gridDim.x * gridDim.y);
}

__global__ void add_k(const bf16_raw* __restrict__ a, const bf16_raw* __restrict__ b, bf16_raw* __restrict__ o,
                      long n, int act) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    o[i] = f2bf(apply_act(bf2f(a[i]) + bf2f(b[i]), act));
}

extern "C" int hopsx_dropout_fwd(const void* x, void* y, long n, float p, const unsigned long long* rng,
                                 unsigned salt, hipStream_t st) {
  hipLaunchKernelGGL(dropout_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, n, p, rng,
                     salt);
  return (int)hipGetLastError();
}
// the backward of dropout is the same mask applied to dy
extern "C" int hopsx_dropout_bwd(const void* dy, void* dx, long n, float p, const unsigned long long* rng,
                                 unsigned salt, hipStream_t st) {
  return hopsx_dropout_fwd(dy, dx, n, p, rng, salt, st);
}
extern "C" int hopsx_rng_advance(unsigned long long* rng, hipStream_t st) {
  hipLaunchKernelGGL(rng_adv_k, dim3(1), dim3(1), 0, st, rng);
  return (int)hipGetLastError();
}
extern "C" int hopsx_cast_f32_bf16(const float* x, void* y, long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_k, dim3(ew_grid(n)), dim3(256), 0, st, x, (bf16_raw*)y, n);
  return (int)hipGetLastError();
}
extern "C" int hopsx_cast_bf16_f32(const void* x, float* y, long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_bf16_f32_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)x, y, n);
  return (int)hipGetLastError();
}
extern "C" int hopsx_u8_normalize_chan(const unsigned char* x, void* y, long pixels, int C, const float* scale,
                                       const float* shift, int rev, int cout, hipStream_t st) {
  if (C < 1 || C > 4 || pixels < 0 || (cout != C && cout != 8) || (cout == 8 && (uintptr_t)y % 16)) return -2;
  ChanAffine a{};
  for (int c = 0; c < C; ++c) {
    a.scale[c] = scale[c];
    a.shift[c] = shift[c];
  }
  long g = (pixels + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (cout == 8)
    hipLaunchKernelGGL(u8_norm_chan8_k, dim3((unsigned)g), dim3(256), 0, st, x, (bf16_raw*)y, pixels, C, a, rev);
  else
    hipLaunchKernelGGL(u8_norm_chan_k, dim3((unsigned)g), dim3(256), 0, st, x, (bf16_raw*)y, pixels, C, a, rev);
  return (int)hipGetLastError();
}
extern "C" int hopsx_u8_normalize(const unsigned char* x, void* y, long n, float scale, float shift, hipStream_t st) {
  const int vec = ((uintptr_t)x % 8 == 0) && ((uintptr_t)y % 16 == 0);
  hipLaunchKernelGGL(u8_norm_k, dim3(ew_grid(n, vec ? 8 : 1)), dim3(256), 0, st, x, (bf16_raw*)y, n, scale, shift,
                     vec);
  return (int)hipGetLastError();
}
extern "C" int hopsx_colsum_bf16_scalar(const void* x, float* out, int M, int N, hipStream_t st) {
  const int gx = (N + 63) / 64;
  int gy = (M + 255) / 256;
  const int max_gy = (1024 + gx - 1) / gx;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  const int rpb = (M + gy - 1) / gy;
  hipLaunchKernelGGL(colsum_k, dim3(gx, gy), dim3(256), 0, st, (const bf16_raw*)x, out, M, N, rpb);
  return (int)hipGetLastError();
}
extern "C" int hopsx_act_bwd(const void* dy, const void* y, void* dx, long n, int act, hipStream_t st) {
  hipLaunchKernelGGL(act_bwd_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)y,
                     (bf16_raw*)dx, n, act);
  return (int)hipGetLastError();
}
extern "C" int hopsx_act_bwd_colsum_scalar(const void* dy, const void* y, void* dx, int M, int N, int act, float* colsum,
                                    hipStream_t st) {
  const int gx = (N + 63) / 64;
  int gy = (M + 255) / 256;
  const int max_gy = (2048 + gx - 1) / gx;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  const int rpb = (M + gy - 1) / gy;
  hipLaunchKernelGGL(act_bwd_colsum_k, dim3(gx, gy), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)y,
                     (bf16_raw*)dx, M, N, act, colsum, rpb);
  return (int)hipGetLastError();
}
extern "C" int hopsx_add_bf16(const void* a, const void* b, void* out, long n, int act, hipStream_t st) {
  hipLaunchKernelGGL(add_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)a, (const bf16_raw*)b,
                     (bf16_raw*)out, n, act);
  return (int)hipGetLastError();
}


// Zero-fill as a KERNEL node.  hipMemsetAsync inside a captured hipGraph becomes a runtime
// blit node; replays showed it intermittently not ordered before the split-K atomics that
// follow it (garbage accumulators -> exploding logits), so every in-graph clear goes through
// this kernel instead.
__global__ __launch_bounds__(256) void zero_k(uint32_t* __restrict__ p, long n32) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n128 = ((uintptr_t)p % 16 == 0) ? (n32 >> 2) : 0;
  for (long j = i; j < n128; j += stride) ((uint4*)p)[j] = make_uint4(0u, 0u, 0u, 0u);
  for (long j = (n128 << 2) + i; j < n32; j += stride) p[j] = 0u;
}

extern "C" int hopsx_zero(void* p, long bytes, hipStream_t st) {
  if (!p || bytes <= 0) return 0;
  const long n32 = bytes / 4;  // callers clear fp32 / int32 buffers
  long g = (n32 / 4 + 255) / 256;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(zero_k, dim3(g), dim3(256), 0, st, (uint32_t*)p, n32);
  return (int)hipGetLastError();
}

// Health pill (the tfdbg NaN/Inf legend): out[0] += #NaN, out[1] += #Inf over an
// fp32 or bf16 tensor, one read pass (16-B vector loads), wave-reduced counts and one atomic
// pair per workgroup.  Graph-capturable: the caller zeroes `out` with hopsx_zero in the same stream.
template <typename T>
__global__ __launch_bounds__(256) void nonfinite_k(const T* __restrict__ x, long n, unsigned* __restrict__ out) {
  unsigned nan_c = 0, inf_c = 0;
  const long stride = (long)gridDim.x * blockDim.x;
  auto chk = [&](float v) {
    nan_c += (v != v) ? 1u : 0u;
    inf_c += (fabsf(v) == INFINITY) ? 1u : 0u;
  };
  constexpr int PER = 16 / sizeof(T);
  const long nv = ((uintptr_t)x % 16 == 0) ? n / PER : 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const uint4 q = ((const uint4*)x)[i];
    const T* e = (const T*)&q;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if constexpr (sizeof(T) == 4) chk(((const float*)e)[j]);
      else chk(bf2f(((const uint16_t*)e)[j]));
    }
  }
  for (long i = nv * PER + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if constexpr (sizeof(T) == 4) chk(((const float*)x)[i]);
    else chk(bf2f(((const uint16_t*)x)[i]));
  }
  for (int o = 32; o > 0; o >>= 1) {
    nan_c += __shfl_xor(nan_c, o, 64);
    inf_c += __shfl_xor(inf_c, o, 64);
  }
  __shared__ unsigned red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red[0][wave] = nan_c; red[1][wave] = inf_c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const unsigned b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    if (a) atomicAdd(out, a);
    if (b) atomicAdd(out + 1, b);
  }
}

extern "C" int hopsx_nonfinite(const void* x, long n, int is_bf16, unsigned* out, hipStream_t st) {
  if (n <= 0) return 0;
  long g = (n / (is_bf16 ? 8 : 4) + 255) / 256;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  if (is_bf16) hipLaunchKernelGGL(nonfinite_k<uint16_t>, dim3(g), dim3(256), 0, st, (const uint16_t*)x, n, out);
  else hipLaunchKernelGGL(nonfinite_k<float>, dim3(g), dim3(256), 0, st, (const float*)x, n, out);
  return (int)hipGetLastError();
}

// ---- input-channel padding of an image stem's conv weight (ops/functional.py _PadCinFn) ----------
// forward: w fp32 [R][C] -> out fp32 [R][cp] and its bf16 copy (what the conv kernels read), the channels
// C..cp-1 zero: ONE launch instead of a zero fill + a strided copy + a cast
__global__ __launch_bounds__(256) void pad_cin_k(const float* __restrict__ w, long R, int C, int cp,
                                                 float* __restrict__ out, bf16_raw* __restrict__ out16) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < R * cp; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cp;
    const int c = (int)(i - r * cp);
    const float v = c < C ? w[r * C + c] : 0.f;
    out[i] = v;
    out16[i] = f2bf(v);
  }
}

// backward: tgt[R][C] += g[R][:C] (the parameter's arena gradient), g re-zeroed (a zero-at-rest
// weight-gradient buffer the conv accumulates into): one launch instead of a zero fill + an add
__global__ __launch_bounds__(256) void unpad_cin_add_k(float* __restrict__ g, long R, int C, int cp,
                                                       float* __restrict__ tgt) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < R * cp; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cp;
    const int c = (int)(i - r * cp);
    if (c < C && tgt) tgt[r * C + c] += g[i];
    g[i] = 0.f;
  }
}

extern "C" int hopsx_pad_cin(const float* w, long R, int C, int cp, float* out, void* out16, hipStream_t st) {
  if (R <= 0 || C <= 0 || cp < C) return -1;
  long g = (R * cp + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(pad_cin_k, dim3(g), dim3(256), 0, st, w, R, C, cp, out, (bf16_raw*)out16);
  return (int)hipGetLastError();
}

extern "C" int hopsx_unpad_cin_add(float* gpad, long R, int C, int cp, float* tgt, hipStream_t st) {
  if (R <= 0 || C <= 0 || cp < C) return -1;
  long g = (R * cp + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(unpad_cin_add_k, dim3(g), dim3(256), 0, st, gpad, R, C, cp, tgt);
  return (int)hipGetLastError();
}
