// NHWC pooling. Max-pool keeps a 1-byte window-argmax per output element; the
// backward is a deterministic gather (no atomics) that also applies the
// derivative of the activation feeding the pool and emits that conv layer's
// bias gradient (per-channel column sum) — conv->act->pool backprop in one pass.
#include "common.h"
#include "ops_api.h"

static inline int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

__global__ __launch_bounds__(256) void maxpool_fwd_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                     unsigned char* __restrict__ am, int B, int H, int W, int C,
                                                     int OH, int OW, int KH, int KW, int sh, int sw, int ph,
                                                     int pw) {
  const long total = (long)B * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = i % C;
    long t = i / C;
    const int ow = t % OW;
    t /= OW;
    const int oh = t % OH;
    const int b = t / OH;
    float best = -INFINITY;
    int bi = 0;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * sh - ph + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * sw - pw + kw;
        if (iw < 0 || iw >= W) continue;
        const float v = bf2f(x[(((long)b * H + ih) * W + iw) * C + c]);
        if (v > best) { best = v; bi = kh * KW + kw; }
      }
    }
    y[i] = f2bf(best);
    if (am) am[i] = (unsigned char)bi;
  }
}

// one thread per input element; gathers from every window that covers it
__global__ __launch_bounds__(256) void maxpool_bwd_k(const bf16_raw* __restrict__ dy, const unsigned char* __restrict__ am,
                                                     const bf16_raw* __restrict__ x, bf16_raw* __restrict__ dx, int B,
                                                     int H, int W, int C, int OH, int OW, int KH, int KW, int sh,
                                                     int sw, int ph, int pw, int act, float* __restrict__ colsum) {
  extern __shared__ float scs[];  // per-block channel partial sums (C floats)
  const long total = (long)B * H * W * C;
  if (colsum) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) scs[c] = 0.f;
    __syncthreads();
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = i % C;
    long t = i / C;
    const int iw = t % W;
    t /= W;
    const int ih = t % H;
    const int b = t / H;
    // output windows covering (ih, iw): oh*sh - ph <= ih < oh*sh - ph + KH
    const int oh_lo = max(0, (ih + ph - KH + sh) / sh), oh_hi = min(OH - 1, (ih + ph) / sh);
    const int ow_lo = max(0, (iw + pw - KW + sw) / sw), ow_hi = min(OW - 1, (iw + pw) / sw);
    float g = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = ih - (oh * sh - ph);
      if (kh < 0 || kh >= KH) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = iw - (ow * sw - pw);
        if (kw < 0 || kw >= KW) continue;
        const long o = (((long)b * OH + oh) * OW + ow) * C + c;
        if (am[o] == kh * KW + kw) g += bf2f(dy[o]);
      }
    }
    if (act != ACT_NONE && x) g *= act_grad_from_out(bf2f(x[i]), act);
    dx[i] = f2bf(g);
    if (colsum) atomicAdd(&scs[c], g);
  }
  if (colsum) {
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x)
      if (scs[c] != 0.f) atomicAdd(colsum + c, scs[c]);
  }
}

__global__ void gap_fwd_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y, int B, int HW, int C) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += bf2f(x[((long)b * HW + p) * C + c]);
    y[(long)b * C + c] = f2bf(s / HW);
  }
}

__global__ void gap_bwd_k(const bf16_raw* __restrict__ dy, bf16_raw* __restrict__ dx, int B, int HW, int C) {
  const long total = (long)B * HW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = i % C;
    const long b = i / ((long)HW * C);
    dx[i] = f2bf(bf2f(dy[b * C + c]) / HW);
  }
}

extern "C" int hopsx_maxpool2d_fwd(const void* x, void* y, unsigned char* argmax, int B, int H, int W, int C, int OH,
                                   int OW, int KH, int KW, int sh, int sw, int ph, int pw, hipStream_t st) {
  const long n = (long)B * OH * OW * C;
  hipLaunchKernelGGL(maxpool_fwd_k, dim3(grid_for(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, argmax, B,
                     H, W, C, OH, OW, KH, KW, sh, sw, ph, pw);
  return (int)hipGetLastError();
}

extern "C" int hopsx_maxpool2d_bwd(const void* dy, const unsigned char* argmax, const void* x, void* dx, int B, int H,
                                   int W, int C, int OH, int OW, int KH, int KW, int sh, int sw, int ph, int pw,
                                   int act, float* colsum, hipStream_t st) {
  const long n = (long)B * H * W * C;
  const size_t shm = colsum ? (size_t)C * sizeof(float) : 0;
  hipLaunchKernelGGL(maxpool_bwd_k, dim3(grid_for(n, 256) > 1024 ? 1024 : grid_for(n, 256)), dim3(256), shm, st, (const bf16_raw*)dy, argmax,
                     (const bf16_raw*)x, (bf16_raw*)dx, B, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, act, colsum);
  return (int)hipGetLastError();
}

extern "C" int hopsx_avgpool_global_fwd(const void* x, void* y, int B, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gap_fwd_k, dim3(B), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, B, HW, C);
  return (int)hipGetLastError();
}

extern "C" int hopsx_avgpool_global_bwd(const void* dy, void* dx, int B, int HW, int C, hipStream_t st) {
  const long n = (long)B * HW * C;
  hipLaunchKernelGGL(gap_bwd_k, dim3(grid_for(n)), dim3(256), 0, st, (const bf16_raw*)dy, (bf16_raw*)dx, B, HW, C);
  return (int)hipGetLastError();
}
