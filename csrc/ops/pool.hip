// NHWC pooling. Max-pool keeps a 1-byte window-argmax per output element; the
// backward is a deterministic gather (no atomics) that also applies the
// derivative of the activation feeding the pool and emits that conv layer's
// bias gradient (per-channel column sum) — conv->act->pool backprop in one pass.
#include "common.h"
#include "ops_api.h"

HOPSX_DET_TU(pool)

static inline int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

__global__ __launch_bounds__(256) void maxpool_fwd_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                     unsigned char* __restrict__ am, int B, int H, int W, int C,
                                                     int OH, int OW, int KH, int KW, int sh, int sw, int ph,
                                                     int pw, float p, const unsigned long long* __restrict__ rng,
                                                     unsigned salt) {
  const long total = (long)B * OH * OW * C;
  const uint64_t key = p > 0.f ? drop_key(rng, salt) : 0;
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
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
    if (p > 0.f) best = uniform01(key, i) >= p ? best * dscale : 0.f;
    y[i] = f2bf(best);
    if (am) am[i] = (unsigned char)bi;
  }
}

// one thread per input element; gathers from every window that covers it
__global__ __launch_bounds__(256) void maxpool_bwd_k(const bf16_raw* __restrict__ dy, const unsigned char* __restrict__ am,
                                                     const bf16_raw* __restrict__ x, bf16_raw* __restrict__ dx, int B,
                                                     int H, int W, int C, int OH, int OW, int KH, int KW, int sh,
                                                     int sw, int ph, int pw, int act, float* __restrict__ colsum,
                                                     float p, const unsigned long long* __restrict__ rng,
                                                     unsigned salt) {
  extern __shared__ float scs[];
  const uint64_t key = p > 0.f ? drop_key(rng, salt) : 0;
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;  // per-block channel partial sums (C floats)
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
        const unsigned a = am[o];
        if (hx_check(a < (unsigned)(KH * KW)) && a == (unsigned)(kh * KW + kw)) {
          float d = bf2f(dy[o]);
          if (p > 0.f) d = uniform01(key, o) >= p ? d * dscale : 0.f;
          g += d;
        }
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

// ---------------------------------------------------------------------------
// Fast path: non-overlapping windows (stride == kernel, no padding — every
// reference CNN), C % 8 == 0.  One thread per (output pixel, 8 channels): 16-B
// loads/stores, argmax packed as 8 bytes.  The backward writes each window
// exactly once (value at the argmax, zero elsewhere, plus the floor-mode
// remainder rows/cols), so it needs no gather and no zero-fill pass; bias-grad
// partials stay in registers (channel group is fixed per thread because the
// grid stride is a multiple of C/8) and hit LDS/global atomics once per thread.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void maxpool_fwd8_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                      unsigned char* __restrict__ am, int B, int H, int W, int C,
                                                      int OH, int OW, int KH, int KW, float p,
                                                      const unsigned long long* __restrict__ rng, unsigned salt) {
  const int G = C >> 3;
  const long total = (long)B * OH * OW * G;
  const uint64_t key = p > 0.f ? drop_key(rng, salt) : 0;
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = t % G;
    const long pix = t / G;
    const int ow = pix % OW;
    const long r = pix / OW;
    const int oh = r % OH;
    const int b = r / OH;
    float best[8];
    unsigned char bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < KH; ++kh)
      for (int kw = 0; kw < KW; ++kw) {
        const bf16x8 v = *(const bf16x8*)(x + (((long)b * H + oh * KH + kh) * W + ow * KW + kw) * C + cg * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f((uint16_t)v[j]);
          if (f > best[j]) { best[j] = f; bi[j] = (unsigned char)(kh * KW + kw); }
        }
      }
    const long o = pix * C + cg * 8;
    bf16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = best[j];
      if (p > 0.f) f = uniform01(key, o + j) >= p ? f * dscale : 0.f;
      out[j] = (short)f2bf(f);
    }
    *(bf16x8*)(y + o) = out;
    if (am) {
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
      *(uint2*)(am + o) = packed;
    }
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd8_k(const bf16_raw* __restrict__ dy, const unsigned char* __restrict__ am,
                                                      const bf16_raw* __restrict__ x, bf16_raw* __restrict__ dx, int B,
                                                      int H, int W, int C, int OH, int OW, int KH, int KW, int act,
                                                      float* __restrict__ colsum, float p,
                                                      const unsigned long long* __restrict__ rng, unsigned salt) {
  extern __shared__ float scs[];
  const int G = C >> 3;
  const long total = (long)B * OH * OW * G;
  const uint64_t key = p > 0.f ? drop_key(rng, salt) : 0;
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (colsum) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) scs[c] = 0.f;
    __syncthreads();
  }
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int my_cg = -1;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = t % G;
    my_cg = cg;
    const long pix = t / G;
    const int ow = pix % OW;
    const long r = pix / OW;
    const int oh = r % OH;
    const int b = r / OH;
    const long o = pix * C + cg * 8;
    const bf16x8 dv = *(const bf16x8*)(dy + o);
    const uint2 pk = *(const uint2*)(am + o);
    float d[8];
    int a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = bf2f((uint16_t)dv[j]);
      if (p > 0.f) f = uniform01(key, o + j) >= p ? f * dscale : 0.f;
      d[j] = f;
      a[j] = ((j < 4 ? pk.x : pk.y) >> (8 * (j & 3))) & 0xff;
    }
    const int h1 = (oh == OH - 1) ? H : oh * KH + KH;
    const int w1 = (ow == OW - 1) ? W : ow * KW + KW;
    for (int ih = oh * KH; ih < h1; ++ih)
      for (int iw = ow * KW; iw < w1; ++iw) {
        const int kh = ih - oh * KH, kw = iw - ow * KW;
        const bool inwin = kh < KH && kw < KW;
        const int pos = kh * KW + kw;
        const long xi = (((long)b * H + ih) * W + iw) * C + cg * 8;
        bf16x8 xv = {0, 0, 0, 0, 0, 0, 0, 0};
        if (inwin && act != ACT_NONE && x) xv = *(const bf16x8*)(x + xi);
        bf16x8 outv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float g = (inwin && a[j] == pos) ? d[j] : 0.f;
          if (act != ACT_NONE && x && g != 0.f) g *= act_grad_from_out(bf2f((uint16_t)xv[j]), act);
          outv[j] = (short)f2bf(g);
          cs[j] += g;
        }
        *(bf16x8*)(dx + xi) = outv;
      }
  }
  if (colsum) {
    if (my_cg >= 0)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (cs[j] != 0.f) atomicAdd(&scs[my_cg * 8 + j], cs[j]);
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x)
      if (scs[c] != 0.f) atomicAdd(colsum + c, scs[c]);
  }
}

// ---------------------------------------------------------------------------
// Vectorized general windows (overlapping / padded, e.g. the ResNet stem 3x3/2 pad 1), C % 8 == 0:
// one thread per (pixel, 8 channels) with 16-B loads/stores and the 8 argmax bytes packed; the
// backward gathers over the <= ceil(K/s)^2 windows covering each input pixel.  Replaces the
// scalar kernels above, which moved 2 bytes per lane.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void maxpool_fwdv_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                      unsigned char* __restrict__ am, int B, int H, int W, int C,
                                                      int OH, int OW, int KH, int KW, int sh, int sw, int ph, int pw,
                                                      float p, const unsigned long long* __restrict__ rng,
                                                      unsigned salt) {
  const int G = C >> 3;
  const long total = (long)B * OH * OW * G;
  const uint64_t key = p > 0.f ? drop_key(rng, salt) : 0;
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % G);
    const long pix = t / G;
    const int ow = (int)(pix % OW);
    const long r = pix / OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * sh - ph + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * sw - pw + kw;
        if (iw < 0 || iw >= W) continue;
        const bf16x8 v = *(const bf16x8*)(x + (((long)b * H + ih) * W + iw) * C + cg * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f((uint16_t)v[j]);
          if (f > best[j]) { best[j] = f; bi[j] = kh * KW + kw; }
        }
      }
    }
    const long o = pix * C + cg * 8;
    bf16x8 out;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = best[j];
      if (p > 0.f) f = uniform01(key, o + j) >= p ? f * dscale : 0.f;
      out[j] = (short)f2bf(f);
      if (j < 4) lo |= (uint32_t)bi[j] << (8 * j);
      else hi |= (uint32_t)bi[j] << (8 * (j - 4));
    }
    *(bf16x8*)(y + o) = out;
    if (am) *(uint2*)(am + o) = make_uint2(lo, hi);
  }
}

__global__ __launch_bounds__(256) void maxpool_bwdv_k(const bf16_raw* __restrict__ dy, const unsigned char* __restrict__ am,
                                                      const bf16_raw* __restrict__ x, bf16_raw* __restrict__ dx, int B,
                                                      int H, int W, int C, int OH, int OW, int KH, int KW, int sh,
                                                      int sw, int ph, int pw, int act, float p,
                                                      const unsigned long long* __restrict__ rng, unsigned salt) {
  const int G = C >> 3;
  const long total = (long)B * H * W * G;
  const uint64_t key = p > 0.f ? drop_key(rng, salt) : 0;
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % G);
    const long pix = t / G;
    const int iw = (int)(pix % W);
    const long r = pix / W;
    const int ih = (int)(r % H);
    const int b = (int)(r / H);
    const int oh_lo = max(0, (ih + ph - KH + sh) / sh), oh_hi = min(OH - 1, (ih + ph) / sh);
    const int ow_lo = max(0, (iw + pw - KW + sw) / sw), ow_hi = min(OW - 1, (iw + pw) / sw);
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = ih - (oh * sh - ph);
      if (kh < 0 || kh >= KH) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = iw - (ow * sw - pw);
        if (kw < 0 || kw >= KW) continue;
        const long o = (((long)b * OH + oh) * OW + ow) * C + cg * 8;
        const bf16x8 d = *(const bf16x8*)(dy + o);
        const uint2 pk = *(const uint2*)(am + o);
        const int want = kh * KW + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int a = ((j < 4 ? pk.x : pk.y) >> (8 * (j & 3))) & 0xff;
          if (a == want) {
            float f = bf2f((uint16_t)d[j]);
            if (p > 0.f) f = uniform01(key, o + j) >= p ? f * dscale : 0.f;
            g[j] += f;
          }
        }
      }
    }
    const long i = pix * C + cg * 8;
    if (act != ACT_NONE && x) {
      const bf16x8 xv = *(const bf16x8*)(x + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] *= act_grad_from_out(bf2f((uint16_t)xv[j]), act);
    }
    bf16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (short)f2bf(g[j]);
    *(bf16x8*)(dx + i) = out;
  }
}

// global average pool over HW, 8 channels per thread (16-B loads), fp32 sums
__global__ __launch_bounds__(256) void gap_fwdv_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y, int HW,
                                                  int C) {
  const int G = C >> 3;
  const int b = blockIdx.y, cg = blockIdx.x * blockDim.x + threadIdx.x;
  if (cg >= G) return;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16_raw* p = x + (long)b * HW * C + cg * 8;
  int q = 0;
  for (; q + 4 <= HW; q += 4) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const bf16x8*)(p + (long)(q + u) * C);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f((uint16_t)v[u][j]);
  }
  for (; q < HW; ++q) {
    const bf16x8 v = *(const bf16x8*)(p + (long)q * C);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += bf2f((uint16_t)v[j]);
  }
  bf16x8 out;
  const float inv = 1.f / HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (short)f2bf(s[j] * inv);
  *(bf16x8*)(y + (long)b * C + cg * 8) = out;
}

__global__ __launch_bounds__(256) void gap_bwdv_k(const bf16_raw* __restrict__ dy, bf16_raw* __restrict__ dx, int B,
                                                  int HW, int C) {
  const int G = C >> 3;
  const long total = (long)B * HW * G;
  const float inv = 1.f / HW;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % G);
    const long b = t / ((long)HW * G);
    const bf16x8 d = *(const bf16x8*)(dy + b * C + cg * 8);
    bf16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (short)f2bf(bf2f((uint16_t)d[j]) * inv);
    *(bf16x8*)(dx + (t / G) * C + cg * 8) = out;
  }
}

static bool pool_vec(int C, const void* a, const void* b, const void* c, const void* d) {
  return !hopsx_disabled("poolv") && C % 8 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)d) % 16 == 0) &&
         ((uintptr_t)c % 8 == 0);
}

static bool pool_fast(int C, int KH, int KW, int sh, int sw, int ph, int pw, const void* a, const void* b,
                      const void* c, const void* d) {
  return !hopsx_disabled("pool8") && C % 8 == 0 && (256 % (C / 8) == 0) && sh == KH && sw == KW && ph == 0 &&
         pw == 0 && KH * KW <= 255 &&
         (((uintptr_t)a | (uintptr_t)b | (uintptr_t)d) % 16 == 0) && ((uintptr_t)c % 8 == 0);
}

extern "C" int hopsx_maxpool2d_fwd(const void* x, void* y, unsigned char* argmax, int B, int H, int W, int C, int OH,
                                   int OW, int KH, int KW, int sh, int sw, int ph, int pw, float p,
                                   const unsigned long long* rng, unsigned salt, hipStream_t st) {
  if (argmax && pool_fast(C, KH, KW, sh, sw, ph, pw, x, y, argmax, nullptr)) {
    const long n8 = (long)B * OH * OW * (C / 8);
    hipLaunchKernelGGL(maxpool_fwd8_k, dim3(grid_for(n8)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, argmax,
                       B, H, W, C, OH, OW, KH, KW, p, rng, salt);
    return (int)hipGetLastError();
  }
  if (KH * KW <= 255 && pool_vec(C, x, y, argmax, nullptr)) {
    const long n8 = (long)B * OH * OW * (C / 8);
    hipLaunchKernelGGL(maxpool_fwdv_k, dim3(grid_for(n8)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, argmax,
                       B, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, p, rng, salt);
    return (int)hipGetLastError();
  }
  const long n = (long)B * OH * OW * C;
  hipLaunchKernelGGL(maxpool_fwd_k, dim3(grid_for(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, argmax, B,
                     H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, p, rng, salt);
  return (int)hipGetLastError();
}

extern "C" int hopsx_maxpool2d_bwd(const void* dy, const unsigned char* argmax, const void* x, void* dx, int B, int H,
                                   int W, int C, int OH, int OW, int KH, int KW, int sh, int sw, int ph, int pw,
                                   int act, float* colsum, float p, const unsigned long long* rng, unsigned salt,
                                   hipStream_t st) {
  if (colsum && hopsx_deterministic()) {
    // the fused column sum adds through LDS float atomics (unordered even within a workgroup):
    // deterministic mode sums the stored input gradient in a second, turn-ordered pass instead
    const int e = hopsx_maxpool2d_bwd(dy, argmax, x, dx, B, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, act, nullptr, p,
                                      rng, salt, st);
    return e ? e : hopsx_colsum_bf16(dx, colsum, B * H * W, C, st);
  }
  const size_t shm = colsum ? (size_t)C * sizeof(float) : 0;
  // (a thread per pooled output walks its whole window: with few outputs and big windows — the E1 model's
  // 4x4 pool, 6,400 threads in 25 workgroups, 28 us — the per-input-pixel kernel below fills the GPU)
  const bool few_big = (long)B * OH * OW * (C / 8) < 32768 && KH * KW >= 9 && !colsum;
  if (!few_big && pool_fast(C, KH, KW, sh, sw, ph, pw, dy, dx, argmax, x)) {
    const long n8 = (long)B * OH * OW * (C / 8);
    int g = grid_for(n8);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(maxpool_bwd8_k, dim3(g), dim3(256), shm, st, (const bf16_raw*)dy, argmax, (const bf16_raw*)x,
                       (bf16_raw*)dx, B, H, W, C, OH, OW, KH, KW, act, colsum, p, rng, salt);
    return (int)hipGetLastError();
  }
  if (!colsum && KH * KW <= 255 && pool_vec(C, dy, dx, argmax, x)) {
    const long n8 = (long)B * H * W * (C / 8);
    hipLaunchKernelGGL(maxpool_bwdv_k, dim3(grid_for(n8)), dim3(256), 0, st, (const bf16_raw*)dy, argmax,
                       (const bf16_raw*)x, (bf16_raw*)dx, B, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, act, p, rng, salt);
    return (int)hipGetLastError();
  }
  const long n = (long)B * H * W * C;
  hipLaunchKernelGGL(maxpool_bwd_k, dim3(grid_for(n, 256) > 1024 ? 1024 : grid_for(n, 256)), dim3(256), shm, st, (const bf16_raw*)dy, argmax,
                     (const bf16_raw*)x, (bf16_raw*)dx, B, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, act, colsum, p, rng, salt);
  return (int)hipGetLastError();
}

extern "C" int hopsx_avgpool_global_fwd(const void* x, void* y, int B, int HW, int C, hipStream_t st) {
  if (pool_vec(C, x, y, nullptr, nullptr)) {
    const int G = C / 8;
    hipLaunchKernelGGL(gap_fwdv_k, dim3((G + 255) / 256, B), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, HW, C);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(gap_fwd_k, dim3(B), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, B, HW, C);
  return (int)hipGetLastError();
}

extern "C" int hopsx_avgpool_global_bwd(const void* dy, void* dx, int B, int HW, int C, hipStream_t st) {
  if (pool_vec(C, dy, dx, nullptr, nullptr)) {
    const long n8 = (long)B * HW * (C / 8);
    hipLaunchKernelGGL(gap_bwdv_k, dim3(grid_for(n8)), dim3(256), 0, st, (const bf16_raw*)dy, (bf16_raw*)dx, B, HW, C);
    return (int)hipGetLastError();
  }
  const long n = (long)B * HW * C;
  hipLaunchKernelGGL(gap_bwd_k, dim3(grid_for(n)), dim3(256), 0, st, (const bf16_raw*)dy, (bf16_raw*)dx, B, HW, C);
  return (int)hipGetLastError();
}
