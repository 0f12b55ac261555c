// Implicit-GEMM conv2d (NHWC activations, [Cout][KH][KW][Cin] weights) on MFMA.
//   fwd   : Y[m=(b,oh,ow)][co]      = im2col(X)[m][k=(kh,kw,ci)] . W[co][k]
//   dgrad : dX[m=(b,ih,iw)][ci]     = gatherT(dY)[m][k=(kh,kw,co)] . W^T[k][ci]
//   wgrad : dW[co][k=(kh,kw,ci)]   += dY^T[co][m] . im2col(X)[m][k]     (split-K, fp32 atomics)
// The gathers run inside the LDS staging of gemm_core.h, so no im2col buffer
// ever touches HBM.
#include "gemm_core.h"
#include "ops_api.h"

using namespace hopsx;

static ConvGeom make_geom(const int* g) {
  ConvGeom c;
  c.B = g[0]; c.H = g[1]; c.W = g[2]; c.C = g[3];
  c.OH = g[4]; c.OW = g[5]; c.CO = g[6];
  c.KH = g[7]; c.KW = g[8]; c.sh = g[9]; c.sw = g[10]; c.ph = g[11]; c.pw = g[12]; c.dh = g[13]; c.dw = g[14];
  return c;
}

// ---------------------------------------------------------------------------
// Direct conv for tiny reductions (K = KH*KW*Cin <= 64: the Cin=1 input layers
// of every MNIST model, K = 4/9/16/25).  As an implicit GEMM these waste
// >= 60 % of each BK=64 MFMA tile on zero padding and pay a scalar im2col
// gather per element; here each thread owns (pixel, 4 output channels), the
// weights sit in LDS as fp32, and outputs leave as 8-byte stores.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_direct_fwd_k(const bf16_raw* __restrict__ x,
                                                         const bf16_raw* __restrict__ w,
                                                         const float* __restrict__ bias, bf16_raw* __restrict__ y,
                                                         ConvGeom g, int act) {
  extern __shared__ float sw[];  // [K][CO]
  const int K = g.KH * g.KW * g.C;
  for (int i = threadIdx.x; i < K * g.CO; i += blockDim.x) {
    const int co = i % g.CO, k = i / g.CO;
    sw[i] = bf2f(w[(long)co * K + k]);
  }
  __syncthreads();
  const int G = g.CO >> 2;
  const long total = (long)g.B * g.OH * g.OW * G;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = t % G;
    const long pix = t / G;
    const int ow = pix % g.OW;
    const long r = pix / g.OW;
    const int oh = r % g.OH;
    const int b = r / g.OH;
    float acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bias ? bias[cg * 4 + j] : 0.f;
    int k = 0;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.sh - g.ph + kh * g.dh;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.sw - g.pw + kw * g.dw;
        const bool in = ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const bf16_raw* xp = x + (((long)b * g.H + ih) * g.W + iw) * g.C;
        for (int ci = 0; ci < g.C; ++ci, ++k) {
          const float xv = in ? bf2f(xp[ci]) : 0.f;
          const float* wr = sw + k * g.CO + cg * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] += xv * wr[j];
        }
      }
    }
    const uint32_t lo = (uint32_t)f2bf(apply_act(acc[0], act)) | ((uint32_t)f2bf(apply_act(acc[1], act)) << 16);
    const uint32_t hi = (uint32_t)f2bf(apply_act(acc[2], act)) | ((uint32_t)f2bf(apply_act(acc[3], act)) << 16);
    *(uint2*)(y + pix * g.CO + cg * 4) = make_uint2(lo, hi);
  }
}

// dW[co][k] += sum_m dY[m][co] * im2col(X)[m][k] for K*CO <= 1024: one thread per
// (k, co) output, pixel tiles of 64 staged in LDS, ONE atomic per thread per workgroup.
__global__ __launch_bounds__(1024) void conv_direct_wgrad_k(const bf16_raw* __restrict__ dy,
                                                            const bf16_raw* __restrict__ x, float* __restrict__ dw,
                                                            ConvGeom g, int pix_per_block) {
  constexpr int TP = 64;
  extern __shared__ float sm[];
  const int K = g.KH * g.KW * g.C;
  float* sdy = sm;             // [TP][CO]
  float* sx = sm + TP * g.CO;  // [TP][K]
  const int M = g.B * g.OH * g.OW;
  const int m0 = blockIdx.x * pix_per_block, m1 = min(M, m0 + pix_per_block);
  const int tid = threadIdx.x;
  const int co = tid % g.CO, k = tid / g.CO;
  const bool active = k < K;
  float acc = 0.f;
  for (int mb = m0; mb < m1; mb += TP) {
    const int np = min(TP, m1 - mb);
    for (int i = tid; i < TP * g.CO; i += blockDim.x) {
      const int p = i / g.CO, c = i % g.CO;
      sdy[i] = p < np ? bf2f(dy[(long)(mb + p) * g.CO + c]) : 0.f;
    }
    for (int i = tid; i < TP * K; i += blockDim.x) {
      const int p = i / K, kk = i % K;
      float v = 0.f;
      if (p < np) {
        const int m = mb + p;
        const int ohw = g.OH * g.OW;
        const int b = m / ohw, rem = m - b * ohw;
        const int oh = rem / g.OW, ow = rem - oh * g.OW;
        const int ci = kk % g.C, t = kk / g.C;
        const int kw = t % g.KW, kh = t / g.KW;
        const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
        if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) v = bf2f(x[(((long)b * g.H + ih) * g.W + iw) * g.C + ci]);
      }
      sx[i] = v;
    }
    __syncthreads();
    if (active)
#pragma unroll 8
      for (int p = 0; p < TP; ++p) acc += sdy[p * g.CO + co] * sx[p * K + k];
    __syncthreads();
  }
  if (active && acc != 0.f) atomicAdd(dw + (long)co * K + k, acc);
}

static bool direct_ok(const ConvGeom& g) {
  const int K = g.KH * g.KW * g.C;
  return K <= 64 && g.CO % 4 == 0 && g.CO <= 256 && K * g.CO <= 1024 && !hopsx_disabled("direct_conv");
}

extern "C" int hopsx_conv2d_fwd(const void* x, const void* w, const int* geom, int epi, void* out,
                                const float* bias, int act, float* colsum, hipStream_t st) {
  ConvGeom g = make_geom(geom);
  const int M = g.B * g.OH * g.OW, N = g.CO, K = g.KH * g.KW * g.C;
  if (epi == EPI_STORE_BF16 && !colsum && direct_ok(g) && ((uintptr_t)out % 8 == 0)) {
    long total = (long)M * (N / 4);
    long grid = (total + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(conv_direct_fwd_k, dim3(grid), dim3(256), (size_t)K * N * sizeof(float), st,
                       (const bf16_raw*)x, (const bf16_raw*)w, bias, (bf16_raw*)out, g, act);
    return (int)hipGetLastError();
  }
  Im2colLoader al{(const bf16_raw*)x, g, (g.C % 8 == 0) && ((uintptr_t)x % 16 == 0)};
  DenseLoader bl{(const bf16_raw*)w, K, is_vec_ok(w, K)};
  if (epi == EPI_STORE_BF16) {
    EpiStoreBF16 e{(bf16_raw*)out, N, bias, 1.f, act, colsum};
    launch_gemm<true, true>(al, bl, e, M, N, K, false, st);
  } else if (epi == EPI_STORE_F32) {
    EpiStoreF32 e{(float*)out, N, bias, 1.f, 0.f, act, colsum};
    launch_gemm<true, true>(al, bl, e, M, N, K, false, st);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

// dX = conv_transpose(dY, W).  If `yprev` is given, the result is multiplied by
// act'(yprev) — the backward of the activation that produced this conv's input
// — and `colsum` receives that layer's bias gradient.
extern "C" int hopsx_conv2d_dgrad(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                  int act, float* colsum, hipStream_t st) {
  ConvGeom g = make_geom(geom);
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.CO;
  ConvDgradALoader al{(const bf16_raw*)dy, g, (g.CO % 8 == 0) && ((uintptr_t)dy % 16 == 0)};
  ConvWeightTLoader bl{(const bf16_raw*)w, g, (g.C % 8 == 0) && ((uintptr_t)w % 16 == 0)};
  EpiDActBF16 e{(bf16_raw*)dx, N, (const bf16_raw*)yprev, N, act, colsum};
  launch_gemm<true, false>(al, bl, e, M, N, K, false, st);
  return (int)hipGetLastError();
}

// dW[co][k] += sum_m dY[m][co] * im2col(X)[m][k]; db[co] += sum_m dY[m][co] when colsum given
extern "C" int hopsx_conv2d_wgrad(const void* dy, const void* x, const int* geom, float* dw, float* dbias,
                                  hipStream_t st) {
  ConvGeom g = make_geom(geom);
  const int M = g.CO, N = g.KH * g.KW * g.C, K = g.B * g.OH * g.OW;
  if (direct_ok(g)) {
    const int threads = ((N * M + 63) / 64) * 64;
    // ~2 workgroups per CU; each handles >= 64 pixels (one LDS tile)
    long blocks = (K + 63) / 64;
    if (blocks > 512) blocks = 512;
    if (blocks < 1) blocks = 1;
    const int ppb = (int)((K + blocks - 1) / blocks);
    const size_t shm = (size_t)64 * (M + N) * sizeof(float);
    hipLaunchKernelGGL(conv_direct_wgrad_k, dim3(blocks), dim3(threads), shm, st, (const bf16_raw*)dy,
                       (const bf16_raw*)x, dw, g, ppb);
    return (int)hipGetLastError();
  }
  DenseLoader al{(const bf16_raw*)dy, g.CO, is_vec_ok(dy, g.CO)};
  Im2colLoader bl{(const bf16_raw*)x, g, (g.C % 8 == 0) && ((uintptr_t)x % 16 == 0)};
  EpiAtomicF32 e{dw, N, 1.f, nullptr};
  launch_gemm<false, false>(al, bl, e, M, N, K, true, st);
  (void)dbias;  // bias gradient of a conv is produced by the consumer's fused column sum
  return (int)hipGetLastError();
}
