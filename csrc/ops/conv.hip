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

extern "C" int hopsx_conv2d_fwd(const void* x, const void* w, const int* geom, int epi, void* out,
                                const float* bias, int act, float* colsum, hipStream_t st) {
  ConvGeom g = make_geom(geom);
  const int M = g.B * g.OH * g.OW, N = g.CO, K = g.KH * g.KW * g.C;
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
  DenseLoader al{(const bf16_raw*)dy, g.CO, is_vec_ok(dy, g.CO)};
  Im2colLoader bl{(const bf16_raw*)x, g, (g.C % 8 == 0) && ((uintptr_t)x % 16 == 0)};
  EpiAtomicF32 e{dw, N, 1.f, nullptr};
  launch_gemm<false, false>(al, bl, e, M, N, K, true, st);
  (void)dbias;  // bias gradient of a conv is produced by the consumer's fused column sum
  return (int)hipGetLastError();
}
