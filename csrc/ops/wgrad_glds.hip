// Convolution weight gradient on the gg engine (gemm_glds.h):
//   dW[co][k = (kh, kw, ci)] += sum_m dY[m][co] * im2col(X)[m][k]      (m = output pixel)
// Both operands are pixel-major, so both LDS images are RC ([64 pixels][128 columns], read with
// ds_read_b64_tr_b16) and the reduction runs over the pixel axis, split-K over the launch with fp32
// atomics into dW.  With CO < 128 the GEMM is run transposed (dW^T = im2col(X)^T dY) so the 128-row
// side of the tile is not half empty.
// Scope: no activation mask on dY and no bias gradient (the ResNet convolutions: conv -> BN);
// CO % 8 == 0, C % 8 == 0, 16-B aligned tensors.  Everything else keeps gemm_core.h's engine.
#include "gemm_glds.h"
#include "ops_api.h"

HOPSX_DET_TU(wgrad_glds)

using namespace hopsx;

extern "C" int hopsx_conv_wgrad_glds_ok(const int* geom) {
  const int C = geom[3], CO = geom[6];
  const long K = (long)geom[0] * geom[4] * geom[5];
  const long N = (long)geom[7] * geom[8] * C;
  return !hopsx_disabled("wgrad_glds") && C % 8 == 0 && CO % 8 == 0 && CO >= 64 && N >= 64 && K >= 512 &&
         K < (1L << 31) / 2;
}

// force: launch however few workgroups the shape gives (numerics tests); else -2 below the engine's
// workgroup floor and the caller keeps gemm_core.h's kernels
extern "C" int hopsx_conv2d_wgrad_glds(const void* dy, const void* x, const int* geom, float* dw, int force,
                                       hipStream_t st) {
  if (!hopsx_conv_wgrad_glds_ok(geom) || ((uintptr_t)dy | (uintptr_t)x) % 16) return -2;
  ConvGeom g;
  g.B = geom[0]; g.H = geom[1]; g.W = geom[2]; g.C = geom[3];
  g.OH = geom[4]; g.OW = geom[5]; g.CO = geom[6];
  g.KH = geom[7]; g.KW = geom[8]; g.sh = geom[9]; g.sw = geom[10]; g.ph = geom[11]; g.pw = geom[12];
  g.dh = geom[13]; g.dw = geom[14];
  g.init_div();
  const int CO = g.CO, N = g.KH * g.KW * g.C, K = g.B * g.OH * g.OW;
  const GgDense dsrc{(const bf16_raw*)dy, (long)CO, K, CO};
  const long mw = force ? 1 : -1;
  auto run = [&](const auto& xsrc) {
    if (CO >= 128 || N < 128)
      return launch_gg<false, false>(dsrc, xsrc, EpiAtomicF32{dw, (long)N, 1.f, nullptr}, CO, N, K, true, st, mw);
    return launch_gg<false, false>(xsrc, dsrc, EpiAtomicF32T{dw, (long)N, 1.f, nullptr}, N, CO, K, true, st, mw);
  };
  // a 1x1 / stride-1 / unpadded conv's im2col IS X viewed as [pixels][C]: no gather
  const bool dense = g.KH == 1 && g.KW == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0;
  const bool ok = dense ? run(GgDense{(const bf16_raw*)x, (long)g.C, K, N}) : run(GgIm2col{(const bf16_raw*)x, g, K, N});
  if (!ok) return -2;
  return (int)hipGetLastError();
}
