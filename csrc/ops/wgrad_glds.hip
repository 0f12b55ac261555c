// Convolution weight gradient on gfx950 with LDS-DMA staging:
//   dW[co][k = (kh, kw, ci)] += sum_m dY[m][co] * im2col(X)[m][k]      (m = output pixel)
//
// The generic implicit-GEMM engine (gemm_core.h) stages both operands through registers in 4-wave
// workgroups and reached ~100 TFLOP/s on the ResNet-50 weight gradients, 26 % of the B=64 step
// (profiles/r3s3_resnet50_b64_kernels.txt).  The weight gradient is the one GEMM of the
// network whose reduction runs over the huge pixel axis with both operands pixel-major, so it gets
// its own kernel built around the CDNA4 idioms (cdna_hip_programming.md §5):
//   * 512 threads (8 waves, 2 co x 4 k), a 128 x 128 fp32 output tile per workgroup, BK = 64 pixels
//     per k-step, split-K over the pixels so a launch fills the chip; fp32 hardware atomics merge
//     the splits (few: every split covers >= 8 k-steps);
//   * both operand tiles move global -> LDS by `global_load_lds_dwordx4` (16 B per lane, no register
//     staging): dY rows are contiguous in co, im2col(X) rows are 8-channel chunks of one (kh, kw)
//     tap (C % 8 == 0), out-of-image taps and the tile edges read a zero page; double-buffered, the
//     next k-step's DMA is in flight while the MFMAs of this one run;
//   * the LDS images are [64 pixels][128 columns] with 256-B rows; the pixel axis is the MFMA
//     reduction axis, so fragments come out of LDS with `ds_read_b64_tr_b16` (hardware transpose,
//     T10).  Rows are XOR-swizzled on 16-B chunks (chunk ^ ((row&3)<<2 | (row>>2)&3), the T10 (b)
//     image); because the DMA writes lane-linearly the swizzle is applied to the SOURCE address of
//     each lane (guide rule 21: linear destination, permuted source, permuted read);
//   * v_mfma_f32_16x16x32_bf16, a 64 x 32 wave tile (4 x 2 fragments), fp32 accumulation.
// Scope: no activation mask on dY and no bias gradient (the ResNet convolutions: conv -> BN);
// CO % 8 == 0, C % 8 == 0, 16-B aligned tensors.  Everything else keeps the generic engine.
#include "gemm_core.h"
#include "ops_api.h"

using namespace hopsx;

namespace {

constexpr int WB_M = 128;       // co per tile
constexpr int WB_N = 128;       // k per tile
constexpr int WB_K = 64;        // pixels per k-step
constexpr int WB_THREADS = 512;
constexpr int WB_ROWB = 256;    // bytes per LDS image row (128 bf16)
constexpr int WB_IMG = WB_K * WB_ROWB;          // 16 KiB per operand image
constexpr int WB_STAGE = 2 * WB_IMG;            // A + B
constexpr int WB_LDS = 2 * WB_STAGE;            // double buffered: 64 KiB

__device__ __attribute__((aligned(64))) uint4 g_wb_zero[4];  // zero page for out-of-range chunks

typedef __attribute__((address_space(3))) void* lds_void_ptr;

struct WbArgs {
  const bf16_raw* dy;
  const bf16_raw* x;
  float* dw;
  ConvGeom g;
  int M, N;   // CO, KH*KW*C
  int K;      // pixels
  int kps;    // pixels per split (multiple of WB_K)
  int tiles_n, tiles;
};

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// Per-lane DMA source addresses, branch-free (a divergent branch around the DMA would split it
// into several partial-EXEC instructions): an out-of-range chunk reads the zero page.
__device__ __forceinline__ const void* a_src(const WbArgs& a, int m, int col) {
  const bool ok = m < a.K && col < a.M;
  const uintptr_t p = (uintptr_t)(a.dy + (long)(ok ? m : 0) * a.M + (ok ? col : 0));
  return (const void*)(ok ? p : (uintptr_t)g_wb_zero);
}

__device__ __forceinline__ const void* b_src(const WbArgs& a, int m, int k) {
  const ConvGeom& g = a.g;
  const int mc = m < a.K ? m : 0, kc = k < a.N ? k : 0;
  const int b = g.fOHW.div(mc), rem = mc - b * (g.OH * g.OW);
  const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
  const int t = g.fC.div(kc), ci = kc - t * g.C;
  const int kh = g.fKW.div(t), kw = t - kh * g.KW;
  const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
  const bool ok = m < a.K && k < a.N && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
  const long off = (((long)b * g.H + (ok ? ih : 0)) * g.W + (ok ? iw : 0)) * g.C + ci;
  const uintptr_t p = (uintptr_t)(a.x + off);
  return (const void*)(ok ? p : (uintptr_t)g_wb_zero);
}

// 4 x 16 (rows x cols) block at logical (row, col) of a swizzled 256-B-row image, transposed read
__device__ __forceinline__ bf16x4 tr_read(const unsigned char* img, int row, int col) {
  const unsigned char* p = img + row * WB_ROWB + 16 * ((col >> 3) ^ swz(row)) + 2 * (col & 7);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p));
}

__global__ __launch_bounds__(WB_THREADS) void conv_wgrad_glds_k(WbArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[WB_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // 2 x 4 waves: 64 co x 32 k each
  // blocks of one tile are consecutive ids (tile-major): its splits spread over XCDs round-robin
  const int bid = blockIdx.x;
  const int tile = bid % a.tiles, split = bid / a.tiles;
  const int co0 = (tile / a.tiles_n) * WB_M, n0 = (tile % a.tiles_n) * WB_N;
  const int kbeg = split * a.kps;
  const int kend = min(a.K, kbeg + a.kps);
  if (kbeg >= kend) return;
  const int nt = (kend - kbeg + WB_K - 1) / WB_K;

  // DMA roles: wave-instruction i of wave w fills rows 4*(w + 8 i) .. +3; lane -> (row, physical chunk)
  const int prow = lane >> 4, pch = lane & 15;
  auto stage = [&](int buf, int m0) {
    unsigned char* A = smem + buf * WB_STAGE;
    unsigned char* Bm = A + WB_IMG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = 4 * (wave + 8 * i);
      const int row = r0 + prow;
      const int lc = pch ^ swz(row);  // the logical chunk that lands at this lane's physical slot
      __builtin_amdgcn_global_load_lds(a_src(a, m0 + row, co0 + 8 * lc), (lds_void_ptr)(A + r0 * WB_ROWB), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(b_src(a, m0 + row, n0 + 8 * lc), (lds_void_ptr)(Bm + r0 * WB_ROWB), 16, 0,
                                       0);
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int tq = (lane & 15) >> 2, tp = lane & 3;

  stage(0, kbeg);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const unsigned char* A = smem + cur * WB_STAGE;
    const unsigned char* Bm = A + WB_IMG;
    // every fragment of this k-step first: a DMA issued before an LDS read makes hipcc wait for
    // it (vmcnt(0)) ahead of the read, which would serialise the prefetch
    bf16x8 af[2][4], bf[2][2];
#pragma unroll
    for (int kk = 0; kk < WB_K / 32; ++kk) {
      const int r1 = kk * 32 + 8 * fq + tq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wm * 64 + i * 16 + 4 * tp;
        const bf16x4 v1 = tr_read(A, r1, col), v2 = tr_read(A, r1 + 4, col);
        af[kk][i] = (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wn * 32 + j * 16 + 4 * tp;
        const bf16x4 v1 = tr_read(Bm, r1, col), v2 = tr_read(Bm, r1 + 4, col);
        bf[kk][j] = (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) stage(cur ^ 1, kbeg + (t + 1) * WB_K);  // lands while the MFMAs below run
#pragma unroll
    for (int kk = 0; kk < WB_K / 32; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bf[kk][j], acc[i][j], 0, 0, 0);
    // keep every MFMA ahead of the DMA wait (hipcc otherwise sinks most of them past the barrier
    // and waits for the DMA right after the first two: the prefetch would not overlap compute)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next k-step's DMA has landed
    __syncthreads();
  }

  // D[row = co][col = k]: lane holds rows 4 fq + r of column fr of each fragment
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = n0 + wn * 32 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 64 + i * 16 + 4 * fq + r;
        const float v = acc[i][j][r];
        if (co < a.M && k < a.N && v != 0.f) unsafeAtomicAdd(a.dw + (long)co * a.N + k, v);
      }
    }
}

}  // namespace

extern "C" int hopsx_conv_wgrad_glds_ok(const int* geom) {
  const int C = geom[3], CO = geom[6];
  const long K = (long)geom[0] * geom[4] * geom[5];
  const long N = (long)geom[7] * geom[8] * C;
  return !hopsx_disabled("wgrad_glds") && C % 8 == 0 && CO % 8 == 0 && CO >= 64 && N >= 64 && K >= 8L * WB_K &&
         K < (1L << 31) / 2;
}

extern "C" int hopsx_conv2d_wgrad_glds(const void* dy, const void* x, const int* geom, float* dw, hipStream_t st) {
  if (!hopsx_conv_wgrad_glds_ok(geom) || ((uintptr_t)dy | (uintptr_t)x) % 16) return -2;
  WbArgs a{};
  a.dy = (const bf16_raw*)dy;
  a.x = (const bf16_raw*)x;
  a.dw = dw;
  ConvGeom& g = a.g;
  g.B = geom[0]; g.H = geom[1]; g.W = geom[2]; g.C = geom[3];
  g.OH = geom[4]; g.OW = geom[5]; g.CO = geom[6];
  g.KH = geom[7]; g.KW = geom[8]; g.sh = geom[9]; g.sw = geom[10]; g.ph = geom[11]; g.pw = geom[12];
  g.dh = geom[13]; g.dw = geom[14];
  g.init_div();
  a.M = g.CO;
  a.N = g.KH * g.KW * g.C;
  a.K = g.B * g.OH * g.OW;
  a.tiles_n = (a.N + WB_N - 1) / WB_N;
  a.tiles = ((a.M + WB_M - 1) / WB_M) * a.tiles_n;
  // splits: ~2 workgroups per CU over the whole launch, each split >= 8 k-steps of 64 pixels;
  // HOPSX_WGRAD_GLDS_TARGET overrides the workgroup target (A/B knob)
  static const long target = hopsx_env_int("HOPSX_WGRAD_GLDS_TARGET", 512);
  long s = (target + a.tiles - 1) / a.tiles;
  const long maxs = (a.K + 8L * WB_K - 1) / (8L * WB_K);
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  long kps = (a.K + s - 1) / s;
  kps = (kps + WB_K - 1) / WB_K * WB_K;
  a.kps = (int)kps;
  s = (a.K + kps - 1) / kps;
  hipLaunchKernelGGL(conv_wgrad_glds_k, dim3((unsigned)(a.tiles * s)), dim3(WB_THREADS), 0, st, a);
  return (int)hipGetLastError();
}
