// Direct MFMA convolutions for short reductions (K = KH*KW*Cin <= 512, Cin % 8 == 0 for the
// forward, Cout % 8 == 0 for dgrad; the 32->64 channel second conv of every MNIST model,
// K = 128 / 288 / 512).  As an implicit GEMM these layers are latency-bound: 2-8 K-tiles per
// workgroup, each paying an LDS staging round trip and two barriers.  Here:
//   * the (tiny) weight matrix is staged ONCE per workgroup into LDS in MFMA B-fragment
//     order (16-B chunks, XOR-swizzled so a 16-lane ds_read_b128 group hits 16 distinct slots),
//   * each wave owns 16-pixel groups and loads its A fragments straight from global memory
//     into registers — one 16-B im2col (fwd) / col2im (dgrad) gather per lane per 32-deep
//     K-step, two groups in flight per trip, no barriers in the loop,
//   * v_mfma_f32_16x16x32_bf16 over all Cout fragments, then a fused epilogue (bias + act
//     for fwd; act'(yprev) mask + previous layer's bias gradient for dgrad) written through
//     a per-wave LDS transpose so the stores leave as 16-B vectors.
#include <algorithm>
#include <cstdlib>

#include "gemm_core.h"
#include "ops_api.h"
#include "optim_slice.h"

HOPSX_DET_TU(conv_mfma)

using namespace hopsx;

namespace {

// per-workgroup phase timestamps (100 MHz wall clock), written only when HOPSX_PHASE_DBG is set:
// tools/dbg_wgrad.py reads them back to split a launch into load / compute / reduce / atomics
__device__ unsigned long long g_wgrad_dbg[2048 * 4];
__device__ __forceinline__ void phase_mark(int on, int slot) {
  if (on && threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 2048) g_wgrad_dbg[blockIdx.x * 4 + slot] = wall_clock64();
}

constexpr int CM_WAVES = 4;
constexpr int CM_UN = 2;  // pixel groups per wave per trip
constexpr int CM_RSLOTS = CM_WAVES * 4;  // dgrad column-sum partials: one per (wave, 16-lane row)

// LDS row stride (in 16-B chunks) of a weight image with cpr chunks per row: rows of >= 16
// chunks are padded to a multiple of 16 so the XOR swizzle below never leaves its row
__host__ __device__ constexpr int cm_rs(int cpr) { return cpr >= 16 ? (cpr + 15) / 16 * 16 : cpr; }

// swizzled chunk index for row `r` of a [rows][cpr chunks] LDS image: 16 consecutive rows
// reading the same logical chunk land on 16 different 16-B slots of the 256-B bank row
__device__ __forceinline__ int cm_swz(int r, int c, int cpr) {
  if (cpr >= 16) return c ^ (r & 15);
  const int rows_per_line = 16 / cpr;  // 2 (cpr 8), 4 (cpr 4)
  return c ^ ((r / rows_per_line) & (cpr - 1));
}

// ---------------------------------------------------------------------------- forward
// POOL: a 2x2/stride-2 max-pool (+ dropout) fused into the epilogue.  The 16 A rows of a pixel
// group are then 4 pooled outputs x their 4 window taps (row = 4*pooled + tap), so in the C
// fragment each lane's 4 accumulator registers ARE one pooling window of one channel: max /
// argmax in registers, only the pooled tensor (a quarter of the conv output) and the 1-byte
// argmax are written.  With a ReLU the argmax of an all-zero window is stored as 0xFF, so every
// pool backward (which routes the gradient to the tap equal to the argmax) applies ReLU' for
// free and the full conv output is never needed again.
// PK = 4: a 4x4/stride-4 pool.  The 16 rows of a group are ONE pooled output's 16 window taps
// (row = tap = 4*kh + kw), so lane (fr, fq) holds window row kh = fq of channel nf*16+fr in its 4
// registers: max over them, then over the 4 lane quads by two xor shuffles (ties to the lower tap,
// the unfused pool's raster order).  Both pool sizes use floor windows (a remainder row / column of
// the conv output that no window covers is never computed).
struct PoolEpi {
  unsigned char* am;
  const unsigned long long* rng;
  unsigned salt;
  float p;
  int dbg;  // HOPSX_PHASE_DBG: per-workgroup phase stamps (tools/dbg_convfwd.py)
};

// BNS: the output feeds a training-mode BatchNorm — the epilogue also accumulates per-channel sum and
// sum of squares of the stored (bf16) outputs into the zero-at-rest replicas
// bnacc[blockIdx % HOPSX_BN_NREP][2 CO] (norm.hip bn_apply_fin8_k finishes them), so the BN never
// re-reads its input for statistics.
//
// T0 > 0 (IN0): this conv's input is the output of the network's input layer (Cin0 = 1, stride 1, <= 9 taps:
// the 2x2 / 3x3 first conv of the MNIST models), and that layer is computed INSIDE the operand
// gather instead of by its own launch: each lane's 8-channel A chunk at (b, ih, iw) is
// act0(b0 + sum_taps px * w0) from the raw uint8 pixels with the input affine applied, in the
// same fp32 order as conv.hip conv_direct_fwd_k, rounded to bf16.  Every input-layer element is
// also stored once (for the backward: this conv's weight gradient and the input layer's ReLU'):
// by the lane whose conv tap is the first one covering it (kh == 0, or the last output row).
struct In0 {
  const void* x0;  // input-layer pixels [B][H0][W0] (C0 = 1), uint8
  float xscale, xshift;  // the input affine, applied on the fly (xscale != 0)
  const bf16_raw* w0;  // [C][KH0*KW0] bf16 (C = this conv's Cin)
  const float* b0;
  bf16_raw* y1;  // input-layer output [B][H][W][C], written here; nullptr: not kept (inference)
  int H0, W0, KH0, KW0, ph0, pw0, act0;
};

// IBN: this conv's input is act(bn(z)) of a training BatchNorm (stride 1 only) whose statistics the conv
// that produced z accumulated (acc: the zero-at-rest replica rows [HOPSX_BN_NREP][2C] + arrival words), and
// that BN's apply launch (norm.hip bn_apply_fin8_k) is folded in here: every workgroup folds the replicas
// into per-channel scale / shift in LDS with bn_apply_fin8_k's arithmetic, the operand gather reads z and
// applies act(z * scale + shift) in registers (bf16-rounded, as the apply stores it), and each BN output
// element is stored once for the backward (the In0 designated-lane rule: the lane whose tap is the first
// covering it).  Workgroup 0 publishes mean / rstd and the running statistics; the last workgroup to have
// read the replicas re-zeroes them.  x is z; the BN output goes to `a`.
typedef float cm_f32x2 __attribute__((ext_vector_type(2)));
typedef short cm_i16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 cm_bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t cm_u32x4 __attribute__((ext_vector_type(4)));

struct InBn {
  float* acc;
  const float* gamma;
  const float* beta;
  float *mean_out, *rstd_out, *rmean, *rvar;
  float momentum, eps;
  bf16_raw* a;  // the BN output [B][H][W][C]
  int M;        // BN rows (B*H*W)
  int act;
};

template <int NF, int KS, bool POOL = false, int UN = CM_UN, bool BNS = false, int T0 = 0, int PK = 2,
          bool IBN = false>
__global__ __launch_bounds__(256) void conv_fwd_mfma_k(const bf16_raw* __restrict__ x, const bf16_raw* __restrict__ w,
                                                      const float* __restrict__ bias, bf16_raw* __restrict__ y,
                                                      ConvGeom g, int act, int K, PoolEpi pe = PoolEpi{},
                                                      float* __restrict__ bnacc = nullptr, In0 i0 = In0{},
                                                      InBn ib = InBn{}) {
  constexpr int CO = NF * 16;
  extern __shared__ __attribute__((aligned(16))) bf16_raw cm_smem[];
  constexpr int cpr = KS * 4;  // 16-B chunks per weight row (K padded to 32*KS)
  constexpr int RS = cm_rs(cpr);  // row stride in chunks: the XOR swizzle stays inside the row
  bf16_raw* sw = cm_smem;                                 // [CO][RS*8]
  bf16_raw* scratch = cm_smem + CO * RS * 8;              // [waves][16][CO]
  // T0: input-layer weights [taps][C] and bias [C] as fp32 after the scratch
  float* sw0 = (float*)(scratch + CM_WAVES * 16 * CO);
  phase_mark(pe.dbg, 0);
  if constexpr (T0 > 0) {
    const int taps = T0 * T0;
    for (int i = threadIdx.x; i < (taps + 1) * g.C; i += 256) {
      const int t = i / g.C, c = i - t * g.C;
      sw0[i] = t < taps ? bf2f(i0.w0[c * taps + t]) : (i0.b0 ? i0.b0[c] : 0.f);
    }
  }
  __shared__ int ib_last;
  if constexpr (IBN) {
    // IBN: scale [C] and shift [C] in sw0's place, as bn_apply_fin8_k folds them
    for (int c = threadIdx.x; c < g.C; c += 256) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int r = 0; r < HOPSX_BN_NREP; ++r) {
        s += ib.acc[(long)r * 2 * g.C + c];
        q += ib.acc[(long)r * 2 * g.C + g.C + c];
      }
      const float mu = s / ib.M;
      const float var = fmaxf(q / ib.M - mu * mu, 0.f);
      const float rs = rsqrtf(var + ib.eps);
      const float scl = rs * (ib.gamma ? ib.gamma[c] : 1.f);
      sw0[c] = scl;
      sw0[g.C + c] = fmaf(-mu, scl, ib.beta ? ib.beta[c] : 0.f);
      if (blockIdx.x == 0) {
        ib.mean_out[c] = mu;
        ib.rstd_out[c] = rs;
        if (ib.rmean) {
          const float unb = ib.M > 1 ? var * ib.M / (ib.M - 1) : var;
          ib.rmean[c] = (1.f - ib.momentum) * ib.rmean[c] + ib.momentum * mu;
          ib.rvar[c] = (1.f - ib.momentum) * ib.rvar[c] + ib.momentum * unb;
        }
      }
    }
  }
  {
    // every staging load leaves before the first LDS write: one memory round trip, not one per
    // chunk (a load + ds_write loop waits for each load in turn)
    constexpr int NCHK = CO * cpr, NPT = (NCHK + 255) / 256;
    bf16x8 wv[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int co = i / cpr, c = i - co * cpr;
      const bool ok = i < NCHK && 8 * c < K;  // K % 8 == 0 (Cin % 8 == 0)
      wv[j] = *(const bf16x8*)(w + (ok ? (long)co * K + 8 * c : 0));
      wv[j] = zero_unless(wv[j], ok);
    }
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int co = i / cpr, c = i - co * cpr;
      if (i < NCHK) *(bf16x8*)(sw + co * RS * 8 + 8 * cm_swz(co, c, cpr)) = wv[j];
    }
  }
  __syncthreads();
  // IBN: every replica value this workgroup needs has been consumed (re-zeroed at the end by the last
  // arriver).  common.h grid_arrive_last's sharded protocol split in two: the shard ticket is taken here and
  // first used at the end, so its round trip hides behind the trip's loads (one word for every workgroup
  // serialised ~1024 arrivals, ~12 us, in front of the loads of a one-trip grid)
  unsigned ib_ticket = 0;
  unsigned* const ib_arr = (unsigned*)(ib.acc + (long)HOPSX_BN_NREP * 2 * g.C);
  if (IBN && threadIdx.x == 0) ib_ticket = atomicAdd(ib_arr + 32u * ((blockIdx.x & 7u) + 1u), 1u);
  phase_mark(pe.dbg, 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  static_assert(PK == 2 || (PK == 4 && T0 == 0), "pool 4x4 without the fused input layer");
  static_assert(!IBN || (T0 == 0 && !POOL), "input BN without the fused input layer / pool");
  const int PH = g.OH / PK, PW = g.OW / PK;
  const int M = POOL ? g.B * PH * PW * PK * PK : g.B * g.OH * g.OW;  // A rows (pooled: PK*PK taps per output)
  const int ngroups = (M + 15) / 16;
  bf16_raw* sc = scratch + wave * 16 * CO;
  float bv[NF];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) bv[nf] = bias ? bias[nf * 16 + fr] : 0.f;
  const uint64_t dkey = POOL && pe.p > 0.f ? drop_key(pe.rng, pe.salt) : 0;
  // IBN: this lane's 8 input channels are the same at every tap (32 % C == 0: ci = 8*fq mod C), so their
  // scale / shift pairs live in registers
  cm_f32x2 isc[4], ish[4];
  if constexpr (IBN) {
    const int ci0 = (8 * fq) & (g.C - 1);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      isc[p] = (cm_f32x2){sw0[ci0 + 2 * p], sw0[ci0 + 2 * p + 1]};
      ish[p] = (cm_f32x2){sw0[g.C + ci0 + 2 * p], sw0[g.C + ci0 + 2 * p + 1]};
    }
  }
  float st1[NF], st2[NF];  // BNS: this lane's channel partials (channel nf*16 + fr)
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) { st1[nf] = 0.f; st2[nf] = 0.f; }
  for (int g0 = (blockIdx.x * CM_WAVES + wave) * UN; g0 < ngroups; g0 += gridDim.x * CM_WAVES * UN) {
    bf16x8 a[UN][KS];
    // T0: the input layer's pixels / lane bookkeeping of this trip (sized 1 when unused)
    constexpr int TU = T0 > 0 || IBN ? UN : 1, TK = T0 > 0 || IBN ? KS : 1, TT = T0 > 0 ? T0 * T0 : 1;
    unsigned i0px[TU][TK][TT];
    int i0ci[TU][TK];
    long i0off[TU][TK];
    bool i0ok[TU][TK], i0wr[TU][TK];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int px = (g0 + u) * 16 + fr;
      const bool pok = (g0 + u) < ngroups && px < M;
      const int pp = pok ? px : 0;
      int b, oh, ow;
      if constexpr (POOL) {
        constexpr int SH = PK == 2 ? 2 : 4;  // log2 of the taps per window
        const int po = pp >> SH, tap = pp & (PK * PK - 1);  // pooled output index, window tap
        const int pr = po / PW, pw_ = po - pr * PW;
        b = pr / PH;
        oh = PK * (pr - b * PH) + tap / PK;
        ow = PK * pw_ + tap % PK;
      } else {
        b = g.fOHW.div(pp);
        const int rem = pp - b * (g.OH * g.OW);
        oh = g.fOW.div(rem);
        ow = rem - oh * g.OW;
      }
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const int k0 = kk * 32 + 8 * fq;
        const int kc = k0 < K ? k0 : 0;
        const int t = g.fC.div(kc), ci = kc - t * g.C;
        const int kh = g.fKW.div(t), kw = t - kh * g.KW;
        const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
        const bool ok = pok && k0 < K && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const long off = ok ? (((long)b * g.H + ih) * g.W + iw) * g.C + ci : 0;
        if constexpr (T0 > 0) {
          // input layer at (b, ih, iw): issue its T0 x T0 pixel loads now, evaluate after the loop
          // (every load of the trip in flight before the first use)
          i0ok[u][kk] = ok;
          i0ci[u][kk] = ci;
          i0off[u][kk] = off;
          i0wr[u][kk] = ok && (kh == 0 || oh == g.OH - 1) && (kw == 0 || ow == g.OW - 1);
#pragma unroll
          for (int a0 = 0; a0 < T0; ++a0)
#pragma unroll
            for (int c0 = 0; c0 < T0; ++c0) {
              const int y0 = ih - i0.ph0 + a0, x0c = iw - i0.pw0 + c0;
              const bool in = ok && y0 >= 0 && y0 < i0.H0 && x0c >= 0 && x0c < i0.W0;
              const long pi = in ? ((long)b * i0.H0 + y0) * i0.W0 + x0c : 0;
              const unsigned raw = ((const uint8_t*)i0.x0)[pi];  // one unconditional byte load per tap
              i0px[u][kk][a0 * T0 + c0] = in ? raw : 0xFFFFFFFFu;
            }
        } else if constexpr (IBN) {
          a[u][kk] = *(const bf16x8*)(x + off);  // z: the BN applied after the loop
          i0ok[u][kk] = ok;
          i0off[u][kk] = off;
          i0wr[u][kk] = ok && (kh == 0 || oh == g.OH - 1) && (kw == 0 || ow == g.OW - 1);
        } else {
          a[u][kk] = zero_unless(*(const bf16x8*)(x + off), ok);
        }
      }
    }
    if constexpr (IBN) {
      // act(z * scale + shift) rounded to bf16: bn_apply_fin8_k's fp32 fma per element, two at a time
      // (v_pk_fma_f32), the round-to-nearest-even by the conversion instruction (common.h f2bf's bits for
      // every finite value) and the ReLU on the bf16 bits (max_i16 with 0: a negative bf16 is a negative
      // int16) — the gather visits every element once per tap, so this runs KH*KW times per element;
      // padding taps stay zero
      const bool relu = ib.act == ACT_RELU;
#pragma unroll
      for (int u = 0; u < UN; ++u)
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const cm_u32x4 r = __builtin_bit_cast(cm_u32x4, a[u][kk]);
          cm_u32x4 o;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            cm_f32x2 v = {__uint_as_float(r[p] << 16), __uint_as_float(r[p] & 0xffff0000u)};
            v = __builtin_elementwise_fma(v, isc[p], ish[p]);
            cm_i16x2 b = __builtin_bit_cast(cm_i16x2, __builtin_convertvector(v, cm_bf16x2));
            if (relu) b = __builtin_elementwise_max(b, (cm_i16x2){0, 0});
            o[p] = __builtin_bit_cast(uint32_t, b);
          }
          const bf16x8 t = __builtin_bit_cast(bf16x8, o);
          a[u][kk] = zero_unless(t, i0ok[u][kk]);
          if (i0wr[u][kk]) *(bf16x8*)(ib.a + i0off[u][kk]) = t;
        }
    }
    if constexpr (T0 > 0) {
      // input layer: act0(b0 + sum_taps px * w0) in conv_direct_fwd_k's fp32 order, bf16-rounded;
      // stored once (designated lane) for the backward
#pragma unroll
      for (int u = 0; u < UN; ++u)
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int ci = i0ci[u][kk];
          float acc[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = sw0[T0 * T0 * g.C + ci + j];
#pragma unroll
          for (int t = 0; t < T0 * T0; ++t) {
            const unsigned raw = i0px[u][kk][t];
            const float pv = raw == 0xFFFFFFFFu ? 0.f : fmaf((float)raw, i0.xscale, i0.xshift);
            const float* wr = sw0 + t * g.C + ci;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = fmaf(pv, wr[j], acc[j]);
          }
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(apply_act(acc[j], i0.act0));
          a[u][kk] = zero_unless(v, i0ok[u][kk]);
          if (i0.y1 && i0wr[u][kk]) *(bf16x8*)(i0.y1 + i0off[u][kk]) = v;
        }
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      if (g0 + u >= ngroups) break;
      f32x4 acc[NF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[nf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const int co = nf * 16 + fr;
          const bf16x8 bfr = *(const bf16x8*)(sw + co * RS * 8 + 8 * cm_swz(co, kk * 4 + fq, cpr));
          acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][kk], bfr, acc[nf], 0, 0, 0);
        }
      }
      if (u == 0) phase_mark(pe.dbg, 2);
      if constexpr (POOL && PK == 4) {
        // lane (fr, fq): window row fq of pooled output g0+u, channel nf*16+fr; the 4 quads' maxima
        // combined by xor shuffles, then lane (fr, fq) stores channel nf*16+fr for nf % 4 == fq (a
        // 128-B row per 4 fragments)
        const long po = g0 + u;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          float best = -INFINITY;
          int bi = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = bf2f(f2bf(apply_act(acc[nf][r] + bv[nf], act)));
            if (v > best) { best = v; bi = fq * 4 + r; }
          }
#pragma unroll
          for (int d = 16; d <= 32; d *= 2) {
            const float ob = __shfl_xor(best, d, 64);
            const int oi = __shfl_xor(bi, d, 64);
            if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
          }
          if (act == ACT_RELU && !(best > 0.f)) bi = 0xFF;
          const int co = nf * 16 + fr;
          if ((nf & 3) == fq) {
            if (pe.p > 0.f)
              best = uniform01(dkey, (uint64_t)(po * CO + co)) >= pe.p ? best * (1.f / (1.f - pe.p)) : 0.f;
            y[po * CO + co] = f2bf(best);
            pe.am[po * CO + co] = (unsigned char)bi;
          }
        }
        continue;
      }
      if constexpr (POOL) {
        // lane (fr, fq): channel nf*16+fr of pooled output 4*(g0+u)+fq; acc[nf][0..3] = its window
        const int po = (g0 + u) * 4 + fq;
        unsigned char* sa = (unsigned char*)(sc + 4 * CO);  // [4][CO] argmax bytes after [4][CO] bf16
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          float best = -INFINITY;
          int bi = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // round to bf16 first: ties and the stored max follow the unfused conv -> pool chain
            const float v = bf2f(f2bf(apply_act(acc[nf][r] + bv[nf], act)));
            if (v > best) { best = v; bi = r; }
          }
          if (act == ACT_RELU && !(best > 0.f)) bi = 0xFF;  // ReLU'(window) == 0: no gradient
          const int co = nf * 16 + fr;
          if (pe.p > 0.f)
            best = uniform01(dkey, (uint64_t)((long)po * CO + co)) >= pe.p ? best * (1.f / (1.f - pe.p)) : 0.f;
          sc[fq * CO + co] = f2bf(best);
          sa[fq * CO + co] = (unsigned char)bi;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int nout = g.B * PH * PW;
        const int pbase = (g0 + u) * 4;
        for (int c = lane; c < 4 * CO / 8; c += 64) {  // 4 pooled rows x CO, 16-B vectors
          const int row = c / (CO / 8), col = (c - row * (CO / 8)) * 8;
          if (pbase + row < nout) *(bf16x8*)(y + (long)(pbase + row) * CO + col) = *(const bf16x8*)(sc + row * CO + col);
        }
        for (int c = lane; c < 4 * CO / 8; c += 64) {  // argmax bytes, 8-B vectors
          const int row = c / (CO / 8), col = (c - row * (CO / 8)) * 8;
          if (pbase + row < nout) *(uint2*)(pe.am + (long)(pbase + row) * CO + col) = *(const uint2*)(sa + row * CO + col);
        }
        __builtin_amdgcn_wave_barrier();
        continue;
      }
      // epilogue through the wave's LDS scratch: C map col = lane&15 (co), row = (lane>>4)*4 + r (pixel)
      const int base = (g0 + u) * 16;
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bf16_raw o = f2bf(apply_act(acc[nf][r] + bv[nf], act));
          sc[(fq * 4 + r) * CO + nf * 16 + fr] = o;
          if constexpr (BNS) {
            const float v = base + fq * 4 + r < M ? bf2f(o) : 0.f;
            st1[nf] += v;
            st2[nf] = fmaf(v, v, st2[nf]);
          }
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes landed
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = lane; c < 16 * CO / 8; c += 64) {
        const int row = c / (CO / 8), col = (c - row * (CO / 8)) * 8;
        if (base + row < M) *(bf16x8*)(y + (long)(base + row) * CO + col) = *(const bf16x8*)(sc + row * CO + col);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if constexpr (BNS) {
    // fold the 4 pixel quads of each channel (lanes fr, fr+16, fr+32, fr+48), then the 4 waves in
    // LDS (the staging scratch is free once every wave left the loop), one atomic per channel and
    // statistic per workgroup into this workgroup's replica row
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) {
      st1[nf] += __shfl_xor(st1[nf], 16, 64);
      st1[nf] += __shfl_xor(st1[nf], 32, 64);
      st2[nf] += __shfl_xor(st2[nf], 16, 64);
      st2[nf] += __shfl_xor(st2[nf], 32, 64);
    }
    __syncthreads();
    float* red = (float*)scratch;  // [CM_WAVES][2][CO] floats <= the [CM_WAVES][16][CO] bf16 scratch
    if (fq == 0) {
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        red[(wave * 2) * CO + nf * 16 + fr] = st1[nf];
        red[(wave * 2 + 1) * CO + nf * 16 + fr] = st2[nf];
      }
    }
    __syncthreads();
    float* dst = bnacc + (long)(blockIdx.x % HOPSX_BN_NREP) * 2 * CO;
    const bool det = det_on();
    if (det) det_turn_begin(DET_BN_FWD, blockIdx.x);
    for (int e = threadIdx.x; e < 2 * CO; e += 256) {
      const int which = e / CO, c = e - which * CO;
      float t = 0.f;
#pragma unroll
      for (int wv = 0; wv < CM_WAVES; ++wv) t += red[(wv * 2 + which) * CO + c];
      atomicAdd(dst + e, t);
    }
    if (det) det_turn_end(DET_BN_FWD, blockIdx.x, gridDim.x);
  }
  if constexpr (IBN) {
    if (threadIdx.x == 0) {
      const unsigned G = gridDim.x, shard = blockIdx.x & 7u;
      int last = 0;
      if (ib_ticket == (G - shard + 7u) / 8u - 1u) {  // this shard's last member: arrive on the top word
        atomicExch(ib_arr + 32u * (shard + 1u), 0u);
        if (atomicAdd(ib_arr, 1u) == (G < 8u ? G : 8u) - 1u) {
          atomicExch(ib_arr, 0u);
          last = 1;
        }
      }
      ib_last = last;
    }
    __syncthreads();
    if (ib_last)
      for (int i = threadIdx.x; i < HOPSX_BN_NREP * 2 * g.C; i += 256) ib.acc[i] = 0.f;
  }
  if (pe.dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    phase_mark(pe.dbg, 3);
  }
}

// ---------------------------------------------------------------------------- dgrad
// dX[b,ih,iw,ci] = sum_{kh,kw,co} dY'[b,oh,ow,co] W[co,kh,kw,ci]  (stride 1:
// oh = ih + ph - kh*dh), dY' = dY * act'(y); output masked by act'(yprev) and its
// per-channel sums accumulated into `colsum` (the previous layer's bias gradient).
//
// K0 > 0 fuses the weight gradient of the PREVIOUS layer into the epilogue: when that layer is
// the network's input layer (its input needs no gradient) with a K0 = KH0*KW0*1-tap reduction,
// dX here is only ever consumed by that layer's wgrad, so instead of storing dX the epilogue
// multiplies each masked dX row by the input layer's im2col row (K0 raw pixels, uint8 with the
// fused affine or bf16) and accumulates dW0[ci][k] in registers; the previous layer's bias
// gradient is the existing colsum.  Saves the dX write/re-read and a whole launch.
struct DgradArgs {
  const bf16_raw* dy;
  const bf16_raw* w;
  bf16_raw* dx;
  const bf16_raw* yprev;
  int act_prev;
  float* colsum;
  const bf16_raw* y;
  int yact;
  ConvGeom g;
  int K;
  int wvec;
  const void* x0;
  float xscale, xshift;
  ConvGeom gi;
  float* dw0;
  int dbg;
  // optional gradient of the same input from another consumer (a ResNet block's identity shortcut):
  // added before the act'(yprev) mask, replacing autograd's separate add launch
  const bf16_raw* addend;
  // 1: XCD-aware block order (consecutive pixel groups, which share dY halo rows, on one XCD's L2)
  int xcd;
  // BN column reduction in the epilogue (bnacc != null): this conv's input is the output of a training
  // BatchNorm whose only autograd consumer is this conv, so the stored dX (after the addend and the
  // act'(yprev) mask) IS that BN's masked output gradient g.  The epilogue adds sum g and
  // sum g * (z - mean) * rstd (z = the BN input, bnz) per channel into the zero-at-rest replica rows
  // bnacc[bid % HOPSX_BN_NREP][2C] that norm.hip bn_bwd_apply_fin8_k folds: the BN backward's own
  // column-reduction launch (bn_colred8_k) disappears.
  const bf16_raw* bnz;
  const float* bnmean;
  const float* bnrstd;
  float* bnacc;
};

// bid / nblk: this workgroup's index and the number of workgroups doing dgrad work (a paired
// launch, conv_bwd_pair_k, hands the remaining workgroups to the weight gradient)
template <int NF, int KS, int K0, int UN>
__device__ __forceinline__ void conv_dgrad_body(const DgradArgs& A, int bid, int nblk) {
  if (A.xcd) bid = xcd_remap(bid, nblk);
  const bf16_raw* __restrict__ dy = A.dy;
  const bf16_raw* __restrict__ w = A.w;
  bf16_raw* __restrict__ dx = A.dx;
  const bf16_raw* __restrict__ yprev = A.yprev;
  const int act_prev = A.act_prev;
  float* __restrict__ colsum = A.colsum;
  const bf16_raw* __restrict__ y = A.y;
  const int yact = A.yact;
  const ConvGeom& g = A.g;
  const int K = A.K, wvec = A.wvec;
  const void* __restrict__ x0 = A.x0;
  const float xscale = A.xscale, xshift = A.xshift;
  const ConvGeom& gi = A.gi;
  float* __restrict__ dw0 = A.dw0;
  const int dbg = A.dbg;
  phase_mark(dbg, 0);
  constexpr int CI = NF * 16;
  extern __shared__ __attribute__((aligned(16))) bf16_raw cm_smem[];
  constexpr int cpr = KS * 4;
  constexpr int RS = cm_rs(cpr);
  // W image [KP = 32*KS rows k = (kh,kw,co)][CI] rc-swizzled: every 16-B chunk of W (8 ci of one
  // (co,kh,kw) row) lands whole in image row k, so staging is one 16-B load + one ds_write_b128 per
  // chunk; the MFMA B fragments (8 consecutive k at one ci) come back via ds_read_b64_tr_b16.
  (void)RS;
  bf16_raw* sw = cm_smem;                     // [KP][CI]
  bf16_raw* scratch = cm_smem + CI * RS * 8;  // [waves][16][CI]   (CI*RS*8 >= KP*CI)
  float* csum = (float*)(scratch + CM_WAVES * 16 * CI);  // [CI]
  constexpr int CPR = CI / 8;  // 16-B chunks per image row
  const int T = g.KH * g.KW;
  for (int i = threadIdx.x; i < (cpr * 8 - K) * CPR; i += blockDim.x) {  // zero the K padding rows
    const int kk = K + i / CPR, c8 = i % CPR;
    *(bf16x8*)(sw + kk * CI + 8 * (c8 ^ rc_swz(kk, CPR))) = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  }
  if (wvec) {
    // a batch's loads all leave before its LDS writes (one round trip per batch, not per chunk)
    constexpr int NPT = (32 * KS * CPR + 255) / 256, BAT = NPT < 8 ? NPT : 8;
    const int nch = K * CPR;
#pragma unroll
    for (int j0 = 0; j0 < NPT; j0 += BAT) {
      bf16x8 wv[BAT];
#pragma unroll
      for (int j = 0; j < BAT; ++j) {
        const int i = threadIdx.x + 256 * (j0 + j);
        wv[j] = *(const bf16x8*)(w + (i < nch ? (long)i * 8 : 0));
      }
#pragma unroll
      for (int j = 0; j < BAT; ++j) {
        const int i = threadIdx.x + 256 * (j0 + j);
        if (i < nch) {
          const int r = i / CPR, c8 = i - r * CPR;  // source row r = co*T + t
          const int co = r / T, t = r - co * T;
          const int kk = t * g.CO + co;
          *(bf16x8*)(sw + kk * CI + 8 * (c8 ^ rc_swz(kk, CPR))) = wv[j];
        }
      }
    }
  } else {
    for (int i = threadIdx.x; i < K * CI; i += blockDim.x) {
      const int ci = i % CI, r = i / CI;
      const int co = r / T, t = r - co * T;
      const int kk = t * g.CO + co;
      sw[kk * CI + 8 * ((ci >> 3) ^ rc_swz(kk, CPR)) + (ci & 7)] = w[i];
    }
  }
  float* cwsum = csum + CM_RSLOTS * CI;  // [slot][CI][K0] (K0 > 0); csum is [slot][CI]
  const bool bn = A.bnacc != nullptr;
  float* csum2 = cwsum + CM_RSLOTS * CI * (K0 > 0 ? K0 : 0);  // [slot][CI] (bn): sum g * xhat
  // per (K step, fq) gather constants, built once per workgroup: output-pixel displacement of the
  // tap and the element offset relative to the lane's own pixel (x: dh, y: dw, z: offset, w: valid)
  int4* ktab = (int4*)(csum2 + (bn ? CM_RSLOTS * CI : 0));
  for (int i = threadIdx.x; i < KS * 4; i += blockDim.x) {
    const int kk = i >> 2, q = i & 3;
    const int k0 = kk * 32 + 8 * q;
    const int kc = k0 < K ? k0 : 0;
    const int t = g.fCO.div(kc), co = kc - t * g.CO;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const int dh = g.ph - kh * g.dh, dwv = g.pw - kw * g.dw;  // stride 1: oh = ih + dh, ow = iw + dw
    ktab[i] = make_int4(dh, dwv, (dh * g.OW + dwv) * g.CO + co, k0 < K);
  }
  __syncthreads();
  phase_mark(dbg, 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int M = g.B * g.H * g.W;
  const int ngroups = (M + 15) / 16;
  const bf16_raw* yp = y ? y : dy;
  const bf16_raw* ypp = yprev ? yprev : dx;
  bf16_raw* sc = scratch + wave * 16 * CI;
  float cacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // bn: sum g * xhat, and the batch mean / rstd of this lane's 8 fixed output channels
  float cacc2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, bmu[8], brs[8];
  if (bn) {
    const int col = (lane % (CI / 8)) * 8;  // (lane + 64 q) % (CI / 8): CI / 8 divides 64
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmu[j] = A.bnmean[col + j];
      brs[j] = A.bnrstd[col + j];
    }
  }
  float cw[8][K0 > 0 ? K0 : 1];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k < (K0 > 0 ? K0 : 1); ++k) cw[j][k] = 0.f;
  constexpr int NCH = 16 * CI / 8;      // 16-B output chunks per 16-pixel group
  constexpr int CPL = (NCH + 63) / 64;  // of which this lane stores CPL (c = lane + 64 q)
  constexpr int XK = K0 > 0 ? K0 : 1;
  int bo1[NF], bo2[NF];  // this lane's B-fragment LDS offsets at K step 0
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int col = nf * 16 + 4 * (lane & 3);
    const int k1 = 8 * fq + ((lane & 15) >> 2), k2 = k1 + 4;
    bo1[nf] = k1 * CI + 8 * ((col >> 3) ^ rc_swz(k1, CPR)) + (col & 7);
    bo2[nf] = k2 * CI + 8 * ((col >> 3) ^ rc_swz(k2, CPR)) + (col & 7);
  }
  for (int g0 = (bid * CM_WAVES + wave) * UN; g0 < ngroups; g0 += nblk * CM_WAVES * UN) {
    bf16x8 a[UN][KS];
    bf16x8 pmv[UN][CPL];  // epilogue operands prefetched with the A fragments: one round trip
    bf16x8 bzv[UN][CPL];  // bn: the BN input z at the stored chunks
    // input-layer pixels for the fused wgrad: RAW loads (uint8 or bf16 bits) with the validity kept
    // aside and the conversion at the consumer — a conversion next to its load makes the compiler
    // wait for each load in turn (one full memory round trip per tap)
    unsigned xk[UN][CPL][XK];
    unsigned long long xin = 0;  // bit (u*CPL+q)*XK+k
    unsigned okm = 0;            // A-fragment validity, bit u*KS+kk
    static_assert(UN * CPL * XK <= 64 && UN * KS <= 32, "validity masks");
    // 32-bit index math throughout (host: every tensor < 2^31 elements), tap constants from ktab
    int4 kt[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) kt[kk] = ktab[kk * 4 + fq];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int px = (g0 + u) * 16 + fr;
      const bool pok = (g0 + u) < ngroups && px < M;
      const int pp = pok ? px : 0;
      const int b = g.fHW.div(pp), rem = pp - b * (g.H * g.W);
      const int ih = g.fW.div(rem), iw = rem - ih * g.W;
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int c = lane + 64 * q;
        const int row = c / (CI / 8), col = (c - row * (CI / 8)) * 8;
        const int p = (g0 + u) * 16 + row;
        const bool okc = c < NCH && (g0 + u) < ngroups && p < M;
        const int pc = okc ? p : 0;
        pmv[u][q] = *(const bf16x8*)(ypp + (pc * CI + (okc ? col : 0)));  // unconditional (ypp = yprev or dx)
        if (bn) bzv[u][q] = *(const bf16x8*)(A.bnz + (pc * CI + (okc ? col : 0)));
        if constexpr (K0 > 0) {
          // im2col row of the input layer at this pixel (= the input layer's output pixel)
          const int bb = g.fHW.div(pc), rr = pc - bb * (g.H * g.W);
          const int oh = g.fW.div(rr), ow = rr - oh * g.W;
          const int ohs = oh * gi.sh - gi.ph, ows = ow * gi.sw - gi.pw, rowb = bb * gi.H;
          int xo[K0];
#pragma unroll
          for (int k = 0; k < K0; ++k) {
            const int kh = gi.fKW.div(k), kw = k - kh * gi.KW;  // Cin = 1 (uniform: scalar ops)
            const int ih0 = ohs + kh * gi.dh, iw0 = ows + kw * gi.dw;
            const bool in = okc && (unsigned)ih0 < (unsigned)gi.H && (unsigned)iw0 < (unsigned)gi.W;
            xo[k] = in ? (rowb + ih0) * gi.W + iw0 : 0;
            xin |= (unsigned long long)in << ((u * CPL + q) * XK + k);
          }
          if (xscale != 0.f) {  // uniform: the K0 loads of either form leave together
#pragma unroll
            for (int k = 0; k < K0; ++k) xk[u][q][k] = ((const uint8_t*)x0)[xo[k]];
          } else {
#pragma unroll
            for (int k = 0; k < K0; ++k) xk[u][q][k] = ((const bf16_raw*)x0)[xo[k]];
          }
        }
      }
      // raw gathers, validity kept aside and applied at the MFMA: no ALU op on a loaded value
      // (and no branch) between the loads, so all of a trip's gathers are in flight together
      const int pix = ((b * g.OH + ih) * g.OW + iw) * g.CO;
      int ao[KS];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const int oh = ih + kt[kk].x, ow = iw + kt[kk].y;
        const bool ok = pok && kt[kk].w && (unsigned)oh < (unsigned)g.OH && (unsigned)ow < (unsigned)g.OW;
        ao[kk] = ok ? pix + kt[kk].z : 0;
        okm |= (unsigned)ok << (u * KS + kk);
      }
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) a[u][kk] = *(const bf16x8*)(dy + ao[kk]);
      if (y) {  // uniform: no load when dY is pre-masked
        bf16x8 yv[KS];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) yv[kk] = *(const bf16x8*)(yp + ao[kk]);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) mask8(a[u][kk], yv[kk], yact);
      }
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      if (g0 + u >= ngroups) break;
      f32x4 acc[NF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[nf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          // transposed read (T10): lane 4q+p addresses rows k1 = 32kk+8fq+q (+4), ci = 16nf+4p..+3;
          // rc_swz looks at k bits 0, 1 and 3 only, so the 32kk row step is a constant offset
          const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(sw + bo1[nf] + kk * 32 * CI));
          const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(sw + bo2[nf] + kk * 32 * CI));
          const bf16x8 bfr = (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
          acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(zero_unless(a[u][kk], (okm >> (u * KS + kk)) & 1), bfr,
                                                             acc[nf], 0, 0, 0);
        }
      }
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[(fq * 4 + r) * CI + nf * 16 + fr] = f2bf(acc[nf][r]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int base = (g0 + u) * 16;
#pragma unroll
      for (int q = 0; q < CPL; ++q) {  // a lane always lands on the same 8 columns
        const int c = lane + 64 * q;
        const int row = c / (CI / 8), col = (c - row * (CI / 8)) * 8;
        if (c < NCH && base + row < M) {
          bf16x8 v = *(const bf16x8*)(sc + row * CI + col);
          if (A.addend) {  // bf16 + bf16 -> bf16, exactly autograd's accumulation of the two parts
            const bf16x8 a = *(const bf16x8*)(A.addend + (long)(base + row) * CI + col);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(bf2f((uint16_t)v[j]) + bf2f((uint16_t)a[j]));
          }
          if (yprev) mask8(v, pmv[u][q], act_prev);
          if constexpr (K0 > 0) {
            float xv[K0];
#pragma unroll
            for (int k = 0; k < K0; ++k) {
              const unsigned r = xk[u][q][k];
              const float f = xscale != 0.f ? fmaf((float)r, xscale, xshift) : bf2f((uint16_t)r);
              xv[k] = (xin >> ((u * CPL + q) * XK + k)) & 1 ? f : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float d = bf2f((uint16_t)v[j]);
              cacc[j] += d;
#pragma unroll
              for (int k = 0; k < K0; ++k) cw[j][k] = fmaf(d, xv[k], cw[j][k]);
            }
          } else {
            *(bf16x8*)(dx + (long)(base + row) * CI + col) = v;
#pragma unroll
            for (int j = 0; j < 8; ++j) cacc[j] += bf2f((uint16_t)v[j]);
            if (bn) {  // the stored bf16 g, as bn_colred8_k would read it back
#pragma unroll
              for (int j = 0; j < 8; ++j)
                cacc2[j] = fmaf(bf2f((uint16_t)v[j]), (bf2f((uint16_t)bzv[u][q][j]) - bmu[j]) * brs[j], cacc2[j]);
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  phase_mark(dbg, 2);
  if (colsum || bn) {
    // lanes l, l + CI/8, l + 2*CI/8, ... own the same 8 columns: fold them inside each 16-lane row
    // with DPP rotations (plain VALU; ds_bpermute shuffles were ~160 LDS round trips here), then
    // one LDS partial per (wave, row), summed after one barrier
    constexpr int CW = CI / 8 < 16 ? CI / 8 : 16;
    const int slot = wave * 4 + (lane >> 4), rl = lane & 15;
#pragma unroll
    for (int j = 0; j < 8; ++j) cacc[j] = row_fold<CW>(cacc[j]);
    if (rl < CW) {
#pragma unroll
      for (int j = 0; j < 8; ++j) csum[slot * CI + rl * 8 + j] = cacc[j];
    }
    if (bn) {
#pragma unroll
      for (int j = 0; j < 8; ++j) cacc2[j] = row_fold<CW>(cacc2[j]);
      if (rl < CW) {
#pragma unroll
        for (int j = 0; j < 8; ++j) csum2[slot * CI + rl * 8 + j] = cacc2[j];
      }
    }
    if constexpr (K0 > 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < K0; ++k) cw[j][k] = row_fold<CW>(cw[j][k]);
      if (rl < CW) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int k = 0; k < K0; ++k) cwsum[slot * CI * K0 + (rl * 8 + j) * K0 + k] = cw[j][k];
      }
    }
    __syncthreads();
    const bool det = det_on();
    if (det) det_turn_begin(DET_DGRAD_COLSUM, (unsigned)bid);
    // bn: this workgroup's replica row of the BN accumulator ([sum g | sum g * xhat]), else the bias
    // gradient (the host never asks for both)
    float* d1 = bn ? A.bnacc + (long)(bid % HOPSX_BN_NREP) * 2 * CI : colsum;
    for (int i = threadIdx.x; i < CI; i += blockDim.x) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < CM_RSLOTS; ++r) v += csum[r * CI + i];
      if (v != 0.f) atomicAdd(d1 + i, v);
    }
    if (bn)
      for (int i = threadIdx.x; i < CI; i += blockDim.x) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < CM_RSLOTS; ++r) v += csum2[r * CI + i];
        if (v != 0.f) atomicAdd(d1 + CI + i, v);
      }
    if constexpr (K0 > 0) {
      // no-return f32 atomics: ~1 us for ~200 workgroups into these few rows (row 'Global float atomics')
      for (int i = threadIdx.x; i < CI * K0; i += blockDim.x) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < CM_RSLOTS; ++r) v += cwsum[r * CI * K0 + i];
        if (v != 0.f) atomicAdd(dw0 + i, v);
      }
    }
    if (det) det_turn_end(DET_DGRAD_COLSUM, (unsigned)bid, (unsigned)nblk);
  }
  if (dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    phase_mark(dbg, 3);
  }
}


template <int NF, int KS, int K0, int UN>
__global__ __launch_bounds__(256) void conv_dgrad_mfma_k(DgradArgs A) {
  conv_dgrad_body<NF, KS, K0, UN>(A, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------- wgrad
// dW[co][k] += sum_px dY'[px][co] * im2col(X)[px][k] (dY' = dY * act'(y)), db[co] += sum_px dY'[px][co]
// for short convs (CO <= 64, C % 8 == 0).  The generic split-K GEMM walks 4+ K-tiles per
// workgroup with a workgroup barrier and a dependent global round trip each.  Here:
//   * grid = (pixel groups, 16*NFKW-column blocks of K): a workgroup owns a CO x 16*NFKW
//     output block and a contiguous run of 32-pixel chunks (the MFMA K), split over its 4 waves;
//   * each wave stages its chunk (dY' and the 16-B im2col gathers of X) into a wave-private
//     LDS image (no workgroup barrier in the loop) while the next chunk's loads are in flight,
//     and reads both MFMA operands back transposed with ds_read_b64_tr_b16 (T10): the
//     reduction runs over pixels, the rows of the NHWC images;
//   * the waves meet once: lane-major float4 partials in LDS (conflict-free), summed, restaged
//     row-major, and the workgroup leaves one coalesced no-return f32 atomic per output element.
// (LDS float atomics were measured at ~200 cycles per ds_add_f32 here: not used.)
constexpr int WG_PX = 32;  // pixels per wave chunk (= MFMA K)

struct WgradArgs {
  const bf16_raw* dy;
  const bf16_raw* x;
  const bf16_raw* y;
  int yact;
  float* dw;
  float* dbias;
  ConvGeom g;
  int K, cpw, dbg;
};

// (bx, by): pixel-group and column-block coordinates of this workgroup
template <int NFC, int NFKW>
__device__ __forceinline__ void conv_wgrad_body(const WgradArgs& A, int bx, int by, int nbx, int nby) {
  const bf16_raw* __restrict__ dy = A.dy;
  const bf16_raw* __restrict__ x = A.x;
  const bf16_raw* __restrict__ y = A.y;
  const int yact = A.yact;
  float* __restrict__ dw = A.dw;
  float* __restrict__ dbias = A.dbias;
  const ConvGeom& g = A.g;
  const int K = A.K, cpw = A.cpw, dbg = A.dbg;
  phase_mark(dbg, 0);
  constexpr int CO = NFC * 16, KB = NFKW * 16;
  constexpr int DCH = WG_PX * CO / 8 / 64;  // 16-B dY chunks per lane per pixel chunk
  constexpr int XCH = WG_PX * KB / 8 / 64;  // 16-B im2col chunks per lane per pixel chunk
  static_assert(DCH >= 1 && XCH >= 1, "tile too small");
  constexpr int NFR = NFC * NFKW;           // output fragments per wave
  extern __shared__ __attribute__((aligned(16))) bf16_raw cm_smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bf16_raw* sA = cm_smem + wave * WG_PX * (CO + KB);  // [px][CO]  rc-swizzled
  bf16_raw* sB = sA + WG_PX * CO;                     // [px][KB]  rc-swizzled
  const int kb0 = by * KB;
  const int M = g.B * g.OH * g.OW;
  const int nchunks = (M + WG_PX - 1) / WG_PX;
  // this lane's fixed columns: dY chunk column dc (8 channels), im2col chunk column xc (8 ci of one tap)
  const int dc = lane % (CO / 8);
  const int xc = lane % (KB / 8);
  const int kcol = kb0 + xc * 8;
  const bool kin = kcol < K;
  const int tap = kin ? g.fC.div(kcol) : 0, ci0 = kin ? kcol - tap * g.C : 0;
  const int kh = g.fKW.div(tap), kw = tap - kh * g.KW;
  const bool do_bias = dbias != nullptr && by == 0;
  f32x4 acc[NFC][NFKW];
#pragma unroll
  for (int i = 0; i < NFC; ++i)
#pragma unroll
    for (int j = 0; j < NFKW; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float cacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;

  bf16x8 dv[DCH], xv[XCH];
  auto load = [&](int c) {
#pragma unroll
    for (int i = 0; i < DCH; ++i) {
      const int p = c * WG_PX + (lane + 64 * i) / (CO / 8);
      const bool ok = p < M;
      const long o = (long)(ok ? p : 0) * CO + dc * 8;
      bf16x8 v = zero_unless(*(const bf16x8*)(dy + o), ok);
      if (y) mask8(v, *(const bf16x8*)(y + o), yact);
      dv[i] = v;
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int p = c * WG_PX + (lane + 64 * i) / (KB / 8);
      const int pc = p < M ? p : 0;
      const int b = g.fOHW.div(pc), rem = pc - b * (g.OH * g.OW);
      const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
      const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
      const bool ok = kin && p < M && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const long o = ok ? (((long)b * g.H + ih) * g.W + iw) * g.C + ci0 : 0;
      xv[i] = zero_unless(*(const bf16x8*)(x + o), ok);
    }
  };
  // transposed fragment read (T10): lane 4q+p addresses row 8fq+q (+4), columns col0+4p..+3
  auto frag = [&](const bf16_raw* sm, int col0, int ROWS) -> bf16x8 {
    const int cpr = ROWS / 8;
    const int col = col0 + 4 * tp;
    const int k1 = 8 * fq + tq, k2 = k1 + 4;
    const bf16_raw* p1 = sm + k1 * ROWS + 8 * ((col >> 3) ^ rc_swz(k1, cpr)) + (col & 7);
    const bf16_raw* p2 = sm + k2 * ROWS + 8 * ((col >> 3) ^ rc_swz(k2, cpr)) + (col & 7);
    bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p1));
    bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p2));
    return (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  };

  const int cbeg = (bx * 4 + wave) * cpw;
  const int cend = min(nchunks, cbeg + cpw);
  if (cbeg < cend) load(cbeg);
  for (int c = cbeg; c < cend; ++c) {  // wave-uniform: EXEC stays full for the tr reads
#pragma unroll
    for (int i = 0; i < DCH; ++i) {
      const int px = (lane + 64 * i) / (CO / 8);
      *(bf16x8*)(sA + px * CO + 8 * (dc ^ rc_swz(px, CO / 8))) = dv[i];
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) cacc[j] += bf2f((uint16_t)dv[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int px = (lane + 64 * i) / (KB / 8);
      *(bf16x8*)(sB + px * KB + 8 * (xc ^ rc_swz(px, KB / 8))) = xv[i];
    }
    if (c + 1 < cend) load(c + 1);  // in flight behind this chunk's MFMAs
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    bf16x8 af[NFC], bfr[NFKW];
#pragma unroll
    for (int i = 0; i < NFC; ++i) af[i] = frag(sA, i * 16, CO);
#pragma unroll
    for (int j = 0; j < NFKW; ++j) bfr[j] = frag(sB, j * 16, KB);
#pragma unroll
    for (int i = 0; i < NFC; ++i)
#pragma unroll
      for (int j = 0; j < NFKW; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next chunk's writes
    __builtin_amdgcn_wave_barrier();
  }
  // ---- cross-wave reduction (the staging images are free after this barrier)
  phase_mark(dbg, 1);
  __syncthreads();
  f32x4* red4 = (f32x4*)cm_smem;  // [wave][NFR][64] lane-major: conflict-free 16-B accesses
#pragma unroll
  for (int i = 0; i < NFC; ++i)
#pragma unroll
    for (int j = 0; j < NFKW; ++j) red4[(wave * NFR + i * NFKW + j) * 64 + lane] = acc[i][j];
  float* bsum = (float*)(red4 + 4 * NFR * 64);  // [4][CO] per-wave bias partials
  if (do_bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      for (int off = CO / 8; off < 64; off <<= 1) cacc[j] += __shfl_xor(cacc[j], off, 64);
    if (lane < CO / 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) bsum[wave * CO + lane * 8 + j] = cacc[j];
    }
  }
  __syncthreads();
  // sum the 4 waves' copies, restage row-major [CO][KB] behind them
  float* rowm = (float*)(bsum + 4 * CO);
  for (int e = threadIdx.x; e < NFR * 64; e += 256) {
    const int f = e >> 6, l = e & 63;
    f32x4 v = red4[f * 64 + l];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const f32x4 u = red4[(w * NFR + f) * 64 + l];
      v[0] += u[0]; v[1] += u[1]; v[2] += u[2]; v[3] += u[3];
    }
    const int i = f / NFKW, j = f - i * NFKW;
#pragma unroll
    for (int r = 0; r < 4; ++r) rowm[(i * 16 + (l >> 4) * 4 + r) * KB + j * 16 + (l & 15)] = v[r];
  }
  __syncthreads();
  phase_mark(dbg, 2);
  // deterministic mode: the pixel-chunk groups (bx) of every column block add in workgroup order
  const bool det = det_on();
  const unsigned dmy = (unsigned)(by * nbx + bx);
  if (det) det_turn_begin(DET_WGRAD, dmy);
  for (int e = threadIdx.x; e < CO * KB; e += 256) {
    const int co = e / KB, col = e - co * KB;
    const float v = rowm[e];
    if (kb0 + col < K && v != 0.f) atomicAdd(dw + (long)co * K + kb0 + col, v);
  }
  if (do_bias)
    for (int e = threadIdx.x; e < CO; e += 256) {
      const float v = bsum[e] + bsum[CO + e] + bsum[2 * CO + e] + bsum[3 * CO + e];
      if (v != 0.f) atomicAdd(dbias + e, v);
    }
  if (det) det_turn_end(DET_WGRAD, dmy, (unsigned)(nbx * nby));
  if (dbg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    phase_mark(dbg, 3);
  }
}

template <int NFC, int NFKW>
__global__ __launch_bounds__(256) void conv_wgrad_mfma_k(WgradArgs A) {
  conv_wgrad_body<NFC, NFKW>(A, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y);
}

// Horizontal fusion of one conv layer's backward: the input-gradient workgroups (first nA) and
// the weight-gradient workgroups (the rest, nBx x nBy) share ONE launch.  The two GEMMs are
// independent and each alone leaves most CUs idle at small batch; a second stream would run them
// concurrently too, but a cross-queue dependency costs ~10 us per replayed graph, a launch ~1.5.
//
// os.kind >= 0: os.nblk more workgroups run a fused optimizer's update of an arena slice whose
// gradients are final (optim_slice.h) — first in the grid (opt_first) or after the conv part.
// (OPT: only the instantiation that takes a slice contains the call — the out-of-line optimizer body
// needs a scratch stack, which the plain pair launches must not pay for)
template <int NF, int KS, int K0, int NFC, bool OPT = false>
__global__ __launch_bounds__(256, 2) void conv_bwd_pair_k(DgradArgs A, WgradArgs B, int nA, int nBx,
                                                          OptSlice os, int opt_first) {
  int bid = blockIdx.x;
  if constexpr (OPT) {
    if (opt_first) {
      if (bid < os.nblk) {
        opt_slice_run(os, bid);
        return;
      }
      bid -= os.nblk;
    } else if (bid >= (int)gridDim.x - os.nblk) {
      opt_slice_run(os, bid - ((int)gridDim.x - os.nblk));
      return;
    }
  }
  if (bid < nA) {
    conv_dgrad_body<NF, KS, K0, 2>(A, bid, nA);
  } else {
    const int j = bid - nA;
    conv_wgrad_body<NFC, 2>(B, j % nBx, j / nBx, nBx, ((int)gridDim.x - (OPT ? os.nblk : 0) - nA) / nBx);
  }
}

// The same horizontal fusion for layers whose input gradient takes the implicit GEMM (stride 2, or
// KH*KW*CO > 512: ResNet stage-3 3x3x64 and the strided / projection convs): the first nA
// workgroups are the dgrad GEMM's tiles (mfma_gemm_body, one K split), the rest the direct MFMA
// weight gradient.  Each part alone leaves most CUs idle at these sizes.
template <int BM, int NFC, class EP = EpiDActBF16>
__global__ __launch_bounds__(256) void conv_bwd_pair_gemm_k(ConvDgradALoader al, ConvWeightTLoader bl, EP ep,
                                                           int M, int N, int K, int kps, int nA, WgradArgs B,
                                                           int nBx) {
  if ((int)blockIdx.x < nA) {
    mfma_gemm_body<BM, BM, 2, true, false>(al, bl, ep, M, N, K, kps, nullptr, blockIdx.x, nA, 0, 1);
  } else {
    const int j = blockIdx.x - nA;
    conv_wgrad_body<NFC, 2>(B, j % nBx, j / nBx, nBx, ((int)gridDim.x - nA) / nBx);
  }
}

// supported K-step counts (K is zero-padded up to one of them)
int cm_ks(int ks) { return ks <= 2 ? 2 : ks <= 4 ? 4 : ks <= 8 ? 8 : ks <= 9 ? 9 : 16; }
// + a 5-step variant (K = 129..160: the 3x3, 16-channel convs of ResNet stage 1, K = 144) for the
// plain forward, the plain dgrad and the pair, which would otherwise pad K to 256 and spend 3/8 of
// their gathers and MFMAs on zeros; the pooled / fused-input variants keep cm_ks
int cm_ks5(int ks) { return ks == 5 && !hopsx_disabled("ks5") ? 5 : cm_ks(ks); }

int cm_grid(long ngroups, int un = CM_UN) {
  long blocks = (ngroups + CM_WAVES * un - 1) / (CM_WAVES * un);
  static const long cap = hopsx_env_int("HOPSX_CM_MAXWG", 1024);  // A/B knob: workgroups of the direct convs
  if (blocks > cap) blocks = cap;
  return (int)(blocks < 1 ? 1 : blocks);
}

}  // namespace

// K = KH*KW*C <= 512, C % 8 == 0, CO in {16, 32, 64, 128}
bool hopsx_conv_fwd_mfma_ok(const int* geom) {
  const int C = geom[3], CO = geom[6], K = geom[7] * geom[8] * C;
  return C % 8 == 0 && K <= 512 && (CO == 16 || CO == 32 || CO == 64 || CO == 128) &&
         !hopsx_disabled("conv_mfma");
}

// conv (act none / relu) -> pk x pk stride-pk max-pool (+ dropout p) in one launch (POOL epilogue):
// needs the plain MFMA forward; pk = 2 (any output size >= 2, floor windows) or 4 (output >= 4)
bool hopsx_conv_fwd_pool_ok(const int* geom, int act, int pk) {
  return hopsx_conv_fwd_mfma_ok(geom) && (pk == 2 || (pk == 4 && !hopsx_disabled("conv_pool4"))) && geom[4] >= pk &&
         geom[5] >= pk && (act == ACT_NONE || act == ACT_RELU) && !hopsx_disabled("conv_pool");
}

// stride 1 only; K = KH*KW*CO <= 512, CO % 8 == 0, C in {16, 32, 64, 128}
bool hopsx_conv_dgrad_mfma_ok(const int* geom) {
  const int C = geom[3], CO = geom[6], K = geom[7] * geom[8] * CO;
  const long nx = (long)geom[0] * geom[1] * geom[2] * C, ny = (long)geom[0] * geom[4] * geom[5] * CO;
  return geom[9] == 1 && geom[10] == 1 && CO % 8 == 0 && K <= 512 && (C == 16 || C == 32 || C == 64 || C == 128) &&
         nx < (1L << 31) && ny < (1L << 31) &&  // 32-bit gather offsets
         !hopsx_disabled("conv_mfma");
}

extern "C" int hopsx_conv2d_fwd_mfma(const void* x, const void* w, const int* geom, void* out, const float* bias,
                                     int act, hipStream_t st) {
  return hopsx_conv2d_fwd_mfma_ex(x, w, geom, out, bias, act, nullptr, st);
}

// bnacc != null: also accumulate the BatchNorm statistics of the output (conv_fwd_mfma_k BNS)
extern "C" int hopsx_conv2d_fwd_mfma_ex(const void* x, const void* w, const int* geom, void* out, const float* bias,
                                        int act, float* bnacc, hipStream_t st) {
  ConvGeom g;
  g.B = geom[0]; g.H = geom[1]; g.W = geom[2]; g.C = geom[3]; g.OH = geom[4]; g.OW = geom[5]; g.CO = geom[6];
  g.KH = geom[7]; g.KW = geom[8]; g.sh = geom[9]; g.sw = geom[10]; g.ph = geom[11]; g.pw = geom[12];
  g.dh = geom[13]; g.dw = geom[14];
  g.init_div();
  const int K = g.KH * g.KW * g.C;
  const int KS = cm_ks5((K + 31) / 32);
  const long M = (long)g.B * g.OH * g.OW;
  const int grid = cm_grid((M + 15) / 16);
  const size_t shm = (size_t)(g.CO * cm_rs(KS * 4) * 8 + CM_WAVES * 16 * g.CO) * sizeof(bf16_raw);
#define HOPSX_CMF(NF, KSV)                                                                                     \
  if (bnacc)                                                                                                   \
    hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV, false, CM_UN, true>), dim3(grid), dim3(256), shm, st,          \
                       (const bf16_raw*)x, (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K, PoolEpi{}, bnacc); \
  else                                                                                                         \
    hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV>), dim3(grid), dim3(256), shm, st, (const bf16_raw*)x,          \
                       (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K)
#define HOPSX_CMF_NF(NF)          \
  switch (KS) {                   \
    case 2: HOPSX_CMF(NF, 2); break;  \
    case 4: HOPSX_CMF(NF, 4); break;  \
    case 5: HOPSX_CMF(NF, 5); break;  \
    case 8: HOPSX_CMF(NF, 8); break;  \
    case 9: HOPSX_CMF(NF, 9); break;  \
    default: HOPSX_CMF(NF, 16); break; \
  }
  switch (g.CO / 16) {
    case 1: HOPSX_CMF_NF(1); break;
    case 2: HOPSX_CMF_NF(2); break;
    case 4: HOPSX_CMF_NF(4); break;
    case 8: HOPSX_CMF_NF(8); break;
    default: return -2;
  }
#undef HOPSX_CMF_NF
#undef HOPSX_CMF
  return (int)hipGetLastError();
}

// conv_fwd_mfma_k IBN: z -> a = act(bn(z)) (stored for the backward) -> conv -> out, with out's BN statistics
// into bnacc; the input BN's statistics come from inacc (re-zeroed here; != bnacc).  -2: not this path
// (stride / dilation != 1, the shape has no MFMA forward, act other than none / relu).
extern "C" int hopsx_conv2d_fwd_mfma_inbn(const void* z, void* a, const void* w, const int* geom, void* out,
                                          float* bnacc, float* inacc, const float* gamma, const float* beta,
                                          float* mean_out, float* rstd_out, float* rmean, float* rvar, float momentum,
                                          float eps, int act, hipStream_t st) {
  if (!hopsx_conv_fwd_mfma_ok(geom) || hopsx_disabled("bn_fold") || !bnacc || !inacc || bnacc == inacc || !a ||
      !mean_out || !rstd_out || (act != ACT_NONE && act != ACT_RELU))
    return -2;
  ConvGeom g;
  g.B = geom[0]; g.H = geom[1]; g.W = geom[2]; g.C = geom[3]; g.OH = geom[4]; g.OW = geom[5]; g.CO = geom[6];
  g.KH = geom[7]; g.KW = geom[8]; g.sh = geom[9]; g.sw = geom[10]; g.ph = geom[11]; g.pw = geom[12];
  g.dh = geom[13]; g.dw = geom[14];
  g.init_div();
  if (g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1 || g.OH < 1 || g.OW < 1) return -2;
  if (32 % g.C != 0) return -2;  // C in {8, 16, 32}: a lane's channels are the same at every tap (InBn)
  if (((uintptr_t)z | (uintptr_t)a | (uintptr_t)w | (uintptr_t)out) % 16 != 0) return -2;
  const long nx = (long)g.B * g.H * g.W * g.C;
  if (nx >= (1L << 31) || (long)g.B * g.H * g.W >= (1L << 31)) return -2;
  const int K = g.KH * g.KW * g.C;
  const int KS = cm_ks5((K + 31) / 32);
  const long M = (long)g.B * g.OH * g.OW;
  const int grid = cm_grid((M + 15) / 16);
  const size_t shm = (size_t)(g.CO * cm_rs(KS * 4) * 8 + CM_WAVES * 16 * g.CO) * sizeof(bf16_raw) + 2 * g.C * sizeof(float);
  const InBn ib{inacc, gamma, beta, mean_out, rstd_out, rmean, rvar, momentum, eps, (bf16_raw*)a,
                (int)(g.B * g.H * g.W), act};
#define HOPSX_CMI(NF, KSV)                                                                                       \
  hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV, false, CM_UN, true, 0, 2, true>), dim3(grid), dim3(256), shm, st, \
                     (const bf16_raw*)z, (const bf16_raw*)w, nullptr, (bf16_raw*)out, g, 0, K, PoolEpi{}, bnacc,   \
                     In0{}, ib)
#define HOPSX_CMI_NF(NF)          \
  switch (KS) {                   \
    case 2: HOPSX_CMI(NF, 2); break;  \
    case 4: HOPSX_CMI(NF, 4); break;  \
    case 5: HOPSX_CMI(NF, 5); break;  \
    case 8: HOPSX_CMI(NF, 8); break;  \
    case 9: HOPSX_CMI(NF, 9); break;  \
    default: HOPSX_CMI(NF, 16); break; \
  }
  switch (g.CO / 16) {
    case 1: HOPSX_CMI_NF(1); break;
    case 2: HOPSX_CMI_NF(2); break;
    case 4: HOPSX_CMI_NF(4); break;
    default: return -2;
  }
#undef HOPSX_CMI_NF
#undef HOPSX_CMI
  return (int)hipGetLastError();
}

static ConvGeom cm_geom(const int* geom) {
  ConvGeom g;
  g.B = geom[0]; g.H = geom[1]; g.W = geom[2]; g.C = geom[3]; g.OH = geom[4]; g.OW = geom[5]; g.CO = geom[6];
  g.KH = geom[7]; g.KW = geom[8]; g.sh = geom[9]; g.sw = geom[10]; g.ph = geom[11]; g.pw = geom[12];
  g.dh = geom[13]; g.dw = geom[14];
  g.init_div();
  return g;
}

// the dgrad of this conv (geom) can carry the wgrad of the input layer feeding it (geom0)
bool hopsx_conv_dgrad_fused_wgrad_ok(const int* geom, const int* geom0) {
  const int K0 = geom0[7] * geom0[8] * geom0[3];
  return hopsx_conv_dgrad_mfma_ok(geom) && geom[3] <= 64 && geom0[3] == 1 && (K0 == 4 || K0 == 9) &&
         geom0[0] == geom[0] && geom0[4] == geom[1] && geom0[5] == geom[2] && geom0[6] == geom[3] &&
         geom[7] * geom[8] * geom[6] <= 256 && !hopsx_disabled("fused_wgrad0");
}

extern "C" int hopsx_conv2d_dgrad_mfma(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                       int act_prev, float* colsum, const void* y, int yact, hipStream_t st) {
  return hopsx_conv2d_dgrad_mfma_ex(dy, w, geom, dx, yprev, act_prev, colsum, y, yact, nullptr, nullptr, 0.f, 0.f,
                                    nullptr, st);
}

static int dgrad_mfma_impl(const void* dy, const void* w, const int* geom, void* dx, const void* yprev, int act_prev,
                           float* colsum, const void* y, int yact, const int* geom0, const void* x0, float xscale,
                           float xshift, float* dw0, const void* addend, const void* bnz, const float* bnmean,
                           const float* bnrstd, float* bnacc, hipStream_t st);

extern "C" int hopsx_conv2d_dgrad_mfma_ex(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                          int act_prev, float* colsum, const void* y, int yact, const int* geom0,
                                          const void* x0, float xscale, float xshift, float* dw0, hipStream_t st) {
  return dgrad_mfma_impl(dy, w, geom, dx, yprev, act_prev, colsum, y, yact, geom0, x0, xscale, xshift, dw0, nullptr,
                         nullptr, nullptr, nullptr, nullptr, st);
}

// the direct MFMA dgrad with the input BN's backward column sums in its epilogue (DgradArgs bnacc) and an
// optional shortcut gradient added before the act'(yprev) mask; -2: not this kernel's shape (nothing launched)
extern "C" int hopsx_conv2d_dgrad_mfma_bn(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                          int act_prev, const void* addend, const void* bnz, const float* bnmean,
                                          const float* bnrstd, float* bnacc, hipStream_t st) {
  if (!hopsx_conv_dgrad_mfma_ok(geom) || !bnacc || !bnz || !bnmean || !bnrstd ||
      ((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)yprev | (uintptr_t)addend | (uintptr_t)bnz) % 16)
    return -2;
  return dgrad_mfma_impl(dy, w, geom, dx, yprev, act_prev, nullptr, nullptr, 0, nullptr, nullptr, 0.f, 0.f, nullptr,
                         addend, bnz, bnmean, bnrstd, bnacc, st);
}

static int dgrad_mfma_impl(const void* dy, const void* w, const int* geom, void* dx, const void* yprev, int act_prev,
                           float* colsum, const void* y, int yact, const int* geom0, const void* x0, float xscale,
                           float xshift, float* dw0, const void* addend, const void* bnz, const float* bnmean,
                           const float* bnrstd, float* bnacc, hipStream_t st) {
  const bool fused = geom0 != nullptr;
  if (fused && (!hopsx_conv_dgrad_fused_wgrad_ok(geom, geom0) || !yprev || !colsum || !dw0 || !x0)) return -4;
  ConvGeom g0 = fused ? cm_geom(geom0) : ConvGeom{};
  const int K0 = fused ? geom0[7] * geom0[8] : 0;
  ConvGeom g = cm_geom(geom);
  const int K = g.KH * g.KW * g.CO;
  const int KS = fused ? cm_ks((K + 31) / 32) : cm_ks5((K + 31) / 32);
  const long M = (long)g.B * g.H * g.W;
  // two 16-pixel groups per wave per trip (HOPSX_DGRAD_UN=1: one)
  static const int un_env = getenv("HOPSX_DGRAD_UN") ? atoi(getenv("HOPSX_DGRAD_UN")) : 0;
  const long ngroups = (M + 15) / 16;
  const int un = un_env == 1 ? 1 : 2;  // UN=1 measured slower at the MNIST shape (more colsum atomics)
  long blocks = (ngroups + CM_WAVES * un - 1) / (CM_WAVES * un);
  if (blocks > 1024) blocks = 1024;
  if (colsum && blocks > 512) blocks = 512;  // one colsum atomic per channel per workgroup
  const size_t shm = (size_t)(g.C * cm_rs(KS * 4) * 8 + CM_WAVES * 16 * g.C) * sizeof(bf16_raw) +
                     (size_t)CM_RSLOTS * g.C * (1 + K0 + (bnacc ? 1 : 0)) * sizeof(float) + (size_t)KS * 4 * 16;
  if (shm > 160u * 1024u) return -2;  // gfx950 LDS per workgroup (C = 128 at K = 512 with the BN sums: 161 KB)
  const int wvec = (uintptr_t)w % 16 == 0;
  static const int dbg = getenv("HOPSX_PHASE_DBG") ? 1 : 0;
  const DgradArgs DA{(const bf16_raw*)dy, (const bf16_raw*)w, (bf16_raw*)dx, (const bf16_raw*)yprev, act_prev, colsum,
                     (const bf16_raw*)y, yact, g, K, wvec, x0, xscale, xshift, g0, dw0, dbg, (const bf16_raw*)addend,
                     (int)hopsx_env_int("HOPSX_DGRAD_XCD", 0), (const bf16_raw*)bnz, bnmean, bnrstd, bnacc};
#define HOPSX_CMD(NF, KSV, K0V)                                                                                \
  if (un == 1) hipLaunchKernelGGL((conv_dgrad_mfma_k<NF, KSV, K0V, 1>), dim3(blocks), dim3(256), shm, st, DA); \
  else hipLaunchKernelGGL((conv_dgrad_mfma_k<NF, KSV, K0V, 2>), dim3(blocks), dim3(256), shm, st, DA)
#define HOPSX_CMD_NF(NF)          \
  switch (KS) {                   \
    case 2: HOPSX_CMD(NF, 2, 0); break;  \
    case 4: HOPSX_CMD(NF, 4, 0); break;  \
    case 5: HOPSX_CMD(NF, 5, 0); break;  \
    case 8: HOPSX_CMD(NF, 8, 0); break;  \
    case 9: HOPSX_CMD(NF, 9, 0); break;  \
    default: HOPSX_CMD(NF, 16, 0); break; \
  }
#define HOPSX_CMD_FUSED(NF, K0V)  \
  switch (KS) {                   \
    case 2: HOPSX_CMD(NF, 2, K0V); break;  \
    case 4: HOPSX_CMD(NF, 4, K0V); break;  \
    default: HOPSX_CMD(NF, 8, K0V); break;  \
  }
  if (fused) {  // K <= 256: KS in {2, 4, 8}
    if (g.C != 16 && g.C != 32 && g.C != 64) return -2;
    if (K0 == 4) {
      if (g.C == 16) { HOPSX_CMD_FUSED(1, 4); } else if (g.C == 32) { HOPSX_CMD_FUSED(2, 4); } else { HOPSX_CMD_FUSED(4, 4); }
    } else {
      if (g.C == 16) { HOPSX_CMD_FUSED(1, 9); } else if (g.C == 32) { HOPSX_CMD_FUSED(2, 9); } else { HOPSX_CMD_FUSED(4, 9); }
    }
    return (int)hipGetLastError();
  }
  switch (g.C / 16) {
    case 1: HOPSX_CMD_NF(1); break;
    case 2: HOPSX_CMD_NF(2); break;
    case 4: HOPSX_CMD_NF(4); break;
    case 8: HOPSX_CMD_NF(8); break;
    default: return -2;
  }
#undef HOPSX_CMD_FUSED
#undef HOPSX_CMD_NF
#undef HOPSX_CMD
  return (int)hipGetLastError();
}

// short-conv weight gradient on MFMA: C % 8 == 0, CO in {16, 32, 64}, K = KH*KW*C <= 256
bool hopsx_conv_wgrad_mfma_ok(const int* geom) {
  const int C = geom[3], CO = geom[6], K = geom[7] * geom[8] * C;
  static const long maxk = hopsx_env_int("HOPSX_WGRAD_MFMA_MAXK", 640);  // 640: ResNet-20 +2 %, ResNet-56 +3.4 %, R50 flat
  return C % 8 == 0 && K <= maxk && (CO == 16 || CO == 32 || CO == 64) && !hopsx_disabled("wgrad_mfma");
}

extern "C" int hopsx_conv2d_wgrad_mfma(const void* dy, const void* x, const int* geom, float* dw, float* dbias,
                                       const void* y, int yact, hipStream_t st) {
  ConvGeom g = cm_geom(geom);
  const int K = g.KH * g.KW * g.C;
  const long M = (long)g.B * g.OH * g.OW;
  const long nchunks = (M + WG_PX - 1) / WG_PX;
  static const int dbg = getenv("HOPSX_PHASE_DBG") ? 1 : 0;
  static const int nfkw_env = getenv("HOPSX_WGRAD_NFKW") ? atoi(getenv("HOPSX_WGRAD_NFKW")) : 2;
  const int NFKW = nfkw_env == 4 ? 4 : 2, KB = NFKW * 16;  // 32-column blocks: 8 KB of atomics per workgroup
  const int colblk = (K + KB - 1) / KB;
  // ~384 workgroups in all: each wave walks a run of cpw chunks with one chunk of prefetch
  static const int cpw_env = getenv("HOPSX_WGRAD_CPW") ? atoi(getenv("HOPSX_WGRAD_CPW")) : 0;
  const long want_groups = std::max(1L, 384L / colblk);
  int cpw = cpw_env > 0 ? cpw_env : (int)std::max(1L, (nchunks + 4 * want_groups - 1) / (4 * want_groups));
  const long groups = (nchunks + 4L * cpw - 1) / (4L * cpw);
  dim3 grid((unsigned)groups, (unsigned)colblk);
  const size_t stage = (size_t)4 * WG_PX * (g.CO + KB) * sizeof(bf16_raw);
  const int NFR = (g.CO / 16) * NFKW;
  const size_t redb = ((size_t)4 * NFR * 64 * 4 + 4 * g.CO + (size_t)g.CO * KB) * sizeof(float);
  const size_t shm = std::max(stage, redb);
  const WgradArgs WA{(const bf16_raw*)dy, (const bf16_raw*)x, (const bf16_raw*)y, yact, dw, dbias, g, K, cpw, dbg};
#define HOPSX_CWM(NFC)                                                                                     \
  if (NFKW == 4) hipLaunchKernelGGL((conv_wgrad_mfma_k<NFC, 4>), grid, dim3(256), shm, st, WA); \
  else hipLaunchKernelGGL((conv_wgrad_mfma_k<NFC, 2>), grid, dim3(256), shm, st, WA)
  switch (g.CO) {
    case 16: HOPSX_CWM(1); break;
    case 32: HOPSX_CWM(2); break;
    case 64: HOPSX_CWM(4); break;
    default: return -2;
  }
#undef HOPSX_CWM
  return (int)hipGetLastError();
}

extern "C" int hopsx_wgrad_debug_times(unsigned long long* host_out, int n) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wgrad_dbg), sizeof(unsigned long long) * (size_t)n, 0,
                                  hipMemcpyDeviceToHost);
}

// wgrad part of a paired launch: 32-column blocks, chunks per wave sized for ~`slots` workgroups
static void pair_wgrad_plan(const ConvGeom& g, long slots, int& cpw, long& nBx, int& colblk, size_t& shm) {
  const int Kw = g.KH * g.KW * g.C;
  const long nchunks = ((long)g.B * g.OH * g.OW + WG_PX - 1) / WG_PX;
  constexpr int KB = 32;
  colblk = (Kw + KB - 1) / KB;
  const long want_groups = std::max(1L, slots / colblk);
  cpw = (int)std::max(1L, (nchunks + 4 * want_groups - 1) / (4 * want_groups));
  nBx = (nchunks + 4L * cpw - 1) / (4L * cpw);
  const size_t stage = (size_t)4 * WG_PX * (g.CO + KB) * sizeof(bf16_raw);
  const size_t redb = ((size_t)4 * (g.CO / 16) * 2 * 64 * 4 + 4 * g.CO + (size_t)g.CO * KB) * sizeof(float);
  shm = std::max(stage, redb);
}

// The BN whose output is this conv's input (DgradArgs bnz / bnmean / bnrstd / bnacc); acc == null: none
struct BnPre {
  const void* z;
  const float* mean;
  const float* rstd;
  float* acc;
};

// dgrad on the implicit GEMM + wgrad on the direct MFMA kernel in one launch (conv_bwd_pair_gemm_k);
// bp.acc: the input BN's backward column sums in the dgrad epilogue (EpiDgradBnBF16; yprev = x)
static int conv_bwd_pair_gemm(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                              int act_prev, float* colsum, const void* y, int yact, const void* x, float* dw,
                              float* dbias, const void* addend, hipStream_t st, const BnPre& bp = BnPre{}) {
  if (hopsx_disabled("bwd_pair_gemm")) return -2;
  ConvGeom g = cm_geom(geom);
  if (g.C % 8 != 0 || g.CO % 8 != 0 || ((uintptr_t)dy | (uintptr_t)y | (uintptr_t)x | (uintptr_t)w) % 16 != 0)
    return -2;
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.CO;
  const GemmPlan p = plan_gemm(M, N, K, false);
  if (p.cfg == 0 || p.split != 1) return -2;  // 128x128 tiles: the GEMM fills the chip on its own
  const int BM = p.cfg == 1 ? 64 : 32;
  const long nA = (long)((M + BM - 1) / BM) * ((N + BM - 1) / BM);
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
  }
  int cpw, colblk;
  long nBx;
  size_t shm;
  pair_wgrad_plan(g, nA >= 2L * n_cu ? 384L : std::max(64L, 2L * n_cu - nA), cpw, nBx, colblk, shm);
  const long total = nA + nBx * colblk;
  if (shm > 65536 || total > (1L << 20)) return -2;
  static const int dbg = getenv("HOPSX_PHASE_DBG") ? 1 : 0;
  const WgradArgs WA{(const bf16_raw*)dy, (const bf16_raw*)x, (const bf16_raw*)y, yact, dw, dbias, g,
                     g.KH * g.KW * g.C, cpw, dbg};
  ConvDgradALoader al{(const bf16_raw*)dy, g, 1, (const bf16_raw*)y, yact};
  ConvWeightTLoader bl{(const bf16_raw*)w, g, 1};
  // addend: another consumer's gradient of x, added after the dgrad (no act' of a producing layer here)
  EpiDActBF16 e{(bf16_raw*)dx, N, (const bf16_raw*)yprev, N, act_prev, colsum, (const bf16_raw*)addend};
  const EpiDgradBnBF16 eb{(bf16_raw*)dx, N, (const bf16_raw*)yprev, act_prev, (const bf16_raw*)addend,
                          (const bf16_raw*)bp.z, bp.mean, bp.rstd, bp.acc};
#define HOPSX_PG(BMv, NFCv)                                                                                   \
  if (BM == BMv && g.CO / 16 == NFCv) {                                                                     \
    if (bp.acc)                                                                                             \
      hipLaunchKernelGGL((conv_bwd_pair_gemm_k<BMv, NFCv, EpiDgradBnBF16>), dim3((unsigned)total), dim3(256), shm, \
                         st, al, bl, eb, M, N, K, p.kps, (int)nA, WA, (int)nBx);                              \
    else                                                                                                    \
      hipLaunchKernelGGL((conv_bwd_pair_gemm_k<BMv, NFCv>), dim3((unsigned)total), dim3(256), shm, st, al, bl, e, \
                         M, N, K, p.kps, (int)nA, WA, (int)nBx);                                              \
    return (int)hipGetLastError();                                                                          \
  }
  HOPSX_PG(32, 1) HOPSX_PG(32, 2) HOPSX_PG(32, 4) HOPSX_PG(64, 1) HOPSX_PG(64, 2) HOPSX_PG(64, 4)
#undef HOPSX_PG
  return -2;
}

// One launch for a conv layer's whole backward: dgrad (optionally carrying the input layer's
// weight gradient, geom0 != null) + the layer's own weight gradient.  Same argument meaning as
// hopsx_conv2d_dgrad_mfma_ex and hopsx_conv2d_wgrad_mfma; returns -2 for shapes outside the
// instantiated set (the caller then issues the two launches).
static int conv2d_bwd_pair_impl(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                int act_prev, float* colsum, const void* y, int yact, const int* geom0, const void* x0,
                                float xscale, float xshift, float* dw0, const void* x, float* dw, float* dbias,
                                const void* addend, const OptSlice& os, int opt_first, hipStream_t st,
                                const BnPre& bp = BnPre{});

// the paired backward can also reduce the input BatchNorm's backward column sums (BnPre): either dgrad
// variant (direct MFMA or implicit GEMM), no fused input layer, no bias gradient
extern "C" int hopsx_conv2d_bwd_pair_bn_ok(const int* geom) {
  // (the implicit-GEMM dgrad variant may still refuse a shape at launch: -2, nothing launched)
  return hopsx_conv_wgrad_mfma_ok(geom) && geom[3] % 8 == 0 && !hopsx_disabled("bwd_pair") &&
                 !hopsx_disabled("bn_dgrad_sums") && hopsx_bn_prestats_ok(geom[3])
             ? 1
             : 0;
}

extern "C" int hopsx_conv2d_bwd_pair(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                     int act_prev, float* colsum, const void* y, int yact, const int* geom0,
                                     const void* x0, float xscale, float xshift, float* dw0, const void* x,
                                     float* dw, float* dbias, const void* addend, const void* bnz,
                                     const float* bnmean, const float* bnrstd, float* bnacc, hipStream_t st) {
  OptSlice none{};
  none.kind = -1;
  return conv2d_bwd_pair_impl(dy, w, geom, dx, yprev, act_prev, colsum, y, yact, geom0, x0, xscale, xshift, dw0, x, dw,
                              dbias, addend, none, 0, st, BnPre{bnz, bnmean, bnrstd, bnacc});
}

// The same launch + a fused optimizer's update of the arena slice [p, p + n) (its gradients final),
// as `nblk` extra workgroups (optim_slice.h).  f[0..7] = the optimizer's hyper-parameter vector.
// Returns -2 when the pair kernel does not take the shape (nothing launched: the caller runs the
// unfused backward and the whole optimizer).
extern "C" int hopsx_conv2d_bwd_pair_opt(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                         int act_prev, float* colsum, const void* y, int yact, const int* geom0,
                                         const void* x0, float xscale, float xshift, float* dw0, const void* x,
                                         float* dw, float* dbias, const void* addend, int kind, float* p, float* g,
                                         float* s1, float* s2, float* s3, void* shadow, long n, const float* f,
                                         const float* hp_dev, const float* step_dev, int nblk, int opt_first,
                                         hipStream_t st) {
  if (kind < 0 || kind > 6 || n <= 0 || n % 4 || nblk < 1 ||
      ((uintptr_t)p | (uintptr_t)g | (uintptr_t)s1 | (uintptr_t)s2 | (uintptr_t)s3) % 16 || (uintptr_t)shadow % 8)
    return -3;
  OptSlice os{};
  os.kind = kind;
  os.nblk = nblk;
  os.p = p;
  os.g = g;
  os.s1 = s1;
  os.s2 = s2;
  os.s3 = s3;
  os.shadow = (bf16_raw*)shadow;
  os.n4 = n / 4;
  os.h = OptHP{f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]};
  os.hp_dev = hp_dev;
  os.step_dev = step_dev;
  return conv2d_bwd_pair_impl(dy, w, geom, dx, yprev, act_prev, colsum, y, yact, geom0, x0, xscale, xshift, dw0, x, dw,
                              dbias, addend, os, opt_first, st);
}

static int conv2d_bwd_pair_impl(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                int act_prev, float* colsum, const void* y, int yact, const int* geom0, const void* x0,
                                float xscale, float xshift, float* dw0, const void* x, float* dw, float* dbias,
                                const void* addend, const OptSlice& os, int opt_first, hipStream_t st,
                                const BnPre& bp) {
  if (hopsx_disabled("bwd_pair") || !hopsx_conv_wgrad_mfma_ok(geom)) return -2;
  const bool fused = geom0 != nullptr;
  if (fused && addend) return -2;
  const bool bn = bp.acc != nullptr;
  if (bn && (fused || colsum || !dx || !bp.z || !bp.mean || !bp.rstd || !hopsx_conv2d_bwd_pair_bn_ok(geom) ||
             (uintptr_t)bp.z % 16 || os.kind >= 0))
    return -2;
  if ((uintptr_t)addend % 16 != 0) return -3;
  if (!hopsx_conv_dgrad_mfma_ok(geom)) {
    // the GEMM variant adds an addend in its epilogue after the dgrad; with an act' of the producing
    // layer (yprev) the sum would have to come first: call again without it and add afterwards
    // (bn: the BN epilogue adds first, then masks)
    if (addend && yprev && !bn) return -3;
    if (os.kind >= 0) return -2;
    return fused ? -2
                 : conv_bwd_pair_gemm(dy, w, geom, dx, yprev, act_prev, colsum, y, yact, x, dw, dbias, addend, st, bp);
  }
  if (fused && (!hopsx_conv_dgrad_fused_wgrad_ok(geom, geom0) || !yprev || !colsum || !dw0 || !x0)) return -4;
  if (((uintptr_t)dy | (uintptr_t)y | (uintptr_t)x | (uintptr_t)dx | (uintptr_t)yprev) % 16 != 0) return -2;
  ConvGeom g = cm_geom(geom);
  ConvGeom g0 = fused ? cm_geom(geom0) : ConvGeom{};
  const int K0 = fused ? geom0[7] * geom0[8] : 0;
  // ---- dgrad part
  const int Kd = g.KH * g.KW * g.CO;
  const int KS = cm_ks5((Kd + 31) / 32);
  const long Md = (long)g.B * g.H * g.W;
  long nA = ((Md + 15) / 16 + CM_WAVES * 2 - 1) / (CM_WAVES * 2);
  static const long pair_cap = hopsx_env_int("HOPSX_PAIR_DGRAD_MAXWG", 1024);  // A/B knob
  if (nA > pair_cap) nA = pair_cap;
  if (colsum && nA > 512) nA = 512;
  const size_t shmA = (size_t)(g.C * cm_rs(KS * 4) * 8 + CM_WAVES * 16 * g.C) * sizeof(bf16_raw) +
                      (size_t)CM_RSLOTS * g.C * (1 + K0 + (bn ? 1 : 0)) * sizeof(float) + (size_t)KS * 4 * 16;
  static const int dbg = getenv("HOPSX_PHASE_DBG") ? 1 : 0;
  const DgradArgs DA{(const bf16_raw*)dy, (const bf16_raw*)w, (bf16_raw*)dx, (const bf16_raw*)yprev, act_prev, colsum,
                     (const bf16_raw*)y, yact, g, Kd, (int)((uintptr_t)w % 16 == 0), x0, xscale, xshift, g0, dw0, dbg,
                     (const bf16_raw*)addend, (int)hopsx_env_int("HOPSX_DGRAD_XCD", 0), (const bf16_raw*)bp.z,
                     bp.mean, bp.rstd, bp.acc};
  // ---- wgrad part (32-column blocks)
  const int Kw = g.KH * g.KW * g.C;
  const long nchunks = ((long)g.B * g.OH * g.OW + WG_PX - 1) / WG_PX;
  constexpr int KB = 32;
  const int colblk = (Kw + KB - 1) / KB;
  // size the weight-gradient part so the whole launch is resident at once (2 workgroups per CU at
  // <= 256 VGPRs): otherwise its last workgroups only start when the first ones retire and the
  // launch's tail is a second wave of them (measured: 340 of them started up to 8.4 us late)
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
  }
  // When the dgrad part alone already fills every slot (nA >= 2 per CU, e.g. ResNet-20 stage 1:
  // 1024 dgrad workgroups) the launch runs in several waves anyway: size the weight-gradient part
  // by work (~384 workgroups) — squeezing it into the leftover slots made 12 x 5 workgroups walk
  // 2048 chunks (86 us instead of 27 us per launch).
  static const int cpw_env = getenv("HOPSX_PAIR_CPW") ? atoi(getenv("HOPSX_PAIR_CPW")) : 0;
  const long slots = nA >= 2L * n_cu ? 384L : std::max(64L, 2L * n_cu - nA);
  const long want_groups = std::max(1L, slots / colblk);
  const int cpw = cpw_env > 0 ? cpw_env : (int)std::max(1L, (nchunks + 4 * want_groups - 1) / (4 * want_groups));
  const long nBx = (nchunks + 4L * cpw - 1) / (4L * cpw);
  const size_t stage = (size_t)4 * WG_PX * (g.CO + KB) * sizeof(bf16_raw);
  const size_t redb = ((size_t)4 * (g.CO / 16) * 2 * 64 * 4 + 4 * g.CO + (size_t)g.CO * KB) * sizeof(float);
  const size_t shm = std::max(shmA, std::max(stage, redb));
  const WgradArgs WA{(const bf16_raw*)dy, (const bf16_raw*)x, (const bf16_raw*)y, yact, dw, dbias, g, Kw, cpw, dbg};
  const long total = nA + nBx * colblk + (os.kind >= 0 ? os.nblk : 0);
  if (shm > 65536 || total > (1L << 20)) return -2;
  const int NF = g.C / 16, NFC = g.CO / 16;
#define HOPSX_PAIR(NFv, KSv, K0v, NFCv)                                                                      \
  if (NF == NFv && KS == KSv && K0 == K0v && NFC == NFCv) {                                                  \
    if (os.kind >= 0) {                                                                                      \
      if (NFv != 2 || KSv != 8 || K0v != 4 || NFCv != 4) return -2; /* slice only on the flagship shape */  \
      hipLaunchKernelGGL((conv_bwd_pair_k<2, 8, 4, 4, true>), dim3((unsigned)total), dim3(256), shm, st, DA, WA, \
                         (int)nA, (int)nBx, os, opt_first);                                                  \
    } else {                                                                                                 \
      hipLaunchKernelGGL((conv_bwd_pair_k<NFv, KSv, K0v, NFCv>), dim3((unsigned)total), dim3(256), shm, st, DA, \
                         WA, (int)nA, (int)nBx, os, opt_first);                                              \
    }                                                                                                        \
    return (int)hipGetLastError();                                                                           \
  }
#define HOPSX_PAIR_K0(NFv, KSv, NFCv) HOPSX_PAIR(NFv, KSv, 0, NFCv) HOPSX_PAIR(NFv, KSv, 4, NFCv)
#define HOPSX_PAIR_NFC(NFv, KSv) HOPSX_PAIR_K0(NFv, KSv, 1) HOPSX_PAIR_K0(NFv, KSv, 2) HOPSX_PAIR_K0(NFv, KSv, 4)
  HOPSX_PAIR_NFC(1, 4) HOPSX_PAIR_NFC(1, 8) HOPSX_PAIR_NFC(2, 4) HOPSX_PAIR_NFC(2, 8) HOPSX_PAIR_NFC(4, 4)
  HOPSX_PAIR_NFC(4, 8) HOPSX_PAIR_K0(2, 9, 2) HOPSX_PAIR(1, 5, 0, 1)
#undef HOPSX_PAIR_NFC
#undef HOPSX_PAIR_K0
#undef HOPSX_PAIR
  return -2;
}

extern "C" int hopsx_conv2d_fwd_pool(const void* x, const void* w, const int* geom, void* out, void* am,
                                     const float* bias, int act, float p, const unsigned long long* rng, unsigned salt,
                                     int pk, hipStream_t st) {
  if (!hopsx_conv_fwd_pool_ok(geom, act, pk)) return -2;
  ConvGeom g;
  g.B = geom[0]; g.H = geom[1]; g.W = geom[2]; g.C = geom[3]; g.OH = geom[4]; g.OW = geom[5]; g.CO = geom[6];
  g.KH = geom[7]; g.KW = geom[8]; g.sh = geom[9]; g.sw = geom[10]; g.ph = geom[11]; g.pw = geom[12];
  g.dh = geom[13]; g.dw = geom[14];
  g.init_div();
  const int K = g.KH * g.KW * g.C;
  const int KS = cm_ks((K + 31) / 32);
  const long rows = (long)g.B * (g.OH / pk) * (g.OW / pk) * pk * pk;
  // one 16-row group per wave per trip when two would leave CUs idle (HOPSX_CMP_UN=1/2 forces)
  static const int un_env = getenv("HOPSX_CMP_UN") ? atoi(getenv("HOPSX_CMP_UN")) : 0;
  const long ngr = (rows + 15) / 16;
  const int un = un_env == 1 || un_env == 2 ? un_env : (ngr < 2L * CM_WAVES * CM_UN * 256 ? 1 : 2);
  const int grid = cm_grid(ngr, un);
  const size_t shm = (size_t)(g.CO * cm_rs(KS * 4) * 8 + CM_WAVES * 16 * g.CO) * sizeof(bf16_raw);
  static const int dbg = getenv("HOPSX_PHASE_DBG") ? 1 : 0;
  const PoolEpi pe{(unsigned char*)am, rng, salt, p, dbg};
#define HOPSX_CMP(NF, KSV)                                                                                      \
  if (pk == 4 && un == 1)                                                                                       \
    hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV, true, 1, false, 0, 4>), dim3(grid), dim3(256), shm, st,         \
                       (const bf16_raw*)x, (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K, pe);            \
  else if (pk == 4)                                                                                             \
    hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV, true, 2, false, 0, 4>), dim3(grid), dim3(256), shm, st,         \
                       (const bf16_raw*)x, (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K, pe);            \
  else if (un == 1)                                                                                             \
    hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV, true, 1>), dim3(grid), dim3(256), shm, st, (const bf16_raw*)x,  \
                       (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K, pe);                                \
  else                                                                                                          \
    hipLaunchKernelGGL((conv_fwd_mfma_k<NF, KSV, true, 2>), dim3(grid), dim3(256), shm, st, (const bf16_raw*)x,  \
                       (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K, pe)
#define HOPSX_CMP_NF(NF)              \
  switch (KS) {                       \
    case 2: HOPSX_CMP(NF, 2); break;  \
    case 4: HOPSX_CMP(NF, 4); break;  \
    case 8: HOPSX_CMP(NF, 8); break;  \
    case 9: HOPSX_CMP(NF, 9); break;  \
    default: HOPSX_CMP(NF, 16); break; \
  }
  switch (g.CO / 16) {
    case 1: HOPSX_CMP_NF(1); break;
    case 2: HOPSX_CMP_NF(2); break;
    case 4: HOPSX_CMP_NF(4); break;
    case 8: HOPSX_CMP_NF(8); break;
    default: return -2;
  }
#undef HOPSX_CMP_NF
#undef HOPSX_CMP
  return (int)hipGetLastError();
}

// input layer (geom0: Cin 1, stride 1, dilation 1, a 2x2 or 3x3 kernel) -> this conv + act + 2x2 max-pool
// (+ dropout) in ONE launch (conv_fwd_mfma_k IN0); geom is this conv's geometry over the input
// layer's output (stride 1, dilation 1)
bool hopsx_conv_fwd_pool_in_ok(const int* geom0, const int* geom, int act) {
  return hopsx_conv_fwd_pool_ok(geom, act, 2) && geom[4] % 2 == 0 && geom[5] % 2 == 0 && geom0[3] == 1 && geom0[9] == 1 && geom0[10] == 1 && geom0[13] == 1 &&
         geom0[14] == 1 && geom0[7] == geom0[8] && (geom0[7] == 2 || geom0[7] == 3) && geom0[4] == geom[1] && geom0[5] == geom[2] &&
         geom0[6] == geom[3] && geom0[0] == geom[0] && geom[9] == 1 && geom[10] == 1 && geom[13] == 1 &&
         geom[14] == 1 && geom[6] == 64 && geom[3] % 8 == 0 && geom[3] <= 64 &&
         (cm_ks((geom[7] * geom[8] * geom[3] + 31) / 32) == 2 || cm_ks((geom[7] * geom[8] * geom[3] + 31) / 32) == 4 ||
          cm_ks((geom[7] * geom[8] * geom[3] + 31) / 32) == 9) &&
         !hopsx_disabled("conv_in_pool");
}

extern "C" int hopsx_conv2d_fwd_pool_in(const void* x0, float xscale, float xshift, const void* w0, const float* b0,
                                        int act0, const int* geom0, void* y1, const void* w, const int* geom,
                                        void* out, void* am, const float* bias, int act, float p,
                                        const unsigned long long* rng, unsigned salt, hipStream_t st) {
  if (!hopsx_conv_fwd_pool_in_ok(geom0, geom, act)) return -2;
  if (((uintptr_t)w | (uintptr_t)out | (uintptr_t)y1) % 16 != 0 || xscale == 0.f) return -3;
  ConvGeom g = cm_geom(geom);
  const int K = g.KH * g.KW * g.C;
  const int KS = cm_ks((K + 31) / 32);
  const long rows = (long)g.B * (g.OH / 2) * (g.OW / 2) * 4;
  // one 16-row group per wave per trip: the trip holds T0*T0 pixels per K-step in registers
  const long ngr = (rows + 15) / 16;
  const int grid = cm_grid(ngr, 1);
  const int taps = geom0[7] * geom0[8];
  const size_t shm = (size_t)(g.CO * cm_rs(KS * 4) * 8 + CM_WAVES * 16 * g.CO) * sizeof(bf16_raw) +
                     (size_t)(taps + 1) * g.C * sizeof(float);
  static const int dbg = getenv("HOPSX_PHASE_DBG") ? 1 : 0;
  const PoolEpi pe{(unsigned char*)am, rng, salt, p, dbg};
  const In0 i0{x0, xscale, xshift, (const bf16_raw*)w0, b0, (bf16_raw*)y1, geom0[1], geom0[2], geom0[7], geom0[8],
               geom0[11], geom0[12], act0};
#define HOPSX_CMPI(KSV, T0V)                                                                                      \
  hipLaunchKernelGGL((conv_fwd_mfma_k<4, KSV, true, 1, false, T0V>), dim3(grid), dim3(256), shm, st, nullptr,      \
                     (const bf16_raw*)w, bias, (bf16_raw*)out, g, act, K, pe, nullptr, i0)
  const int t0 = geom0[7];
  switch (KS * 4 + t0) {
    case 2 * 4 + 2: HOPSX_CMPI(2, 2); break;
    case 4 * 4 + 2: HOPSX_CMPI(4, 2); break;
    case 9 * 4 + 2: HOPSX_CMPI(9, 2); break;
    case 2 * 4 + 3: HOPSX_CMPI(2, 3); break;
    case 4 * 4 + 3: HOPSX_CMPI(4, 3); break;
    case 9 * 4 + 3: HOPSX_CMPI(9, 3); break;
    default: return -2;
  }
#undef HOPSX_CMPI
  return (int)hipGetLastError();
}
