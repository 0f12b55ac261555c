// hopsx "gg" GEMM engine: LDS-DMA (global_load_lds) staged, 3-stage pipelined MFMA GEMM for the big
// conv GEMMs of gfx950 (cdna_hip_programming.md §5 "Pipelining across barriers", "glds vs register
// staging", rule 21; MI355X_MICROARCH.md §LDS).
//
// Why a second engine next to gemm_core.h: the register-staged 4-wave core tops out near
// 100-300 TFLOP/s on the ResNet-50 shapes (profiles/r3s6_wgrad_layers_b64.jsonl) because every
// k-step waits for its own global loads.  Here:
//  * 512 threads (8 waves as 2 (M) x 4 (N)), tiles 256x128 / 128x256 / 128x128, BK = 64,
//    v_mfma_f32_16x16x32_bf16 with fp32 accumulators;
//  * both operand tiles go global -> LDS by `global_load_lds_dwordx4` (16 B per lane, no VGPR
//    staging) into a 3-deep ring: two k-steps are in flight while the MFMAs of the third run.
//    The ring is retired with a COUNTED `s_waitcnt vmcnt(G)` (G = DMA instructions per stage per
//    wave) and a raw `s_barrier` — never `__syncthreads()`, whose fence would drain every DMA;
//  * fragments are read with inline-asm `ds_read_b128` / `ds_read_b64_tr_b16`: hipcc cannot tell
//    an LDS read from a builtin apart from the ring slot a DMA is writing, and waits vmcnt(0) before
//    it (which serialises the ring); the asm reads are waited for by hand (lgkmcnt + sched_barrier,
//    guide rule 18);
//  * LDS images (one __shared__ array, guide §5 item 4(a)):
//      KC ("K contiguous", operand stored [rows][K])  [rows][64 k], 128-B rows, 16-B chunk c of row r
//          stored at chunk c ^ (r & 7): every 16-lane group of a ds_read_b128 hits 16 distinct
//          16-B bank slots;
//      RC ("row contiguous", operand stored [K][cols]) [64 k][128 cols] sub-images, 256-B rows, chunk
//          c of k-row r at c ^ swz(r), read transposed by ds_read_b64_tr_b16 (T10);
//    the DMA writes lane-linearly, so the swizzle is applied to each lane's SOURCE address (rule 21);
//  * operand "sources" return the address of an 8-element chunk or nullptr (-> a zero page): the
//    im2col / transposed-conv gathers, padding and tile edges cost one select per lane, no branch
//    around the DMA.
// Epilogues are gemm_core.h's functors (per-element operator(), column sums for BN statistics).
#pragma once
#include "gemm_core.h"

namespace hopsx {

static __device__ __attribute__((aligned(64))) uint4 g_gg_zero[4];  // zero page, never written
static __device__ float g_gg_sink;                                   // HOPSX_GG_DIAG target

typedef __attribute__((address_space(3))) void* gg_lds_ptr;

__device__ __forceinline__ uint32_t gg_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(gg_lds_ptr)(p);
}

template <int OFF>
__device__ __forceinline__ bf16x8 gg_read_b128(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

template <int OFF>
__device__ __forceinline__ bf16x4 gg_read_tr(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  bf16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt at their maxima), N < 16
template <int N>
__device__ __forceinline__ void gg_wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

__device__ __forceinline__ int gg_rc_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// ---------------------------------------------------------------------------------------------
// Operand sources.  A logical operand is [O][I] with I contiguous in memory; the KC role stages
// rows (o fixed per DMA lane, i = k advancing 64 per k-step), the RC role stages k-rows (o = k
// advancing, i = column fixed per lane).  Everything that does not change along the k loop is
// decoded ONCE per lane into a GgSlot before the loop (the per-k-step address work is what the
// DMA issue competes with: MFMAs leave a SIMD's VALU issue half its cycles), then kc_at / rc_at
// return the chunk address for k-offset dk, or the zero page outside the operand, the conv
// geometry or the split's k range.
// ---------------------------------------------------------------------------------------------
struct GgSlot {
  const bf16_raw* q;  // base pointer of this lane
  int a, b, c, k0;    // source-specific invariants
  int rem;            // valid k-offsets: dk < rem
  bool ok;            // the fixed index is inside the operand
};

struct GgDense {  // [O][I] row-major, ld elements per row (ld % 8 == 0, base 16-B aligned)
  const bf16_raw* p;
  long ld;
  int olim, ilim;
  __device__ __forceinline__ GgSlot kc(int row, int k, int kend) const {
    const bool ok = row < olim;
    return GgSlot{p + (long)(ok ? row : 0) * ld + k, 0, 0, 0, k, min(ilim, kend) - k, ok};
  }
  __device__ __forceinline__ const void* kc_at(const GgSlot& s, int dk) const {
    return (s.ok && dk < s.rem) ? (const void*)(s.q + dk) : (const void*)g_gg_zero;
  }
  __device__ __forceinline__ GgSlot rc(int k, int col, int kend) const {
    const bool ok = col < ilim;
    return GgSlot{p + (long)k * ld + (ok ? col : 0), 0, 0, 0, k, min(olim, kend) - k, ok};
  }
  __device__ __forceinline__ const void* rc_at(const GgSlot& s, int dk) const {
    return (s.ok && dk < s.rem) ? (const void*)(s.q + (long)dk * ld) : (const void*)g_gg_zero;
  }
};

// im2col(X): (o = output pixel m, i = k = (kh, kw, ci)); C % 8 == 0
struct GgIm2col {
  const bf16_raw* x;
  ConvGeom g;
  int olim, ilim;  // pixels, KH*KW*C
  // KC (forward A): the pixel is fixed -> image base and the window origin
  __device__ __forceinline__ GgSlot kc(int m, int k, int kend) const {
    const bool ok = m < olim;
    const int mc = ok ? m : 0;
    const int b = g.fOHW.div(mc), rem = mc - b * (g.OH * g.OW);
    const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
    const bool in = ok && hx_check(b < g.B && oh < g.OH && ow < g.OW);  // (the fast divisions)
    return GgSlot{x + (long)b * g.H * g.W * g.C, oh * g.sh - g.ph, ow * g.sw - g.pw, 0, k, min(ilim, kend) - k, in};
  }
  __device__ __forceinline__ const void* kc_at(const GgSlot& s, int dk) const {
    const int k = s.k0 + dk;
    const int kc = k < ilim ? k : 0;
    const int t = g.fC.div(kc), ci = kc - t * g.C;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const int ih = s.a + kh * g.dh, iw = s.b + kw * g.dw;
    const bool ok = s.ok && dk < s.rem && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W &&
                    hx_check(kh < g.KH && ci < g.C);
    return ok ? (const void*)(s.q + (ih * g.W + iw) * g.C + ci) : (const void*)g_gg_zero;
  }
  // RC (weight-gradient B): the column k = (kh, kw, ci) is fixed -> channel and tap offsets
  __device__ __forceinline__ GgSlot rc(int m, int col, int kend) const {
    const bool ok = col < ilim;
    const int kc = ok ? col : 0;
    const int t = g.fC.div(kc), ci = kc - t * g.C;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    return GgSlot{x + ci, kh * g.dh - g.ph, kw * g.dw - g.pw, 0, m, min(olim, kend) - m, ok};
  }
  __device__ __forceinline__ const void* rc_at(const GgSlot& s, int dk) const {
    const int m = s.k0 + dk;
    const int mc = m < olim ? m : 0;
    const int b = g.fOHW.div(mc), rem = mc - b * (g.OH * g.OW);
    const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
    const int ih = oh * g.sh + s.a, iw = ow * g.sw + s.b;
    const bool ok = s.ok && dk < s.rem && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W &&
                    hx_check(b < g.B);
    return ok ? (const void*)(s.q + (((long)b * g.H + ih) * g.W + iw) * g.C) : (const void*)g_gg_zero;
  }
};

// dgrad A (KC): (o = input pixel (b, ih, iw), i = k = (kh, kw, co)) -> dY[b, oh, ow, co] where
// oh * sh = ih + ph - kh * dh (nullptr when not integral / outside); CO % 8 == 0
struct GgDgradA {
  const bf16_raw* dy;
  ConvGeom g;
  int olim, ilim;  // B*H*W, KH*KW*CO
  __device__ __forceinline__ GgSlot kc(int m, int k, int kend) const {
    const bool ok = m < olim;
    const int mc = ok ? m : 0;
    const int b = g.fHW.div(mc), rem = mc - b * (g.H * g.W);
    const int ih = g.fW.div(rem), iw = rem - ih * g.W;
    const bool in = ok && hx_check(b < g.B && ih < g.H && iw < g.W);
    return GgSlot{dy + (long)b * g.OH * g.OW * g.CO, ih + g.ph, iw + g.pw, 0, k, min(ilim, kend) - k, in};
  }
  __device__ __forceinline__ const void* kc_at(const GgSlot& s, int dk) const {
    const int k = s.k0 + dk;
    const int kc = k < ilim ? k : 0;
    const int t = g.fCO.div(kc), co = kc - t * g.CO;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const int hn = s.a - kh * g.dh, wn = s.b - kw * g.dw;
    const int hc = hn > 0 ? hn : 0, wc = wn > 0 ? wn : 0;
    const int oh = g.sh == 1 ? hc : g.fSH.div(hc), ow = g.sw == 1 ? wc : g.fSW.div(wc);
    const bool ok = s.ok && dk < s.rem && hn >= 0 && wn >= 0 && oh * g.sh == hn && ow * g.sw == wn && oh < g.OH &&
                    ow < g.OW && hx_check(kh < g.KH && co < g.CO);
    return ok ? (const void*)(s.q + (oh * g.OW + ow) * g.CO + co) : (const void*)g_gg_zero;
  }
};

// dgrad B (RC): W[co][kh][kw][ci] viewed as (o = k = (kh, kw, co), i = ci); C % 8 == 0
struct GgWeightT {
  const bf16_raw* w;
  ConvGeom g;
  int olim, ilim;  // KH*KW*CO, C
  __device__ __forceinline__ GgSlot rc(int k, int col, int kend) const {
    const bool ok = col < ilim;
    return GgSlot{w + (ok ? col : 0), 0, 0, 0, k, min(olim, kend) - k, ok};
  }
  __device__ __forceinline__ const void* rc_at(const GgSlot& s, int dk) const {
    const int k = s.k0 + dk;
    const int kc = k < olim ? k : 0;
    const int t = g.fCO.div(kc), co = kc - t * g.CO;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const bool ok = s.ok && dk < s.rem && hx_check(kh < g.KH && co < g.CO);
    return ok ? (const void*)(s.q + ((co * g.KH + kh) * g.KW + kw) * g.C) : (const void*)g_gg_zero;
  }
};

// ---- strided dgrad by input-pixel parity class (stride s > 1, dilation 1) ----
// dX[ih] gathers dY[oh] W[kh] over ih + ph - kh = s * oh: an input pixel with ih mod s = py only
// ever meets the taps kh = (py + ph) mod s (+ s, + 2s, ...).  So each of the s_h * s_w classes is a
// DENSE implicit GEMM over 1/(s_h s_w) of the pixels with ~1/(s_h s_w) of the taps, where the
// zero-inserting GgDgradA stages and multiplies the whole KH x KW window for every pixel (3 of 4
// taps of a 3x3 / stride-2 dgrad are zeros: the 2.5-3.2x gap to PyTorch in
// profiles/r3s7_conv_gemm_vs_torch.txt).
struct GgParGeom {
  int py, px;      // the class: ih mod sh, iw mod sw
  int kh0, kw0;    // first tap of the class per axis; taps kh0 + sh * t
  int nkh, nkw;    // taps per axis
  int Hp, Wp;      // input rows / columns of the class
  FastDiv fWp, fHWp, fNKW;
};

// A (KC): (o = class pixel (b, ihh, iww), i = k = (th, tw, co)) -> dY[b, oh, ow, co]
struct GgDgradParA {
  const bf16_raw* dy;
  ConvGeom g;
  GgParGeom c;
  int olim, ilim;  // B*Hp*Wp, nkh*nkw*CO
  __device__ __forceinline__ GgSlot kc(int m, int k, int kend) const {
    const bool ok = m < olim;
    const int mc = ok ? m : 0;
    const int b = c.fHWp.div(mc), rem = mc - b * (c.Hp * c.Wp);
    const int ihh = c.fWp.div(rem), iww = rem - ihh * c.Wp;
    const bool in = ok && hx_check(b < g.B && ihh < c.Hp && iww < c.Wp);
    return GgSlot{dy + (long)b * g.OH * g.OW * g.CO, g.sh * ihh + c.py + g.ph, g.sw * iww + c.px + g.pw, 0, k,
                  min(ilim, kend) - k, in};
  }
  __device__ __forceinline__ const void* kc_at(const GgSlot& s, int dk) const {
    const int k = s.k0 + dk;
    const int kc = k < ilim ? k : 0;
    const int t = g.fCO.div(kc), co = kc - t * g.CO;
    const int th = c.fNKW.div(t), tw = t - th * c.nkw;
    const int hn = s.a - (c.kh0 + g.sh * th), wn = s.b - (c.kw0 + g.sw * tw);  // multiples of s
    const int oh = g.fSH.div(hn > 0 ? hn : 0), ow = g.fSW.div(wn > 0 ? wn : 0);
    const bool ok = s.ok && dk < s.rem && hn >= 0 && wn >= 0 && oh < g.OH && ow < g.OW &&
                    hx_check(oh * g.sh == hn && ow * g.sw == wn && co < g.CO);  // (the class's taps only)
    return ok ? (const void*)(s.q + (oh * g.OW + ow) * g.CO + co) : (const void*)g_gg_zero;
  }
};

// B (RC): the class's taps of W[co][kh][kw][ci] as (o = k = (th, tw, co), i = ci)
struct GgWeightTPar {
  const bf16_raw* w;
  ConvGeom g;
  GgParGeom c;
  int olim, ilim;  // nkh*nkw*CO, C
  __device__ __forceinline__ GgSlot rc(int k, int col, int kend) const {
    const bool ok = col < ilim;
    return GgSlot{w + (ok ? col : 0), 0, 0, 0, k, min(olim, kend) - k, ok};
  }
  __device__ __forceinline__ const void* rc_at(const GgSlot& s, int dk) const {
    const int k = s.k0 + dk;
    const int kc = k < olim ? k : 0;
    const int t = g.fCO.div(kc), co = kc - t * g.CO;
    const int th = c.fNKW.div(t), tw = t - th * c.nkw;
    const int kh = c.kh0 + g.sh * th, kw = c.kw0 + g.sw * tw;
    const bool ok = s.ok && dk < s.rem && hx_check(kh < g.KH && kw < g.KW && co < g.CO);
    return ok ? (const void*)(s.q + ((co * g.KH + kh) * g.KW + kw) * g.C) : (const void*)g_gg_zero;
  }
};

// the class's rows land on their own pixels of dX: EpiDActBF16's act' / added gradient / column sum
struct EpiDgradParBF16 {
  static constexpr bool kVec8 = true;
  bf16_raw* out;
  const bf16_raw* yprev;
  int act;
  float* colsum;
  const bf16_raw* add;
  int C, H, W, Wp, HWp, py, px, sh, sw;
  FastDiv fWp, fHWp;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    const int b = fHWp.div(m), r = m - b * HWp;
    const int ihh = fWp.div(r), iww = r - ihh * Wp;
    const long pos = (((long)b * H + sh * ihh + py) * W + sw * iww + px) * C + n;
    if (yprev) v *= act_grad_from_out(bf2f(yprev[pos]), act);
    if (add) v += bf2f(add[pos]);
    out[pos] = f2bf(v);
    return v;
  }
  __host__ __device__ bool vec8_ok() const {
    return C % 8 == 0 && (uintptr_t)out % 16 == 0 && (uintptr_t)yprev % 16 == 0 && (uintptr_t)add % 16 == 0 && !colsum;
  }
  __device__ __forceinline__ void store8(int m, int n, const float* v) const {
    const int b = fHWp.div(m), r = m - b * HWp;
    const int ihh = fWp.div(r), iww = r - ihh * Wp;
    const long pos = (((long)b * H + sh * ihh + py) * W + sw * iww + px) * C + n;
    const bf16x8 yv = yprev ? *(const bf16x8*)(yprev + pos) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    const bf16x8 av = add ? *(const bf16x8*)(add + pos) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j];
      if (yprev) t *= act_grad_from_out(bf2f((uint16_t)yv[j]), act);
      if (add) t += bf2f((uint16_t)av[j]);
      q[j] = (short)f2bf(t);
    }
    *(bf16x8*)(out + pos) = q;
  }
};

// dW^T orientation of a weight gradient: the GEMM computes D[m = k][n = co], stored to out[n][m]
struct EpiAtomicF32T {
  float* out;
  long ldo;
  float alpha;
  float* colsum;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    v *= alpha;
    atomicAdd(out + (long)n * ldo + m, v);
    return v;
  }
};

// dgrad of a 1x1 / stride-s / unpadded conv as a DENSE GEMM over dY's pixels (M = B*OH*OW): the
// input pixel (oh*sh, ow*sw) gets the product, the rest of its s x s block only zeros (the implicit
// GEMM over dX's pixels would stage and multiply zero taps for (s*s - 1) / (s*s) of its rows).
// Requires H == OH*sh, W == OW*sw (the blocks tile dX exactly); act' of yprev and the added gradient
// as EpiDActBF16; no column sum.
struct EpiDgradScatterBF16 {
  bf16_raw* out;
  const bf16_raw* yprev;
  int act;
  const bf16_raw* add;
  int C, W, OW, OHW, sh, sw;
  FastDiv fOW, fOHW;
  float* colsum;  // always null (interface)
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    const int b = fOHW.div(m), r = m - b * OHW;
    const int oh = fOW.div(r), ow = r - oh * OW;
    const long H = (long)OHW / OW * sh;
    const long base = (((long)b * H + (long)oh * sh) * W + (long)ow * sw) * C + n;
    for (int dy = 0; dy < sh; ++dy)
      for (int dx = 0; dx < sw; ++dx) {
        const long pos = base + ((long)dy * W + dx) * C;
        float val = 0.f;
        if (dy == 0 && dx == 0) val = yprev ? v * act_grad_from_out(bf2f(yprev[pos]), act) : v;
        if (add) val += bf2f(add[pos]);
        out[pos] = f2bf(val);
      }
    return v;
  }
};

// ---------------------------------------------------------------------------------------------
// Kernel
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int S, bool BKC = true>
struct GgCfg {
  static constexpr int BK = 64;
  // B rows held in LDS: a 64-column RC (n-contiguous) operand still loads a whole 128-column sub-image (its
  // upper half is masked to the zero page, n >= N), so the RC DMA roles and swizzle stay those of 128
  static constexpr int BL = (BKC || BN >= 128) ? BN : 128;
  // 8 waves with 64-row wave tiles: 256x128 -> 4 x 2 waves of 64x64, 128x256 -> 2 x 4 of 64x64,
  // 128x128 -> 2 x 4 of 64x32
  static constexpr int WAVES_M = BM / 64, WAVES_N = 8 / WAVES_M;
  static constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BL * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int LDS = S * STAGE;
  // (BN = 64: the narrow-N tile, 256x64 -> 4 x 2 waves of 64x32)
  static_assert(BM % 128 == 0 && (BN % 128 == 0 || BN == 64), "tiles are multiples of 128 (or 64 columns)");
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <bool KC>
__device__ __forceinline__ constexpr int gg_dma_per_wave(int rows) {
  // KC: rows x 128 B = rows / 8 wave-instructions over 8 waves; RC: rows / 128 sub-images x 16 over 8
  return KC ? rows / 64 : (rows / 128) * 2;
}

// DMA lane roles of one operand tile (rows = BM or BN of the tile, starting at r0):
//   KC: wave-instruction i of wave w fills rows 8 (w + 8 i) .. +7 (128 B each); lane -> (row, chunk)
//   RC: sub-image s, wave-instruction i fills k-rows 4 (w + 8 i) .. +3 (256 B each)
template <bool KC, int ROWS>
struct GgLanes {
  static constexpr int N = KC ? ROWS / 64 : (ROWS / 128) * 2;
};

template <bool KC, int ROWS, class SRC>
__device__ __forceinline__ void gg_slots(const SRC& src, GgSlot* sl, int r0, int kbeg, int kend, int wave, int lane) {
  if constexpr (KC) {
    const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
    for (int i = 0; i < ROWS / 64; ++i) {
      const int row = 8 * (wave + 8 * i) + prow;
      sl[i] = src.kc(r0 + row, kbeg + 8 * (pch ^ (row & 7)), kend);
    }
  } else {
    const int prow = lane >> 4, pch = lane & 15;
#pragma unroll
    for (int s = 0; s < ROWS / 128; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kr = 4 * (wave + 8 * i) + prow;
        sl[s * 2 + i] = src.rc(kbeg + kr, r0 + s * 128 + 8 * (pch ^ gg_rc_swz(kr)), kend);
      }
  }
}

template <bool KC, int ROWS, class SRC>
__device__ __forceinline__ void gg_stage_operand(const SRC& src, const GgSlot* sl, unsigned char* img, int dk,
                                                 int wave) {
  if constexpr (KC) {
#pragma unroll
    for (int i = 0; i < ROWS / 64; ++i) {
      const void* p = src.kc_at(sl[i], dk);
      __builtin_amdgcn_global_load_lds(p, (gg_lds_ptr)(img + 8 * (wave + 8 * i) * 128), 16,
                                       0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < ROWS / 128; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const void* p = src.rc_at(sl[s * 2 + i], dk);
        __builtin_amdgcn_global_load_lds(p,
                                         (gg_lds_ptr)(img + s * 16384 + 4 * (wave + 8 * i) * 256), 16, 0, 0);
      }
  }
}

// One DMA of the stage (slot i of the operand's lane roles, see gg_slots)
template <bool KC, class SRC>
__device__ __forceinline__ void gg_dma1(const SRC& src, const GgSlot& sl, unsigned char* img, int i, int wave,
                                        int dk) {
  const void* p;
  unsigned char* dst;
  if constexpr (KC) {
    p = src.kc_at(sl, dk);
    dst = img + 8 * (wave + 8 * i) * 128;
  } else {
    p = src.rc_at(sl, dk);
    dst = img + (i >> 1) * 16384 + 4 * (wave + 8 * (i & 1)) * 256;
  }
  __builtin_amdgcn_global_load_lds(p, (gg_lds_ptr)dst, 16, 0, 0);
}

// Per-lane fragment readers (16 rows x 32 k MFMA fragments of a wave's 64-row strip).  All the
// swizzle arithmetic is loop-invariant: off[] holds each lane's byte offset of every fragment read
// of k-half 0; k-half 1 is +8192 B (RC: 32 k-rows of 256 B) or a fixed chunk flip (KC, kept as a
// second offset set), folded into the ds_read `offset:` immediate.  Per ring slot, at(base) adds
// the slot's LDS base once (one VALU per read address, shared by both k-halves).
//   KC: row = rbase + 16 i + fr, chunk (4 kk + fq) ^ (row & 7): fragment i = +2048 B.
//   RC: T10 lane roles (row q = tq of a 4-row block, columns 4 tp ..): fragment i moves the column
//       by 16, i.e. chunk ^ 2i (the strip's chunk bits 1-2 are free of the swizzle's carries); the two
//       4-row halves of a fragment have their own swizzle.
template <bool KC, int F>
struct GgReader {
  static constexpr int NA = KC ? 2 : 2 * F;  // address registers: KC one per k-half, RC one per (fragment, half)
  uint32_t off[NA];
  uint32_t adr[NA];
  __device__ __forceinline__ void init(int rbase, int fr, int fq, int tq, int tp) {
    if constexpr (KC) {
      const int row = rbase + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) off[kk] = row * 128 + 16 * ((kk * 4 + fq) ^ (row & 7));
    } else {
      const int col = rbase + 4 * tp;
      const int c = col & 127;
#pragma unroll
      for (int i = 0; i < F; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 8 * fq + tq + 4 * h;
          off[2 * i + h] = ((col >> 7) * 16384 + r * 256 + 16 * ((c >> 3) ^ gg_rc_swz(r)) + 2 * (c & 7)) ^ (32 * i);
        }
    }
  }
  __device__ __forceinline__ void at(uint32_t base) {
#pragma unroll
    for (int q = 0; q < NA; ++q) adr[q] = base + off[q];
  }
  template <int KK>
  __device__ __forceinline__ bf16x8 read(int i) const {
    if constexpr (KC) {
      // i * 2048 is a compile-time constant after unrolling only; keep it in the address add
      return gg_read_b128<0>(adr[KK] + i * 2048);
    } else {
      const bf16x4 v1 = gg_read_tr<KK * 8192>(adr[2 * i]);
      const bf16x4 v2 = gg_read_tr<KK * 8192>(adr[2 * i + 1]);
      return (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
    }
  }
};

template <int BM, int BN, int S, bool A_KC, bool B_KC, class AS, class BS, class EP>
__global__ __launch_bounds__(512) void gg_kernel(const AS as, const BS bs, const EP ep, int M, int N, int K, int kps,
                                                 int tiles_n, int tiles, int diag) {
  using C = GgCfg<BM, BN, S, B_KC>;
  constexpr int BK = C::BK, FM = C::FM, FN = C::FN, BL = C::BL;
  constexpr int G = gg_dma_per_wave<A_KC>(BM) + gg_dma_per_wave<B_KC>(BL);
  __shared__ __attribute__((aligned(1024))) unsigned char smem[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WAVES_N, wn = wave % C::WAVES_N;
  // XCD-aware: consecutive virtual ids (neighbouring tiles of one split) share an XCD's L2
  const int v = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = v % tiles, split = v / tiles;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int kbeg = split * kps;
  const int kend = min(K, kbeg + kps);
  if (kbeg >= kend) return;
  const int nt = (kend - kbeg + BK - 1) / BK;

  constexpr int GA = GgLanes<A_KC, BM>::N;
  GgSlot sa[GA], sb[GgLanes<B_KC, BL>::N];
  gg_slots<A_KC, BM>(as, sa, m0, kbeg, kend, wave, lane);
  gg_slots<B_KC, BL>(bs, sb, n0, kbeg, kend, wave, lane);
  // DMA q (0 .. G-1) of the stage of k-step ks into ring slot ks % S.  Stages past the last k-step
  // are issued too: every lane is then masked to the zero page (dk >= rem), so they only write
  // zeros into a slot nobody reads, and the loop needs no branch and a constant vmcnt.
  auto dma = [&](int q, int ks) {
    unsigned char* img = smem + (ks % S) * C::STAGE;
    const int dk = ks * BK;
    if (q < GA) gg_dma1<A_KC>(as, sa[q], img, q, wave, dk);
    else gg_dma1<B_KC>(bs, sb[q - GA], img + C::A_BYTES, q - GA, wave, dk);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const uint32_t base = gg_lds_addr(smem);
  GgReader<A_KC, FM> ra;
  GgReader<B_KC, FN> rb;
  ra.init(wm * C::WTM, fr, fq, tq, tp);
  rb.init(wn * C::WTN, fr, fq, tq, tp);

  // fragments: k-half 0 and k-half 1 of the current k-step (8 VGPR x (FM + FN) each)
  bf16x8 a0[FM], b0[FN], a1[FM], b1[FN];
  constexpr int NH = FM + FN;  // fragments per k-half
  auto read_k0 = [&](int f) {
    if (f < FM) a0[f] = ra.template read<0>(f);
    else b0[f - FM] = rb.template read<0>(f - FM);
  };
  auto read_k1 = [&](int f) {
    if (f < FM) a1[f] = ra.template read<1>(f);
    else b1[f - FM] = rb.template read<1>(f - FM);
  };
  auto point = [&](uint32_t slot_base) {  // readers -> ring slot
    ra.at(slot_base);
    rb.at(slot_base + C::A_BYTES);
  };

  // Software pipeline, one barrier per k-step.  Entering step t, a0/b0 hold its k-half 0:
  //   phase 1: k-half-0 MFMAs; in their gaps the DMAs of stage t+2 (ring slot of step t-1) and the
  //            reads of this step's k-half 1 into a1/b1 (slot t, visible since the last barrier)
  //   lgkmcnt(0) + vmcnt(G) (this wave's stage t+1 landed, t+2 in flight) + s_barrier
  //   phase 2: k-half-1 MFMAs; in their gaps the reads of step t+1's k-half 0 into a0/b0
  //   lgkmcnt(0)
  // WAR: slot (t+2) % 3 = (t-1) % 3 was last read before the previous step's barrier (every read
  // is retired by an lgkmcnt(0) before the barrier that follows it).
  auto step = [&](int t) {
    constexpr int NQ = FM * FN;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
        const int q = i * FN + j;
        if (q < G) dma(q, t + 2);
#pragma unroll
        for (int f = q * NH / NQ; f < (q + 1) * NH / NQ; ++f) read_k1(f);
        __builtin_amdgcn_sched_barrier(0);
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): a1/b1
    gg_wait_vm<G>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    point(base + ((t + 1) % S) * C::STAGE);  // the readers keep this slot for the next phase 1
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
        const int q = i * FN + j;
#pragma unroll
        for (int f = q * NH / NQ; f < (q + 1) * NH / NQ; ++f) read_k0(f);
        __builtin_amdgcn_sched_barrier(0);
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): a0/b0
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: stages 0 and 1 in flight, wait for stage 0, read step 0's k-half 0
#pragma unroll
  for (int q = 0; q < G; ++q) dma(q, 0);
#pragma unroll
  for (int q = 0; q < G; ++q) dma(q, 1);
  gg_wait_vm<G>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  point(base);
#pragma unroll
  for (int f = 0; f < NH; ++f) read_k0(f);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  for (int t = 0; t < nt; ++t) step(t);
  gg_wait_vm<0>();  // the trailing (all-zero) stages: no DMA may outlive the workgroup's LDS

  if (diag) {  // diagnostic (HOPSX_GG_DIAG=1): main loop only, one atomic per lane keeps the MFMAs live
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 1.2345e-30f) atomicAdd(&g_gg_sink, s);
    return;
  }
  // vectorized epilogue (epilogues with store8, no column sum, N % 8 == 0): the tile goes through LDS
  // as fp32 rows and leaves as 16-B stores of 8 consecutive columns (the fragment layout stores 2-B
  // values, four 32-B pieces per wave instruction) — also 16-B loads of the act' / addend operands
  // BN-backward dgrad epilogue (EpiDgradBnBF16): the same LDS-staged 16-B path, and each thread's column
  // sums (its 8-column chunk is fixed: 512 threads, BN / 8 chunks per row) meet in LDS in a fixed order
  // before one atomic pair per column into this tile's replica row
  if constexpr (has_bn2<EP>::value) {
    constexpr int SR = BN + 4;
    static_assert(BM * SR * 4 <= C::LDS && 512 * 16 * 4 <= C::LDS, "BN epilogue staging must fit the tile's LDS");
    if (N % 8 == 0 && ep.vec8_ok()) {
      float* st = (float*)smem;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            st[(wm * C::WTM + i * 16 + fq * 4 + r) * SR + wn * C::WTN + j * 16 + fr] = acc[i][j][r];
      __syncthreads();
      constexpr int CPR = BN / 8;
      static_assert(512 % CPR == 0, "a thread's column chunk must stay fixed");
      float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int c = tid; c < BM * CPR; c += 512) {
        const int row = c / CPR, col = (c - row * CPR) * 8;
        const int m = m0 + row, n = n0 + col;
        if (m < M && n < N) {
          const f32x4 v0 = *(const f32x4*)(st + row * SR + col), v1 = *(const f32x4*)(st + row * SR + col + 4);
          const float vv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          ep.store8_bn(m, n, vv, s1, s2);
        }
      }
      __syncthreads();  // the staged tile is consumed: its LDS takes the per-thread sums
      float* red = (float*)smem;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[tid * 16 + j] = s1[j];
        red[tid * 16 + 8 + j] = s2[j];
      }
      __syncthreads();
      const bool det = det_on();
      if (det) det_turn_begin(DET_GG_COLSUM, (unsigned)blockIdx.x);
      if (tid < BN && n0 + tid < N) {
        const int ch = tid >> 3, j = tid & 7;
        float a = 0.f, b = 0.f;
        for (int q = ch; q < 512; q += CPR) {
          a += red[q * 16 + j];
          b += red[q * 16 + 8 + j];
        }
        float* d = ep.colsum + (long)(v % HOPSX_BN_NREP) * 2 * N;
        atomicAdd(d + n0 + tid, a);
        atomicAdd(d + N + n0 + tid, b);
      }
      if (det) det_turn_end(DET_GG_COLSUM, (unsigned)blockIdx.x, gridDim.x);
      return;
    }
  }
  if constexpr (has_vec8<EP>::value && !has_bn2<EP>::value) {
    constexpr int SR = BN + 4;  // fp32 row stride (bank offset 4 between the fragment's 4 rows)
    static_assert(BM * SR * 4 <= C::LDS, "vector epilogue staging must fit the tile's LDS");
    if (N % 8 == 0 && ep.vec8_ok()) {
      float* st = (float*)smem;
      __syncthreads();  // every wave's last fragment reads of the main loop are done
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            st[(wm * C::WTM + i * 16 + fq * 4 + r) * SR + wn * C::WTN + j * 16 + fr] = acc[i][j][r];
      __syncthreads();
      constexpr int CPR = BN / 8;  // 8-column chunks per row
#pragma unroll 4
      for (int c = tid; c < BM * CPR; c += 512) {
        const int row = c / CPR, col = (c - row * CPR) * 8;
        const int m = m0 + row, n = n0 + col;
        if (m < M && n < N) {
          const f32x4 v0 = *(const f32x4*)(st + row * SR + col), v1 = *(const f32x4*)(st + row * SR + col + 4);
          const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          ep.store8(m, n, v);
        }
      }
      return;
    }
  }
  // epilogue: lane holds D[row = 16 i + 4 fq + r][col = 16 j + fr] of its wave tile
  float cs[FN], cs2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { cs[j] = 0.f; cs2[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * C::WTN + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * C::WTM + i * 16 + fq * 4 + r;
        if (m < M && n < N) {
          const float vv = ep(m, n, acc[i][j][r]);
          cs[j] += vv;
          if constexpr (has_bn2<EP>::value) cs2[j] += ep.second(m, n, vv);
          else if constexpr (has_sq<EP>::value) cs2[j] = fmaf(vv, vv, cs2[j]);
        }
      }
    }
  }
  if (ep.colsum) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = cs[j];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const int n = n0 + wn * C::WTN + j * 16 + fr;
      if constexpr (has_sq<EP>::value) {
        float q = cs2[j];
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        float* d = ep.colsum + (long)(v % HOPSX_BN_NREP) * 2 * N;
        if (fq == 0 && n < N) {
          atomicAdd(d + n, s);
          atomicAdd(d + N + n, q);
        }
      } else {
        if (fq == 0 && n < N) atomicAdd(ep.colsum + n, s);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Host side: tile choice + split-K, then launch.  Returns false (nothing launched) when the shape
// is too small to fill the chip with these tiles — the caller keeps gemm_core.h's engine.
// ---------------------------------------------------------------------------------------------
struct GgPlan {
  int cfg;  // 0: 256x128, 1: 128x256, 2: 128x128, 3: 256x64 (N <= 64, both operands k-contiguous)
  int split, kps, tiles_n, tiles;
};

inline bool gg_plan(long M, long N, long K, bool allow_split, GgPlan& p, long min_wg_override = -1,
                    int num_cu = 256, bool narrow_ok = false) {
  static const long force = hopsx_env_int("HOPSX_GG_CFG", -1);
  // 64: the stage-4 ResNet-50 shapes (7x7, 100 tiles of 128x128) run 1.5-2.2x faster on gg than on
  // gemm_core.h even at 0.4 workgroups per CU (profiles/r4_gg_min_wg_ab.txt); 32 (round 5): the B=8
  // shapes with 32-63 tiles too (ResNet-50 B=8 +1.5 %, B=64 / CIFAR flat: profiles/r5_gemm_knobs_b8_ab.txt)
  static const long min_wg_env = hopsx_env_int("HOPSX_GG_MIN_WG", 32);
  const long min_wg = min_wg_override >= 0 ? min_wg_override : min_wg_env;
  static const long split_target = hopsx_env_int("HOPSX_GG_SPLIT_TARGET", 1);
  static const long min_ks = hopsx_env_int("HOPSX_GG_SPLIT_MINKT", 8);
  auto ntiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  const long t0 = ntiles(256, 128), t1 = ntiles(128, 256), t2 = ntiles(128, 128);
  if (force >= 0 && force <= 2) {
    p.cfg = (int)force;
  } else if (narrow_ok && N <= 64 && (allow_split || ntiles(256, 64) >= num_cu)) {
    // a 64-column output (the stage-1 3x3 convs of ResNet-50, their weight gradients' 64 output channels):
    // a 128-wide tile would waste half its MFMAs
    p.cfg = 3;
  } else if (allow_split) {
    // split-K GEMMs get their parallelism from K: the biggest tile the output shape allows
    p.cfg = (M >= 256 && M >= N) ? 0 : (N >= 256 ? 1 : 2);
  } else {
    // one tile per CU at least when the big tiles can have it, else 128x128
    if (M >= 256 && t0 >= num_cu && t0 <= t1) p.cfg = 0;
    else if (N >= 256 && t1 >= num_cu) p.cfg = 1;
    else p.cfg = 2;
  }
  const int bm = p.cfg == 0 || p.cfg == 3 ? 256 : 128, bn = p.cfg == 1 ? 256 : (p.cfg == 3 ? 64 : 128);
  p.tiles_n = (int)((N + bn - 1) / bn);
  p.tiles = (int)((M + bm - 1) / bm) * p.tiles_n;
  long s = 1;
  if (allow_split) {
    const long target = split_target * num_cu;
    if (p.tiles < target) s = (target + p.tiles - 1) / p.tiles;
    const long maxs = (K + min_ks * 64 - 1) / (min_ks * 64);
    static const long smax = hopsx_env_int("HOPSX_GG_SPLIT_MAX", 64);
    if (s > maxs) s = maxs;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
  }
  long kps = (K + s - 1) / s;
  kps = (kps + 63) / 64 * 64;
  p.kps = (int)(kps > 0 ? kps : 64);
  p.split = (int)((K + p.kps - 1) / p.kps);
  if (p.split < 1) p.split = 1;
  const long wgs = (long)p.tiles * p.split;
  (void)t2;
  return wgs >= min_wg && wgs < (1L << 31);
}

template <bool A_KC, bool B_KC, class AS, class BS, class EP>
inline bool launch_gg(const AS& as, const BS& bs, const EP& ep, int M, int N, int K, bool allow_split,
                      hipStream_t st, long min_wg_override = -1) {
  // deterministic mode keeps gemm_core.h's engine (one K slice per tile, turn-ordered column sums)
  if (M <= 0 || N <= 0 || K <= 0 || hopsx_disabled("gg") || hopsx_deterministic()) return false;
  GgPlan p;
  static const bool narrow = !hopsx_disabled("gg_n64");
  if (!gg_plan(M, N, K, allow_split, p, min_wg_override, 256, narrow)) return false;
  static const int diag = (int)hopsx_env_int("HOPSX_GG_DIAG", 0);
  const dim3 grid((unsigned)(p.tiles * p.split));
  switch (p.cfg) {
    case 0:
      hipLaunchKernelGGL((gg_kernel<256, 128, 3, A_KC, B_KC, AS, BS, EP>), grid, dim3(512), 0, st, as, bs, ep, M, N, K,
                         p.kps, p.tiles_n, p.tiles, diag);
      break;
    case 1:
      hipLaunchKernelGGL((gg_kernel<128, 256, 3, A_KC, B_KC, AS, BS, EP>), grid, dim3(512), 0, st, as, bs, ep, M, N, K,
                         p.kps, p.tiles_n, p.tiles, diag);
      break;
    case 3:
      hipLaunchKernelGGL((gg_kernel<256, 64, 3, A_KC, B_KC, AS, BS, EP>), grid, dim3(512), 0, st, as, bs, ep, M, N, K,
                         p.kps, p.tiles_n, p.tiles, diag);
      break;
    default:
      hipLaunchKernelGGL((gg_kernel<128, 128, 3, A_KC, B_KC, AS, BS, EP>), grid, dim3(512), 0, st, as, bs, ep, M, N, K,
                         p.kps, p.tiles_n, p.tiles, diag);
      break;
  }
  return true;
}

}  // namespace hopsx
