// hopsx MFMA GEMM engine for gfx950 (MI355X).
//
// One templated main loop serves every matmul-shaped op in the framework:
// dense GEMM (Linear fwd / dgrad / wgrad), implicit-GEMM conv2d fwd / dgrad /
// wgrad and the wide&deep / MLP towers.  The operand *loaders* are functors
// that return 8 consecutive bf16 values along the operand's contiguous axis,
// so im2col / transposed-conv gathers happen on the fly while a tile is
// staged into LDS — nothing is materialised in HBM.
//
// Design (see /opt/skills/guides/cdna_hip_programming.md §3, §5):
//  * v_mfma_f32_16x16x32_bf16, fp32 accumulate, 4 waves (256 threads) per
//    workgroup, BK = 64.
//  * Two LDS images per operand:
//      KC  ("K contiguous")  [rows][64 k]   read with ds_read_b128,
//                                            16-B chunk XOR-swizzled c^(row&7)
//                                            -> conflict-free (4 LDS cycles).
//      RC  ("row contiguous") [64 k][rows]  read with ds_read_b64_tr_b16 (T10)
//                                            hardware transpose, chunk XOR
//                                            swizzle keyed on k.
//    So a transposed operand (dgrad's W, wgrad's dY and X) never needs a
//    transposed copy in HBM.
//  * Register-staged double buffer (T14): tile t+1's global loads are issued
//    before tile t's MFMAs and written to the other LDS buffer afterwards.
//  * XCD-aware bijective workgroup remap (T1) and split-K over gridDim.y with
//    fp32 atomics for reduction-heavy shapes (wgrad with K = batch*pixels).
//  * Fused epilogues: bias + activation, bf16/fp32 store, fp32 atomic
//    accumulate (gradient buffers), activation-derivative mask, and an
//    optional per-column sum (bias gradient) reduced in-wave + one atomic per
//    column per wave.
#pragma once
#include "common.h"

namespace hopsx {

constexpr int GEMM_BK = 64;

__device__ __forceinline__ int rc_swz(int k, int cpr) {
  return (2 * ((k & 3) | (((k >> 3) & 1) << 2))) & (cpr - 1);
}

// ----------------------------------------------------------------------------
// Loaders: bf16x8 load(outer, inner, outer_lim, inner_lim) returns elements
// (outer, inner .. inner+7) — 8 consecutive along the contiguous axis, zero
// outside [0, lim).  inner is always a multiple of 8.
// ----------------------------------------------------------------------------
// Prologue fusion: multiply a loaded operand by act'(y) (y = the activation
// output with the operand's layout) so backward GEMMs consume dY directly and
// the separate activation-backward pass disappears.
// (the act switch is hoisted out of the element loop: one uniform branch per call, straight-line
// element code — a per-element switch compiled to ~8 branches per call)
__device__ __forceinline__ void mask8(bf16x8& v, const bf16x8& y, int act) {
  if (act == ACT_RELU) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (short)y[j] > 0 ? v[j] : (short)0;  // bf16 > 0 <=> positive int16 bits
  } else if (act != ACT_NONE) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (short)f2bf(bf2f((uint16_t)v[j]) * act_grad_from_out(bf2f((uint16_t)y[j]), act));
  }
}

struct DenseLoader {
  const bf16_raw* p;
  long ld;
  int vec;               // ld % 8 == 0 and base 16-B aligned
  const bf16_raw* y;     // optional activation output for the fused act' mask (same layout as p)
  int act;
  __device__ __forceinline__ bf16x8 load(int o, int i, int olim, int ilim) const {
    bf16x8 r = {0, 0, 0, 0, 0, 0, 0, 0};
    if (o >= olim) return r;
    const long off = (long)o * ld + i;
    const bf16_raw* q = p + off;
    if (vec && i + 8 <= ilim) {
      r = *(const bf16x8*)q;
      if (y) mask8(r, *(const bf16x8*)(y + off), act);
      return r;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j < ilim) {
        if (y) r[j] = (short)f2bf(bf2f(q[j]) * act_grad_from_out(bf2f(y[off + j]), act));
        else r[j] = (short)q[j];
      }
    }
    return r;
  }
};

// Multiply-high "magic number" division (Granlund-Montgomery): the im2col /
// transposed-conv gathers decode (b, oh, ow) and (kh, kw, ci) for every staged
// element; hardware has no integer divider, so a generic '/' costs ~40 VALU
// ops while this costs 3.
struct FastDiv {
  uint32_t d, mul, shift;
  void init(uint32_t dd) {
    d = dd ? dd : 1;
    shift = 0;
    while ((1ull << shift) < d) ++shift;
    mul = (uint32_t)((((1ull << 32) * ((1ull << shift) - d)) / d) + 1);
  }
  __device__ __forceinline__ int div(int n) const {
    return (int)((((uint64_t)__umulhi((uint32_t)n, mul)) + (uint32_t)n) >> shift);
  }
};

struct ConvGeom {
  int B, H, W, C;      // input NHWC
  int OH, OW, CO;      // output NHWC
  int KH, KW, sh, sw, ph, pw, dh, dw;
  FastDiv fC, fCO, fKW, fOW, fOHW, fW, fHW, fSH, fSW;
  void init_div() {
    fC.init(C); fCO.init(CO); fKW.init(KW); fOW.init(OW); fOHW.init(OH * OW);
    fW.init(W); fHW.init(H * W); fSH.init(sh); fSW.init(sw);
  }
};

// im2col view of X: (outer = output pixel m, inner = k = (kh, kw, ci))
struct Im2colLoader {
  const bf16_raw* x;
  ConvGeom g;
  int vec;  // C % 8 == 0 and aligned
  __device__ __forceinline__ short at(int b, int oh, int ow, int k) const {
    const int t = g.fC.div(k);
    const int ci = k - t * g.C;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const int ih = oh * g.sh - g.ph + kh * g.dh;
    const int iw = ow * g.sw - g.pw + kw * g.dw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return 0;
    return (short)x[(((long)b * g.H + ih) * g.W + iw) * g.C + ci];
  }
  __device__ __forceinline__ bf16x8 load(int m, int k, int olim, int ilim) const {
    bf16x8 r = {0, 0, 0, 0, 0, 0, 0, 0};
    if (m >= olim) return r;
    const int ohw = g.OH * g.OW;
    const int b = g.fOHW.div(m), rem = m - b * ohw;
    const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
    if (vec && k + 8 <= ilim) {
      const int t = g.fC.div(k);
      const int ci = k - t * g.C;
      const int kh = g.fKW.div(t), kw = t - kh * g.KW;
      const int ih = oh * g.sh - g.ph + kh * g.dh;
      const int iw = ow * g.sw - g.pw + kw * g.dw;
      if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return r;
      return *(const bf16x8*)(x + (((long)b * g.H + ih) * g.W + iw) * g.C + ci);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (k + j < ilim) ? at(b, oh, ow, k + j) : (short)0;
    return r;
  }
};

// dgrad A operand: (outer = input pixel (b, ih, iw), inner = k = (kh, kw, co))
// value = dY[b, oh, ow, co] with oh*sh = ih + ph - kh*dh (zero if not integral)
struct ConvDgradALoader {
  const bf16_raw* dy;
  ConvGeom g;
  int vec;            // CO % 8 == 0 and aligned
  const bf16_raw* y;  // optional: this conv's activation output -> fused act' mask on dY
  int act;
  __device__ __forceinline__ short at(int b, int ih, int iw, int k) const {
    const int t = g.fCO.div(k);
    const int co = k - t * g.CO;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const int hn = ih + g.ph - kh * g.dh, wn = iw + g.pw - kw * g.dw;
    if (hn < 0 || wn < 0) return 0;
    const int oh = g.fSH.div(hn), ow = g.fSW.div(wn);
    if (oh * g.sh != hn || ow * g.sw != wn || oh >= g.OH || ow >= g.OW) return 0;
    const long o = (((long)b * g.OH + oh) * g.OW + ow) * g.CO + co;
    if (y) return (short)f2bf(bf2f(dy[o]) * act_grad_from_out(bf2f(y[o]), act));
    return (short)dy[o];
  }
  __device__ __forceinline__ bf16x8 load(int m, int k, int olim, int ilim) const {
    bf16x8 r = {0, 0, 0, 0, 0, 0, 0, 0};
    if (m >= olim) return r;
    const int hw = g.H * g.W;
    const int b = g.fHW.div(m), rem = m - b * hw;
    const int ih = g.fW.div(rem), iw = rem - ih * g.W;
    if (vec && k + 8 <= ilim) {
      const int t = g.fCO.div(k);
      const int co = k - t * g.CO;
      const int kh = g.fKW.div(t), kw = t - kh * g.KW;
      const int hn = ih + g.ph - kh * g.dh, wn = iw + g.pw - kw * g.dw;
      if (hn < 0 || wn < 0) return r;
      const int oh = g.fSH.div(hn), ow = g.fSW.div(wn);
      if (oh * g.sh != hn || ow * g.sw != wn || oh >= g.OH || ow >= g.OW) return r;
      const long o = (((long)b * g.OH + oh) * g.OW + ow) * g.CO + co;
      r = *(const bf16x8*)(dy + o);
      if (y) mask8(r, *(const bf16x8*)(y + o), act);
      return r;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (k + j < ilim) ? at(b, ih, iw, k + j) : (short)0;
    return r;
  }
};

// dgrad B operand: W[co][kh][kw][ci] viewed as (outer = k = (kh, kw, co), inner = ci)
struct ConvWeightTLoader {
  const bf16_raw* w;
  ConvGeom g;
  int vec;  // C % 8 == 0 and aligned
  __device__ __forceinline__ bf16x8 load(int k, int ci, int olim, int ilim) const {
    bf16x8 r = {0, 0, 0, 0, 0, 0, 0, 0};
    if (k >= olim) return r;
    const int t = g.fCO.div(k);
    const int co = k - t * g.CO;
    const int kh = g.fKW.div(t), kw = t - kh * g.KW;
    const bf16_raw* q = w + (((long)co * g.KH + kh) * g.KW + kw) * g.C + ci;
    if (vec && ci + 8 <= ilim) return *(const bf16x8*)q;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (ci + j < ilim) ? (short)q[j] : (short)0;
    return r;
  }
};

// ----------------------------------------------------------------------------
// Epilogues.  operator()(m, n, v) handles one output element and returns the
// value that should enter the optional column sum.
// ----------------------------------------------------------------------------
struct EpiStoreBF16 {  // out = act(alpha*acc + bias[n])
  static constexpr bool kVec8 = true;
  bf16_raw* out;
  long ldo;
  const float* bias;
  float alpha;
  int act;
  float* colsum;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    v = v * alpha + (bias ? bias[n] : 0.f);
    v = apply_act(v, act);
    out[(long)m * ldo + n] = f2bf(v);
    return v;
  }
  // the vectorized epilogue (gemm_glds.h): 8 consecutive columns n..n+7 of row m, one 16-B store
  __host__ __device__ bool vec8_ok() const { return ldo % 8 == 0 && (uintptr_t)out % 16 == 0 && !colsum; }
  __device__ __forceinline__ void store8(int m, int n, const float* v) const {
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = (short)f2bf(apply_act(v[j] * alpha + (bias ? bias[n + j] : 0.f), act));
    *(bf16x8*)(out + (long)m * ldo + n) = q;
  }
};

// out = bf16(acc) for a conv feeding a training BatchNorm: the column statistics (sum and sum of
// squares of the stored bf16 values) go to colsum = the replicas [HOPSX_BN_NREP][2N] (kSq)
struct EpiBnStatsBF16 {
  static constexpr bool kSq = true;
  bf16_raw* out;
  long ldo;
  float* colsum;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    const bf16_raw b = f2bf(v);
    out[(long)m * ldo + n] = b;
    return bf2f(b);
  }
};

struct EpiStoreF32 {  // out = act(alpha*acc + bias[n]) + beta*out
  float* out;
  long ldo;
  const float* bias;
  float alpha, beta;
  int act;
  float* colsum;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    v = v * alpha + (bias ? bias[n] : 0.f);
    v = apply_act(v, act);
    float* o = out + (long)m * ldo + n;
    if (beta != 0.f) v += beta * *o;
    *o = v;
    return v;
  }
};

struct EpiAtomicF32 {  // out += alpha*acc (split-K safe)
  float* out;
  long ldo;
  float alpha;
  float* colsum;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    v *= alpha;
    atomicAdd(out + (long)m * ldo + n, v);
    return v;
  }
};

// Split-K with an in-launch finish: every K-slice adds into the fp32 workspace `out`
// (persistent, zero at rest); the slice that draws the last ticket of its tile reads the
// tile back, applies the real epilogue (bias/act/bf16 store, dact mask, colsum) and
// re-zeroes the workspace tile and its counter — no memset node, no finishing kernel.
// epilogue ids of ops_api.h's GemmEpi (this header does not depend on the C ABI header)
constexpr int kEpiStoreBF16 = 0, kEpiStoreF32 = 1, kEpiDActBF16 = 3;
constexpr int kEpiBnStatsBF16 = 4;  // (finish only) bf16 store + BN sums of the stored values (EpiBnStatsBF16)

struct SplitFinish {
  unsigned* cnt;  // one counter per output tile, zero at rest
  int epi;        // EPI_STORE_BF16 / EPI_STORE_F32 / EPI_DACT_BF16 / kEpiBnStatsBF16
  void* out;
  long ldo;
  const float* bias;
  float alpha, beta;
  int act;
  const bf16_raw* aux;
  long ldaux;
  float* colsum;        // plain column sums; for kEpiBnStatsBF16 the replicas [HOPSX_BN_NREP][2N]
  const bf16_raw* add;  // kEpiDActBF16: a gradient to add (EpiDActBF16::add), layout of out
};

struct EpiAtomicTicket {
  float* out;  // workspace [M][N]
  long ldo;
  float alpha;
  float* colsum;  // unused in the slice pass
  SplitFinish fin;
  static constexpr bool kTicket = true;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    atomicAdd(out + (long)m * ldo + n, v);
    return v;
  }
};

template <class EP, class = void>
struct has_vec8 { static constexpr bool value = false; };
template <class EP>
struct has_vec8<EP, decltype((void)EP::kVec8)> { static constexpr bool value = EP::kVec8; };

template <class EP, class = void>
struct has_ticket { static constexpr bool value = false; };
template <class EP>
struct has_ticket<EP, decltype((void)EP::kTicket)> { static constexpr bool value = EP::kTicket; };
template <class EP, class = void>
struct has_sq { static constexpr bool value = false; };
template <class EP>
struct has_sq<EP, decltype((void)EP::kSq)> { static constexpr bool value = EP::kSq; };
template <class EP, class = void>
struct has_pre { static constexpr bool value = false; };
template <class EP>
struct has_pre<EP, decltype((void)EP::kPre)> { static constexpr bool value = EP::kPre; };

// out = acc * act'(y[m,n])  (backprop through the activation whose OUTPUT is y)
struct EpiDActBF16 {
  static constexpr bool kVec8 = true;
  bf16_raw* out;
  long ldo;
  const bf16_raw* y;
  long ldy;
  int act;
  float* colsum;        // optional: bias gradient of the layer that produced y
  const bf16_raw* add;  // optional: a gradient to add (a ResNet identity shortcut's), same layout as out
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    if (y) v *= act_grad_from_out(bf2f(y[(long)m * ldy + n]), act);
    if (add) v += bf2f(add[(long)m * ldo + n]);
    out[(long)m * ldo + n] = f2bf(v);
    return v;
  }
  __host__ __device__ bool vec8_ok() const {
    return ldo % 8 == 0 && (uintptr_t)out % 16 == 0 && (!y || (ldy % 8 == 0 && (uintptr_t)y % 16 == 0)) &&
           (uintptr_t)add % 16 == 0 && !colsum;
  }
  __device__ __forceinline__ void store8(int m, int n, const float* v) const {
    const bf16x8 yv = y ? *(const bf16x8*)(y + (long)m * ldy + n) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    const bf16x8 av = add ? *(const bf16x8*)(add + (long)m * ldo + n) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j];
      if (y) t *= act_grad_from_out(bf2f((uint16_t)yv[j]), act);
      if (add) t += bf2f((uint16_t)av[j]);
      q[j] = (short)f2bf(t);
    }
    *(bf16x8*)(out + (long)m * ldo + n) = q;
  }
};

// Conv dgrad whose input x is a training BatchNorm's output consumed only by this conv (see
// conv_mfma.hip DgradArgs bnacc): g = act'(y) * (acc + add) is stored (bf16) and its column sums
// sum g (the plain colsum) and sum g * (z - mean) * rstd (second()) go to the BN accumulator's replica
// rows colsum[HOPSX_BN_NREP][2N] (kSq layout), which the BN's apply-only backward folds.
struct EpiDgradBnBF16 {
  static constexpr bool kSq = true;
  static constexpr bool kBn2 = true;
  bf16_raw* out;
  long ldo;
  const bf16_raw* y;    // the BN output (= this conv's input), for act'; null: no activation
  int act;
  const bf16_raw* add;  // optional: a shortcut's gradient of x, added before the mask
  const bf16_raw* z;    // the BN input, layout of out
  const float* mean;
  const float* rstd;
  float* colsum;
  __device__ __forceinline__ float operator()(int m, int n, float v) const {
    const long o = (long)m * ldo + n;
    if (add) v += bf2f(add[o]);
    if (y) v *= act_grad_from_out(bf2f(y[o]), act);
    const bf16_raw b = f2bf(v);
    out[o] = b;
    return bf2f(b);  // the sums see the stored value, as the BN's own reduction would
  }
  __device__ __forceinline__ float second(int m, int n, float g) const {
    return g * ((bf2f(z[(long)m * ldo + n]) - mean[n]) * rstd[n]);
  }
  // the gg engine's 16-B epilogue (gemm_glds.h): 8 columns n..n+7 of row m, their g and g * xhat added
  // to the caller's per-thread column sums s1 / s2
  static constexpr bool kVec8 = true;
  __host__ __device__ bool vec8_ok() const {
    return ldo % 8 == 0 && (uintptr_t)out % 16 == 0 && (uintptr_t)y % 16 == 0 && (uintptr_t)add % 16 == 0 &&
           (uintptr_t)z % 16 == 0;
  }
  __device__ __forceinline__ void store8_bn(int m, int n, const float* v, float* s1, float* s2) const {
    const long o = (long)m * ldo + n;
    const bf16x8 zero = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    const bf16x8 av = add ? *(const bf16x8*)(add + o) : zero;
    const bf16x8 yv = y ? *(const bf16x8*)(y + o) : zero;
    const bf16x8 zv = *(const bf16x8*)(z + o);
    const f32x4 mu0 = *(const f32x4*)(mean + n), mu1 = *(const f32x4*)(mean + n + 4);
    const f32x4 rs0 = *(const f32x4*)(rstd + n), rs1 = *(const f32x4*)(rstd + n + 4);
    const float mu[8] = {mu0[0], mu0[1], mu0[2], mu0[3], mu1[0], mu1[1], mu1[2], mu1[3]};
    const float rs[8] = {rs0[0], rs0[1], rs0[2], rs0[3], rs1[0], rs1[1], rs1[2], rs1[3]};
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j];
      if (add) t += bf2f((uint16_t)av[j]);
      if (y) t *= act_grad_from_out(bf2f((uint16_t)yv[j]), act);
      q[j] = (short)f2bf(t);
      const float g = bf2f((uint16_t)q[j]);
      s1[j] += g;
      s2[j] = fmaf(g, (bf2f((uint16_t)zv[j]) - mu[j]) * rs[j], s2[j]);
    }
    *(bf16x8*)(out + o) = q;
  }
};

template <class EP, class = void>
struct has_bn2 { static constexpr bool value = false; };
template <class EP>
struct has_bn2<EP, decltype((void)EP::kBn2)> { static constexpr bool value = EP::kBn2; };

// Linear dgrad whose input came from a non-overlapping max-pool (exact windows): the epilogue IS
// the pool backward — each pooled-gradient element (row m, column n = (ph, pw, c)) is routed to
// its argmax position of the pool input (dropout mask regenerated, ReLU' of the pool input
// applied), the rest of the window gets zeros.  Removes the pool-backward launch and the dX
// round trip between them.  Floor windows: the last pooled row / column also zero-fills the
// remainder rows / columns of the pool input that no window covers (as maxpool_bwd8_k).
struct EpiPoolScatterBF16 {
  static constexpr bool kPre = true;  // two-phase: all gathers issued before any dX store
  bf16_raw* dx;                 // pool-input gradient [B][H][W][C]
  const unsigned char* am;      // argmax bytes [B][PH][PW][C]
  const bf16_raw* y;            // pooled output = this Linear's input [B][N] (ReLU' mask), or null
  int act;
  const unsigned long long* rng;
  unsigned salt;
  float p;                      // dropout probability of the pool (0: none)
  int N, C, PW, KH, KW, H, W;
  float* colsum;                // unused (kept for the epilogue interface)
  int PH;
  // phase 1: argmax byte | ReLU'(pooled value) << 8.  The pooled value is positive iff the window
  // max is (dropout only scales or zeroes it, and a zeroed element has no gradient anyway).
  __device__ __forceinline__ unsigned pre(int m, int n) const {
    const long o = (long)m * N + n;
    unsigned keep = 1u;
    if (y && act != ACT_NONE) {
      const unsigned short r = y[o];
      keep = (r & 0x8000u) == 0 && (r & 0x7fffu) != 0;
    }
    return (unsigned)am[o] | (keep << 8);
  }
  __device__ __forceinline__ float apply(int m, int n, float v, unsigned aux) const {
    const long o = (long)m * N + n;
    const int c = n % C, t = n / C;
    const int pw = t % PW, ph = t / PW;
    if (p > 0.f) v = uniform01(drop_key(rng, salt), (uint64_t)o) >= p ? v * (1.f / (1.f - p)) : 0.f;
    const int a = aux & 0xff;
    const float g = (aux >> 8) ? v : 0.f;
    bf16_raw* base = dx + (((long)m * H + ph * KH) * W + pw * KW) * C + c;
    const int eh = ph == PH - 1 ? H - ph * KH : KH, ew = pw == PW - 1 ? W - pw * KW : KW;
    const int ah = a / KW, aw = a - ah * KW;  // a = 0xFF (ReLU' == 0 from a fused conv-pool) matches no tap
    for (int qh = 0; qh < eh; ++qh)
      for (int qw = 0; qw < ew; ++qw) base[((long)qh * W + qw) * C] = f2bf(qh == ah && qw == aw ? g : 0.f);
    return v;
  }
};

// ----------------------------------------------------------------------------
// Main loop
// ----------------------------------------------------------------------------
// Body with explicit block coordinates (bx of gx tiles, by of gy K-splits) so several GEMMs can
// share one launch (mfma_gemm_pair_k); mfma_gemm_kernel passes the builtins.
template <int BM, int BN, int WAVES_M, bool A_KC, bool B_KC, class AL, class BL, class EP>
__device__ __forceinline__ void mfma_gemm_body(const AL& al, const BL& bl, const EP& ep, int M, int N, int K, int kps,
                                               float* rowsum_a, int bx, int gx, int by, int gy) {
  // rowsum_a (RC-A only): rowsum_a[m] += sum_k A[m][k] of the staged (masked) A
  // operand — in wgrad dW = dY^T X that is the bias gradient sum_b dY[b][m],
  // accumulated while the tiles pass through registers, by the tn == 0 blocks.
  constexpr int BK = GEMM_BK;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave tile must hold a 16x16 fragment");
  constexpr int A_CH = BM * BK / 8, B_CH = BN * BK / 8;  // 16-B chunks per tile
  constexpr int A_PT = (A_CH + 255) / 256, B_PT = (B_CH + 255) / 256;
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;

  __shared__ __attribute__((aligned(16))) bf16_raw smem[2 * (A_ELEMS + B_ELEMS)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  const int ntn = (N + BN - 1) / BN;
  const int bid = xcd_remap(bx, gx);
  const int tm = bid / ntn, tn = bid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = by * kps;
  const int kend = min(K, kbeg + kps);
  if (kbeg >= kend) return;
  const int nt = (kend - kbeg + BK - 1) / BK;

  bf16x8 ra[A_PT], rb[B_PT];
  const bool do_rs = !A_KC && rowsum_a != nullptr && tn == 0;
  float rs[A_PT][8];
#pragma unroll
  for (int i = 0; i < A_PT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[i][j] = 0.f;

  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < A_CH) {
        if (A_KC) {
          const int r = idx >> 3, c = idx & 7;
          ra[i] = al.load(m0 + r, k0 + 8 * c, M, kend);
        } else {
          const int cpr = BM / 8;
          const int kr = idx / cpr, c = idx - kr * cpr;
          ra[i] = al.load(k0 + kr, m0 + 8 * c, kend, M);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < B_CH) {
        if (B_KC) {
          const int r = idx >> 3, c = idx & 7;
          rb[i] = bl.load(n0 + r, k0 + 8 * c, N, kend);
        } else {
          const int cpr = BN / 8;
          const int kr = idx / cpr, c = idx - kr * cpr;
          rb[i] = bl.load(k0 + kr, n0 + 8 * c, kend, N);
        }
      }
    }
  };
  auto lstore = [&](int buf) {
    bf16_raw* sa = smem + buf * (A_ELEMS + B_ELEMS);
    bf16_raw* sb = sa + A_ELEMS;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < A_CH) {
        int off;
        if (A_KC) {
          const int r = idx >> 3, c = idx & 7;
          off = r * BK + 8 * (c ^ (r & 7));
        } else {
          const int cpr = BM / 8;
          const int kr = idx / cpr, c = idx - kr * cpr;
          off = kr * BM + 8 * (c ^ rc_swz(kr, cpr));
        }
        *(bf16x8*)(sa + off) = ra[i];
        if (!A_KC && do_rs)
#pragma unroll
          for (int j = 0; j < 8; ++j) rs[i][j] += bf2f((uint16_t)ra[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < B_CH) {
        int off;
        if (B_KC) {
          const int r = idx >> 3, c = idx & 7;
          off = r * BK + 8 * (c ^ (r & 7));
        } else {
          const int cpr = BN / 8;
          const int kr = idx / cpr, c = idx - kr * cpr;
          off = kr * BN + 8 * (c ^ rc_swz(kr, cpr));
        }
        *(bf16x8*)(sb + off) = rb[i];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // tr-read lane roles (T10): lane 4q+p of a 16-lane group addresses row q, cols 4p..4p+3
  const int tq = (lane & 15) >> 2, tp = lane & 3;

  auto frag_kc = [&](const bf16_raw* s, int row, int kk) -> bf16x8 {
    const int chunk = kk * 4 + fq;
    return *(const bf16x8*)(s + row * BK + 8 * (chunk ^ (row & 7)));
  };
  auto frag_rc = [&](const bf16_raw* s, int col0, int kk, int ROWS) -> bf16x8 {
    // rows of the LDS image are k, columns are m (or n); ROWS = BM or BN
    const int cpr = ROWS / 8;
    const int col = col0 + 4 * tp;
    const int k1 = kk * 32 + 8 * fq + tq;
    const int k2 = k1 + 4;
    const bf16_raw* p1 = s + k1 * ROWS + 8 * ((col >> 3) ^ rc_swz(k1, cpr)) + (col & 7);
    const bf16_raw* p2 = s + k2 * ROWS + 8 * ((col >> 3) ^ rc_swz(k2, cpr)) + (col & 7);
    bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p1));
    bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p2));
    return (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
  };

  gload(kbeg);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) gload(kbeg + (t + 1) * BK);
    const bf16_raw* sa = smem + cur * (A_ELEMS + B_ELEMS);
    const bf16_raw* sb = sa + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int rbase = wm * WTM + i * 16;
        af[i] = A_KC ? frag_kc(sa, rbase + fr, kk) : frag_rc(sa, rbase, kk, BM);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int cbase = wn * WTN + j * 16;
        bfr[j] = B_KC ? frag_kc(sb, cbase + fr, kk) : frag_rc(sb, cbase, kk, BN);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nt) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  if (!A_KC && do_rs) {
    // reduce the per-thread row sums over the k-rows of the RC image through LDS
    // (the staging buffers are free after the last barrier of the main loop)
    float* red = (float*)smem;  // [BK][BM] floats = 2*BK*BM*2 bytes <= smem size
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int idx = tid + 256 * i;
      if (idx < A_CH) {
        const int cpr = BM / 8;
        const int kr = idx / cpr, c = idx - kr * cpr;
#pragma unroll
        for (int j = 0; j < 8; ++j) red[kr * BM + 8 * c + j] = rs[i][j];
      }
    }
    __syncthreads();
    for (int m = tid; m < BM; m += 256) {
      float s = 0.f;
      for (int kr = 0; kr < BK; ++kr) s += red[kr * BM + m];
      if (m0 + m < M && s != 0.f) atomicAdd(rowsum_a + m0 + m, s);
    }
  }

  // epilogue: C/D map col = lane&15, row = (lane>>4)*4 + reg
  float cs[FN], cs2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { cs[j] = 0.f; cs2[j] = 0.f; }
  if constexpr (has_pre<EP>::value) {
    // gather-then-scatter epilogues: issue every gather first (the scatter stores may alias them
    // as far as the compiler knows, which would serialise one load latency per element)
    unsigned aux[FM][FN][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
          aux[i][j][r] = (m < M && n < N) ? ep.pre(m, n) : 0u;
        }
      }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
          if (m < M && n < N) cs[j] += ep.apply(m, n, acc[i][j][r], aux[i][j][r]);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
          if (m < M && n < N) {
            const float v = ep(m, n, acc[i][j][r]);
            cs[j] += v;
            if constexpr (has_bn2<EP>::value) cs2[j] += ep.second(m, n, v);
            else if constexpr (has_sq<EP>::value) cs2[j] = fmaf(v, v, cs2[j]);
          }
        }
      }
    }
  }
  if constexpr (!has_ticket<EP>::value) {
    if (ep.colsum) {
      // deterministic mode: the column-sum atomics of this launch's tiles in workgroup order (no
      // split-K there, so every tile of the launch reaches this point exactly once)
      const bool det = det_on();
      const unsigned dmy = (unsigned)(by * gx + bx), dtot = (unsigned)(gx * gy);
      if (WAVES_M > 1 && det) {
        // the WAVES_M waves of a column add to the same addresses: in deterministic mode they first meet
        // in LDS (fixed order), and only the wm == 0 waves issue the atomics
        float* red = (float*)smem;  // [WAVES_M][2][BN] (the staging tiles are free after the main loop)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float v = cs[j], q = cs2[j];
          v += __shfl_xor(v, 16, 64);
          v += __shfl_xor(v, 32, 64);
          q += __shfl_xor(q, 16, 64);
          q += __shfl_xor(q, 32, 64);
          if (fq == 0) {
            red[(wm * 2) * BN + wn * WTN + j * 16 + fr] = v;
            red[(wm * 2 + 1) * BN + wn * WTN + j * 16 + fr] = q;
          }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float v = 0.f, q = 0.f;
#pragma unroll
          for (int w = 0; w < WAVES_M; ++w) {
            v += red[(w * 2) * BN + wn * WTN + j * 16 + fr];
            q += red[(w * 2 + 1) * BN + wn * WTN + j * 16 + fr];
          }
          // lanes fr of quarter 0 of the wm == 0 waves hold the column totals below
          cs[j] = (wm == 0 && fq == 0) ? v : 0.f;
          cs2[j] = (wm == 0 && fq == 0) ? q : 0.f;
        }
      }
      if (det) det_turn_begin(DET_GEMM_COLSUM, dmy);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float v = cs[j];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int n = n0 + wn * WTN + j * 16 + fr;
        if (WAVES_M > 1 && det && wm != 0) continue;  // (their sums went through LDS above)
        if constexpr (has_sq<EP>::value) {
          float q = cs2[j];
          q += __shfl_xor(q, 16, 64);
          q += __shfl_xor(q, 32, 64);
          float* d = ep.colsum + (long)(bid % HOPSX_BN_NREP) * 2 * N;
          if (fq == 0 && n < N) {
            atomicAdd(d + n, v);
            atomicAdd(d + N + n, q);
          }
        } else {
          if (fq == 0 && n < N) atomicAdd(ep.colsum + n, v);
        }
      }
      if (det) det_turn_end(DET_GEMM_COLSUM, dmy, dtot);
    }
  } else {
    // ---- in-launch split-K finish (agent-scope release per slice, acquire in the last one)
    int* flag = (int*)smem;  // the staging array is free now; never a second __shared__ object
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(ep.fin.cnt + bid, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = (t == (unsigned)gy - 1) ? 1 : 0;
    }
    __syncthreads();
    if (flag[0] == 0) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ep.fin.cnt[bid] = 0u;
    }
    __syncthreads();
    const SplitFinish& f = ep.fin;
    const int c = tid % BN;  // BN divides 256: a thread keeps one column
    float csum = 0.f, csq = 0.f;
    for (int idx = tid; idx < BM * BN; idx += 256) {
      const int m = m0 + idx / BN, n = n0 + c;
      if (m >= M || n >= N) continue;
      float* wp = ep.out + (long)m * ep.ldo + n;
      float v = *wp;
      *wp = 0.f;
      if (f.epi == kEpiDActBF16) {
        if (f.aux) v *= act_grad_from_out(bf2f(f.aux[(long)m * f.ldaux + n]), f.act);
        if (f.add) v += bf2f(f.add[(long)m * f.ldo + n]);
        ((bf16_raw*)f.out)[(long)m * f.ldo + n] = f2bf(v);
      } else if (f.epi == kEpiBnStatsBF16) {
        const bf16_raw b = f2bf(v);  // statistics of the stored bf16 value, as EpiBnStatsBF16
        ((bf16_raw*)f.out)[(long)m * f.ldo + n] = b;
        v = bf2f(b);
        csq = fmaf(v, v, csq);
      } else {
        v = apply_act(v * f.alpha + (f.bias ? f.bias[n] : 0.f), f.act);
        if (f.epi == kEpiStoreBF16) {
          ((bf16_raw*)f.out)[(long)m * f.ldo + n] = f2bf(v);
        } else {
          float* o = (float*)f.out + (long)m * f.ldo + n;
          *o = (f.beta != 0.f) ? v + f.beta * *o : v;
        }
      }
      csum += v;
    }
    if (f.colsum) {
      float* red = (float*)smem;
      const bool sq = f.epi == kEpiBnStatsBF16;
      __syncthreads();
      red[tid] = csum;
      if (sq) red[256 + tid] = csq;
      __syncthreads();
      if (tid < BN && n0 + tid < N) {
        float t = 0.f, t2 = 0.f;
        for (int q = tid; q < 256; q += BN) {
          t += red[q];
          if (sq) t2 += red[256 + q];
        }
        if (sq) {
          float* d = f.colsum + (long)(bid % HOPSX_BN_NREP) * 2 * N;
          atomicAdd(d + n0 + tid, t);
          atomicAdd(d + N + n0 + tid, t2);
        } else {
          atomicAdd(f.colsum + n0 + tid, t);
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------
// Host-side config selection + launch
// ----------------------------------------------------------------------------
template <int BM, int BN, int WAVES_M, bool A_KC, bool B_KC, class AL, class BL, class EP>
__global__ __launch_bounds__(256) void mfma_gemm_kernel(const AL al, const BL bl, const EP ep, int M, int N,
                                                       int K, int kps, float* rowsum_a) {
  mfma_gemm_body<BM, BN, WAVES_M, A_KC, B_KC, AL, BL, EP>(al, bl, ep, M, N, K, kps, rowsum_a, blockIdx.x, gridDim.x,
                                                          blockIdx.y, gridDim.y);
}

struct GemmPlan {
  int cfg;    // 0: 128x128, 1: 64x64, 2: 32x32
  int split;  // split-K factor (only honoured for atomic epilogues)
  int kps;    // K per split (multiple of BK)
};

inline GemmPlan plan_gemm(long M, long N, long K, bool allow_split, int num_cu = 256) {
  GemmPlan p;
  if (hopsx_deterministic()) allow_split = false;  // one producer per output element
  const long t128 = ((M + 127) / 128) * ((N + 127) / 128);
  const long t64 = ((M + 63) / 64) * ((N + 63) / 64);
  // A/B knobs (host side, read once): HOPSX_GEMM_T64_MIN / _T128_MIN = the tile count below which a
  // non-split GEMM drops to the next smaller tile (fewer, bigger tiles leave CUs idle on small-M
  // convs); HOPSX_GEMM_SPLIT_CFG = tile config of the big-K split GEMMs (1: 64x64,
  // 0: 128x128 where M, N >= 128); HOPSX_GEMM_SPLIT_TARGET = workgroups per CU a split aims at.
  // default 2 x num_cu 64x64 tiles (two per CU) before a non-split GEMM uses them: vs the old floor
  // num_cu/2, ResNet-20 +6 %, ResNet-50 B=8 +18 %, B=64 +3 % (profiles/r2s7_gemm_plan_ab.txt,
  // r2s7_verify2_ab.txt); the old floor left half the CUs idle on small-M convs
  static const long t64_min = hopsx_env_int("HOPSX_GEMM_T64_MIN", 2L * num_cu);
  static const long t128_min = hopsx_env_int("HOPSX_GEMM_T128_MIN", num_cu);
  static const long split_cfg = hopsx_env_int("HOPSX_GEMM_SPLIT_CFG", 1);
  // 4 (was 2): ResNet-50 B=8 +1 %, with HOPSX_GG_MIN_WG=32 +1.7 %; B=64 / CIFAR flat (profiles/r5_gemm_knobs_b8_ab.txt)
  static const long split_target = hopsx_env_int("HOPSX_GEMM_SPLIT_TARGET", 4);
  const long t64_lim = t64_min >= 0 ? t64_min : num_cu / 2;
  if (M >= 128 && N >= 128 && t128 >= t128_min) p.cfg = 0;
  else if (M >= 48 && N >= 48 && t64 >= t64_lim) p.cfg = 1;
  else if (M > 32 && N > 32 && t64 >= 32 && !(t64_min >= 0 && t64 < t64_min)) p.cfg = 1;
  // split-K GEMMs (weight gradients, K = batch*pixels) get their parallelism from
  // the K split, so use the bigger tile: every operand element is then fetched by
  // fewer workgroups (64x64 halves the operand traffic of 32x32 tiles)
  else if (allow_split && M >= 48 && N >= 48 && K >= 8192)
    p.cfg = (split_cfg == 0 && M >= 128 && N >= 128) ? 0 : 1;
  else p.cfg = 2;
  const int bm = p.cfg == 0 ? 128 : (p.cfg == 1 ? 64 : 32);
  const long tiles = ((M + bm - 1) / bm) * ((N + bm - 1) / bm);
  p.split = 1;
  if (allow_split) {
    const long target = split_target * num_cu;
    if (tiles < target) {
      long s = (target + tiles - 1) / tiles;
      static const int minkt = [] {
        const char* e = std::getenv("HOPSX_SPLIT_MINKT");
        return e ? std::atoi(e) : 4;
      }();
      const long maxs = (K + minkt * GEMM_BK - 1) / (minkt * GEMM_BK);  // >= minkt k-tiles per split
      if (s > maxs) s = maxs;
      if (s < 1) s = 1;
      p.split = (int)s;
    }
  }
  long kps = (K + p.split - 1) / p.split;
  kps = ((kps + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.kps = (int)(kps > 0 ? kps : GEMM_BK);
  p.split = (int)((K + p.kps - 1) / p.kps);
  if (p.split < 1) p.split = 1;
  return p;
}

template <bool A_KC, bool B_KC, class AL, class BL, class EP>
inline void launch_gemm(const AL& al, const BL& bl, const EP& ep, int M, int N, int K, bool allow_split,
                        hipStream_t st, float* rowsum_a = nullptr) {
  if (M <= 0 || N <= 0) return;
  if (K <= 0) K = 1;  // degenerate: zero-length reduction still runs the epilogue
  GemmPlan p = plan_gemm(M, N, K, allow_split);
  const int bm = p.cfg == 0 ? 128 : (p.cfg == 1 ? 64 : 32);
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bm - 1) / bm);
  dim3 grid((unsigned)tiles, (unsigned)p.split);
  switch (p.cfg) {
    case 0:
      hipLaunchKernelGGL((mfma_gemm_kernel<128, 128, 2, A_KC, B_KC, AL, BL, EP>), grid, dim3(256), 0, st, al, bl,
                         ep, M, N, K, p.kps, rowsum_a);
      break;
    case 1:
      hipLaunchKernelGGL((mfma_gemm_kernel<64, 64, 2, A_KC, B_KC, AL, BL, EP>), grid, dim3(256), 0, st, al, bl, ep,
                         M, N, K, p.kps, rowsum_a);
      break;
    default:
      hipLaunchKernelGGL((mfma_gemm_kernel<32, 32, 2, A_KC, B_KC, AL, BL, EP>), grid, dim3(256), 0, st, al, bl, ep,
                         M, N, K, p.kps, rowsum_a);
      break;
  }
}

inline int is_vec_ok(const void* p, long ld) { return (ld % 8 == 0) && ((uintptr_t)p % 16 == 0); }

}  // namespace hopsx
