// The Chicago-taxi wide & deep training step, v2: bf16 MFMA on an LDS-resident model, with the
// wide table and every optimizer state on chip for the whole launch.
//
// Why v2 (widedeep_step.hip is v1, kept for data-parallel gradients and non-default shapes): v1 runs
// the deep GEMMs on the f32-input MFMA, which on gfx950 issues at 1/16 of the bf16 rate, so one
// CU needs ~9 us of pure MFMA time a step; its wide rows make four L2 round trips a step (gradient
// atomics, a claiming exchange, the FTRL stores, the next step's gather); and its 1024-thread
// layout spills ~600 B a lane.  The step is a dependent chain (4 forward layers, loss, 3 dX layers,
// the W0 update, the next step) of ~2.7 M MACs: spreading it over CUs would put a cross-CU
// hand-off (~1 us) on each link, so v2 keeps ONE workgroup and shortens the chain:
//
//   * mixed precision like the rest of the framework (bf16 operands, fp32 accumulation, fp32
//     master weights, fp32 optimizer state): activations, gradients and weights are bf16 images
//     in LDS, read as `v_mfma_f32_16x16x32_bf16` / `16x16x16` operands — row reads for the forward
//     and dX products, `ds_read_b64_tr_b16` transposed reads for dX's W operand and both dW
//     operands, so each tensor has ONE image.  Row strides are odd multiples of 16 elements: the
//     transposed reads of 8 rows land on 8 distinct bank groups.
//   * the forward pass and the dX chain of 16 examples depend only on those 16 rows: "tile waves"
//     0..2 each own one 16-row batch tile and run its whole forward (4 layers, logits, loss, the
//     logit gradient) with no barrier at all, then one dX layer per backward phase.  The weight
//     gradients sum over all rows, so "gradient waves" 3..7 compute them one phase behind the G
//     they read.  Five barriers a step: FWD, B3, B2, B1, B0.
//   * every deep parameter (weight or bias) is owned by the gradient-wave lane whose dW
//     accumulator holds its gradient (static tile -> wave map): fp32 weight + Adagrad state live in
//     that lane's registers for the whole launch and the update happens as the gradient leaves the
//     MFMA; the new bf16 image entry is written one phase later, once that layer's dX has read the
//     old weight.  Biases ride the GEMMs as a ones column of A (db = that column of dW) but are
//     applied in fp32 in the forward epilogue.  The logits layer (34 -> 1) is the dot product of
//     the last hidden tile with w4 in the forward wave; its backward is G4 = g w4 relu'.
//   * the wide (linear) part: the 6,287-row weight table lives in LDS (fp32).  Per step the tile waves
//     gather their examples' 13 rows (FWD) while the otherwise idle gradient waves find each entry's
//     leader — the first example of the batch with the same id in that column (the 13 columns' id
//     ranges are disjoint) — from an LDS id table; in B3 the gradient waves sum each leader's example
//     gradients in example order (no atomics: deterministic), and in B0 the leader applies FTRL-proximal
//     with (z, n) from a kernel-private float2 copy in memory (fetched in B3) and writes the new weight
//     back to the table.
//   * the launch loads / stores the deep parameters through an LDS staging copy of their arena span
//     (coalesced), so per-launch overhead stays small next to the 20-32 steps it runs.
//
// Numerics = a bf16 layer-by-layer training step with fp32 accumulation (the layerwise TrainStep
// path of this framework); tests/test_taxi_v2_gpu.py checks it against a bf16-emulating fp64
// reference of the same step.  HOPSX_TAXI_KERNEL=v1 selects the fp32 v1 kernel.
// Parity: the reference's TFX taxi trainer (README.md:99-112): DNNLinearCombinedClassifier,
// hidden [100, 70, 48, 34], FTRL on the wide part, Adagrad on the deep part, batch 40.
#include <cstdint>
#include <type_traits>

#include "common.h"
#include "optim_core.h"

namespace taxi2 {

constexpr int NT = 512;  // 8 waves: 2 per SIMD, 256 registers a lane for the owned optimizer state
constexpr int NW = NT / 64;
constexpr int NTW = 3;   // tile waves (batch tiles of 16 rows)
constexpr int BP = 48;   // batch rows (B <= 48)
constexpr int NWIDE = 13;
constexpr int WJ = 13;  // wide rows per thread
constexpr int MAXROWS = NT * WJ;
constexpr int D0 = 3, D1 = 100, D2 = 70, D3 = 48, D4 = 34;  // dense input + hidden widths (logits: 1)

constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
constexpr int pad32(int x) { return (x + 31) & ~31; }
// dW tile rounds a lane owns (the deep exchange payload's slots; = NSLOT below, checked there)
constexpr int NSLOT_X = cdiv(cdiv(D4, 16) * cdiv(D3 + 1, 16), NT / 64) + cdiv(cdiv(D3, 16) * cdiv(D2 + 1, 16), NT / 64) +
                        cdiv(cdiv(D2, 16) * cdiv(D1 + 1, 16), NT / 64) + 1;

// ---- LDS images (bf16 element offsets); strides are odd multiples of 16 elements
constexpr int SA0 = 16, SA1 = 144, SA2 = 112, SA3 = 80, SA4 = 48, SG = 112;
constexpr int OFF_A0 = 0;                        // [2][BP][SA0] (double-buffered input)
constexpr int OFF_A1 = OFF_A0 + 2 * BP * SA0;    // [BP][SA1]
constexpr int OFF_A2 = OFF_A1 + BP * SA1;
constexpr int OFF_A3 = OFF_A2 + BP * SA2;
constexpr int OFF_A4 = OFF_A3 + BP * SA3;
constexpr int OFF_GX = OFF_A4 + BP * SA4;        // G4, G2
constexpr int OFF_GY = OFF_GX + BP * SG;         // G3, G1
constexpr int W0R = 16 * cdiv(D1, 16);           // W0 rows (no dX for layer 0)
constexpr int W1R = pad32(D2), W2R = pad32(D3), W3R = pad32(D4);  // K of dX = rows
constexpr int OFF_W0 = OFF_GY + BP * SG;
constexpr int OFF_W1 = OFF_W0 + W0R * SA0;
constexpr int OFF_W2 = OFF_W1 + W1R * SA1;
constexpr int OFF_W3 = OFF_W2 + W2R * SA2;
constexpr int BF_END = OFF_W3 + W3R * SA3;
constexpr int BF_BYTES = BF_END * 2;
// ---- fp32 region (float offsets from BF_BYTES)
constexpr int F_B0 = 0, F_B1 = F_B0 + 16 * cdiv(D1, 16), F_B2 = F_B1 + 16 * cdiv(D2, 16),
              F_B3 = F_B2 + 16 * cdiv(D3, 16), F_W4 = F_B3 + 16 * cdiv(D4, 16), F_MISC = F_W4 + 48,
              F_RED = F_MISC + 16, F_DW4 = F_RED + 16, F_GV = F_DW4 + 3 * 48, F_IDT = F_GV + BP, F_LT = F_IDT + 16 * BP,
              F_GS = F_LT + 16 * BP, F_WTAB = F_GS + 16 * BP, F_VD = F_WTAB + MAXROWS, F_END = F_VD + 4;
constexpr int LDS_BYTES = BF_BYTES + F_END * 4;
constexpr int STAGE_MAX = LDS_BYTES / 4;  // floats of the deep arena span staged through LDS
static_assert(BF_BYTES % 16 == 0 && LDS_BYTES <= 160 * 1024, "taxi2 LDS budget");

// ---- data-parallel instantiation (DP = true; world 2..8 ranks, models/widedeep.py TaxiExchange) ----
// Each rank runs this one-workgroup step on ITS OWN batch.  The weight gradients are not applied as
// they leave the MFMAs: every owner lane PUSHES its dW accumulators (16 B a tile round) into every
// rank's uncached exchange buffer at slot [this rank] (system-scope write-through stores, off the
// critical path while the backward continues); the gradient waves push every wide entry's (id, summed
// gradient).  After the backward: drain, raise this rank's flag word in every peer's flag page, poll
// the own page.  Then each owner lane sums the W ranks' gradients of its elements in RANK ORDER and
// applies Adagrad in registers (so every replica computes bit-identical weights), and the wide rows
// touched by ANY rank get ONE FTRL update each with the rank-order sum of their gradients (an LDS
// gradient/tag table in the dead activation region, one pass per rank).  One cross-rank hop a step.
// Payloads are double-buffered by the parity of the global step epoch (a rank cannot push step s + 2
// before every peer raised step s + 1, which they do after reading step s).
constexpr int XMAX = 8;
constexpr int XD_BYTES = NSLOT_X * NT * 16;           // deep dW: [slot][thread] f32x4 (owner-lane-major)
constexpr int XL4_OFF = XD_BYTES;                      // logits-layer gradient: [64] floats (wave 7 lanes)
constexpr int XW_OFF = XL4_OFF + 64 * 4;               // wide entries: [13 col][BP] (id | -1, gradient)
constexpr int XPAY = XW_OFF + NWIDE * BP * 8;          // bytes per (parity, slot)
constexpr long X_BYTES = 2L * XMAX * XPAY;
constexpr int XF_WORDS = 64;                           // flag page: word r = rank r's step epoch

struct Args {
  float* master;
  bf16_raw* shadow;
  float* ada_s;
  float* ftrl_z;
  float* ftrl_n;
  const float* dense;     // [nbatch][B][3]
  const long long* cat;   // [nbatch][B][13] global one-hot ids
  const float* label;     // [nbatch][B]
  long long* cursor;      // batch of the first step (advanced by nsteps), or null
  float* loss;
  int* correct;
  float* step_ada;
  float* step_ftrl;
  unsigned long long* rng;
  unsigned long long* dbg;  // phase stamps or null
  float2* zn;               // [rows] FTRL (z, n) interleaved: kernel-private copy, one access per touched row
  int B, nbatch, nsteps, rows, rng_bumps;
  int ada_rsq;  // Adagrad as w -= lr g rsq(s): wd == 0 and eps below fp32 resolution of sqrt(s) (host-checked)
  long wide_off, deep_lo, deep_hi;
  long woff[5], boff[5];
  int rw[5], rb[5];  // woff / boff relative to deep_lo (staging-copy offsets)
  OptHP ada, ftrl;
  // data parallel (DP instantiation)
  int world, rank, loopback;   // loopback: one process plays every rank (the peers' buffers are its own)
  long long tmo;               // wall-clock ticks the exchange wait polls before it gives up
  unsigned* err;               // sticky error word (0 = ok)
  long long* xstep;            // global step counter: the exchange epoch base (advanced by nsteps)
  unsigned char* xbuf[XMAX];   // exchange buffers of ranks 0..world-1 (own at [rank])
  unsigned* xflag[XMAX];       // flag pages of ranks 0..world-1
};

typedef __attribute__((address_space(3))) bf16x4* lds4_t;

__device__ __forceinline__ bf16_raw f2b(float f) { return __builtin_bit_cast(bf16_raw, (__bf16)f); }
__device__ __forceinline__ float b2f(short v) { return __uint_as_float(((uint32_t)(uint16_t)v) << 16); }
__device__ __forceinline__ float rbf(float f) { return b2f((short)f2b(f)); }  // round to bf16
__device__ __forceinline__ f32x4 mma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// operand with K along the row: lane l takes row r0 + (l & 15), 8 (or 4) consecutive k
__device__ __forceinline__ bf16x8 rd8(const bf16_raw* img, int S, int r0, int k0, int lane) {
  return *(const bf16x8*)(img + (r0 + (lane & 15)) * S + k0 + 8 * (lane >> 4));
}
__device__ __forceinline__ bf16x4 rd4(const bf16_raw* img, int S, int r0, int k0, int lane) {
  return *(const bf16x4*)(img + (r0 + (lane & 15)) * S + k0 + 4 * (lane >> 4));
}
// operand with K down the rows (T10 transposed read): lane l gets column c0 + (l & 15) of rows
// k0 + 4 (l >> 4) + j (x16) or k0 + 8 (l >> 4) + j (x32).  EXEC must be full: never call under a
// lane-dependent branch.
__device__ __forceinline__ bf16x4 tr4(const bf16_raw* img, int S, int k0, int c0, int lane) {
  const int i = lane & 15;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t)(img + (k0 + 4 * (lane >> 4) + (i >> 2)) * S + c0 + 4 * (i & 3)));
}
__device__ __forceinline__ bf16x8 tr8(const bf16_raw* img, int S, int k0, int c0, int lane) {
  const int i = lane & 15;
  const bf16_raw* p = img + (k0 + 8 * (lane >> 4) + (i >> 2)) * S + c0 + 4 * (i & 3);
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t)p);
  const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t)(p + 4 * S));
  return (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
}
__device__ __forceinline__ void st4(bf16_raw* p, float a, float b, float c, float d) {
  *(bf16x4*)p = (bf16x4){(short)f2b(a), (short)f2b(b), (short)f2b(c), (short)f2b(d)};
}
__device__ __forceinline__ float sel(bool c, float a, float b) { return c ? a : b; }

// Workgroup barrier that waits only for LDS traffic: the next batch's loads stay in flight across
// it (a __syncthreads() would drain them at every phase)
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// keeps the compiler from moving LDS accesses across it (this wave's own write -> read order)
__device__ __forceinline__ void fence_c() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ float adagrad(float w, float g, float& s, const OptHP& h) {
  g = fmaf(h.wd, w, g);
  s = fmaf(g, g, s);
  return w - h.lr * g * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(s) + h.a);
}
// the same update when wd == 0 and eps is below the fp32 resolution of sqrt(s) (the accumulator never
// drops below its initial value): one transcendental instead of two, 5 VALU an element
__device__ __forceinline__ float adagrad_rsq(float w, float g, float& s, float nlr) {
  s = fmaf(g, g, s);
  return fmaf(nlr * g, __builtin_amdgcn_rsqf(s), w);
}

// An opaque copy of x: the LDS addresses of a phase's tasks derive from it, so the compiler recomputes
// them in the phase instead of hoisting ~200 loop-invariant addresses out of the step loop (which
// spilled them to scratch)
__device__ __forceinline__ int fresh(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ int fresh_s(int x) {  // (the same for wave-uniform values, in SGPRs)
  asm volatile("" : "+s"(x));
  return x;
}

__device__ __forceinline__ void stamp(const Args& a, int slot) {
  if (a.dbg && threadIdx.x == 0) a.dbg[slot] = wall_clock64();
}
// (HOPSX_PHASE_DBG) the shader clock next to the 100 MHz wall clock, for the clock rate of a launch
__device__ __forceinline__ void stamp_clk(const Args& a, int slot) {
  if (a.dbg && threadIdx.x == 0) a.dbg[slot] = __builtin_amdgcn_s_memtime();
}
// (HOPSX_PHASE_DBG) a stamp from lane 0 of wave w: tile wave 0 / gradient wave 3 inside a phase
__device__ __forceinline__ void stampw(const Args& a, int slot, int w) {
  if (a.dbg && threadIdx.x == 64 * w) a.dbg[slot] = wall_clock64();
}

// ------------------------------------------------------------------------------- layer geometry
// layer l: IN -> OUT, A_l image (OFFA, SA), W_l image (OFFW, stride SA), output image (OFFZ, SZ),
// fp32 bias at FB.  KF = forward K (x16 for layer 0).
template <int L_, int IN_, int OUT_, int OFFA_, int SA_, int OFFW_, int OFFZ_, int SZ_, int FB_>
struct Layer {
  static constexpr int L = L_, IN = IN_, OUT = OUT_, OFFA = OFFA_, SA = SA_, OFFW = OFFW_, OFFZ = OFFZ_,
                       SZ = SZ_, FB = FB_;
  static constexpr bool X16 = IN_ < 16;
  static constexpr int KF = X16 ? 16 : pad32(IN_ + 1);
  static constexpr int OT = cdiv(OUT_, 16);       // output-feature tiles
  static constexpr int ITW = cdiv(IN_ + 1, 16);   // dW input tiles (bias column included)
  static constexpr int ITX = cdiv(IN_, 16);       // dX input tiles
  static constexpr int KX = pad32(OUT_);          // dX K (= W image rows)
  static constexpr int NDW = OT * ITW;
  static_assert(KF <= SA_ && 16 * ITW <= SA_, "layer image width");
};
using L0 = Layer<0, D0, D1, OFF_A0, SA0, OFF_W0, OFF_A1, SA1, F_B0>;
using L1 = Layer<1, D1, D2, OFF_A1, SA1, OFF_W1, OFF_A2, SA2, F_B1>;
using L2 = Layer<2, D2, D3, OFF_A2, SA2, OFF_W2, OFF_A3, SA3, F_B2>;
using L3 = Layer<3, D3, D4, OFF_A3, SA3, OFF_W3, OFF_A4, SA4, F_B3>;
static_assert(L1::KX <= W1R && L2::KX <= W2R && L3::KX <= W3R && 16 * L0::OT <= W0R, "W image rows");
constexpr int NDW4 = cdiv(D4 + 1, 16);  // logits layer dW tiles (output column 0)

// dW tiles -> waves: tile t of a phase goes to the wave w with (w + 5) % 8 == t % 8, round t / 8, so the
// tile waves (busy with dX) get the lighter share of each phase; dW0 (7 tiles): waves 0..6, one each.
// The logits layer's 35 gradients are VALU row sums in the tile waves (FWD), owned by wave 7's lanes.
constexpr int R3 = cdiv(L3::NDW, NW), R2 = cdiv(L2::NDW, NW), R1 = cdiv(L1::NDW, NW);
static_assert(L0::NDW < NW && NW == 8, "tile map");
constexpr int S3 = 0, S2 = S3 + R3, S1 = S2 + R2, S0 = S1 + R1, NSLOT = S0 + 1;
static_assert(NSLOT == NSLOT_X, "exchange payload slots");

// ---- cross-rank exchange primitives (DP): system-scope (sc0 sc1) buffer stores / loads on the uncached
// exchange buffers, system-scope relaxed flag words (the persistent MNIST step's hand-off form)
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));
typedef unsigned __attribute__((address_space(1))) gu32_t;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xrsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void xst16(const void* base, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), xrsrc(base), off, 0, 17);
}
__device__ __forceinline__ void xst8(const void* base, int off, int a, float b) {
  __builtin_amdgcn_raw_buffer_store_b64((v2i_t){a, __float_as_int(b)}, xrsrc(base), off, 0, 17);
}
__device__ __forceinline__ void xst4(const void* base, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), xrsrc(base), off, 0, 17);
}
__device__ __forceinline__ f32x4 xld16(const void* base, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrsrc(base), off, 0, 17));
}
__device__ __forceinline__ v2i_t xld8(const void* base, int off) {
  return __builtin_amdgcn_raw_buffer_load_b64(xrsrc(base), off, 0, 17);
}
__device__ __forceinline__ float xld4(const void* base, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrsrc(base), off, 0, 17));
}
__device__ __forceinline__ int perm8(int wave) { return (wave + 5) & 7; }

struct Own {
  float w[NSLOT][4], s[NSLOT][4];
  float w4, s4;  // (wave 7, lanes 0..34) logits weight / bias and its Adagrad state
};

// dW tile t of layer Ly: i-tile t / OT, o-tile t % OT (element r: i = i0 + 4 (lane >> 4) + r, o = o0 + lane & 15)
template <class Ly>
__device__ __forceinline__ void dw_coords(int t, int lane, int& i, int& o) {
  i = (t / Ly::OT) * 16 + 4 * (lane >> 4);
  o = (t % Ly::OT) * 16 + (lane & 15);
}

// staging-copy offset (arena index - deep_lo) of element (i, o) of layer Ly's dW tile, or -1 (padding)
template <class Ly, class AR>
__device__ __forceinline__ int pidx(const AR& a, int i, int o) {
  if (o >= Ly::OUT || i > Ly::IN) return -1;
  return i == Ly::IN ? a.rb[Ly::L] + o : a.rw[Ly::L] + o * Ly::IN + i;
}
template <class AR>
__device__ __forceinline__ int pidx4(const AR& a, int i, int o) {  // logits layer
  if (o != 0 || i > D4) return -1;
  return i == D4 ? a.rb[4] : a.rw[4] + i;
}

// owned values <-> the LDS staging copy of the deep arena span (write: w or s of the slot)
template <class Ly, class AR>
__device__ __forceinline__ void own_get(const AR& a, const float* stage, int t, int lane, float (&v)[4]) {
  int i, o;
  dw_coords<Ly>(t, lane, i, o);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int x = pidx<Ly, AR>(a, i + r, o);
    v[r] = x >= 0 ? stage[x] : 0.f;
  }
}
template <class Ly, class AR>
__device__ __forceinline__ void own_put(const AR& a, float* stage, int t, int lane, const float (&v)[4]) {
  int i, o;
  dw_coords<Ly>(t, lane, i, o);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int x = pidx<Ly, AR>(a, i + r, o);
    if (x >= 0) stage[x] = v[r];
  }
}
// put owned elements into the bf16 W image (4 consecutive i of row o) and the fp32 bias array
template <class Ly>
__device__ __forceinline__ void put_w(bf16_raw* Lb, float* LF, int t, int lane, const float (&w)[4]) {
  int i, o;
  dw_coords<Ly>(t, lane, i, o);
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = sel((o < Ly::OUT) & (i + r < Ly::IN), w[r], 0.f);
  st4(Lb + Ly::OFFW + o * Ly::SA + i, v[0], v[1], v[2], v[3]);
  // the bias element (i + r == IN) can only be register IN % 4 (i is a multiple of 4)
  constexpr int rb = Ly::IN % 4;
  if ((o < Ly::OUT) & (i + rb == Ly::IN)) LF[Ly::FB + o] = w[rb];
}
// ---- dW: the R rounds of this wave in a phase, tiles t = p + 8 j (p = perm8(wave)), x16 MFMAs over the 48
// batch rows, Adagrad on the owned elements as the gradient leaves the accumulator (branch-free; a round
// past the layer's tile count runs a clamped dummy tile whose update is discarded).  Operands are
// double-buffered: the next round's transposed reads are in flight during this round's MFMAs (fence_c
// keeps the compiler from hoisting every round's reads at once, which would not fit the registers).
struct DwOps {
  bf16x4 a[BP / 16], g[BP / 16];
};
template <class Ly>
__device__ __forceinline__ DwOps dw_load(const bf16_raw* Aimg, const bf16_raw* G, int t, int lane) {
  t = t < Ly::NDW ? t : Ly::NDW - 1;
  const int i0 = (t / Ly::OT) * 16, o0 = (t % Ly::OT) * 16;
  DwOps d;
#pragma unroll
  for (int k = 0; k < BP / 16; ++k) {
    d.a[k] = tr4(Aimg, Ly::SA, 16 * k, i0, lane);
    d.g[k] = tr4(G, SG, 16 * k, o0, lane);
  }
  return d;
}
// (DP) this lane's dW accumulator of exchange slot `slot` into every rank's buffer at [parity][this rank]
__device__ __forceinline__ void xpush_dw(int slot, int par, f32x4 acc);
template <class Ly, int R, bool RSQ, bool DP = false>
__device__ __forceinline__ void dw_seq(const bf16_raw* Aimg, const bf16_raw* G, int p, int lane, float (*w)[4],
                                       float (*s)[4], const OptHP& h, int sbase = 0, int par = 0) {
  // padding elements (o >= OUT, i > IN) and a dummy round update registers nothing ever reads (put_w and
  // the write-back skip them), so no validity selects here
  DwOps cur = dw_load<Ly>(Aimg, G, p, lane);
  const float nlr = -h.lr;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int t = p + 8 * j;
    DwOps nxt = cur;
    if (j + 1 < R) nxt = dw_load<Ly>(Aimg, G, t + 8, lane);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < BP / 16; ++k) acc = mma16(cur.a[k], cur.g[k], acc);
    if constexpr (DP) {
      // the update waits for every rank's gradient (apply phase): push this one (a dummy round owns nothing)
      if (t < Ly::NDW) xpush_dw(sbase + j, par, acc);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (RSQ) w[j][r] = adagrad_rsq(w[j][r], acc[r] * h.gscale, s[j][r], nlr);
        else w[j][r] = adagrad(w[j][r], acc[r] * h.gscale, s[j][r], h);
      }
    }
    cur = nxt;
    fence_c();
  }
}
// the R rounds' images (a uniform branch per round: an out-of-range round owns nothing)
template <class Ly, int R>
__device__ __forceinline__ void put_seq(bf16_raw* Lb, float* LF, int p, int lane, float (*w)[4]) {
#pragma unroll
  for (int j = 0; j < R; ++j)
    if (p + 8 * j < Ly::NDW) put_w<Ly>(Lb, LF, p + 8 * j, lane, w[j]);
}

// ---- dX for batch tile b0 of layer Ly: dX^T[i][b] = sum_o W[o][i] G[b][o]; G_l[b][i] = dX relu'(A_l[b][i])
template <class Ly>
__device__ __forceinline__ void dx_tile(bf16_raw* Lb, const bf16_raw* G, bf16_raw* Gout, int b0, int lane) {
  constexpr int NK = Ly::KX / 32;
  bf16x8 gop[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) gop[k] = rd8(G, SG, b0, 32 * k, lane);
  const int b = b0 + (lane & 15);
  bf16x8 cur[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) cur[k] = tr8(Lb + Ly::OFFW, Ly::SA, 32 * k, 0, lane);
#pragma unroll
  for (int it = 0; it < Ly::ITX; ++it) {
    bf16x8 nxt[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) nxt[k] = it + 1 < Ly::ITX ? tr8(Lb + Ly::OFFW, Ly::SA, 32 * k, 16 * (it + 1), lane) : cur[k];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NK; ++k) acc = mma32(cur[k], gop[k], acc);
    const int i = 16 * it + 4 * (lane >> 4);
    const bf16x4 av = *(const bf16x4*)(Lb + Ly::OFFA + b * Ly::SA + i);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = sel(b2f(av[r]) > 0.f, acc[r], 0.f);  // (cols >= IN: A is 0 or the
    // ones column, whose dX is 0 since W's column IN is 0 in the image)
    st4(Gout + b * SG + i, v[0], v[1], v[2], v[3]);
#pragma unroll
    for (int k = 0; k < NK; ++k) cur[k] = nxt[k];
    fence_c();
  }
}

// ---- forward of layer Ly for batch tile b0: Z^T[o][b] = sum_k W[o][k] A[b][k] + bias[o], relu ->
// A_{l+1} rows b0...  No masks: W rows >= OUT are 0 and the fp32 bias array holds 1 at OUT (the ones
// column the next layer's db needs) and -1e30 beyond (relu -> 0); rows >= B hold finite garbage that
// only ever meets zero gradient rows (g_b = 0 for b >= B).  KEEP: also returns the activations.
template <class Ly, bool KEEP>
__device__ __forceinline__ void fwd_tile(bf16_raw* Lb, const float* LF, const bf16_raw* Ain, int b0, int lane, int B,
                                         float (*out)[4]) {
  constexpr int NK = Ly::X16 ? 1 : Ly::KF / 32;
  const int b = b0 + (lane & 15);
  if constexpr (Ly::X16) {
    const bf16x4 aop = rd4(Ain, Ly::SA, b0, 0, lane);
    bf16x4 w[Ly::OT];
#pragma unroll
    for (int ot = 0; ot < Ly::OT; ++ot) w[ot] = rd4(Lb + Ly::OFFW, Ly::SA, 16 * ot, 0, lane);
#pragma unroll
    for (int ot = 0; ot < Ly::OT; ++ot) {
      const f32x4 acc = mma16(w[ot], aop, (f32x4){0.f, 0.f, 0.f, 0.f});
      const int o = 16 * ot + 4 * (lane >> 4);
      const f32x4 bias = *(const f32x4*)(LF + Ly::FB + o);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[r] + bias[r], 0.f);
      st4(Lb + Ly::OFFZ + b * Ly::SZ + o, v[0], v[1], v[2], v[3]);
    }
  } else {
    bf16x8 aop[NK], cur[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      aop[k] = rd8(Ain, Ly::SA, b0, 32 * k, lane);
      cur[k] = rd8(Lb + Ly::OFFW, Ly::SA, 0, 32 * k, lane);
    }
#pragma unroll
    for (int ot = 0; ot < Ly::OT; ++ot) {
      bf16x8 nxt[NK];
#pragma unroll
      for (int k = 0; k < NK; ++k) nxt[k] = ot + 1 < Ly::OT ? rd8(Lb + Ly::OFFW, Ly::SA, 16 * (ot + 1), 32 * k, lane) : cur[k];
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NK; ++k) acc = mma32(cur[k], aop[k], acc);
      const int o = 16 * ot + 4 * (lane >> 4);
      const f32x4 bias = *(const f32x4*)(LF + Ly::FB + o);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[r] + bias[r], 0.f);
      st4(Lb + Ly::OFFZ + b * Ly::SZ + o, v[0], v[1], v[2], v[3]);
      if constexpr (KEEP) {
#pragma unroll
        for (int r = 0; r < 4; ++r) out[ot][r] = v[r];
      }
#pragma unroll
      for (int k = 0; k < NK; ++k) cur[k] = nxt[k];
      fence_c();
    }
  }
}

// the kernel's arguments read where used, through an opaque copy of the kernarg pointer (held in
// SGPRs across the step loop they spilled).  The pointer stays in the constant address space: the
// reads are scalar loads (a generic pointer made them flat vector loads, each a memory round trip
// that also waited for every outstanding store)
typedef const __attribute__((address_space(4))) Args* kargs_t;
__device__ __forceinline__ kargs_t cold_p() {
  kargs_t p = (kargs_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
#define COLD (*cold_p())

__device__ __forceinline__ void xpush_dw(int slot, int par, f32x4 acc) {
  const auto& C = COLD;
  const int off = (slot * NT + (int)threadIdx.x) * 16;
  for (int r = 0; r < C.world; ++r) {
    const int sl = C.loopback ? r : C.rank;
    xst16(C.xbuf[r] + (long)(par * XMAX + sl) * XPAY, off, acc);
  }
}

template <bool GET, bool PASS_S>
__device__ __forceinline__ void own_stage(float* stage, Own& own, int wave, int lane) {
  const auto& C = COLD;
  auto& v = PASS_S ? own.s : own.w;
  const int p = perm8(wave);
#pragma unroll
  for (int j = 0; j < R3; ++j)
    if (p + 8 * j < L3::NDW) {
      if (GET) own_get<L3>(C, stage, p + 8 * j, lane, v[S3 + j]);
      else own_put<L3>(C, stage, p + 8 * j, lane, v[S3 + j]);
    }
#pragma unroll
  for (int j = 0; j < R2; ++j)
    if (p + 8 * j < L2::NDW) {
      if (GET) own_get<L2>(C, stage, p + 8 * j, lane, v[S2 + j]);
      else own_put<L2>(C, stage, p + 8 * j, lane, v[S2 + j]);
    }
#pragma unroll
  for (int j = 0; j < R1; ++j)
    if (p + 8 * j < L1::NDW) {
      if (GET) own_get<L1>(C, stage, p + 8 * j, lane, v[S1 + j]);
      else own_put<L1>(C, stage, p + 8 * j, lane, v[S1 + j]);
    }
  if (wave < L0::NDW) {
    if (GET) own_get<L0>(C, stage, wave, lane, v[S0]);
    else own_put<L0>(C, stage, wave, lane, v[S0]);
  }
  if (wave == NW - 1 && lane <= D4) {  // logits layer: lane i < 34 weight i, lane 34 the bias
    const int x = lane < D4 ? C.rw[4] + lane : C.rb[4];
    float& o = PASS_S ? own.s4 : own.w4;
    if (GET) o = stage[x];
    else stage[x] = o;
  }
}

// dst[0..n) = src[0..n) into LDS, 8 loads of a thread in flight at once (a plain strided loop waits
// for each load before the next: ~25 round trips for the deep span); 16-byte loads when src is aligned
__device__ __forceinline__ void gather_in(float* dst, const float* src, int n, int tid) {
  constexpr int PER = 8;
  if (((uintptr_t)src & 15) == 0) {
    const int n4 = n >> 2;
    for (int base = 0; base < n4; base += NT * PER) {
      f32x4 v[PER];  // (native vectors: an array of HIP's float4 struct stays in scratch)
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int e = base + tid + NT * k;
        v[k] = ((const f32x4*)src)[e < n4 ? e : 0];
      }
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (base + tid + NT * k < n4) ((f32x4*)dst)[base + tid + NT * k] = v[k];
    }
    for (int e = 4 * n4 + tid; e < n; e += NT) dst[e] = src[e];
    return;
  }
  for (int base = 0; base < n; base += NT * PER) {
    float v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = base + tid + NT * k;
      v[k] = e < n ? src[e] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (base + tid + NT * k < n) dst[base + tid + NT * k] = v[k];
  }
}
constexpr unsigned SENT = 0xFFFFFFFFu;  // staging sentinel (a NaN no owner writes): "not owned, keep"

// OUT a multiple of 16: no epilogue tile reaches the ones column (the next layer's bias input), which is
// then constant — written at the launch start (and, data parallel, again after each step's apply phase,
// whose gradient table borrows the activation images)
__device__ __forceinline__ void ones_columns(bf16_raw* Lb, int B, int tid) {
  if (tid < B) {
    if (D1 % 16 == 0) Lb[OFF_A1 + tid * SA1 + D1] = f2b(1.f);
    if (D2 % 16 == 0) Lb[OFF_A2 + tid * SA2 + D2] = f2b(1.f);
    if (D3 % 16 == 0) Lb[OFF_A3 + tid * SA3 + D3] = f2b(1.f);
    if (D4 % 16 == 0) Lb[OFF_A4 + tid * SA4 + D4] = f2b(1.f);
  }
}

// (DP) the step's exchange: drain this wave's pushes, barrier (every payload store of the workgroup has
// completed at the system coherence point: the release for them), raise this rank's flag word in every
// peer's page, then wave 0 polls the own page until every peer's word has reached `epoch` (wrap-safe),
// bounded by the wall clock and the sticky error word.  Returns the verdict to the whole workgroup.
__device__ __forceinline__ bool exchange_step(const Args& A, long long epoch64, int step, unsigned char* lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const auto& C = COLD;
  const bool last = step + 1 == C.nsteps;
  if (last) stamp(A, 31);
  const unsigned ep = (unsigned)epoch64;
  volatile int* verdict = (volatile int*)(lds + BF_BYTES + F_VD * 4);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (lane < C.world && lane != C.rank)
      __hip_atomic_store((gu32_t*)(C.xflag[lane] + (C.loopback ? lane : C.rank)), ep, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* page = C.xflag[C.rank];
    int good = 1;
    const long long t0 = wall_clock64();
    for (unsigned spins = 0;; ++spins) {
      const bool peer = lane < C.world && lane != C.rank;
      const int ok = !peer || (int)(__hip_atomic_load((gu32_t*)(page + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - ep) >= 0;
      if (__all(ok)) break;
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32_t*)C.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u) {
        good = 0;
        break;
      }
      if ((spins & 15u) == 15u && wall_clock64() - t0 > C.tmo) {
        if (lane == 0) atomicCAS(C.err, 0u, 0x80000000u | ((unsigned)step & 0xFFFFFFu));
        good = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) *verdict = good;
  }
  __syncthreads();
  if (last) stamp(A, 25);
  return *verdict != 0;
}
static_assert(MAXROWS * 4 <= (OFF_W0 - OFF_A1) * 2, "DP wide gradient table fits the activation images");

// (DP) owner lanes: the rank-order sum of every rank's dW for each owned element, Adagrad in registers, the
// new W images / biases / logits weights; then the wide rows: the rank-order sum of every rank's entry
// gradients per distinct id (gradient + first-rank tag tables in the activation images, dead until the next
// forward), and ONE FTRL update per id touched by any rank, by the lane holding its first occurrence.
// (DP) is exchange slot S (a dW tile round) owned by this wave?  S -> (layer, round j): S3.. L3, S2.. L2,
// S1.. L1, S0 L0 (p = perm8(wave); L0: waves 0..6 own one tile each)
template <int S>
__device__ __forceinline__ bool slot_owned(int p, int wave) {
  if constexpr (S < S2) return p + 8 * (S - S3) < L3::NDW;
  else if constexpr (S < S1) return p + 8 * (S - S2) < L2::NDW;
  else if constexpr (S < S0) return p + 8 * (S - S1) < L1::NDW;
  else return wave < L0::NDW;
}
// (DP) the deep apply streams this lane's gradients of every rank from the uncached exchange buffer, 4
// 16-B loads a unit (latency-bound: the next unit's loads are in flight while one is summed):
//   NR = 8 (3..8 ranks): unit U = slot U / 2 from rank group U % 2 (ranks 4g .. 4g + 3);
//   NR = 2 (2 ranks):    unit U = slots 2U and 2U + 1 from both ranks — half the units, half the trips.
constexpr int XG = 4;
static_assert(2 * XG == XMAX && NSLOT % 2 == 0, "unit geometry");
template <int NR>
constexpr int n_units() { return NR == 2 ? NSLOT / 2 : 2 * NSLOT; }
template <int NR, int U>
__device__ __forceinline__ void load_unit(f32x4 (&v)[XG], const unsigned char* X, int W, int tid, int p, int wave) {
  if constexpr (NR == 2) {
#pragma unroll
    for (int q = 0; q < XG; ++q) {
      constexpr int S0_ = 2 * U;
      const int S = S0_ + q / 2, r = q % 2;
      const bool on = (q / 2 ? slot_owned<2 * U + 1>(p, wave) : slot_owned<2 * U>(p, wave)) && r < W;
      v[q] = on ? xld16(X + (long)r * XPAY, (S * NT + tid) * 16) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  } else {
    constexpr int S = U / 2, G = U % 2;
    const bool on = slot_owned<S>(p, wave) && G * XG < W;
#pragma unroll
    for (int r = 0; r < XG; ++r)
      v[r] = on && G * XG + r < W ? xld16(X + (long)(G * XG + r) * XPAY, (S * NT + tid) * 16) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
}
template <int S, bool RSQ>
__device__ __forceinline__ void adagrad_slot(Own& own, const f32x4& g, const OptHP& h) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if constexpr (RSQ) own.w[S][e] = adagrad_rsq(own.w[S][e], g[e] * h.gscale, own.s[S][e], -h.lr);
    else own.w[S][e] = adagrad(own.w[S][e], g[e] * h.gscale, own.s[S][e], h);
  }
}
template <int NR, int U, bool RSQ>
__device__ __forceinline__ void sum_unit(Own& own, f32x4& g, const f32x4 (&v)[XG], int W, int p, int wave,
                                         const OptHP& h) {
  if constexpr (NR == 2) {  // both ranks of two slots: rank order v0 + v1
    if (slot_owned<2 * U>(p, wave)) adagrad_slot<2 * U, RSQ>(own, v[0] + v[1], h);
    if (slot_owned<2 * U + 1>(p, wave)) adagrad_slot<2 * U + 1, RSQ>(own, v[2] + v[3], h);
  } else {
    constexpr int S = U / 2, G = U % 2;
    if (!(slot_owned<S>(p, wave) && G * XG < W)) return;
    // rank order: ((v0 + v1) + v2) + ... across both groups
#pragma unroll
    for (int r = 0; r < XG; ++r)
      if (G * XG + r < W) g = (G == 0 && r == 0) ? v[r] : g + v[r];
    if (G == 1 || W <= XG) adagrad_slot<S, RSQ>(own, g, h);  // the slot's last group: every rank is in g
  }
}
// the units software-pipelined: unit U + 1's loads are in flight while unit U is summed and applied
template <int NR, int U, bool RSQ>
__device__ __forceinline__ void apply_units(Own& own, f32x4& g, f32x4 (&cur)[XG], const unsigned char* X, int W,
                                            int tid, int p, int wave, const OptHP& h) {
  constexpr int NU = n_units<NR>();
  if constexpr (U < NU) {
    f32x4 nxt[XG];
    if constexpr (U + 1 < NU) load_unit<NR, U + 1>(nxt, X, W, tid, p, wave);
    sum_unit<NR, U, RSQ>(own, g, cur, W, p, wave, h);
    if constexpr (U + 1 < NU) {
#pragma unroll
      for (int r = 0; r < XG; ++r) cur[r] = nxt[r];
    }
    fence_c();
    apply_units<NR, U + 1, RSQ>(own, g, cur, X, W, tid, p, wave, h);
  }
}

template <bool RSQ, int NR>
__device__ __forceinline__ void apply_dp(Own& own, unsigned char* lds, int par, int wave, int lane, int tid) {
  const auto& C = COLD;
  bf16_raw* const Lb = (bf16_raw*)lds;
  float* const LF = (float*)(lds + BF_BYTES);
  const int W = C.world;
  constexpr int XR = NR == 2 ? 2 : XMAX;  // ranks the wide-entry registers cover
  const unsigned char* X = C.xbuf[C.rank] + (long)par * XMAX * XPAY;  // own buffer, slots 0..W-1
  // ---- wide entries of every rank (this thread: entries tid, tid + 512 of each rank): loads issued first,
  // in flight during the deep apply
  constexpr int NE = NWIDE * BP;
  int eid[XR][2];
  float eg[XR][2];
#pragma unroll
  for (int r = 0; r < XR; ++r)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + NT * k;
      v2i_t q = (v2i_t){-1, 0};
      if (r < W && e < NE) q = xld8(X + (long)r * XPAY, XW_OFF + e * 8);
      eid[r][k] = q[0];
      eg[r][k] = __int_as_float(q[1]);
    }
  // ---- deep: rank-order sums + Adagrad, software-pipelined over the owned slots
  {
    const OptHP ha = {C.ada.lr, C.ada.gscale, C.ada.wd, C.ada.a, C.ada.b, C.ada.c, C.ada.d, C.ada.e};
    const int p = perm8(wave);
    f32x4 cur[XG], g = {0.f, 0.f, 0.f, 0.f};
    load_unit<NR, 0>(cur, X, W, tid, p, wave);
    apply_units<NR, 0, RSQ>(own, g, cur, X, W, tid, p, wave, ha);
    if (C.dbg && tid == 0) C.dbg[28] = wall_clock64();  // (HOPSX_PHASE_DBG: every step overwrites; the last stays)
    if (wave == NW - 1 && lane <= D4) {
      float g = 0.f;
      for (int r = 0; r < W; ++r) g += xld4(X + (long)r * XPAY, XL4_OFF + lane * 4);
      own.w4 = RSQ ? adagrad_rsq(own.w4, g * ha.gscale, own.s4, -ha.lr) : adagrad(own.w4, g * ha.gscale, own.s4, ha);
    }
  }
  // ---- the wide rows' gradient table over the dead activation images (A1 .. GY): one pass per rank in
  // rank order (within a rank the leader ids are distinct, so no two lanes touch a row); the first pass that
  // touches a row finds the sentinel and marks the entry as the row's updater.  Every entry's (z, n) is
  // fetched first (in flight during the passes; only the updater's is used)
  constexpr unsigned GSENT = 0x7FC0DEADu;  // a NaN no gradient sum produces
  float* gacc = (float*)(lds + OFF_A1 * 2);
  float2 zn[XR][2];
#pragma unroll
  for (int r = 0; r < XR; ++r)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      zn[r][k] = C.zn[eid[r][k] >= 0 ? eid[r][k] : 0];  // (unconditional: a predicated load kept zn in scratch)
#pragma unroll
  for (int r = 0; r < XR; ++r)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (eid[r][k] >= 0) gacc[eid[r][k]] = __uint_as_float(GSENT);
  __syncthreads();
  unsigned mine = 0u;
#pragma unroll
  for (int r = 0; r < XR; ++r) {
    if (r < W) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (eid[r][k] >= 0) {
          const int id = eid[r][k];
          const float o = gacc[id];
          const bool first = __float_as_uint(o) == GSENT;
          gacc[id] = first ? eg[r][k] : o + eg[r][k];
          mine |= first ? 1u << (2 * r + k) : 0u;
        }
      __syncthreads();
    }
  }
  // FTRL-proximal once per distinct row, by the lane holding its first occurrence; (z, n) from the private copy
  const OptHP hf = {C.ftrl.lr, C.ftrl.gscale, C.ftrl.wd, C.ftrl.a, C.ftrl.b, C.ftrl.c, C.ftrl.d, C.ftrl.e};
  const float ilr = __builtin_amdgcn_rcpf(hf.lr);
#pragma unroll
  for (int r = 0; r < XR; ++r)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (mine & (1u << (2 * r + k))) {
        const int id = eid[r][k];
        const float g = gacc[id] * hf.gscale;
        gacc[id] = 0.f;  // (the row's only reader: its slot is padding-clean again for the forward)
        const float wo = LF[F_WTAB + id];
        const float n0 = zn[r][k].y;
        const float nn = fmaf(g, g, n0);
        const float rs = __builtin_amdgcn_sqrtf(nn);
        const float zz = zn[r][k].x + g - (rs - __builtin_amdgcn_sqrtf(n0)) * ilr * wo;
        const float den = (hf.c + rs) * ilr + 2.f * hf.b;
        LF[F_WTAB + id] = (fabsf(zz) <= hf.a) ? 0.f : -(zz - copysignf(hf.a, zz)) * __builtin_amdgcn_rcpf(den);
        C.zn[id] = make_float2(zz, nn);
      }
  // ---- give the activation images back as the forward expects them: every table slot was zeroed by its
  // row's updater above (padding columns the MFMAs read must hold 0, never the sentinel NaN); the constant
  // ones columns 1 again
  __syncthreads();
  ones_columns(Lb, C.B, tid);
  // ---- the new bf16 W images, fp32 biases and logits weights for the next forward
  const int p = perm8(wave);
  put_seq<L3, R3>(Lb, LF, p, lane, own.w + S3);
  put_seq<L2, R2>(Lb, LF, p, lane, own.w + S2);
  put_seq<L1, R1>(Lb, LF, p, lane, own.w + S1);
  if (wave < L0::NDW) put_w<L0>(Lb, LF, wave, lane, own.w[S0]);
  if (wave == NW - 1 && lane <= D4) LF[lane < D4 ? F_W4 + lane : F_MISC] = own.w4;
}

template <bool RSQ, bool DP, int NR = 8>
__global__ __launch_bounds__(NT) void taxi_step_k(Args A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  bf16_raw* const Lb = (bf16_raw*)lds;
  float* const LF = (float*)(lds + BF_BYTES);
  float* const stage = (float*)lds;
  int* const idt = (int*)(LF + F_IDT);  // [16][BP] the step's wide ids by (column, example), -1: none
  int* const ltab = (int*)(LF + F_LT);  // [16][BP] each entry's leader: first example with the same id
  const int tid = threadIdx.x;
  int lane = tid & 63;
  const int wave0 = __builtin_amdgcn_readfirstlane(tid >> 6);
  int wave = wave0, b0 = 16 * wave0;  // b0: (tile waves) batch tile
  const bool tw = wave0 < NTW;  // tile wave
  const int B = A.B;
  const OptHP ha = A.ada;
  stamp(A, 0);

  // ------------------------------------------------------------------ launch prologue
  Own own;
  {
    const auto& C = COLD;
    const int span = (int)(C.deep_hi - C.deep_lo);
    // deep parameters and their Adagrad state, each through a coalesced LDS staging copy of the span
    gather_in(stage, C.master + C.deep_lo, span, tid);
    bar();
    own_stage<true, false>(stage, own, wave, lane);
    bar();
    gather_in(stage, C.ada_s + C.deep_lo, span, tid);
    bar();
    own_stage<true, true>(stage, own, wave, lane);
    bar();
    // the kernel-private (z, n) copy of the FTRL state (leaders read / write one float2 per row a step):
    // 4 rows a lane, 16-byte accesses (a single CU's store path is the limit here)
    const float* zs = C.ftrl_z + C.wide_off;
    const float* ns = C.ftrl_n + C.wide_off;
    const int r4 = ((((uintptr_t)zs | (uintptr_t)ns) & 15) == 0) ? C.rows >> 2 : 0;
    for (int q = tid; q < r4; q += NT) {
      const f32x4 z4 = ((const f32x4*)zs)[q], n4 = ((const f32x4*)ns)[q];
      ((f32x4*)C.zn)[2 * q] = (f32x4){z4[0], n4[0], z4[1], n4[1]};
      ((f32x4*)C.zn)[2 * q + 1] = (f32x4){z4[2], n4[2], z4[3], n4[3]};
    }
    for (int r = 4 * r4 + tid; r < C.rows; r += NT) C.zn[r] = make_float2(zs[r], ns[r]);
  }
  // the batch (tile waves): lane -> example b = b0 + (lane & 15), columns c = (lane >> 4) + 4 m
  const int eb = b0 + (lane & 15), eg = lane >> 4;
  const bool evb = tw && eb < B;
  const long long bi0 = A.cursor ? A.cursor[0] : 0;
  int cid[4], nid[4];
  float yv = 0.f, ny = 0.f, nd = 0.f;
  int bnx = (int)(bi0 % A.nbatch);  // the batch the "next" registers hold (advanced by fetch, no modulo)
  auto fetch = [&](bool advance) {  // the next batch -> the "next" registers
    const auto& C = COLD;
    if (advance) bnx = bnx + 1 == C.nbatch ? 0 : bnx + 1;
    const long long bi = bnx;
    const long long* cb = C.cat + (bi * B + (evb ? eb : 0)) * NWIDE;
#pragma unroll
    for (int m = 0; m < 4; ++m) nid[m] = evb && eg + 4 * m < NWIDE ? (int)cb[eg + 4 * m] : -1;
    ny = evb ? C.label[bi * B + eb] : 0.f;
    nd = evb && eg < D0 ? C.dense[(bi * B + eb) * D0 + eg] : 0.f;
  };
  if (tw) {
    fetch(false);
#pragma unroll
    for (int m = 0; m < 4; ++m) cid[m] = nid[m];
    yv = ny;
  }
  {
    uint4* z = (uint4*)lds;
    for (int e = tid; e < LDS_BYTES / 16; e += NT) z[e] = make_uint4(0u, 0u, 0u, 0u);
  }
  bar();
  // the input's ones column (db0); the fp32 bias arrays' constant tail: 1 at OUT makes the forward
  // epilogue write the next layer's ones column, -1e30 beyond makes it write zeros
  if (tid < B) {
    Lb[OFF_A0 + tid * SA0 + D0] = f2b(1.f);
    Lb[OFF_A0 + BP * SA0 + tid * SA0 + D0] = f2b(1.f);
  }
  if (tid < 16) {
    if (D1 + tid < 16 * L0::OT) LF[F_B0 + D1 + tid] = tid ? -1e30f : 1.f;
    if (D2 + tid < 16 * L1::OT) LF[F_B1 + D2 + tid] = tid ? -1e30f : 1.f;
    if (D3 + tid < 16 * L2::OT) LF[F_B2 + D3 + tid] = tid ? -1e30f : 1.f;
    if (D4 + tid < 16 * L3::OT) LF[F_B3 + D4 + tid] = tid ? -1e30f : 1.f;
  }
  ones_columns(Lb, B, tid);
  if (evb && eg < D0) Lb[OFF_A0 + eb * SA0 + eg] = f2b(nd);
  {
    const int p = perm8(wave);
    put_seq<L3, R3>(Lb, LF, p, lane, own.w + S3);
    put_seq<L2, R2>(Lb, LF, p, lane, own.w + S2);
    put_seq<L1, R1>(Lb, LF, p, lane, own.w + S1);
    if (wave == NW - 1 && lane <= D4) LF[lane < D4 ? F_W4 + lane : F_MISC] = own.w4;
  }
  if (wave < L0::NDW) put_w<L0>(Lb, LF, wave, lane, own.w[S0]);
  if (tw) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (eg + 4 * m < NWIDE) idt[(eg + 4 * m) * BP + eb] = cid[m];  // (-1 for examples >= B)
  }
  gather_in(LF + F_WTAB, A.master + A.wide_off, A.rows, tid);
  // (the zn copy's stores need not land here: B3 waits for them before a leader reads (z, n))
  bar();
  stamp(A, 1);

  float lsum = 0.f, csum = 0.f, gb = 0.f;
  // data parallel: every replica's gradient carries 1 / (global batch), so the rank-order sum of the W
  // replicas' gradients is the gradient of the global-batch mean loss (MirroredStrategy semantics)
  const float invB = 1.f / (float)(DP ? B * A.world : B);
  const long long xs0 = DP ? A.xstep[0] : 0;
  stamp_clk(A, 20);
  float wv[4], zl[4], nl[4];  // (tile waves) gathered wide weights; FTRL state of the rows this lane leads
  unsigned lead = 0u;
  // entries e = gl + 320 k of the gradient waves' leader passes: column e / BP, example e % BP
  auto gl_entry = [&](int k, int& c, int& b) {
    const int e = (wave - NTW) * 64 + lane + (NW - NTW) * 64 * k;
    c = e / BP;
    b = e - c * BP;
  };
  for (int step = 0; step < A.nsteps; ++step) {
    const bool last = step + 1 == A.nsteps;
    const int par = (int)((xs0 + step) & 1);  // (DP) exchange-buffer parity of this step
    const bf16_raw* A0 = Lb + OFF_A0 + (step & 1) * BP * SA0;
    if (last) stamp(A, 7);
    // ============================================================ FWD: tile waves, no barrier inside | leaders
    lane = fresh(tid & 63);
    wave = fresh_s(wave0);
    b0 = 16 * wave;
    if (tw) {
      // this lane's wide rows (kept: the FTRL of the rows it leads needs the old weight), their sum
      // folded over the 4 lane groups in a fixed order
      float ws = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        wv[m] = cid[m] >= 0 ? LF[F_WTAB + cid[m]] : 0.f;
        ws += wv[m];
      }
      fwd_tile<L0, false>(Lb, LF, A0, b0, lane, B, nullptr);
      fence_c();
      if (last) stampw(A, 8, 0);
      fwd_tile<L1, false>(Lb, LF, Lb + L1::OFFA, b0, lane, B, nullptr);
      fence_c();
      if (last) stampw(A, 9, 0);
      fwd_tile<L2, false>(Lb, LF, Lb + L2::OFFA, b0, lane, B, nullptr);
      fence_c();
      if (last) stampw(A, 10, 0);
      float a4[L3::OT][4];
      fwd_tile<L3, true>(Lb, LF, Lb + L3::OFFA, b0, lane, B, a4);
      if (last) stampw(A, 11, 0);
      // logits = a4 . w4 + b4 (a4 as the bf16 image holds it), + the wide sum
      float zd = 0.f;
#pragma unroll
      for (int ot = 0; ot < L3::OT; ++ot) {
        const f32x4 w4 = *(const f32x4*)(LF + F_W4 + 16 * ot + 4 * eg);  // zero beyond D4 (ones column too)
#pragma unroll
        for (int r = 0; r < 4; ++r) zd = fmaf(rbf(a4[ot][r]), w4[r], zd);
      }
      zd += __shfl_xor(zd, 16, 64);
      zd += __shfl_xor(zd, 32, 64);
      ws += __shfl_xor(ws, 16, 64);
      ws += __shfl_xor(ws, 32, 64);
      const bool vb = eb < B;
      const float z = zd + LF[F_MISC] + ws;
      const float e = __expf(-fabsf(z));
      const float re = __builtin_amdgcn_rcpf(1.f + e);
      const float p = z >= 0.f ? re : e * re;
      gb = vb ? (p - yv) * invB : 0.f;
      if (eg == 0) LF[F_GV + eb] = gb;  // (the wide rows' gradients, summed per leader in B3)
      // G4[b][o] = g w4[o] relu'(a4[b][o]) (K columns 0..47 of dX3; 48..63 meet zero W3 rows)
#pragma unroll
      for (int ot = 0; ot < L3::OT; ++ot) {
        const f32x4 w4 = *(const f32x4*)(LF + F_W4 + 16 * ot + 4 * eg);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = sel(a4[ot][r] > 0.f, gb * w4[r], 0.f);
        st4(Lb + OFF_GX + eb * SG + 16 * ot + 4 * eg, v[0], v[1], v[2], v[3]);
      }
      // logits-layer gradient partials over this tile's 16 examples: sum_b g_b a4[b][o] (the ones
      // column o = 34 gives db4), a fixed-order DPP row sum, one row-leader lane per 4 columns
#pragma unroll
      for (int ot = 0; ot < L3::OT; ++ot) {
        float q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = row_fold<1>(gb * rbf(a4[ot][r]));
        if ((lane & 15) == 0) *(f32x4*)(LF + F_DW4 + wave * 48 + 16 * ot + 4 * eg) = (f32x4){q[0], q[1], q[2], q[3]};
      }
      if (last && eg == 0 && vb) {
        lsum = fmaxf(z, 0.f) - z * yv + __logf(1.f + e);
        csum = (float)((p > 0.5f) == (yv > 0.5f));
      }
      if (last) stampw(A, 12, 0);
    } else {
      // each entry's leader: the smallest example index with the same id in its column (ids of
      // different columns never coincide), from the column read 4 ids at a time
#pragma unroll
      for (int k = 0; k < 2; ++k) {  // 2 x 320 lanes >= 13 x 48 entries
        int c, b;
        gl_entry(k, c, b);
        if (c < NWIDE) {
          const int id = idt[c * BP + b];
          int L = b;
#pragma unroll
          for (int q = 0; q < BP / 4; ++q) {
            const int4 v = *(const int4*)(idt + c * BP + 4 * q);
            L = (v.w == id && 4 * q + 3 < L) ? 4 * q + 3 : L;
            L = (v.z == id && 4 * q + 2 < L) ? 4 * q + 2 : L;
            L = (v.y == id && 4 * q + 1 < L) ? 4 * q + 1 : L;
            L = (v.x == id && 4 * q < L) ? 4 * q : L;
          }
          ltab[c * BP + b] = id >= 0 ? L : -1;
        }
      }
    }
    bar();
    if (last) stamp(A, 2);
    // ============================================================ B3: dX3 ; leaders fetch (z, n) | dW3, dW4, leader sums
    lane = fresh(tid & 63);
    wave = fresh_s(wave0);
    b0 = 16 * wave;
    if (tw) {
      dx_tile<L3>(Lb, Lb + OFF_GX, Lb + OFF_GY, b0, lane);
      if (last) stampw(A, 13, 0);
      // the previous step's (z, n) stores (same CU) completed before these loads: by now the wait is free
      lead = 0u;
      if constexpr (!DP) {  // (data parallel: the apply phase updates every touched row after the exchange)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const auto& C = COLD;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int c = eg + 4 * m, r = cid[m];
          if (r >= 0 && ltab[c * BP + eb] == eb) {
            lead |= 1u << m;
            const float2 q = C.zn[r];
            zl[m] = q.x;
            nl[m] = q.y;
          }
        }
      }
      if (last) stampw(A, 14, 0);
      if (step + 1 < A.nsteps) fetch(true);  // the next batch, in flight during the backward
    } else {
      // the summed example gradient of every leader entry, in example order
#pragma unroll
      for (int k = 0; k < 2; ++k) {  // 2 x 320 lanes >= 13 x 48 entries
        int c, b;
        gl_entry(k, c, b);
        const bool ld = c < NWIDE && ltab[c * BP + b] == b;
        float g = 0.f;
        if (ld) {
#pragma unroll
          for (int q = 0; q < BP / 4; ++q) {
            const int4 l4 = *(const int4*)(ltab + c * BP + 4 * q);
            const f32x4 g4 = *(const f32x4*)(LF + F_GV + 4 * q);
            g += l4.x == b ? g4[0] : 0.f;
            g += l4.y == b ? g4[1] : 0.f;
            g += l4.z == b ? g4[2] : 0.f;
            g += l4.w == b ? g4[3] : 0.f;
          }
          if constexpr (!DP) LF[F_GS + c * BP + b] = g;
        }
        if constexpr (DP) {
          // every entry of the step (id of a leader, -1 otherwise) with its summed gradient, to every rank
          if (c < NWIDE) {
            const auto& C = COLD;
            const int id = ld ? idt[c * BP + b] : -1;
            for (int r = 0; r < C.world; ++r)
              xst8(C.xbuf[r] + (long)(par * XMAX + (C.loopback ? r : C.rank)) * XPAY, XW_OFF + (c * BP + b) * 8, id, g);
          }
        }
      }
    }
    dw_seq<L3, R3, RSQ, DP>(Lb + L3::OFFA, Lb + OFF_GX, perm8(wave), lane, own.w + S3, own.s + S3, ha, S3, par);
    if (last) stampw(A, 15, 3);
    if (wave == NW - 1) {  // the logits layer: sum the tiles' partials in order, Adagrad, new w4 / b4 now
      const int i = lane <= D4 ? lane : 0;
      const float g = (LF[F_DW4 + i] + LF[F_DW4 + 48 + i]) + LF[F_DW4 + 96 + i];
      if constexpr (DP) {
        const auto& C = COLD;
        if (lane <= D4)
          for (int r = 0; r < C.world; ++r)
            xst4(C.xbuf[r] + (long)(par * XMAX + (C.loopback ? r : C.rank)) * XPAY, XL4_OFF + lane * 4, g);
      } else {
      float s1 = own.s4;
      const float wn = RSQ ? adagrad_rsq(own.w4, g * ha.gscale, s1, -ha.lr) : adagrad(own.w4, g * ha.gscale, s1, ha);
      if (lane <= D4) {
        own.w4 = wn;
        own.s4 = s1;
        LF[lane < D4 ? F_W4 + lane : F_MISC] = wn;
      }
      }
    }
    bar();
    if (last) stamp(A, 3);
    // ============================================================ B2: dX2 | W3 image, dW2
    lane = fresh(tid & 63);
    wave = fresh_s(wave0);
    b0 = 16 * wave;
    if (tw) dx_tile<L2>(Lb, Lb + OFF_GY, Lb + OFF_GX, b0, lane);
    if constexpr (!DP) put_seq<L3, R3>(Lb, LF, perm8(wave), lane, own.w + S3);
    dw_seq<L2, R2, RSQ, DP>(Lb + L2::OFFA, Lb + OFF_GY, perm8(wave), lane, own.w + S2, own.s + S2, ha, S2, par);
    bar();
    if (last) stamp(A, 4);
    // ============================================================ B1: dX1 | W2 image, dW1
    lane = fresh(tid & 63);
    wave = fresh_s(wave0);
    b0 = 16 * wave;
    if (tw) dx_tile<L1>(Lb, Lb + OFF_GX, Lb + OFF_GY, b0, lane);
    if (last) stampw(A, 16, 0);
    if constexpr (!DP) put_seq<L2, R2>(Lb, LF, perm8(wave), lane, own.w + S2);
    dw_seq<L1, R1, RSQ, DP>(Lb + L1::OFFA, Lb + OFF_GX, perm8(wave), lane, own.w + S1, own.s + S1, ha, S1, par);
    if (last) stampw(A, 17, 3);
    bar();
    if (last) stamp(A, 5);
    // ============================================================ B0: dW0 (+ image) ; FTRL ; next batch | W1 image
    lane = fresh(tid & 63);
    wave = fresh_s(wave0);
    b0 = 16 * wave;
    if (wave < L0::NDW) {
      dw_seq<L0, 1, RSQ, DP>(A0, Lb + OFF_GY, wave, lane, own.w + S0, own.s + S0, ha, S0, par);
      if constexpr (!DP) put_w<L0>(Lb, LF, wave, lane, own.w[S0]);
    }
    if constexpr (!DP) put_seq<L1, R1>(Lb, LF, perm8(wave), lane, own.w + S1);
    if (tw) {
      // FTRL-proximal on the rows this lane leads: the summed gradient from the leader sums, the old
      // weight in wv; the new weight goes back to the table, (z, n) to the private copy
      const auto& C = COLD;
      const OptHP hf = {C.ftrl.lr, C.ftrl.gscale, C.ftrl.wd, C.ftrl.a, C.ftrl.b, C.ftrl.c, C.ftrl.d, C.ftrl.e};
      const float ilr = __builtin_amdgcn_rcpf(hf.lr);
      float w1[4], z1[4], n1[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if constexpr (DP) break;  // (the apply phase updates the rows after the exchange)
        const float g = LF[F_GS + (eg + 4 * m) * BP + eb] * hf.gscale;
        const float nn = fmaf(g, g, nl[m]);
        const float rs = __builtin_amdgcn_sqrtf(nn);
        const float zz = zl[m] + g - (rs - __builtin_amdgcn_sqrtf(nl[m])) * ilr * wv[m];
        const float den = (hf.c + rs) * ilr + 2.f * hf.b;
        w1[m] = (fabsf(zz) <= hf.a) ? 0.f : -(zz - copysignf(hf.a, zz)) * __builtin_amdgcn_rcpf(den);
        z1[m] = zz;
        n1[m] = nn;
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (!DP && (lead & (1u << m))) LF[F_WTAB + cid[m]] = w1[m];
      // the next batch (loaded during B3) into registers / the other A0 image / the id table BEFORE the
      // (z, n) stores: a wait for these loads must not include those stores (conditional: the compiler
      // would wait for every outstanding access)
      int cn[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) cn[m] = nid[m];
      const float yn = ny;
      if (!last && evb && eg < D0) Lb[OFF_A0 + ((step + 1) & 1) * BP * SA0 + eb * SA0 + eg] = f2b(nd);
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (eg + 4 * m < NWIDE) idt[(eg + 4 * m) * BP + eb] = cn[m];
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (!DP && (lead & (1u << m))) C.zn[cid[m]] = make_float2(z1[m], n1[m]);
#pragma unroll
      for (int m = 0; m < 4; ++m) cid[m] = cn[m];
      yv = yn;
      if (last) stampw(A, 18, 0);
    }
    bar();
    if (last) stamp(A, 6);
    if constexpr (DP) {
      // ========================================================== exchange: every rank's gradients, then apply
      if (!exchange_step(A, xs0 + step + 1, step, lds)) return;  // (sticky error word set; state partial)
      lane = fresh(tid & 63);
      wave = fresh_s(wave0);
      apply_dp<RSQ, NR>(own, lds, par, wave, lane, tid);
      bar();
      if (last) stamp(A, 30);
    }
  }
  stamp_clk(A, 21);

  // ------------------------------------------------------------------ write-back
  if (tw) {
    lsum = wave_sum(lsum);
    csum = wave_sum(csum);
    if (lane == 0) {
      LF[F_RED + wave] = lsum;
      LF[F_RED + 8 + wave] = csum;
    }
  }
  bar();
  {
    const auto& C = COLD;
    if (tid == 0) {
      float l = 0.f, c = 0.f;
      for (int w = 0; w < NTW; ++w) {
        l += LF[F_RED + w];
        c += LF[F_RED + 8 + w];
      }
      if (C.loss) C.loss[0] = l / (float)B;
      if (C.correct) C.correct[0] = (int)c;
    }
    // deep parameters and state through the staging copy: sentinel-filled, the owners' values written,
    // then copied out coalesced where not the sentinel (the span's alignment gaps keep their values)
    stamp(A, 22);
    const int span = (int)(C.deep_hi - C.deep_lo);
    unsigned* su = (unsigned*)stage;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      float* dst = (pass ? C.ada_s : C.master) + C.deep_lo;
      for (int e = tid; e < span; e += NT) su[e] = SENT;
      bar();
      stamp(A, 23 + 3 * pass);
      if (pass) own_stage<false, true>(stage, own, wave, lane);
      else own_stage<false, false>(stage, own, wave, lane);
      bar();
      stamp(A, 24 + 3 * pass);
      // 4 elements a lane: one 16-byte store (+ 8-byte shadow) where all 4 are owned (the alignment gaps
      // between tensors are the only exceptions)
      const bool al = ((uintptr_t)dst & 15) == 0;
      for (int e4 = tid; 4 * e4 < span; e4 += NT) {
        const int e = 4 * e4;
        bool all = al && e + 3 < span;
#pragma unroll
        for (int k = 0; k < 4; ++k) all = all && su[e + k] != SENT;
        if (all) {
          const f32x4 v = *(const f32x4*)(stage + e);
          *(f32x4*)(dst + e) = v;
          if (!pass && C.shadow) st4(C.shadow + C.deep_lo + e, v[0], v[1], v[2], v[3]);
        } else {
          for (int k = 0; k < 4 && e + k < span; ++k)
            if (su[e + k] != SENT) {
              dst[e + k] = stage[e + k];
              if (!pass && C.shadow) C.shadow[C.deep_lo + e + k] = f2b(stage[e + k]);
            }
        }
      }
      bar();
    }
    stamp(A, 29);
    // the wide part: weights from the table, (z, n) from the private copy; 4 rows a lane, 16-byte stores
    {
      float* wm = C.master + C.wide_off;
      float* zs = C.ftrl_z + C.wide_off;
      float* ns = C.ftrl_n + C.wide_off;
      bf16_raw* sh = C.shadow ? C.shadow + C.wide_off : nullptr;
      const int r4 = ((((uintptr_t)wm | (uintptr_t)zs | (uintptr_t)ns) & 15) == 0 && (((uintptr_t)sh) & 7) == 0)
                         ? C.rows >> 2 : 0;
      for (int q = tid; q < r4; q += NT) {
        const f32x4 a = ((const f32x4*)C.zn)[2 * q], b = ((const f32x4*)C.zn)[2 * q + 1];
        const f32x4 w = *(const f32x4*)(LF + F_WTAB + 4 * q);
        ((f32x4*)wm)[q] = w;
        ((f32x4*)zs)[q] = (f32x4){a[0], a[2], b[0], b[2]};
        ((f32x4*)ns)[q] = (f32x4){a[1], a[3], b[1], b[3]};
        if (sh) st4(sh + 4 * q, w[0], w[1], w[2], w[3]);
      }
      for (int r = 4 * r4 + tid; r < C.rows; r += NT) {
        const float w = LF[F_WTAB + r];
        const float2 t = C.zn[r];
        wm[r] = w;
        zs[r] = t.x;
        ns[r] = t.y;
        if (sh) sh[r] = f2b(w);
      }
    }
    if (tid == 0) {
      if (C.step_ada) C.step_ada[0] += (float)C.nsteps;
      if (C.step_ftrl) C.step_ftrl[0] += (float)C.nsteps;
      if (C.rng) C.rng[1] += (unsigned long long)C.rng_bumps * (unsigned long long)C.nsteps;
      if (C.cursor) C.cursor[0] = (bi0 + C.nsteps) % C.nbatch;
      if (DP) C.xstep[0] = xs0 + C.nsteps;
    }
  }
  stamp(A, 19);
}

// iv: L B nbatch nwide wide_off apply_opt rng_bumps dims[L+1] woff[L] boff[L] [nsteps] (widedeep_step.hip's
// contract); fv: ada(8) ftrl(8).  0 = this kernel takes the configuration.
int fill(Args& a, const long* iv, int ni, const float* fv, int nf, long rows) {
  if (ni < 7 || nf != 16 || rows < 1 || rows > MAXROWS) return -1;
  const int L = (int)iv[0];
  const int nbase = 7 + (L + 1) + 2 * L;
  if (L != 5 || (ni != nbase && ni != nbase + 1)) return -1;
  const int dims[6] = {D0, D1, D2, D3, D4, 1};
  for (int i = 0; i <= L; ++i)
    if (iv[7 + i] != dims[i]) return -1;
  a.B = (int)iv[1];
  a.nbatch = (int)iv[2];
  if (iv[3] != NWIDE || iv[5] != 1 || a.B < 1 || a.B > BP || a.nbatch < 1) return -1;
  a.wide_off = iv[4];
  a.rng_bumps = (int)iv[6];
  a.deep_lo = iv[8 + L];
  a.deep_hi = a.deep_lo;
  for (int i = 0; i < L; ++i) {
    a.woff[i] = iv[8 + L + i];
    a.boff[i] = iv[8 + 2 * L + i];
    const long dims_in = dims[i], dims_out = dims[i + 1];
    a.deep_lo = a.woff[i] < a.deep_lo ? a.woff[i] : a.deep_lo;
    a.deep_lo = a.boff[i] < a.deep_lo ? a.boff[i] : a.deep_lo;
    const long we = a.woff[i] + dims_in * dims_out, be = a.boff[i] + dims_out;
    a.deep_hi = we > a.deep_hi ? we : a.deep_hi;
    a.deep_hi = be > a.deep_hi ? be : a.deep_hi;
  }
  if (a.deep_hi - a.deep_lo > STAGE_MAX || a.deep_lo < 0) return -1;
  for (int i = 0; i < L; ++i) {
    a.rw[i] = (int)(a.woff[i] - a.deep_lo);
    a.rb[i] = (int)(a.boff[i] - a.deep_lo);
  }
  // the wide slice must not overlap the deep span (the owners write both)
  if (a.wide_off < a.deep_hi && a.wide_off + rows > a.deep_lo) return -1;
  a.nsteps = ni == nbase + 1 ? (int)iv[nbase] : 1;
  if (a.nsteps < 1) return -1;
  a.rows = (int)rows;
  a.ada = OptHP{fv[0], fv[1], fv[2], fv[3], fv[4], fv[5], fv[6], fv[7]};
  a.ftrl = OptHP{fv[8], fv[9], fv[10], fv[11], fv[12], fv[13], fv[14], fv[15]};
  return 0;
}

}  // namespace taxi2

// rows = wide table rows.  Returns the LDS bytes if the v2 kernel takes this configuration, else -1.
// exchange geometry for the host (models/widedeep.py TaxiExchange): buffer bytes, flag words, max ranks
extern "C" void hopsx_taxi_step2_xgeom(long* g) {
  g[0] = taxi2::X_BYTES;
  g[1] = taxi2::XF_WORDS;
  g[2] = taxi2::XMAX;
  g[3] = taxi2::XPAY;
}
extern "C" long hopsx_taxi_step2_ok(const long* iv, int ni, long rows) {
  taxi2::Args a{};
  const float f[16] = {};
  if (taxi2::fill(a, iv, ni, f, 16, rows)) return -1;
  return taxi2::LDS_BYTES;
}

// ptrs: master grad shadow ada_s ftrl_z ftrl_n dense cat label cursor loss correct step_ada step_ftrl rng dbg
// (widedeep_step.hip's order; grad is unused: the gradients never leave the kernel), zn ([rows] float2
// scratch), rsq (nonzero: the host checked wd == 0 and eps < 1e-7 sqrt(initial Adagrad accumulator));
// data parallel (np = 22 + 2 world): world | rank << 8 | loopback << 16, timeout_ms, err, xstep,
// xbuf[world], xflag[world]
extern "C" int hopsx_taxi_step2(const uint64_t* p, int np, const long* iv, int ni, const float* fv, int nf, long rows,
                                hipStream_t st) {
  taxi2::Args a{};
  if (np < 18 || taxi2::fill(a, iv, ni, fv, nf, rows)) return -2;
  bool dp = false;
  if (np > 18) {
    a.world = (int)(p[18] & 0xFF);
    a.rank = (int)((p[18] >> 8) & 0xFF);
    a.loopback = (int)((p[18] >> 16) & 0xFF);
    if (a.world < 2 || a.world > taxi2::XMAX || a.rank >= a.world || np != 22 + 2 * a.world) return -2;
    a.tmo = (long long)p[19] * 100000ll;  // ms -> 100 MHz ticks
    a.err = (unsigned*)p[20];
    a.xstep = (long long*)p[21];
    for (int r = 0; r < a.world; ++r) {
      a.xbuf[r] = (unsigned char*)p[22 + r];
      a.xflag[r] = (unsigned*)p[22 + a.world + r];
      if (!a.xbuf[r] || !a.xflag[r] || ((uint64_t)a.xbuf[r] & 15)) return -2;
    }
    if (!a.err || !a.xstep || a.tmo <= 0) return -2;
    dp = true;
  } else {
    a.world = 1;
  }
  a.master = (float*)p[0];
  a.shadow = (bf16_raw*)p[2];
  a.ada_s = (float*)p[3];
  a.ftrl_z = (float*)p[4];
  a.ftrl_n = (float*)p[5];
  a.dense = (const float*)p[6];
  a.cat = (const long long*)p[7];
  a.label = (const float*)p[8];
  a.cursor = (long long*)p[9];
  a.loss = (float*)p[10];
  a.correct = (int*)p[11];
  a.step_ada = (float*)p[12];
  a.step_ftrl = (float*)p[13];
  a.rng = (unsigned long long*)p[14];
  a.dbg = (unsigned long long*)p[15];
  a.zn = (float2*)p[16];
  a.ada_rsq = p[17] ? 1 : 0;
  if (!a.master || !a.ada_s || !a.ftrl_z || !a.ftrl_n || !a.dense || !a.cat || !a.label || !a.zn) return -2;
  if (a.ada_rsq && a.ada.wd != 0.f) return -2;
  static bool attr = false;
  if (!attr) {
    const void* fns[6] = {(const void*)taxi2::taxi_step_k<true, false>, (const void*)taxi2::taxi_step_k<false, false>,
                          (const void*)taxi2::taxi_step_k<true, true>, (const void*)taxi2::taxi_step_k<false, true>,
                          (const void*)taxi2::taxi_step_k<true, true, 2>, (const void*)taxi2::taxi_step_k<false, true, 2>};
    for (const void* f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, taxi2::LDS_BYTES);
    attr = true;
  }
  const size_t lds = (size_t)taxi2::LDS_BYTES;
  if (dp && a.world == 2) {  // (the deep apply's two-rank unit shape)
    if (a.ada_rsq) hipLaunchKernelGGL((taxi2::taxi_step_k<true, true, 2>), dim3(1), dim3(taxi2::NT), lds, st, a);
    else hipLaunchKernelGGL((taxi2::taxi_step_k<false, true, 2>), dim3(1), dim3(taxi2::NT), lds, st, a);
  } else if (dp) {
    if (a.ada_rsq) hipLaunchKernelGGL((taxi2::taxi_step_k<true, true>), dim3(1), dim3(taxi2::NT), lds, st, a);
    else hipLaunchKernelGGL((taxi2::taxi_step_k<false, true>), dim3(1), dim3(taxi2::NT), lds, st, a);
  } else {
    if (a.ada_rsq) hipLaunchKernelGGL((taxi2::taxi_step_k<true, false>), dim3(1), dim3(taxi2::NT), lds, st, a);
    else hipLaunchKernelGGL((taxi2::taxi_step_k<false, false>), dim3(1), dim3(taxi2::NT), lds, st, a);
  }
  return (int)hipGetLastError();
}
