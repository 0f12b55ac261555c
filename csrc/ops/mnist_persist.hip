// hopsx: the flagship MNIST CNN training step as ONE persistent launch per `nsteps` steps (gfx950).
//
// Model (reference E3/E5, notebooks/ml/Distributed_Training/mirrored_strategy/
// mirroredstrategy_mnist_example.ipynb:189-207): uint8 28x28 -> x/255 - .5 -> Conv32 k2 relu ->
// Conv64 k2 relu -> MaxPool2 -> Dropout(.01) -> Dense128 relu -> Dense10 -> sparse softmax CE
// (mean over the batch) -> Adadelta(lr, rho, eps) (:210-222 compile/fit).  B = 32 images per step.
//
// Why one launch.  The whole step is ~1.35 GFLOP (0.5 us of MFMA time at bf16 peak) spread over six
// dependent ops: as separate kernels it is latency-bound (six launches, each re-reading its operands
// and the 1.38 M-parameter fc1 weight / Adadelta state from HBM: ~36 MB per step).  Here every
// workgroup keeps its share of the model ON CHIP for all `nsteps` steps and hands off only the small
// activations between phases.
//
// Partition (the design decision everything else follows from): workgroup p < 169 owns pooled
// position p = (ph, pw) of the 13x13 map, for all 32 images and all 64 channels.  Then
//   * its conv1 -> conv2 -> pool receptive field is a private 4x4 input patch (conv1 and conv2 are
//     recomputed per position, no halo exchange);
//   * the fc1 weight columns it multiplies (W1[:, p*64 .. p*64+63], 8192 params) are touched by no
//     other workgroup: forward partial product, weight gradient AND the Adadelta update are local,
//     and its fp32 master + two Adadelta accumulators live in the lane registers of the fc1 wgrad
//     MFMA output layout (96 VGPRs per lane) for the whole launch (written back once at the end);
//   * the fc1 input gradient for its 64 pooled inputs is local too, so the whole conv backward is.
// What must cross workgroups per step (4 hand-offs, the critical path):
//   A  fc1 partial sums  [32 x 128] fp32 per position  -> 32 head workgroups (one per image) reduce
//      them in a fixed order, add the bias, relu, Dense10, softmax CE, dlogits, dh;
//   B  dh (+ h, dlogits, loss) of each image -> every position workgroup (and every head: each head
//      recomputes the fc2 / fc1-bias gradient from all 32 payloads and applies the SAME Adadelta
//      update to its replicated copy of those 1,418 params — bit-identical, no reduction hop);
//   C  conv-parameter gradient partials (8,416 fp32) per position -> 162 slice owners (52 params
//      each) reduce over the 169 partials in a fixed order and run Adadelta on their slice;
//   D  the updated conv parameters -> every position workgroup (next step's forward).
// Hand-off form: MI355X_MICROARCH.md "Valid forms" table, row 1 (cdna_hip_programming §6 G16 R1):
// payload stored write-through (16-B `sc1` buffer stores), every storing wave drains vmcnt, a
// workgroup barrier, ONE lane stores the flag (agent-scope relaxed = `global_store sc1`); the consumer
// polls the flags relaxed from one wave, then a barrier, then EVERY payload load is an `sc1` buffer
// load.  Flag epochs grow across launches (epoch = base + step + 1, the 64-bit base kept after the flag
// rows and advanced by nsteps at the end of each launch), so no memset precedes a launch.  Every
// poll is bounded (wall clock) and also watches a sticky error word, so a fault drains the grid.
// Payload buffers are double-buffered by step parity.
//
// Determinism: no float atomics anywhere — every cross-workgroup sum is a fixed-order loop, so two
// runs from the same state are bit-identical.
#include "common.h"
#include "optim_core.h"

namespace mnistp {

constexpr int B = 32;  // images per step
constexpr int C1 = 32, C2 = 64, HID = 128, NCLS = 10;
constexpr int PH = 13, NPOS = PH * PH;  // pooled positions = position workgroups
constexpr int KIN = NPOS * C2;          // 10816 fc1 inputs (NHWC flatten: (ph*13 + pw)*64 + c)
constexpr int NCONV = C2 * 128 + C2 + C1 * 4 + C1;  // 8416 conv params: [w2 | b2 | w1 | b1]
constexpr int OFF_B2 = C2 * 128, OFF_W1 = OFF_B2 + C2, OFF_B1 = OFF_W1 + C1 * 4;
constexpr int SLICE = 52, NSLICE = (NCONV + SLICE - 1) / SLICE;  // 162 slice owners
constexpr int NRED = 19;                                           // partial groups in the slice reduce
constexpr int NHEAD = B;
constexpr int GRID = NPOS + NHEAD;  // 201 workgroups, one per CU
constexpr int PAY = 272;            // head payload floats
constexpr int PAY_DH = 0, PAY_H = 128, PAY_DL = 256, PAY_LOSS = 268, PAY_COR = 269;
constexpr int FL_A = 0, FL_B = 256, FL_C = 512, FL_D = 768, FL_WORDS = 1024;
constexpr int FL_EPOCH = FL_WORDS - 2;  // 64-bit epoch base after the flag rows (8-B aligned)
// D payload (updated conv parameters): the conv2 weights as bf16 (what the MFMAs read), then the 224
// small fp32 parameters [b2 | conv1 w | conv1 b]
constexpr int D_F32 = OFF_B2 * 2;                 // byte offset of the fp32 part
constexpr int D_BYTES = D_F32 + (NCONV - OFF_B2) * 4;

// LDS row strides (bf16 elements), padded by 16 B against bank conflicts of the fragment reads
constexpr int W1S = 72, W2S = 136, C1S = 40, PLS = 72, DHS = 136, DCS = 136;

// position-workgroup LDS map (bytes, every offset a multiple of 16)
constexpr int L_W1 = 0;                           // bf16 [128 n][W1S]   fc1 slice
constexpr int L_W2 = L_W1 + HID * W1S * 2;        // bf16 [64 co][W2S]  conv2 weights (OHWI rows)
constexpr int L_CW1 = L_W2 + C2 * W2S * 2;        // f32  [32][4]       conv1 weights
constexpr int L_CB1 = L_CW1 + C1 * 4 * 4;         // f32  [32]
constexpr int L_CB2 = L_CB1 + C1 * 4;             // f32  [64]
constexpr int L_XIN = L_CB2 + C2 * 4;             // f32  [32 b][16]    input patch
constexpr int L_C1 = L_XIN + B * 16 * 4;          // bf16 [32 b][9 pos][C1S] conv1 output
constexpr int L_POOL = L_C1 + B * 9 * C1S * 2;    // bf16 [32 b][PLS]   pooled (+dropout)
constexpr int L_AM = L_POOL + B * PLS * 2;        // u8   [32 b][64]    argmax tap / 0xFF = no grad
constexpr int L_DH = L_AM + B * C2;               // bf16 [32 b][DHS]
constexpr int L_DC2 = L_DH + B * DHS * 2;         // bf16 [64 co][DCS] conv2 output grad, (b,q) cols
constexpr int L_STG = L_DC2 + C2 * DCS * 2;       // f32  staging: A partial [32][128] / C grads [8416]
constexpr int L_RED = L_STG + NCONV * 4;          // f32  [NRED][SLICE] slice reduce / conv1 grad halves
constexpr int L_SL = L_RED + 1024 * 4;            // f32  [3][SLICE] owned conv slice: master, s1, s2
constexpr int L_KEEP = L_SL + 3 * 64 * 4;         // u8   [32 b][64] next step's dropout keep mask
constexpr int LDS_BYTES = L_KEEP + B * C2;

// head-workgroup LDS map (aliases the same allocation)
constexpr int H_W2 = 0;                       // f32 [3][10*128] fc2 weight: master, s1, s2
constexpr int H_B2 = H_W2 + 3 * NCLS * HID * 4;  // f32 [3][16]
constexpr int H_B1 = H_B2 + 3 * 16 * 4;       // f32 [3][128]
constexpr int H_RED = H_B1 + 3 * HID * 4;     // f32 [8][128]
constexpr int H_H = H_RED + 8 * HID * 4;      // f32 [128]
constexpr int H_LOG = H_H + HID * 4;          // f32 [16]
constexpr int H_PAY = H_LOG + 16 * 4;         // f32 [PAY]
constexpr int H_ALL = H_PAY + PAY * 4;        // f32 [32][PAY]
constexpr int H_END = H_ALL + NHEAD * PAY * 4;
constexpr int H_DHS = H_END;                  // bf16 [32][DHS] dh staging (head 0, data-parallel)
static_assert(H_DHS + B * DHS * 2 <= LDS_BYTES, "head LDS map must fit the position map");

// ---- data-parallel exchange (DP instantiation, world > 1) ----
// Each rank owns one uncached (UC) exchange buffer and one UC flag page, IPC-mapped by every peer.
// A producer PUSHES its payload into every peer's buffer at slot [its rank] (system-scope write-through
// stores), drains, and raises its flag word in every peer's page; a consumer polls its OWN page and
// reads its OWN buffer (local memory, no L2 copies to go stale).  Flags carry a global step epoch that
// grows across launches (never reset), payloads are double-buffered by step parity.
constexpr int XMAX = 8;                                         // ranks (one node)
constexpr long XS_POOL = (long)NPOS * 4 * 64 * 16;              // fc1-wgrad B fragments of all positions
constexpr long XS_DHT = 8L * 64 * 16;                           // fc1-wgrad A fragments (dh^T), 8 n-blocks
constexpr int NFC2 = NCLS * HID + HID + NCLS, NFC2P = 1424;     // [fc2 w | fc1 b | fc2 b] gradient
constexpr long XS_FC2 = NFC2P * 4;
constexpr long XS_CONV = (long)NSLICE * SLICE * 4;              // conv slice gradient sums
constexpr long XO_POOL = 0, XO_DHT = XO_POOL + 2L * XMAX * XS_POOL, XO_FC2 = XO_DHT + 2L * XMAX * XS_DHT,
               XO_CONV = XO_FC2 + 2L * XMAX * XS_FC2, X_BYTES = XO_CONV + 2L * XMAX * XS_CONV;
constexpr int XF_POOL = 0, XF_H = XMAX * NPOS, XF_CONV = XF_H + XMAX, XF_WORDS = XF_CONV + XMAX * NSLICE;
static_assert(NFC2 <= NFC2P && NFC2P % 4 == 0 && X_BYTES < 0x7fffffffL, "exchange geometry");
static_assert(LDS_BYTES <= 160 * 1024, "one workgroup per CU: 160 KiB LDS");
static_assert(L_RED + NRED * SLICE * 4 <= L_SL && 2 * 32 * 5 * 4 <= 1024 * 4, "reduce scratch");
static_assert(NRED * 13 <= 256 && NSLICE * SLICE >= NCONV && NSLICE <= NPOS, "slice geometry");

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned __attribute__((address_space(1))) gu32;

struct Args {
  float* master;      // arena fp32 parameters
  bf16_raw* shadow;   // arena bf16 copy the other kernels read
  float* s1;          // Adadelta E[g^2]
  float* s2;          // Adadelta E[dx^2]
  long off[8];        // arena offsets: conv1.w conv1.b conv2.w conv2.b fc1.w fc1.b fc2.w fc2.b
  const unsigned char* xs;  // uint8 [nbatch][32][28][28]
  const long long* ys;      // int64 [nbatch][32]
  long nbatch;
  long long* cursor;         // next batch index (advanced by nsteps at the end)
  unsigned long long* rng;   // {seed, step counter} (dropout key; advanced by nsteps)
  float* step_dev;           // optimizer step count (advanced by nsteps), may be null
  const float* hp_dev;       // device hyper-parameters (OptHP layout), may be null
  float* slabA;  // [2][169][32][128]
  float* slabB;  // [2][32][PAY]
  float* slabC;  // [2][169][NCONV]
  float* slabD;  // [2][D_BYTES / 4]
  unsigned* flags;  // [FL_WORDS]: flag rows + the epoch base (zeroed once at allocation)
  unsigned* err;    // sticky error word (0 = ok)
  float* out;       // [nsteps][2]: mean loss, correct count
  unsigned long long* dbg;  // optional [GRID][nsteps][16] wall-clock phase stamps
  OptHP hp;
  float drop_p, xscale, xshift;
  unsigned salt;
  int nsteps;
  int acquire;  // 1: agent-scope acquire after every poll (diagnostic; the sc1 form needs none)
  long long tmo;  // wall-clock ticks a poll waits before it declares the producer lost
  long long tmo0;  // the same for step 0's purely local waits (co-residency: HOPSX_PERSIST_START_MS)
  int pollw, stagger;  // waves polling a hand-off wait and their start offsets (HOPSX_PERSIST_POLLW / _STAGGER)
  int pollw_a, pollw_b, pollw_c, pollw_d;  // per hand-off (HOPSX_PERSIST_POLLW_A.._D, default POLLW; C: 4)
  int head1w;          // 1: one wave computes the head from registers and publishes B (HOPSX_PERSIST_HEAD1W)
  float inv_gb;   // 1 / global batch (world * B): the loss is the mean over every replica's images
  // data parallel (DP instantiation)
  int world, rank;
  int loopback;                 // 1: one process plays every rank (peers = this rank's own buffers)
  int xfence;                   // 1: system-scope release fence before raising peer flags
  long long* xstep;             // global step counter (epoch base of the exchange flags)
  unsigned char* xbuf[XMAX];    // exchange buffers of ranks 0..world-1 (own at [rank])
  unsigned* xflag[XMAX];        // flag pages of ranks 0..world-1
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// write-through (sc1) 16-B store / sc1 16-B load (L1 bypass): the hand-off payload path
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, byte_off, 0, 16);
}
__device__ __forceinline__ void st_sc1x2(__amdgpu_buffer_rsrc_t r, int byte_off, float x, float y) {
  typedef int v2i __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64((v2i){__float_as_int(x), __float_as_int(y)}, r, byte_off, 0, 16);
}
__device__ __forceinline__ f32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void flag_store(unsigned* f, unsigned v) {
  __hip_atomic_store((gu32*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned flag_load(const unsigned* f) {
  return __hip_atomic_load((gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// system-scope (sc0 sc1) 16-B / 4-B buffer store and load: the cross-rank exchange path
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, int byte_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, byte_off, 0, 17);
}
__device__ __forceinline__ void st_sys1(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, byte_off, 0, 17);
}
__device__ __forceinline__ f32x4 ld_sys(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 17));
}
__device__ __forceinline__ float ld_sys1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 17));
}
__device__ __forceinline__ void xflag_store(unsigned* f, unsigned v) {
  __hip_atomic_store((gu32*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned xflag_load(const unsigned* f) {
  return __hip_atomic_load((gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// slot a push lands in: the producer's rank (loopback: the simulated peer's, so every slot fills)
__device__ __forceinline__ int xslot(const Args& a, int peer) { return a.loopback ? peer : a.rank; }

// Wave 0 polls flags[0..n) until every word equals `epoch` (relaxed sc1 loads + s_sleep); gives up
// on the sticky error word or after a.tmo ticks (recording `code`).  Returns the verdict to the
// whole workgroup (uniform).
// pollw > 1 (HOPSX_PERSIST_POLLW): that many waves poll, their first polls staggered by `stagger` x 64
// cycles, so a flag that lands between two polls of one wave is seen by the next wave's poll — the
// detection delay shrinks from ~half a poll round trip toward ~half of that over pollw.  The first
// wave to see every flag (or the error) tells the others through the LDS word s_ok[1], set to this
// wait's `code` (unique per phase and step, never 0); s_ok[0] carries the verdict as before.
__device__ __forceinline__ bool wait_all(const unsigned* flags, int n, unsigned epoch, unsigned* err, unsigned code,
                                      int acquire, int* s_ok, long long tmo, int pollw = 1, int stagger = 0) {
  if (pollw <= 1) {
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      int good = 1;
      const long long t0 = wall_clock64();
      for (unsigned spins = 0;; ++spins) {
        int ok = 1;
        for (int k = lane; k < n; k += 64) ok &= flag_load(flags + k) == epoch;
        if (__all(ok)) break;
        if (__builtin_amdgcn_readfirstlane(flag_load(err)) != 0u) {
          good = 0;
          break;
        }
        if ((spins & 15u) == 15u && wall_clock64() - t0 > tmo) {
          if (lane == 0) atomicCAS(err, 0u, code);
          good = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (acquire && good) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain();
      if (lane == 0) *s_ok = good;
    }
    __syncthreads();
    const int g = *s_ok;
    return g != 0;
  }
  volatile int* gen = s_ok + 1;
  const int wave = threadIdx.x >> 6;
  if (wave < pollw) {
    const int lane = threadIdx.x & 63;
    int good = 1;
    // (the stagger checks the done word too: when the flags are already there, wave 0's first poll ends
    // the wait and the later waves must not sleep out their offsets before the barrier)
    for (int d = 0; d < wave * stagger && __builtin_amdgcn_readfirstlane(*gen) != (int)code; ++d)
      __builtin_amdgcn_s_sleep(1);
    const long long t0 = wall_clock64();
    for (unsigned spins = 0;; ++spins) {
      if (__builtin_amdgcn_readfirstlane(*gen) == (int)code) break;  // another wave saw it
      int ok = 1;
      for (int k = lane; k < n; k += 64) ok &= flag_load(flags + k) == epoch;
      if (__all(ok)) {
        if (lane == 0) {
          s_ok[0] = 1;
          *gen = (int)code;
        }
        break;
      }
      if (__builtin_amdgcn_readfirstlane(flag_load(err)) != 0u) good = 0;
      if ((spins & 15u) == 15u && wall_clock64() - t0 > tmo) {
        if (lane == 0) atomicCAS(err, 0u, code);
        good = 0;
      }
      if (!good) {
        if (lane == 0) {
          s_ok[0] = 0;
          *gen = (int)code;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain();
  }
  __syncthreads();
  const int g = s_ok[0];
  return g != 0;
}

// Wave 0 polls this rank's flag page until word base + r * stride has reached `epoch` for every peer
// r != rank (the epoch grows across launches: "reached" is a wrap-safe >=).  Same failure handling
// and uniform verdict as wait_all.
__device__ __forceinline__ bool wait_peers(const Args& a, int base, int stride, unsigned epoch, unsigned code,
                                        int* s_ok) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned* page = a.xflag[a.rank];
    int good = 1;
    const long long t0 = wall_clock64();
    for (unsigned spins = 0;; ++spins) {
      const bool mine = lane < a.world && lane != a.rank;
      const int ok = !mine || (int)(xflag_load(page + base + lane * stride) - epoch) >= 0;
      if (__all(ok)) break;
      if (__builtin_amdgcn_readfirstlane(flag_load(a.err)) != 0u) {
        good = 0;
        break;
      }
      if ((spins & 15u) == 15u && wall_clock64() - t0 > a.tmo) {
        if (lane == 0) atomicCAS(a.err, 0u, code);
        good = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    drain();
    if (lane == 0) *s_ok = good;
  }
  __syncthreads();
  const int g = *s_ok;
  return g != 0;
}
// raise this rank's flag word base + slot * stride in every peer's page (after the payload drained)
// The payload stores are system-scope write-through (sc0 sc1) and drained (vmcnt 0) by every storing
// wave before this: that completes them at the system coherence point, the release for exactly these
// stores.  The optional fence (HOPSX_PERSIST_XFENCE=1) also writes back other dirty L2 lines.
__device__ __forceinline__ void raise_peers(const Args& a, int base, int stride, unsigned epoch) {
  if (a.xfence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: buffer_wbl2 sc0 sc1 + drain
  const int r = threadIdx.x & 63;
  if (r < a.world && r != a.rank) xflag_store(a.xflag[r] + base + xslot(a, r) * stride, epoch);
}

// Adadelta (optim_core.h upd<3>, rho = a, eps = b) with the hardware square root / reciprocal square
// root (1 ulp) instead of the correctly rounded sqrt + division sequences: ~8 instead of ~35 VALU ops
// an element, and the fc1 slice update (32 elements a lane) sits on the step's critical path
__device__ __forceinline__ float adadelta(float w, float g, float& s1, float& s2, const OptHP& h) {
  g = fmaf(h.wd, w, g);
  s1 = fmaf(h.a, s1, (1.f - h.a) * g * g);
  const float delta = g * __builtin_amdgcn_sqrtf(s2 + h.b) * __builtin_amdgcn_rsqf(s1 + h.b);
  s2 = fmaf(h.a, s2, (1.f - h.a) * delta * delta);
  return fmaf(-h.lr, delta, w);
}

__device__ __forceinline__ unsigned ecode(int phase, int s) {
  return 0x80000000u | ((unsigned)phase << 24) | (((unsigned)s & 0xFFFu) << 12) | (blockIdx.x & 0xFFFu);
}

// fp32 -> bf16 round-to-nearest-even by the gfx950 conversion instruction (v_cvt_pk_bf16_f32):
// the same bits as common.h's f2bf for every finite value, one instruction instead of five
__device__ __forceinline__ bf16_raw f2bf(float f) { return __builtin_bit_cast(bf16_raw, (__bf16)f); }

__device__ __forceinline__ bf16x8 lds8(const bf16_raw* p) { return *(const bf16x8*)p; }
// transposed fragment read (ds_read_b64_tr_b16): this lane addresses row (k) 8*fq + tq (p1) and
// 8*fq + tq + 4 (p2), 4 consecutive columns 4*tp..; the result holds column (lane & 15)'s 8 k values
__device__ __forceinline__ bf16x8 lds_tr(const bf16_raw* p1, const bf16_raw* p2) {
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p1));
  const bf16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_ptr)(p2));
  return (bf16x8){v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
}
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ long conv_idx(const Args& a, int j) {
  if (j < OFF_B2) return a.off[2] + j;
  if (j < OFF_W1) return a.off[3] + (j - OFF_B2);
  if (j < OFF_B1) return a.off[0] + (j - OFF_W1);
  return a.off[1] + (j - OFF_B1);
}

__device__ __forceinline__ void stamp(const Args& a, int s, int ph) {
  if (a.dbg && threadIdx.x == 0) a.dbg[((long)blockIdx.x * a.nsteps + s) * 16 + ph] = (unsigned long long)wall_clock64();
}

// ------------------------------------------------------------------------------------------------
// position workgroup p: conv1 -> conv2 -> pool -> fc1 partial; backward of all of it; fc1 slice
// Adadelta; conv-parameter slice owner
// ------------------------------------------------------------------------------------------------
template <bool DP>
__device__ __forceinline__ void position_wg(const Args& a, unsigned char* smem, int* s_ok, const OptHP& hp,
                                            long long cur0, unsigned long long seed, unsigned long long ctr0,
                                            long long xs0, unsigned long long eb) {
  const int p = blockIdx.x, ph = p / PH, pw = p - ph * PH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int tq = fr >> 2, tp = fr & 3;
  bf16_raw* W1 = (bf16_raw*)(smem + L_W1);
  bf16_raw* W2 = (bf16_raw*)(smem + L_W2);
  float* CW1 = (float*)(smem + L_CW1);
  float* CB1 = (float*)(smem + L_CB1);
  float* CB2 = (float*)(smem + L_CB2);
  float* XIN = (float*)(smem + L_XIN);
  bf16_raw* C1 = (bf16_raw*)(smem + L_C1);
  bf16_raw* POOL = (bf16_raw*)(smem + L_POOL);
  unsigned char* AM = smem + L_AM;
  bf16_raw* DH = (bf16_raw*)(smem + L_DH);
  bf16_raw* DC2 = (bf16_raw*)(smem + L_DC2);
  float* STG = (float*)(smem + L_STG);
  float* RED = (float*)(smem + L_RED);
  float* SLm = (float*)(smem + L_SL);
  float* SL1 = SLm + 64;
  float* SL2 = SLm + 128;

  // ---- fc1 slice: lane-owned (rows n = (2w+ii)*16 + fq*4 + r, column co = j*16 + fr) ----
  float wm[2][4][4], g1[2][4][4], g2[2][4][4];
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = (2 * w + ii) * 16 + fq * 4 + r, co = j * 16 + fr;
        const long ai = a.off[4] + (long)n * KIN + p * C2 + co;
        wm[ii][j][r] = a.master[ai];
        g1[ii][j][r] = a.s1[ai];
        g2[ii][j][r] = a.s2[ai];
        W1[n * W1S + co] = f2bf(wm[ii][j][r]);
      }
  // ---- conv parameters (every position needs all of them) ----
  auto put_conv = [&](int j, float v) {
    if (j < OFF_B2) W2[(j >> 7) * W2S + (j & 127)] = f2bf(v);
    else if (j < OFF_W1) CB2[j - OFF_B2] = v;
    else if (j < OFF_B1) CW1[j - OFF_W1] = v;
    else CB1[j - OFF_B1] = v;
  };
  {
    // every load in flight before the LDS stores: a load -> store loop waited out one memory round trip per
    // iteration (33 of them: the launch prologue measured 16 us, tools/persist_check.py "launch:")
    constexpr int NJ = (NCONV + 255) / 256;
    float cv[NJ];
#pragma unroll
    for (int q = 0; q < NJ; ++q) {
      const int j = tid + 256 * q;
      cv[q] = j < NCONV ? a.master[conv_idx(a, j)] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < NJ; ++q) {
      const int j = tid + 256 * q;
      if (j < NCONV) put_conv(j, cv[q]);
    }
  }
  const bool owner = p < NSLICE;
  if (owner && tid < SLICE) {
    const int e = p * SLICE + tid;
    if (e < NCONV) {
      const long ci = conv_idx(a, e);
      SLm[tid] = a.master[ci];
      SL1[tid] = a.s1[ci];
      SL2[tid] = a.s2[ci];
    }
  }
  // ---- input patch: thread -> (image xb, patch row xr, column pair xh) ----
  const int xb = tid >> 3, xr = (tid >> 1) & 3, xh = tid & 1;
  auto xload = [&](int s) -> unsigned {
    const long bt = (long)((cur0 + s) % a.nbatch);
    const unsigned char* q = a.xs + (bt * B + xb) * 784 + (2 * ph + xr) * 28 + 2 * pw + 2 * xh;
    return *(const unsigned short*)q;
  };
  unsigned xv = xload(0);
  const float P = a.drop_p, inv = P > 0.f ? 1.f / (1.f - P) : 1.f;
  unsigned char* KEEP = smem + L_KEEP;
  // the dropout keep mask of step s for this position (common.h drop_key / uniform01 on the NHWC
  // index of the pooled element): it depends only on the step, so it is drawn while the previous
  // step waits for its D hand-off, off the critical path
  auto draw_keep = [&](int s) {
    const unsigned long long ctr = ctr0 + (unsigned long long)s;
    const uint64_t dkey = (uint64_t)seed ^ ((uint64_t)a.salt * 0xD1B54A32D192ED03ull) ^
                          ((uint64_t)ctr * 0x8CB92BA72F3D8DD7ull);
    for (int e = threadIdx.x; e < B * C2; e += 256) {
      const int b = e >> 6, co = e & 63;
      const long gb = (long)a.rank * B + b;  // global image index: every replica draws its own masks
      KEEP[e] = P > 0.f ? (unsigned char)(uniform01(dkey, (uint64_t)((gb * NPOS + p) * C2 + co)) >= P) : 1;
    }
  };
  draw_keep(0);
  __syncthreads();

  for (int s = 0; s < a.nsteps; ++s) {
    const unsigned ep = (unsigned)(eb + (unsigned long long)s + 1ull);
    const int par = s & 1;
    // lane indices re-derived from an opaque zero every step: otherwise the compiler hoists every
    // LDS address of the step body out of the loop and runs out of registers (spills to scratch)
    int oz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
    const int tid = threadIdx.x + oz, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
    const int tq = fr >> 2, tp = fr & 3, xb = tid >> 3, xr = (tid >> 1) & 3, xh = tid & 1;
    stamp(a, s, 0);
    XIN[xb * 16 + xr * 4 + 2 * xh] = (float)(xv & 0xFFu) * a.xscale + a.xshift;
    XIN[xb * 16 + xr * 4 + 2 * xh + 1] = (float)(xv >> 8) * a.xscale + a.xshift;
    __syncthreads();
    // ---- conv1 (VALU): 32 images x 3x3 positions x 32 channels ----
    {
      const int ci = tid & 31, bg = tid >> 5;
      const float k0 = CW1[ci * 4 + 0], k1 = CW1[ci * 4 + 1], k2 = CW1[ci * 4 + 2], k3 = CW1[ci * 4 + 3];
      const float bias = CB1[ci];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int b = bg * 4 + u;
        const float* xi = XIN + b * 16;
#pragma unroll
        for (int py = 0; py < 3; ++py)
#pragma unroll
          for (int px = 0; px < 3; ++px) {
            float v = bias;
            v = fmaf(xi[py * 4 + px], k0, v);
            v = fmaf(xi[py * 4 + px + 1], k1, v);
            v = fmaf(xi[(py + 1) * 4 + px], k2, v);
            v = fmaf(xi[(py + 1) * 4 + px + 1], k3, v);
            C1[(b * 9 + py * 3 + px) * C1S + ci] = f2bf(fmaxf(v, 0.f));
          }
      }
    }
    __syncthreads();
    // ---- conv2 (MFMA, rows (b, q) = b*4 + q, k = tap*32 + ci) + bias + relu + max-pool + dropout ----
    {
      f32x4 acc[2][4];
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ii][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int di = kk >> 1, dj = kk & 1;
        bf16x8 af[2];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int b = 4 * (2 * w + ii) + (fr >> 2), q = fr & 3;
          const int pos = ((q >> 1) + di) * 3 + (q & 1) + dj;
          af[ii] = lds8(C1 + (b * 9 + pos) * C1S + fq * 8);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8 bfr = lds8(W2 + (j * 16 + fr) * W2S + kk * 32 + fq * 8);
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) acc[ii][j] = mfma(af[ii], bfr, acc[ii][j]);
        }
      }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int b = 4 * (2 * w + ii) + fq, co = j * 16 + fr;
          const float bias = CB2[co];
          float best = -INFINITY;
          int bi = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = bf2f(f2bf(fmaxf(acc[ii][j][r] + bias, 0.f)));  // bf16 conv output, as unfused
            if (v > best) {
              best = v;
              bi = r;
            }
          }
          if (!(best > 0.f)) bi = 0xFF;
          if (KEEP[b * C2 + co]) {
            best *= inv;
          } else {
            best = 0.f;
            bi = 0xFF;
          }
          POOL[b * PLS + co] = f2bf(best);
          AM[b * C2 + co] = (unsigned char)bi;
        }
    }
    __syncthreads();
    stamp(a, s, 1);
    // ---- fc1 partial product over this position's 64 inputs: part[b][n] ----
    {
      f32x4 acc[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = lds8(POOL + (i * 16 + fr) * PLS + kk * 32 + fq * 8);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) bfr[jj] = lds8(W1 + ((2 * w + jj) * 16 + fr) * W1S + kk * 32 + fq * 8);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mfma(af[i], bfr[jj], acc[i][jj]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) STG[(i * 16 + fq * 4 + r) * HID + (2 * w + jj) * 16 + fr] = acc[i][jj][r];
    }
    __syncthreads();
    {  // publish A
      const auto R = rsrc(a.slabA + ((long)par * NPOS + p) * (B * HID));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = tid + 256 * k;
        st_sc1(R, idx * 16, *(const f32x4*)(STG + idx * 4));
      }
      drain();
      __syncthreads();
      if (tid == 0) flag_store(a.flags + FL_A + p, ep);
    }
    const unsigned gep = (unsigned)(xs0 + s + 1);  // cross-rank epoch (grows across launches)
    if constexpr (DP) {
      // push this position's pooled activations to every peer, already in the fc1-wgrad B-fragment
      // layout (wave w: column block j = w; k = image), for the peers' fc1 weight gradient at the end
      // of the step; off the critical path (the peers read them after their conv backward)
      const int c0 = w * 16 + 4 * tp;
      const f32x4 f = __builtin_bit_cast(f32x4, lds_tr(POOL + (8 * fq + tq) * PLS + c0, POOL + (8 * fq + tq + 4) * PLS + c0));
      for (int r = 0; r < a.world; ++r) {
        if (r == a.rank) continue;
        st_sys(rsrc(a.xbuf[r] + XO_POOL + (par * XMAX + xslot(a, r)) * XS_POOL + (long)p * 4096), (w * 64 + lane) * 16, f);
      }
      // (flags raised after the B wait: by then the stores have long completed, so the drain is free)
    }
    if (s + 1 < a.nsteps) xv = xload(s + 1);  // next step's patch, consumed next iteration
    stamp(a, s, 2);
    // ---- B: dh of all 32 images ----
    // (step 0: the heads run on this GPU only, so a B that has not come within tmo0 means workgroups of
    // this launch are not resident — fail fast with the co-residency code instead of waiting out tmo)
    if (!wait_all(a.flags + FL_B, NHEAD, ep, a.err, s ? ecode(2, s) : ecode(12, 0), a.acquire, s_ok,
                  s ? a.tmo : a.tmo0, a.pollw_b, a.stagger))
      return;
    if constexpr (DP) {
      drain();
      __syncthreads();
      if (tid < 64) raise_peers(a, XF_POOL + p, NPOS, gep);
    }
    stamp(a, s, 3);
    {
      const auto R = rsrc(a.slabB + (long)par * NHEAD * PAY);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = tid + 256 * k, b = idx >> 5, n4 = idx & 31;
        const f32x4 v = ld_sc1(R, (b * PAY + PAY_DH + n4 * 4) * 4);
        *(bf16x4*)(DH + b * DHS + n4 * 4) =
            (bf16x4){(short)f2bf(v[0]), (short)f2bf(v[1]), (short)f2bf(v[2]), (short)f2bf(v[3])};
      }
    }
    __syncthreads();
    // ---- fc1 weight gradient (lane-owned layout) and input gradient ----
    f32x4 gw[2][4], dp[2];
    {
      // data parallel: the weight gradient sums every replica's images in rank order at the end of
      // the step (below); here only the input gradient
      if constexpr (!DP) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {  // A = dh^T (row n, k = b)
        const int n0 = (2 * w + ii) * 16 + 4 * tp;
        const bf16x8 af = lds_tr(DH + (8 * fq + tq) * DHS + n0, DH + (8 * fq + tq + 4) * DHS + n0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // B = pooled (col co, k = b)
          const int c0 = j * 16 + 4 * tp;
          const bf16x8 bfr = lds_tr(POOL + (8 * fq + tq) * PLS + c0, POOL + (8 * fq + tq + 4) * PLS + c0);
          gw[ii][j] = mfma(af, bfr, (f32x4){0.f, 0.f, 0.f, 0.f});
        }
      }
      }
      dp[0] = dp[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {  // A = dh (row b, k = n), B = W1^T (col co, k = n)
        const int k1 = kk * 32 + 8 * fq + tq;
        const bf16x8 bfr = lds_tr(W1 + k1 * W1S + w * 16 + 4 * tp, W1 + (k1 + 4) * W1S + w * 16 + 4 * tp);
#pragma unroll
        for (int i = 0; i < 2; ++i) dp[i] = mfma(lds8(DH + (i * 16 + fr) * DHS + kk * 32 + fq * 8), bfr, dp[i]);
      }
    }
    // (no barrier: the phases up to the C publish write neither DH, POOL nor W1)
    // ---- dropout / max-pool / relu backward -> dconv2[(b,q)][co]; conv2 bias gradient ----
    {
      const int co = w * 16 + fr;
      float db = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = i * 16 + fq * 4 + r;
          const int am = AM[b * C2 + co];
          const bf16_raw gb = am != 0xFF ? f2bf(dp[i][r] * inv) : (bf16_raw)0;
          db += bf2f(gb);
          // the image's 4 window taps are adjacent columns of row co: one 8-byte store
          *(bf16x4*)(DC2 + co * DCS + b * 4) = (bf16x4){(short)(am == 0 ? gb : 0), (short)(am == 1 ? gb : 0),
                                                        (short)(am == 2 ? gb : 0), (short)(am == 3 ? gb : 0)};
        }
      db += __shfl_xor(db, 16, 64);
      db += __shfl_xor(db, 32, 64);
      if (fq == 0) STG[OFF_B2 + co] = db;
    }
    __syncthreads();
    stamp(a, s, 4);
    // ---- conv2 weight gradient: dW2[co][(t,ci)] = sum_(b,q) dconv2[(b,q)][co] im2col[(b,q)][(t,ci)] ----
    {
      f32x4 acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k1 = kk * 32 + 8 * fq + tq, b1 = k1 >> 2, q1 = k1 & 3;  // k1 + 4 = image b1 + 1, same q
        const bf16x8 af = lds8(DC2 + (w * 16 + fr) * DCS + kk * 32 + fq * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int t = j >> 1, ci0 = (j & 1) * 16 + 4 * tp;
          const int pos = ((q1 >> 1) + (t >> 1)) * 3 + (q1 & 1) + (t & 1);
          const bf16x8 bfr = lds_tr(C1 + (b1 * 9 + pos) * C1S + ci0, C1 + ((b1 + 1) * 9 + pos) * C1S + ci0);
          acc[j] = mfma(af, bfr, acc[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) STG[(w * 16 + fq * 4 + r) * 128 + j * 16 + fr] = acc[j][r];
    }
    __syncthreads();
    {  // publish C, part 1: the conv2 weight gradient (8192 floats) now; its write-through stores drain
       // while the conv2 input gradient and the conv1 gradient below are computed
      const auto R = rsrc(a.slabC + ((long)par * NPOS + p) * NCONV);
#pragma unroll
      for (int k = 0; k < OFF_B2 / 4 / 256; ++k) {
        const int idx = tid + 256 * k;
        st_sc1(R, idx * 16, *(const f32x4*)(STG + idx * 4));
      }
    }
    // ---- conv2 input gradient -> col2im -> relu' -> conv1 weight / bias gradient ----
    {
      const int mh = w >> 1, h = w & 1;
      f32x4 acc[4][4];  // [M tile mh*4+i][tap t (N tile 2t+h)]
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4];
        const int k1 = kk * 32 + 8 * fq + tq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m0 = (mh * 4 + i) * 16 + 4 * tp;
          af[i] = lds_tr(DC2 + k1 * DCS + m0, DC2 + (k1 + 4) * DCS + m0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int c0 = (2 * t + h) * 16 + 4 * tp;
          const bf16x8 bfr = lds_tr(W2 + k1 * W2S + c0, W2 + (k1 + 4) * W2S + c0);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][t] = mfma(af[i], bfr, acc[i][t]);
        }
      }
      const int ci = h * 16 + fr;
      float gk[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 4 * (mh * 4 + i) + fq;
        float d[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) d[((q >> 1) + (t >> 1)) * 3 + (q & 1) + (t & 1)] += acc[i][t][q];
        const float* xi = XIN + b * 16;
#pragma unroll
        for (int py = 0; py < 3; ++py)
#pragma unroll
          for (int px = 0; px < 3; ++px) {
            const int pos = py * 3 + px;
            const float dd = (short)C1[(b * 9 + pos) * C1S + ci] > 0 ? d[pos] : 0.f;  // relu' of conv1
            gk[0] = fmaf(dd, xi[py * 4 + px], gk[0]);
            gk[1] = fmaf(dd, xi[py * 4 + px + 1], gk[1]);
            gk[2] = fmaf(dd, xi[(py + 1) * 4 + px], gk[2]);
            gk[3] = fmaf(dd, xi[(py + 1) * 4 + px + 1], gk[3]);
            gk[4] += dd;
          }
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        gk[k] += __shfl_xor(gk[k], 16, 64);
        gk[k] += __shfl_xor(gk[k], 32, 64);
      }
      if (fq == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) RED[(mh * 32 + ci) * 5 + k] = gk[k];
      }
    }
    __syncthreads();
    if (tid < 32 * 5) {
      const int ci = tid / 5, k = tid - ci * 5;
      const float v = RED[ci * 5 + k] + RED[(32 + ci) * 5 + k];
      if (k < 4) STG[OFF_W1 + ci * 4 + k] = v;
      else STG[OFF_B1 + ci] = v;
    }
    __syncthreads();
    stamp(a, s, 5);
    {  // publish C, part 2: the 224 small gradients [b2 | conv1 w | conv1 b]; every wave drains both parts
      const auto R = rsrc(a.slabC + ((long)par * NPOS + p) * NCONV);
      const int idx = OFF_B2 / 4 + tid;
      if (idx < NCONV / 4) st_sc1(R, idx * 16, *(const f32x4*)(STG + idx * 4));
      drain();
      __syncthreads();
      if (tid == 0) flag_store(a.flags + FL_C + p, ep);
    }
    stamp(a, s, 6);
    // ---- slice owners: fixed-order reduce of 52 params over the 169 partials, Adadelta, publish D ----
    if (owner) {
      if (!wait_all(a.flags + FL_C, NPOS, ep, a.err, ecode(3, s), a.acquire, s_ok, a.tmo, a.pollw_c, a.stagger)) return;
      stamp(a, s, 7);
      const int e0 = p * SLICE;
      if (tid < 13 * NRED) {
        const int j = tid % 13, g = tid / 13;
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (e0 + 4 * j < NCONV) {
          const auto R = rsrc(a.slabC + (long)par * NPOS * NCONV);
          constexpr int NK = (NPOS + NRED - 1) / NRED;  // 9 partials per thread, all in flight
          f32x4 v[NK];
#pragma unroll
          for (int k = 0; k < NK; ++k) {
            const int pp = g + NRED * k;
            v[k] = pp < NPOS ? ld_sc1(R, (pp * NCONV + e0 + 4 * j) * 4) : (f32x4){0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int k = 0; k < NK; ++k) acc += v[k];
        }
        *(f32x4*)(RED + g * SLICE + 4 * j) = acc;
      }
      __syncthreads();
      const int e = e0 + tid;
      float gs = 0.f;
      if (tid < SLICE) {
        for (int g = 0; g < NRED; ++g) gs += RED[g * SLICE + tid];
      }
      if constexpr (DP) {
        // this rank's slice sum to every peer, then every replica's, summed in rank order (identical
        // on every rank, so the replicas stay bit-identical)
        if (tid < 64) {
          if (tid < SLICE) {
            for (int r = 0; r < a.world; ++r) {
              if (r == a.rank) continue;
              st_sys1(rsrc(a.xbuf[r] + XO_CONV + (par * XMAX + xslot(a, r)) * XS_CONV), e * 4, gs);
            }
          }
          drain();
          raise_peers(a, XF_CONV + p, NSLICE, gep);
        }
        if (!wait_peers(a, XF_CONV + p, NSLICE, gep, ecode(6, s), s_ok)) return;
        if (tid < SLICE) {
          const auto X = rsrc(a.xbuf[a.rank] + XO_CONV + (long)par * XMAX * XS_CONV);
          float v[XMAX];  // every peer's value in flight before the rank-order sum
#pragma unroll
          for (int r = 0; r < XMAX; ++r) v[r] = r < a.world && r != a.rank ? ld_sys1(X, (int)(r * XS_CONV) + e * 4) : gs;
          float t = 0.f;
#pragma unroll
          for (int r = 0; r < XMAX; ++r)
            if (r < a.world) t += v[r];
          gs = t;
        }
      }
      if (tid < SLICE) {  // wave 0
        float wn = 0.f;
        if (e < NCONV) {
          SLm[tid] = adadelta(SLm[tid], gs * hp.gscale, SL1[tid], SL2[tid], hp);
          wn = SLm[tid];
        }
        // the D payload: conv2 weights as bf16 pairs (slices start at even indices), the rest fp32; every
        // store a 4-byte write-through (sc1) store
        const float wnext = __shfl_down(wn, 1, 64);
        unsigned char* D = (unsigned char*)a.slabD + (long)par * D_BYTES;
        if (e < OFF_B2) {
          if (!(tid & 1))
            __hip_atomic_store((gu32*)(D + e * 2), (unsigned)f2bf(wn) | ((unsigned)f2bf(wnext) << 16),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (e < NCONV) {
          __hip_atomic_store((gu32*)(D + D_F32 + (e - OFF_B2) * 4), __float_as_uint(wn), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (w == 0) {
        drain();
        if (lane == 0) flag_store(a.flags + FL_D + p, ep);
      }
      stamp(a, s, 8);
    }
    if constexpr (DP) {
      // ---- fc1 weight gradient over every replica's images: dh^T fragments (each rank's head 0) and
      // pooled fragments (each rank's position p); one MFMA product per replica, summed in rank order
      // (the per-replica gradients, added exactly as an all-reduce in rank order would).  After the
      // owner phase: placed before the owners' C wait it delayed the D publish (measured +2 us at 8
      // loopback ranks: the exchange-buffer loads take longer than that wait) ----
      if (!wait_peers(a, XF_H, 1, gep, ecode(7, s), s_ok)) return;
      if (!wait_peers(a, XF_POOL + p, NPOS, gep, ecode(8, s), s_ok)) return;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) gw[ii][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      const auto XP = rsrc(a.xbuf[a.rank] + XO_POOL + (long)par * XMAX * XS_POOL + (long)p * 4096);
      const auto XD = rsrc(a.xbuf[a.rank] + XO_DHT + (long)par * XMAX * XS_DHT);
      // rank r's fragments: own from LDS, a peer's from this rank's exchange buffer; loaded two ranks
      // ahead of the MFMAs that consume them (three register sets, indices fixed by the unrolled loop;
      // four — three peers' loads in flight — measured no faster at 8 loopback ranks: 34.2 vs 33.6 us/step)
      constexpr int PF = 3;
      bf16x8 af[PF][2], bfr[PF][4];
      auto fetch = [&](int r, int b) {
        if (r == a.rank) {
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) {
            const int n0 = (2 * w + ii) * 16 + 4 * tp;
            af[b][ii] = lds_tr(DH + (8 * fq + tq) * DHS + n0, DH + (8 * fq + tq + 4) * DHS + n0);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c0 = j * 16 + 4 * tp;
            bfr[b][j] = lds_tr(POOL + (8 * fq + tq) * PLS + c0, POOL + (8 * fq + tq + 4) * PLS + c0);
          }
        } else {
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
            af[b][ii] = __builtin_bit_cast(bf16x8, ld_sys(XD, (int)(r * XS_DHT) + ((2 * w + ii) * 64 + lane) * 16));
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bfr[b][j] = __builtin_bit_cast(bf16x8, ld_sys(XP, (int)(r * XS_POOL) + (j * 64 + lane) * 16));
        }
      };
#pragma unroll
      for (int r = 0; r < PF - 1; ++r)
        if (r < a.world) fetch(r, r);
#pragma unroll
      for (int r = 0; r < XMAX; ++r) {
        if (r < a.world) {
          if (r + PF - 1 < XMAX && r + PF - 1 < a.world) fetch(r + PF - 1, (r + PF - 1) % PF);
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              gw[ii][j] += mfma(af[r % PF][ii], bfr[r % PF][j], (f32x4){0.f, 0.f, 0.f, 0.f});
        }
      }
    }
    // ---- Adadelta on the fc1 slice (registers) and the new bf16 weights for the next forward: off the
    // critical path, while this workgroup waits for the D hand-off (W1 is next read after it) ----
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          wm[ii][j][r] = adadelta(wm[ii][j][r], gw[ii][j][r] * hp.gscale, g1[ii][j][r], g2[ii][j][r], hp);
          W1[((2 * w + ii) * 16 + fq * 4 + r) * W1S + j * 16 + fr] = f2bf(wm[ii][j][r]);
        }
    if (s + 1 < a.nsteps) draw_keep(s + 1);  // KEEP is next read after the D wait's barrier
    stamp(a, s, 9);
    // ---- D: the updated conv parameters for the next step ----
    if (!wait_all(a.flags + FL_D, NSLICE, ep, a.err, ecode(4, s), a.acquire, s_ok, a.tmo, a.pollw_d, a.stagger)) return;
    stamp(a, s, 10);
    {
      const auto R = rsrc((const unsigned char*)a.slabD + (long)par * D_BYTES);
      constexpr int NB = OFF_B2 * 2 / 16;        // 1024 16-B chunks of bf16 conv2 weights
      constexpr int NF = (NCONV - OFF_B2) / 4;   // 56 16-B chunks of fp32
      f32x4 dv[NB / 256 + 1];
#pragma unroll
      for (int k = 0; k < NB / 256; ++k) dv[k] = ld_sc1(R, (tid + 256 * k) * 16);
      dv[NB / 256] = tid < NF ? ld_sc1(R, D_F32 + tid * 16) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NB / 256; ++k) {
        const int c = tid + 256 * k;  // chunk c: conv2 row c >> 4, 8 values from column (c & 15) * 8
        *(f32x4*)(W2 + (c >> 4) * W2S + (c & 15) * 8) = dv[k];
      }
      if (tid < NF) {
        const int j = OFF_B2 + tid * 4;  // 4 params never straddle a region (8256, 8384 are multiples of 4)
        float* dst = j < OFF_W1 ? CB2 + (j - OFF_B2) : (j < OFF_B1 ? CW1 + (j - OFF_W1) : CB1 + (j - OFF_B1));
        *(f32x4*)dst = dv[NB / 256];
      }
    }
    __syncthreads();
    stamp(a, s, 11);
  }

  // ---- write back: fc1 slice and the owned conv slice (master, state, bf16 shadow) ----
#pragma unroll
  for (int ii = 0; ii < 2; ++ii)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = (2 * w + ii) * 16 + fq * 4 + r, co = j * 16 + fr;
        const long ai = a.off[4] + (long)n * KIN + p * C2 + co;
        a.master[ai] = wm[ii][j][r];
        a.s1[ai] = g1[ii][j][r];
        a.s2[ai] = g2[ii][j][r];
        a.shadow[ai] = f2bf(wm[ii][j][r]);
      }
  if (owner && tid < SLICE) {
    const int e = p * SLICE + tid;
    if (e < NCONV) {
      const long ci = conv_idx(a, e);
      a.master[ci] = SLm[tid];
      a.s1[ci] = SL1[tid];
      a.s2[ci] = SL2[tid];
      a.shadow[ci] = f2bf(SLm[tid]);
    }
  }
  stamp(a, a.nsteps - 1, 14);  // (debug stamps: write-back issued)
  // every workgroup has started (D of the last step needs C of every position, which needs B of
  // every head): the run-state words can advance
  if (p == 0 && tid == 0) {
    if constexpr (DP) a.xstep[0] = xs0 + a.nsteps;
    a.cursor[0] = (cur0 + a.nsteps) % a.nbatch;
    *(unsigned long long*)(a.flags + FL_EPOCH) = eb + (unsigned long long)a.nsteps;
    a.rng[1] = ctr0 + (unsigned long long)a.nsteps;
    if (a.step_dev) a.step_dev[0] += (float)a.nsteps;
  }
}

// ------------------------------------------------------------------------------------------------
// head workgroup i (image i): fc1 reduce + bias + relu, Dense10, softmax CE, dh; replicated
// fc2 / fc1-bias Adadelta from all 32 payloads
// ------------------------------------------------------------------------------------------------
template <bool DP>
__device__ __forceinline__ void head_wg(const Args& a, unsigned char* smem, int* s_ok, const OptHP& hp,
                                        long long cur0, long long xs0, unsigned long long eb) {
  const int i = blockIdx.x - NPOS;
  const int tid = threadIdx.x, lane = tid & 63;
  float* HW = (float*)(smem + H_W2);
  float* HW1 = HW + NCLS * HID;
  float* HW2 = HW1 + NCLS * HID;
  float* HB2 = (float*)(smem + H_B2);  // [0,16) master [16,32) s1 [32,48) s2
  float* HB1 = (float*)(smem + H_B1);  // [0,128) master [128,256) s1 [256,384) s2
  float* RED = (float*)(smem + H_RED);
  float* HH = (float*)(smem + H_H);
  float* LOG = (float*)(smem + H_LOG);
  float* PAYL = (float*)(smem + H_PAY);
  float* ALL = (float*)(smem + H_ALL);
  {
    constexpr int NJ = NCLS * HID / 256;  // (all loads in flight before the LDS stores)
    float v0[NJ], v1[NJ], v2[NJ];
#pragma unroll
    for (int q = 0; q < NJ; ++q) {
      const long ai = a.off[6] + tid + 256 * q;
      v0[q] = a.master[ai];
      v1[q] = a.s1[ai];
      v2[q] = a.s2[ai];
    }
#pragma unroll
    for (int q = 0; q < NJ; ++q) {
      HW[tid + 256 * q] = v0[q];
      HW1[tid + 256 * q] = v1[q];
      HW2[tid + 256 * q] = v2[q];
    }
  }
  if (tid < NCLS) {
    const long ai = a.off[7] + tid;
    HB2[tid] = a.master[ai];
    HB2[16 + tid] = a.s1[ai];
    HB2[32 + tid] = a.s2[ai];
  }
  if (tid < HID) {
    const long ai = a.off[5] + tid;
    HB1[tid] = a.master[ai];
    HB1[128 + tid] = a.s1[ai];
    HB1[256 + tid] = a.s2[ai];
  }
  if (tid == 0) {
    PAYL[266] = PAYL[267] = PAYL[270] = PAYL[271] = 0.f;
  }
  __syncthreads();

  for (int s = 0; s < a.nsteps; ++s) {
    const unsigned ep = (unsigned)(eb + (unsigned long long)s + 1ull);
    const int par = s & 1;
    const int y = (int)a.ys[((cur0 + s) % a.nbatch) * B + i];
    // ---- A: reduce the 169 fc1 partial rows of image i (fixed order) ----
    if (!wait_all(a.flags + FL_A, NPOS, ep, a.err, s ? ecode(1, s) : ecode(12, 0), a.acquire, s_ok,
                  s ? a.tmo : a.tmo0, a.pollw_a, a.stagger))
      return;
    stamp(a, s, 0);
    {
      const int n4 = tid & 31, g = tid >> 5;
      const auto R = rsrc(a.slabA + (long)par * NPOS * B * HID);
      // all 22 loads in flight before the (fixed-order) sum: a load -> add chain serialises 22 L2 trips
      constexpr int NK = (NPOS + 7) / 8;
      f32x4 v[NK];
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const int pp = g + 8 * k;
        v[k] = pp < NPOS ? ld_sc1(R, ((pp * B + i) * HID + n4 * 4) * 4) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      f32x4 acc = v[0];
#pragma unroll
      for (int k = 1; k < NK; ++k) acc += v[k];
      *(f32x4*)(RED + g * HID + n4 * 4) = acc;
    }
    __syncthreads();
    if (a.head1w) {
      // one wave does the whole head from registers (HOPSX_PERSIST_HEAD1W): lane l owns hidden units 2l,
      // 2l+1, the 10 logits are wave sums, softmax / dlogits / dh in registers, and the B payload leaves
      // as 8-B write-through stores from this wave alone (its drain then its flag: no barrier, no LDS
      // round trip) — four barriers and three LDS passes off the critical A -> B chain
      if (tid < 64) {
        const int n0 = 2 * lane;
        float h[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float v = 0.f;
#pragma unroll
          for (int g = 0; g < 8; ++g) v += RED[g * HID + n0 + u];
          h[u] = fmaxf(v + HB1[n0 + u], 0.f);
        }
        float z[NCLS];
#pragma unroll
        for (int c = 0; c < NCLS; ++c)
          z[c] = wave_sum(fmaf(h[1], HW[c * HID + n0 + 1], h[0] * HW[c * HID + n0])) + HB2[c];
        float m = z[0];
#pragma unroll
        for (int c = 1; c < NCLS; ++c) m = fmaxf(m, z[c]);
        float e[NCLS], se = 0.f, zy = 0.f;
        int am = NCLS;
#pragma unroll
        for (int c = NCLS - 1; c >= 0; --c) {
          e[c] = __expf(z[c] - m);
          if (z[c] == m) am = c;  // the first maximum
          if (c == y) zy = z[c];
        }
#pragma unroll
        for (int c = 0; c < NCLS; ++c) se += e[c];
        const float inv_se = 1.f / se;
        float dl[NCLS];
#pragma unroll
        for (int c = 0; c < NCLS; ++c) dl[c] = (e[c] * inv_se - (c == y ? 1.f : 0.f)) * a.inv_gb;
        float dh[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float d = 0.f;
#pragma unroll
          for (int c = 0; c < NCLS; ++c) d = fmaf(dl[c], HW[c * HID + n0 + u], d);
          dh[u] = h[u] > 0.f ? d : 0.f;
        }
        const auto R = rsrc(a.slabB + ((long)par * NHEAD + i) * PAY);
        st_sc1x2(R, (PAY_DH + n0) * 4, dh[0], dh[1]);
        st_sc1x2(R, (PAY_H + n0) * 4, h[0], h[1]);
        float p0 = 0.f, p1 = 0.f;
#pragma unroll
        for (int c = 0; c < NCLS; c += 2)
          if (lane == c / 2) {
            p0 = dl[c];
            p1 = dl[c + 1];
          }
        if (lane < NCLS / 2) st_sc1x2(R, (PAY_DL + 2 * lane) * 4, p0, p1);
        if (lane == NCLS / 2) st_sc1x2(R, PAY_LOSS * 4, __logf(se) + m - zy, am == y ? 1.f : 0.f);
        drain();
        if (lane == 0) flag_store(a.flags + FL_B + i, ep);
      }
    }
    if (!a.head1w) {
    if (tid < HID) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v += RED[g * HID + tid];
      HH[tid] = fmaxf(v + HB1[tid], 0.f);
    }
    __syncthreads();
    {  // logits: 16 lanes per class
      const int c = tid >> 4, part = tid & 15;
      float v = 0.f;
      if (c < NCLS) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v = fmaf(HH[part + 16 * k], HW[c * HID + part + 16 * k], v);
      }
      v = row_fold<1>(v);
      if (part == 0 && c < NCLS) LOG[c] = v + HB2[c];
    }
    __syncthreads();
    if (tid < 64) {  // softmax cross-entropy of image i (mean over the batch: 1/B)
      const float z = lane < NCLS ? LOG[lane] : -INFINITY;
      const float m = wave_max(z);
      const float e = lane < NCLS ? __expf(z - m) : 0.f;
      const float se = wave_sum(e);
      const unsigned long long hit = __ballot(lane < NCLS && z == m);
      const int am = __ffsll((long long)hit) - 1;
      if (lane < NCLS) PAYL[PAY_DL + lane] = (e / se - (lane == y ? 1.f : 0.f)) * a.inv_gb;
      if (lane == 0) {
        PAYL[PAY_LOSS] = __logf(se) + m - LOG[y];
        PAYL[PAY_COR] = am == y ? 1.f : 0.f;
      }
    }
    __syncthreads();
    if (tid < HID) {
      const float h = HH[tid];
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) d = fmaf(PAYL[PAY_DL + c], HW[c * HID + tid], d);
      PAYL[PAY_DH + tid] = h > 0.f ? d : 0.f;
      PAYL[PAY_H + tid] = h;
    }
    __syncthreads();
    {  // publish B
      const auto R = rsrc(a.slabB + ((long)par * NHEAD + i) * PAY);
      if (tid < PAY / 4) st_sc1(R, tid * 16, *(const f32x4*)(PAYL + tid * 4));
      drain();
      __syncthreads();
      if (tid == 0) flag_store(a.flags + FL_B + i, ep);
    }
    }
    stamp(a, s, 1);
    // ---- replicated fc2 / fc1-bias update from every image's payload ----
    if (!wait_all(a.flags + FL_B, NHEAD, ep, a.err, s ? ecode(5, s) : ecode(12, 0), a.acquire, s_ok,
                  s ? a.tmo : a.tmo0, a.pollw, a.stagger))
      return;
    {
      const auto R = rsrc(a.slabB + (long)par * NHEAD * PAY);
      constexpr int NK = (NHEAD * PAY / 4 + 255) / 256;
      f32x4 v[NK];
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const int idx = tid + 256 * k;
        v[k] = idx < NHEAD * PAY / 4 ? ld_sc1(R, idx * 16) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const int idx = tid + 256 * k;
        if (idx < NHEAD * PAY / 4) *(f32x4*)(ALL + idx * 4) = v[k];
      }
    }
    __syncthreads();
    // this replica's fc2 / fc1-bias / fc2-bias gradients: element tid + 256 k of fc2.weight (k < 5),
    // fc1.bias[tid], fc2.bias[tid]
    constexpr int NW = NCLS * HID / 256;
    static_assert(NCLS * HID == NW * 256, "fc2 weight split");
    float gl[NW + 2];
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int j = tid + 256 * k, c = j / HID, n = j - c * HID;
      float g = 0.f;
#pragma unroll 8
      for (int b = 0; b < B; ++b) g = fmaf(ALL[b * PAY + PAY_DL + c], ALL[b * PAY + PAY_H + n], g);
      gl[k] = g;
    }
    gl[NW] = gl[NW + 1] = 0.f;
    if (tid < HID) {
#pragma unroll 8
      for (int b = 0; b < B; ++b) gl[NW] += ALL[b * PAY + PAY_DH + tid];
    }
    if (tid < NCLS) {
      for (int b = 0; b < B; ++b) gl[NW + 1] += ALL[b * PAY + PAY_DL + tid];
    }
    if constexpr (DP) {
      const unsigned gep = (unsigned)(xs0 + s + 1);
      if (i == 0) {
        // head 0 pushes this replica's head gradients and dh^T (fc1-wgrad A fragments, bf16, the layout
        // the position workgroups read from their own LDS) to every peer
        bf16_raw* DS = (bf16_raw*)(smem + H_DHS);
        for (int e = tid; e < B * HID; e += 256) DS[(e >> 7) * DHS + (e & 127)] = f2bf(ALL[(e >> 7) * PAY + PAY_DH + (e & 127)]);
        __syncthreads();
        const int w = tid >> 6, fr = lane & 15, fq = lane >> 4, tq = fr >> 2, tp = fr & 3;
        f32x4 fd[2];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int n0 = (2 * w + ii) * 16 + 4 * tp;
          fd[ii] = __builtin_bit_cast(f32x4, lds_tr(DS + (8 * fq + tq) * DHS + n0, DS + (8 * fq + tq + 4) * DHS + n0));
        }
        for (int r = 0; r < a.world; ++r) {
          if (r == a.rank) continue;
          const int sl = xslot(a, r);
          const auto XG = rsrc(a.xbuf[r] + XO_FC2 + (par * XMAX + sl) * XS_FC2);
#pragma unroll
          for (int k = 0; k < NW; ++k) st_sys1(XG, (tid + 256 * k) * 4, gl[k]);
          if (tid < HID) st_sys1(XG, (NCLS * HID + tid) * 4, gl[NW]);
          if (tid < NCLS) st_sys1(XG, (NCLS * HID + HID + tid) * 4, gl[NW + 1]);
          const auto XD = rsrc(a.xbuf[r] + XO_DHT + (par * XMAX + sl) * XS_DHT);
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) st_sys(XD, ((2 * w + ii) * 64 + lane) * 16, fd[ii]);
        }
        drain();
        __syncthreads();
        if (tid < 64) raise_peers(a, XF_H, 1, gep);
      }
      if (!wait_peers(a, XF_H, 1, gep, ecode(9, s), s_ok)) return;
      // every replica's gradient, summed in rank order
      const auto X = rsrc(a.xbuf[a.rank] + XO_FC2 + (long)par * XMAX * XS_FC2);
      float t[NW + 2];
#pragma unroll
      for (int k = 0; k < NW + 2; ++k) t[k] = 0.f;
      float v[XMAX][NW + 2];  // every peer's gradients in flight before the rank-order sums
#pragma unroll
      for (int r = 0; r < XMAX; ++r) {
        const bool peer = r < a.world && r != a.rank;
        const int o = (int)(r * XS_FC2);
#pragma unroll
        for (int k = 0; k < NW; ++k) v[r][k] = peer ? ld_sys1(X, o + (tid + 256 * k) * 4) : gl[k];
        v[r][NW] = peer && tid < HID ? ld_sys1(X, o + (NCLS * HID + tid) * 4) : gl[NW];
        v[r][NW + 1] = peer && tid < NCLS ? ld_sys1(X, o + (NCLS * HID + HID + tid) * 4) : gl[NW + 1];
      }
#pragma unroll
      for (int r = 0; r < XMAX; ++r)
        if (r < a.world) {
#pragma unroll
          for (int k = 0; k < NW + 2; ++k) t[k] += v[r][k];
        }
#pragma unroll
      for (int k = 0; k < NW + 2; ++k) gl[k] = t[k];
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int j = tid + 256 * k;
      HW[j] = adadelta(HW[j], gl[k] * hp.gscale, HW1[j], HW2[j], hp);
    }
    if (tid < HID) HB1[tid] = adadelta(HB1[tid], gl[NW] * hp.gscale, HB1[128 + tid], HB1[256 + tid], hp);
    if (tid < NCLS) HB2[tid] = adadelta(HB2[tid], gl[NW + 1] * hp.gscale, HB2[16 + tid], HB2[32 + tid], hp);
    if (i == 0 && tid == 255) {
      float l = 0.f, cc = 0.f;
      for (int b = 0; b < B; ++b) {
        l += ALL[b * PAY + PAY_LOSS];
        cc += ALL[b * PAY + PAY_COR];
      }
      a.out[2 * s] = l * (1.f / B);
      a.out[2 * s + 1] = cc;
    }
    __syncthreads();
    stamp(a, s, 2);
  }
  if (i == 0) {
    for (int j = tid; j < NCLS * HID; j += 256) {
      const long ai = a.off[6] + j;
      a.master[ai] = HW[j];
      a.s1[ai] = HW1[j];
      a.s2[ai] = HW2[j];
      a.shadow[ai] = f2bf(HW[j]);
    }
    if (tid < NCLS) {
      const long ai = a.off[7] + tid;
      a.master[ai] = HB2[tid];
      a.s1[ai] = HB2[16 + tid];
      a.s2[ai] = HB2[32 + tid];
      a.shadow[ai] = f2bf(HB2[tid]);
    }
    if (tid < HID) {
      const long ai = a.off[5] + tid;
      a.master[ai] = HB1[tid];
      a.s1[ai] = HB1[128 + tid];
      a.s2[ai] = HB1[256 + tid];
      a.shadow[ai] = f2bf(HB1[tid]);
    }
  }
}

template <bool DP>
__global__ __launch_bounds__(256, 1) void mnist_persist_k(const Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_ok[2];  // [0] a wait's verdict, [1] the multi-wave wait's done word (wait_all)
  stamp(a, 0, 13);  // (debug stamps: workgroup entry, before the launch prologue)
  if (threadIdx.x == 0) s_ok[0] = s_ok[1] = 0;  // (read after the first barrier of either role)
  const OptHP hp = load_hp(a.hp, a.hp_dev);
  const long long cur0 = a.cursor[0];
  const long long xs0 = DP ? a.xstep[0] : 0;
  const unsigned long long eb = *(const unsigned long long*)(a.flags + FL_EPOCH);
  if (blockIdx.x < NPOS) {
    position_wg<DP>(a, smem, s_ok, hp, cur0, a.rng[0], a.rng[1], xs0, eb);
  } else {
    head_wg<DP>(a, smem, s_ok, hp, cur0, xs0, eb);
  }
}

}  // namespace mnistp

// ptrs: master shadow s1 s2 xs ys cursor rng step_dev hp_dev slabA slabB slabC slabD flags err out dbg(0 = none)
//       [xstep xbuf[world] xflag[world]]   (world > 1: the data-parallel instantiation)
// iv:   off[8] nbatch salt nsteps batch acquire world rank loopback timeout_ms xfence
// fv:   drop_p xscale xshift lr gscale wd rho eps
static int g_persist_reload = 0;
extern "C" void hopsx_mnist_persist_reload_knobs() { g_persist_reload = 1; }

extern "C" int hopsx_mnist_persist(const uint64_t* p, int np, const long* iv, int ni, const float* fv, int nf,
                                   hipStream_t st) {
  using namespace mnistp;
  if (np < 18 || ni < 18 || nf < 8) return (int)hipErrorInvalidValue;
  if (iv[11] != B || iv[10] < 1 || iv[8] < 1) return (int)hipErrorInvalidValue;
  const int world = (int)iv[13], rank = (int)iv[14];
  if (world < 1 || world > XMAX || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
  const bool dp = world > 1;
  if (dp && np < 19 + 2 * world) return (int)hipErrorInvalidValue;
  Args a{};
  a.master = (float*)p[0];
  a.shadow = (bf16_raw*)p[1];
  a.s1 = (float*)p[2];
  a.s2 = (float*)p[3];
  a.xs = (const unsigned char*)p[4];
  a.ys = (const long long*)p[5];
  a.cursor = (long long*)p[6];
  a.rng = (unsigned long long*)p[7];
  a.step_dev = (float*)p[8];
  a.hp_dev = (const float*)p[9];
  a.slabA = (float*)p[10];
  a.slabB = (float*)p[11];
  a.slabC = (float*)p[12];
  a.slabD = (float*)p[13];
  a.flags = (unsigned*)p[14];
  a.err = (unsigned*)p[15];
  a.out = (float*)p[16];
  a.dbg = (unsigned long long*)p[17];
  for (int k = 0; k < 8; ++k) a.off[k] = iv[k];
  a.nbatch = iv[8];
  a.salt = (unsigned)iv[9];
  a.nsteps = (int)iv[10];
  a.acquire = (int)iv[12];
  a.world = world;
  a.rank = rank;
  a.loopback = (int)iv[15];
  a.xfence = (int)iv[17];
  a.tmo = (long long)iv[16] * 100000ll;  // ms -> 100 MHz ticks
  a.tmo0 = a.tmo;
  // launch knobs (environment), read once and again after hopsx_mnist_persist_reload_knobs (tools/persist_ab.py)
  static int kn_ok = 0, kn_pollw, kn_stagger, kn_a, kn_b, kn_c, kn_d, kn_head1w, kn_memset, kn_coop;
  static long kn_start_ms;
  if (!kn_ok || g_persist_reload) {
    auto pw = [&](const char* name, long dflt) {
      const long v = hopsx_env_int(name, dflt);
      return (int)(v >= 1 && v <= 4 ? v : 1);
    };
    kn_pollw = pw("HOPSX_PERSIST_POLLW", 1);
    kn_stagger = (int)hopsx_env_int("HOPSX_PERSIST_STAGGER", 12);
    // per hand-off: the slice owners' wait on the 169 conv-gradient partials polls from 4 waves by default
    // (C hop 2.6 -> 1.9 us, 27.6 -> 26.0 us/step: profiles/r5_persist_pollw_ab.txt); the same on the other
    // waits measured slower (more pollers on the flag lines)
    kn_a = pw("HOPSX_PERSIST_POLLW_A", kn_pollw);
    kn_b = pw("HOPSX_PERSIST_POLLW_B", kn_pollw);
    kn_c = pw("HOPSX_PERSIST_POLLW_C", 4);
    kn_d = pw("HOPSX_PERSIST_POLLW_D", kn_pollw);
    kn_head1w = (int)hopsx_env_int("HOPSX_PERSIST_HEAD1W", 1);  // 25.8 -> 25.5 us/step (same profile)
    kn_memset = (int)hopsx_env_int("HOPSX_PERSIST_MEMSET", 0);  // (the round-4 form, for A/B)
    // co-residency: step 0's local hand-offs give up after HOPSX_PERSIST_START_MS (every workgroup starts
    // within microseconds when the grid is resident; anything else means a concurrent kernel holds CUs the
    // grid needs): measured 50 ms to the co-residency error with a kernel holding 128 CUs, instead of the
    // 2 s / 60 s hand-off timeout.  HOPSX_PERSIST_COOP=1 launches cooperatively instead: ROCm then checks
    // the grid against the device's capacity only (what launchable() already does), not against kernels
    // already resident, and costs 0.6 us/step at 32 steps per launch (1.226M -> 1.200M img/s,
    // profiles/r6_persist_dp_sim.txt), so it is off by default
    kn_coop = (int)hopsx_env_int("HOPSX_PERSIST_COOP", 0);
    kn_start_ms = hopsx_env_int("HOPSX_PERSIST_START_MS", 50);
    kn_ok = 1;
    g_persist_reload = 0;
  }
  a.pollw = kn_pollw;
  a.stagger = kn_stagger;
  a.pollw_a = kn_a;
  a.pollw_b = kn_b;
  a.pollw_c = kn_c;
  a.pollw_d = kn_d;
  a.head1w = kn_head1w;
  if (kn_start_ms > 0 && kn_start_ms * 100000ll < a.tmo) a.tmo0 = kn_start_ms * 100000ll;
  a.inv_gb = 1.f / (float)(world * B);
  if (dp) {
    a.xstep = (long long*)p[18];
    for (int r = 0; r < world; ++r) {
      a.xbuf[r] = (unsigned char*)p[19 + r];
      a.xflag[r] = (unsigned*)p[19 + world + r];
      if (!a.xbuf[r] || !a.xflag[r] || ((uint64_t)a.xbuf[r] & 15)) return (int)hipErrorInvalidValue;
    }
  }
  a.drop_p = fv[0];
  a.xscale = fv[1];
  a.xshift = fv[2];
  a.hp = OptHP{fv[3], fv[4], fv[5], fv[6], fv[7], 0.f, 0.f, 0.f};
  static bool attr[2] = {false, false};
  const void* fn = dp ? (const void*)mnist_persist_k<true> : (const void*)mnist_persist_k<false>;
  if (!attr[dp]) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr[dp] = true;
  }
  if (kn_memset) {  // (the round-4 form, for A/B: zeroed flags each launch)
    const hipError_t e = hipMemsetAsync(a.flags, 0, FL_WORDS * sizeof(unsigned), st);
    if (e != hipSuccess) return (int)e;
  }
  if (kn_coop) {
    // cooperative launch: refused at once (hipErrorCooperativeLaunchTooLarge) when the device cannot hold
    // all GRID workgroups together, instead of workgroups spinning on hand-offs that cannot come
    void* kargs[] = {(void*)&a};
    const hipError_t e = hipLaunchCooperativeKernel(fn, dim3(GRID), dim3(256), kargs, LDS_BYTES, st);
    if (e != hipSuccess) {
      (void)hipGetLastError();  // clear the sticky launch error; the caller raises on the return code
      return (int)e;
    }
    return (int)hipSuccess;
  }
  if (dp)
    hipLaunchKernelGGL(mnist_persist_k<true>, dim3(GRID), dim3(256), LDS_BYTES, st, a);
  else
    hipLaunchKernelGGL(mnist_persist_k<false>, dim3(GRID), dim3(256), LDS_BYTES, st, a);
  return (int)hipGetLastError();
}

// Workgroups of the persistent kernel one CU can hold at once (registers, LDS, wave slots): the
// launch hands data between workgroups, so all GRID of them must be co-resident — the host requires
// this >= 1 and CUs >= GRID before it picks the persistent engine (runtime/persist.py launchable()).
extern "C" int hopsx_mnist_persist_occupancy(int dp) {
  using namespace mnistp;
  const void* fn = dp ? (const void*)mnist_persist_k<true> : (const void*)mnist_persist_k<false>;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) != hipSuccess) return -1;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, LDS_BYTES) != hipSuccess) return -1;
  return n;
}

// geometry for the host wrapper (buffer sizes) and the tests
extern "C" void hopsx_mnist_persist_geom(long* g) {
  using namespace mnistp;
  g[0] = B;
  g[1] = NPOS;
  g[2] = NHEAD;
  g[3] = GRID;
  g[4] = NCONV;
  g[5] = NSLICE;
  g[6] = SLICE;
  g[7] = PAY;
  g[8] = FL_WORDS;
  g[9] = LDS_BYTES;
  g[10] = D_BYTES;
  g[11] = X_BYTES;
  g[12] = XF_WORDS;
  g[13] = XMAX;
  // exchange-buffer layout (runtime/persist_sim.py): region offset, per-slot bytes, for the pooled
  // fragments, dh^T fragments, head gradients and conv slice sums ([2 parities][XMAX slots] each)
  g[14] = XO_POOL;
  g[15] = XS_POOL;
  g[16] = XO_DHT;
  g[17] = XS_DHT;
  g[18] = XO_FC2;
  g[19] = XS_FC2;
  g[20] = XO_CONV;
  g[21] = XS_CONV;
}
