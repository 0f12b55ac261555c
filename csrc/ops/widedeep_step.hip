// The whole wide & deep training step (the Chicago-taxi DNNLinearCombinedClassifier) in ONE
// workgroup of one CU.  The model is tiny (18.9 k parameters, batch 40): as a chain of library
// launches every op — five Linear forwards, five paired backwards, the embedding bag forward and
// backward, the loss, two optimizers, three input copies — costs a kernel boundary and an HBM
// round trip for a few KB of work (measured ~90 us/step, 22 launches).  Here:
//   * the deep weights (fp32 master, ~50 KB) and every activation of the batch (~60 KB) live in
//     LDS for the whole step; gradients overwrite the activations they replace in place,
//   * the GEMMs (forward, dX, dW) run on v_mfma_f32_16x16x4_f32 straight from LDS — fp32 operands,
//     so the fused step is at least as precise as the bf16 layer-by-layer path; row strides are
//     odd (padded dim + 1) so the three operand access patterns are all bank-conflict free,
//   * the wide part (13 embedding rows per example) is gathered from the fp32 master and its
//     gradient scattered with L2 atomics,
//   * with apply_opt the optimizers run in the same launch: Adagrad on each dW fragment as it
//     leaves the MFMA (the deep gradient never touches memory), FTRL on the touched wide rows
//     (each row claimed once by an atomic exchange of its summed gradient, which also leaves
//     the gradient buffer zero), step counters / RNG bumps as the optimizer kernels would,
//   * the batch is read straight from the HBM-resident epoch at a device cursor that the
//     kernel advances itself: no copy launches;
//   * ``nsteps`` > 1 (Keras steps_per_execution): the launch runs that many consecutive steps on
//     consecutive batches — the deep weights and their Adagrad state stay in registers / LDS
//     between steps (written back once, after the last), the wide rows' FTRL updates go through
//     memory (the next step gathers them) — so a step costs neither a launch nor a reload.
// Data parallel runs use apply_opt = 0: gradients land in the arena grad buffer for the RCCL
// all-reduce and the regular optimizer kernels.
// Parity: the reference's TFX taxi trainer (README.md:99-112) — same model,
// optimizers (FTRL on the wide part, Adagrad on the deep part) and loss.
#include <cstdint>

#include "common.h"
#include "ops_api.h"
#include "optim_core.h"

namespace {

constexpr int WD_MAXL = 8;      // linear layers (hidden + logits)
constexpr int WD_THREADS = 1024;
constexpr int WD_WAVES = WD_THREADS / 64;
constexpr int WD_MAXT = 4;      // dW / dX tiles a wave holds in registers across the in-place barrier
constexpr int WD_PF = 16;       // deep parameters per thread prefetched into registers (span <= 16 K)
constexpr int WD_DX = 1;        // dense-input image elements per thread (Bp * (dpad(d0) + 1) <= 1 K: taxi 48 x 17)
constexpr int WD_LDS_MAX = 160 * 1024;

struct WideDeepArgs {
  float* master;
  float* grad;
  bf16_raw* shadow;
  float* ada_s;   // Adagrad accumulator over the whole arena (indexed by arena offset)
  float* ftrl_z;  // FTRL state (arena-indexed)
  float* ftrl_n;
  int L, B, Bp;
  int dims[WD_MAXL + 1];
  long woff[WD_MAXL], boff[WD_MAXL];
  long wide_off;
  int nwide;
  const float* dense;       // resident [nbatch][B][dims[0]]
  const long long* cat;     // resident [nbatch][B][nwide] (global one-hot ids)
  const float* label;       // resident [nbatch][B]
  long long* cursor;        // batch index (advanced in-kernel), or null: batch 0
  int nbatch;
  OptHP ada, ftrl;
  float* loss;
  int* correct;
  float* step_ada;
  float* step_ftrl;
  unsigned long long* rng;
  int rng_bumps;
  int apply_opt;
  int nsteps;               // consecutive steps in this launch (1 unless apply_opt)
  unsigned long long* dbg;  // phase timestamps (wall clock, 100 MHz), or null
  const int* slot;          // [deep span]: LDS slot of each deep arena element (-1: padding), host-built
};

__host__ __device__ inline int pad16(int x) { return (x + 15) & ~15; }
// padded width of an activation of d features: one extra constant-1 column (the bias rides in the
// GEMMs as weight column d, and db falls out of the dW GEMM as its column d)
__host__ __device__ inline int dpad(int d) { return pad16(d + 1); }

struct Lay {
  int act[WD_MAXL + 1];  // LDS float offset of A_l [Bp][dpad(d_l) + 1] (column d_l = 1)
  int w[WD_MAXL];        // [W_l | b_l] [dpad(out)][dpad(in) + 1]
  int wsum;              // wide sums [Bp]
  int red;               // loss / correct partials [2 * WD_WAVES]
  int total;
};

__host__ __device__ inline Lay wd_layout(const WideDeepArgs& a, int L) {
  Lay l;
  int o = 0;
#pragma unroll
  for (int i = 0; i <= L; ++i) {
    l.act[i] = o;
    o += a.Bp * (dpad(a.dims[i]) + 1);
  }
#pragma unroll
  for (int i = 0; i < L; ++i) {
    l.w[i] = o;
    o += dpad(a.dims[i + 1]) * (dpad(a.dims[i]) + 1);
  }
  l.wsum = o;
  o += a.Bp;
  l.red = o;
  o += 2 * WD_WAVES;
  l.total = o;
  return l;
}

__device__ __forceinline__ void wd_mark(const WideDeepArgs& A, int slot) {
  if (A.dbg && threadIdx.x == 0) A.dbg[slot] = wall_clock64();
}

// Adagrad / FTRL-proximal (optim_core.h upd<5> / upd<6>) with the hardware square root and reciprocal
// (1 ulp) instead of the correctly rounded sqrt + division sequences: the update phase runs ~16 deep
// parameters a lane and the touched wide rows every step, on the step's critical path
__device__ __forceinline__ float adagrad_fast(float w, float g, float& s1, const OptHP& h) {
  g = fmaf(h.wd, w, g);
  s1 = fmaf(g, g, s1);
  return w - h.lr * g * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(s1) + h.a);
}
__device__ __forceinline__ float ftrl_fast(float w, float g, float& z, float& n, const OptHP& h) {
  const float nn = fmaf(g, g, n);
  const float rs = __builtin_amdgcn_sqrtf(nn);
  const float sigma = (rs - __builtin_amdgcn_sqrtf(n)) * __builtin_amdgcn_rcpf(h.lr);
  z += g - sigma * w;
  n = nn;
  const float den = (h.c + rs) * __builtin_amdgcn_rcpf(h.lr) + 2.f * h.b;
  return (fabsf(z) <= h.a) ? 0.f : -(z - copysignf(h.a, z)) * __builtin_amdgcn_rcpf(den);
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() also waits for every outstanding global
// access (vmcnt 0), which would put the wide rows' gradient atomics and the next batch's prefetch
// loads on the critical path of every layer's barrier
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// NL (the layer count) is a template parameter so every per-layer loop unrolls and the layout /
// dims / offsets stay in scalar registers (a runtime-indexed struct would live in scratch memory)
template <int NL>
__global__ __launch_bounds__(WD_THREADS) void widedeep_step_k(WideDeepArgs A) {
  extern __shared__ __attribute__((aligned(16))) float wd_lds[];
  constexpr int L = NL;
  const Lay Ly = wd_layout(A, NL);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int B = A.B, Bp = A.Bp;
  const long long bi0 = A.cursor ? A.cursor[0] : 0;
  const long deep_lo = A.woff[0], deep_hi = A.boff[L - 1] + A.dims[L];
  wd_mark(A, 0);

  // ---------------------------------------------------------------- stage
  // Every global load of the step is issued here, independent of each other (one memory round
  // trip): this thread's deep parameters + Adagrad state (kept in registers until the update —
  // and across the steps of a multi-step launch), its wide (example, column) entry with that
  // row's FTRL state, the batch.
  float pw[WD_PF], ps[WD_PF];
  int psl[WD_PF];
#pragma unroll
  for (int k = 0; k < WD_PF; ++k) {
    const long x = deep_lo + tid + (long)k * WD_THREADS;
    const long xc = x < deep_hi ? x : deep_lo;
    pw[k] = A.master[xc];
    ps[k] = A.apply_opt ? A.ada_s[xc] : 0.f;
    psl[k] = x < deep_hi ? A.slot[xc - deep_lo] : -1;
  }
  // the batch of step s in registers: this thread's wide id, label and dense-image elements; step
  // s + 1's are loaded during step s's backward (they do not depend on its updates)
  const bool wide_t = tid < B * A.nwide;
  const int d0 = A.dims[0], s0 = dpad(d0) + 1;
  long long cid = 0;
  float yv = 0.f, dxv[WD_DX];
  auto prefetch = [&](int s) {
    const long long bi = (bi0 + s) % A.nbatch;
    cid = wide_t ? A.cat[bi * (long long)B * A.nwide + tid] : 0;
    yv = tid < B ? A.label[bi * (long long)B + tid] : 0.f;
    const float* xb = A.dense + bi * (long long)B * d0;
#pragma unroll
    for (int j = 0; j < WD_DX; ++j) {
      const int e = tid + j * WD_THREADS, b = e / s0, i = e - b * s0;
      dxv[j] = e < Bp * s0 && b < B && i < d0 ? xb[(long)b * d0 + i] : 0.f;
    }
  };
  prefetch(0);
  for (int step = 0; step < A.nsteps; ++step) {
  const bool last = step + 1 == A.nsteps;
  if (step) __syncthreads();  // the previous step's wide-row updates (same CU) are visible after this
  const long wrow = A.wide_off + cid;
  const float wv = A.master[wrow];
  float wz = 0.f, wn = 0.f;
  if (A.apply_opt) {
    wz = A.ftrl_z[wrow];
    wn = A.ftrl_n[wrow];
  }
  const float ylab = yv;
  {
#pragma unroll
    for (int j = 0; j < WD_DX; ++j) {
      const int e = tid + j * WD_THREADS, b = e / s0, i = e - b * s0;
      if (e < Bp * s0) wd_lds[Ly.act[0] + e] = b < B && i == d0 ? 1.f : dxv[j];
    }
    // zero the weight / bias images (their padding must read 0) and the wide sums
    for (int e = Ly.w[0] + tid; e < Ly.wsum + Bp; e += WD_THREADS) wd_lds[e] = 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < WD_PF; ++k)
    if (psl[k] >= 0) wd_lds[psl[k]] = pw[k];
  if (wide_t) atomicAdd(wd_lds + Ly.wsum + tid / A.nwide, wv);  // sum of the example's 13 rows
  __syncthreads();
  wd_mark(A, 1);

  // ---------------------------------------------------------------- forward
  // layer loops NOT unrolled: unrolled, the 5 layers' live ranges spilled 1.4 KB per lane to scratch
  // at the 128-VGPR budget of a 1024-thread workgroup (0.66 KB rolled: 25.3k -> 26.9k steps/s)
#pragma unroll 1
  for (int l = 0; l < L; ++l) {
    const int in = A.dims[l], out = A.dims[l + 1];
    const int sa = dpad(in) + 1, sz = dpad(out) + 1, sw = sa;
    const int tm = Bp / 16, tn = dpad(out) / 16, ks = dpad(in) / 4;
    const float* Ap = wd_lds + Ly.act[l];
    const float* Wp = wd_lds + Ly.w[l];
    float* Zp = wd_lds + Ly.act[l + 1];
    const bool relu = l + 1 < L;
    for (int t = wave; t < tm * tn; t += WD_WAVES) {
      const int m0 = (t / tn) * 16, n0 = (t % tn) * 16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int k = 0; k < ks; ++k)
        acc = mfma4(Ap[(m0 + fr) * sa + 4 * k + fq], Wp[(n0 + fr) * sw + 4 * k + fq], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = m0 + 4 * fq + r, o = n0 + fr;
        float v = acc[r];  // bias included (constant-1 input column)
        if (relu) v = fmaxf(v, 0.f);
        Zp[b * sz + o] = b < B ? (o < out ? v : (o == out && relu ? 1.f : 0.f)) : 0.f;
      }
    }
    __syncthreads();
    wd_mark(A, 2 + l);
  }

  // ---------------------------------------------------------------- loss (sigmoid CE on logits)
  {
    float* Zp = wd_lds + Ly.act[L];  // [Bp][17]; column 0 = deep logit
    const int sz = dpad(A.dims[L]) + 1;
    float lsum = 0.f;
    int csum = 0;
    if (tid < B) {
      const int b = tid;
      const float z = Zp[b * sz] + wd_lds[Ly.wsum + b];
      const float p = 1.f / (1.f + __expf(-z));
      lsum = fmaxf(z, 0.f) - z * ylab + __logf(1.f + __expf(-fabsf(z)));
      csum = ((p > 0.5f) == (ylab > 0.5f));
      Zp[b * sz] = (p - ylab) / (float)B;  // G_L in place of the logits
    }
    lsum = wave_sum(lsum);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o, 64);
    if (lane == 0) {
      wd_lds[Ly.red + wave] = lsum;
      wd_lds[Ly.red + WD_WAVES + wave] = (float)csum;
    }
    __syncthreads();
    if (wide_t) atomicAdd(A.grad + wrow, Zp[(tid / A.nwide) * sz]);  // wide gradient (summed per row)
    if (step + 1 < A.nsteps) prefetch(step + 1);  // in flight during the backward (LDS-only barriers)
    if (tid == 0) {
      float l = 0.f, c = 0.f;
      for (int w = 0; w < WD_WAVES; ++w) {
        l += wd_lds[Ly.red + w];
        c += wd_lds[Ly.red + WD_WAVES + w];
      }
      if (A.loss) A.loss[0] = l / (float)B;
      if (A.correct) A.correct[0] = (int)c;
    }
    wd_mark(A, 10);
  }

  // ---------------------------------------------------------------- backward
  // Per layer: phase A computes dW (o x i tiles) and dX (b x i tiles) from LDS into registers and
  // db into the (dead) bias image; phase B — after every reader of A_{l-1} and W_l is done — writes
  // G_{l-1} = dX * relu'(A_{l-1}) over A_{l-1} and dW over W_l.
#pragma unroll 1
  for (int l = L - 1; l >= 0; --l) {
    const int in = A.dims[l], out = A.dims[l + 1];
    const int sg = dpad(out) + 1, sa = dpad(in) + 1, sw = sa;
    const float* Gp = wd_lds + Ly.act[l + 1];
    float* Ap = wd_lds + Ly.act[l];
    float* Wp = wd_lds + Ly.w[l];
    const int tni = dpad(in) / 16;
    const int tdw = (dpad(out) / 16) * tni;  // includes the bias column: db = dW[:, in]
    const int tdx = l > 0 ? (Bp / 16) * tni : 0;
    f32x4 hw[WD_MAXT], hx[WD_MAXT];
#pragma unroll
    for (int j = 0; j < WD_MAXT; ++j) {
      const int t = wave + j * WD_WAVES;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (t < tdw) {  // dW[o][i] = sum_b G[b][o] A[b][i]
        const int o0 = (t / tni) * 16, i0 = (t % tni) * 16;
#pragma unroll 4
        for (int k = 0; k < Bp / 4; ++k)
          acc = mfma4(Gp[(4 * k + fq) * sg + o0 + fr], Ap[(4 * k + fq) * sa + i0 + fr], acc);
      }
      hw[j] = acc;
      f32x4 acx = {0.f, 0.f, 0.f, 0.f};
      if (t < tdx) {  // dX[b][i] = sum_o G[b][o] W[o][i]
        const int b0 = (t / tni) * 16, i0 = (t % tni) * 16;
#pragma unroll 4
        for (int k = 0; k < dpad(out) / 4; ++k)
          acx = mfma4(Gp[(b0 + fr) * sg + 4 * k + fq], Wp[(4 * k + fq) * sw + i0 + fr], acx);
      }
      hx[j] = acx;
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < WD_MAXT; ++j) {
      const int t = wave + j * WD_WAVES;
      if (t < tdw) {
        const int o0 = (t / tni) * 16, i0 = (t % tni) * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) Wp[(o0 + 4 * fq + r) * sw + i0 + fr] = hw[j][r];
      }
      if (t < tdx) {
        const int b0 = (t / tni) * 16, i0 = (t % tni) * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* p = Ap + (b0 + 4 * fq + r) * sa + i0 + fr;
          *p = *p > 0.f ? hx[j][r] : 0.f;  // relu' of the hidden activation (0 on padding)
        }
      }
    }
    lds_barrier();
    wd_mark(A, 11 + l);
  }

  // ---------------------------------------------------------------- updates + bookkeeping
  // (the LDS weight images now hold dW, the bias images db)
#pragma unroll
  for (int k = 0; k < WD_PF; ++k) {
    const long x = deep_lo + tid + (long)k * WD_THREADS;
    {
      const int sl = psl[k];
      if (sl >= 0) {
        const float g = wd_lds[sl];
        if (A.apply_opt) {
          float s1 = ps[k];
          const float w = adagrad_fast(pw[k], g * A.ada.gscale, s1, A.ada);
          pw[k] = w;  // the next step of this launch starts from the updated weight
          ps[k] = s1;
          if (last) {
            A.master[x] = w;
            A.ada_s[x] = s1;
            if (A.shadow) A.shadow[x] = f2bf(w);
          }
        } else {
          A.grad[x] = g;
        }
      }
    }
  }
  // every wave's wide-gradient atomics complete before any claim reads a row
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (A.apply_opt && wide_t) {
    // the summed gradient of this row, claimed by exactly one thread (and left zero); its state
    // was prefetched at the start (no other thread touches the row before the claim)
    const float g = atomicExch(A.grad + wrow, 0.f);
    if (g != 0.f) {
      float z = wz, n = wn;
      const float w = ftrl_fast(wv, g * A.ftrl.gscale, z, n, A.ftrl);
      A.master[wrow] = w;
      A.ftrl_z[wrow] = z;
      A.ftrl_n[wrow] = n;
      if (A.shadow) A.shadow[wrow] = f2bf(w);
    }
  }
  }  // steps
  if (tid == 0) {
    if (A.apply_opt) {
      if (A.step_ada) A.step_ada[0] += (float)A.nsteps;
      if (A.step_ftrl) A.step_ftrl[0] += (float)A.nsteps;
      if (A.rng) A.rng[1] += (unsigned long long)A.rng_bumps * (unsigned long long)A.nsteps;
    }
    if (A.cursor) A.cursor[0] = (bi0 + A.nsteps) % A.nbatch;
  }
  wd_mark(A, 19);
}

int wd_fill(WideDeepArgs& a, const uint64_t* p, int np, const long* iv, int ni, const float* fv, int nf) {
  // ptrs: master grad shadow ada_s ftrl_z ftrl_n dense cat label cursor loss correct step_ada step_ftrl rng
  if (np != 17 || nf != 16) return -2;
  a.dbg = (unsigned long long*)p[15];
  a.slot = (const int*)p[16];
  a.master = (float*)p[0];
  a.grad = (float*)p[1];
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
  // ints: L B nbatch nwide wide_off apply_opt rng_bumps dims[L+1] woff[L] boff[L] [nsteps]
  if (ni < 7) return -2;
  a.L = (int)iv[0];
  a.B = (int)iv[1];
  a.nbatch = (int)iv[2];
  a.nwide = (int)iv[3];
  a.wide_off = iv[4];
  a.apply_opt = (int)iv[5];
  a.rng_bumps = (int)iv[6];
  const int nbase = 7 + (a.L + 1) + 2 * a.L;
  if (a.L < 1 || a.L > WD_MAXL || (ni != nbase && ni != nbase + 1) || a.B < 1 || a.nbatch < 1) return -2;
  a.nsteps = ni == nbase + 1 ? (int)iv[nbase] : 1;
  if (a.nsteps < 1 || (a.nsteps > 1 && !a.apply_opt)) return -2;  // DP: gradients leave after every step
  for (int i = 0; i <= a.L; ++i) a.dims[i] = (int)iv[7 + i];
  for (int i = 0; i < a.L; ++i) {
    a.woff[i] = iv[8 + a.L + i];
    a.boff[i] = iv[8 + 2 * a.L + i];
  }
  a.Bp = pad16(a.B);
  // floats: ada(lr gscale wd eps + 4 unused) ftrl(lr gscale wd l1 l2 beta + 2 unused)
  a.ada = OptHP{fv[0], fv[1], fv[2], fv[3], fv[4], fv[5], fv[6], fv[7]};
  a.ftrl = OptHP{fv[8], fv[9], fv[10], fv[11], fv[12], fv[13], fv[14], fv[15]};
  return 0;
}

}  // namespace

// The fused step applies when the whole batch + model fit one workgroup's LDS, the logits
// layer has one output, and a wave's dX tiles fit its register budget.
extern "C" long hopsx_widedeep_step_lds(const long* iv, int ni) {
  WideDeepArgs a{};
  const uint64_t p[17] = {};
  const float f[16] = {};
  if (wd_fill(a, p, 17, iv, ni, f, 16)) return -1;
  if (a.dims[a.L] != 1 || (long)a.B * a.nwide > WD_THREADS || a.B > WD_THREADS) return -1;
  if ((long)a.Bp * (dpad(a.dims[0]) + 1) > (long)WD_DX * WD_THREADS) return -1;
  if (a.boff[a.L - 1] + a.dims[a.L] - a.woff[0] > (long)WD_PF * WD_THREADS) return -1;
  for (int l = 0; l < a.L; ++l) {
    const int tn = dpad(a.dims[l]) / 16;
    if ((a.Bp / 16) * tn > WD_WAVES * WD_MAXT || (dpad(a.dims[l + 1]) / 16) * tn > WD_WAVES * WD_MAXT) return -1;
  }
  const long bytes = (long)wd_layout(a, a.L).total * 4;
  return bytes <= WD_LDS_MAX ? bytes : -1;
}

// The slot table the kernel reads: LDS float offset of every deep arena element (weights
// W_l[o][i] -> W image row o col i, biases -> bias image), -1 for the arena's alignment padding.
extern "C" int hopsx_widedeep_slots(const long* iv, int ni, int* out, long n) {
  WideDeepArgs a{};
  const uint64_t p[17] = {};
  const float f[16] = {};
  if (wd_fill(a, p, 17, iv, ni, f, 16)) return -2;
  const Lay Ly = wd_layout(a, a.L);
  const long lo = a.woff[0];
  if (a.boff[a.L - 1] + a.dims[a.L] - lo != n) return -2;
  for (long x = 0; x < n; ++x) out[x] = -1;
  for (int l = 0; l < a.L; ++l) {
    const int in = a.dims[l], out_ = a.dims[l + 1];
    for (int o = 0; o < out_; ++o) {
      const int row = Ly.w[l] + o * (dpad(in) + 1);
      for (int i = 0; i <= in; ++i) out[(i < in ? a.woff[l] + (long)o * in + i : a.boff[l] + o) - lo] = row + i;
    }
  }
  return 0;
}

extern "C" int hopsx_widedeep_step(const uint64_t* ptrs, int np, const long* iv, int ni, const float* fv, int nf,
                                   hipStream_t st) {
  WideDeepArgs a{};
  if (wd_fill(a, ptrs, np, iv, ni, fv, nf)) return -2;
  const long bytes = hopsx_widedeep_step_lds(iv, ni);
  if (bytes < 0) return -2;
  static bool attr[WD_MAXL + 1] = {};
#define HOPSX_WD(NLV)                                                                                           \
  case NLV:                                                                                                     \
    if (!attr[NLV]) {                                                                                           \
      hipFuncSetAttribute((const void*)widedeep_step_k<NLV>, hipFuncAttributeMaxDynamicSharedMemorySize,        \
                          WD_LDS_MAX);                                                                          \
      attr[NLV] = true;                                                                                         \
    }                                                                                                           \
    hipLaunchKernelGGL(widedeep_step_k<NLV>, dim3(1), dim3(WD_THREADS), (size_t)bytes, st, a);                 \
    break;
  switch (a.L) {
    HOPSX_WD(1) HOPSX_WD(2) HOPSX_WD(3) HOPSX_WD(4) HOPSX_WD(5) HOPSX_WD(6) HOPSX_WD(7) HOPSX_WD(8)
    default: return -2;
  }
#undef HOPSX_WD
  return (int)hipGetLastError();
}
