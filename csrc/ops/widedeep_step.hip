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
//     kernel advances itself: no copy launches.
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
constexpr int WD_MAXT = 8;      // dX tiles a wave holds in registers across the in-place barrier
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
};

__host__ __device__ inline int pad16(int x) { return (x + 15) & ~15; }

struct Lay {
  int act[WD_MAXL + 1];  // LDS float offset of A_l [Bp][pad16(d_l) + 1]
  int w[WD_MAXL];        // W_l [pad16(out)][pad16(in) + 1]
  int b[WD_MAXL];        // bias_l [pad16(out)]
  int wsum;              // wide sums [Bp]
  int red;               // loss / correct partials [2 * WD_WAVES]
  int total;
};

__host__ __device__ inline Lay wd_layout(const WideDeepArgs& a) {
  Lay l;
  int o = 0;
  for (int i = 0; i <= a.L; ++i) {
    l.act[i] = o;
    o += a.Bp * (pad16(a.dims[i]) + 1);
  }
  for (int i = 0; i < a.L; ++i) {
    l.w[i] = o;
    o += pad16(a.dims[i + 1]) * (pad16(a.dims[i]) + 1);
    l.b[i] = o;
    o += pad16(a.dims[i + 1]);
  }
  l.wsum = o;
  o += a.Bp;
  l.red = o;
  o += 2 * WD_WAVES;
  l.total = o;
  return l;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(WD_THREADS) void widedeep_step_k(WideDeepArgs A) {
  extern __shared__ __attribute__((aligned(16))) float wd_lds[];
  const Lay Ly = wd_layout(A);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int B = A.B, Bp = A.Bp, L = A.L;
  const long long bi = A.cursor ? A.cursor[0] : 0;

  // ---------------------------------------------------------------- stage
  {
    const int d0 = A.dims[0], s0 = pad16(d0) + 1;
    const float* xb = A.dense + bi * (long long)B * d0;
    for (int e = tid; e < Bp * s0; e += WD_THREADS) {
      const int b = e / s0, i = e - b * s0;
      wd_lds[Ly.act[0] + e] = (b < B && i < d0) ? xb[(long)b * d0 + i] : 0.f;
    }
    for (int l = 0; l < L; ++l) {
      const int in = A.dims[l], out = A.dims[l + 1], sw = pad16(in) + 1, op = pad16(out);
      const float* wg = A.master + A.woff[l];
      for (int e = tid; e < op * sw; e += WD_THREADS) {
        const int o = e / sw, i = e - o * sw;
        wd_lds[Ly.w[l] + e] = (o < out && i < in) ? wg[(long)o * in + i] : 0.f;
      }
      for (int o = tid; o < op; o += WD_THREADS) wd_lds[Ly.b[l] + o] = o < out ? A.master[A.boff[l] + o] : 0.f;
    }
    const long long* cb = A.cat + bi * (long long)B * A.nwide;
    for (int b = tid; b < Bp; b += WD_THREADS) {
      float s = 0.f;
      if (b < B)
        for (int j = 0; j < A.nwide; ++j) s += A.master[A.wide_off + cb[(long)b * A.nwide + j]];
      wd_lds[Ly.wsum + b] = s;
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- forward
  for (int l = 0; l < L; ++l) {
    const int in = A.dims[l], out = A.dims[l + 1];
    const int sa = pad16(in) + 1, sz = pad16(out) + 1, sw = sa;
    const int tm = Bp / 16, tn = pad16(out) / 16, ks = pad16(in) / 4;
    const float* Ap = wd_lds + Ly.act[l];
    const float* Wp = wd_lds + Ly.w[l];
    const float* bp = wd_lds + Ly.b[l];
    float* Zp = wd_lds + Ly.act[l + 1];
    const bool relu = l + 1 < L;
    for (int t = wave; t < tm * tn; t += WD_WAVES) {
      const int m0 = (t / tn) * 16, n0 = (t % tn) * 16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < ks; ++k)
        acc = mfma4(Ap[(m0 + fr) * sa + 4 * k + fq], Wp[(n0 + fr) * sw + 4 * k + fq], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = m0 + 4 * fq + r, o = n0 + fr;
        float v = acc[r] + bp[o];
        if (relu) v = fmaxf(v, 0.f);
        Zp[b * sz + o] = (b < B && o < out) ? v : 0.f;
      }
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- loss (sigmoid CE on logits)
  {
    float* Zp = wd_lds + Ly.act[L];  // [Bp][17]; column 0 = deep logit
    const int sz = pad16(A.dims[L]) + 1;
    const long long* cb = A.cat + bi * (long long)B * A.nwide;
    const float* yb = A.label + bi * (long long)B;
    float lsum = 0.f;
    int csum = 0;
    for (int b = tid; b < B; b += WD_THREADS) {
      const float z = Zp[b * sz] + wd_lds[Ly.wsum + b];
      const float y = yb[b];
      const float p = 1.f / (1.f + __expf(-z));
      lsum += fmaxf(z, 0.f) - z * y + __logf(1.f + __expf(-fabsf(z)));
      csum += ((p > 0.5f) == (y > 0.5f));
      const float g = (p - y) / (float)B;
      Zp[b * sz] = g;  // G_L in place of the logits
      for (int j = 0; j < A.nwide; ++j) atomicAdd(A.grad + A.wide_off + cb[(long)b * A.nwide + j], g);
    }
    lsum = wave_sum(lsum);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o, 64);
    if (lane == 0) {
      wd_lds[Ly.red + wave] = lsum;
      wd_lds[Ly.red + WD_WAVES + wave] = (float)csum;
    }
    __syncthreads();
    if (tid == 0) {
      float l = 0.f, c = 0.f;
      for (int w = 0; w < WD_WAVES; ++w) {
        l += wd_lds[Ly.red + w];
        c += wd_lds[Ly.red + WD_WAVES + w];
      }
      if (A.loss) A.loss[0] = l / (float)B;
      if (A.correct) A.correct[0] = (int)c;
    }
  }

  // ---------------------------------------------------------------- backward
  for (int l = L - 1; l >= 0; --l) {
    const int in = A.dims[l], out = A.dims[l + 1];
    const int sg = pad16(out) + 1, sa = pad16(in) + 1, sw = sa;
    const float* Gp = wd_lds + Ly.act[l + 1];  // G_l [Bp][sg] (already masked by relu')
    float* Ap = wd_lds + Ly.act[l];            // A_{l-1} [Bp][sa]
    const float* Wp = wd_lds + Ly.w[l];
    const int tdw = (pad16(out) / 16) * (pad16(in) / 16);           // dW tiles (o x i)
    const int tdx = l > 0 ? (Bp / 16) * (pad16(in) / 16) : 0;       // dX tiles (b x i)
    const int tni = pad16(in) / 16;
    for (int t = wave; t < tdw; t += WD_WAVES) {
      // dW[o][i] = sum_b G[b][o] A[b][i]   (M = o, N = i, K = b), optimizer applied on the fragment
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int o0 = (t / tni) * 16, i0 = (t % tni) * 16;
      for (int k = 0; k < Bp / 4; ++k)
        acc = mfma4(Gp[(4 * k + fq) * sg + o0 + fr], Ap[(4 * k + fq) * sa + i0 + fr], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + 4 * fq + r, i = i0 + fr;
        if (o < out && i < in) {
          const long idx = A.woff[l] + (long)o * in + i;
          if (A.apply_opt) {
            float s1 = A.ada_s[idx], s2 = 0.f, s3 = 0.f;
            const float w = upd<5>(A.master[idx], acc[r] * A.ada.gscale, s1, s2, s3, A.ada, 1.f, 1.f);
            A.master[idx] = w;
            A.ada_s[idx] = s1;
            if (A.shadow) A.shadow[idx] = f2bf(w);
          } else {
            A.grad[idx] = acc[r];
          }
        }
      }
    }
    // dX[b][i] = sum_o G[b][o] W[o][i]   (M = b, N = i, K = o): held in registers (static indices)
    // until every reader of A_{l-1} is done, then written over it as G_{l-1}
    f32x4 hold[WD_MAXT];
#pragma unroll
    for (int j = 0; j < WD_MAXT; ++j) {
      const int tt = wave + j * WD_WAVES;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (tt < tdx) {
        const int b0 = (tt / tni) * 16, i0 = (tt % tni) * 16;
        for (int k = 0; k < pad16(out) / 4; ++k)
          acc = mfma4(Gp[(b0 + fr) * sg + 4 * k + fq], Wp[(4 * k + fq) * sw + i0 + fr], acc);
      }
      hold[j] = acc;
    }
    // bias gradient: db[o] = sum_b G[b][o]
    for (int o = tid; o < out; o += WD_THREADS) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += Gp[b * sg + o];
      const long idx = A.boff[l] + o;
      if (A.apply_opt) {
        float s1 = A.ada_s[idx], s2 = 0.f, s3 = 0.f;
        const float w = upd<5>(A.master[idx], s * A.ada.gscale, s1, s2, s3, A.ada, 1.f, 1.f);
        A.master[idx] = w;
        A.ada_s[idx] = s1;
        if (A.shadow) A.shadow[idx] = f2bf(w);
      } else {
        A.grad[idx] = s;
      }
    }
    if (l == 0) break;
    __syncthreads();  // every reader of A_{l-1} (dW) is done: overwrite it with G_{l-1}
#pragma unroll
    for (int j = 0; j < WD_MAXT; ++j) {
      const int tt = wave + j * WD_WAVES;
      if (tt >= tdx) break;
      const int b0 = (tt / tni) * 16, i0 = (tt % tni) * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = b0 + 4 * fq + r, i = i0 + fr;
        float* p = Ap + b * sa + i;
        *p = *p > 0.f ? hold[j][r] : 0.f;  // relu' of the hidden activation (0 on padding)
      }
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- wide FTRL + bookkeeping
  __syncthreads();
  if (A.apply_opt) {
    const long long* cb = A.cat + bi * (long long)B * A.nwide;
    for (int e = tid; e < B * A.nwide; e += WD_THREADS) {
      const long idx = A.wide_off + cb[e];
      // the summed gradient of this row, claimed by exactly one thread (and left zero)
      const float g = atomicExch(A.grad + idx, 0.f);
      if (g != 0.f) {
        float z = A.ftrl_z[idx], n = A.ftrl_n[idx], s3 = 0.f;
        const float w = upd<6>(A.master[idx], g * A.ftrl.gscale, z, n, s3, A.ftrl, 1.f, 1.f);
        A.master[idx] = w;
        A.ftrl_z[idx] = z;
        A.ftrl_n[idx] = n;
        if (A.shadow) A.shadow[idx] = f2bf(w);
      }
    }
  }
  if (tid == 0) {
    if (A.apply_opt) {
      if (A.step_ada) A.step_ada[0] += 1.f;
      if (A.step_ftrl) A.step_ftrl[0] += 1.f;
      if (A.rng) A.rng[1] += (unsigned long long)A.rng_bumps;
    }
    if (A.cursor) A.cursor[0] = (bi + 1) % A.nbatch;
  }
}

int wd_fill(WideDeepArgs& a, const uint64_t* p, int np, const long* iv, int ni, const float* fv, int nf) {
  // ptrs: master grad shadow ada_s ftrl_z ftrl_n dense cat label cursor loss correct step_ada step_ftrl rng
  if (np != 15 || nf != 16) return -2;
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
  // ints: L B nbatch nwide wide_off apply_opt rng_bumps dims[L+1] woff[L] boff[L]
  if (ni < 7) return -2;
  a.L = (int)iv[0];
  a.B = (int)iv[1];
  a.nbatch = (int)iv[2];
  a.nwide = (int)iv[3];
  a.wide_off = iv[4];
  a.apply_opt = (int)iv[5];
  a.rng_bumps = (int)iv[6];
  if (a.L < 1 || a.L > WD_MAXL || ni != 7 + (a.L + 1) + 2 * a.L || a.B < 1 || a.nbatch < 1) return -2;
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
  const uint64_t p[15] = {};
  const float f[16] = {};
  if (wd_fill(a, p, 15, iv, ni, f, 16)) return -1;
  if (a.dims[a.L] != 1) return -1;
  for (int l = 1; l < a.L; ++l)
    if ((a.Bp / 16) * (pad16(a.dims[l]) / 16) > WD_WAVES * WD_MAXT) return -1;
  const long bytes = (long)wd_layout(a).total * 4;
  return bytes <= WD_LDS_MAX ? bytes : -1;
}

extern "C" int hopsx_widedeep_step(const uint64_t* ptrs, int np, const long* iv, int ni, const float* fv, int nf,
                                   hipStream_t st) {
  WideDeepArgs a{};
  if (wd_fill(a, ptrs, np, iv, ni, fv, nf)) return -2;
  const long bytes = hopsx_widedeep_step_lds(iv, ni);
  if (bytes < 0) return -2;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)widedeep_step_k, hipFuncAttributeMaxDynamicSharedMemorySize, WD_LDS_MAX);
    attr = true;
  }
  hipLaunchKernelGGL(widedeep_step_k, dim3(1), dim3(WD_THREADS), (size_t)bytes, st, a);
  return (int)hipGetLastError();
}
