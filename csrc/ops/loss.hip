// Fused loss forward+backward.  The gradient w.r.t. the logits is written in the
// same pass (already scaled by grad_scale, e.g. 1/batch for a mean loss), the
// reported loss is sum * grad_scale, and the correct-prediction count is
// produced alongside so the metric all-reduce moves 8 bytes per replica.
//
// Two shapes of parallelism:
//   * C <= 32 (MNIST 10 classes, binary heads): one THREAD per row — a wave
//     processes 64 rows with no cross-lane reductions at all;
//   * C  > 32 (ImageNet-style 1000-way heads): one WAVE per row with shuffles.
// Small problems run as ONE workgroup that overwrites the totals (no zero-fill
// node in the graph); large ones use many workgroups + one atomic each after a
// memset of the two accumulators.
//   kind 0  softmax cross-entropy, int64 labels   (Keras sparse CE / torch log_softmax+NLL)
//   kind 1  softmax cross-entropy, dense targets  (Keras categorical_crossentropy on one-hot)
//   kind 2  sigmoid + binary CE from logits
//   kind 3  mean squared error
//   kind 4  binary CE on probabilities (Keras sigmoid output + binary_crossentropy)
#include "common.h"
#include "ops_api.h"

HOPSX_DET_TU(loss)

__device__ __forceinline__ float ld_logit(const void* p, int f32, long i) {
  return f32 ? ((const float*)p)[i] : bf2f(((const bf16_raw*)p)[i]);
}
__device__ __forceinline__ void st_grad(void* p, int f32, long i, float v) {
  if (f32) ((float*)p)[i] = v;
  else ((bf16_raw*)p)[i] = f2bf(v);
}

// elementwise kinds (2,3,4): loss and grad of one element
__device__ __forceinline__ void elem_loss(int kind, float z, float y, float& l, float& g, int& c) {
  if (kind == 2) {
    const float p = 1.f / (1.f + __expf(-z));
    l = fmaxf(z, 0.f) - z * y + __logf(1.f + __expf(-fabsf(z)));
    g = p - y;
    c = ((p > 0.5f) == (y > 0.5f));
  } else if (kind == 3) {
    const float d = z - y;
    l = d * d;
    g = 2.f * d;
    c = 0;
  } else {
    const float eps = 1e-7f;
    const float p = fminf(fmaxf(z, eps), 1.f - eps);
    l = -(y * __logf(p) + (1.f - y) * __logf(1.f - p));
    g = (z <= eps || z >= 1.f - eps) ? 0.f : (p - y) / (p * (1.f - p));
    c = ((z > 0.5f) == (y > 0.5f));
  }
}

// ---- one thread per row (C <= 32) ----
__device__ __forceinline__ void row_thread(int kind, const void* logits, int lf32, const void* target, long row, int C,
                                           float gs, void* dl, int df32, float& lacc, int& cacc) {
  const long base = row * C;
  if (kind == 0 || kind == 1) {
    float mx = -INFINITY;
    int amx = 0;
    for (int c = 0; c < C; ++c) {
      const float v = ld_logit(logits, lf32, base + c);
      if (v > mx) { mx = v; amx = c; }
    }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(ld_logit(logits, lf32, base + c) - mx);
    const float lse = mx + __logf(se);
    if (kind == 0) {
      const long lab = ((const long*)target)[row];
      // a label outside [0, C) (kernels.debug_errors names it) reads no logit: it contributes lse
      const float zl = hx_guard((unsigned long)lab < (unsigned long)C) ? ld_logit(logits, lf32, base + lab) : 0.f;
      if (dl)
        for (int c = 0; c < C; ++c)
          st_grad(dl, df32, base + c, (__expf(ld_logit(logits, lf32, base + c) - lse) - (c == lab ? 1.f : 0.f)) * gs);
      lacc += lse - zl;
      cacc += (amx == lab);
    } else {
      const float* t = (const float*)target;
      float tz = 0.f, ts = 0.f, tmx = -INFINITY;
      int tam = 0;
      for (int c = 0; c < C; ++c) {
        const float y = t[base + c];
        tz += y * ld_logit(logits, lf32, base + c);
        ts += y;
        if (y > tmx) { tmx = y; tam = c; }
      }
      if (dl)
        for (int c = 0; c < C; ++c)
          st_grad(dl, df32, base + c, (__expf(ld_logit(logits, lf32, base + c) - lse) * ts - t[base + c]) * gs);
      lacc += ts * lse - tz;
      cacc += (amx == tam);
    }
  } else {
    const float* t = (const float*)target;
    for (int c = 0; c < C; ++c) {
      float l, g;
      int cc;
      elem_loss(kind, ld_logit(logits, lf32, base + c), t[base + c], l, g, cc);
      lacc += l;
      cacc += cc;
      if (dl) st_grad(dl, df32, base + c, g * gs);
    }
  }
}

// ---- one wave per row (C > 32) ----
__device__ __forceinline__ void row_wave(int kind, const void* logits, int lf32, const void* target, long row, int C,
                                         float gs, void* dl, int df32, int lane, float& lacc, int& cacc) {
  const long base = row * C;
  if (kind == 0 || kind == 1) {
    float mx = -INFINITY;
    int amx = 0;
    for (int c = lane; c < C; c += 64) {
      const float v = ld_logit(logits, lf32, base + c);
      if (v > mx) { mx = v; amx = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // wave argmax, first max wins on ties
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(amx, o, 64);
      if (om > mx || (om == mx && oa < amx)) { mx = om; amx = oa; }
    }
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += __expf(ld_logit(logits, lf32, base + c) - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    if (kind == 0) {
      const long lab = ((const long*)target)[row];
      if (dl)
        for (int c = lane; c < C; c += 64)
          st_grad(dl, df32, base + c, (__expf(ld_logit(logits, lf32, base + c) - lse) - (c == lab ? 1.f : 0.f)) * gs);
      if (lane == 0) {
        lacc += lse - (hx_guard((unsigned long)lab < (unsigned long)C) ? ld_logit(logits, lf32, base + lab) : 0.f);
        cacc += (amx == lab);
      }
    } else {
      const float* t = (const float*)target;
      float tz = 0.f, ts = 0.f, tmx = -INFINITY;
      int tam = 0;
      for (int c = lane; c < C; c += 64) {
        const float y = t[base + c];
        tz += y * ld_logit(logits, lf32, base + c);
        ts += y;
        if (y > tmx) { tmx = y; tam = c; }
      }
      tz = wave_sum(tz);
      ts = wave_sum(ts);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float om = __shfl_xor(tmx, o, 64);
        const int oa = __shfl_xor(tam, o, 64);
        if (om > tmx || (om == tmx && oa < tam)) { tmx = om; tam = oa; }
      }
      if (dl)
        for (int c = lane; c < C; c += 64)
          st_grad(dl, df32, base + c, (__expf(ld_logit(logits, lf32, base + c) - lse) * ts - t[base + c]) * gs);
      if (lane == 0) {
        lacc += ts * lse - tz;
        cacc += (amx == tam);
      }
    }
  } else {
    const float* t = (const float*)target;
    float ls = 0.f;
    int cs = 0;
    for (int c = lane; c < C; c += 64) {
      float l, g;
      int cc;
      elem_loss(kind, ld_logit(logits, lf32, base + c), t[base + c], l, g, cc);
      ls += l;
      cs += cc;
      if (dl) st_grad(dl, df32, base + c, g * gs);
    }
    ls = wave_sum(ls);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o, 64);
    if (lane == 0) {
      lacc += ls;
      cacc += cs;
    }
  }
}

__global__ __launch_bounds__(1024) void loss_k(int kind, const void* __restrict__ logits, int lf32,
                                               const void* __restrict__ target, int B, int C, float gscale,
                                               float* __restrict__ loss_sum, int* __restrict__ correct,
                                               void* __restrict__ dl, int df32, int per_thread) {
  __shared__ float sl[16];
  __shared__ int sc[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  float lacc = 0.f;
  int cacc = 0;
  if (per_thread) {
    for (long row = (long)blockIdx.x * blockDim.x + threadIdx.x; row < B; row += (long)gridDim.x * blockDim.x)
      row_thread(kind, logits, lf32, target, row, C, gscale, dl, df32, lacc, cacc);
    lacc = wave_sum(lacc);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cacc += __shfl_xor(cacc, o, 64);
  } else {
    for (long row = (long)blockIdx.x * nw + wave; row < B; row += (long)gridDim.x * nw)
      row_wave(kind, logits, lf32, target, row, C, gscale, dl, df32, lane, lacc, cacc);
  }
  if (lane == 0) {
    sl[wave] = lacc;
    sc[wave] = cacc;
  }
  __syncthreads();
  const bool det = gridDim.x > 1 && det_on();  // deterministic mode: the loss partials in block order
  if (det) det_turn_begin(DET_COLSUM, blockIdx.x);
  if (threadIdx.x == 0) {
    float l = 0.f;
    int c = 0;
    for (int w = 0; w < nw; ++w) {
      l += sl[w];
      c += sc[w];
    }
    l *= gscale;  // reported loss = sum * grad_scale (= the mean when grad_scale = 1/count)
    if (gridDim.x == 1) {  // single workgroup: overwrite, no memset / atomics needed
      if (loss_sum) *loss_sum = l;
      if (correct) *correct = c;
    } else {
      if (loss_sum) atomicAdd(loss_sum, l);
      if (correct) atomicAdd(correct, c);
    }
  }
  if (det) det_turn_end(DET_COLSUM, blockIdx.x, gridDim.x);
}

extern "C" int hopsx_loss_fwd_bwd(int kind, const void* logits, int logits_f32, const void* target, int B, int C,
                                  float grad_scale, float* loss_sum, int* correct, void* dlogits, int dlogits_f32,
                                  hipStream_t st) {
  const int per_thread = C <= 32 && !hopsx_disabled("loss_thread");
  int grid, block;
  if (per_thread) {
    block = B <= 1024 ? ((B + 63) / 64) * 64 : 256;
    if (block < 64) block = 64;
    grid = (B + block - 1) / block;
    if (grid > 1024) grid = 1024;
  } else {
    block = B <= 16 ? 1024 : 256;
    grid = B <= 16 ? 1 : (B + 3) / 4;
    if (grid > 1024) grid = 1024;
  }
  if (grid > 1) {
    if (loss_sum) hopsx_zero(loss_sum, sizeof(float), st);
    if (correct) hopsx_zero(correct, sizeof(int), st);
  }
  hipLaunchKernelGGL(loss_k, dim3(grid), dim3(block), 0, st, kind, logits, logits_f32, target, B, C, grad_scale,
                     loss_sum, correct, dlogits, dlogits_f32, per_thread);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Classifier head, fused: for logits = h . W^T + b (the last Dense layer, C <= 32 classes) one
// launch computes the loss, the correct count and dlogits (kept in LDS, never written), then
//   dW[n][k] += sum_r dl[r][n] h[r][k],  db[n] += sum_r dl[r][n],  dh[r][k] = sum_n dl[r][n] W[n][k]
// i.e. the loss kernel, the head's dgrad GEMM and its wgrad GEMM (three latency-bound launches at
// small batch) become one.  One workgroup per 64 rows; dW/db partials leave as f32 atomics.
constexpr int HEAD_ROWS = 32;
constexpr int HEAD_CMAX = 32;

// Several row blocks (B > HEAD_ROWS): each (bx, 0) workgroup leaves its loss / correct partial in a slot
// and the last to arrive sums the slots in row-block order and STORES the totals (no zeroing launches of
// the two outputs before the kernel, no float atomics, a deterministic sum).  <= HEAD_PART_MAX blocks.
constexpr int HEAD_PART_MAX = 64;
__device__ float g_head_part_l[HEAD_PART_MAX];
__device__ int g_head_part_c[HEAD_PART_MAX];
__device__ unsigned g_head_arrive;

// LDS: h tile [HEAD_ROWS][KD] bf16 | W [C][KD] bf16 | dlogits [HEAD_ROWS][C] f32 (dynamic size)
// The body takes its block coordinates explicitly (bx of gx row blocks, by of gy column blocks) so
// the fused Dense -> head kernel (mlp_head_k) can run it in its last workgroup; h == nullptr: the
// caller has already placed the h tile in the LDS image.
__device__ inline void head_ce_body(int kind, const void* __restrict__ logits, int lf32,
                                    const void* __restrict__ target, int B, int C, int KD, float gs,
                                    const bf16_raw* __restrict__ h, const bf16_raw* __restrict__ w,
                                    float* __restrict__ dw, float* __restrict__ db, bf16_raw* __restrict__ dh,
                                    float* __restrict__ loss_sum, int* __restrict__ correct, int vec,
                                    const float* __restrict__ bias, void* __restrict__ lout, int bx, int by, int gx,
                                    int gy, float dp = 0.f, const unsigned long long* __restrict__ drng = nullptr,
                                    unsigned dsalt = 0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char head_smem[];
  bf16_raw* sh = (bf16_raw*)head_smem;
  bf16_raw* sw = sh + HEAD_ROWS * KD;
  float* sdl = (float*)(sw + ((C * KD + 7) / 8) * 8);
  float* slog = sdl + HEAD_ROWS * C;  // forward mode: the logits computed here
  __shared__ float sl[16];
  __shared__ int sc[16];
  const int r0 = bx * HEAD_ROWS;
  const int nr = min(HEAD_ROWS, B - r0);
  // stage the h tile and W (one round trip of independent 16-B loads)
  if (vec) {
    const int hch = h ? nr * KD / 8 : 0, wch = C * KD / 8;
    for (int i = threadIdx.x; i < hch + wch; i += blockDim.x) {
      if (i < hch) ((bf16x8*)sh)[i] = ((const bf16x8*)(h + (long)r0 * KD))[i];
      else ((bf16x8*)sw)[i - hch] = ((const bf16x8*)w)[i - hch];
    }
  } else {
    if (h)
      for (int i = threadIdx.x; i < nr * KD; i += blockDim.x) sh[i] = h[(long)r0 * KD + i];
    for (int i = threadIdx.x; i < C * KD; i += blockDim.x) sw[i] = w[i];
  }
  // dp > 0: a Dropout between the previous layer and this head, folded in: h is the dropout's INPUT, the
  // staged tile gets dropout_k's mask and rounding, and the input gradient below the same mask (so dh is
  // the gradient of the dropout's input): neither dropout launch remains
  const uint64_t dkey = dp > 0.f ? drop_key(drng, dsalt) : 0;
  const float dscale = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  if (dp > 0.f && h) {
    __syncthreads();
    for (int i = threadIdx.x; i < nr * KD; i += blockDim.x)
      sh[i] = f2bf(bf2f(sh[i]) * (uniform01(dkey, (uint64_t)((long)r0 * KD + i)) >= dp ? dscale : 0.f));
    __syncthreads();
  }
  if (lout) {
    // forward mode: the head layer's own GEMM (logits = h W^T + b) runs here from the staged
    // operands, so the layer needs no forward launch; block y == 0 stores the logits
    __syncthreads();
    for (int e = threadIdx.x; e < nr * C; e += blockDim.x) {
      const int r = e / C, n = e - r * C;
      float s0 = 0.f, s1 = 0.f;
      int k = 0;
      if (vec)
        for (; k + 8 <= KD; k += 8) {
          const bf16x8 a = *(const bf16x8*)(sh + r * KD + k), b = *(const bf16x8*)(sw + n * KD + k);
#pragma unroll
          for (int u = 0; u < 8; u += 2) {
            s0 = fmaf(bf2f(a[u]), bf2f(b[u]), s0);
            s1 = fmaf(bf2f(a[u + 1]), bf2f(b[u + 1]), s1);
          }
        }
      for (; k < KD; ++k) s0 = fmaf(bf2f(sh[r * KD + k]), bf2f(sw[n * KD + k]), s0);
      float v = s0 + s1 + (bias ? bias[n] : 0.f);
      if (!lf32) v = bf2f(f2bf(v));  // the loss sees exactly the stored logits
      slog[e] = v;
      if (by == 0) {
        if (lf32) ((float*)lout)[(long)r0 * C + e] = v;
        else ((bf16_raw*)lout)[(long)r0 * C + e] = f2bf(v);
      }
    }
    __syncthreads();
  }
  float lacc = 0.f;
  int cacc = 0;
  if ((int)threadIdx.x < nr) {
    const void* lg = lout ? (const void*)slog
                          : lf32 ? (const void*)((const float*)logits + (long)r0 * C)
                                 : (const void*)((const bf16_raw*)logits + (long)r0 * C);
    const void* tg = kind == 0 ? (const void*)((const long*)target + r0)
                               : (const void*)((const float*)target + (long)r0 * C);
    row_thread(kind, lg, lout ? 1 : lf32, tg, threadIdx.x, C, gs, sdl, 1, lacc, cacc);
  }
  lacc = wave_sum(lacc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cacc += __shfl_xor(cacc, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sl[wave] = lacc;
    sc[wave] = cacc;
  }
  __syncthreads();
  // deterministic mode: the loss and head weight-gradient atomics of the row blocks in block order
  const bool det = gx > 1 && det_on();
  const unsigned dmy = (unsigned)(by * gx + bx);
  if (det) det_turn_begin(DET_COLSUM, dmy);
  if (threadIdx.x == 0 && by == 0) {
    float l = 0.f;
    int c = 0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
      l += sl[q];
      c += sc[q];
    }
    l *= gs;
    if (gx == 1) {
      if (loss_sum) *loss_sum = l;
      if (correct) *correct = c;
    } else if (gx <= HEAD_PART_MAX) {  // (deterministic as it is: a fixed-order sum)
      g_head_part_l[bx] = l;
      g_head_part_c[bx] = c;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const unsigned t = __hip_atomic_fetch_add(&g_head_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == (unsigned)gx - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        float lt = 0.f;
        int ct = 0;
        for (int q = 0; q < gx; ++q) {
          lt += __hip_atomic_load(g_head_part_l + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ct += __hip_atomic_load(g_head_part_c + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (loss_sum) *loss_sum = lt;
        if (correct) *correct = ct;
        __hip_atomic_store(&g_head_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      if (loss_sum) atomicAdd(loss_sum, l);
      if (correct) atomicAdd(correct, c);
    }
  }
  // weight / bias gradient of the head, all operands in LDS; 8 rows' loads in flight per step.
  // blockIdx.y owns columns [k0, k0 + kw) of KD (the dl recompute per column block is ~free)
  const int kw = (KD + gy - 1) / gy;
  const int k0 = by * kw, kn = min(kw, KD - k0);
  for (int e = threadIdx.x; e < C * kn; e += blockDim.x) {
    const int n = e / kn, k = k0 + (e - n * kn);
    float s0 = 0.f, s1 = 0.f;
    int r = 0;
    for (; r + 8 <= nr; r += 8) {
      float a[8], v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = sdl[(r + u) * C + n];
        v[u] = bf2f(sh[(r + u) * KD + k]);
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        s0 = fmaf(a[u], v[u], s0);
        s1 = fmaf(a[u + 1], v[u + 1], s1);
      }
    }
    for (; r < nr; ++r) s0 = fmaf(sdl[r * C + n], bf2f(sh[r * KD + k]), s0);
    const float s = s0 + s1;
    if (s != 0.f) atomicAdd(dw + (long)n * KD + k, s);
  }
  if (db && by == 0)
    for (int n = threadIdx.x; n < C; n += blockDim.x) {
      float s = 0.f;
      for (int r = 0; r < nr; ++r) s += sdl[r * C + n];
      if (s != 0.f) atomicAdd(db + n, s);
    }
  if (det) det_turn_end(DET_COLSUM, dmy, (unsigned)(gx * gy));
  // input gradient of the head (the previous layer applies its own act' mask)
  for (int e = threadIdx.x; e < nr * kn; e += blockDim.x) {
    const int r = e / kn, k = k0 + (e - r * kn);
    float s0 = 0.f, s1 = 0.f;
    int n = 0;
    for (; n + 8 <= C; n += 8) {
      float a[8], v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = sdl[r * C + n + u];
        v[u] = bf2f(sw[(n + u) * KD + k]);
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        s0 = fmaf(a[u], v[u], s0);
        s1 = fmaf(a[u + 1], v[u + 1], s1);
      }
    }
    for (; n < C; ++n) s0 = fmaf(sdl[r * C + n], bf2f(sw[n * KD + k]), s0);
    float v = s0 + s1;
    if (dp > 0.f)  // (the unfused chain: bf16 dX, then dropout_k on it)
      v = bf2f(f2bf(v)) * (uniform01(dkey, (uint64_t)((long)(r0 + r) * KD + k)) >= dp ? dscale : 0.f);
    dh[(long)(r0 + r) * KD + k] = f2bf(v);
  }
}

__global__ __launch_bounds__(1024) void head_ce_k(int kind, const void* __restrict__ logits, int lf32,
                                                 const void* __restrict__ target, int B, int C, int KD, float gs,
                                                 const bf16_raw* __restrict__ h, const bf16_raw* __restrict__ w,
                                                 float* __restrict__ dw, float* __restrict__ db,
                                                 bf16_raw* __restrict__ dh, float* __restrict__ loss_sum,
                                                 int* __restrict__ correct, int vec, const float* __restrict__ bias,
                                                 void* __restrict__ lout, float dp,
                                                 const unsigned long long* __restrict__ drng, unsigned dsalt) {
  head_ce_body(kind, logits, lf32, target, B, C, KD, gs, h, w, dw, db, dh, loss_sum, correct, vec, bias, lout,
               blockIdx.x, blockIdx.y, gridDim.x, gridDim.y, dp, drng, dsalt);
}

static size_t head_lds_bytes(int C, int KD) {
  return (size_t)HEAD_ROWS * KD * 2 + (size_t)((C * KD + 7) / 8) * 8 * 2 + (size_t)HEAD_ROWS * C * 4 * 2;
}

bool hopsx_head_ce_ok(int C, int KD) { return C >= 1 && C <= HEAD_CMAX && KD >= 1 && head_lds_bytes(C, KD) <= 65536; }

extern "C" int hopsx_head_ce(int kind, const void* logits, int logits_f32, const void* target, int B, int C, int KD,
                             float grad_scale, const void* h, const void* w, float* dw, float* db, void* dh,
                             float* loss_sum, int* correct, const float* bias, void* logits_out, float drop_p,
                             const unsigned long long* drop_rng, unsigned drop_salt, hipStream_t st) {
  if (!hopsx_head_ce_ok(C, KD) || B < 1) return -2;
  if (drop_p > 0.f && (!drop_rng || !h || drop_p >= 1.f)) return -3;
  const int grid = (B + HEAD_ROWS - 1) / HEAD_ROWS;
  // column blocks of >= 32 columns so a small batch still spreads over several CUs
  int gy = KD / 32;
  if (gy > 8) gy = 8;
  if (gy < 1) gy = 1;
  // (up to HEAD_PART_MAX row blocks the totals are stored, see g_head_part_l; more: atomics into zeroed totals)
  if (grid > HEAD_PART_MAX) {
    if (loss_sum) hopsx_zero(loss_sum, sizeof(float), st);
    if (correct) hopsx_zero(correct, sizeof(int), st);
  }
  const int vec = KD % 8 == 0 && ((uintptr_t)h % 16 == 0) && ((uintptr_t)w % 16 == 0);
  hipLaunchKernelGGL(head_ce_k, dim3(grid, gy), dim3(1024), head_lds_bytes(C, KD), st, kind, logits, logits_f32, target, B, C,
                     KD, grad_scale, (const bf16_raw*)h, (const bf16_raw*)w, dw, db, (bf16_raw*)dh, loss_sum,
                     correct, vec, bias, logits_out, drop_p, drop_rng, drop_salt);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused last hidden Dense layer + classifier head (training step, batch <= 32):
//   y   = act(x . W1^T + b1)                      [B, N1]  (stored bf16: dense1's backward reads it)
//   out = y . W2^T + b2,  loss, correct, dlogits  (head_ce_body)
//   dW2 += dl^T y,  db2 += sum dl,  dh = dl . W2  (the gradient dense1's backward starts from)
// At batch 32 the Dense layer is a K = 10,816 reduction onto 32 x 128 outputs: latency-bound, and
// the head is three more tiny GEMMs.  Three launches (split-K GEMM, its finish, the head) become
// one: every workgroup takes 128-deep K chunks, loads its MFMA fragments straight from global
// memory (16-B rows of x and W1 — no LDS staging, every load of the chunk in flight at once),
// adds its fp32 partial tile into a zero-at-rest workspace (memory-side float atomics), and the
// last workgroup to arrive (per-XCD sharded counter) reads the sums back with atomic exchanges
// (re-zeroing the workspace), applies bias + activation, and runs the head from LDS.
struct MlpHeadArgs {
  const bf16_raw* x;
  const bf16_raw* w1;
  const float* b1;
  int act1;
  bf16_raw* y;
  float* ws;         // fp32 [B][N1], zero at rest
  unsigned* arrive;  // kArriveWords, zero at rest
  int B, K, N1;
  int kind;
  const void* target;
  int C;
  float gs;
  const bf16_raw* w2;
  const float* b2;
  float* dw2;
  float* db2;
  bf16_raw* dh;
  float* loss_sum;
  int* correct;
  void* lout;
  int lf32;
  int vec2;
  unsigned long long* dbg;
  int rot;  // rotate each workgroup's workspace atomics (HOPSX_MLP_ROT, default on)
  // dp > 0: a Dropout between the Dense and the head (as head_ce_k's): y stays the Dense output (dense1's
  // backward reads its act' from it), the head reads dropout(y), and dh is the gradient of y
  float dp;
  const unsigned long long* drng;
  unsigned dsalt;
};


// phase stamps for tools/dbg_mlp_head.py (s_memrealtime, 100 MHz): null in production
static unsigned long long* g_mlp_dbg = nullptr;
extern "C" void hopsx_mlp_head_debug(void* p) { g_mlp_dbg = (unsigned long long*)p; }
__device__ inline void mlp_stamp(unsigned long long* dbg, int i) {
  if (dbg && threadIdx.x == 0) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: never waits on this thread's global stores
    dbg[i] = wall_clock64();
  }
}

// The last workgroup's part (256 threads): bias + activation, then the head from LDS.  Every loop
// is shaped for independent 16-B LDS reads and the LDS rows are padded by 16 B (a 256-B row
// stride puts every row's chunk k in the same banks).  Measured per phase with
// tools/dbg_mlp_head.py: scalar per-element loops chained ~300 dependent LDS reads per thread
// (31 us), unpadded 16-B loops 13 us.
constexpr int MLP_PAD = 8;  // bf16 elements of row padding
// dynamic LDS of mlp_head_k (byte offsets, 16-B aligned):
//   sh y bf16 [32][N1+8] | sw W2 bf16 [C][N1+8] | sdl f32 [32][C] | slog f32 [32][C] | sb1 f32 [N1] |
//   sb2 f32 [C] | stg targets (int64 [32] or f32 [32][C]) | st GEMM tile f32 [32][N1+4]
struct MlpLds {
  unsigned sh, sw, sdl, slog, sb1, sb2, stg, st, total;
  __host__ __device__ MlpLds(int C, int N1) {
    auto al = [](unsigned x) { return (x + 15u) / 16u * 16u; };
    const unsigned RS = N1 + MLP_PAD;
    sh = 0;
    sw = sh + HEAD_ROWS * RS * 2;
    sdl = al(sw + C * RS * 2);
    slog = sdl + HEAD_ROWS * C * 4;
    sb1 = al(slog + HEAD_ROWS * C * 4);
    sb2 = al(sb1 + N1 * 4);
    stg = al(sb2 + C * 4);
    st = al(stg + HEAD_ROWS * (C * 4 > 8 ? C * 4 : 8));
    total = al(st + HEAD_ROWS * (N1 + 4) * 4);
  }
};
static size_t mlp_lds_bytes(int C, int N1) { return MlpLds(C, N1).total; }

// loss + dlogits of one row per 16-lane group (C <= 16): max / sum / argmax by shuffles.  Kinds
// 0/1 (softmax CE), 2/3/4 elementwise.  Adds this lane's loss / correct contributions.
__device__ inline void mlp_loss16(int kind, const float* slog, const void* target, int B, int C, float gs,
                                  float* sdl, float& lacc, int& cacc) {
  for (int t0 = 0; t0 < B * 16; t0 += blockDim.x) {
    const int t = t0 + threadIdx.x;
    const int r = t >> 4, c = t & 15;
    const bool ok = r < B && c < C;
    const float z = ok ? slog[r * C + c] : -INFINITY;
    if (kind == 0 || kind == 1) {
      float mx = z;
      int am = ok ? c : 1 << 20;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float om = __shfl_xor(mx, o, 64);
        const int oa = __shfl_xor(am, o, 64);
        if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
      }
      float se = ok ? __expf(z - mx) : 0.f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) se += __shfl_xor(se, o, 64);
      const float lse = mx + __logf(se);
      const float p = ok ? __expf(z - lse) : 0.f;
      if (kind == 0) {
        long lab = r < B ? ((const long*)target)[r] : -1;
        if (r < B && c == 0 && !hx_guard((unsigned long)lab < (unsigned long)C)) lab = -1;
        if (ok) {
          sdl[r * C + c] = (p - (c == lab ? 1.f : 0.f)) * gs;
          if (c == lab) lacc += lse - z;
          if (c == 0) cacc += (am == lab);
        }
      } else {
        const float y = ok ? ((const float*)target)[(long)r * C + c] : 0.f;
        float tz = y * (ok ? z : 0.f), ts = y, tm = ok ? y : -INFINITY;
        int ta = ok ? c : 1 << 20;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          tz += __shfl_xor(tz, o, 64);
          ts += __shfl_xor(ts, o, 64);
          const float om = __shfl_xor(tm, o, 64);
          const int oa = __shfl_xor(ta, o, 64);
          if (om > tm || (om == tm && oa < ta)) { tm = om; ta = oa; }
        }
        if (ok) {
          sdl[r * C + c] = (p * ts - y) * gs;
          if (c == 0) {
            lacc += ts * lse - tz;
            cacc += (am == ta);
          }
        }
      }
    } else if (ok) {
      float l, g;
      int cc;
      elem_loss(kind, z, ((const float*)target)[(long)r * C + c], l, g, cc);
      sdl[r * C + c] = g * gs;
      lacc += l;
      cacc += cc;
    }
  }
}

// head operands that do not depend on the GEMM (W2, b1, b2, targets) -> LDS, by the waves the
// GEMM part leaves idle, while the W1 stream is in flight: the tail then has ONE global round trip
__device__ inline void mlp_prefetch(const MlpHeadArgs& a, int t, int nt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char head_smem[];
  const MlpLds L(a.C, a.N1);
  const int N1 = a.N1, C = a.C, N8 = N1 / 8, RS = N1 + MLP_PAD;
  bf16_raw* sw = (bf16_raw*)(head_smem + L.sw);
  for (int i = t; i < C * N8; i += nt) {
    const int c = i / N8, c8 = (i - c * N8) * 8;
    bf16x8 q;
    if (a.vec2) {
      q = *(const bf16x8*)(a.w2 + (long)c * N1 + c8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = (short)a.w2[(long)c * N1 + c8 + j];
    }
    *(bf16x8*)(sw + c * RS + c8) = q;
  }
  float* sb1 = (float*)(head_smem + L.sb1);
  float* sb2 = (float*)(head_smem + L.sb2);
  for (int i = t; i < N1; i += nt) sb1[i] = a.b1 ? a.b1[i] : 0.f;
  for (int i = t; i < C; i += nt) sb2[i] = a.b2 ? a.b2[i] : 0.f;
  if (a.kind == 0) {
    long* tg = (long*)(head_smem + L.stg);
    for (int i = t; i < a.B; i += nt) tg[i] = ((const long*)a.target)[i];
  } else {
    float* tg = (float*)(head_smem + L.stg);
    for (int i = t; i < a.B * C; i += nt) tg[i] = ((const float*)a.target)[i];
  }
}

// the input gradient of the dropout's input at element o (the unfused chain: bf16 dX, then dropout_k on it)
__device__ __forceinline__ float mlp_drop_grad(const MlpHeadArgs& a, float v, long o) {
  if (!(a.dp > 0.f)) return v;
  return bf2f(f2bf(v)) * (uniform01(drop_key(a.drng, a.dsalt), (uint64_t)o) >= a.dp ? 1.f / (1.f - a.dp) : 0.f);
}

__device__ inline void mlp_tail(const MlpHeadArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char head_smem[];
  const MlpLds L(a.C, a.N1);
  const int B = a.B, N1 = a.N1, C = a.C, tid = threadIdx.x, nt = blockDim.x;
  const int N8 = N1 / 8, RS = N1 + MLP_PAD;
  bf16_raw* sh = (bf16_raw*)(head_smem + L.sh);  // y  [B][RS]
  bf16_raw* sw = (bf16_raw*)(head_smem + L.sw);  // W2 [C][RS] (prefetched)
  float* sdl = (float*)(head_smem + L.sdl);      // dl [B][C]
  float* slog = (float*)(head_smem + L.slog);    // logits [B][C]
  const float* sb1 = (const float*)(head_smem + L.sb1);
  const float* sb2 = (const float*)(head_smem + L.sb2);
  const void* stg = head_smem + L.stg;
  __shared__ float sl[16];
  __shared__ int sc[16];
  // the workspace sums: every workgroup added to every line, so no stale copy survives in an L2
  // (float atomics execute at the memory side).  All loads first (one round trip), then re-zero.
  constexpr int MAXI = (HEAD_ROWS * 256 / 8 + 255) / 256;  // chunks per thread at B <= 32, N1 <= 256
  float4 v[MAXI][2];
#pragma unroll
  for (int u = 0; u < MAXI; ++u) {
    const int i = tid + u * nt;
    if (i < B * N8) {
      const float4* wp = (const float4*)(a.ws + (long)(i / N8) * N1 + (i % N8) * 8);
      v[u][0] = wp[0];
      v[u][1] = wp[1];
    }
  }
#pragma unroll
  for (int u = 0; u < MAXI; ++u) {
    const int i = tid + u * nt;
    if (i < B * N8) {
      const int r = i / N8, c8 = (i - r * N8) * 8;
      float4* wp = (float4*)(a.ws + (long)r * N1 + c8);
      wp[0] = make_float4(0.f, 0.f, 0.f, 0.f);
      wp[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      const float f[8] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w, v[u][1].x, v[u][1].y, v[u][1].z, v[u][1].w};
      bf16x8 q;
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = (short)f2bf(apply_act(f[j] + sb1[c8 + j], a.act1));
      *(bf16x8*)(a.y + (long)r * N1 + c8) = q;
      if (a.dp > 0.f) {  // (dropout_k's mask and rounding)
        const uint64_t key = drop_key(a.drng, a.dsalt);
        const float sc = 1.f / (1.f - a.dp);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          q[j] = (short)f2bf(bf2f((uint16_t)q[j]) * (uniform01(key, (uint64_t)((long)r * N1 + c8 + j)) >= a.dp ? sc : 0.f));
      }
      *(bf16x8*)(sh + r * RS + c8) = q;
    }
  }
  mlp_stamp(a.dbg, 4);
  __syncthreads();
  mlp_stamp(a.dbg, 5);
  const int lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int ncf = N1 >> 4;
  // C <= 16 with 16 waves: the three head GEMMs on MFMA (bf16 logits; fp32 16x16x4 for the
  // gradients, so dlogits keep fp32 precision) instead of per-thread FMA loops
  const bool mf = C <= 16 && nt == 1024;
  if (mf) {
    if (wave < 2) {  // logits rows 16*wave..: y [32 x N1] . W2^T [N1 x 16]
      f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < N1 / 32; ++ks) {
        const bf16x8 av = *(const bf16x8*)(sh + (wave * 16 + fr) * RS + ks * 32 + 8 * fq);
        const bf16x8 bv = zero_unless(*(const bf16x8*)(sw + (fr < C ? fr : 0) * RS + ks * 32 + 8 * fq), fr < C);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
      }
      if (N1 % 32) {  // a trailing 16-deep step (N1 % 32 == 16): zero the upper half of k
        const int k = (N1 / 32) * 32 + 8 * fq;
        const bool ok = k < N1;
        const bf16x8 av = zero_unless(*(const bf16x8*)(sh + (wave * 16 + fr) * RS + (ok ? k : 0)), ok);
        const bf16x8 bv = zero_unless(*(const bf16x8*)(sw + (fr < C ? fr : 0) * RS + (ok ? k : 0)), ok && fr < C);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 16 + 4 * fq + r;
        if (row < B && fr < C) {
          float v2 = acc[r] + sb2[fr];
          if (!a.lf32) v2 = bf2f(f2bf(v2));  // the loss sees exactly the stored logits
          const int o = row * C + fr;
          slog[o] = v2;
          if (a.lf32) ((float*)a.lout)[o] = v2;
          else ((bf16_raw*)a.lout)[o] = f2bf(v2);
        }
      }
    }
  } else {
  // logits: 4 lanes per output (a quarter of N1 each, combined by shuffles)
  const int nq = N8 % 4 == 0 ? 4 : 1;
  const int per = N8 / nq;
  for (int t0 = 0; t0 < B * C * nq; t0 += nt) {
    const int t = t0 + tid;
    const int o = t / nq, q = t - o * nq;
    float s0 = 0.f, s1 = 0.f;
    if (o < B * C) {
      const int r = o / C, c = o - r * C;
#pragma unroll 4
      for (int k8 = q * per; k8 < (q + 1) * per; ++k8) {
        const bf16x8 hv = *(const bf16x8*)(sh + r * RS + k8 * 8), wv = *(const bf16x8*)(sw + c * RS + k8 * 8);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          s0 = fmaf(bf2f((uint16_t)hv[j]), bf2f((uint16_t)wv[j]), s0);
          s1 = fmaf(bf2f((uint16_t)hv[j + 1]), bf2f((uint16_t)wv[j + 1]), s1);
        }
      }
    }
    float s = s0 + s1;
    if (nq == 4) {
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
    }
    if (o < B * C && q == 0) {
      const int c = o % C;
      float v2 = s + sb2[c];
      if (!a.lf32) v2 = bf2f(f2bf(v2));  // the loss sees exactly the stored logits
      slog[o] = v2;
      if (a.lf32) ((float*)a.lout)[o] = v2;
      else ((bf16_raw*)a.lout)[o] = f2bf(v2);
    }
  }
  }
  __syncthreads();
  mlp_stamp(a.dbg, 6);
  // loss, correct count, dlogits
  float lacc = 0.f;
  int cacc = 0;
  if (C <= 16) {
    mlp_loss16(a.kind, slog, stg, B, C, a.gs, sdl, lacc, cacc);
  } else if (tid < B) {
    row_thread(a.kind, slog, 1, stg, tid, C, a.gs, sdl, 1, lacc, cacc);
  }
  lacc = wave_sum(lacc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cacc += __shfl_xor(cacc, o, 64);
  if (lane == 0 && wave < 16) {
    sl[wave] = lacc;
    sc[wave] = cacc;
  }
  __syncthreads();
  if (wave == 0) {  // 16 wave partials: one shuffle tree, not a serial LDS loop
    const int nw = nt >> 6;
    float l = lane < nw && lane < 16 ? sl[lane] : 0.f;
    int c = lane < nw && lane < 16 ? sc[lane] : 0;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      l += __shfl_xor(l, o, 64);
      c += __shfl_xor(c, o, 64);
    }
    if (lane == 0) {
      if (a.loss_sum) *a.loss_sum = l * a.gs;
      if (a.correct) *a.correct = c;
    }
  }
  mlp_stamp(a.dbg, 7);
  if (mf) {
    // dW2 [C x N1] += dl^T [C x B] . y [B x N1]: wave w owns column fragment w (fp32 MFMA, K = B)
    if (wave < ncf) {
      f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int kb = 0; kb < B; kb += 4) {
        const int b = kb + fq;  // A[c = fr][k = fq] = dl[kb + fq][fr];  B[k = fq][n = fr] = y[kb + fq][16 w + fr]
        const float av = (b < B && fr < C) ? sdl[b * C + fr] : 0.f;
        const float bv = b < B ? bf2f(sh[b * RS + wave * 16 + fr]) : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 4 * fq + r;
        if (c < C && acc[r] != 0.f) atomicAdd(a.dw2 + (long)c * N1 + wave * 16 + fr, acc[r]);
      }
    }
    if (a.db2 && wave == (ncf < 16 ? 15 : 0) && lane < C) {
      float sm = 0.f;
      for (int r = 0; r < B; ++r) sm += sdl[r * C + lane];
      if (sm != 0.f) atomicAdd(a.db2 + lane, sm);
    }
    mlp_stamp(a.dbg, 8);
    // dh [B x N1] = dl [B x C] . W2 [C x N1]: tasks (row fragment, column fragment), K = C <= 16
    for (int tsk = wave; tsk < ((B + 15) / 16) * ncf; tsk += 16) {
      const int rf = tsk / ncf, f = tsk - rf * ncf;
      f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < 16; kc += 4) {
        const int c = kc + fq, b = rf * 16 + fr;  // A[b = fr][k = fq] = dl[b][c];  B[k][n] = W2[c][16 f + fr]
        const float av = (c < C && b < B) ? sdl[b * C + c] : 0.f;
        const float bv = c < C ? bf2f(sw[c * RS + f * 16 + fr]) : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rf * 16 + 4 * fq + r;
        if (b < B) a.dh[(long)b * N1 + f * 16 + fr] = f2bf(mlp_drop_grad(a, acc[r], (long)b * N1 + f * 16 + fr));
      }
    }
    return;
  }
  // dW2[c][k..k+8] += sum_r dl[r][c] y[r][k..k+8];  db2[c] += sum_r dl[r][c]
  for (int t = tid; t < C * N8 + C; t += nt) {
    if (t < C * N8) {
      const int c = t / N8, k = (t - c * N8) * 8;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int r = 0; r < B; ++r) {
        const float d = sdl[r * C + c];
        const bf16x8 hv = *(const bf16x8*)(sh + r * RS + k);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(d, bf2f((uint16_t)hv[j]), acc[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (acc[j] != 0.f) atomicAdd(a.dw2 + (long)c * N1 + k + j, acc[j]);
    } else if (a.db2) {
      const int c = t - C * N8;
      float s = 0.f;
      for (int r = 0; r < B; ++r) s += sdl[r * C + c];
      if (s != 0.f) atomicAdd(a.db2 + c, s);
    }
  }
  mlp_stamp(a.dbg, 8);
  // dh[r][k..k+8] = sum_c dl[r][c] W2[c][k..k+8]  (dense1's backward applies its own act')
  for (int t = tid; t < B * N8; t += nt) {
    const int r = t / N8, k = (t - r * N8) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int c = 0; c < C; ++c) {
      const float d = sdl[r * C + c];
      const bf16x8 wv = *(const bf16x8*)(sw + c * RS + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(d, bf2f((uint16_t)wv[j]), acc[j]);
    }
    bf16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = (short)f2bf(mlp_drop_grad(a, acc[j], (long)r * N1 + k + j));
    *(bf16x8*)(a.dh + (long)r * N1 + k) = q;
  }
}

// 1024 threads: waves 0-3 run the split-K GEMM part, all 16 waves the last workgroup's head (with
// one wave per SIMD every LDS read of the head's loops was exposed: 12 us for the tail)
template <int RF, int CF, int KS>
__global__ __launch_bounds__(1024) void mlp_head_k(MlpHeadArgs a) {
  unsigned long long* dbg0 = blockIdx.x == 0 ? a.dbg : nullptr;
  mlp_stamp(dbg0, 0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  extern __shared__ __attribute__((aligned(16))) unsigned char head_smem[];
  const MlpLds L(a.C, a.N1);
  float* st = (float*)(head_smem + L.st);  // this workgroup's partial tile [B][N1 + 4]
  const int SR = a.N1 + 4;
  if (wave >= 4) mlp_prefetch(a, threadIdx.x - 256, blockDim.x - 256);
  if (wave < 4) {
  const int fr = lane & 15, fq = lane >> 4;
  const int ncf = a.N1 >> 4;  // 16-column fragments; wave w owns fragments w, w + 4, ...
  f32x4 acc[RF][CF];
#pragma unroll
  for (int rf = 0; rf < RF; ++rf)
#pragma unroll
    for (int cf = 0; cf < CF; ++cf) acc[rf][cf] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = blockIdx.x * (KS * 32); k0 < a.K; k0 += gridDim.x * (KS * 32)) {
    bf16x8 av[RF][KS], bv[CF][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = k0 + ks * 32 + 8 * fq;
      const bool kok = k < a.K;  // K % 8 == 0: an 8-wide chunk is all in or all out
      const int kc = kok ? k : 0;
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) {
        const int r = rf * 16 + fr;
        const bool ok = kok && r < a.B;
        av[rf][ks] = zero_unless(*(const bf16x8*)(a.x + (long)(ok ? r : 0) * a.K + kc), ok);
      }
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const int f = wave + 4 * cf;
        const bool ok = kok && f < ncf;
        bv[cf][ks] = zero_unless(*(const bf16x8*)(a.w1 + (long)(ok ? f * 16 + fr : 0) * a.K + kc), ok);
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int rf = 0; rf < RF; ++rf)
#pragma unroll
        for (int cf = 0; cf < CF; ++cf)
          acc[rf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[rf][ks], bv[cf][ks], acc[rf][cf], 0, 0, 0);
  }
  mlp_stamp(dbg0, 1);
  // partial tile -> LDS (lane holds D[16 rf + 4 fq + r][16 f + fr]), then to the workspace as
  // whole-row atomics: every wave instruction adds 256 contiguous bytes (the full-rate shape of
  // memory-side float atomics; the fragment layout would issue 64-B pieces of 4 rows)
#pragma unroll
  for (int rf = 0; rf < RF; ++rf)
#pragma unroll
    for (int cf = 0; cf < CF; ++cf) {
      const int f = wave + 4 * cf;
      if (f >= ncf) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) st[(rf * 16 + 4 * fq + r) * SR + f * 16 + fr] = acc[rf][cf][r];
    }
  }
  __syncthreads();
  // every workgroup adds to every line of the workspace: start each one at a different 64-float
  // line (a.rot != 0) so the memory-side atomics of concurrent workgroups hit different addresses
  // instead of all queueing on the same line in the same order
  const int tot = a.B * a.N1;
  // deterministic mode: the split-K partial tiles are added in workgroup order
  const bool det = det_on();
  if (det) det_turn_begin(DET_MLP_WS, blockIdx.x);
  const int rot = a.rot ? (int)(((unsigned)blockIdx.x * 64u) % (unsigned)tot) & ~63 : 0;
  for (int i0 = threadIdx.x; i0 < tot; i0 += blockDim.x) {
    int i = i0 + rot;
    if (i >= tot) i -= tot;
    const int row = i / a.N1, col = i - row * a.N1;
    atomicAdd(a.ws + i, st[row * SR + col]);
  }
  if (det) det_turn_end(DET_MLP_WS, blockIdx.x, gridDim.x);
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's atomics are done
  __syncthreads();
  mlp_stamp(dbg0, 2);
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    s_last = grid_arrive_last(a.arrive) ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  mlp_stamp(a.dbg, 3);
  mlp_tail(a);
  mlp_stamp(a.dbg, 9);
}

extern "C" int hopsx_mlp_head(const void* x, const void* w1, const float* b1, int act1, void* y, float* ws,
                              unsigned* arrive, int B, int K, int N1, int kind, const void* target, int C,
                              float grad_scale, const void* w2, const float* b2, float* dw2, float* db2, void* dh,
                              float* loss_sum, int* correct, void* logits_out, int logits_f32, float drop_p,
                              const unsigned long long* drop_rng, unsigned drop_salt, hipStream_t st) {
  if (hopsx_disabled("mlp_head") || B < 1 || B > HEAD_ROWS || N1 < 16 || N1 % 16 || N1 > 256 || K < 8 || K % 8 ||
      !hopsx_head_ce_ok(C, N1) || !ws || !arrive || !logits_out ||
      ((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)y | (uintptr_t)dh | (uintptr_t)ws) % 16)
    return -2;
  // K chunk per workgroup: 128 (4 MFMA k-steps).  At the flagship shape (K 10,816) the launch took
  // 17.0 / 15.3 / 16.3 us at 64 / 128 / 256 (169 / 85 / 43 workgroups: more workgroups add float
  // atomics and arrival skew, fewer serialise the W1 stream); HOPSX_MLP_KS=2|4|8 overrides
  static const int ksenv = getenv("HOPSX_MLP_KS") ? atoi(getenv("HOPSX_MLP_KS")) : 0;
  const int ks = ksenv == 2 || ksenv == 4 || ksenv == 8 ? ksenv : 4;
  int G = (K + ks * 32 - 1) / (ks * 32);
  if (G > 256) G = 256;
  const int vec2 = N1 % 8 == 0 && (uintptr_t)w2 % 16 == 0;
  static const int rot_on = (int)hopsx_env_int("HOPSX_MLP_ROT", 1);
  MlpHeadArgs a{(const bf16_raw*)x, (const bf16_raw*)w1, b1, act1, (bf16_raw*)y, ws, arrive, B, K, N1, kind, target, C,
                grad_scale, (const bf16_raw*)w2, b2, dw2, db2, (bf16_raw*)dh, loss_sum, correct, logits_out,
                logits_f32, vec2, g_mlp_dbg, rot_on, drop_p, drop_rng, drop_salt};
  if (drop_p > 0.f && (!drop_rng || drop_p >= 1.f)) return -3;
  const size_t lds = mlp_lds_bytes(C, N1);
  const int rf = B > 16 ? 2 : 1, cf = (N1 / 16 + 3) / 4;
#define MLP_CASE(R, F)                                                                     \
  if (rf == R && cf == F) {                                                                \
    if (ks == 2) hipLaunchKernelGGL((mlp_head_k<R, F, 2>), dim3(G), dim3(1024), lds, st, a); \
    else if (ks == 4) hipLaunchKernelGGL((mlp_head_k<R, F, 4>), dim3(G), dim3(1024), lds, st, a); \
    else hipLaunchKernelGGL((mlp_head_k<R, F, 8>), dim3(G), dim3(1024), lds, st, a);         \
    return (int)hipGetLastError();                                                         \
  }
  MLP_CASE(1, 1) MLP_CASE(1, 2) MLP_CASE(1, 3) MLP_CASE(1, 4)
  MLP_CASE(2, 1) MLP_CASE(2, 2) MLP_CASE(2, 3) MLP_CASE(2, 4)
#undef MLP_CASE
  return -2;
}
