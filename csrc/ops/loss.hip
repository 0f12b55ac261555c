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
      const float zl = ld_logit(logits, lf32, base + lab);
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
        lacc += lse - ld_logit(logits, lf32, base + lab);
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

// LDS: h tile [HEAD_ROWS][KD] bf16 | W [C][KD] bf16 | dlogits [HEAD_ROWS][C] f32 (dynamic size)
__global__ __launch_bounds__(1024) void head_ce_k(int kind, const void* __restrict__ logits, int lf32,
                                                 const void* __restrict__ target, int B, int C, int KD, float gs,
                                                 const bf16_raw* __restrict__ h, const bf16_raw* __restrict__ w,
                                                 float* __restrict__ dw, float* __restrict__ db,
                                                 bf16_raw* __restrict__ dh, float* __restrict__ loss_sum,
                                                 int* __restrict__ correct, int vec, const float* __restrict__ bias,
                                                 void* __restrict__ lout) {
  extern __shared__ __attribute__((aligned(16))) unsigned char head_smem[];
  bf16_raw* sh = (bf16_raw*)head_smem;
  bf16_raw* sw = sh + HEAD_ROWS * KD;
  float* sdl = (float*)(sw + ((C * KD + 7) / 8) * 8);
  float* slog = sdl + HEAD_ROWS * C;  // forward mode: the logits computed here
  __shared__ float sl[16];
  __shared__ int sc[16];
  const int r0 = blockIdx.x * HEAD_ROWS;
  const int nr = min(HEAD_ROWS, B - r0);
  // stage the h tile and W (one round trip of independent 16-B loads)
  if (vec) {
    const int hch = nr * KD / 8, wch = C * KD / 8;
    for (int i = threadIdx.x; i < hch + wch; i += blockDim.x) {
      if (i < hch) ((bf16x8*)sh)[i] = ((const bf16x8*)(h + (long)r0 * KD))[i];
      else ((bf16x8*)sw)[i - hch] = ((const bf16x8*)w)[i - hch];
    }
  } else {
    for (int i = threadIdx.x; i < nr * KD; i += blockDim.x) sh[i] = h[(long)r0 * KD + i];
    for (int i = threadIdx.x; i < C * KD; i += blockDim.x) sw[i] = w[i];
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
      if (blockIdx.y == 0) {
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
  if (threadIdx.x == 0 && blockIdx.y == 0) {
    float l = 0.f;
    int c = 0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
      l += sl[q];
      c += sc[q];
    }
    l *= gs;
    if (gridDim.x == 1) {
      if (loss_sum) *loss_sum = l;
      if (correct) *correct = c;
    } else {
      if (loss_sum) atomicAdd(loss_sum, l);
      if (correct) atomicAdd(correct, c);
    }
  }
  // weight / bias gradient of the head, all operands in LDS; 8 rows' loads in flight per step.
  // blockIdx.y owns columns [k0, k0 + kw) of KD (the dl recompute per column block is ~free)
  const int kw = (KD + gridDim.y - 1) / gridDim.y;
  const int k0 = blockIdx.y * kw, kn = min(kw, KD - k0);
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
  if (db && blockIdx.y == 0)
    for (int n = threadIdx.x; n < C; n += blockDim.x) {
      float s = 0.f;
      for (int r = 0; r < nr; ++r) s += sdl[r * C + n];
      if (s != 0.f) atomicAdd(db + n, s);
    }
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
    dh[(long)(r0 + r) * KD + k] = f2bf(s0 + s1);
  }
}

static size_t head_lds_bytes(int C, int KD) {
  return (size_t)HEAD_ROWS * KD * 2 + (size_t)((C * KD + 7) / 8) * 8 * 2 + (size_t)HEAD_ROWS * C * 4 * 2;
}

bool hopsx_head_ce_ok(int C, int KD) { return C >= 1 && C <= HEAD_CMAX && KD >= 1 && head_lds_bytes(C, KD) <= 65536; }

extern "C" int hopsx_head_ce(int kind, const void* logits, int logits_f32, const void* target, int B, int C, int KD,
                             float grad_scale, const void* h, const void* w, float* dw, float* db, void* dh,
                             float* loss_sum, int* correct, const float* bias, void* logits_out, hipStream_t st) {
  if (!hopsx_head_ce_ok(C, KD) || B < 1) return -2;
  const int grid = (B + HEAD_ROWS - 1) / HEAD_ROWS;
  // column blocks of >= 32 columns so a small batch still spreads over several CUs
  int gy = KD / 32;
  if (gy > 8) gy = 8;
  if (gy < 1) gy = 1;
  if (grid > 1) {  // (one row block: the blockIdx.y == 0 workgroup overwrites the totals)
    if (loss_sum) hopsx_zero(loss_sum, sizeof(float), st);
    if (correct) hopsx_zero(correct, sizeof(int), st);
  }
  const int vec = KD % 8 == 0 && ((uintptr_t)h % 16 == 0) && ((uintptr_t)w % 16 == 0);
  hipLaunchKernelGGL(head_ce_k, dim3(grid, gy), dim3(1024), head_lds_bytes(C, KD), st, kind, logits, logits_f32, target, B, C,
                     KD, grad_scale, (const bf16_raw*)h, (const bf16_raw*)w, dw, db, (bf16_raw*)dh, loss_sum,
                     correct, vec, bias, logits_out);
  return (int)hipGetLastError();
}
