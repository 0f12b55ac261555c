// Fused loss forward+backward: one wave per row, online max/sum, the gradient
// w.r.t. the logits is written in the same pass, the loss and the
// correct-prediction count are reduced per workgroup and added with ONE atomic
// per workgroup (the metric all-reduce then moves 8 bytes per replica).
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

__global__ __launch_bounds__(256) void loss_k(int kind, const void* __restrict__ logits, int lf32,
                                              const void* __restrict__ target, int B, int C, float gscale,
                                              float* __restrict__ loss_sum, int* __restrict__ correct,
                                              void* __restrict__ dl, int df32) {
  __shared__ float sl[4];
  __shared__ int sc[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float lacc = 0.f;
  int cacc = 0;
  for (long row = (long)blockIdx.x * 4 + wave; row < B; row += (long)gridDim.x * 4) {
    const long base = row * C;
    if (kind == 0 || kind == 1) {
      float mx = -INFINITY;
      int amx = 0;
      for (int c = lane; c < C; c += 64) {
        const float v = ld_logit(logits, lf32, base + c);
        if (v > mx) { mx = v; amx = c; }
      }
      // wave argmax (first max wins on ties)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
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
        float zl = 0.f;
        for (int c = lane; c < C; c += 64) {
          const float z = ld_logit(logits, lf32, base + c);
          const float p = __expf(z - lse);
          if (c == lab) zl = z;
          if (dl) st_grad(dl, df32, base + c, (p - (c == lab ? 1.f : 0.f)) * gscale);
        }
        zl = wave_sum(zl);
        if (lane == 0) { lacc += lse - zl; cacc += (amx == lab); }
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
          for (int c = lane; c < C; c += 64) {
            const float p = __expf(ld_logit(logits, lf32, base + c) - lse);
            st_grad(dl, df32, base + c, (p * ts - t[base + c]) * gscale);
          }
        // CE = -sum y*(z - lse) = ts*lse - tz ; for normalised targets ts == 1
        if (lane == 0) { lacc += ts * lse - tz; cacc += (amx == tam); }
      }
    } else {
      const float* t = (const float*)target;
      float ls = 0.f;
      int cs = 0;
      for (int c = lane; c < C; c += 64) {
        const float z = ld_logit(logits, lf32, base + c);
        const float y = t[base + c];
        float g, l;
        if (kind == 2) {
          const float p = 1.f / (1.f + __expf(-z));
          l = fmaxf(z, 0.f) - z * y + __logf(1.f + __expf(-fabsf(z)));
          g = p - y;
          cs += ((p > 0.5f) == (y > 0.5f));
        } else if (kind == 3) {
          const float d = z - y;
          l = d * d;
          g = 2.f * d;
        } else {
          const float eps = 1e-7f;
          const float p = fminf(fmaxf(z, eps), 1.f - eps);
          l = -(y * __logf(p) + (1.f - y) * __logf(1.f - p));
          g = (z <= eps || z >= 1.f - eps) ? 0.f : (p - y) / (p * (1.f - p));
          cs += ((z > 0.5f) == (y > 0.5f));
        }
        ls += l;
        if (dl) st_grad(dl, df32, base + c, g * gscale);
      }
      ls = wave_sum(ls);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o, 64);
      if (lane == 0) { lacc += ls; cacc += cs; }
    }
  }
  if (lane == 0) { sl[wave] = lacc; sc[wave] = cacc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l = sl[0] + sl[1] + sl[2] + sl[3];
    const int c = sc[0] + sc[1] + sc[2] + sc[3];
    if (loss_sum) atomicAdd(loss_sum, l);
    if (correct) atomicAdd(correct, c);
  }
}

extern "C" int hopsx_loss_fwd_bwd(int kind, const void* logits, int logits_f32, const void* target, int B, int C,
                                  float grad_scale, float* loss_sum, int* correct, void* dlogits, int dlogits_f32,
                                  hipStream_t st) {
  int grid = (B + 3) / 4;
  if (grid > 1024) grid = 1024;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(loss_k, dim3(grid), dim3(256), 0, st, kind, logits, logits_f32, target, B, C, grad_scale,
                     loss_sum, correct, dlogits, dlogits_f32);
  return (int)hipGetLastError();
}
