// Fused "multi-tensor" optimizers over ONE flat fp32 parameter buffer.
// Every model parameter is a view into a single contiguous master buffer, so an
// optimizer step is one memory-bound launch over the whole model (after the
// gradient all-reduce of the same flat buffer), which also:
//   * scales the gradient (1/world_size for a mean all-reduce, loss scaling),
//   * refreshes the bf16 shadow copy the MFMA kernels read,
//   * zeroes the gradient in place for the next step's atomic accumulation.
// The step counter lives on the device so the whole step is hipGraph-capturable.
#include "common.h"
#include "ops_api.h"

struct OptHP {
  float lr, gscale, wd, a, b, c, d, e;
};

__global__ void step_inc_k(float* step) { step[0] += 1.f; }

template <int KIND>
__global__ __launch_bounds__(256) void optim_k(float* __restrict__ p, float* __restrict__ g, float* __restrict__ s1,
                                               float* __restrict__ s2, float* __restrict__ s3,
                                               bf16_raw* __restrict__ shadow, long n, OptHP h,
                                               const float* __restrict__ step_dev, int zero_grad) {
  const float t = step_dev ? step_dev[0] : 1.f;
  float bc1 = 1.f, bc2 = 1.f;
  if (KIND == 1 || KIND == 2) {
    bc1 = 1.f - __powf(h.a, t);
    bc2 = 1.f - __powf(h.b, t);
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float w = p[i];
    float gr = g[i] * h.gscale;
    if (zero_grad) g[i] = 0.f;
    if (KIND == 0) {  // SGD + momentum (+ nesterov), L2 weight decay
      gr += h.wd * w;
      if (h.a != 0.f) {
        float buf = h.a * s1[i] + (1.f - h.b) * gr;
        s1[i] = buf;
        gr = (h.c != 0.f) ? gr + h.a * buf : buf;
      }
      w -= h.lr * gr;
    } else if (KIND == 1 || KIND == 2) {  // Adam / AdamW
      if (KIND == 1) gr += h.wd * w;
      else w -= h.lr * h.wd * w;
      const float m = h.a * s1[i] + (1.f - h.a) * gr;
      const float v = h.b * s2[i] + (1.f - h.b) * gr * gr;
      s1[i] = m;
      s2[i] = v;
      w -= h.lr * (m / bc1) / (sqrtf(v / bc2) + h.c);
    } else if (KIND == 3) {  // Adadelta
      gr += h.wd * w;
      const float ag = h.a * s1[i] + (1.f - h.a) * gr * gr;
      const float delta = sqrtf(s2[i] + h.b) / sqrtf(ag + h.b) * gr;
      s1[i] = ag;
      s2[i] = h.a * s2[i] + (1.f - h.a) * delta * delta;
      w -= h.lr * delta;
    } else if (KIND == 4) {  // RMSprop (optionally centered, momentum)
      gr += h.wd * w;
      const float v = h.a * s1[i] + (1.f - h.a) * gr * gr;
      s1[i] = v;
      float avg;
      if (h.d != 0.f) {
        const float ga = h.a * s3[i] + (1.f - h.a) * gr;
        s3[i] = ga;
        avg = sqrtf(fmaxf(v - ga * ga, 0.f)) + h.b;
      } else {
        avg = sqrtf(v) + h.b;
      }
      if (h.c != 0.f) {
        const float buf = h.c * s2[i] + gr / avg;
        s2[i] = buf;
        w -= h.lr * buf;
      } else {
        w -= h.lr * gr / avg;
      }
    } else if (KIND == 5) {  // Adagrad
      gr += h.wd * w;
      const float s = s1[i] + gr * gr;
      s1[i] = s;
      w -= h.lr * gr / (sqrtf(s) + h.a);
    } else if (KIND == 6) {  // FTRL-proximal (lr_power = -0.5), s1 = z, s2 = n
      const float nn = s2[i] + gr * gr;
      const float sigma = (sqrtf(nn) - sqrtf(s2[i])) / h.lr;
      const float z = s1[i] + gr - sigma * w;
      s1[i] = z;
      s2[i] = nn;
      w = (fabsf(z) <= h.a) ? 0.f : -(z - copysignf(h.a, z)) / ((h.c + sqrtf(nn)) / h.lr + 2.f * h.b);
    }
    p[i] = w;
    if (shadow) shadow[i] = f2bf(w);
  }
}

extern "C" int hopsx_optim_step(int kind, float* param, float* grad, float* s1, float* s2, float* s3,
                                void* shadow_bf16, long n, const float* hp, int nhp, float* step_dev, int zero_grad,
                                hipStream_t st) {
  OptHP h{0, 1, 0, 0, 0, 0, 0, 0};
  float* hv = &h.lr;
  for (int i = 0; i < nhp && i < 8; ++i) hv[i] = hp[i];
  if (step_dev) hipLaunchKernelGGL(step_inc_k, dim3(1), dim3(1), 0, st, step_dev);
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  bf16_raw* sh = (bf16_raw*)shadow_bf16;
#define OPT_CASE(K) \
  case K: hipLaunchKernelGGL(optim_k<K>, dim3(g), dim3(256), 0, st, param, grad, s1, s2, s3, sh, n, h, step_dev, zero_grad); break;
  switch (kind) {
    OPT_CASE(0) OPT_CASE(1) OPT_CASE(2) OPT_CASE(3) OPT_CASE(4) OPT_CASE(5) OPT_CASE(6)
    default: return -2;
  }
#undef OPT_CASE
  return (int)hipGetLastError();
}
