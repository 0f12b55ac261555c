// Per-element optimizer update rules shared by the flat-arena optimizer kernel (optim.hip) and
// the fused whole-step kernels (widedeep_step.hip): one definition, bit-identical updates.
#pragma once
#include "common.h"

struct OptHP {
  float lr, gscale, wd, a, b, c, d, e;
};

template <int KIND>
__device__ __forceinline__ float upd(float w, float gr, float& s1, float& s2, float& s3, const OptHP& h, float bc1,
                                     float bc2) {
  if (KIND == 0) {  // SGD + momentum (+ nesterov), L2 weight decay
    gr += h.wd * w;
    if (h.a != 0.f) {
      const float buf = h.a * s1 + (1.f - h.b) * gr;
      s1 = buf;
      gr = (h.c != 0.f) ? gr + h.a * buf : buf;
    }
    w -= h.lr * gr;
  } else if (KIND == 1 || KIND == 2) {  // Adam / AdamW
    if (KIND == 1) gr += h.wd * w;
    else w -= h.lr * h.wd * w;
    s1 = h.a * s1 + (1.f - h.a) * gr;
    s2 = h.b * s2 + (1.f - h.b) * gr * gr;
    w -= h.lr * (s1 / bc1) / (sqrtf(s2 / bc2) + h.c);
  } else if (KIND == 3) {  // Adadelta
    gr += h.wd * w;
    s1 = h.a * s1 + (1.f - h.a) * gr * gr;
    const float delta = sqrtf(s2 + h.b) / sqrtf(s1 + h.b) * gr;
    s2 = h.a * s2 + (1.f - h.a) * delta * delta;
    w -= h.lr * delta;
  } else if (KIND == 4) {  // RMSprop (optionally centered, momentum)
    gr += h.wd * w;
    s1 = h.a * s1 + (1.f - h.a) * gr * gr;
    float avg;
    if (h.d != 0.f) {
      s3 = h.a * s3 + (1.f - h.a) * gr;
      avg = sqrtf(fmaxf(s1 - s3 * s3, 0.f)) + h.b;
    } else {
      avg = sqrtf(s1) + h.b;
    }
    if (h.c != 0.f) {
      s2 = h.c * s2 + gr / avg;
      w -= h.lr * s2;
    } else {
      w -= h.lr * gr / avg;
    }
  } else if (KIND == 5) {  // Adagrad
    gr += h.wd * w;
    s1 += gr * gr;
    w -= h.lr * gr / (sqrtf(s1) + h.a);
  } else if (KIND == 6) {  // FTRL-proximal (lr_power = -0.5), s1 = z, s2 = n
    const float nn = s2 + gr * gr;
    const float sigma = (sqrtf(nn) - sqrtf(s2)) / h.lr;
    s1 += gr - sigma * w;
    s2 = nn;
    w = (fabsf(s1) <= h.a) ? 0.f : -(s1 - copysignf(h.a, s1)) / ((h.c + sqrtf(nn)) / h.lr + 2.f * h.b);
  }
  return w;
}
