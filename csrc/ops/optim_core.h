// Per-element optimizer update rules shared by the flat-arena optimizer kernel (optim.hip) and
// the fused whole-step kernels (widedeep_step.hip): one definition, bit-identical updates.
#pragma once
#include "common.h"

struct OptHP {
  float lr, gscale, wd, a, b, c, d, e;
};

// The hyper-parameters of a launch: from device memory when the optimizer keeps them there (a
// replayed hipGraph then sees learning-rate changes made after capture), else the by-value copy.
__device__ __forceinline__ OptHP load_hp(const OptHP& h, const float* hp_dev) {
  if (!hp_dev) return h;
  const OptHP* d = reinterpret_cast<const OptHP*>(hp_dev);
  return *d;
}

// Fused input prefetch (HBM-resident datasets): after its update each workgroup copies a slice of
// batch (cursor + 1) % nbatch of up to two resident tensors (images, labels) into the step's
// static input buffers, and the last-arriving workgroup advances the cursor.  The optimizer is the
// last kernel of a replayed training step, so nothing reads the inputs any more: the next batch
// lands with no launch and no copy engine on the critical path.
struct PrefetchJob {
  const unsigned char* src;  // batch 0 of the resident tensor; batch i at src + i * bytes
  unsigned char* dst;        // static input buffer
  long bytes;                // per batch (multiple of 16, 16-B aligned buffers)
};
struct Prefetch {
  PrefetchJob job[2];
  long long* cursor;  // device: index of the batch currently in dst
  int nbatch;
  int njobs;
};

// this workgroup's share of the next-batch copy (every workgroup reads the cursor before the
// last one arrives and advances it)
__device__ inline void prefetch_copy(const Prefetch& pf) {
  if (!pf.njobs) return;
  const long stride = (long)gridDim.x * blockDim.x;
  const long long next = (pf.cursor[0] + 1) % pf.nbatch;
  for (int j = 0; j < pf.njobs; ++j) {
    const uint4* src = (const uint4*)(pf.job[j].src + next * pf.job[j].bytes);
    uint4* dst = (uint4*)pf.job[j].dst;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < pf.job[j].bytes / 16; i += stride) dst[i] = src[i];
  }
}

// The last workgroup to arrive bumps the completed-step counter (bias correction), the dropout
// RNG counter and the prefetch cursor, so a captured step needs no bookkeeping launches.
// Arrival counter: kArriveWords uint32 (common.h grid_arrive_last: per-XCD shards, zero at rest);
// with one arrival word the fan-in cost 2.8 us of the flagship's optimizer launch, sharded 1.2.
__device__ inline void step_bookkeeping(unsigned* arrive, float* step_dev, float t, unsigned long long* rng,
                                        const Prefetch& pf) {
  if (!arrive) return;
  __syncthreads();
  if (threadIdx.x == 0 && grid_arrive_last(arrive)) {
    if (step_dev) step_dev[0] = t;
    if (rng) rng[1] += 1ull;
    if (pf.njobs) pf.cursor[0] = (pf.cursor[0] + 1) % pf.nbatch;
  }
}

// Adam-family bias corrections for step t
template <int KIND>
__device__ __forceinline__ void bias_corr(const OptHP& h, float t, float& bc1, float& bc2) {
  bc1 = 1.f;
  bc2 = 1.f;
  if (KIND == 1 || KIND == 2) {
    bc1 = 1.f - __powf(h.a, t);
    bc2 = 1.f - __powf(h.b, t);
  }
}

template <int KIND>
constexpr int nstate() {
  return KIND == 0 ? 1 : (KIND == 4 ? 3 : (KIND == 5 ? 1 : 2));
}

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
