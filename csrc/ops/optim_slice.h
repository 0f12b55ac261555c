// A fused optimizer's update of one contiguous slice of the flat parameter arena, run by extra
// workgroups of ANOTHER launch (horizontal fusion of the optimizer with the last backward kernel).
//
// In a single-GPU training step the optimizer is the last, memory-bound launch, and every layer
// above the network's input layer has its final gradient before the last backward launch (the
// input-side conv pair) starts.  That launch is latency-bound and leaves CUs idle, so it takes the
// update of those layers' arena slice as extra workgroups; the optimizer launch that follows only
// updates the remaining prefix (the input-side layers) and does the step bookkeeping.  Same
// per-element rule (optim_core.h upd<KIND>) and the same step count t (read before the optimizer
// launch bumps it): the result equals the unfused step's up to the FMA contractions the compiler
// picks for the same rule in the two kernels (tests/test_opt_colaunch_gpu.py).
#pragma once
#include "optim_core.h"

struct OptSlice {
  int kind;  // optim.hip kind; -1: no slice
  int nblk;  // workgroups given to the slice
  float* p;
  float* g;
  float* s1;
  float* s2;
  float* s3;
  bf16_raw* shadow;
  long n4;  // float4 elements (the slice is 16-B aligned, its length a multiple of 4)
  OptHP h;
  const float* hp_dev;
  const float* step_dev;  // completed steps (this step is t = step + 1)
};

template <int KIND>
__device__ __forceinline__ void opt_slice_body(const OptSlice& o, int blk) {
  const float t = (o.step_dev ? o.step_dev[0] : 0.f) + 1.f;
  const OptHP h = load_hp(o.h, o.hp_dev);
  float bc1, bc2;
  bias_corr<KIND>(h, t, bc1, bc2);
  constexpr int NS = nstate<KIND>();
  constexpr int UN = 2;
  const long stride = (long)o.nblk * blockDim.x;
  for (long i0 = (long)blk * blockDim.x + threadIdx.x; i0 < o.n4; i0 += UN * stride) {
    float4 w[UN], gr[UN], a[UN], b[UN], c[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const long i = i0 + u * stride;
      const long ic = i < o.n4 ? i : 0;
      w[u] = ((const float4*)o.p)[ic];
      gr[u] = ((const float4*)o.g)[ic];
      a[u] = NS >= 1 ? ((const float4*)o.s1)[ic] : make_float4(0, 0, 0, 0);
      b[u] = NS >= 2 ? ((const float4*)o.s2)[ic] : make_float4(0, 0, 0, 0);
      c[u] = NS >= 3 ? ((const float4*)o.s3)[ic] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const long i = i0 + u * stride;
      if (i >= o.n4) break;
      ((float4*)o.g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 ww = w[u], aa = a[u], bb = b[u], cc = c[u];
      ww.x = upd<KIND>(ww.x, gr[u].x * h.gscale, aa.x, bb.x, cc.x, h, bc1, bc2);
      ww.y = upd<KIND>(ww.y, gr[u].y * h.gscale, aa.y, bb.y, cc.y, h, bc1, bc2);
      ww.z = upd<KIND>(ww.z, gr[u].z * h.gscale, aa.z, bb.z, cc.z, h, bc1, bc2);
      ww.w = upd<KIND>(ww.w, gr[u].w * h.gscale, aa.w, bb.w, cc.w, h, bc1, bc2);
      ((float4*)o.p)[i] = ww;
      if (NS >= 1) ((float4*)o.s1)[i] = aa;
      if (NS >= 2) ((float4*)o.s2)[i] = bb;
      if (NS >= 3) ((float4*)o.s3)[i] = cc;
      if (o.shadow) {
        const uint32_t lo = (uint32_t)f2bf(ww.x) | ((uint32_t)f2bf(ww.y) << 16);
        const uint32_t hi = (uint32_t)f2bf(ww.z) | ((uint32_t)f2bf(ww.w) << 16);
        ((uint2*)o.shadow)[i] = make_uint2(lo, hi);
      }
    }
  }
}

// one out-of-line copy per translation unit: the host kernel's own hot path keeps its registers
__device__ __noinline__ inline void opt_slice_run(const OptSlice& o, int blk) {
  switch (o.kind) {
    case 0: opt_slice_body<0>(o, blk); break;
    case 1: opt_slice_body<1>(o, blk); break;
    case 2: opt_slice_body<2>(o, blk); break;
    case 3: opt_slice_body<3>(o, blk); break;
    case 4: opt_slice_body<4>(o, blk); break;
    case 5: opt_slice_body<5>(o, blk); break;
    case 6: opt_slice_body<6>(o, blk); break;
    default: break;
  }
}
