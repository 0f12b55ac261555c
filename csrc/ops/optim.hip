// Fused "multi-tensor" optimizers over ONE flat fp32 parameter buffer.
// Every model parameter is a view into a single contiguous master buffer, so an
// optimizer step is one memory-bound launch over the whole model (after the
// gradient all-reduce of the same flat buffer), which also:
//   * scales the gradient (1/world_size for a mean all-reduce, loss scaling),
//   * refreshes the bf16 shadow copy the MFMA kernels read,
//   * zeroes the gradient in place for the next step's atomic accumulation,
//   * bumps the device step counter and the dropout RNG counter (last-arriving
//     workgroup), so a captured step needs no extra bookkeeping launches.
// Streams are moved as float4 (16 B/lane); the grid is capped at 2 workgroups
// per CU so the single arrival counter sees only ~512 atomics.
#include <cstdlib>

#include "common.h"
#include "ops_api.h"
#include "optim_core.h"



typedef float f4v __attribute__((ext_vector_type(4)));
__device__ inline void st_nt(float* dst, long i, const float4& v) {
  const f4v x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(dst) + i);
}

template <int KIND, int UN>
__global__ __launch_bounds__(256) void optim_k(float* __restrict__ p, float* __restrict__ g, float* __restrict__ s1,
                                               float* __restrict__ s2, float* __restrict__ s3,
                                               bf16_raw* __restrict__ shadow, long n, OptHP h,
                                               float* __restrict__ step_dev, unsigned* __restrict__ arrive,
                                               unsigned long long* __restrict__ rng, int zero_grad, int vec,
                                               Prefetch pf, int nt, const float* __restrict__ hp_dev,
                                               int pf_early) {
  // step_dev holds the number of COMPLETED steps; this step is t = step + 1.
  // Every workgroup reads it before its final barrier; the last workgroup to
  // finish bumps it (and the dropout RNG counter).
  const float t = (step_dev ? step_dev[0] : 0.f) + 1.f;
  h = load_hp(h, hp_dev);
  float bc1, bc2;
  bias_corr<KIND>(h, t, bc1, bc2);
  constexpr int NS = nstate<KIND>();
  // RMSprop without momentum and not centered (Keras' default, the benchmark notebook's RMSprop(0.2))
  // needs only the square average: skip the momentum / mean-gradient streams (42 -> 26 B per parameter
  // of HBM traffic).  Decided on the device hyper-parameters, so a captured graph follows a later change.
  const bool s23 = KIND != 4 || h.c != 0.f || h.d != 0.f;
  // HOPSX_OPT_PF_EARLY=1: the next batch's copy first: its cursor -> source -> store
  // chain does not depend on the update and nothing reads the input buffers any more, so its round
  // trips overlap the update's instead of following them
  if (pf_early) prefetch_copy(pf);
  const long n4 = vec ? (n >> 2) : 0;
  const long stride = (long)gridDim.x * blockDim.x;
  // UN float4 per thread per trip with every load issued before the first update: the launcher
  // picks UN so that a small arena (the 1.4 M-parameter flagship at 256 workgroups) is ONE trip —
  // one memory round trip instead of two dependent ones
  for (long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x; i0 < n4; i0 += UN * stride) {
    float4 w[UN], gr[UN], a[UN], b[UN], c[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const long i = i0 + u * stride;
      const long ic = i < n4 ? i : 0;  // clamped, unconditional loads
      w[u] = ((const float4*)p)[ic];
      gr[u] = ((const float4*)g)[ic];
      a[u] = NS >= 1 ? ((const float4*)s1)[ic] : make_float4(0, 0, 0, 0);
      b[u] = NS >= 2 && s23 ? ((const float4*)s2)[ic] : make_float4(0, 0, 0, 0);
      c[u] = NS >= 3 && s23 ? ((const float4*)s3)[ic] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const long i = i0 + u * stride;
      if (i >= n4) break;
      if (zero_grad) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 ww = w[u], aa = a[u], bb = b[u], cc = c[u];
      ww.x = upd<KIND>(ww.x, gr[u].x * h.gscale, aa.x, bb.x, cc.x, h, bc1, bc2);
      ww.y = upd<KIND>(ww.y, gr[u].y * h.gscale, aa.y, bb.y, cc.y, h, bc1, bc2);
      ww.z = upd<KIND>(ww.z, gr[u].z * h.gscale, aa.z, bb.z, cc.z, h, bc1, bc2);
      ww.w = upd<KIND>(ww.w, gr[u].w * h.gscale, aa.w, bb.w, cc.w, h, bc1, bc2);
      if (nt) {
        // master and optimizer state are next read by this kernel one step later: stream them
        // past L2 so the shadow, the zeroed grad and the activations keep it
        st_nt(p, i, ww);
        if (NS >= 1) st_nt(s1, i, aa);
        if (NS >= 2 && s23) st_nt(s2, i, bb);
        if (NS >= 3 && s23) st_nt(s3, i, cc);
      } else {
        ((float4*)p)[i] = ww;
        if (NS >= 1) ((float4*)s1)[i] = aa;
        if (NS >= 2 && s23) ((float4*)s2)[i] = bb;
        if (NS >= 3 && s23) ((float4*)s3)[i] = cc;
      }
      if (shadow) {
        const uint32_t lo = (uint32_t)f2bf(ww.x) | ((uint32_t)f2bf(ww.y) << 16);
        const uint32_t hi = (uint32_t)f2bf(ww.z) | ((uint32_t)f2bf(ww.w) << 16);
        ((uint2*)shadow)[i] = make_uint2(lo, hi);
      }
    }
  }
  for (long i = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float a = NS >= 1 ? s1[i] : 0.f, b = NS >= 2 && s23 ? s2[i] : 0.f, c = NS >= 3 && s23 ? s3[i] : 0.f;
    const float gr = g[i] * h.gscale;
    if (zero_grad) g[i] = 0.f;
    const float w = upd<KIND>(p[i], gr, a, b, c, h, bc1, bc2);
    p[i] = w;
    if (NS >= 1) s1[i] = a;
    if (NS >= 2 && s23) s2[i] = b;
    if (NS >= 3 && s23) s3[i] = c;
    if (shadow) shadow[i] = f2bf(w);
  }
  if (!pf_early) prefetch_copy(pf);
  step_bookkeeping(arrive, step_dev, t, rng, pf);
}

__global__ void bump_k(float* step_dev, unsigned long long* rng) {
  if (step_dev) step_dev[0] += 1.f;
  if (rng) rng[1] += 1ull;
}

extern "C" int hopsx_optim_step(int kind, float* param, float* grad, float* s1, float* s2, float* s3,
                                void* shadow_bf16, long n, const float* hp, int nhp, float* step_dev,
                                unsigned* arrive, unsigned long long* rng, int zero_grad, const void* const* pf_src,
                                void* const* pf_dst, const long* pf_bytes, int pf_njobs, long long* pf_cursor,
                                int pf_nbatch, const float* hp_dev, hipStream_t st) {
  Prefetch pf{};
  pf.njobs = 0;
  if (pf_njobs > 0 && pf_cursor && pf_nbatch > 0 && arrive) {  // the cursor advance needs the arrival counter
    for (int j = 0; j < pf_njobs && j < 2; ++j) {
      if (((uintptr_t)pf_src[j] | (uintptr_t)pf_dst[j] | (uintptr_t)pf_bytes[j]) % 16 != 0) return -5;
      pf.job[j] = PrefetchJob{(const unsigned char*)pf_src[j], (unsigned char*)pf_dst[j], pf_bytes[j]};
    }
    pf.njobs = pf_njobs < 2 ? pf_njobs : 2;
    pf.cursor = pf_cursor;
    pf.nbatch = pf_nbatch;
  }
  OptHP h{0, 1, 0, 0, 0, 0, 0, 0};
  float* hv = &h.lr;
  for (int i = 0; i < nhp && i < 8; ++i) hv[i] = hp[i];
  // 16-B vector path needs 16-B aligned streams
  const bool aligned = ((uintptr_t)param | (uintptr_t)grad | (uintptr_t)s1 | (uintptr_t)s2 | (uintptr_t)s3) % 16 == 0 &&
                       ((uintptr_t)shadow_bf16 % 8 == 0);
  long g = ((aligned ? n / 4 : n) + 255) / 256;
  // grid cap 512 (two workgroups per CU).  With the per-XCD sharded arrival counter the flagship
  // step measured 256: 0.0875, 384: 0.0859, 512: 0.0848, 768: 0.0849, 1024: 0.0850 ms
  // (profiles/r2s2_optim_grid_sweep.txt); with one arrival word 256 had been best (the fan-in
  // grew with the grid)
  static const int genv = getenv("HOPSX_OPT_GRID") ? atoi(getenv("HOPSX_OPT_GRID")) : 0;
  const int gcap = genv > 0 ? genv : 512;
  static const int nt = getenv("HOPSX_OPT_NT") ? atoi(getenv("HOPSX_OPT_NT")) : 0;
  static const int pf_early = (int)hopsx_env_int("HOPSX_OPT_PF_EARLY", 0);  // measured neutral (profiles/r3s7_flagship_ab.txt)
  if (g > gcap) g = gcap;
  if (g < 1) g = 1;
  // 6 float4 per thread when that covers the whole arena in one trip, else 3 (VGPR budget)
  static const int unenv = getenv("HOPSX_OPT_UN") ? atoi(getenv("HOPSX_OPT_UN")) : 0;
  const long n4 = aligned ? n / 4 : 0;
  const int un = unenv == 3 || unenv == 6 ? unenv : (n4 > 3L * g * 256 && n4 <= 6L * g * 256 ? 6 : 3);
  bf16_raw* sh = (bf16_raw*)shadow_bf16;
  // without an arrival counter the bookkeeping needs its own tiny launch
  unsigned* arr = (step_dev || rng) ? arrive : nullptr;
#define OPT_CASE(K)                                                                                             \
  case K:                                                                                                       \
    if (un == 6)                                                                                                \
      hipLaunchKernelGGL((optim_k<K, 6>), dim3(g), dim3(256), 0, st, param, grad, s1, s2, s3, sh, n, h, step_dev, \
                         arr, rng, zero_grad, (int)aligned, pf, nt, hp_dev, pf_early);                           \
    else                                                                                                        \
      hipLaunchKernelGGL((optim_k<K, 3>), dim3(g), dim3(256), 0, st, param, grad, s1, s2, s3, sh, n, h, step_dev, \
                         arr, rng, zero_grad, (int)aligned, pf, nt, hp_dev, pf_early);                           \
    break;
  switch (kind) {
    OPT_CASE(0) OPT_CASE(1) OPT_CASE(2) OPT_CASE(3) OPT_CASE(4) OPT_CASE(5) OPT_CASE(6)
    default: return -2;
  }
#undef OPT_CASE
  if ((step_dev || rng) && !arrive) hipLaunchKernelGGL(bump_k, dim3(1), dim3(1), 0, st, step_dev, rng);
  return (int)hipGetLastError();
}
