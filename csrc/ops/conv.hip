// Implicit-GEMM conv2d (NHWC activations, [Cout][KH][KW][Cin] weights) on MFMA.
//   fwd   : Y[m=(b,oh,ow)][co]      = im2col(X)[m][k=(kh,kw,ci)] . W[co][k]
//   dgrad : dX[m=(b,ih,iw)][ci]     = gatherT(dY)[m][k=(kh,kw,co)] . W^T[k][ci]
//   wgrad : dW[co][k=(kh,kw,ci)]   += dY^T[co][m] . im2col(X)[m][k]     (split-K, fp32 atomics)
// The gathers run inside the LDS staging of gemm_core.h, so no im2col buffer
// ever touches HBM.
#include "gemm_core.h"
#include "gemm_glds.h"
#include "ops_api.h"

HOPSX_DET_TU(conv)

using namespace hopsx;

static ConvGeom make_geom(const int* g) {
  ConvGeom c;
  c.B = g[0]; c.H = g[1]; c.W = g[2]; c.C = g[3];
  c.OH = g[4]; c.OW = g[5]; c.CO = g[6];
  c.KH = g[7]; c.KW = g[8]; c.sh = g[9]; c.sw = g[10]; c.ph = g[11]; c.pw = g[12]; c.dh = g[13]; c.dw = g[14];
  c.init_div();
  return c;
}

// ---------------------------------------------------------------------------
// Direct conv for tiny reductions (K = KH*KW*Cin <= 64: the Cin=1 input layers
// of every MNIST model, K = 4/9/16/25).  As an implicit GEMM these waste
// >= 60 % of each BK=64 MFMA tile on zero padding and pay a scalar im2col
// gather per element; here each thread owns (pixel, 4 output channels), the
// weights sit in LDS as fp32, and outputs leave as 8-byte stores.
// ---------------------------------------------------------------------------
// Input element of the direct kernels: bf16 activations, or raw uint8 pixels scaled on
// the fly (the u8->[0,1] normalisation of the input layer fused away: xscale != 0).
__device__ __forceinline__ float in_at(const void* x, float xscale, float xshift, long i) {
  return xscale != 0.f ? fmaf((float)((const uint8_t*)x)[i], xscale, xshift) : bf2f(((const bf16_raw*)x)[i]);
}

__global__ __launch_bounds__(256) void conv_direct_fwd_k(const void* __restrict__ x, float xscale, float xshift,
                                                         const bf16_raw* __restrict__ w,
                                                         const float* __restrict__ bias, bf16_raw* __restrict__ y,
                                                         ConvGeom g, int act) {
  extern __shared__ float sw[];  // [K][CO]
  const int K = g.KH * g.KW * g.C;
  for (int i = threadIdx.x; i < K * g.CO; i += blockDim.x) {
    const int co = i % g.CO, k = i / g.CO;
    sw[i] = bf2f(w[(long)co * K + k]);
  }
  __syncthreads();
  const int G = g.CO >> 2;
  const long total = (long)g.B * g.OH * g.OW * G;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int cg = t % G;
    const long pix = t / G;
    const int ow = pix % g.OW;
    const long r = pix / g.OW;
    const int oh = r % g.OH;
    const int b = r / g.OH;
    float acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bias ? bias[cg * 4 + j] : 0.f;
    int k = 0;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.sh - g.ph + kh * g.dh;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.sw - g.pw + kw * g.dw;
        const bool in = ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const long xo = (((long)b * g.H + ih) * g.W + iw) * g.C;
        for (int ci = 0; ci < g.C; ++ci, ++k) {
          const float xv = in ? in_at(x, xscale, xshift, xo + ci) : 0.f;
          const float* wr = sw + k * g.CO + cg * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] += xv * wr[j];
        }
      }
    }
    const uint32_t lo = (uint32_t)f2bf(apply_act(acc[0], act)) | ((uint32_t)f2bf(apply_act(acc[1], act)) << 16);
    const uint32_t hi = (uint32_t)f2bf(apply_act(acc[2], act)) | ((uint32_t)f2bf(apply_act(acc[3], act)) << 16);
    *(uint2*)(y + pix * g.CO + cg * 4) = make_uint2(lo, hi);
  }
}

// dW[co][k] += sum_m dY'[m][co] * im2col(X)[m][k] for K*CO <= 1024 (dY' = dY * act'(y)
// when y is given; dbias[co] += sum_m dY'[m][co]).  Threads = R replicas x K x CO;
// each thread walks a strided pixel subset straight from global memory with an
// incremental (b, oh, ow) decode (no divisions in the loop, no LDS staging, no
// barriers), replicas are reduced through LDS and every (co, k) gets ONE atomic
// per workgroup.
__global__ __launch_bounds__(1024) void conv_direct_wgrad_k(const bf16_raw* __restrict__ dy,
                                                            const bf16_raw* __restrict__ x, float* __restrict__ dw,
                                                            float* __restrict__ dbias, const bf16_raw* __restrict__ y,
                                                            int yact, ConvGeom g, int pix_per_block, int R,
                                                            float* __restrict__ slab) {
  extern __shared__ float red[];  // [R][K*CO + CO]
  const int K = g.KH * g.KW * g.C;
  const int KC = K * g.CO;
  const int tid = threadIdx.x;
  const int rep = tid / KC, r = tid % KC;
  const int co = r % g.CO, k = r / g.CO;
  const int M = g.B * g.OH * g.OW;
  const int m0 = blockIdx.x * pix_per_block, m1 = min(M, m0 + pix_per_block);
  float acc0 = 0.f, acc1 = 0.f, b0 = 0.f, b1 = 0.f;
  if (rep < R) {
    const int ci = k % g.C, t = k / g.C;
    const int kw = t % g.KW, kh = t / g.KW;
    // two independent pixel streams per thread (m and m + R) for memory-level parallelism
    int m = m0 + rep;
    const int ohw = g.OH * g.OW;
    int b = m / ohw, rem = m - b * ohw;
    int oh = rem / g.OW, ow = rem - oh * g.OW;
    auto advance = [&](int step) {
      ow += step;
      while (ow >= g.OW) {
        ow -= g.OW;
        if (++oh == g.OH) { oh = 0; ++b; }
      }
    };
    auto term = [&](int mm, int bb, int hh, int ww, float& acc, float& bacc) {
      float d = bf2f(dy[(long)mm * g.CO + co]);
      if (y) d *= act_grad_from_out(bf2f(y[(long)mm * g.CO + co]), yact);
      const int ih = hh * g.sh - g.ph + kh * g.dh, iw = ww * g.sw - g.pw + kw * g.dw;
      const float xv = (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
                           ? bf2f(x[(((long)bb * g.H + ih) * g.W + iw) * g.C + ci]) : 0.f;
      acc += d * xv;
      bacc += d;
    };
    for (; m + R < m1; m += 2 * R) {
      const int bA = b, hA = oh, wA = ow;
      advance(R);
      term(m, bA, hA, wA, acc0, b0);
      term(m + R, b, oh, ow, acc1, b1);
      advance(R);
    }
    if (m < m1) term(m, b, oh, ow, acc0, b0);
    red[rep * (KC + g.CO) + r] = acc0 + acc1;
    if (k == 0) red[rep * (KC + g.CO) + KC + co] = b0 + b1;
  }
  __syncthreads();
  const bool det = !slab && det_on();  // deterministic mode: the atomic path adds in workgroup order
  if (det) det_turn_begin(DET_WGRAD, blockIdx.x);
  if (rep == 0) {
    float s = 0.f, sb = 0.f;
    for (int q = 0; q < R; ++q) {
      s += red[q * (KC + g.CO) + r];
      if (k == 0) sb += red[q * (KC + g.CO) + KC + co];
    }
    if (slab) {  // plain stores; slab_reduce_k sums the workgroups (no same-address atomics)
      slab[(long)blockIdx.x * (KC + g.CO) + r] = s;
      if (k == 0) slab[(long)blockIdx.x * (KC + g.CO) + KC + co] = sb;
    } else {
      if (s != 0.f) atomicAdd(dw + (long)co * K + k, s);
      if (dbias && k == 0 && sb != 0.f) atomicAdd(dbias + co, sb);
    }
  }
  if (det) det_turn_end(DET_WGRAD, blockIdx.x, gridDim.x);
}

// Small-K weight gradient (K = KH*KW*C <= 16, CO % 8 == 0): the input layers of the MNIST
// models.  Work item = (output pixel, group of 8 output channels); a thread owns one channel
// group for its whole life (the grid stride is a multiple of CO/8), loads dY (and y for the
// fused act' mask) as 16-B vectors, keeps acc[8][K+1] (last column = bias) in registers and
// processes UNROLL items per trip with all loads issued up front, so the loads are
// independent (the old (k, co)-per-thread walk was a chain of dependent L2 round trips).
// Lanes with the same channel group are reduced with xor-shuffles, waves through LDS, each
// workgroup writes its partial row to a slab, and the last workgroup to finish (ticket
// counter, agent-scope release/acquire) sums the rows into dW/db — no same-address atomics
// (91+ workgroups hammering 160 addresses cost ~15 us) and no second kernel.
template <int KK>
__global__ __launch_bounds__(256) void conv_wgrad_smallk_k(const bf16_raw* __restrict__ dy, const void* __restrict__ x,
                                                          float xscale, float xshift, float* __restrict__ dw,
                                                          float* __restrict__ dbias, const bf16_raw* __restrict__ y,
                                                          int yact, ConvGeom g, long total, float* __restrict__ slab,
                                                          unsigned* __restrict__ counter) {
  constexpr int UNROLL = 4;
  const int G = g.CO >> 3;
  const bf16_raw* yp = y ? y : dy;
  const int cg = threadIdx.x % G;
  float acc[8][KK + 1];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k <= KK; ++k) acc[j][k] = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long base = (long)blockIdx.x * blockDim.x + threadIdx.x; base < total; base += UNROLL * stride) {
    bf16x8 dv[UNROLL], yv[UNROLL];
    float xv[UNROLL][KK];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const long idx = base + u * stride;
      const bool ok = idx < total;
      const int pi = ok ? (int)(idx / G) : 0;  // clamped: every load below is unconditional
      dv[u] = zero_unless(*(const bf16x8*)(dy + (long)pi * g.CO + cg * 8), ok);
      yv[u] = *(const bf16x8*)(yp + (long)pi * g.CO + cg * 8);  // unconditional (yp = y or dy)
      const int b = g.fOHW.div(pi), rem = pi - b * (g.OH * g.OW);
      const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
#pragma unroll
      for (int k = 0; k < KK; ++k) {
        const int ci = k % g.C, t = k / g.C;  // KK is small; the compiler folds what it can
        const int kw = t % g.KW, kh = t / g.KW;
        const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
        const bool in = ok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const long xi = in ? (((long)b * g.H + ih) * g.W + iw) * g.C + ci : 0;
        const float xval = in_at(x, xscale, xshift, xi);
        xv[u][k] = in ? xval : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = bf2f((uint16_t)dv[u][j]);
        if (y) d *= act_grad_from_out(bf2f((uint16_t)yv[u][j]), yact);
#pragma unroll
        for (int k = 0; k < KK; ++k) acc[j][k] += d * xv[u][k];
        acc[j][KK] += d;
      }
    }
  }
  // lanes l, l+G, l+2G, ... hold the same channel group
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k <= KK; ++k)
      for (int o = G; o < 64; o <<= 1) acc[j][k] += __shfl_xor(acc[j][k], o, 64);
  __shared__ float red[4 * 32 * 8 * (KK + 1) + 1];  // [wave][group][8*(K+1)] + the "last arriver" flag
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = 32 * 8 * (KK + 1);
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k <= KK; ++k) red[wave * per + lane * 8 * (KK + 1) + j * (KK + 1) + k] = acc[j][k];
  }
  __syncthreads();
  const int nel = G * 8 * (KK + 1);  // element e = grp*8*(K+1) + j*(K+1) + k
  for (int e = threadIdx.x; e < nel; e += blockDim.x)
    slab[(long)blockIdx.x * nel + e] = red[e] + red[per + e] + red[2 * per + e] + red[3 * per + e];
  // in-launch combine (one agent-scope release per workgroup, one acquire in the last one):
  // the last workgroup to draw a ticket sums every slab row; it also re-arms the counter
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    red[4 * per] = (t == gridDim.x - 1) ? 1.f : 0.f;
  }
  __syncthreads();
  if (red[4 * per] == 0.f) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *counter = 0u;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nel; e += blockDim.x) {
    float s = 0.f;
#pragma unroll 16
    for (int b = 0; b < (int)gridDim.x; ++b) s += slab[(long)b * nel + e];
    const int grp = e / (8 * (KK + 1)), r = e - grp * (8 * (KK + 1));
    const int j = r / (KK + 1), k = r - j * (KK + 1);
    const int co = grp * 8 + j;
    if (k < KK) dw[(long)co * KK + k] += s;
    else if (dbias) dbias[co] += s;
  }
}

// Weight gradient of a ONE-channel input layer (C = 1, K = KH*KW <= 25 taps, CO in {8,16,32,64}): the E1 /
// HPO MNIST models' 4x4 input conv (mnist.ipynb:154-164), 20,000 pixels x 32 channels x 17 outputs at
// batch 32 — ~11 M MACs that the channel-group kernel above spent 65 us on (25-way xor-shuffle trees per
// accumulator, a 128-row single-workgroup combine: profiles/r6_e1_fit_kernels.txt).  Here:
//   * workgroup = a contiguous range of PPW pixels; it stages d = dY * act'(y) for them [PPW][CO] fp32
//     and the im2col rows of the input [PPW][K] in LDS (16-B dY loads, every load in flight at once);
//   * thread (co, tap group): accumulates its <= 7 (tap, co) outputs (the bias as tap K) over the range
//     from LDS — no shuffles, no atomics;
//   * partial rows -> the slab; a two-level ticket combine: the last of each group of 16 workgroups sums
//     its group's rows in row order, the last group sums the group rows in order and adds dW / db —
//     deterministic (fixed summation order) and ~2 L2 round trips instead of one per 16 rows.
constexpr int C1_GROUP = 16;
// the combine's partial rows cross workgroups (and XCDs, each with its own L2) inside one launch: written
// write-through (sc1) and read with sc1 loads, after a vmcnt drain and a relaxed ticket, so neither an
// agent-scope release (an L2 write-back) nor an acquire (an L2 invalidate) is needed per level
__device__ __forceinline__ __amdgpu_buffer_rsrc_t c1_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void c1_st(__amdgpu_buffer_rsrc_t r, long e, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(e * 4), 0, 16);
}
__device__ __forceinline__ float c1_ld(__amdgpu_buffer_rsrc_t r, long e) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(e * 4), 0, 16));
}

__global__ __launch_bounds__(256) void conv_wgrad_c1_k(const bf16_raw* __restrict__ dy, const void* __restrict__ x,
                                                      float xscale, float xshift, float* __restrict__ dw,
                                                      float* __restrict__ dbias, const bf16_raw* __restrict__ y,
                                                      int yact, ConvGeom g, int P, int PPW, float* __restrict__ slab,
                                                      unsigned* __restrict__ counter, int stop) {
  extern __shared__ float c1s[];
  const int CO = g.CO, K = g.KH * g.KW, NE = CO * (K + 1);
  float* D = c1s;                  // [PPW][CO] masked dY
  float* XS = c1s + PPW * CO;      // [PPW][K] input taps
  __shared__ int last;
  const int m0 = blockIdx.x * PPW, np = min(PPW, P - m0);
  // ---- stage d and the taps
  // (every load of a thread is issued before any LDS store: a load -> store loop waits out one memory
  // round trip per iteration)
  const int G8 = CO >> 3;
  constexpr int QD = 8, QX = 20;  // per-thread items: PPW * CO / 8 / 256 <= 8, PPW * K / 256 <= 20
  {
    bf16x8 dv[QD], yv[QD];
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int pi = min(i / G8, np - 1), cg = i % G8;
      const long o = (long)(m0 + pi) * CO + cg * 8;
      dv[q] = *(const bf16x8*)(dy + o);
      yv[q] = y ? *(const bf16x8*)(y + o) : dv[q];
    }
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      const int i = threadIdx.x + 256 * q;
      if (i < np * G8) {
        const int pi = i / G8, cg = i - pi * G8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = bf2f((uint16_t)dv[q][j]);
          if (y) d *= act_grad_from_out(bf2f((uint16_t)yv[q][j]), yact);
          D[pi * CO + cg * 8 + j] = d;
        }
      }
    }
  }
  {
    float xv[QX];
#pragma unroll
    for (int q = 0; q < QX; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int pi = i / K, k = i - pi * K;
      const int m = m0 + min(pi, np - 1);
      const int b = g.fOHW.div(m), rem = m - b * (g.OH * g.OW);
      const int oh = g.fOW.div(rem), ow = rem - oh * g.OW;
      const int kw = k % g.KW, kh = k / g.KW;
      const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
      const bool in = i < np * K && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const float v = in_at(x, xscale, xshift, in ? ((long)b * g.H + ih) * g.W + iw : 0);
      xv[q] = in ? v : 0.f;
    }
#pragma unroll
    for (int q = 0; q < QX; ++q) {
      const int i = threadIdx.x + 256 * q;
      if (i < np * K) XS[i] = xv[q];
    }
  }
  __syncthreads();
  if (stop == 1) return;  // (HOPSX_C1_STOP: timing of the phases, tools/c1_wgrad_bench.py)
  // ---- accumulate: thread (co, pixel lane pl) sums ALL K + 1 outputs of channel co over pixels pl, pl + PL,
  // ... (a thread walking every pixel for a few taps was a 179-deep LDS-latency chain at one wave per SIMD)
  constexpr int KMAX = 25;
  const int PL = 256 / CO, co = threadIdx.x % CO, pl = threadIdx.x / CO;
  float acc[KMAX + 1];
#pragma unroll
  for (int k = 0; k <= KMAX; ++k) acc[k] = 0.f;
  for (int pi = pl; pi < np; pi += PL) {
    const float d = D[pi * CO + co];
    const float* xr = XS + pi * K;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < K) acc[k] = fmaf(d, xr[k], acc[k]);
    acc[KMAX] += d;
  }
  __syncthreads();  // (D / XS are read; their LDS becomes the pixel-lane reduction buffer)
  float* RD = c1s;  // [PL][CO][K + 1]
#pragma unroll
  for (int k = 0; k <= KMAX; ++k) {
    if (k < K) RD[(pl * CO + co) * (K + 1) + k] = acc[k];
  }
  RD[(pl * CO + co) * (K + 1) + K] = acc[KMAX];
  __syncthreads();
  // rows padded to whole 128-B lines: a line is only ever written by one workgroup, so no reader's L2 can
  // hold a copy of it filled before that write
  const int NEP = (NE + 31) & ~31;
  const auto SR = c1_rsrc(slab);
  for (int e = threadIdx.x; e < NE; e += 256) {
    float t = 0.f;
    for (int q = 0; q < PL; ++q) t += RD[q * NE + e];  // pixel-lane order: deterministic
    c1_st(SR, (long)blockIdx.x * NEP + e, t);
  }
  if (stop == 2) return;
  // ---- level 1: the last workgroup of this group of 16 sums the group's rows (row order)
  const int ngrp = (gridDim.x + C1_GROUP - 1) / C1_GROUP, grp = blockIdx.x / C1_GROUP;
  const int g0 = grp * C1_GROUP, g1 = min((int)gridDim.x, g0 + C1_GROUP);
  const long s2 = (long)gridDim.x * NEP;  // slab2 = slab + s2: [ngrp][NEP]
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's rows written through
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter + 1 + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (unsigned)(g1 - g0 - 1);
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) counter[1 + grp] = 0u;  // re-armed for the next launch
  for (int e = threadIdx.x; e < NE; e += 256) {
    float v[C1_GROUP];
#pragma unroll
    for (int q = 0; q < C1_GROUP; ++q) v[q] = g0 + q < g1 ? c1_ld(SR, (long)(g0 + q) * NEP + e) : 0.f;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < C1_GROUP; ++q) t += v[q];
    c1_st(SR, s2 + (long)grp * NEP + e, t);
  }
  // ---- level 2: the last group sums the group rows (group order) into dW / db
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (unsigned)(ngrp - 1);
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) counter[0] = 0u;
  for (int e = threadIdx.x; e < NE; e += 256) {
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = q < ngrp ? c1_ld(SR, s2 + (long)q * NEP + e) : 0.f;  // (ngrp <= 14)
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += v[q];
    const int c = e / (K + 1), k = e - c * (K + 1);
    if (k < K) dw[(long)c * K + k] += t;
    else if (dbias) dbias[c] += t;
  }
}

// sums the per-workgroup partials: element e < KC is dW[co][k] (slab index r = k*CO + co),
// e >= KC the bias of channel e - KC
// one workgroup per output element: 256 lanes stride over the workgroup partials
// (coalescing is poor but every load is independent), wave + LDS tree reduction
__global__ __launch_bounds__(256) void slab_reduce_k(const float* __restrict__ slab, int nblk, int KC, int CO, int K,
                                                     float* __restrict__ dw, float* __restrict__ dbias) {
  const int e = blockIdx.x;
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) s += slab[(long)b * (KC + CO) + e];
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  s = red[0] + red[1] + red[2] + red[3];
  if (e < KC) {
    const int co = e % CO, k = e / CO;
    dw[(long)co * K + k] += s;
  } else if (dbias) {
    dbias[e - KC] += s;
  }
}

// ---- small-M split-K for the forward / dgrad GEMMs of gemm_core.h's engine ------------------------
// The stage-3/4 ResNet-50 convs at small batch (batch 8: 392 / 1,568 output pixels, K up to 4,608)
// give a few hundred 32x32 tiles that each walk all of K alone: 58-72 us for the 7x7 3x3 layers vs
// PyTorch's 25-28 (profiles/r5_conv_gemm_vs_torch.txt).  When plan_gemm would split K, the GEMM runs
// as EpiAtomicTicket: every K-slice adds into a persistent zero-at-rest fp32 workspace and the slice
// that draws the tile's last ticket applies the real epilogue (bf16 store + BN sums, or act' mask +
// addend) and re-zeroes the tile — one launch, no memset node.  The workspaces are module-scope device
// arrays, one per role (forward, dgrad: both only ever run on the main stream, never concurrently).
constexpr long kConvWs = 4L << 20;  // fp32 elements per role (M x N of the GEMM)
constexpr int kConvTk = 16384;      // tile tickets per role
__device__ float g_conv_ws[2][kConvWs];
__device__ unsigned g_conv_tk[2][kConvTk];

static bool conv_split(int role, long M, long N, long K, float** ws, unsigned** tk) {
  if (hopsx_deterministic() || hopsx_disabled("conv_splitk")) return false;
  // only GEMMs with fewer tiles than CUs and a long K: at 392 tiles / K 1,024-2,304 (stage-3 convs at
  // batch 8) the split's workspace round trip cost more than it won (profiles/r5_conv_splitk_b8.txt)
  static const long min_k = hopsx_env_int("HOPSX_CONV_SPLIT_MINK", 2048);
  const GemmPlan p0 = plan_gemm(M, N, K, false);
  const int bm0 = p0.cfg == 0 ? 128 : (p0.cfg == 1 ? 64 : 32);
  if (((M + bm0 - 1) / bm0) * ((N + bm0 - 1) / bm0) >= 256 || K < min_k) return false;
  const GemmPlan p = plan_gemm(M, N, K, true);
  if (p.split < 2) return false;
  const int bm = p.cfg == 0 ? 128 : (p.cfg == 1 ? 64 : 32);
  const long tiles = ((M + bm - 1) / bm) * ((N + bm - 1) / bm);
  if (M * N > kConvWs || tiles > kConvTk) return false;
  static float* wsp = nullptr;
  static unsigned* tkp = nullptr;
  if (!wsp) {
    void *a = nullptr, *b = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_conv_ws)) != hipSuccess ||
        hipGetSymbolAddress(&b, HIP_SYMBOL(g_conv_tk)) != hipSuccess)
      return false;
    wsp = (float*)a;
    tkp = (unsigned*)b;
  }
  *ws = wsp + role * kConvWs;
  *tk = tkp + role * kConvTk;
  return true;
}

static bool direct_ok(const ConvGeom& g) {
  const int K = g.KH * g.KW * g.C;
  return K <= 64 && g.CO % 4 == 0 && g.CO <= 256 && K * g.CO <= 1024 && !hopsx_disabled("direct_conv");
}

// The gg engine (gemm_glds.h: LDS-DMA ring, 128x256 / 256x128 tiles) for the conv GEMMs it fills the
// chip with; false -> nothing launched, the caller keeps gemm_core.h's engine.  A 1x1 / stride-1 /
// unpadded conv reads X (forward) and dY (dgrad) as plain [pixels][channels] matrices.
static bool gg_1x1(const ConvGeom& g) {
  return g.KH == 1 && g.KW == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0;
}

// im2col convs with a narrow GEMM (N = output columns < HOPSX_GG_MIN_N, default 65) stay on gemm_core.h's
// engine: the ResNet-50 stage-1 3x3 64->64 conv measured 210 vs 248 us forward and 249 vs 294 us dgrad
// at B=256 there (profiles/r3s7_conv_gemm_vs_torch.txt); gg keeps every wider shape
static bool gg_narrow(const ConvGeom& g, int N) {
  static const int min_n = (int)hopsx_env_int("HOPSX_GG_MIN_N", 65);
  // (64 output columns: the 256x64 tile, gg_plan cfg 3)
  static const bool n64 = !hopsx_disabled("gg_n64");
  return !(g.KH == 1 && g.KW == 1) && N < min_n && !(N == 64 && n64);
}

// A spatial (KH*KW > 1) conv with 64 output channels, K >= 256 and >= 8 rounds of the gg engine's 256x64 tiles
// (the ResNet-50 7x7 stem at batch >= 16: 802,816 output pixels at batch 64): the tiled engine rather than
// the direct MFMA kernel, whose per-wave 16-pixel groups re-gather every A row from L2 (211 us per stem
// forward at batch 64, profiles/r6_resnet50_b64_kernels.txt)
static bool gg_big_spatial(const int* geom) {
  const long M = (long)geom[0] * geom[4] * geom[5];
  const int K = geom[7] * geom[8] * geom[3];
  return geom[7] * geom[8] > 1 && geom[6] == 64 && K >= 256 && M >= 8L * 256 * 256 && geom[3] % 8 == 0 &&
         !hopsx_disabled("gg_stem") && !hopsx_disabled("gg_n64") && !hopsx_deterministic();
}

template <class EP>
static bool gg_conv_fwd(const void* x, const void* w, const ConvGeom& g, const EP& e, hipStream_t st) {
  const int M = g.B * g.OH * g.OW, N = g.CO, K = g.KH * g.KW * g.C;
  if (g.C % 8 || g.CO % 8 || ((uintptr_t)x | (uintptr_t)w) % 16 || hopsx_disabled("gg_fwd") || gg_narrow(g, N))
    return false;
  const GgDense ws{(const bf16_raw*)w, (long)K, N, K};
  if (gg_1x1(g)) return launch_gg<true, true>(GgDense{(const bf16_raw*)x, (long)g.C, M, K}, ws, e, M, N, K, false, st);
  return launch_gg<true, true>(GgIm2col{(const bf16_raw*)x, g, M, K}, ws, e, M, N, K, false, st);
}

// The pixels of parity classes that no tap reaches (a 1x1 / stride-2 conv: all but the (0, 0)
// class) get dX = 0, or the added gradient: 16-B chunks, `live` = bitmask of the classes with taps.
__global__ __launch_bounds__(256) void dgrad_par_fill_k(bf16_raw* __restrict__ out, const bf16_raw* __restrict__ add,
                                                        long nch, int C8, int W, int H, int sh, int sw, unsigned live) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nch; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C8;
    const int iw = (int)(pix % W), ih = (int)((pix / W) % H);
    if ((live >> ((ih % sh) * sw + iw % sw)) & 1u) continue;
    *(bf16x8*)(out + i * 8) = add ? *(const bf16x8*)(add + i * 8) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// Strided dgrad as sh*sw dense parity-class GEMMs (gemm_glds.h GgDgradParA); classes without taps
// are filled (dgrad_par_fill_k).  All class plans are checked before anything is launched.
static bool gg_dgrad_par(const void* dy, const void* w, const ConvGeom& g, const EpiDActBF16& e, hipStream_t st) {
  if ((g.sh == 1 && g.sw == 1) || g.dh != 1 || g.dw != 1 || g.sh > 4 || g.sw > 4 || hopsx_disabled("dgrad_par"))
    return false;
  if ((uintptr_t)e.out % 16 || (uintptr_t)e.add % 16) return false;
  GgParGeom cls[16];
  int n = 0;
  unsigned live = 0;
  for (int py = 0; py < g.sh; ++py)
    for (int px = 0; px < g.sw; ++px) {
      GgParGeom c{};
      c.py = py;
      c.px = px;
      c.kh0 = (py + g.ph) % g.sh;
      c.kw0 = (px + g.pw) % g.sw;
      c.nkh = c.kh0 < g.KH ? (g.KH - c.kh0 + g.sh - 1) / g.sh : 0;
      c.nkw = c.kw0 < g.KW ? (g.KW - c.kw0 + g.sw - 1) / g.sw : 0;
      c.Hp = (g.H - py + g.sh - 1) / g.sh;
      c.Wp = (g.W - px + g.sw - 1) / g.sw;
      if (c.Hp <= 0 || c.Wp <= 0) return false;
      if (c.nkh <= 0 || c.nkw <= 0) continue;  // no tap reaches this class: filled below
      c.fWp.init(c.Wp);
      c.fHWp.init(c.Hp * c.Wp);
      c.fNKW.init(c.nkw);
      GgPlan p;
      if (!gg_plan((long)g.B * c.Hp * c.Wp, g.C, (long)c.nkh * c.nkw * g.CO, false, p, 1)) return false;
      live |= 1u << (py * g.sw + px);
      cls[n++] = c;
    }
  if (n == 0) return false;
  if (n < g.sh * g.sw) {
    const long nch = (long)g.B * g.H * g.W * (g.C / 8);
    long blocks = (nch + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(dgrad_par_fill_k, dim3((unsigned)blocks), dim3(256), 0, st, e.out, e.add, nch, g.C / 8, g.W,
                       g.H, g.sh, g.sw, live);
  }
  for (int i = 0; i < n; ++i) {
    const GgParGeom& c = cls[i];
    const int M = g.B * c.Hp * c.Wp, K = c.nkh * c.nkw * g.CO;
    const GgDgradParA as{(const bf16_raw*)dy, g, c, M, K};
    const GgWeightTPar bs{(const bf16_raw*)w, g, c, K, g.C};
    const EpiDgradParBF16 ep{e.out, e.y, e.act, e.colsum, e.add, g.C, g.H, g.W, c.Wp, c.Hp * c.Wp,
                             c.py, c.px, g.sh, g.sw, c.fWp, c.fHWp};
    if (!launch_gg<true, false>(as, bs, ep, M, g.C, K, false, st, 1)) return false;  // (plans checked above)
  }
  return true;
}

static bool gg_conv_dgrad(const void* dy, const void* w, const ConvGeom& g, const EpiDActBF16& e, hipStream_t st) {
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.CO;
  if (g.C % 8 || g.CO % 8 || ((uintptr_t)dy | (uintptr_t)w) % 16 || hopsx_disabled("gg_dgrad") || gg_narrow(g, N))
    return false;
  // stride > 1: the dense parity-class GEMMs instead of the zero-inserting gather (when the whole
  // shape would take gg; the class GEMMs are launched however few workgroups each gives)
  {
    GgPlan p;
    if (e.ldo == g.C && (!e.y || e.ldy == g.C) && gg_plan(M, N, K, false, p) && gg_dgrad_par(dy, w, g, e, st))
      return true;
  }
  const GgWeightT ws{(const bf16_raw*)w, g, K, N};
  if (g.KH == 1 && g.KW == 1 && g.ph == 0 && g.pw == 0 && (g.sh > 1 || g.sw > 1) && g.H == g.OH * g.sh &&
      g.W == g.OW * g.sw && !e.colsum && !hopsx_disabled("dgrad_scatter")) {
    const int Mo = g.B * g.OH * g.OW;
    EpiDgradScatterBF16 es{e.out, e.y, e.act, e.add, g.C, g.W, g.OW, g.OH * g.OW, g.sh, g.sw, {}, {}, nullptr};
    es.fOW.init(g.OW);
    es.fOHW.init(g.OH * g.OW);
    return launch_gg<true, false>(GgDense{(const bf16_raw*)dy, (long)g.CO, Mo, K}, ws, es, Mo, N, K, false, st);
  }
  if (gg_1x1(g))
    return launch_gg<true, false>(GgDense{(const bf16_raw*)dy, (long)g.CO, M, K}, ws, e, M, N, K, false, st);
  return launch_gg<true, false>(GgDgradA{(const bf16_raw*)dy, g, M, K}, ws, e, M, N, K, false, st);
}

extern "C" int hopsx_conv2d_fwd(const void* x, const void* w, const int* geom, int epi, void* out,
                                const float* bias, int act, float* colsum, float xscale, float xshift,
                                hipStream_t st) {
  ConvGeom g = make_geom(geom);
  const int M = g.B * g.OH * g.OW, N = g.CO, K = g.KH * g.KW * g.C;
  const bool direct = epi == EPI_STORE_BF16 && !colsum && direct_ok(g) && ((uintptr_t)out % 8 == 0);
  if (xscale != 0.f && !direct) return -3;  // uint8 inputs are only fused into the direct kernel
  if (direct) {
    long total = (long)M * (N / 4);
    long grid = (total + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(conv_direct_fwd_k, dim3(grid), dim3(256), (size_t)K * N * sizeof(float), st, x, xscale,
                       xshift, (const bf16_raw*)w, bias, (bf16_raw*)out, g, act);
    return (int)hipGetLastError();
  }
  if (epi == EPI_STORE_BF16 && !colsum && hopsx_conv_fwd_mfma_ok(geom) && !gg_big_spatial(geom) && ((uintptr_t)x % 16 == 0) &&
      ((uintptr_t)w % 16 == 0) && ((uintptr_t)out % 16 == 0))
    return hopsx_conv2d_fwd_mfma(x, w, geom, out, bias, act, st);
  Im2colLoader al{(const bf16_raw*)x, g, (g.C % 8 == 0) && ((uintptr_t)x % 16 == 0)};
  DenseLoader bl{(const bf16_raw*)w, K, is_vec_ok(w, K)};
  if (epi == EPI_STORE_BF16) {
    EpiStoreBF16 e{(bf16_raw*)out, N, bias, 1.f, act, colsum};
    if (gg_conv_fwd(x, w, g, e, st)) return (int)hipGetLastError();
    float* ws;
    unsigned* tk;
    if (conv_split(0, M, N, K, &ws, &tk)) {
      const SplitFinish f{tk, kEpiStoreBF16, out, N, bias, 1.f, 0.f, act, nullptr, 0, colsum, nullptr};
      launch_gemm<true, true>(al, bl, EpiAtomicTicket{ws, N, 1.f, nullptr, f}, M, N, K, true, st);
      return (int)hipGetLastError();
    }
    launch_gemm<true, true>(al, bl, e, M, N, K, false, st);
  } else if (epi == EPI_STORE_F32) {
    EpiStoreF32 e{(float*)out, N, bias, 1.f, 0.f, act, colsum};
    launch_gemm<true, true>(al, bl, e, M, N, K, false, st);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int hopsx_conv2d_fwd_bnstats(const void* x, const void* w, const int* geom, void* out, float* bnacc,
                                        hipStream_t st) {
  if (!bnacc || hopsx_disabled("bnstats") || !hopsx_bn_prestats_ok(geom[6])) return -2;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)out) % 16 != 0) return -2;
  if (hopsx_conv_fwd_mfma_ok(geom) && !gg_big_spatial(geom))
    return hopsx_conv2d_fwd_mfma_ex(x, w, geom, out, nullptr, 0, bnacc, st);
  ConvGeom g = make_geom(geom);
  if (g.C % 8 != 0) return -2;
  const int M = g.B * g.OH * g.OW, N = g.CO, K = g.KH * g.KW * g.C;
  Im2colLoader al{(const bf16_raw*)x, g, 1};
  DenseLoader bl{(const bf16_raw*)w, K, is_vec_ok(w, K)};
  EpiBnStatsBF16 e{(bf16_raw*)out, N, bnacc};
  if (gg_conv_fwd(x, w, g, e, st)) return (int)hipGetLastError();
  float* ws;
  unsigned* tk;
  if (conv_split(0, M, N, K, &ws, &tk)) {
    const SplitFinish f{tk, kEpiBnStatsBF16, out, N, nullptr, 1.f, 0.f, 0, nullptr, 0, bnacc, nullptr};
    launch_gemm<true, true>(al, bl, EpiAtomicTicket{ws, N, 1.f, nullptr, f}, M, N, K, true, st);
    return (int)hipGetLastError();
  }
  launch_gemm<true, true>(al, bl, e, M, N, K, false, st);
  return (int)hipGetLastError();
}

extern "C" int hopsx_conv2d_fwd_bnstats_inbn(const void* z, void* a, const void* w, const int* geom, void* out,
                                             float* bnacc, float* inacc, const float* gamma, const float* beta,
                                             float* mean_out, float* rstd_out, float* rmean, float* rvar,
                                             float momentum, float eps, int act, hipStream_t st) {
  if (!bnacc || hopsx_disabled("bnstats") || !hopsx_bn_prestats_ok(geom[6]) || !hopsx_bn_prestats_ok(geom[3]) ||
      gg_big_spatial(geom))
    return -2;
  return hopsx_conv2d_fwd_mfma_inbn(z, a, w, geom, out, bnacc, inacc, gamma, beta, mean_out, rstd_out, rmean, rvar,
                                    momentum, eps, act, st);
}

// dX = conv_transpose(dY, W).  If `yprev` is given, the result is multiplied by
// act'(yprev) — the backward of the activation that produced this conv's input
// — and `colsum` receives that layer's bias gradient.
extern "C" int hopsx_conv2d_dgrad(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                  int act, float* colsum, const void* y, int yact, const void* addend,
                                  hipStream_t st) {
  if (!addend && hopsx_conv_dgrad_mfma_ok(geom) && ((uintptr_t)dy % 16 == 0) && ((uintptr_t)y % 16 == 0) &&
      ((uintptr_t)dx % 16 == 0) && ((uintptr_t)yprev % 16 == 0))
    return hopsx_conv2d_dgrad_mfma(dy, w, geom, dx, yprev, act, colsum, y, yact, st);
  ConvGeom g = make_geom(geom);
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.CO;
  ConvDgradALoader al{(const bf16_raw*)dy, g,
                      (g.CO % 8 == 0) && ((uintptr_t)dy % 16 == 0) && ((uintptr_t)y % 16 == 0),
                      (const bf16_raw*)y, yact};
  ConvWeightTLoader bl{(const bf16_raw*)w, g, (g.C % 8 == 0) && ((uintptr_t)w % 16 == 0)};
  EpiDActBF16 e{(bf16_raw*)dx, N, (const bf16_raw*)yprev, N, act, colsum, (const bf16_raw*)addend};
  if (!y && gg_conv_dgrad(dy, w, g, e, st)) return (int)hipGetLastError();
  float* ws;
  unsigned* tk;
  if (conv_split(1, M, N, K, &ws, &tk)) {
    const SplitFinish f{tk, kEpiDActBF16, dx, N, nullptr, 1.f, 0.f, act, (const bf16_raw*)yprev, N, colsum,
                        (const bf16_raw*)addend};
    launch_gemm<true, false>(al, bl, EpiAtomicTicket{ws, N, 1.f, nullptr, f}, M, N, K, true, st);
    return (int)hipGetLastError();
  }
  launch_gemm<true, false>(al, bl, e, M, N, K, false, st);
  return (int)hipGetLastError();
}

// dX of a conv whose input x is a training BatchNorm's output consumed only by this conv: the epilogue
// adds `addend` (a shortcut's gradient of x), masks by act_prev'(yprev = x), stores g and reduces the
// BN's backward column sums (sum g, sum g * xhat) into the replica rows bnacc[HOPSX_BN_NREP][2C]
// (gemm_core.h EpiDgradBnBF16; conv_mfma.hip DgradArgs bnacc for the direct MFMA shapes).  Stride-1
// convs on the direct MFMA kernel, the gg engine (1x1 and implicit-GEMM gathers) or gemm_core.h's
// engine without split-K; anything else (strided parity GEMMs, split-K) returns -2 with nothing
// launched and the caller runs the plain dgrad + the full BN backward.
extern "C" int hopsx_conv2d_dgrad_bn(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                     int act_prev, const void* addend, const void* bnz, const float* bnmean,
                                     const float* bnrstd, float* bnacc, hipStream_t st) {
  ConvGeom g = make_geom(geom);
  if (!bnacc || !bnz || !bnmean || !bnrstd || hopsx_disabled("bn_dgrad_sums") || g.sh != 1 || g.sw != 1 ||
      g.C % 8 || g.CO % 8 || !hopsx_bn_prestats_ok(g.C) ||
      ((uintptr_t)dy | (uintptr_t)w | (uintptr_t)dx | (uintptr_t)yprev | (uintptr_t)addend | (uintptr_t)bnz) % 16)
    return -2;
  const int r = hopsx_conv2d_dgrad_mfma_bn(dy, w, geom, dx, yprev, act_prev, addend, bnz, bnmean, bnrstd, bnacc, st);
  if (r != -2) return r;
  const int M = g.B * g.H * g.W, N = g.C, K = g.KH * g.KW * g.CO;
  const EpiDgradBnBF16 e{(bf16_raw*)dx, N, (const bf16_raw*)yprev, act_prev, (const bf16_raw*)addend,
                         (const bf16_raw*)bnz, bnmean, bnrstd, bnacc};
  if (!hopsx_disabled("gg_dgrad") && !gg_narrow(g, N)) {
    const GgWeightT ws{(const bf16_raw*)w, g, K, N};
    if (gg_1x1(g) ? launch_gg<true, false>(GgDense{(const bf16_raw*)dy, (long)g.CO, M, K}, ws, e, M, N, K, false, st)
                  : launch_gg<true, false>(GgDgradA{(const bf16_raw*)dy, g, M, K}, ws, e, M, N, K, false, st))
      return (int)hipGetLastError();
  }
  float* sws;
  unsigned* stk;
  if (conv_split(1, M, N, K, &sws, &stk)) return -2;  // the plain dgrad would split K: keep it
  ConvDgradALoader al{(const bf16_raw*)dy, g, 1, nullptr, 0};
  ConvWeightTLoader bl{(const bf16_raw*)w, g, 1};
  launch_gemm<true, false>(al, bl, e, M, N, K, false, st);
  return (int)hipGetLastError();
}

// dW[co][k] += sum_m dY[m][co] * im2col(X)[m][k]; db[co] += sum_m dY[m][co] when colsum given
static bool smallk_ok(const ConvGeom& g, const void* dy, const void* y, const float* ws, long ws_elems,
                      const unsigned* counter) {
  const int K = g.KH * g.KW * g.C;
  // input layers only (C < 8: the MNIST uint8 inputs): a 1x1 conv with K = C = 16 is a plain
  // short reduction that the MFMA wgrad does faster (CIFAR ResNet-20 77.4k -> 82.0k img/s)
  return (K == 4 || K == 9 || K == 16) && g.C < 8 && g.CO % 8 == 0 && g.CO <= 256 && ((uintptr_t)dy % 16 == 0) &&
         ((uintptr_t)y % 16 == 0) && counter && ws && ws_elems >= 128L * g.CO * (K + 1) &&
         !hopsx_disabled("smallk_wgrad");
}

extern "C" int hopsx_conv2d_wgrad(const void* dy, const void* x, const int* geom, float* dw, float* dbias,
                                  const void* y, int yact, float* ws, long ws_elems, float xscale, float xshift,
                                  unsigned* counter, hipStream_t st) {
  ConvGeom g = make_geom(geom);
  const int M = g.CO, N = g.KH * g.KW * g.C, K = g.B * g.OH * g.OW;
  // one-channel input layers: the pixel-range kernel (conv_wgrad_c1_k)
  if (g.C == 1 && N <= 25 && (g.CO == 8 || g.CO == 16 || g.CO == 32 || g.CO == 64) && (uintptr_t)dy % 16 == 0 &&
      (uintptr_t)y % 16 == 0 && counter && ws && !hopsx_disabled("c1_wgrad")) {
    const int NE = g.CO * (N + 1), NEP = (NE + 31) & ~31;  // rows padded to 128-B lines
    // <= 224 workgroups + their <= 14 group rows fit the caller's 256-row slab (kernels.conv2d_wgrad)
    int nwg = (K + 63) / 64;
    if (nwg > 224) nwg = 224;
    if (nwg < 1) nwg = 1;
    const int ppw = (K + nwg - 1) / nwg;
    const int ngrp = (nwg + C1_GROUP - 1) / C1_GROUP;
    size_t lds = (size_t)ppw * (g.CO + N) * sizeof(float);
    const size_t lds_red = (size_t)256 * (N + 1) * sizeof(float);  // the pixel-lane reduction [PL][CO][K+1]
    if (lds < lds_red) lds = lds_red;
    // (the staging loops' per-thread item counts are compile-time: 8 dY vectors, 20 taps)
    if (ws_elems >= (long)(nwg + ngrp) * NEP && lds <= 64 * 1024 && (long)ppw * (g.CO / 8) <= 8 * 256 &&
        (long)ppw * N <= 20 * 256) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)conv_wgrad_c1_k, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        attr = true;
      }
      static const int stop = (int)hopsx_env_int("HOPSX_C1_STOP", 0);
      hipLaunchKernelGGL(conv_wgrad_c1_k, dim3(nwg), dim3(256), lds, st, (const bf16_raw*)dy, x, xscale, xshift, dw,
                         dbias, (const bf16_raw*)y, yact, g, K, ppw, ws, counter, stop);
      return (int)hipGetLastError();
    }
  }
  if (smallk_ok(g, dy, y, ws, ws_elems, counter)) {
    const long total = (long)K * (g.CO / 8);
    // ~16 work items per thread: the in-launch combine then reads only blocks x CO x (K+1)
    // floats (one row per workgroup; ~23 rows at the MNIST batch of 32).  At 16 taps (the E1 / HPO
    // models' 4x4 input convs) a thread holds 8 x 17 accumulators (one wave per SIMD): 2 items per thread
    // instead, ~6x the workgroups (E1 keras fit 131 k -> 158 k img/s: profiles/r5_e1_fit_kernels.txt)
    static const long items_env = hopsx_env_int("HOPSX_SMALLK_ITEMS", 0);
    const long items = items_env > 0 ? items_env : (N >= 16 ? 2 : 16);
    long blocks = (total + 256 * items - 1) / (256 * items);
    if (blocks > 128) blocks = 128;
    if (blocks < 1) blocks = 1;
#define HOPSX_SMALLK(KK)                                                                                      \
  hipLaunchKernelGGL(conv_wgrad_smallk_k<KK>, dim3(blocks), dim3(256), 0, st, (const bf16_raw*)dy, x, xscale, xshift, dw, \
                     dbias, (const bf16_raw*)y, yact, g, total, ws, counter)
    if (N == 4) HOPSX_SMALLK(4);
    else if (N == 9) HOPSX_SMALLK(9);
    else HOPSX_SMALLK(16);
#undef HOPSX_SMALLK
    return (int)hipGetLastError();
  }
  if (xscale != 0.f) return -3;
  // LDS-DMA 128x128 kernel (wgrad_glds.hip) for the conv -> BN layers (no dY mask, no bias grad);
  // the small-CO direct-MFMA kernel keeps its shapes unless HOPSX_WGRAD_GLDS_FIRST=1 (A/B knob)
  static const int glds_first = hopsx_env_int("HOPSX_WGRAD_GLDS_FIRST", 0);
  // ... up to a size: past ~32M pixel-columns (ResNet-50 at B=64: the stage-1 3x3, the 8-channel stem)
  // the LDS-DMA engine wins even at CO = 64 (profiles/r4_stem_wgrad_ab.txt: +1.7 % per step); the CIFAR
  // ResNets' convs (<= 19M) keep the short-conv kernel
  static const long mfma_max_mk = hopsx_env_int("HOPSX_WGRAD_MFMA_MAX_MK", 32L << 20);
  const bool mfma_ok = hopsx_conv_wgrad_mfma_ok(geom) && (long)K * N < mfma_max_mk && (uintptr_t)dy % 16 == 0 &&
                       (uintptr_t)y % 16 == 0 && (uintptr_t)x % 16 == 0;
  if (!y && !dbias && (glds_first || !mfma_ok) && hopsx_conv_wgrad_glds_ok(geom) &&
      hopsx_conv2d_wgrad_glds(dy, x, geom, dw, 0, st) == 0)
    return 0;
  if (mfma_ok) return hopsx_conv2d_wgrad_mfma(dy, x, geom, dw, dbias, y, yact, st);
  // the direct kernel re-loads dY and X per (k, co) thread: cheap for small pixel counts and the
  // only path for uint8 inputs; past 16k pixels the implicit-GEMM MFMA path wins (the CIFAR
  // ResNet stem, 131k pixels: 89 us direct)
  if (direct_ok(g) && (xscale != 0.f || K <= 16384) && !hopsx_disabled("direct_wgrad")) {
    const int KC = N * M;
    int R = 1024 / KC;
    if (R > 8) R = 8;
    if (R < 1) R = 1;
    const int threads = ((KC * R + 63) / 64) * 64;
    // with a slab workspace: up to 1024 workgroups of >= 128 pixels, partials reduced by
    // a second pass; without one: <= 128 workgroups so same-address atomics stay cheap
    const bool use_slab = ws && ws_elems >= 1024L * (KC + M);
    const long cap = use_slab ? 1024 : 128;
    long blocks = (K + 127) / 128;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const int ppb = (int)((K + blocks - 1) / blocks);
    blocks = (K + ppb - 1) / ppb;
    const size_t shm = (size_t)R * (KC + M) * sizeof(float);
    hipLaunchKernelGGL(conv_direct_wgrad_k, dim3(blocks), dim3(threads), shm, st, (const bf16_raw*)dy,
                       (const bf16_raw*)x, dw, dbias, (const bf16_raw*)y, yact, g, ppb, R, use_slab ? ws : nullptr);
    if (use_slab)
      hipLaunchKernelGGL(slab_reduce_k, dim3(KC + M), dim3(256), 0, st, ws, (int)blocks, KC, M, N, dw,
                         dbias);
    return (int)hipGetLastError();
  }
  DenseLoader al{(const bf16_raw*)dy, g.CO, is_vec_ok(dy, g.CO) && is_vec_ok(y ? y : dy, g.CO), (const bf16_raw*)y,
                 yact};
  Im2colLoader bl{(const bf16_raw*)x, g, (g.C % 8 == 0) && ((uintptr_t)x % 16 == 0)};
  EpiAtomicF32 e{dw, N, 1.f, nullptr};
  // A = dY^T is staged as an RC image: its row sums are the conv bias gradient
  launch_gemm<false, false>(al, bl, e, M, N, K, true, st, dbias);
  return (int)hipGetLastError();
}
