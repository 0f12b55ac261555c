// BatchNorm over NHWC activations viewed as [M = B*H*W, C] (channel-fastest),
// with the residual add and the activation fused into the apply pass
// (ResNet: y = act(bn(x) + residual)) and into the backward.
#include <algorithm>
#include <initializer_list>

#include "common.h"
#include "ops_api.h"

HOPSX_DET_TU(norm)

// column sums of x and x^2 (stats) -- one workgroup per (64-column strip, row slab)
__global__ __launch_bounds__(256) void bn_stats_k(const bf16_raw* __restrict__ x, float* __restrict__ s1,
                                                  float* __restrict__ s2, int M, int C, int rpb) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  float a = 0.f, b = 0.f;
  if (c < C)
    for (int m = r0 + (threadIdx.x >> 6); m < r1; m += 4) {
      const float v = bf2f(x[(long)m * C + c]);
      a += v;
      b += v * v;
    }
  __shared__ float ra[4][64], rb[4][64];
  ra[threadIdx.x >> 6][threadIdx.x & 63] = a;
  rb[threadIdx.x >> 6][threadIdx.x & 63] = b;
  __syncthreads();
  const bool det = det_on();
  const unsigned dmy = blockIdx.y * gridDim.x + blockIdx.x;
  if (det) det_turn_begin(DET_BN_STATS, dmy);
  if (threadIdx.x < 64 && c < C) {
    const int t = threadIdx.x;
    atomicAdd(s1 + c, ra[0][t] + ra[1][t] + ra[2][t] + ra[3][t]);
    atomicAdd(s2 + c, rb[0][t] + rb[1][t] + rb[2][t] + rb[3][t]);
  }
  if (det) det_turn_end(DET_BN_STATS, dmy, gridDim.x * gridDim.y);
}

// turn (sum, sumsq) into (mean, rstd) in place; update running stats (unbiased var)
__global__ void bn_finalize_k(float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ rmean,
                              float* __restrict__ rvar, float momentum, float eps, int M, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mu = mean[c] / M;
  const float var = fmaxf(rstd[c] / M - mu * mu, 0.f);
  mean[c] = mu;
  rstd[c] = rsqrtf(var + eps);
  if (rmean) {
    const float unb = M > 1 ? var * M / (M - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  }
}

__global__ __launch_bounds__(256) void bn_apply_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  const float* __restrict__ mean, const float* __restrict__ rstd,
                                                  int var_mode, float eps, long n, int C,
                                                  const bf16_raw* __restrict__ res, int act) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = i % C;
    const float rs = var_mode ? rsqrtf(rstd[c] + eps) : rstd[c];
    float v = (bf2f(x[i]) - mean[c]) * rs * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
    if (res) v += bf2f(res[i]);
    y[i] = f2bf(apply_act(v, act));
  }
}

// backward reduce: ws[0:C] = sum(dz), ws[C:2C] = sum(dz * xhat), dz = dy * act'(y)
__global__ __launch_bounds__(256) void bn_bwd_reduce_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ x,
                                                       const bf16_raw* __restrict__ y, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, float* __restrict__ ws, int M,
                                                       int C, int rpb, int act) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  float a = 0.f, b = 0.f;
  if (c < C) {
    const float mu = mean[c], rs = rstd[c];
    for (int m = r0 + (threadIdx.x >> 6); m < r1; m += 4) {
      const long i = (long)m * C + c;
      float dz = bf2f(dy[i]);
      if (act != ACT_NONE) dz *= act_grad_from_out(bf2f(y[i]), act);
      a += dz;
      b += dz * (bf2f(x[i]) - mu) * rs;
    }
  }
  __shared__ float ra[4][64], rb[4][64];
  ra[threadIdx.x >> 6][threadIdx.x & 63] = a;
  rb[threadIdx.x >> 6][threadIdx.x & 63] = b;
  __syncthreads();
  const bool det = det_on();
  const unsigned dmy = blockIdx.y * gridDim.x + blockIdx.x;
  if (det) det_turn_begin(DET_BN_BWD, dmy);
  if (threadIdx.x < 64 && c < C) {
    const int t = threadIdx.x;
    atomicAdd(ws + c, ra[0][t] + ra[1][t] + ra[2][t] + ra[3][t]);
    atomicAdd(ws + C + c, rb[0][t] + rb[1][t] + rb[2][t] + rb[3][t]);
  }
  if (det) det_turn_end(DET_BN_BWD, dmy, gridDim.x * gridDim.y);
}

__global__ __launch_bounds__(256) void bn_bwd_apply_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ x,
                                                      const bf16_raw* __restrict__ y, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ ws, bf16_raw* __restrict__ dx,
                                                      bf16_raw* __restrict__ dres, long n, int M, int C, int act) {
  const float invM = 1.f / M;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = i % C;
    float dz = bf2f(dy[i]);
    if (act != ACT_NONE) dz *= act_grad_from_out(bf2f(y[i]), act);
    if (dres) dres[i] = f2bf(dz);
    const float xh = (bf2f(x[i]) - mean[c]) * rstd[c];
    const float g = gamma ? gamma[c] : 1.f;
    dx[i] = f2bf(g * rstd[c] * (dz - ws[c] * invM - xh * ws[C + c] * invM));
  }
}

__global__ void bn_grad_acc_k(const float* __restrict__ ws, float* __restrict__ dgamma, float* __restrict__ dbeta,
                              int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dbeta) dbeta[c] += ws[c];
  if (dgamma) dgamma[c] += ws[C + c];
}

// ---------------------------------------------------------------------------------------------
// Vectorized path (C % 8 == 0, C/8 a power of two <= 256, 16-B aligned tensors): every lane moves
// 8 channels (16 B) per access, a workgroup covers all C columns and 256/(C/8) rows per pass with
// UNR rows' loads in flight, and per-channel partials go to one of NREP replica rows of a
// zero-at-rest accumulator (NREP-fold less same-address atomic contention); the finalize
// kernels fold the replicas, re-zero them and (fwd) update the running statistics, so no
// memset launches remain.  The scalar kernels above serve odd channel counts.
constexpr int BN_NREP = HOPSX_BN_NREP;
constexpr int BN_UNR = 4;

// The forward's per-channel shift, one explicit fma: the backward recomputes it bit-identically, so a
// ReLU BN without residual takes its act' mask from z (t = z * sc + sh > 0, exactly the forward's test)
// instead of reading y back (zmask: one tensor less in both backward passes).
__device__ __forceinline__ float bn_shift(float beta, float mu, float sc) { return fmaf(-mu, sc, beta); }

__device__ __forceinline__ void ld8f(const bf16_raw* p, float* v) {
  const bf16x8 q = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f((uint16_t)q[j]);
}
__device__ __forceinline__ void st8f(bf16_raw* p, const float* v) {
  bf16x8 q;
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = (short)f2bf(v[j]);
  *(bf16x8*)p = q;
}

// MODE 0 (stats): acc[rep][0:C] += x, acc[rep][C:2C] += x^2
// MODE 1 (bwd):   acc[rep][0:C] += dz, acc[rep][C:2C] += dz * xhat, dz = dy * act'(y)
// The launch also FINISHES the statistics (no separate finalize launch): the last workgroup to
// arrive (per-XCD sharded counter after the BN_NREP x 2C replicas, common.h grid_arrive_last)
// folds the replicas with atomic exchanges (read + re-zero at the memory side, where the float
// atomics landed) and writes mean / rstd + running statistics (MODE 0) or the two bwd sums + the
// dgamma / dbeta accumulation (MODE 1).
struct BnFin {
  float* mean_out;  // MODE 0
  float* rstd_out;
  float* rmean;
  float* rvar;
  float momentum, eps;
  float* ws;  // MODE 1: [sum dz | sum dz*xhat]
  float* dgamma;
  float* dbeta;
  int defer;  // 1: leave the replicas for the consuming apply kernel (bn_apply_fin8_k / bn_bwd_apply_fin8_k)
};

// Fold a workgroup's per-lane column partials (8 channels c0..c0+7 of channel group threadIdx % CG,
// sums s1 / s2) and add them to this workgroup's replica row dst[0:2C] (red: >= 256*16 floats LDS).
__device__ __forceinline__ void bn_block_colsum_body(float* s1, float* s2, float* red, float* dst, int C, int CG,
                                                     int RPI);
// deterministic mode: the workgroups add their partials in workgroup order (common.h det_turn_*)
__device__ __forceinline__ void bn_block_colsum(float* s1, float* s2, float* red, float* dst, int C, int CG,
                                                int RPI) {
  const bool det = det_on();
  if (det) det_turn_begin(DET_BN_STATS, blockIdx.x);
  bn_block_colsum_body(s1, s2, red, dst, C, CG, RPI);
  if (det) det_turn_end(DET_BN_STATS, blockIdx.x, gridDim.x);
}
__device__ __forceinline__ void bn_block_colsum_body(float* s1, float* s2, float* red, float* dst, int C, int CG,
                                                     int RPI) {
  if (CG < 64) {
    // lanes of a wave with the same channel group (lane % CG) fold with xor shuffles, log2(64/CG)
    // steps; then 4 wave partials per channel meet in LDS.  (A serial walk over the RPI row
    // partials by 2C threads cost RPI dependent LDS round trips: 128 of them at C = 16.)
    for (int o = CG; o < 64; o <<= 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += __shfl_xor(s1[j], o, 64);
        s2[j] += __shfl_xor(s2[j], o, 64);
      }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane < CG) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wave * CG + lane) * 16 + j] = s1[j];
        red[(wave * CG + lane) * 16 + 8 + j] = s2[j];
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * C; e += 256) {  // e < C: sum1 of channel e, else sum2 of channel e - C
      const int which = e >= C, c = e - which * C;
      const int g = c >> 3, j = c & 7;
      const float t = red[g * 16 + which * 8 + j] + red[(CG + g) * 16 + which * 8 + j] +
                      red[(2 * CG + g) * 16 + which * 8 + j] + red[(3 * CG + g) * 16 + which * 8 + j];
      if (t != 0.f) atomicAdd(dst + e, t);
    }
  } else {  // RPI <= 4 row partials per channel
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[threadIdx.x * 16 + j] = s1[j];
      red[threadIdx.x * 16 + 8 + j] = s2[j];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * C; e += 256) {
      const int which = e >= C, c = e - which * C;
      const int g = c >> 3, j = c & 7;
      float t = 0.f;
      for (int q = 0; q < RPI; ++q) t += red[(q * CG + g) * 16 + which * 8 + j];
      if (t != 0.f) atomicAdd(dst + e, t);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void bn_colred8_k(const bf16_raw* __restrict__ a, const bf16_raw* __restrict__ x,
                                                    const bf16_raw* __restrict__ y, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, float* __restrict__ acc, int M,
                                                    int C, int rpb, int act, BnFin fin,
                                                    const float* __restrict__ gamma = nullptr,
                                                    const float* __restrict__ zbeta = nullptr) {
  const int CG = C >> 3, RPI = 256 / CG;
  const int cg = threadIdx.x % CG, rsub = threadIdx.x / CG;
  const int c0 = cg * 8;
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float s1[8], s2[8], mu[8], rs[8], zs[8], zh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; mu[j] = 0.f; rs[j] = 0.f; zs[j] = 0.f; zh[j] = 0.f; }
  const bool zmask = MODE == 1 && zbeta != nullptr && act == ACT_RELU;  // act' from z (bn_shift)
  if (MODE == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
    if (zmask)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        zs[j] = rs[j] * (gamma ? gamma[c0 + j] : 1.f);
        zh[j] = bn_shift(zbeta[c0 + j], mu[j], zs[j]);
      }
  }
  for (int r = r0 + rsub; r < r1; r += BN_UNR * RPI) {
    float va[BN_UNR][8], vx[BN_UNR][8], vy[BN_UNR][8];
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {  // all loads of the trip first
      const int rr = r + u * RPI;
      const long o = (long)(rr < r1 ? rr : r0) * C + c0;
      ld8f(a + o, va[u]);
      if (MODE == 1) {
        ld8f(x + o, vx[u]);
        if (act != ACT_NONE && !zmask) ld8f(y + o, vy[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      if (r + u * RPI >= r1) break;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MODE == 0) {
          s1[j] += va[u][j];
          s2[j] = fmaf(va[u][j], va[u][j], s2[j]);
        } else {
          float dz = va[u][j];
          if (zmask) dz = fmaf(vx[u][j], zs[j], zh[j]) > 0.f ? dz : 0.f;
          else if (act != ACT_NONE) dz *= act_grad_from_out(vy[u][j], act);
          s1[j] += dz;
          s2[j] = fmaf(dz, (vx[u][j] - mu[j]) * rs[j], s2[j]);
        }
      }
    }
  }
  __shared__ float red[256 * 16];
  float* dst = acc + (long)(blockIdx.x % BN_NREP) * 2 * C;
  bn_block_colsum(s1, s2, red, dst, C, CG, RPI);
  if (fin.defer) return;  // the apply launch folds the replicas: no arrival / exchange round trips here
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's atomics are done
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last = grid_arrive_last((unsigned*)(acc + (long)BN_NREP * 2 * C)) ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int r = 0; r < BN_NREP; ++r) {
      s += atomicExch(acc + (long)r * 2 * C + c, 0.f);
      q += atomicExch(acc + (long)r * 2 * C + C + c, 0.f);
    }
    if (MODE == 0) {
      const float mu = s / M;
      const float var = fmaxf(q / M - mu * mu, 0.f);
      fin.mean_out[c] = mu;
      fin.rstd_out[c] = rsqrtf(var + fin.eps);
      if (fin.rmean) {
        const float unb = M > 1 ? var * M / (M - 1) : var;
        fin.rmean[c] = (1.f - fin.momentum) * fin.rmean[c] + fin.momentum * mu;
        fin.rvar[c] = (1.f - fin.momentum) * fin.rvar[c] + fin.momentum * unb;
      }
    } else {
      fin.ws[c] = s;
      fin.ws[C + c] = q;
      if (fin.dbeta) fin.dbeta[c] += s;
      if (fin.dgamma) fin.dgamma[c] += q;
    }
  }
}

// y = act((x - mean) * rstd * gamma + beta + res)  (var_mode: rstd holds a variance -> inference)
__global__ __launch_bounds__(256) void bn_apply8_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd,
                                                   int var_mode, float eps, long nch, int C,
                                                   const bf16_raw* __restrict__ res, int act) {
  const int CG = C >> 3;
  const long stride = (long)gridDim.x * blockDim.x;  // a multiple of CG: the channel group is per-thread
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(i0 % CG) * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float rs = var_mode ? rsqrtf(rstd[c0 + j] + eps) : rstd[c0 + j];
    sc[j] = rs * (gamma ? gamma[c0 + j] : 1.f);
    sh[j] = bn_shift(beta ? beta[c0 + j] : 0.f, mean[c0 + j], sc[j]);
  }
  for (long i = i0; i < nch; i += 2 * stride) {
    float v[2][8], rv[2][8];
    const long i1 = i + stride < nch ? i + stride : i;
    ld8f(x + i * 8, v[0]);
    ld8f(x + i1 * 8, v[1]);
    if (res) {
      ld8f(res + i * 8, rv[0]);
      ld8f(res + i1 * 8, rv[1]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = fmaf(v[u][j], sc[j], sh[j]);
        if (res) t += rv[u][j];
        v[u][j] = apply_act(t, act);
      }
    }
    st8f(y + i * 8, v[0]);
    if (i + stride < nch) st8f(y + i1 * 8, v[1]);
  }
}

// Forward apply whose statistics the PRODUCING conv accumulated in its epilogue (conv_mfma.hip /
// conv.hip `bnacc`: per-channel sum / sum of squares of the bf16 outputs into the zero-at-rest
// replicas acc[BN_NREP][2C]).  Every workgroup folds the replicas into per-channel scale / shift
// in LDS — no statistics pass over x and no finalize round trips on the critical path — workgroup
// 0 publishes mean / rstd (for the backward) and the running statistics, and the last workgroup
// to have read the replicas re-zeroes them (after its own elementwise work).
__global__ __launch_bounds__(256) void bn_apply_fin8_k(const bf16_raw* __restrict__ x, bf16_raw* __restrict__ y,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float* __restrict__ acc, long nch, int M, int C,
                                                       const bf16_raw* __restrict__ res, int act, BnFin fin) {
  __shared__ float ssc[2048], ssh[2048];  // C <= 2048 (bn_vec_ok)
  __shared__ int last;
  const long stride = (long)gridDim.x * blockDim.x;  // a multiple of CG: the channel group is per-thread
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // the first trip's operands are requested BEFORE the replica fold, so their latency overlaps the
  // replica loads' (kept raw: a conversion here would wait for them right away).  apply_grid gives
  // most launches exactly one trip.
  const bool have0 = i0 < nch;
  const long i1 = i0 + stride < nch ? i0 + stride : i0;
  bf16x8 px[2], pr[2];
  if (have0) {
    px[0] = *(const bf16x8*)(x + i0 * 8);
    px[1] = *(const bf16x8*)(x + i1 * 8);
    if (res) {
      pr[0] = *(const bf16x8*)(res + i0 * 8);
      pr[1] = *(const bf16x8*)(res + i1 * 8);
    }
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int r = 0; r < BN_NREP; ++r) {
      s += acc[(long)r * 2 * C + c];
      q += acc[(long)r * 2 * C + C + c];
    }
    const float mu = s / M;
    const float var = fmaxf(q / M - mu * mu, 0.f);
    const float rs = rsqrtf(var + fin.eps);
    const float sc = rs * (gamma ? gamma[c] : 1.f);
    ssc[c] = sc;
    ssh[c] = bn_shift(beta ? beta[c] : 0.f, mu, sc);
    if (blockIdx.x == 0) {
      fin.mean_out[c] = mu;
      fin.rstd_out[c] = rs;
      if (fin.rmean) {
        const float unb = M > 1 ? var * M / (M - 1) : var;
        fin.rmean[c] = (1.f - fin.momentum) * fin.rmean[c] + fin.momentum * mu;
        fin.rvar[c] = (1.f - fin.momentum) * fin.rvar[c] + fin.momentum * unb;
      }
    }
  }
  __syncthreads();  // every replica value this workgroup needs has been consumed
  if (threadIdx.x == 0) last = grid_arrive_last((unsigned*)(acc + (long)BN_NREP * 2 * C)) ? 1 : 0;
  const int CG = C >> 3;
  const int c0 = (int)(i0 % CG) * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = ssc[c0 + j];
    sh[j] = ssh[c0 + j];
  }
  for (long i = i0; i < nch; i += 2 * stride) {
    const long ib = i + stride < nch ? i + stride : i;
    // the next trip's operands are requested before this trip's math and stores (twice the bytes in
    // flight: the big ResNet-50 tensors take ~12 trips per thread, each of which waited out a round trip)
    const long in0 = i + 2 * stride, in1 = in0 + stride < nch ? in0 + stride : in0;
    bf16x8 nx[2], nr[2];
    if (in0 < nch) {
      nx[0] = *(const bf16x8*)(x + in0 * 8);
      nx[1] = *(const bf16x8*)(x + in1 * 8);
      if (res) {
        nr[0] = *(const bf16x8*)(res + in0 * 8);
        nr[1] = *(const bf16x8*)(res + in1 * 8);
      }
    }
    float v[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = fmaf(bf2f((uint16_t)px[u][j]), sc[j], sh[j]);
        if (res) t += bf2f((uint16_t)pr[u][j]);
        v[u][j] = apply_act(t, act);
      }
    }
    st8f(y + i * 8, v[0]);
    if (i + stride < nch) st8f(y + ib * 8, v[1]);
    px[0] = nx[0];
    px[1] = nx[1];
    if (res) {
      pr[0] = nr[0];
      pr[1] = nr[1];
    }
  }
  __syncthreads();
  if (last)
    for (int e = threadIdx.x; e < BN_NREP * 2 * C; e += 256) acc[e] = 0.f;
}

__global__ __launch_bounds__(256) void bn_bwd_apply8_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ x,
                                                       const bf16_raw* __restrict__ y, const float* __restrict__ gamma,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ ws, bf16_raw* __restrict__ dx,
                                                       bf16_raw* __restrict__ dres, long nch, int M, int C, int act) {
  const int CG = C >> 3;
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(i0 % CG) * 8;
  const float invM = 1.f / M;
  float k1[8], k2[8], mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float g = gamma ? gamma[c0 + j] : 1.f;
    rs[j] = rstd[c0 + j];
    mu[j] = mean[c0 + j];
    k1[j] = g * rs[j];                 // dx = k1 * (dz - mean(dz) - xhat * mean(dz*xhat))
    k2[j] = ws[C + c0 + j] * invM;
    mu[j] = mean[c0 + j];
  }
  float md[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) md[j] = ws[c0 + j] * invM;
  for (long i = i0; i < nch; i += stride) {
    float d[8], xv[8], yv[8];
    ld8f(dy + i * 8, d);
    ld8f(x + i * 8, xv);
    if (act != ACT_NONE) {
      ld8f(y + i * 8, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] *= act_grad_from_out(yv[j], act);
    }
    if (dres) st8f(dres + i * 8, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (xv[j] - mu[j]) * rs[j];
      d[j] = k1[j] * (d[j] - md[j] - xh * k2[j]);
    }
    st8f(dx + i * 8, d);
  }
}

// Backward apply that finishes the deferred column reduction itself (bn_colred8_k<1> with
// fin.defer): every workgroup folds the replicas of the two sums into per-channel constants in
// LDS, workgroup 0 publishes ws and accumulates dgamma / dbeta, the last workgroup to have read the
// replicas re-zeroes them.  Saves the reduction launch's arrival + exchange round trips.
__global__ __launch_bounds__(256) void bn_bwd_apply_fin8_k(const bf16_raw* __restrict__ dy,
                                                           const bf16_raw* __restrict__ x,
                                                           const bf16_raw* __restrict__ y,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, float* __restrict__ acc,
                                                           bf16_raw* __restrict__ dx, bf16_raw* __restrict__ dres,
                                                           long nch, int M, int C, int act, BnFin fin,
                                                           const float* __restrict__ zbeta = nullptr) {
  __shared__ float sk1[2048], sk2[2048], smd[2048], smu[2048], srs[2048];  // C <= 2048 (bn_vec_ok)
  const bool zmask = zbeta != nullptr && act == ACT_RELU;  // act' from z (bn_shift), y not read
  __shared__ int last;
  const float invM = 1.f / M;
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // two chunks per trip, the first trip's operands requested before the replica fold (see
  // bn_apply_fin8_k); apply_grid gives most launches exactly one trip
  const long i1 = i0 + stride < nch ? i0 + stride : i0;
  bf16x8 pd[2], px[2], py[2];
  if (i0 < nch) {
    pd[0] = *(const bf16x8*)(dy + i0 * 8);
    pd[1] = *(const bf16x8*)(dy + i1 * 8);
    px[0] = *(const bf16x8*)(x + i0 * 8);
    px[1] = *(const bf16x8*)(x + i1 * 8);
    if (act != ACT_NONE && !zmask) {
      py[0] = *(const bf16x8*)(y + i0 * 8);
      py[1] = *(const bf16x8*)(y + i1 * 8);
    }
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int r = 0; r < BN_NREP; ++r) {
      s += acc[(long)r * 2 * C + c];
      q += acc[(long)r * 2 * C + C + c];
    }
    const float rs = rstd[c];
    sk1[c] = (gamma ? gamma[c] : 1.f) * rs;  // dx = k1 * (dz - mean(dz) - xhat * mean(dz*xhat))
    sk2[c] = q * invM;
    smd[c] = s * invM;
    smu[c] = mean[c];
    srs[c] = rs;
    if (blockIdx.x == 0) {
      fin.ws[c] = s;
      fin.ws[C + c] = q;
      if (fin.dbeta) fin.dbeta[c] += s;
      if (fin.dgamma) fin.dgamma[c] += q;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) last = grid_arrive_last((unsigned*)(acc + (long)BN_NREP * 2 * C)) ? 1 : 0;
  const int CG = C >> 3;
  const int c0 = (int)(i0 % CG) * 8;
  float k1[8], k2[8], md[8], mu[8], rs[8], zs[8], zh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k1[j] = sk1[c0 + j];
    k2[j] = sk2[c0 + j];
    md[j] = smd[c0 + j];
    mu[j] = smu[c0 + j];
    rs[j] = srs[c0 + j];
    zs[j] = zh[j] = 0.f;
    if (zmask) {
      zs[j] = rs[j] * (gamma ? gamma[c0 + j] : 1.f);  // = k1, the forward's scale
      zh[j] = bn_shift(zbeta[c0 + j], mu[j], zs[j]);
    }
  }
  for (long i = i0; i < nch; i += 2 * stride) {
    const long ib = i + stride < nch ? i + stride : i;
    // next trip's operands in flight behind this trip's (see bn_apply_fin8_k)
    const long in0 = i + 2 * stride, in1 = in0 + stride < nch ? in0 + stride : in0;
    bf16x8 nd[2], nx[2], ny[2];
    if (in0 < nch) {
      nd[0] = *(const bf16x8*)(dy + in0 * 8);
      nd[1] = *(const bf16x8*)(dy + in1 * 8);
      nx[0] = *(const bf16x8*)(x + in0 * 8);
      nx[1] = *(const bf16x8*)(x + in1 * 8);
      if (act != ACT_NONE && !zmask) {
        ny[0] = *(const bf16x8*)(y + in0 * 8);
        ny[1] = *(const bf16x8*)(y + in1 * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && i + stride >= nch) break;
      const long o = (u == 0 ? i : ib) * 8;
      float d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        d[j] = bf2f((uint16_t)pd[u][j]);
        if (zmask) d[j] = fmaf(bf2f((uint16_t)px[u][j]), zs[j], zh[j]) > 0.f ? d[j] : 0.f;
        else if (act != ACT_NONE) d[j] *= act_grad_from_out(bf2f((uint16_t)py[u][j]), act);
      }
      if (dres) st8f(dres + o, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (bf2f((uint16_t)px[u][j]) - mu[j]) * rs[j];
        d[j] = k1[j] * (d[j] - md[j] - xh * k2[j]);
      }
      st8f(dx + o, d);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      pd[u] = nd[u];
      px[u] = nx[u];
      py[u] = ny[u];
    }
  }
  __syncthreads();
  if (last)
    for (int e = threadIdx.x; e < BN_NREP * 2 * C; e += 256) acc[e] = 0.f;
}

// ---------------------------------------------------------------------------------------------
// One-launch BN backward for tensors one trip of a resident grid covers (ResNet-20/56 every layer,
// the small ResNet-50 layers): every lane keeps its R rows of dy / x / y in registers, the
// workgroups add their column partials into the replicas, meet at a grid barrier, fold the
// replicas and write dx (+ dres) from the registers — no second launch and no second read of the
// three tensors.  The grid is sized to at most half the device's resident capacity (host side), so
// every workgroup is resident and a concurrent resident-grid kernel (the P2P collectives, <= 1
// workgroup per CU) still fits.  The barrier is sense-reversing on two zero-at-rest words after
// the arrival words (count, generation) and its spin is bounded by the wall clock: a lost
// workgroup cannot hang the device (the timeout is recorded in the third word).
template <int R>
__global__ __launch_bounds__(256) void bn_bwd_coop8_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ x,
                                                      const bf16_raw* __restrict__ y, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      float* __restrict__ acc, bf16_raw* __restrict__ dx,
                                                      bf16_raw* __restrict__ dres, int M, int C, int act, BnFin fin,
                                                      long long spin) {
  const int CG = C >> 3, RPI = 256 / CG;
  const int cg = threadIdx.x % CG, rsub = threadIdx.x / CG;
  const int c0 = cg * 8;
  const int rbase = blockIdx.x * (RPI * R) + rsub;
  float mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
  bf16x8 vd[R], vx[R], vy[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {  // every load of the lane first
    const int r = rbase + u * RPI;
    const long o = (long)(r < M ? r : 0) * C + c0;
    vd[u] = *(const bf16x8*)(dy + o);
    vx[u] = *(const bf16x8*)(x + o);
    if (act != ACT_NONE) vy[u] = *(const bf16x8*)(y + o);
  }
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
#pragma unroll
  for (int u = 0; u < R; ++u) {
    if (rbase + u * RPI >= M) break;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = bf2f((uint16_t)vd[u][j]);
      if (act != ACT_NONE) dz *= act_grad_from_out(bf2f((uint16_t)vy[u][j]), act);
      s1[j] += dz;
      s2[j] = fmaf(dz, (bf2f((uint16_t)vx[u][j]) - mu[j]) * rs[j], s2[j]);
    }
  }
  extern __shared__ float coop_smem[];  // [max(256*16, 5C)] floats
  float* red = coop_smem;
  float* dst = acc + (long)(blockIdx.x % BN_NREP) * 2 * C;
  bn_block_colsum(s1, s2, red, dst, C, CG, RPI);
  // ---- grid barrier (sense reversal; count, generation, timeout flag after the arrival words)
  unsigned* bar = (unsigned*)(acc + (long)BN_NREP * 2 * C) + kArriveWords;
  __shared__ int lastw;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial atomics are done
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned gen0 = __hip_atomic_load(bar + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (atomicAdd(bar, 1u) == gridDim.x - 1) {
      atomicExch(bar, 0u);
      atomicAdd(bar + 32, 1u);
    } else {
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(bar + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
        if ((long long)(wall_clock64() - t0) > spin) {
          atomicExch(bar + 64, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  // ---- fold the replicas (atomic reads: the partials landed at the memory side)
  float* sk1 = coop_smem;  // red is free again
  float* sk2 = sk1 + C;
  float* smd = sk2 + C;
  const float invM = 1.f / M;
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int r = 0; r < BN_NREP; ++r) {
      s += __hip_atomic_load(acc + (long)r * 2 * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      q += __hip_atomic_load(acc + (long)r * 2 * C + C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    sk1[c] = (gamma ? gamma[c] : 1.f) * rstd[c];
    sk2[c] = q * invM;
    smd[c] = s * invM;
    if (blockIdx.x == 0) {
      fin.ws[c] = s;
      fin.ws[C + c] = q;
      if (fin.dbeta) fin.dbeta[c] += s;
      if (fin.dgamma) fin.dgamma[c] += q;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) lastw = grid_arrive_last((unsigned*)(acc + (long)BN_NREP * 2 * C)) ? 1 : 0;
  float k1[8], k2[8], md[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { k1[j] = sk1[c0 + j]; k2[j] = sk2[c0 + j]; md[j] = smd[c0 + j]; }
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int r = rbase + u * RPI;
    if (r >= M) break;
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      d[j] = bf2f((uint16_t)vd[u][j]);
      if (act != ACT_NONE) d[j] *= act_grad_from_out(bf2f((uint16_t)vy[u][j]), act);
    }
    const long o = (long)r * C + c0;
    if (dres) st8f(dres + o, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (bf2f((uint16_t)vx[u][j]) - mu[j]) * rs[j];
      d[j] = k1[j] * (d[j] - md[j] - xh * k2[j]);
    }
    st8f(dx + o, d);
  }
  __syncthreads();
  if (lastw)
    for (int e = threadIdx.x; e < BN_NREP * 2 * C; e += 256) acc[e] = 0.f;
}

static bool bn_vec_ok(int C, std::initializer_list<const void*> ptrs) {
  if (C % 8 != 0 || C / 8 > 256 || (256 % (C / 8)) != 0 || hopsx_disabled("bn_vec")) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16 != 0) return false;
  return true;
}

// Deferred fold (the apply kernel folds the replicas, no arrival round trips in the reduction) costs
// every apply workgroup a read of BN_NREP x 2C floats: cheap at narrow C, a large share of the apply's
// traffic at C = 1024 / 2048.  Above HOPSX_BN_DEFER_MAXC the reduction's last workgroup folds instead.
static int bn_defer(int C) {
  static const long maxc = hopsx_env_int("HOPSX_BN_DEFER_MAXC", 1L << 30);
  return hopsx_disabled("bn_defer") || C > maxc ? 0 : 1;
}

// Wide channels: one small launch folds the replicas once (thread per channel; re-zeroes them) and the
// plain apply kernels read the folded per-channel values, instead of every apply workgroup reading
// BN_NREP x 2C floats.  A/B knob HOPSX_BN_FOLD_MINC (channels from which it applies; default off).
template <int MODE>
__global__ __launch_bounds__(256) void bn_fold_k(float* __restrict__ acc, int M, int C, BnFin fin) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int r = 0; r < BN_NREP; ++r) {
    s += acc[(long)r * 2 * C + c];
    q += acc[(long)r * 2 * C + C + c];
    acc[(long)r * 2 * C + c] = 0.f;
    acc[(long)r * 2 * C + C + c] = 0.f;
  }
  if (MODE == 0) {  // as bn_apply_fin8_k
    const float mu = s / M;
    const float var = fmaxf(q / M - mu * mu, 0.f);
    fin.mean_out[c] = mu;
    fin.rstd_out[c] = rsqrtf(var + fin.eps);
    if (fin.rmean) {
      const float unb = M > 1 ? var * M / (M - 1) : var;
      fin.rmean[c] = (1.f - fin.momentum) * fin.rmean[c] + fin.momentum * mu;
      fin.rvar[c] = (1.f - fin.momentum) * fin.rvar[c] + fin.momentum * unb;
    }
  } else {  // as bn_bwd_apply_fin8_k's workgroup 0
    fin.ws[c] = s;
    fin.ws[C + c] = q;
    if (fin.dbeta) fin.dbeta[c] += s;
    if (fin.dgamma) fin.dgamma[c] += q;
  }
}
static bool bn_fold_first(int C) {
  static const long minc = hopsx_env_int("HOPSX_BN_FOLD_MINC", 1L << 30);
  return C >= minc;
}

static int colred_grid(int M, int C, int& rpb) {
  const int RPI = 256 / (C / 8);
  // ~BN_UNR rows per thread: one trip of loads in flight per lane and >= 256 workgroups on the
  // ResNet-20 stage-1 shapes (8 rows per thread left half the CUs idle there)
  const long rpt = hopsx_env_int("HOPSX_BN_RPT", BN_UNR);
  long g = (M + (long)RPI * rpt - 1) / ((long)RPI * rpt);
  static const long maxg = hopsx_env_int("HOPSX_BN_MAXG", 1024);
  if (g > maxg) g = maxg;
  if (g < 1) g = 1;
  rpb = (int)((M + g - 1) / g);
  return (int)((M + rpb - 1) / rpb);
}

static int apply_grid(long nch, int C) {
  const int CG = C >> 3;
  long g = (nch + 511) / 512;  // two chunks per thread per trip
  // at most 1024 workgroups (several trips per thread on the big ResNet-50 tensors): every workgroup folds
  // the BN_NREP x 2C replica floats first, so fewer of them means less fold traffic — ResNet-50 B=64
  // 5.95 k -> 6.07-6.21 k img/s, B=256 8.48 k -> 8.68 k vs 4096 (profiles/r5_bn_apply_grid_ab.txt); the CIFAR
  // ResNets' tensors need <= 512
  static const long maxg = hopsx_env_int("HOPSX_BN_APPLY_MAXG", 1024);
  if (g > maxg) g = maxg;
  if (g < 1) g = 1;
  // gridDim*256 must be a multiple of CG (per-thread channel group); CG divides 256
  (void)CG;
  return (int)g;
}

static void slab_grid(int M, int C, int& gx, int& gy, int& rpb) {
  gx = (C + 63) / 64;
  gy = (M + 255) / 256;
  const int max_gy = (2048 + gx - 1) / gx;
  if (gy > max_gy) gy = max_gy;
  if (gy < 1) gy = 1;
  rpb = (M + gy - 1) / gy;
}
static int ew_grid(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

// the one-launch backward (bn_bwd_coop8_k) when a resident grid covers the tensor in one trip
template <int R>
static bool bn_coop_try(const void* dy, const void* x, const void* y, const float* gamma, const float* mean,
                        const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int C, int act,
                        void* dres, float* acc, hipStream_t st) {
  static int n_cu = 0, occ = 0;
  const size_t shm = std::max<size_t>(256 * 16, 3 * (size_t)C) * sizeof(float);
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
  }
  static size_t occ_shm = 0;
  if (!occ || occ_shm != shm) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bn_bwd_coop8_k<R>, 256, shm) != hipSuccess) occ = 0;
    occ_shm = shm;
  }
  const int RPI = 256 / (C / 8);
  const long G = ((long)M + (long)RPI * R - 1) / ((long)RPI * R);
  const long cap = (long)n_cu * occ / 2;  // half the resident capacity: see bn_bwd_coop8_k
  if (G < 1 || G > cap) return false;
  const BnFin fin{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, ws, dgamma, dbeta, 1};
  const long long spin = 200000000LL;  // 2 s of the 100 MHz wall clock
  hipLaunchKernelGGL(bn_bwd_coop8_k<R>, dim3((unsigned)G), dim3(256), shm, st, (const bf16_raw*)dy,
                     (const bf16_raw*)x, (const bf16_raw*)y, gamma, mean, rstd, acc, (bf16_raw*)dx, (bf16_raw*)dres, M,
                     C, act, fin, spin);
  return true;
}

static bool bn_bwd_coop(const void* dy, const void* x, const void* y, const float* gamma, const float* mean,
                        const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int C, int act,
                        void* dres, float* acc, hipStream_t st) {
  // off by default: measured SLOWER than the two launches (ResNet-20 111.6k -> 102.7k img/s, ResNet-50
  // B=64 4.15k -> 4.10k; profiles/r2s7_verify2_ab.txt) — fewer workgroups in flight per tensor and the
  // barrier's round trips outweigh the saved launch and re-read.  HOPSX_BN_COOP=1 to A/B.
  static const long on = hopsx_env_int("HOPSX_BN_COOP", 0);
  if (!on) return false;
  return bn_coop_try<1>(dy, x, y, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, C, act, dres, acc, st) ||
         bn_coop_try<2>(dy, x, y, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, C, act, dres, acc, st) ||
         bn_coop_try<4>(dy, x, y, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, C, act, dres, acc, st) ||
         bn_coop_try<8>(dy, x, y, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, C, act, dres, acc, st);
}

// timeout flag of the coop barrier (tests)
extern "C" int hopsx_bn_coop_timeouts(const float* acc, int C) {
  unsigned v = 0;
  const unsigned* bar = (const unsigned*)(acc + (long)BN_NREP * 2 * C) + kArriveWords;
  if (hipMemcpy(&v, bar + 64, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

extern "C" int hopsx_bn_fwd_train(const void* x, void* y, const float* gamma, const float* beta, float* mean_out,
                                  float* rstd_out, float* running_mean, float* running_var, float momentum,
                                  float eps, int M, int C, const void* residual, int act, float* acc,
                                  hipStream_t st) {
  const long n = (long)M * C;
  if (acc && bn_vec_ok(C, {x, y, residual})) {  // acc: BN_NREP x 2C floats + arrival words, zero at rest
    int rpb;
    const int g = colred_grid(M, C, rpb);
    const int defer = bn_defer(C);
    const BnFin fin{mean_out, rstd_out, running_mean, running_var, momentum, eps, nullptr, nullptr, nullptr, defer};
    hipLaunchKernelGGL(bn_colred8_k<0>, dim3(g), dim3(256), 0, st, (const bf16_raw*)x, nullptr, nullptr, nullptr,
                       nullptr, acc, M, C, rpb, 0, fin);
    if (defer)  // the apply folds the replicas (the same launch the conv-epilogue statistics use)
      hipLaunchKernelGGL(bn_apply_fin8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)x,
                         (bf16_raw*)y, gamma, beta, acc, n / 8, M, C, (const bf16_raw*)residual, act, fin);
    else
      hipLaunchKernelGGL(bn_apply8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y,
                         gamma, beta, mean_out, rstd_out, 0, eps, n / 8, C, (const bf16_raw*)residual, act);
    return (int)hipGetLastError();
  }
  hopsx_zero(mean_out, C * sizeof(float), st);
  hopsx_zero(rstd_out, C * sizeof(float), st);
  int gx, gy, rpb;
  slab_grid(M, C, gx, gy, rpb);
  hipLaunchKernelGGL(bn_stats_k, dim3(gx, gy), dim3(256), 0, st, (const bf16_raw*)x, mean_out, rstd_out, M, C, rpb);
  hipLaunchKernelGGL(bn_finalize_k, dim3((C + 255) / 256), dim3(256), 0, st, mean_out, rstd_out, running_mean,
                     running_var, momentum, eps, M, C);
  hipLaunchKernelGGL(bn_apply_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, gamma, beta,
                     mean_out, rstd_out, 0, eps, n, C, (const bf16_raw*)residual, act);
  return (int)hipGetLastError();
}

// Training forward whose statistics are already in `acc` (accumulated by the producing conv's
// epilogue, hopsx_conv2d_fwd_bnstats): one launch, re-zeroes acc.  -2 if the vector path does
// not apply (the caller must not have produced the statistics then: check hopsx_bn_prestats_ok).
extern "C" int hopsx_bn_fwd_apply_fin(const void* x, void* y, const float* gamma, const float* beta, float* mean_out,
                                      float* rstd_out, float* running_mean, float* running_var, float momentum,
                                      float eps, int M, int C, const void* residual, int act, float* acc,
                                      hipStream_t st) {
  if (!acc || !bn_vec_ok(C, {x, y, residual})) return -2;
  const long n = (long)M * C;
  const BnFin fin{mean_out, rstd_out, running_mean, running_var, momentum, eps, nullptr, nullptr, nullptr};
  if (bn_fold_first(C)) {
    hipLaunchKernelGGL(bn_fold_k<0>, dim3((C + 255) / 256), dim3(256), 0, st, acc, M, C, fin);
    hipLaunchKernelGGL(bn_apply8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y,
                       gamma, beta, mean_out, rstd_out, 0, eps, n / 8, C, (const bf16_raw*)residual, act);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_apply_fin8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)x,
                     (bf16_raw*)y, gamma, beta, acc, n / 8, M, C, (const bf16_raw*)residual, act, fin);
  return (int)hipGetLastError();
}

extern "C" int hopsx_bn_prestats_ok(int C) { return bn_vec_ok(C, {}) ? 1 : 0; }

extern "C" int hopsx_bn_fwd_infer(const void* x, void* y, const float* gamma, const float* beta,
                                  const float* running_mean, const float* running_var, float eps, int M, int C,
                                  const void* residual, int act, hipStream_t st) {
  const long n = (long)M * C;
  if (bn_vec_ok(C, {x, y, residual})) {
    hipLaunchKernelGGL(bn_apply8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y,
                       gamma, beta, running_mean, running_var, 1, eps, n / 8, C, (const bf16_raw*)residual, act);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_apply_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, gamma, beta,
                     running_mean, running_var, 1, eps, n, C, (const bf16_raw*)residual, act);
  return (int)hipGetLastError();
}

// The column sums already sit in acc's replica rows (a consumer conv's dgrad epilogue reduced them:
// conv_mfma.hip DgradArgs bnacc) and dy is the masked output gradient: the apply alone, no act' and no
// residual gradient (the caller hands dy itself on as the residual's gradient).
extern "C" int hopsx_bn_bwd_pre(const void* dy, const void* x, const float* gamma, const float* mean,
                                const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int C,
                                float* acc, hipStream_t st) {
  if (!acc || !bn_vec_ok(C, {dy, x, dx})) return -2;
  const long n = (long)M * C;
  const BnFin fin{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, ws, dgamma, dbeta, 1};
  if (bn_fold_first(C)) {
    hipLaunchKernelGGL(bn_fold_k<1>, dim3((C + 255) / 256), dim3(256), 0, st, acc, M, C, fin);
    hipLaunchKernelGGL(bn_bwd_apply8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)dy,
                       (const bf16_raw*)x, (const bf16_raw*)nullptr, gamma, mean, rstd, ws, (bf16_raw*)dx,
                       (bf16_raw*)nullptr, n / 8, M, C, (int)ACT_NONE);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bn_bwd_apply_fin8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)dy,
                     (const bf16_raw*)x, (const bf16_raw*)nullptr, gamma, mean, rstd, acc, (bf16_raw*)dx,
                     (bf16_raw*)nullptr, n / 8, M, C, (int)ACT_NONE, fin, (const float*)nullptr);
  return (int)hipGetLastError();
}

// zbeta: the BN's beta when its forward had no residual (ReLU: act' taken from x, see bn_shift); else null
extern "C" int hopsx_bn_bwd(const void* dy, const void* x, const void* y, const float* gamma, const float* mean,
                            const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int C,
                            int act, void* dresidual, float* acc, const float* zbeta, hipStream_t st) {
  if (hopsx_disabled("bn_zmask")) zbeta = nullptr;
  const long n = (long)M * C;
  if (acc && bn_vec_ok(C, {dy, x, y, dx, dresidual})) {  // acc: BN_NREP x 2C floats + arrival words, zero at rest
    int rpb;
    const int g = colred_grid(M, C, rpb);
    if (bn_bwd_coop(dy, x, y, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, C, act, dresidual, acc, st))
      return (int)hipGetLastError();
    const int defer = bn_defer(C);
    const BnFin fin{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, ws, dgamma, dbeta, defer};
    hipLaunchKernelGGL(bn_colred8_k<1>, dim3(g), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)x,
                       (const bf16_raw*)y, mean, rstd, acc, M, C, rpb, act, fin, gamma, zbeta);
    if (defer && bn_fold_first(C)) {  // (wide channels: y is read, the plain apply has no zmask)
      hipLaunchKernelGGL(bn_fold_k<1>, dim3((C + 255) / 256), dim3(256), 0, st, acc, M, C, fin);
      hipLaunchKernelGGL(bn_bwd_apply8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)dy,
                         (const bf16_raw*)x, (const bf16_raw*)y, gamma, mean, rstd, ws, (bf16_raw*)dx,
                         (bf16_raw*)dresidual, n / 8, M, C, act);
      return (int)hipGetLastError();
    }
    if (defer) {
      hipLaunchKernelGGL(bn_bwd_apply_fin8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)dy,
                         (const bf16_raw*)x, (const bf16_raw*)y, gamma, mean, rstd, acc, (bf16_raw*)dx,
                         (bf16_raw*)dresidual, n / 8, M, C, act, fin, zbeta);
      return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(bn_bwd_apply8_k, dim3(apply_grid(n / 8, C)), dim3(256), 0, st, (const bf16_raw*)dy,
                       (const bf16_raw*)x, (const bf16_raw*)y, gamma, mean, rstd, ws, (bf16_raw*)dx,
                       (bf16_raw*)dresidual, n / 8, M, C, act);
    return (int)hipGetLastError();
  }
  hopsx_zero(ws, 2 * C * sizeof(float), st);
  int gx, gy, rpb;
  slab_grid(M, C, gx, gy, rpb);
  hipLaunchKernelGGL(bn_bwd_reduce_k, dim3(gx, gy), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)x,
                     (const bf16_raw*)y, mean, rstd, ws, M, C, rpb, act);
  hipLaunchKernelGGL(bn_bwd_apply_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)x,
                     (const bf16_raw*)y, gamma, mean, rstd, ws, (bf16_raw*)dx, (bf16_raw*)dresidual, n, M, C, act);
  hipLaunchKernelGGL(bn_grad_acc_k, dim3((C + 255) / 256), dim3(256), 0, st, ws, dgamma, dbeta, C);
  return (int)hipGetLastError();
}
