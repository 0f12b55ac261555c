// BatchNorm over NHWC activations viewed as [M = B*H*W, C] (channel-fastest),
// with the residual add and the activation fused into the apply pass
// (ResNet: y = act(bn(x) + residual)) and into the backward.
#include "common.h"
#include "ops_api.h"

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
  if (threadIdx.x < 64 && c < C) {
    const int t = threadIdx.x;
    atomicAdd(s1 + c, ra[0][t] + ra[1][t] + ra[2][t] + ra[3][t]);
    atomicAdd(s2 + c, rb[0][t] + rb[1][t] + rb[2][t] + rb[3][t]);
  }
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
  if (threadIdx.x < 64 && c < C) {
    const int t = threadIdx.x;
    atomicAdd(ws + c, ra[0][t] + ra[1][t] + ra[2][t] + ra[3][t]);
    atomicAdd(ws + C + c, rb[0][t] + rb[1][t] + rb[2][t] + rb[3][t]);
  }
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

extern "C" int hopsx_bn_fwd_train(const void* x, void* y, const float* gamma, const float* beta, float* mean_out,
                                  float* rstd_out, float* running_mean, float* running_var, float momentum,
                                  float eps, int M, int C, const void* residual, int act, hipStream_t st) {
  hopsx_zero(mean_out, C * sizeof(float), st);
  hopsx_zero(rstd_out, C * sizeof(float), st);
  int gx, gy, rpb;
  slab_grid(M, C, gx, gy, rpb);
  hipLaunchKernelGGL(bn_stats_k, dim3(gx, gy), dim3(256), 0, st, (const bf16_raw*)x, mean_out, rstd_out, M, C, rpb);
  hipLaunchKernelGGL(bn_finalize_k, dim3((C + 255) / 256), dim3(256), 0, st, mean_out, rstd_out, running_mean,
                     running_var, momentum, eps, M, C);
  const long n = (long)M * C;
  hipLaunchKernelGGL(bn_apply_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, gamma, beta,
                     mean_out, rstd_out, 0, eps, n, C, (const bf16_raw*)residual, act);
  return (int)hipGetLastError();
}

extern "C" int hopsx_bn_fwd_infer(const void* x, void* y, const float* gamma, const float* beta,
                                  const float* running_mean, const float* running_var, float eps, int M, int C,
                                  const void* residual, int act, hipStream_t st) {
  const long n = (long)M * C;
  hipLaunchKernelGGL(bn_apply_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)x, (bf16_raw*)y, gamma, beta,
                     running_mean, running_var, 1, eps, n, C, (const bf16_raw*)residual, act);
  return (int)hipGetLastError();
}

extern "C" int hopsx_bn_bwd(const void* dy, const void* x, const void* y, const float* gamma, const float* mean,
                            const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int C,
                            int act, void* dresidual, hipStream_t st) {
  hopsx_zero(ws, 2 * C * sizeof(float), st);
  int gx, gy, rpb;
  slab_grid(M, C, gx, gy, rpb);
  hipLaunchKernelGGL(bn_bwd_reduce_k, dim3(gx, gy), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)x,
                     (const bf16_raw*)y, mean, rstd, ws, M, C, rpb, act);
  const long n = (long)M * C;
  hipLaunchKernelGGL(bn_bwd_apply_k, dim3(ew_grid(n)), dim3(256), 0, st, (const bf16_raw*)dy, (const bf16_raw*)x,
                     (const bf16_raw*)y, gamma, mean, rstd, ws, (bf16_raw*)dx, (bf16_raw*)dresidual, n, M, C, act);
  hipLaunchKernelGGL(bn_grad_acc_k, dim3((C + 255) / 256), dim3(256), 0, st, ws, dgamma, dbeta, C);
  return (int)hipGetLastError();
}
