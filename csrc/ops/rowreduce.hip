// Column reductions over row-major [M, N] bf16 activations — the bias gradient
// of Linear / Conv layers — optionally fused with the activation backward
// (dx = dy * act'(y)).  Vectorised: each lane owns 8 consecutive columns
// (one 16-B load per row), keeps its 8 partial sums in registers across all
// rows of its slab, and a workgroup reduces its lanes through LDS before ONE
// fp32 atomic per column.  Slabs are sized so the grid is ~1-2 workgroups per
// CU: an earlier row-slab design with 2048 workgroups spent most of its time
// in same-address atomics (24.8 us for a 32-column conv bias in the MNIST
// profile, profiles/it2_b32_kernels.txt).
#include "common.h"
#include "ops_api.h"

HOPSX_DET_TU(rowreduce)

extern "C" int hopsx_colsum_bf16_scalar(const void* x, float* out, int M, int N, hipStream_t st);
extern "C" int hopsx_act_bwd_colsum_scalar(const void* dy, const void* y, void* dx, int M, int N, int act,
                                           float* colsum, hipStream_t st);

template <bool WRITE_DX>
__global__ __launch_bounds__(256) void rowreduce8_k(const bf16_raw* __restrict__ dy, const bf16_raw* __restrict__ y,
                                                    bf16_raw* __restrict__ dx, int M, int N, int act,
                                                    float* __restrict__ colsum, int rows_per_block) {
  extern __shared__ float red[];  // [rows_per_pass][N]
  const int g = N >> 3;                  // column groups of 8
  const int rpp = blockDim.x / g;        // rows per pass
  const int tid = threadIdx.x;
  const int cg = tid % g, rl = tid / g;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rl < rpp) {
    for (int m = r0 + rl; m < r1; m += rpp) {
      const long off = (long)m * N + cg * 8;
      bf16x8 v = *(const bf16x8*)(dy + off);
      if (y) {
        const bf16x8 yy = *(const bf16x8*)(y + off);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f((uint16_t)v[j]) * act_grad_from_out(bf2f((uint16_t)yy[j]), act);
          v[j] = (short)f2bf(f);
        }
      }
      if (WRITE_DX) *(bf16x8*)(dx + off) = v;
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f((uint16_t)v[j]);
    }
  }
  if (!colsum) return;
  if (rl < rpp)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rl * N + cg * 8 + j] = s[j];
  __syncthreads();
  const bool det = det_on();
  if (det) det_turn_begin(DET_COLSUM, blockIdx.x);
  for (int c = tid; c < N; c += blockDim.x) {
    float t = 0.f;
    for (int r = 0; r < rpp; ++r) t += red[r * N + c];
    if (t != 0.f) atomicAdd(colsum + c, t);
  }
  if (det) det_turn_end(DET_COLSUM, blockIdx.x, gridDim.x);
}

static int launch_rowreduce(const void* dy, const void* y, void* dx, int M, int N, int act, float* colsum,
                            hipStream_t st) {
  const int g = N / 8;
  const int rpp = 256 / g;
  // ~2 workgroups per CU at most, >= 4 rows per lane-row per workgroup
  long blocks = (M + rpp * 4 - 1) / (rpp * 4);
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  const int rpb = (int)((M + blocks - 1) / blocks);
  blocks = (M + rpb - 1) / rpb;
  const size_t shm = colsum ? (size_t)rpp * N * sizeof(float) : 0;
  if (dx)
    hipLaunchKernelGGL(rowreduce8_k<true>, dim3(blocks), dim3(256), shm, st, (const bf16_raw*)dy, (const bf16_raw*)y,
                       (bf16_raw*)dx, M, N, act, colsum, rpb);
  else
    hipLaunchKernelGGL(rowreduce8_k<false>, dim3(blocks), dim3(256), shm, st, (const bf16_raw*)dy,
                       (const bf16_raw*)y, (bf16_raw*)dx, M, N, act, colsum, rpb);
  return (int)hipGetLastError();
}

static bool vec8_ok(int N, const void* a, const void* b, const void* c) {
  return N % 8 == 0 && N / 8 <= 256 && ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16 == 0 &&
         !hopsx_disabled("rowreduce");
}

extern "C" int hopsx_colsum_bf16(const void* x, float* out, int M, int N, hipStream_t st) {
  if (!vec8_ok(N, x, nullptr, nullptr)) return hopsx_colsum_bf16_scalar(x, out, M, N, st);
  return launch_rowreduce(x, nullptr, nullptr, M, N, 0, out, st);
}

extern "C" int hopsx_act_bwd_colsum(const void* dy, const void* y, void* dx, int M, int N, int act, float* colsum,
                                    hipStream_t st) {
  if (!vec8_ok(N, dy, y, dx)) return hopsx_act_bwd_colsum_scalar(dy, y, dx, M, N, act, colsum, st);
  return launch_rowreduce(dy, y, dx, M, N, act, colsum, st);
}
