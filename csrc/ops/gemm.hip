// Dense GEMM entry points (Linear fwd / dgrad / wgrad, MLP and wide&deep towers).
#include "gemm_core.h"
#include "ops_api.h"

using namespace hopsx;

// Finishing pass of a split-K GEMM whose partial sums were atomically
// accumulated into the fp32 workspace: bias + activation (or activation
// derivative) + dtype cast + optional bias-gradient column sum, one thread per
// output column so the column sum needs a single atomic per column.
__global__ __launch_bounds__(256) void splitk_finish_k(const float* __restrict__ ws, int M, int N, int epi,
                                                       void* __restrict__ out, long ldo, const float* __restrict__ bias,
                                                       float alpha, float beta, int act,
                                                       const bf16_raw* __restrict__ aux, long ldaux,
                                                       float* __restrict__ colsum, int rows_per_block) {
  // block = 4 rows x 64 columns; every thread handles ONE element per row group so
  // the loads are independent (a serial per-column row loop was L2-latency bound)
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int m = blockIdx.y * 4 + (threadIdx.x >> 6);
  __shared__ float red[4][64];
  float cs = 0.f;
  if (n < N && m < M) {
    const float b = bias ? bias[n] : 0.f;
    float v = ws[(long)m * N + n];
    if (epi == EPI_DACT_BF16) {
      if (aux) v *= act_grad_from_out(bf2f(aux[(long)m * ldaux + n]), act);
      ((bf16_raw*)out)[(long)m * ldo + n] = f2bf(v);
    } else {
      v = apply_act(v * alpha + b, act);
      if (epi == EPI_STORE_BF16) {
        ((bf16_raw*)out)[(long)m * ldo + n] = f2bf(v);
      } else {
        float* o = (float*)out + (long)m * ldo + n;
        if (beta != 0.f) v += beta * *o;
        *o = v;
      }
    }
    cs = v;
  }
  if (!colsum) return;
  red[threadIdx.x >> 6][threadIdx.x & 63] = cs;
  __syncthreads();
  if (threadIdx.x < 64 && n < N)
    atomicAdd(colsum + n, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// Small-M / long-K GEMMs (e.g. the MNIST Dense(128) over 10816 features at batch
// 32: 4 output tiles) cannot fill 256 CUs without splitting K.  Non-atomic
// epilogues then go through an fp32 workspace: memset node + atomic split-K
// GEMM + finishing pass (all graph-capturable).
static bool want_splitk(int M, int N, int K) {
  GemmPlan p = plan_gemm(M, N, K, true);
  return p.split >= 4 && !hopsx_disabled("splitk");
}

template <bool AK, bool BK_>
static int dispatch_epi(const DenseLoader& al, const DenseLoader& bl, int M, int N, int K, int epi, void* out,
                        long ldo, const float* bias, float alpha, float beta, int act, const void* aux, long ldaux,
                        float* colsum, hipStream_t st, float* rowsum_a) {
  switch (epi) {
    case EPI_STORE_BF16: {
      EpiStoreBF16 e{(bf16_raw*)out, ldo, bias, alpha, act, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, false, st, rowsum_a);
      break;
    }
    case EPI_STORE_F32: {
      EpiStoreF32 e{(float*)out, ldo, bias, alpha, beta, act, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, false, st, rowsum_a);
      break;
    }
    case EPI_ATOMIC_F32: {
      EpiAtomicF32 e{(float*)out, ldo, alpha, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, true, st, rowsum_a);
      break;
    }
    case EPI_DACT_BF16: {
      EpiDActBF16 e{(bf16_raw*)out, ldo, (const bf16_raw*)aux, ldaux, act, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, false, st, rowsum_a);
      break;
    }
    default:
      return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int hopsx_gemm(const void* A, long lda, int a_kc, const void* B, long ldb, int b_kc, int M, int N, int K,
                          int epi, void* out, long ldo, const float* bias, float alpha, float beta, int act,
                          const void* aux, long ldaux, float* colsum, float* ws, long ws_elems, const void* ay,
                          int aact, float* arowsum, unsigned* tickets, hipStream_t st) {
  // ay/aact: fused act' mask on the A operand (same layout as A); arowsum: row sums of
  // the (masked) A operand — the bias gradient when A = dY^T in a weight-gradient GEMM
  DenseLoader al{(const bf16_raw*)A, lda, is_vec_ok(A, lda) && is_vec_ok(ay ? ay : A, lda), (const bf16_raw*)ay,
                 aact};
  DenseLoader bl{(const bf16_raw*)B, ldb, is_vec_ok(B, ldb)};
  if (ws && tickets && epi != EPI_ATOMIC_F32 && (long)M * N <= ws_elems && want_splitk(M, N, K) &&
      !hopsx_disabled("splitk_ticket")) {
    // ws is persistent and zero at rest (see EpiAtomicTicket)
    SplitFinish f{tickets, epi, out, ldo, bias, alpha, beta, act, (const bf16_raw*)aux, ldaux, colsum};
    EpiAtomicTicket e{ws, N, 1.f, nullptr, f};
    if (a_kc && b_kc) launch_gemm<true, true>(al, bl, e, M, N, K, true, st, arowsum);
    else if (a_kc) launch_gemm<true, false>(al, bl, e, M, N, K, true, st, arowsum);
    else if (b_kc) launch_gemm<false, true>(al, bl, e, M, N, K, true, st, arowsum);
    else launch_gemm<false, false>(al, bl, e, M, N, K, true, st, arowsum);
    return (int)hipGetLastError();
  }
  if (ws && epi != EPI_ATOMIC_F32 && (long)M * N <= ws_elems && want_splitk(M, N, K)) {
    hopsx_zero(ws, (long)M * N * sizeof(float), st);
    int rc = hopsx_gemm(A, lda, a_kc, B, ldb, b_kc, M, N, K, EPI_ATOMIC_F32, ws, N, nullptr, 1.f, 0.f, 0, nullptr, 0,
                        nullptr, nullptr, 0, ay, aact, arowsum, nullptr, st);
    if (rc) return rc;
    const int gx = (N + 63) / 64;
    const int gy = (M + 3) / 4;
    hipLaunchKernelGGL(splitk_finish_k, dim3(gx, gy), dim3(256), 0, st, ws, M, N, epi, out, ldo, bias, alpha, beta,
                       act, (const bf16_raw*)aux, ldaux, colsum, 4);
    return (int)hipGetLastError();
  }
  if (a_kc && b_kc)
    return dispatch_epi<true, true>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum, st, arowsum);
  if (a_kc && !b_kc)
    return dispatch_epi<true, false>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum, st, arowsum);
  if (!a_kc && !b_kc)
    return dispatch_epi<false, false>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum,
                                      st, arowsum);
  return dispatch_epi<false, true>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum, st, arowsum);
}
