// Dense GEMM entry points (Linear fwd / dgrad / wgrad, MLP and wide&deep towers).
#include "gemm_core.h"
#include "ops_api.h"

using namespace hopsx;

template <bool AK, bool BK_>
static int dispatch_epi(const DenseLoader& al, const DenseLoader& bl, int M, int N, int K, int epi, void* out,
                        long ldo, const float* bias, float alpha, float beta, int act, const void* aux, long ldaux,
                        float* colsum, hipStream_t st) {
  switch (epi) {
    case EPI_STORE_BF16: {
      EpiStoreBF16 e{(bf16_raw*)out, ldo, bias, alpha, act, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, false, st);
      break;
    }
    case EPI_STORE_F32: {
      EpiStoreF32 e{(float*)out, ldo, bias, alpha, beta, act, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, false, st);
      break;
    }
    case EPI_ATOMIC_F32: {
      EpiAtomicF32 e{(float*)out, ldo, alpha, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, true, st);
      break;
    }
    case EPI_DACT_BF16: {
      EpiDActBF16 e{(bf16_raw*)out, ldo, (const bf16_raw*)aux, ldaux, act, colsum};
      launch_gemm<AK, BK_>(al, bl, e, M, N, K, false, st);
      break;
    }
    default:
      return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int hopsx_gemm(const void* A, long lda, int a_kc, const void* B, long ldb, int b_kc, int M, int N, int K,
                          int epi, void* out, long ldo, const float* bias, float alpha, float beta, int act,
                          const void* aux, long ldaux, float* colsum, hipStream_t st) {
  DenseLoader al{(const bf16_raw*)A, lda, is_vec_ok(A, lda)};
  DenseLoader bl{(const bf16_raw*)B, ldb, is_vec_ok(B, ldb)};
  if (a_kc && b_kc)
    return dispatch_epi<true, true>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum, st);
  if (a_kc && !b_kc)
    return dispatch_epi<true, false>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum, st);
  if (!a_kc && !b_kc)
    return dispatch_epi<false, false>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum,
                                      st);
  return dispatch_epi<false, true>(al, bl, M, N, K, epi, out, ldo, bias, alpha, beta, act, aux, ldaux, colsum, st);
}
