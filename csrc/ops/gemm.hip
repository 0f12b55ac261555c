// Dense GEMM entry points (Linear fwd / dgrad / wgrad, MLP and wide&deep towers).
#include "gemm_core.h"
#include "ops_api.h"

HOPSX_DET_TU(gemm)

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

// ---------------------------------------------------------------------------
// A Linear layer's whole backward in ONE launch (horizontal fusion): the first gxA*gyA
// workgroups compute dX = (dY*act'(y)) . W (masked by the previous layer's act'), the rest
// dW += (dY*act'(y))^T . X with the bias gradient as the staged operand's row sums.  At small
// batch each GEMM alone is a latency-bound launch on a few hundred workgroups.
template <int BMA, int BMB, class EPA, class EPB>
__global__ __launch_bounds__(256) void linear_bwd_pair_k(DenseLoader aA, DenseLoader bA, EPA eA, int MA,
                                                         int NA, int KA, int kpsA, int gxA, int gyA, DenseLoader aB,
                                                         DenseLoader bB, EPB eB, int MB, int NB, int KB,
                                                         int kpsB, int gxB, int gyB, float* rowsumB) {
  const int nA = gxA * gyA;
  if ((int)blockIdx.x < nA) {
    const int b = blockIdx.x;
    mfma_gemm_body<BMA, BMA, 2, true, false>(aA, bA, eA, MA, NA, KA, kpsA, nullptr, b % gxA, gxA, b / gxA, gyA);
  } else {
    const int b = blockIdx.x - nA;
    mfma_gemm_body<BMB, BMB, 2, false, false>(aB, bB, eB, MB, NB, KB, kpsB, rowsumB, b % gxB, gxB, b / gxB, gyB);
  }
}

static int bm_of(int cfg) { return cfg == 0 ? 128 : (cfg == 1 ? 64 : 32); }

// dy [M,N] (masked by act'(y) when ay), W [N,K], x [M,K]: dx [M,K] (masked by act'(yprev), colsum ->
// previous layer's bias grad), dw [N,K] += , dbias [N] += .  -2: shape better served by two launches.
extern "C" int hopsx_linear_bwd_pair(const void* dy, const void* w, const void* x, void* dx, const void* yprev,
                                     int act_prev, float* colsum, const void* ay, int aact, float* dw, float* dbias,
                                     int M, int N, int K, const int* pool, const unsigned char* pool_am,
                                     const void* pool_x, const unsigned long long* pool_rng, unsigned pool_salt,
                                     float pool_p, int dw_store, hipStream_t st) {
  if (hopsx_disabled("bwd_pair") || M <= 0 || N <= 0 || K <= 0) return -2;
  // dgrad: [M x K] = dy[M x N] . W[N x K]
  if (want_splitk(M, K, N)) return -2;  // the small-M split-K dgrad path keeps its own launch
  GemmPlan pa = plan_gemm(M, K, N, false);
  GemmPlan pb = plan_gemm(N, K, M, true);
  const int bma = bm_of(pa.cfg), bmb = bm_of(pb.cfg);
  const int gxA = ((M + bma - 1) / bma) * ((K + bma - 1) / bma), gyA = pa.split;
  const int gxB = ((N + bmb - 1) / bmb) * ((K + bmb - 1) / bmb), gyB = pb.split;
  const long total = (long)gxA * gyA + (long)gxB * gyB;
  if (total > (1L << 20)) return -2;
  DenseLoader aA{(const bf16_raw*)dy, N, is_vec_ok(dy, N) && is_vec_ok(ay ? ay : dy, N), (const bf16_raw*)ay, aact};
  DenseLoader bA{(const bf16_raw*)w, K, is_vec_ok(w, K)};
  EpiDActBF16 eA{(bf16_raw*)dx, K, (const bf16_raw*)yprev, K, act_prev, colsum};
  // pool = {C, PH, PW, KH, KW, act, H, W}: dx is the pool INPUT gradient [B][H][W][C] (see
  // EpiPoolScatterBF16; H >= PH*KH, W >= PW*KW: floor windows)
  EpiPoolScatterBF16 eP{(bf16_raw*)dx, pool_am, (const bf16_raw*)pool_x, pool ? pool[5] : 0, pool_rng, pool_salt,
                        pool_p, K, pool ? pool[0] : 1, pool ? pool[2] : 1, pool ? pool[3] : 1, pool ? pool[4] : 1,
                        pool ? pool[6] : 1, pool ? pool[7] : 1, nullptr, pool ? pool[1] : 1};
  if (pool && (pool[6] < pool[1] * pool[3] || pool[7] < pool[2] * pool[4] || pool[6] >= (pool[1] + 1) * pool[3] ||
               pool[7] >= (pool[2] + 1) * pool[4]))
    return -3;
  if (pool && pool[0] * pool[1] * pool[2] != K) return -2;
  DenseLoader aB{(const bf16_raw*)dy, N, is_vec_ok(dy, N) && is_vec_ok(ay ? ay : dy, N), (const bf16_raw*)ay, aact};
  DenseLoader bB{(const bf16_raw*)x, K, is_vec_ok(x, K)};
  EpiAtomicF32 eB{dw, K, 1.f, nullptr};
  // the only contribution to a zeroed dW and no K split: plain stores (see ops_api.h)
  const bool store = dw_store && gyB == 1 && !hopsx_disabled("dw_store");
  EpiStoreF32 eS{dw, K, nullptr, 1.f, 0.f, 0, nullptr};
#define HOPSX_LP2(A_, B_, EPA_, ea_)                                                                               \
  if (store)                                                                                                       \
    hipLaunchKernelGGL((linear_bwd_pair_k<A_, B_, EPA_, EpiStoreF32>), dim3((unsigned)total), dim3(256), 0, st, aA, \
                       bA, ea_, M, K, N, pa.kps, gxA, gyA, aB, bB, eS, N, K, M, pb.kps, gxB, gyB, dbias);           \
  else                                                                                                             \
    hipLaunchKernelGGL((linear_bwd_pair_k<A_, B_, EPA_, EpiAtomicF32>), dim3((unsigned)total), dim3(256), 0, st,    \
                       aA, bA, ea_, M, K, N, pa.kps, gxA, gyA, aB, bB, eB, N, K, M, pb.kps, gxB, gyB, dbias);
#define HOPSX_LP(A_, B_)                                   \
  if (bma == A_ && bmb == B_) {                            \
    if (pool) {                                            \
      HOPSX_LP2(A_, B_, EpiPoolScatterBF16, eP)            \
    } else {                                               \
      HOPSX_LP2(A_, B_, EpiDActBF16, eA)                   \
    }                                                      \
    return (int)hipGetLastError();                         \
  }
  HOPSX_LP(32, 32) HOPSX_LP(32, 64) HOPSX_LP(32, 128) HOPSX_LP(64, 32) HOPSX_LP(64, 64) HOPSX_LP(64, 128)
  HOPSX_LP(128, 32) HOPSX_LP(128, 64) HOPSX_LP(128, 128)
#undef HOPSX_LP
#undef HOPSX_LP2
  return -2;
}
