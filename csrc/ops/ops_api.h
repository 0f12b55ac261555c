// C ABI of the hopsx CDNA4 kernel library.  Every entry point takes raw device
// pointers plus the hipStream_t to launch on (PyTorch's current stream), never
// allocates, never synchronises — so whole training steps that call them can
// be captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>

enum GemmEpi : int { EPI_STORE_BF16 = 0, EPI_STORE_F32 = 1, EPI_ATOMIC_F32 = 2, EPI_DACT_BF16 = 3 };

extern "C" {
// ---- GEMM / conv (gemm.hip, conv.hip) ----
int hopsx_gemm(const void* A, long lda, int a_kc, const void* B, long ldb, int b_kc, int M, int N, int K, int epi,
               void* out, long ldo, const float* bias, float alpha, float beta, int act, const void* aux, long ldaux,
               float* colsum, float* ws, long ws_elems, const void* ay, int aact, float* arowsum, unsigned* tickets,
               hipStream_t st);
// xscale != 0: x is uint8 and is read as x * xscale + xshift (input-layer normalisation fused; direct kernel only)
// a Linear layer's dgrad + wgrad (+ bias grad) in one launch; -2: unsupported shape (gemm.hip)
// pool (optional) = {C, PH, PW, KH, KW, act}: x came from a non-overlapping max-pool and dx is the
// POOL INPUT gradient, scattered by the dgrad epilogue (pool_am argmax, pool_x for ReL', dropout p)
// dw_store: dW is this step's only contribution to a zeroed gradient -> plain stores instead of
// float atomics when K is not split (atomics run at the memory side at ~1.3 TB/s, stores ~6 TB/s)
int hopsx_linear_bwd_pair(const void* dy, const void* w, const void* x, void* dx, const void* yprev, int act_prev,
                          float* colsum, const void* ay, int aact, float* dw, float* dbias, int M, int N, int K,
                          const int* pool, const unsigned char* pool_am, const void* pool_x,
                          const unsigned long long* pool_rng, unsigned pool_salt, float pool_p, int dw_store,
                          hipStream_t st);
int hopsx_conv2d_fwd(const void* x, const void* w, const int* geom, int epi, void* out, const float* bias, int act,
                     float* colsum, float xscale, float xshift, hipStream_t st);
// y/yact: this conv's activation output -> fused act' mask on dY (prologue fusion)
int hopsx_conv2d_dgrad(const void* dy, const void* w, const int* geom, void* dx, const void* yprev, int act,
                       float* colsum, const void* y, int yact, const void* addend, hipStream_t st);
// dbias (optional) receives sum over pixels of the (masked) dY = the conv bias gradient
// ws (optional, >= 1024*(K*CO+CO) floats): slab workspace for the small-K direct kernel
int hopsx_conv2d_wgrad(const void* dy, const void* x, const int* geom, float* dw, float* dbias, const void* y,
                       int yact, float* ws, long ws_elems, float xscale, float xshift, unsigned* counter,
                       hipStream_t st);

// ---- pooling (pool.hip) ----
// optional fused dropout on the pooled output (p > 0, rng/salt as hopsx_dropout_fwd)
int hopsx_maxpool2d_fwd(const void* x, void* y, unsigned char* argmax, int B, int H, int W, int C, int OH, int OW,
                        int KH, int KW, int sh, int sw, int ph, int pw, float p, const unsigned long long* rng,
                        unsigned salt, hipStream_t st);
int hopsx_maxpool2d_bwd(const void* dy, const unsigned char* argmax, const void* x, void* dx, int B, int H, int W,
                        int C, int OH, int OW, int KH, int KW, int sh, int sw, int ph, int pw, int act,
                        float* colsum, float p, const unsigned long long* rng, unsigned salt, hipStream_t st);
int hopsx_avgpool_global_fwd(const void* x, void* y, int B, int HW, int C, hipStream_t st);
int hopsx_avgpool_global_bwd(const void* dy, void* dx, int B, int HW, int C, hipStream_t st);

// ---- losses (loss.hip) ----
// kind: 0 softmax cross-entropy (int labels), 1 softmax CE (dense/one-hot targets),
//       2 sigmoid BCE from logits, 3 MSE, 4 BCE on probabilities
// fused classifier head: loss + dlogits (in LDS) + head wgrad/bias grad + input gradient (loss.hip)
bool hopsx_head_ce_ok(int C, int KD);
int hopsx_head_ce(int kind, const void* logits, int logits_f32, const void* target, int B, int C, int KD,
                  float grad_scale, const void* h, const void* w, float* dw, float* db, void* dh, float* loss_sum,
                  int* correct, const float* bias, void* logits_out, float drop_p,
                  const unsigned long long* drop_rng, unsigned drop_salt, hipStream_t st);
// (drop_p > 0: h is the input of a Dropout feeding the head, applied inside with dropout_k's mask; dh is then
// the gradient of that input)
// fused last hidden Dense + head (loss.hip mlp_head_k): y = act(x W1^T + b1) stored, then head_ce from
// LDS; ws fp32 [B][N1] and arrive (kArriveWords) persistent, zero at rest.  -2: shape not supported
int hopsx_mlp_head(const void* x, const void* w1, const float* b1, int act1, void* y, float* ws, unsigned* arrive,
                   int B, int K, int N1, int kind, const void* target, int C, float grad_scale, const void* w2,
                   const float* b2, float* dw2, float* db2, void* dh, float* loss_sum, int* correct,
                   void* logits_out, int logits_f32, float drop_p, const unsigned long long* drop_rng,
                   unsigned drop_salt, hipStream_t st);
int hopsx_loss_fwd_bwd(int kind, const void* logits, int logits_f32, const void* target, int B, int C,
                       float grad_scale, float* loss_sum, int* correct, void* dlogits, int dlogits_f32,
                       hipStream_t st);

// ---- optimizers (optim.hip) ----
// kind: 0 SGD(momentum/nesterov), 1 Adam, 2 AdamW, 3 Adadelta, 4 RMSprop, 5 Adagrad, 6 FTRL
// pf_*: optional fused prefetch of the next batch of up to two HBM-resident tensors (see optim.hip)
// hp_dev: optional device copy of the 8 hyper-parameters (read at run time; overrides hp)
int hopsx_optim_step(int kind, float* param, float* grad, float* s1, float* s2, float* s3, void* shadow_bf16,
                     long n, const float* hp, int nhp, float* step_dev, unsigned* arrive, unsigned long long* rng,
                     int zero_grad, const void* const* pf_src, void* const* pf_dst, const long* pf_bytes,
                     int pf_njobs, long long* pf_cursor, int pf_nbatch, const float* hp_dev, hipStream_t st);

// ---- dropout / RNG (elementwise.hip) ----
int hopsx_dropout_fwd(const void* x, void* y, long n, float p, const unsigned long long* rng, unsigned salt,
                      hipStream_t st);
int hopsx_dropout_bwd(const void* dy, void* dx, long n, float p, const unsigned long long* rng, unsigned salt,
                      hipStream_t st);
int hopsx_rng_advance(unsigned long long* rng, hipStream_t st);

// ---- elementwise / reductions (elementwise.hip) ----
int hopsx_cast_f32_bf16(const float* x, void* y, long n, hipStream_t st);
int hopsx_cast_bf16_f32(const void* x, float* y, long n, hipStream_t st);
int hopsx_u8_normalize(const unsigned char* x, void* y, long n, float scale, float shift, hipStream_t st);
int hopsx_colsum_bf16(const void* x, float* out, int M, int N, hipStream_t st);
int hopsx_act_bwd(const void* dy, const void* y, void* dx, long n, int act, hipStream_t st);
int hopsx_act_bwd_colsum(const void* dy, const void* y, void* dx, int M, int N, int act, float* colsum,
                         hipStream_t st);
int hopsx_add_bf16(const void* a, const void* b, void* out, long n, int act, hipStream_t st);

// ---- batch norm (norm.hip), NHWC, per-channel over M = B*H*W rows ----
int hopsx_bn_fwd_train(const void* x, void* y, const float* gamma, const float* beta, float* mean_out,
                       float* rstd_out, float* running_mean, float* running_var, float momentum, float eps, int M,
                       int C, const void* residual, int act, float* acc, hipStream_t st);
int hopsx_bn_fwd_infer(const void* x, void* y, const float* gamma, const float* beta, const float* running_mean,
                       const float* running_var, float eps, int M, int C, const void* residual, int act,
                       hipStream_t st);
int hopsx_bn_bwd(const void* dy, const void* x, const void* y, const float* gamma, const float* mean,
                 const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int C, int act,
                 void* dresidual, float* acc, const float* zbeta, hipStream_t st);

// ---- direct MFMA convs for short reductions (conv_mfma.hip) ----
// ---- whole wide&deep training step in one workgroup (widedeep_step.hip) ----
long hopsx_widedeep_step_lds(const long* iv, int ni);
int hopsx_widedeep_slots(const long* iv, int ni, int* out, long n);
int hopsx_widedeep_step(const uint64_t* ptrs, int np, const long* iv, int ni, const float* fv, int nf,
                        hipStream_t st);
// ---- taxi step v2: bf16 MFMA, LDS-resident model + wide table, optimizer state in registers (taxi_step.hip) ----
long hopsx_taxi_step2_ok(const long* iv, int ni, long rows);
void hopsx_taxi_step2_xgeom(long* g);
int hopsx_taxi_step2(const uint64_t* ptrs, int np, const long* iv, int ni, const float* fv, int nf, long rows,
                     hipStream_t st);
// ---- flagship MNIST CNN: nsteps whole training steps in one persistent launch (mnist_persist.hip) ----
int hopsx_mnist_persist(const uint64_t* ptrs, int np, const long* iv, int ni, const float* fv, int nf,
                        hipStream_t st);
void hopsx_mnist_persist_geom(long* g);

bool hopsx_conv_fwd_mfma_ok(const int* geom);
bool hopsx_conv_fwd_pool_ok(const int* geom, int act, int pk);
bool hopsx_conv_fwd_pool_in_ok(const int* geom0, const int* geom, int act);
int hopsx_conv2d_fwd_pool_in(const void* x0, float xscale, float xshift, const void* w0, const float* b0, int act0,
                             const int* geom0, void* y1, const void* w, const int* geom, void* out, void* am,
                             const float* bias, int act, float p, const unsigned long long* rng, unsigned salt,
                             hipStream_t st);
// pk = 2 or 4: a pk x pk / stride-pk max-pool with floor windows
int hopsx_conv2d_fwd_pool(const void* x, const void* w, const int* geom, void* out, void* am, const float* bias, int act,
                          float p, const unsigned long long* rng, unsigned salt, int pk, hipStream_t st);
bool hopsx_conv_dgrad_mfma_ok(const int* geom);
int hopsx_conv2d_fwd_mfma(const void* x, const void* w, const int* geom, void* out, const float* bias, int act,
                          hipStream_t st);
int hopsx_conv2d_fwd_mfma_ex(const void* x, const void* w, const int* geom, void* out, const float* bias, int act,
                             float* bnacc, hipStream_t st);
// conv forward (bf16 out, no bias / act) whose epilogue also accumulates the BatchNorm statistics
// of its output into bnacc [HOPSX_BN_NREP][2 CO] (zero at rest; hopsx_bn_fwd_apply_fin consumes and
// re-zeroes it).  -2: not supported for this shape (nothing launched; use the plain BN path).
int hopsx_conv2d_fwd_bnstats(const void* x, const void* w, const int* geom, void* out, float* bnacc, hipStream_t st);
// the same, with the input a = act(bn(z)) of a training BatchNorm (statistics in inacc, from z's producing
// conv) applied inside the operand gather instead of by hopsx_bn_fwd_apply_fin: writes a (for the
// backward), mean / rstd / the running statistics, re-zeroes inacc.  -2: not supported (nothing launched).
int hopsx_conv2d_fwd_bnstats_inbn(const void* z, void* a, const void* w, const int* geom, void* out, float* bnacc,
                                  float* inacc, const float* gamma, const float* beta, float* mean_out,
                                  float* rstd_out, float* rmean, float* rvar, float momentum, float eps, int act,
                                  hipStream_t st);
int hopsx_conv2d_fwd_mfma_inbn(const void* z, void* a, const void* w, const int* geom, void* out, float* bnacc,
                               float* inacc, const float* gamma, const float* beta, float* mean_out, float* rstd_out,
                               float* rmean, float* rvar, float momentum, float eps, int act, hipStream_t st);
int hopsx_bn_fwd_apply_fin(const void* x, void* y, const float* gamma, const float* beta, float* mean_out,
                           float* rstd_out, float* running_mean, float* running_var, float momentum, float eps, int M,
                           int C, const void* residual, int act, float* acc, hipStream_t st);
int hopsx_bn_prestats_ok(int C);
int hopsx_bn_coop_timeouts(const float* acc, int C);
int hopsx_conv2d_dgrad_mfma(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                            int act_prev, float* colsum, const void* y, int yact, hipStream_t st);
// dgrad with the input layer's weight gradient fused into the epilogue (geom0: the input layer,
// x0 its raw input, uint8 when xscale != 0; dw0 its [CO0][K0] grad, colsum its bias grad; dx unused)
bool hopsx_conv_wgrad_mfma_ok(const int* geom);
// one launch for dgrad (+ fused input-layer wgrad when geom0) and this layer's wgrad; -2: unsupported,
// -3: `addend` (added to dX in the epilogue) unsupported for this shape — nothing launched
int hopsx_conv2d_bwd_pair(const void* dy, const void* w, const int* geom, void* dx, const void* yprev, int act_prev,
                          float* colsum, const void* y, int yact, const int* geom0, const void* x0, float xscale,
                          float xshift, float* dw0, const void* x, float* dw, float* dbias, const void* addend,
                          const void* bnz, const float* bnmean, const float* bnrstd, float* bnacc, hipStream_t st);
// dgrad with the input BN's backward column sums in the epilogue (conv.hip; -2: shape not covered, nothing
// launched); the _mfma_bn variant is the direct MFMA kernel alone
int hopsx_conv2d_dgrad_bn(const void* dy, const void* w, const int* geom, void* dx, const void* yprev, int act_prev,
                          const void* addend, const void* bnz, const float* bnmean, const float* bnrstd, float* bnacc,
                          hipStream_t st);
int hopsx_conv2d_dgrad_mfma_bn(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                               int act_prev, const void* addend, const void* bnz, const float* bnmean,
                               const float* bnrstd, float* bnacc, hipStream_t st);
// 1 when hopsx_conv2d_bwd_pair takes bnacc (the input BN's backward column sums in the dgrad epilogue)
int hopsx_conv2d_bwd_pair_bn_ok(const int* geom);
// BN backward whose column sums are already in the replica rows of acc (a consumer conv's dgrad
// epilogue, hopsx_conv2d_bwd_pair bnacc) and whose dy is the masked output gradient: one apply launch
int hopsx_bn_bwd_pre(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                     void* dx, float* dgamma, float* dbeta, float* ws, int M, int C, float* acc, hipStream_t st);
int hopsx_wgrad_debug_times(unsigned long long* host_out, int n);
// conv weight gradient through LDS-DMA staged 128x128 MFMA tiles (wgrad_glds.hip): no dY activation
// mask, no bias gradient, C % 8 == 0, CO % 8 == 0; -2: unsupported (nothing launched)
int hopsx_conv_wgrad_glds_ok(const int* geom);
int hopsx_conv2d_wgrad_glds(const void* dy, const void* x, const int* geom, float* dw, int force, hipStream_t st);
int hopsx_conv2d_wgrad_mfma(const void* dy, const void* x, const int* geom, float* dw, float* dbias, const void* y,
                            int yact, hipStream_t st);
bool hopsx_conv_dgrad_fused_wgrad_ok(const int* geom, const int* geom0);
int hopsx_conv2d_dgrad_mfma_ex(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                               int act_prev, float* colsum, const void* y, int yact, const int* geom0,
                               const void* x0, float xscale, float xshift, float* dw0, hipStream_t st);

// ---- zero-fill kernel (elementwise.hip): graph-safe replacement for hipMemsetAsync ----
int hopsx_zero(void* p, long bytes, hipStream_t st);
// NaN / Inf counts of an fp32 or bf16 tensor: out[0] += #NaN, out[1] += #Inf (elementwise.hip)
int hopsx_nonfinite(const void* x, long n, int is_bf16, unsigned* out, hipStream_t st);

// ---- embedding bag (embedding.hip) ----
int hopsx_embedding_bag_fwd(const float* table, const long* idx, const long* offsets, int nbags, int dim,
                            long nidx, int bag_len, int mode, void* out, int out_f32, long ldo, long rows,
                            hipStream_t st);
int hopsx_embedding_bag_bwd(const void* dout, int dout_f32, long ldo, const long* idx, const long* offsets,
                            int nbags, int dim, long nidx, int bag_len, int mode, float* dtable, long rows,
                            hipStream_t st);

// ---- column statistics for the feature store (stats.hip) ----
int hopsx_column_stats(const float* x, int rows, int cols, float* out_stats, hipStream_t st);
int hopsx_column_hist(const float* x, int rows, int cols, const float* mins, const float* maxs, int bins,
                      unsigned* hist, hipStream_t st);
int hopsx_gram(const float* x, const float* mean, int rows, int cols, float* gram, hipStream_t st);

// ---- TFX Transform apply (transform.hip) ----
// raw fp32 [n][F] (NaN = missing), vids int32 [n][nv] host vocabulary ids; see transform.hip for the
// ints / flts / offs layout.  -2: spec out of range
int hopsx_taxi_transform(const float* raw, const int* vids, long n, const int* ints, const float* flts,
                         const long* offs, float* dense, long* cat, float* label, hipStream_t st);
int hopsx_transform_max_bounds();

// ---- range-window aggregates (window.hip) ----
// P[0..n] = exclusive fp64 prefix sum of v; work >= ceil(n / 4096) doubles
int hopsx_prefix_sum_f64(const double* v, long n, double* P, double* work, hipStream_t st);
// rows sorted by (partition, ts); seg[i] = partition of row i, seg_off[s..s+1) its rows; W windows
// [ts + lo[w], ts + hi[w]] -> sum[i][w] (NaN if empty) and cnt[i][w]
int hopsx_range_window(const long* ts, const int* seg, const long* seg_off, const double* P, long n,
                       const long* lo, const long* hi, int W, double* sum, int* cnt, hipStream_t st);
// fp64 column statistics for the validation rules: [cols][7] = count, sum, sumsq, min, max, #>=0, #>0
int hopsx_column_stats64(const double* x, int rows, int cols, double* out_stats, hipStream_t st);
// per-channel uint8 NHWC -> bf16 image normalisation (C <= 4, optional channel reversal)
int hopsx_u8_normalize_chan(const unsigned char* x, void* y, long pixels, int C, const float* scale,
                            const float* shift, int rev, int cout, hipStream_t st);
// columnar chunk -> row-major fp32 [rows][ld] (columns.hip); dtypes: 0 f32 1 f64 2 i64 3 i32 4 i16 5 i8
// 6 u8 7 f16; k <= 16
int hopsx_cols_to_f32(const void* const* cols, const int* dtypes, int k, long rows, float* out, long ld,
                      hipStream_t st);
}
