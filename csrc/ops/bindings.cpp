// pybind11 module `_hopsx_ops`: thin bindings of the C ABI in ops_api.h.
// Device pointers and the hipStream_t arrive as Python ints (tensor.data_ptr(),
// torch.cuda.current_stream().cuda_stream); shape/dtype validation lives in
// hops_examples_amd/ops/_C.py so this layer stays a zero-cost trampoline.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#if defined(HOPSX_DEBUG) && HOPSX_DEBUG
#define HOPSX_DEBUG_BUILD 1
#else
#define HOPSX_DEBUG_BUILD 0
#endif

#include "ops_api.h"
extern "C" int hopsx_mnist_persist_occupancy(int dp);  // mnist_persist.hip
extern "C" void hopsx_mnist_persist_reload_knobs();     // mnist_persist.hip
extern "C" int hopsx_pad_cin(const float* w, long R, int C, int cp, float* out, void* out16, hipStream_t st);
extern "C" int hopsx_unpad_cin_add(float* gpad, long R, int C, int cp, float* tgt, hipStream_t st);  // elementwise.hip

namespace py = pybind11;
extern "C" void hopsx_mlp_head_debug(void* p);
// conv_mfma.hip: the conv backward pair + a fused optimizer's arena-slice update (optim_slice.h)
extern "C" int hopsx_conv2d_bwd_pair_opt(const void* dy, const void* w, const int* geom, void* dx, const void* yprev,
                                         int act_prev, float* colsum, const void* y, int yact, const int* geom0,
                                         const void* x0, float xscale, float xshift, float* dw0, const void* x,
                                         float* dw, float* dbias, const void* addend, int kind, float* p, float* g,
                                         float* s1, float* s2, float* s3, void* shadow, long n, const float* f,
                                         const float* hp_dev, const float* step_dev, int nblk, int opt_first,
                                         hipStream_t st);  // loss.hip: phase stamps (tools/dbg_mlp_head.py)
using u = uintptr_t;

template <class T>
static inline T* P(u p) {
  return reinterpret_cast<T*>(p);
}
static inline hipStream_t S(u s) { return reinterpret_cast<hipStream_t>(s); }

// deterministic mode: one flag per kernel translation unit (common.h HOPSX_DET_TU)
extern "C" int hopsx_det_set_conv_mfma(int);
extern "C" unsigned hopsx_det_lost_conv_mfma();
extern "C" int hopsx_det_set_loss(int);
extern "C" unsigned hopsx_det_lost_loss();
extern "C" int hopsx_det_set_gemm(int);
extern "C" unsigned hopsx_det_lost_gemm();
extern "C" int hopsx_det_set_norm(int);
extern "C" unsigned hopsx_det_lost_norm();
extern "C" int hopsx_det_set_pool(int);
extern "C" unsigned hopsx_det_lost_pool();
extern "C" int hopsx_det_set_conv(int);
extern "C" unsigned hopsx_det_lost_conv();
extern "C" int hopsx_det_set_elementwise(int);
extern "C" unsigned hopsx_det_lost_elementwise();
extern "C" int hopsx_det_set_rowreduce(int);
extern "C" unsigned hopsx_det_lost_rowreduce();
extern "C" int hopsx_det_set_wgrad_glds(int);
extern "C" unsigned hopsx_det_lost_wgrad_glds();

extern "C" int hopsx_dbg_read_conv_mfma(unsigned* out);
extern "C" int hopsx_dbg_read_loss(unsigned* out);
extern "C" int hopsx_dbg_read_gemm(unsigned* out);
extern "C" int hopsx_dbg_read_norm(unsigned* out);
extern "C" int hopsx_dbg_read_pool(unsigned* out);
extern "C" int hopsx_dbg_read_conv(unsigned* out);
extern "C" int hopsx_dbg_read_elementwise(unsigned* out);
extern "C" int hopsx_dbg_read_rowreduce(unsigned* out);
extern "C" int hopsx_dbg_read_wgrad_glds(unsigned* out);
extern "C" int hopsx_dbg_read_embedding(unsigned* out);

// the debug build (-DHOPSX_DEBUG=1) is the module _hopsx_ops_dbg (same sources, hx_check compiled in)
#ifndef HOPSX_MODNAME
#define HOPSX_MODNAME _hopsx_ops
#endif
#define HX_PYMOD(name) PYBIND11_MODULE(name, m)
HX_PYMOD(HOPSX_MODNAME) {
  m.doc() = "hopsx CDNA4 (gfx950) HIP kernel library";
  m.attr("ARCH") = "gfx950";

  m.def("gemm", [](u A, long lda, int akc, u B, long ldb, int bkc, int M, int N, int K, int epi, u out, long ldo,
                   u bias, float alpha, float beta, int act, u aux, long ldaux, u colsum, u ws, long ws_elems, u ay,
                   int aact, u arowsum, u tickets, u st) {
    return hopsx_gemm(P<void>(A), lda, akc, P<void>(B), ldb, bkc, M, N, K, epi, P<void>(out), ldo, P<float>(bias),
                      alpha, beta, act, P<void>(aux), ldaux, P<float>(colsum), P<float>(ws), ws_elems, P<void>(ay), aact,
                      P<float>(arowsum), P<unsigned>(tickets), S(st));
  });
  m.def("conv2d_fwd", [](u x, u w, std::vector<int> g, int epi, u out, u bias, int act, u colsum, float xscale,
                         float xshift, u st) {
    return hopsx_conv2d_fwd(P<void>(x), P<void>(w), g.data(), epi, P<void>(out), P<float>(bias), act,
                            P<float>(colsum), xscale, xshift, S(st));
  });
  m.def("conv2d_dgrad", [](u dy, u w, std::vector<int> g, u dx, u yprev, int act, u colsum, u y, int yact, u addend,
                           u st) {
    return hopsx_conv2d_dgrad(P<void>(dy), P<void>(w), g.data(), P<void>(dx), P<void>(yprev), act, P<float>(colsum),
                              P<void>(y), yact, P<void>(addend), S(st));
  });
  m.def("widedeep_slots", [](std::vector<long> iv, u out, long n) {
    return hopsx_widedeep_slots(iv.data(), (int)iv.size(), P<int>(out), n);
  });
  m.def("taxi_step2_ok", [](std::vector<long> iv, long rows) { return hopsx_taxi_step2_ok(iv.data(), (int)iv.size(), rows); });
  m.def("taxi_step2_xgeom", []() {
    std::vector<long> g(4);
    hopsx_taxi_step2_xgeom(g.data());
    return g;
  });
  m.def("taxi_step2", [](std::vector<uint64_t> p, std::vector<long> iv, std::vector<float> fv, long rows, u st) {
    return hopsx_taxi_step2(p.data(), (int)p.size(), iv.data(), (int)iv.size(), fv.data(), (int)fv.size(), rows, S(st));
  });
  // launch-argument slots of the v2 taxi step (models/widedeep.py _launch), as mnist_persist_store below
  struct TaxiSlot {
    std::vector<uint64_t> p;
    std::vector<long> iv;
    std::vector<float> fv;
    long rows;
  };
  static std::vector<TaxiSlot> taxi_slots;
  m.def("taxi_step2_store", [](int slot, std::vector<uint64_t> p, std::vector<long> iv, std::vector<float> fv, long rows) {
    if (slot < 0 || slot >= (int)taxi_slots.size()) {
      taxi_slots.push_back({});
      slot = (int)taxi_slots.size() - 1;
    }
    taxi_slots[slot] = TaxiSlot{std::move(p), std::move(iv), std::move(fv), rows};
    return slot;
  });
  m.def("taxi_step2_slot", [](int slot, u st) {
    if (slot < 0 || slot >= (int)taxi_slots.size()) return (int)hipErrorInvalidValue;
    const TaxiSlot& a = taxi_slots[slot];
    return hopsx_taxi_step2(a.p.data(), (int)a.p.size(), a.iv.data(), (int)a.iv.size(), a.fv.data(), (int)a.fv.size(),
                            a.rows, S(st));
  });
  m.def("widedeep_step_lds", [](std::vector<long> iv) { return hopsx_widedeep_step_lds(iv.data(), (int)iv.size()); });
  m.def("set_deterministic", [](int on) {
    int e = 0;
    if (!e) e = hopsx_det_set_conv_mfma(on);
    if (!e) e = hopsx_det_set_loss(on);
    if (!e) e = hopsx_det_set_gemm(on);
    if (!e) e = hopsx_det_set_norm(on);
    if (!e) e = hopsx_det_set_pool(on);
    if (!e) e = hopsx_det_set_conv(on);
    if (!e) e = hopsx_det_set_elementwise(on);
    if (!e) e = hopsx_det_set_rowreduce(on);
    if (!e) e = hopsx_det_set_wgrad_glds(on);
    return e;
  });
  m.attr("DEBUG") = HOPSX_DEBUG_BUILD;
  // device-side check records per translation unit: [(tag, failures, line, workgroup, thread)], cleared
  m.def("dbg_read", []() {
    static const std::pair<const char*, int (*)(unsigned*)> tus[] = {
    {"conv_mfma", hopsx_dbg_read_conv_mfma},
    {"loss", hopsx_dbg_read_loss},
    {"gemm", hopsx_dbg_read_gemm},
    {"norm", hopsx_dbg_read_norm},
    {"pool", hopsx_dbg_read_pool},
    {"conv", hopsx_dbg_read_conv},
    {"elementwise", hopsx_dbg_read_elementwise},
    {"rowreduce", hopsx_dbg_read_rowreduce},
    {"wgrad_glds", hopsx_dbg_read_wgrad_glds},
    {"embedding", hopsx_dbg_read_embedding},
    };
    std::vector<std::tuple<std::string, unsigned, unsigned, unsigned, unsigned>> out;
    for (const auto& t : tus) {
      unsigned v[4] = {0u, 0u, 0u, 0u};
      const int e = t.second(v);
      if (e) throw std::runtime_error(std::string("hopsx dbg_read: hip error ") + std::to_string(e));
      if (v[0]) out.emplace_back(t.first, v[0], v[1], v[2], v[3]);
    }
    return out;
  });
  m.def("det_lost", []() {
    unsigned n = 0;
    n += hopsx_det_lost_conv_mfma();
    n += hopsx_det_lost_loss();
    n += hopsx_det_lost_gemm();
    n += hopsx_det_lost_norm();
    n += hopsx_det_lost_pool();
    n += hopsx_det_lost_conv();
    n += hopsx_det_lost_elementwise();
    n += hopsx_det_lost_rowreduce();
    n += hopsx_det_lost_wgrad_glds();
    return n;
  });
  m.def("mnist_persist", [](std::vector<uint64_t> p, std::vector<long> iv, std::vector<float> fv, u st) {
    return hopsx_mnist_persist(p.data(), (int)p.size(), iv.data(), (int)iv.size(), fv.data(), (int)fv.size(),
                               S(st));
  });
  // launch-argument slots of the persistent step (runtime/persist.py): the argument vectors are converted
  // once per change; a launch then crosses the binding with a slot id and the stream only — at bench.py's
  // 20 steps per launch the host path is inside the timed window while the GPU waits
  struct PersistSlot {
    std::vector<uint64_t> p;
    std::vector<long> iv;
    std::vector<float> fv;
  };
  static std::vector<PersistSlot> persist_slots;
  m.def("mnist_persist_store", [](int slot, std::vector<uint64_t> p, std::vector<long> iv, std::vector<float> fv) {
    if (slot < 0 || slot >= (int)persist_slots.size()) {
      persist_slots.push_back({});
      slot = (int)persist_slots.size() - 1;
    }
    persist_slots[slot] = PersistSlot{std::move(p), std::move(iv), std::move(fv)};
    return slot;
  });
  m.def("mnist_persist_slot", [](int slot, u st) {
    if (slot < 0 || slot >= (int)persist_slots.size()) return (int)hipErrorInvalidValue;
    const PersistSlot& a = persist_slots[slot];
    return hopsx_mnist_persist(a.p.data(), (int)a.p.size(), a.iv.data(), (int)a.iv.size(), a.fv.data(),
                               (int)a.fv.size(), S(st));
  });
  m.def("mnist_persist_reload_knobs", []() { hopsx_mnist_persist_reload_knobs(); });
  m.def("mnist_persist_occupancy", [](int dp) { return hopsx_mnist_persist_occupancy(dp); });
  m.def("pad_cin", [](u w, long R, int C, int cp, u out, u out16, u st) {
    return hopsx_pad_cin(P<float>(w), R, C, cp, P<float>(out), P<void>(out16), S(st));
  });
  m.def("unpad_cin_add", [](u g, long R, int C, int cp, u tgt, u st) {
    return hopsx_unpad_cin_add(P<float>(g), R, C, cp, P<float>(tgt), S(st));
  });
  m.def("mnist_persist_geom", []() {
    std::vector<long> g(22);
    hopsx_mnist_persist_geom(g.data());
    return g;
  });
  m.def("widedeep_step", [](std::vector<uint64_t> p, std::vector<long> iv, std::vector<float> fv, u st) {
    return hopsx_widedeep_step(p.data(), (int)p.size(), iv.data(), (int)iv.size(), fv.data(), (int)fv.size(),
                               S(st));
  });
  m.def("conv2d_fwd_pool_ok", [](std::vector<int> g, int act, int pk) { return hopsx_conv_fwd_pool_ok(g.data(), act, pk); });
  m.def("conv2d_fwd_pool", [](u x, u w, std::vector<int> g, u out, u am, u bias, int act, float p, u rng,
                              unsigned salt, int pk, u st) {
    return hopsx_conv2d_fwd_pool(P<void>(x), P<void>(w), g.data(), P<void>(out), P<void>(am), P<float>(bias), act, p,
                                 P<unsigned long long>(rng), salt, pk, S(st));
  });
  m.def("conv2d_fwd_pool_in_ok", [](std::vector<int> g0, std::vector<int> g, int act) {
    return hopsx_conv_fwd_pool_in_ok(g0.data(), g.data(), act);
  });
  m.def("conv2d_fwd_pool_in", [](u x0, float xscale, float xshift, u w0, u b0, int act0, std::vector<int> g0, u y1,
                                 u w, std::vector<int> g, u out, u am, u bias, int act, float p, u rng, unsigned salt,
                                 u st) {
    return hopsx_conv2d_fwd_pool_in(P<void>(x0), xscale, xshift, P<void>(w0), P<float>(b0), act0, g0.data(),
                                    P<void>(y1), P<void>(w), g.data(), P<void>(out), P<void>(am), P<float>(bias), act,
                                    p, P<unsigned long long>(rng), salt, S(st));
  });
  m.def("conv2d_dgrad_fused_wgrad_ok", [](std::vector<int> g, std::vector<int> g0) {
    return hopsx_conv_dgrad_fused_wgrad_ok(g.data(), g0.data());
  });
  m.def("conv2d_dgrad_fused_wgrad", [](u dy, u w, std::vector<int> g, u yprev, int act, u colsum, u y, int yact,
                                       std::vector<int> g0, u x0, float xscale, float xshift, u dw0, u st) {
    return hopsx_conv2d_dgrad_mfma_ex(P<void>(dy), P<void>(w), g.data(), nullptr, P<void>(yprev), act,
                                      P<float>(colsum), P<void>(y), yact, g0.data(), P<void>(x0), xscale, xshift,
                                      P<float>(dw0), S(st));
  });
  m.def("wgrad_debug_times", [](int n) {
    std::vector<unsigned long long> v((size_t)n);
    hopsx_wgrad_debug_times(v.data(), n);
    return v;
  });
  m.def("head_ce_ok", [](int C, int KD) { return hopsx_head_ce_ok(C, KD); });
  m.def("head_ce", [](int kind, u logits, int lf32, u target, int B, int C, int KD, float gs, u h, u w, u dw, u db,
                      u dh, u loss, u correct, u bias, u lout, float dp, u drng, unsigned dsalt, u st) {
    return hopsx_head_ce(kind, P<void>(logits), lf32, P<void>(target), B, C, KD, gs, P<void>(h), P<void>(w),
                         P<float>(dw), P<float>(db), P<void>(dh), P<float>(loss), P<int>(correct), P<float>(bias),
                         P<void>(lout), dp, P<unsigned long long>(drng), dsalt, S(st));
  });
  m.def("mlp_head_debug", [](u p) { hopsx_mlp_head_debug(P<void>(p)); });
  // upload an instantiated hipGraph's executable to the device now (capture time) instead of at its
  // first launch (inside a timed loop / a latency-critical replay)
  m.def("graph_upload", [](u exec, u st) {
    return (int)hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), S(st));
  });
  m.def("mlp_head", [](u x, u w1, u b1, int act1, u y, u ws, u arrive, int B, int K, int N1, int kind, u target,
                       int C, float gs, u w2, u b2, u dw2, u db2, u dh, u loss, u correct, u lout, int lf32, float dp,
                       u drng, unsigned dsalt, u st) {
    return hopsx_mlp_head(P<void>(x), P<void>(w1), P<float>(b1), act1, P<void>(y), P<float>(ws), P<unsigned>(arrive),
                          B, K, N1, kind, P<void>(target), C, gs, P<void>(w2), P<float>(b2), P<float>(dw2),
                          P<float>(db2), P<void>(dh), P<float>(loss), P<int>(correct), P<void>(lout), lf32, dp,
                          P<unsigned long long>(drng), dsalt, S(st));
  });
  m.def("zero", [](u p, long bytes, u st) { return hopsx_zero(P<void>(p), bytes, S(st)); });
  m.def("nonfinite", [](u x, long n, int is_bf16, u out, u st) {
    return hopsx_nonfinite(P<void>(x), n, is_bf16, P<unsigned>(out), S(st));
  });
  m.def("linear_bwd_pair", [](u dy, u w, u x, u dx, u yprev, int act_prev, u colsum, u ay, int aact, u dw, u db,
                              int M, int N, int K, std::vector<int> pool, u pam, u px, u prng, unsigned psalt,
                              float pp, int dw_store, u st) {
    return hopsx_linear_bwd_pair(P<void>(dy), P<void>(w), P<void>(x), P<void>(dx), P<void>(yprev), act_prev,
                                 P<float>(colsum), P<void>(ay), aact, P<float>(dw), P<float>(db), M, N, K,
                                 pool.empty() ? nullptr : pool.data(), P<unsigned char>(pam), P<void>(px),
                                 P<unsigned long long>(prng), psalt, pp, dw_store, S(st));
  });
  m.def("conv2d_bwd_pair", [](u dy, u w, std::vector<int> g, u dx, u yprev, int act, u colsum, u y, int yact,
                              std::vector<int> g0, u x0, float xscale, float xshift, u dw0, u x, u dw, u db, u add,
                              u bnz, u bnmean, u bnrstd, u bnacc, u st) {
    return hopsx_conv2d_bwd_pair(P<void>(dy), P<void>(w), g.data(), P<void>(dx), P<void>(yprev), act,
                                 P<float>(colsum), P<void>(y), yact, g0.empty() ? nullptr : g0.data(), P<void>(x0),
                                 xscale, xshift, P<float>(dw0), P<void>(x), P<float>(dw), P<float>(db), P<void>(add),
                                 P<void>(bnz), P<float>(bnmean), P<float>(bnrstd), P<float>(bnacc), S(st));
  });
  m.def("conv2d_dgrad_bn", [](u dy, u w, std::vector<int> g, u dx, u yprev, int act_prev, u add, u bnz, u bnmean,
                              u bnrstd, u bnacc, u st) {
    return hopsx_conv2d_dgrad_bn(P<void>(dy), P<void>(w), g.data(), P<void>(dx), P<void>(yprev), act_prev, P<void>(add),
                                 P<void>(bnz), P<float>(bnmean), P<float>(bnrstd), P<float>(bnacc), S(st));
  });
  m.def("conv2d_bwd_pair_bn_ok", [](std::vector<int> g) { return hopsx_conv2d_bwd_pair_bn_ok(g.data()); });
  m.def("bn_bwd_pre", [](u dy, u x, u gamma, u mean, u rstd, u dx, u dgamma, u dbeta, u ws, int M, int C, u acc,
                         u st) {
    return hopsx_bn_bwd_pre(P<void>(dy), P<void>(x), P<float>(gamma), P<float>(mean), P<float>(rstd), P<void>(dx),
                            P<float>(dgamma), P<float>(dbeta), P<float>(ws), M, C, P<float>(acc), S(st));
  });
  m.def("conv2d_bwd_pair_opt", [](u dy, u w, std::vector<int> g, u dx, u yprev, int act, u colsum, u y, int yact,
                                  std::vector<int> g0, u x0, float xscale, float xshift, u dw0, u x, u dw, u db, u add,
                                  int kind, u p, u gr, u s1, u s2, u s3, u sh, long n, std::vector<float> f, u hp_dev,
                                  u step_dev, int nblk, int opt_first, u st) {
    if (f.size() < 8) f.resize(8, 0.f);
    return hopsx_conv2d_bwd_pair_opt(P<void>(dy), P<void>(w), g.data(), P<void>(dx), P<void>(yprev), act,
                                     P<float>(colsum), P<void>(y), yact, g0.empty() ? nullptr : g0.data(), P<void>(x0),
                                     xscale, xshift, P<float>(dw0), P<void>(x), P<float>(dw), P<float>(db),
                                     P<void>(add), kind, P<float>(p), P<float>(gr), P<float>(s1), P<float>(s2),
                                     P<float>(s3), P<void>(sh), n, f.data(), P<float>(hp_dev), P<float>(step_dev), nblk,
                                     opt_first, S(st));
  });
  m.def("conv2d_wgrad", [](u dy, u x, std::vector<int> g, u dw, u db, u y, int yact, u ws, long ws_elems,
                           float xscale, float xshift, u counter, u st) {
    return hopsx_conv2d_wgrad(P<void>(dy), P<void>(x), g.data(), P<float>(dw), P<float>(db), P<void>(y), yact,
                              P<float>(ws), ws_elems, xscale, xshift, P<unsigned>(counter), S(st));
  });
  m.def("conv2d_wgrad_glds", [](u dy, u x, std::vector<int> g, u dw, int force, u st) {
    return hopsx_conv2d_wgrad_glds(P<void>(dy), P<void>(x), g.data(), P<float>(dw), force, S(st));
  });
  m.def("conv_wgrad_glds_ok", [](std::vector<int> g) { return hopsx_conv_wgrad_glds_ok(g.data()); });
  m.def("cols_to_f32", [](std::vector<u> cols, std::vector<int> dtypes, long rows, u out, long ld, u st) {
    std::vector<const void*> cp(cols.size());
    for (size_t j = 0; j < cols.size(); ++j) cp[j] = P<void>(cols[j]);
    if (dtypes.size() != cols.size()) return -2;
    return hopsx_cols_to_f32(cp.data(), dtypes.data(), (int)cols.size(), rows, P<float>(out), ld, S(st));
  });
  m.def("maxpool2d_fwd", [](u x, u y, u am, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int sh,
                            int sw, int ph, int pw, float p, u rng, unsigned salt, u st) {
    return hopsx_maxpool2d_fwd(P<void>(x), P<void>(y), P<unsigned char>(am), B, H, W, C, OH, OW, KH, KW, sh, sw, ph,
                               pw, p, P<unsigned long long>(rng), salt, S(st));
  });
  m.def("maxpool2d_bwd", [](u dy, u am, u x, u dx, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int sh,
                            int sw, int ph, int pw, int act, u colsum, float p, u rng, unsigned salt, u st) {
    return hopsx_maxpool2d_bwd(P<void>(dy), P<unsigned char>(am), P<void>(x), P<void>(dx), B, H, W, C, OH, OW, KH, KW,
                               sh, sw, ph, pw, act, P<float>(colsum), p, P<unsigned long long>(rng), salt, S(st));
  });
  m.def("avgpool_global_fwd", [](u x, u y, int B, int HW, int C, u st) {
    return hopsx_avgpool_global_fwd(P<void>(x), P<void>(y), B, HW, C, S(st));
  });
  m.def("avgpool_global_bwd", [](u dy, u dx, int B, int HW, int C, u st) {
    return hopsx_avgpool_global_bwd(P<void>(dy), P<void>(dx), B, HW, C, S(st));
  });
  m.def("loss_fwd_bwd", [](int kind, u logits, int lf32, u target, int B, int C, float gscale, u loss_sum, u correct,
                           u dl, int df32, u st) {
    return hopsx_loss_fwd_bwd(kind, P<void>(logits), lf32, P<void>(target), B, C, gscale, P<float>(loss_sum),
                              P<int>(correct), P<void>(dl), df32, S(st));
  });
  m.def("optim_step", [](int kind, u p, u g, u s1, u s2, u s3, u shadow, long n, std::vector<float> hp, u step,
                         u arrive, u rng, int zero_grad, std::vector<u> pf_src, std::vector<u> pf_dst,
                         std::vector<long> pf_bytes, u pf_cursor, int pf_nbatch, u hp_dev, u st) {
    const void* srcs[2] = {nullptr, nullptr};
    void* dsts[2] = {nullptr, nullptr};
    long bytes[2] = {0, 0};
    const int nj = (int)std::min<size_t>(2, std::min(pf_src.size(), std::min(pf_dst.size(), pf_bytes.size())));
    for (int j = 0; j < nj; ++j) {
      srcs[j] = P<void>(pf_src[j]);
      dsts[j] = P<void>(pf_dst[j]);
      bytes[j] = pf_bytes[j];
    }
    return hopsx_optim_step(kind, P<float>(p), P<float>(g), P<float>(s1), P<float>(s2), P<float>(s3),
                            P<void>(shadow), n, hp.data(), (int)hp.size(), P<float>(step), P<unsigned>(arrive),
                            P<unsigned long long>(rng), zero_grad, srcs, dsts, bytes, nj, P<long long>(pf_cursor),
                            pf_nbatch, P<float>(hp_dev), S(st));
  });
  m.def("dropout_fwd", [](u x, u y, long n, float p, u rng, unsigned salt, u st) {
    return hopsx_dropout_fwd(P<void>(x), P<void>(y), n, p, P<unsigned long long>(rng), salt, S(st));
  });
  m.def("dropout_bwd", [](u dy, u dx, long n, float p, u rng, unsigned salt, u st) {
    return hopsx_dropout_bwd(P<void>(dy), P<void>(dx), n, p, P<unsigned long long>(rng), salt, S(st));
  });
  m.def("rng_advance", [](u rng, u st) { return hopsx_rng_advance(P<unsigned long long>(rng), S(st)); });
  m.def("cast_f32_bf16", [](u x, u y, long n, u st) { return hopsx_cast_f32_bf16(P<float>(x), P<void>(y), n, S(st)); });
  m.def("cast_bf16_f32", [](u x, u y, long n, u st) { return hopsx_cast_bf16_f32(P<void>(x), P<float>(y), n, S(st)); });
  m.def("u8_normalize", [](u x, u y, long n, float scale, float shift, u st) {
    return hopsx_u8_normalize(P<unsigned char>(x), P<void>(y), n, scale, shift, S(st));
  });
  m.def("colsum_bf16", [](u x, u out, int M, int N, u st) {
    return hopsx_colsum_bf16(P<void>(x), P<float>(out), M, N, S(st));
  });
  m.def("act_bwd", [](u dy, u y, u dx, long n, int act, u st) {
    return hopsx_act_bwd(P<void>(dy), P<void>(y), P<void>(dx), n, act, S(st));
  });
  m.def("act_bwd_colsum", [](u dy, u y, u dx, int M, int N, int act, u colsum, u st) {
    return hopsx_act_bwd_colsum(P<void>(dy), P<void>(y), P<void>(dx), M, N, act, P<float>(colsum), S(st));
  });
  m.def("add_bf16", [](u a, u b, u o, long n, int act, u st) {
    return hopsx_add_bf16(P<void>(a), P<void>(b), P<void>(o), n, act, S(st));
  });
  m.def("bn_fwd_train", [](u x, u y, u g, u b, u mean, u rstd, u rm, u rv, float mom, float eps, int M, int C, u res,
                           int act, u acc, u st) {
    return hopsx_bn_fwd_train(P<void>(x), P<void>(y), P<float>(g), P<float>(b), P<float>(mean), P<float>(rstd),
                              P<float>(rm), P<float>(rv), mom, eps, M, C, P<void>(res), act, P<float>(acc), S(st));
  });
  m.def("bn_fwd_apply_fin", [](u x, u y, u g, u b, u mean, u rstd, u rm, u rv, float mom, float eps, int M, int C,
                               u res, int act, u acc, u st) {
    return hopsx_bn_fwd_apply_fin(P<void>(x), P<void>(y), P<float>(g), P<float>(b), P<float>(mean), P<float>(rstd),
                                  P<float>(rm), P<float>(rv), mom, eps, M, C, P<void>(res), act, P<float>(acc), S(st));
  });
  m.def("bn_prestats_ok", [](int C) { return hopsx_bn_prestats_ok(C); });
  m.def("bn_coop_timeouts", [](u acc, int C) { return hopsx_bn_coop_timeouts(P<float>(acc), C); });
  m.def("conv2d_fwd_bnstats", [](u x, u w, std::vector<int> g, u out, u acc, u st) {
    return hopsx_conv2d_fwd_bnstats(P<void>(x), P<void>(w), g.data(), P<void>(out), P<float>(acc), S(st));
  });
  m.def("conv2d_fwd_bnstats_inbn", [](u z, u a, u w, std::vector<int> g, u out, u acc, u inacc, u gm, u bt, u mean,
                                      u rstd, u rm, u rv, float mom, float eps, int act, u st) {
    return hopsx_conv2d_fwd_bnstats_inbn(P<void>(z), P<void>(a), P<void>(w), g.data(), P<void>(out), P<float>(acc),
                                         P<float>(inacc), P<float>(gm), P<float>(bt), P<float>(mean), P<float>(rstd),
                                         P<float>(rm), P<float>(rv), mom, eps, act, S(st));
  });
  m.def("bn_fwd_infer", [](u x, u y, u g, u b, u rm, u rv, float eps, int M, int C, u res, int act, u st) {
    return hopsx_bn_fwd_infer(P<void>(x), P<void>(y), P<float>(g), P<float>(b), P<float>(rm), P<float>(rv), eps, M, C,
                              P<void>(res), act, S(st));
  });
  m.def("bn_bwd", [](u dy, u x, u y, u g, u mean, u rstd, u dx, u dg, u db, u ws, int M, int C, int act, u dres,
                     u acc, u zbeta, u st) {
    return hopsx_bn_bwd(P<void>(dy), P<void>(x), P<void>(y), P<float>(g), P<float>(mean), P<float>(rstd), P<void>(dx),
                        P<float>(dg), P<float>(db), P<float>(ws), M, C, act, P<void>(dres), P<float>(acc),
                        P<float>(zbeta), S(st));
  });
  m.def("embedding_bag_fwd", [](u table, u idx, u offs, int nbags, int dim, long nidx, int bag_len, int mode, u out,
                                int of32, long ldo, long rows, u st) {
    return hopsx_embedding_bag_fwd(P<float>(table), P<long>(idx), P<long>(offs), nbags, dim, nidx, bag_len, mode,
                                   P<void>(out), of32, ldo, rows, S(st));
  });
  m.def("embedding_bag_bwd", [](u dout, int df32, long ldo, u idx, u offs, int nbags, int dim, long nidx,
                                int bag_len, int mode, u dtable, long rows, u st) {
    return hopsx_embedding_bag_bwd(P<void>(dout), df32, ldo, P<long>(idx), P<long>(offs), nbags, dim, nidx, bag_len,
                                   mode, P<float>(dtable), rows, S(st));
  });
  m.def("column_stats", [](u x, int rows, int cols, u out, u st) {
    return hopsx_column_stats(P<float>(x), rows, cols, P<float>(out), S(st));
  });
  m.def("column_hist", [](u x, int rows, int cols, u mins, u maxs, int bins, u hist, u st) {
    return hopsx_column_hist(P<float>(x), rows, cols, P<float>(mins), P<float>(maxs), bins, P<unsigned>(hist), S(st));
  });
  m.def("gram", [](u x, u mean, int rows, int cols, u gram, u st) {
    return hopsx_gram(P<float>(x), P<float>(mean), rows, cols, P<float>(gram), S(st));
  });
  m.def("taxi_transform", [](u raw, u vids, long n, std::vector<int> ints, std::vector<float> flts,
                             std::vector<long> offs, u dense, u cat, u label, u st) {
    return hopsx_taxi_transform(P<float>(raw), P<int>(vids), n, ints.data(), flts.data(), offs.data(), P<float>(dense),
                                P<long>(cat), P<float>(label), S(st));
  });
  m.def("transform_max_bounds", []() { return hopsx_transform_max_bounds(); });
  m.def("prefix_sum_f64", [](u v, long n, u pref, u work, u st) {
    return hopsx_prefix_sum_f64(P<double>(v), n, P<double>(pref), P<double>(work), S(st));
  });
  m.def("range_window", [](u ts, u seg, u seg_off, u pref, long n, u lo, u hi, int W, u sum, u cnt, u st) {
    return hopsx_range_window(P<long>(ts), P<int>(seg), P<long>(seg_off), P<double>(pref), n, P<long>(lo), P<long>(hi), W,
                              P<double>(sum), P<int>(cnt), S(st));
  });
  m.def("column_stats64", [](u x, int rows, int cols, u out, u st) {
    return hopsx_column_stats64(P<double>(x), rows, cols, P<double>(out), S(st));
  });
  m.def("u8_normalize_chan", [](u x, u y, long pixels, int C, std::vector<float> scale, std::vector<float> shift,
                                int rev, int cout, u st) {
    if ((int)scale.size() < C || (int)shift.size() < C) return -2;
    return hopsx_u8_normalize_chan(P<unsigned char>(x), P<void>(y), pixels, C, scale.data(), shift.data(), rev, cout,
                                   S(st));
  });
}
