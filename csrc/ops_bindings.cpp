// Per-layer HIP kernel ops (generic Keras path).  Pointers in, pointers out; shapes,
// dtypes, alignment and contiguity are validated on the Python side
// (distributed_amd/ops/hip.py) before any launch.  Every op is enqueued on the caller's
// stream (torch's current stream), so it is captured by torch.cuda graphs.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>

#include "gemm.h"
#include "kernels_api.h"
#include "damd_common.h"
#include "layer_ops.h"

namespace py = pybind11;

namespace {
template <typename T>
T* P_(uintptr_t p) { return reinterpret_cast<T*>(p); }

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

namespace damd {
hipError_t spin_stamp(long long ticks, int blocks, unsigned long long* out, int slot, hipStream_t s);
}

void register_kernel_ops(py::module_& m) {
  // diagnostics (csrc/kernels/diag.hip): blocks holding their CU for `ticks` x 10 ns
  m.def("spin_stamp", [](long long ticks, int blocks, uintptr_t out, int slot, uintptr_t s) {
    check(damd::spin_stamp(ticks, blocks, P_<unsigned long long>(out), slot, P_<ihipStream_t>(s)), "spin_stamp");
  });
  m.def(
      "gemm",
      [](int amode, int bmode, int epi, int splits, int tile, uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias,
         uintptr_t stats, uintptr_t R, int M, int N, int K, int lda, int ldb, int ldc, std::vector<int> geo, int kc,
         int k_per_split, uintptr_t stream, int kstep, uintptr_t stats_acc, uintptr_t bnx, uintptr_t bnst,
         int stats_reps, std::vector<uintptr_t> bnin_p, std::vector<float> bnin_v, uintptr_t bnin_y, uintptr_t slab,
         uintptr_t tickets) {
        damd::GemmArgs a{};
        a.slab = P_<float>(slab);
        a.tickets = P_<unsigned>(tickets);
        if (!bnin_p.empty()) {  // BN on the input (A_CONV3 forward): [acc, gamma, beta, st, rmean, rvar]
          if (bnin_p.size() != 6 || bnin_v.size() != 4)
            throw std::invalid_argument("bnin: 6 pointers + [count, eps, momentum, reps]");
          a.bnin.acc = P_<const long long>(bnin_p[0]); a.bnin.gamma = P_<const float>(bnin_p[1]);
          a.bnin.beta = P_<const float>(bnin_p[2]); a.bnin.st = P_<float>(bnin_p[3]);
          a.bnin.rmean = P_<float>(bnin_p[4]); a.bnin.rvar = P_<float>(bnin_p[5]);
          a.bnin.count = bnin_v[0]; a.bnin.eps = bnin_v[1]; a.bnin.mom = bnin_v[2]; a.bnin.reps = (int)bnin_v[3];
          a.bnin_y = P_<uint16_t>(bnin_y);
        }
        a.stats_acc = P_<long long>(stats_acc);
        a.stats_reps = stats_reps;
        a.bnx = P_<const uint16_t>(bnx);
        a.bnst = P_<const float>(bnst);
        a.A = P_<const void>(A);
        a.B = P_<const void>(B);
        a.C = P_<void>(C);
        a.bias = P_<const float>(bias);
        a.stats = P_<float>(stats);
        a.R = P_<const void>(R);
        a.M = M; a.N = N; a.K = K;
        a.lda = lda; a.ldb = ldb; a.ldc = ldc;
        if (geo.size() == 9) {
          a.H = geo[0]; a.W = geo[1]; a.Cin = geo[2]; a.Ho = geo[3]; a.Wo = geo[4];
          a.KH = geo[5]; a.KW = geo[6]; a.stride = geo[7]; a.pad = geo[8];
        } else if (!geo.empty()) {
          throw std::invalid_argument("geo must be [H, W, C, Ho, Wo, KH, KW, stride, pad]");
        }
        a.kc = kc;
        a.k_per_split = k_per_split;
        a.kstep = kstep;
        check(damd::gemm_launch(a, amode, bmode, epi, splits, tile, P_<ihipStream_t>(stream)), "gemm");
      },
      py::arg("amode"), py::arg("bmode"), py::arg("epi"), py::arg("splits"), py::arg("tile"), py::arg("A"),
      py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("stats"), py::arg("R"), py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("geo"), py::arg("kc"), py::arg("k_per_split"),
      py::arg("stream"), py::arg("kstep") = 0, py::arg("stats_acc") = 0, py::arg("bnx") = 0, py::arg("bnst") = 0,
      py::arg("stats_reps") = 1, py::arg("bnin_p") = std::vector<uintptr_t>{},
      py::arg("bnin_v") = std::vector<float>{}, py::arg("bnin_y") = 0, py::arg("slab") = 0, py::arg("tickets") = 0);
  m.def("gemm_stats_tile_rows", &damd::gemm_stats_tile_rows);
  m.def("conv_gemm_kstep", &damd::conv_gemm_kstep);
  m.def("conv3_rows", &damd::conv3_rows);
  m.def("conv3_stamps_enable", [](int on) { check(damd::conv3_stamps_enable(on), "conv3_stamps_enable"); });
  m.def("conv3_stamps_read", [](int blocks) {
    std::vector<unsigned long long> v((size_t)blocks * 4);
    check(damd::conv3_stamps_read(v.data(), blocks), "conv3_stamps_read");
    return v;
  });
  m.def("stem_stamps_enable", [](int on) { check(damd::stem_stamps_enable(on), "stem_stamps_enable"); });
  m.def("stem_stamps_read", [](int blocks) {
    std::vector<unsigned long long> v((size_t)blocks * 8);
    check(damd::stem_stamps_read(v.data(), blocks), "stem_stamps_read");
    return v;
  });
  m.def("wgrad3_stamps_enable", [](int on) { check(damd::wgrad3_stamps_enable(on), "wgrad3_stamps_enable"); });
  m.def("wgrad3_stamps_read", [](int blocks) {
    std::vector<unsigned long long> v((size_t)blocks * 4);
    check(damd::wgrad3_stamps_read(v.data(), blocks), "wgrad3_stamps_read");
    return v;
  });
  m.def("splitk_finish", [](uintptr_t slab, int splits, int M, int N, uintptr_t bias, uintptr_t R, int relu,
                            uintptr_t stats, int rb, uintptr_t out, int ldc, uintptr_t stream, uintptr_t stats_acc,
                            int stats_reps) {
    check(damd::splitk_finish(P_<const float>(slab), splits, M, N, P_<const float>(bias), P_<const uint16_t>(R), relu,
                              P_<float>(stats), rb, P_<uint16_t>(out), ldc, P_<ihipStream_t>(stream),
                              P_<long long>(stats_acc), stats_reps),
          "splitk_finish");
  }, py::arg("slab"), py::arg("splits"), py::arg("M"), py::arg("N"), py::arg("bias"), py::arg("R"), py::arg("relu"),
     py::arg("stats"), py::arg("rb"), py::arg("out"), py::arg("ldc"), py::arg("stream"), py::arg("stats_acc") = 0,
     py::arg("stats_reps") = 1);
  m.def("splitk_finish_f32", [](uintptr_t slab, int splits, int M, int N, uintptr_t bias, int relu, uintptr_t out,
                                int ldc, uintptr_t stream) {
    check(damd::splitk_finish_f32(P_<const float>(slab), splits, M, N, P_<const float>(bias), relu, P_<float>(out),
                                  ldc, P_<ihipStream_t>(stream)),
          "splitk_finish_f32");
  });
  m.def("splitk_reduce", [](uintptr_t slab, int splits, long n, uintptr_t dst, uintptr_t stream, int accumulate) {
    check(damd::splitk_reduce(P_<const float>(slab), splits, n, P_<float>(dst), P_<ihipStream_t>(stream), accumulate),
          "splitk_reduce");
  }, py::arg("slab"), py::arg("splits"), py::arg("n"), py::arg("dst"), py::arg("stream"), py::arg("accumulate") = 1);
  m.def("splitk_reduce_unpad", [](uintptr_t slab, int splits, int R, int C1, int C2, int C1p, int C2p, uintptr_t dst,
                                  uintptr_t stream, int accumulate) {
    check(damd::splitk_reduce_unpad(P_<const float>(slab), splits, R, C1, C2, C1p, C2p, P_<float>(dst),
                                    P_<ihipStream_t>(stream), accumulate),
          "splitk_reduce_unpad");
  });

  using U = uintptr_t;
  using u16 = uint16_t;
  m.def("bn_finalize", [](U part, int T, int C, float count, U gamma, U beta, float eps, float mom, U rmean, U rvar,
                          U st, U s) {
    check(damd::bn_finalize(P_<const float>(part), T, C, count, P_<const float>(gamma), P_<const float>(beta), eps,
                            mom, P_<float>(rmean), P_<float>(rvar), P_<float>(st), P_<ihipStream_t>(s)),
          "bn_finalize");
  });
  m.def("bn_apply", [](U x, U st, U r, U st2, int res_mode, int relu, U y, long M, int C, U s) {
    check(damd::bn_apply(P_<const u16>(x), P_<const float>(st), P_<const u16>(r), P_<const float>(st2), res_mode,
                         relu, P_<u16>(y), M, C, P_<ihipStream_t>(s)),
          "bn_apply");
  });
  m.def("bn_bwd_blocks", &damd::bn_bwd_blocks);
  m.def("bn_bwd_reduce", [](U dy, U y, int relu_mask, U x, U st, U dz, U part, int T, long M, int C, U s) {
    check(damd::bn_bwd_reduce(P_<const u16>(dy), P_<const u16>(y), relu_mask, P_<const u16>(x), P_<const float>(st),
                              P_<u16>(dz), P_<float>(part), T, M, C, P_<ihipStream_t>(s)),
          "bn_bwd_reduce");
  });
  m.def("bn_bwd_finalize", [](U part, int T, int C, float count, U st, U gamma, U dgamma, U dbeta, U co, U s) {
    check(damd::bn_bwd_finalize(P_<const float>(part), T, C, count, P_<const float>(st), P_<const float>(gamma),
                                P_<float>(dgamma), P_<float>(dbeta), P_<float>(co), P_<ihipStream_t>(s)),
          "bn_bwd_finalize");
  });
  m.def("bn_bwd_apply", [](U dy, U y, int relu_mask, U x, U st, U co, U dx, long M, int C, U s) {
    check(damd::bn_bwd_apply(P_<const u16>(dy), P_<const u16>(y), relu_mask, P_<const u16>(x), P_<const float>(st),
                             P_<const float>(co), P_<u16>(dx), M, C, P_<ihipStream_t>(s)),
          "bn_bwd_apply");
  });
  // ---- BatchNorm with the finalize in the consumer (layer_ops.h BNFin / BNBwdFin) ----
  // fin = [acc, gamma, beta, st, rmean, rvar] pointers + [count, eps, momentum]
  // bfin = [acc, dgamma, dbeta, co] pointers + count
  auto mkfin = [](const std::vector<U>& p, const std::vector<float>& v) {
    damd::BNFin f{};
    if (p.empty()) return f;
    if (p.size() != 6 || v.size() != 4) throw std::invalid_argument("fin: 6 pointers + [count, eps, momentum, reps]");
    f.acc = P_<const long long>(p[0]); f.gamma = P_<const float>(p[1]); f.beta = P_<const float>(p[2]);
    f.st = P_<float>(p[3]); f.rmean = P_<float>(p[4]); f.rvar = P_<float>(p[5]);
    f.count = v[0]; f.eps = v[1]; f.mom = v[2]; f.reps = (int)v[3];
    return f;
  };
  auto mkbfin = [](const std::vector<U>& p, float count, int reps) {
    damd::BNBwdFin f{};
    if (p.size() != 4) throw std::invalid_argument("bfin: [acc, dgamma, dbeta, co]");
    f.acc = P_<const long long>(p[0]); f.dgamma = P_<float>(p[1]); f.dbeta = P_<float>(p[2]); f.co = P_<float>(p[3]);
    f.count = count;
    f.reps = reps;
    return f;
  };
  m.def("bn_apply_fin", [mkfin](U x, U r, int res_mode, int relu, U y, long M, int C, std::vector<U> p1,
                                std::vector<float> v1, std::vector<U> p2, std::vector<float> v2, U s) {
    const damd::BNFin a = mkfin(p1, v1), b = mkfin(p2, v2);
    check(damd::bn_apply(P_<const u16>(x), a.st, P_<const u16>(r), b.st, res_mode, relu, P_<u16>(y), M, C,
                         P_<ihipStream_t>(s), &a, &b),
          "bn_apply_fin");
  });
  m.def("bn_reduce_reverse", &damd::bn_reduce_reverse);
  m.def("bn_bwd_reduce_acc", [](U dy, U y, int relu_mask, U x, U st, U dz, U acc, int T, long M, int C, U s,
                                int reps) {
    check(damd::bn_bwd_reduce(P_<const u16>(dy), P_<const u16>(y), relu_mask, P_<const u16>(x), P_<const float>(st),
                              P_<u16>(dz), nullptr, T, M, C, P_<ihipStream_t>(s), P_<long long>(acc), reps),
          "bn_bwd_reduce_acc");
  });
  m.def("bn_bwd_apply_fin", [mkbfin](U dy, U y, int relu_mask, U x, U st, U dx, long M, int C, std::vector<U> bp,
                                     float count, U s, int reps) {
    const damd::BNBwdFin f = mkbfin(bp, count, reps);
    check(damd::bn_bwd_apply(P_<const u16>(dy), P_<const u16>(y), relu_mask, P_<const u16>(x), P_<const float>(st),
                             f.co, P_<u16>(dx), M, C, P_<ihipStream_t>(s), &f),
          "bn_bwd_apply_fin");
  });
  m.def("bn_bwd_reduce_dual_acc", [](U dy, U y, int relu_mask, U x, U x2, U st, U st2, U acc, U acc2, int T, long M,
                                     int C, U s, int reps) {
    check(damd::bn_bwd_reduce_dual(P_<const u16>(dy), P_<const u16>(y), relu_mask, P_<const u16>(x),
                                   P_<const u16>(x2), P_<const float>(st), P_<const float>(st2), T, M, C,
                                   P_<ihipStream_t>(s), P_<long long>(acc), P_<long long>(acc2), reps),
          "bn_bwd_reduce_dual_acc");
  });
  m.def("bn_bwd_apply_dual_fin", [mkbfin](U dy, U y, int relu_mask, U x, U x2, U st, U st2, U dx, U dx2, long M,
                                          int C, std::vector<U> bp, std::vector<U> bp2, float count, U s, int reps) {
    const damd::BNBwdFin f = mkbfin(bp, count, reps), f2 = mkbfin(bp2, count, reps);
    check(damd::bn_bwd_apply_dual(P_<const u16>(dy), P_<const u16>(y), relu_mask, P_<const u16>(x),
                                  P_<const u16>(x2), P_<const float>(st), P_<const float>(st2), P_<u16>(dx),
                                  P_<u16>(dx2), M, C, P_<ihipStream_t>(s), f, f2),
          "bn_bwd_apply_dual_fin");
  });
  m.def("bn_relu_maxpool_fwd_fin", [mkfin](U x, std::vector<int> g, U y, U arg, std::vector<U> p, std::vector<float> v,
                                           U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    const damd::BNFin f = mkfin(p, v);
    check(damd::bn_relu_maxpool_fwd(P_<const u16>(x), f.st, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8],
                                    g[9], g[10], g[11], P_<u16>(y), P_<uint8_t>(arg), P_<ihipStream_t>(s), &f),
          "bn_relu_maxpool_fwd_fin");
  });
  m.def("pool_bn_bwd_reduce_acc", [](U dpool, U arg, std::vector<int> g, U x, U st, U acc, int T, U s, int reps) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::pool_bn_bwd_reduce(P_<const u16>(dpool), P_<const uint8_t>(arg), g[0], g[1], g[2], g[3], g[4], g[5],
                                   g[6], g[7], g[8], g[9], g[10], g[11], P_<const u16>(x), P_<const float>(st),
                                   nullptr, T, P_<ihipStream_t>(s), P_<long long>(acc), reps),
          "pool_bn_bwd_reduce_acc");
  });
  m.def("pool_bn_bwd_apply_fin", [mkbfin](U dpool, U arg, std::vector<int> g, U x, U st, U dx, std::vector<U> bp,
                                          float count, U s, int reps) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    const damd::BNBwdFin f = mkbfin(bp, count, reps);
    check(damd::pool_bn_bwd_apply(P_<const u16>(dpool), P_<const uint8_t>(arg), g[0], g[1], g[2], g[3], g[4], g[5],
                                  g[6], g[7], g[8], g[9], g[10], g[11], P_<const u16>(x), P_<const float>(st), f.co,
                                  P_<u16>(dx), P_<ihipStream_t>(s), &f),
          "pool_bn_bwd_apply_fin");
  });
  m.def("maxpool_fwd", [](U x, std::vector<int> g, U y, U arg, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::maxpool_fwd(P_<const u16>(x), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10],
                            g[11], P_<u16>(y), P_<uint8_t>(arg), P_<ihipStream_t>(s)),
          "maxpool_fwd");
  });
  m.def("maxpool_bwd", [](U dy, U arg, std::vector<int> g, U dx, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::maxpool_bwd(P_<const u16>(dy), P_<const uint8_t>(arg), g[0], g[1], g[2], g[3], g[4], g[5], g[6],
                            g[7], g[8], g[9], g[10], g[11], P_<u16>(dx), P_<ihipStream_t>(s)),
          "maxpool_bwd");
  });
  m.def("bn_relu_maxpool_fwd", [](U x, U st, std::vector<int> g, U y, U arg, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::bn_relu_maxpool_fwd(P_<const u16>(x), P_<const float>(st), g[0], g[1], g[2], g[3], g[4], g[5], g[6],
                                    g[7], g[8], g[9], g[10], g[11], P_<u16>(y), P_<uint8_t>(arg), P_<ihipStream_t>(s)),
          "bn_relu_maxpool_fwd");
  });
  m.def("pool_bn_bwd_reduce", [](U dpool, U arg, std::vector<int> g, U x, U st, U part, int T, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::pool_bn_bwd_reduce(P_<const u16>(dpool), P_<const uint8_t>(arg), g[0], g[1], g[2], g[3], g[4], g[5],
                                   g[6], g[7], g[8], g[9], g[10], g[11], P_<const u16>(x), P_<const float>(st),
                                   P_<float>(part), T, P_<ihipStream_t>(s)),
          "pool_bn_bwd_reduce");
  });
  m.def("pool_bn_bwd_apply", [](U dpool, U arg, std::vector<int> g, U x, U st, U co, U dx, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::pool_bn_bwd_apply(P_<const u16>(dpool), P_<const uint8_t>(arg), g[0], g[1], g[2], g[3], g[4], g[5],
                                  g[6], g[7], g[8], g[9], g[10], g[11], P_<const u16>(x), P_<const float>(st),
                                  P_<const float>(co), P_<u16>(dx), P_<ihipStream_t>(s)),
          "pool_bn_bwd_apply");
  });
  m.def("gap_fwd", [](U x, int N, int HW, int C, U y, int y_f32, U s) {
    check(damd::gap_fwd(P_<const u16>(x), N, HW, C, P_<void>(y), y_f32, P_<ihipStream_t>(s)), "gap_fwd");
  });
  m.def("gap_bwd", [](U dy, int dy_f32, int N, int HW, int C, U dx, U s) {
    check(damd::gap_bwd(P_<const void>(dy), dy_f32, N, HW, C, P_<u16>(dx), P_<ihipStream_t>(s)), "gap_bwd");
  });
  m.def("relu_bwd", [](U dy, U y, U dz, long n, U s) {
    check(damd::relu_bwd(P_<const u16>(dy), P_<const u16>(y), P_<u16>(dz), n, P_<ihipStream_t>(s)), "relu_bwd");
  });
  m.def("act_fwd", [](U x, U y, long n, int kind, U s) {
    check(damd::act_fwd(P_<const u16>(x), P_<u16>(y), n, kind, P_<ihipStream_t>(s)), "act_fwd");
  });
  m.def("act_bwd", [](U dy, U y, U dx, long n, int kind, U s) {
    check(damd::act_bwd(P_<const u16>(dy), P_<const u16>(y), P_<u16>(dx), n, kind, P_<ihipStream_t>(s)), "act_bwd");
  });
  m.def("dropout", [](U x, U y, long n, U ctrl, uint32_t seed, float rate, U s) {
    check(damd::dropout(P_<const u16>(x), P_<u16>(y), n, P_<const damd::Ctrl>(ctrl), seed, rate, P_<ihipStream_t>(s)),
          "dropout");
  });
  m.def("avgpool_fwd", [](U x, std::vector<int> g, U y, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::avgpool_fwd(P_<const u16>(x), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10],
                            g[11], P_<u16>(y), P_<ihipStream_t>(s)),
          "avgpool_fwd");
  });
  m.def("avgpool_bwd", [](U dy, std::vector<int> g, U dx, U s) {
    if (g.size() != 12) throw std::invalid_argument("pool geometry");
    check(damd::avgpool_bwd(P_<const u16>(dy), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10],
                            g[11], P_<u16>(dx), P_<ihipStream_t>(s)),
          "avgpool_bwd");
  });
  m.def("bn_infer_st", [](U rmean, U rvar, U gamma, U beta, float eps, int C, U st, U s) {
    check(damd::bn_infer_st(P_<const float>(rmean), P_<const float>(rvar), P_<const float>(gamma),
                            P_<const float>(beta), eps, C, P_<float>(st), P_<ihipStream_t>(s)),
          "bn_infer_st");
  });
  m.def("logits_store", [](U logits, int ld, int K, int B, U ctrl, U out, U s) {
    check(damd::logits_store(P_<const float>(logits), ld, K, B, P_<const damd::Ctrl>(ctrl), P_<float>(out),
                             P_<ihipStream_t>(s)),
          "logits_store");
  });
  m.def("step_fold", [](U ctrl, U tail, U s) {
    check(damd::step_fold(P_<damd::Ctrl>(ctrl), P_<float>(tail), P_<ihipStream_t>(s)), "step_fold");
  });
  m.def("add_bf16", [](U a, U b, U o, long n, U s) {
    check(damd::add_bf16(P_<const u16>(a), P_<const u16>(b), P_<u16>(o), n, P_<ihipStream_t>(s)), "add_bf16");
  });
  m.def("cast_bf16_f32", [](U x, U y, long n, U s) {
    check(damd::cast_bf16_f32(P_<const u16>(x), P_<float>(y), n, P_<ihipStream_t>(s)), "cast_bf16_f32");
  });
  m.def("cast_f32_bf16", [](U x, U y, long n, U s) {
    check(damd::cast_f32_bf16(P_<const float>(x), P_<u16>(y), n, P_<ihipStream_t>(s)), "cast_f32_bf16");
  });
  m.def("cast_u8_bf16", [](U x, float scale, U y, long n, U s) {
    check(damd::cast_u8_bf16(P_<const uint8_t>(x), scale, P_<u16>(y), n, P_<ihipStream_t>(s)), "cast_u8_bf16");
  });
  m.def("colsum_splits", &damd::colsum_splits);
  m.def("colsum", [](U x, int x_f32, int M, int N, int ld, U out, U s, U ws) {
    check(damd::colsum(P_<const void>(x), x_f32, M, N, ld, P_<float>(out), P_<float>(ws), P_<ihipStream_t>(s)),
          "colsum");
  });
  m.def("softmax_xent", [](U logits, int ld, U labels, int B, int K, float scale, U ctrl, U dl, U tail, U rows, U s,
                           U bias_grad) {
    check(damd::softmax_xent(P_<const float>(logits), ld, P_<const int32_t>(labels), B, K, scale,
                             P_<const damd::Ctrl>(ctrl), P_<u16>(dl), P_<float>(tail), P_<float>(rows),
                             P_<ihipStream_t>(s), P_<float>(bias_grad)),
          "softmax_xent");
  }, py::arg("logits"), py::arg("ld"), py::arg("labels"), py::arg("B"), py::arg("K"), py::arg("scale"),
     py::arg("ctrl"), py::arg("dl"), py::arg("tail"), py::arg("rows"), py::arg("s"), py::arg("bias_grad") = 0);
  m.def("sgd_step", [](U P, U G, U V, U Pb, long n, U ctrl, U tail, U s) {
    check(damd::sgd_step(P_<float>(P), P_<const float>(G), P_<float>(V), P_<u16>(Pb), n, P_<damd::Ctrl>(ctrl),
                         P_<const float>(tail), P_<ihipStream_t>(s)),
          "sgd_step");
  });
  m.def("opt_step", [](U P, U G, U S0, U S1, U S2, U Pb, long n, U ctrl, U tail, int kind, float b1, float b2,
                       float eps, float rho, float mom, int flag, U s, int book) {
    damd::OptArgs o{kind, b1, b2, eps, rho, mom, flag};
    check(damd::opt_step(P_<float>(P), P_<const float>(G), P_<float>(S0), P_<float>(S1), P_<float>(S2), P_<u16>(Pb), n,
                         P_<damd::Ctrl>(ctrl), P_<const float>(tail), o, P_<ihipStream_t>(s), book),
          "opt_step");
  }, py::arg("P"), py::arg("G"), py::arg("S0"), py::arg("S1"), py::arg("S2"), py::arg("Pb"), py::arg("n"),
     py::arg("ctrl"), py::arg("tail"), py::arg("kind"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("rho"),
     py::arg("mom"), py::arg("flag"), py::arg("s"), py::arg("book") = 1);
  m.def("gather_batch", [](U x, int x_u8, float scale, U labels, U ctrl, int per, int HW, int Cin, int Cp, U xb, U yb,
                           U s, U zero, long zero_bytes, U zero2, long zero2_bytes, U pc_src, U pc_dst,
                           std::vector<int> pc_dims) {
    damd::PadCastJob pc{P_<const float>(pc_src), P_<u16>(pc_dst), 0, 0, 0, 0, 0};
    if (pc_src) {
      if (pc_dims.size() != 5) throw std::runtime_error("gather_batch: pc_dims = (R, C1, C2, C1p, C2p)");
      pc.R = pc_dims[0], pc.C1 = pc_dims[1], pc.C2 = pc_dims[2], pc.C1p = pc_dims[3], pc.C2p = pc_dims[4];
    }
    check(damd::gather_batch(P_<const void>(x), x_u8, scale, P_<const int32_t>(labels), P_<damd::Ctrl>(ctrl),
                             per, HW, Cin, Cp, P_<u16>(xb), P_<int32_t>(yb), P_<ihipStream_t>(s), P_<void>(zero),
                             zero_bytes, P_<void>(zero2), zero2_bytes, pc),
          "gather_batch");
  }, py::arg("x"), py::arg("x_u8"), py::arg("scale"), py::arg("labels"), py::arg("ctrl"), py::arg("per"),
     py::arg("HW"), py::arg("Cin"), py::arg("Cp"), py::arg("xb"), py::arg("yb"), py::arg("s"), py::arg("zero") = 0,
     py::arg("zero_bytes") = 0, py::arg("zero2") = 0, py::arg("zero2_bytes") = 0, py::arg("pc_src") = 0,
     py::arg("pc_dst") = 0, py::arg("pc_dims") = std::vector<int>{});
  m.def("pad_cast", [](U src, int R, int C1, int C2, int C1p, int C2p, U dst, U s) {
    check(damd::pad_cast(P_<const float>(src), R, C1, C2, C1p, C2p, P_<u16>(dst), P_<ihipStream_t>(s)), "pad_cast");
  });
  m.def("unpad_add", [](U src, int R, int C1, int C2, int C1p, int C2p, U dst, U s) {
    check(damd::unpad_add(P_<const float>(src), R, C1, C2, C1p, C2p, P_<float>(dst), P_<ihipStream_t>(s)),
          "unpad_add");
  });
  m.def("sgd_flat", [](U P, U G, U V, U Pb, long n, float lr, float mom, int nest, U s) {
    check(damd::sgd_flat(P_<float>(P), P_<const float>(G), P_<float>(V), P_<u16>(Pb), n, lr, mom, nest,
                         P_<ihipStream_t>(s)),
          "sgd_flat");
  });
}
