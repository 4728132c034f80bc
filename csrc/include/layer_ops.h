// Non-GEMM per-layer kernels of the generic path (csrc/kernels/layer_ops.hip).
// Activations are NHWC bf16 (uint16 storage) with the channel count C a multiple of 8,
// parameters / statistics fp32.  All launches are stream-ordered on `s`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace damd {

struct Ctrl;  // kernels_api.h / damd_common.h

// BatchNorm (training) ---------------------------------------------------------------
// Batch statistics without a finalize launch: the producers (conv GEMM epilogue E_STATS
// with GemmArgs::stats_acc, splitk_finish, bn_bwd_reduce / pool_bn_bwd_reduce with `acc`)
// add their per-block fp32 partials into acc[reps][2][C] as int64 fixed point (one word
// per value forward, two backward: damd_common.h bnacc_add1 / bnacc_add2 -- integer
// atomics, so the sums are bitwise independent of the blocks' arrival order); producer
// block / M-tile b adds into replica b % reps, so that same-address atomics --
// serialised at the memory side -- form reps short chains instead of one long one; the
// consumer kernel (bn_apply, bn_relu_maxpool_fwd / bn_bwd_apply, pool_bn_bwd_apply)
// derives the coefficients from acc (replicas summed in order) in its prologue (every
// block, into LDS); its block 0 also writes st / co, the moving statistics and dgamma /
// dbeta.  The accumulators are zeroed once per step (gather_batch's `zero` range).
struct BNFin {
  const long long* acc;  // [reps][2][C] sum, sum of squares (bnacc_add1) + flag plane [2C]; null: the kernel reads st
  const float* gamma;  // may be null (1)
  const float* beta;   // may be null (0)
  float* st;           // [4][C] out (block 0): mean, invstd, scale, shift
  float* rmean;        // moving statistics (block 0), may be null
  float* rvar;
  float count, eps, mom;
  int reps;            // replicas of acc (0 / 1: one)
};
struct BNBwdFin {
  const long long* acc;  // [reps][4][C] sum dz / sum dz * xhat, hi / lo planes (bnacc_add2) + flag plane [4C]; null: co
  float* dgamma;       // += (block 0), may be null
  float* dbeta;
  float* co;           // [3][C] out (block 0)
  float count;
  int reps;
};
// partials [T][2][C] (column sum, sum of squares; from the conv GEMM epilogue) ->
// st[4][C] = mean, invstd, scale = gamma*invstd, shift = beta - mean*scale; moving
// statistics updated Keras-style (m = m*momentum + batch*(1-momentum), biased variance).
hipError_t bn_finalize(const float* part, int T, int C, float count, const float* gamma, const float* beta,
                       float eps, float momentum, float* rmean, float* rvar, float* st, hipStream_t s);
// y = act(x*scale + shift [+ r | + r*scale2 + shift2])   (res_mode 0 / 1 / 2)
hipError_t bn_apply(const uint16_t* x, const float* st, const uint16_t* r, const float* st2, int res_mode,
                    int relu, uint16_t* y, long M, int C, hipStream_t s, const BNFin* f1 = nullptr,
                    const BNFin* f2 = nullptr);
// inference: y = act(x*scale + shift) with scale/shift from the moving statistics
// backward, pass 1: dz = dy * [y > 0] (relu_mask 1; relu_mask 2: y recomputed as
// bf16(relu(x * sc + sh)) from x and st, bitwise the stored bn_apply output, y unread) ; per-block partial sums of dz and
// dz * xhat -> part [T][2][C]; optionally writes dz (bf16).  Returns T via *T_out.
hipError_t bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x,
                         const float* st, uint16_t* dz_out, float* part, int T, long M, int C, hipStream_t s,
                         long long* acc = nullptr, int acc_reps = 1);
int bn_bwd_blocks(long M, int C);
// tests: bn_bwd_reduce launches its row ranges in reversed block order (order independence)
void bn_reduce_reverse(bool on);
// pass 2: dgamma/dbeta (accumulated into the gradient sinks, may be null) and the
// coefficients co[3][C] so that dx = a*dz + b + c*xhat
hipError_t bn_bwd_finalize(const float* part, int T, int C, float count, const float* st, const float* gamma,
                           float* dgamma, float* dbeta, float* co, hipStream_t s);
// pass 3: dx = a*dz + b + c*xhat, dz recomputed from dy and the relu mask (bf16 out)
hipError_t bn_bwd_apply(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x, const float* st,
                        const float* co, uint16_t* dx, long M, int C, hipStream_t s, const BNBwdFin* bf = nullptr);

// Two BatchNorms of the same masked gradient (relu_mask 0 / 1), fixed-point accumulators
// and in-consumer finalize only: one reduce pass and one apply pass for both (bitwise the
// two single-BN launch pairs)
hipError_t bn_bwd_reduce_dual(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x,
                              const uint16_t* x2, const float* st, const float* st2, int T, long M, int C,
                              hipStream_t s, long long* acc, long long* acc2, int acc_reps);
hipError_t bn_bwd_apply_dual(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x,
                             const uint16_t* x2, const float* st, const float* st2, uint16_t* dx, uint16_t* dx2,
                             long M, int C, hipStream_t s, const BNBwdFin& bf, const BNBwdFin& bf2);

// Pooling ----------------------------------------------------------------------------------
hipError_t maxpool_fwd(const uint16_t* x, int N, int H, int W, int C, int ph, int pw, int sh, int sw, int pad_t,
                       int pad_l, int Ho, int Wo, uint16_t* y, uint8_t* arg, hipStream_t s);
hipError_t maxpool_bwd(const uint16_t* dy, const uint8_t* arg, int N, int H, int W, int C, int ph, int pw, int sh,
                       int sw, int pad_t, int pad_l, int Ho, int Wo, uint16_t* dx, hipStream_t s);
// stem fusion (BatchNorm(st) -> ReLU -> MaxPool): the pool reads the conv output x
hipError_t bn_relu_maxpool_fwd(const uint16_t* x, const float* st, int N, int H, int W, int C, int ph, int pw, int sh,
                               int sw, int pad_t, int pad_l, int Ho, int Wo, uint16_t* y, uint8_t* arg, hipStream_t s,
                               const BNFin* f = nullptr);
// its backward: BN-backward partials / apply with the pool routing + ReLU mask recomputed
hipError_t pool_bn_bwd_reduce(const uint16_t* dpool, const uint8_t* arg, int N, int H, int W, int C, int ph, int pw,
                              int sh, int sw, int pad_t, int pad_l, int Ho, int Wo, const uint16_t* x, const float* st,
                              float* part, int T, hipStream_t s, long long* acc = nullptr, int acc_reps = 1);
hipError_t pool_bn_bwd_apply(const uint16_t* dpool, const uint8_t* arg, int N, int H, int W, int C, int ph, int pw,
                             int sh, int sw, int pad_t, int pad_l, int Ho, int Wo, const uint16_t* x, const float* st,
                             const float* co, uint16_t* dx, hipStream_t s, const BNBwdFin* bf = nullptr);
// global average pool over H*W: x [N][HW][C] bf16 -> y [N][C] (bf16 or fp32)
hipError_t gap_fwd(const uint16_t* x, int N, int HW, int C, void* y, int y_f32, hipStream_t s);
hipError_t gap_bwd(const void* dy, int dy_f32, int N, int HW, int C, uint16_t* dx, hipStream_t s);

// Elementwise -----------------------------------------------------------------------------
// dz = dy * [y > 0]  (bf16)
hipError_t relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dz, long n, hipStream_t s);
// y = act(x) / dx = dy * act'(y), kind 0 relu, 1 sigmoid, 2 tanh (bf16, any length, in place ok)
hipError_t act_fwd(const uint16_t* x, uint16_t* y, long n, int kind, hipStream_t s);
hipError_t act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, int kind, hipStream_t s);
// y = x * keep / (1 - rate), keep from a counter hash of (seed, ctrl->cur3, element): the
// same call with the same seed is the backward (dx from dy)
hipError_t dropout(const uint16_t* x, uint16_t* y, long n, const Ctrl* ctrl, uint32_t seed, float rate,
                   hipStream_t s);
// average pooling, divisor = in-bounds taps (TF 'same' semantics)
hipError_t avgpool_fwd(const uint16_t* x, int N, int H, int W, int C, int ph, int pw, int sh, int sw, int pad_t,
                       int pad_l, int Ho, int Wo, uint16_t* y, hipStream_t s);
hipError_t avgpool_bwd(const uint16_t* dy, int N, int H, int W, int C, int ph, int pw, int sh, int sw, int pad_t,
                       int pad_l, int Ho, int Wo, uint16_t* dx, hipStream_t s);
// Inference: BN st rows from the moving statistics; this step's logits rows -> out at the
// device cursor; fold the metric tail into ctrl (tail cleared) and advance the cursor
hipError_t bn_infer_st(const float* rmean, const float* rvar, const float* gamma, const float* beta, float eps, int C,
                       float* st, hipStream_t s);
hipError_t logits_store(const float* logits, int ld, int K, int B, const Ctrl* ctrl, float* out, hipStream_t s);
hipError_t step_fold(Ctrl* ctrl, float* tail, hipStream_t s);
// out = a + b (bf16)
hipError_t add_bf16(const uint16_t* a, const uint16_t* b, uint16_t* out, long n, hipStream_t s);
// fp32 -> bf16, bf16 -> fp32
hipError_t cast_f32_bf16(const float* x, uint16_t* y, long n, hipStream_t s);
hipError_t cast_bf16_f32(const uint16_t* x, float* y, long n, hipStream_t s);
// uint8 (k) -> bf16(k * scale)
hipError_t cast_u8_bf16(const uint8_t* x, float scale, uint16_t* y, long n, hipStream_t s);
// out[n] += sum_m x[m][n]  (x bf16 or fp32, [M][ld]) in a fixed order; when
// colsum_splits(M, N) > 1 the row splits go through ws[splits][N] (fp32 workspace)
int colsum_splits(int M, int N);
hipError_t colsum(const void* x, int x_f32, int M, int N, int ld, float* out, float* ws, hipStream_t s);

// Loss --------------------------------------------------------------------------------------
// Sparse softmax cross-entropy from fp32 logits [B][ld]: dlogits (bf16, [B][K]) =
// (softmax - onehot) * scale; tail[0] += sum loss, tail[1] += sum correct (argmax ==
// label, first max wins), tail[2] += B.  labels int32; a label < 0 masks the row (zero
// gradient, no loss/metric).  ctrl != nullptr: scale = 1 / real rows of the global batch
// (short final batch; see softmax_xent_k), else the given scale.
// dlogits shares the row pitch ld of the logits; its padding columns are left untouched.
// rows: scratch of 3 B floats + one int arrival counter (zero before the first call; the
// kernel re-arms it): the batch sums are formed in a fixed order, not by float atomics.
// bias_grad (optional): += the column sums of the stored dlogits, exactly as colsum with one
// split (the logits layer's bias gradient without a colsum launch)
hipError_t softmax_xent(const float* logits, int ld, const int32_t* labels, int B, int K, float scale,
                        const Ctrl* ctrl, uint16_t* dlogits, float* tail, float* rows, hipStream_t s,
                        float* bias_grad = nullptr);
int colsum_splits(int M, int N);

// Optimizer ---------------------------------------------------------------------------------
// flat multi-tensor Keras SGD over the master buffer: P, V fp32 updated from G; Pb = bf16(P)
hipError_t sgd_flat(float* P, const float* G, float* V, uint16_t* Pb, long n, float lr, float momentum,
                    int nesterov, hipStream_t s);

// one training step's optimizer tail for the graph-captured generic path: hyper-parameters
// from ctrl (lr / momentum / nesterov, so a new lr needs no re-capture); block 0 also
// folds the step's metric tail [loss, correct, count] into the epoch accumulators and
// advances ctrl->cursor / ctrl->iterations.
struct Ctrl;
hipError_t sgd_step(float* P, const float* G, float* V, uint16_t* Pb, long n, Ctrl* ctrl, const float* tail,
                    hipStream_t s);
// kind 0 SGD (S0 momentum; flag = nesterov), 1 Adam (S0 m, S1 v, S2 vhat; flag = amsgrad),
// 2 RMSprop (S0 rms, S1 momentum, S2 mean gradient; flag = centered)
struct OptArgs {
  int kind;
  float b1, b2, eps, rho, mom;
  int flag;
};
hipError_t opt_step(float* P, const float* G, float* S0, float* S1, float* S2, uint16_t* Pb, long n, Ctrl* ctrl,
                    const float* tail, const OptArgs& o, hipStream_t s, int book = 1);

// Data / layout glue -------------------------------------------------------------------------
// the step's rows of the (epoch-permuted) dataset: row = (cursor*global_batch + row0 + i)
// mod nsamples (cursor from ctrl); x fp32 or uint8 (k / scale, i.e. exactly float32(k/255)
// for scale 255) [n][HW][Cin] -> bf16
// [per][HW][Cp] zero-padded channels; labels int32.  zero / zero2 (optional): byte ranges
// (16-byte aligned, multiples of 16 bytes) cleared in the same launch -- the step's
// gradient buffer and BatchNorm statistics accumulators, so no memset launch precedes it.
// A pad_cast (below) run inside gather_batch's launch: the step's first layer's padded bf16
// weights refreshed without a launch of their own (src == nullptr: none).
struct PadCastJob {
  const float* src;
  uint16_t* dst;
  int R, C1, C2, C1p, C2p;
};
hipError_t gather_batch(const void* x, int x_u8, float scale, const int32_t* labels, Ctrl* ctrl, int per,
                        int HW, int Cin, int Cp, uint16_t* xb, int32_t* yb, hipStream_t s, void* zero = nullptr,
                        long zero_bytes = 0, void* zero2 = nullptr, long zero2_bytes = 0,
                        PadCastJob pc = PadCastJob{nullptr, nullptr, 0, 0, 0, 0, 0});
// fp32 [R][C1][C2] -> bf16 [R][C1p][C2p] (zero padding)
hipError_t pad_cast(const float* src, int R, int C1, int C2, int C1p, int C2p, uint16_t* dst, hipStream_t s);
// dst fp32 [R][C1][C2] += src fp32 [R][C1p][C2p] (the un-padded part)
hipError_t unpad_add(const float* src, int R, int C1, int C2, int C1p, int C2p, float* dst, hipStream_t s);

}  // namespace damd
