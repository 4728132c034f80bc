// Host interface of the fused MNIST-CNN step kernels (csrc/kernels/convnet_step2.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace damd {
struct Ctrl;

// ---- sharded gradient exchange of the multi-rank step (world > 1, one GPU per rank) ----
// The dW1 gradient is split into units (slice s, 16-column quarter q) = 96 x 16 values; unit
// u = 4 s + q is owned by rank u % world.  bwd pushes each unit's partial to its owner, the
// owner's bwd sums the world partials in rank order and pushes the reduced unit to every
// rank; the small gradients (conv, b1 / W2 / b2) and the metric tail travel as one message
// per rank that every rank sums in rank order.  All buffers below live in uncached device
// memory exported over IPC (PeerAllreduce's staging), mapped on every rank.
constexpr int kXMaxRanks = 8;
constexpr int kXPSlot = 2048;        // floats per (source, unit) partial slot (fragment layout)
constexpr int kXSmsg = 1408;         // floats per small message: 320 int64 conv | 714 grads | 3 metrics
constexpr long kXGred = 0;           // out: reduced gradient, flat [kConvNetNGrad] (W1 part from owners)
constexpr long kXSmall = 347648;     // out: small messages [2 parity][kXMaxRanks][kXSmsg]
constexpr long kXFlags = kXSmall + 2L * kXMaxRanks * kXSmsg;  // out: flag words (unsigned)
constexpr int kXPFlagPitch = 2 * kXMaxRanks;                  // partial flags [unit][src * 2 + half]
struct XArgs {
  float* in[kXMaxRanks];    // rank p's partial staging [src][unit][kXPSlot]
  float* out[kXMaxRanks];   // rank p's gred | small messages | flags
  unsigned* status;         // local error word (a bounded wait expired)
  unsigned long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
  int world, rank;          // world <= 1: not sharded
  int gbf16;                // DAMD_GRAD_DTYPE=bf16: partials and reduced units travel as bf16
  int ppb;                  // pooled positions per bwd slice (units are 4 per bwd slice)
};
constexpr long kXG16 = kXFlags + 16384;  // out: bf16 reduced dW1 [5408][64] (DAMD_GRAD_DTYPE=bf16)
// floats of `out` the exchange needs for nunits units (<= 909 units: the flag area)
inline long convnet_xout_floats(int nunits) { return kXG16 + 5408L * 64 / 2; }
inline long convnet_xin_floats(int world, int nunits) { return (long)world * nunits * kXPSlot; }
// X / labels are the epoch-permuted copies of the dataset (row g = global sample g).
struct ConvNetBuffers {
  const void* X; const int* labels;  // X: fp32 [n][784], or uint8 [n][784] when x_u8
  int x_u8;
  float* P; float* G; float* V; Ctrl* ctrl;
  float* W1alt; float* V1alt; uint16_t* w1bf;  // W1 double buffer (fp32, velocity) + bf16 copy
  uint16_t* pooled /* [5408][BP] */; uint8_t* code /* [B][5408] */;
  unsigned long long* stamps;  // optional [3][256][16] phase stamps (diagnostics), may be null
  // fixed-point accumulators of the cross-block sums
  long long* hacc;   // [2][B] rows of 64 dense-1 pre-activations x 2^32 (pitch HACC_PITCH), by step parity
  long long* hconv;  // [2][320] conv weight/bias gradient x 2^40, by step parity (both all-reduced)
  float* calt;       // [2][320] alternate conv parameters / velocity (double buffer by parity)
  // no gradient all-reduce (world 1): bwd applies the W1 update as soon as its block has
  // the slice's gradient (fp32 master + velocity in place, bf16 copy); fwd then reads only
  // the bf16 copy.  0: the update is deferred into the next fwd (after the all-reduce of G)
  int eager_w1;
  // read side of the gradient when the peer all-reduce is folded into the step (the
  // all-reduce's `out` staging; G / hconv are then its `in` staging, written by bwd):
  // fwd, bwd's metric fold and flush read Gr / hconv_r.  Null: G / hconv.
  float* Gr;
  long long* hconv_r;
  // sharded multi-rank step (world > 1): the exchange staging of every rank; null otherwise.
  // Then Gr = this rank's gradient staging and hconv_r = the conv-gradient sums that
  // convnet2_launch_gather fills for flush / the host
  const XArgs* xa;
  // next-batch prefetch (B <= 64; both may be null = off): the backward of step t copies the
  // input rows of step t + 1 into xnext ([B][784] in X's dtype) and tags them in *xtag with
  // (ctrl.xgen << 32) | (cursor + 1); the forward of step t + 1 loads them before it has
  // read the ctrl block and keeps them when the tag matches (else it loads X as before)
  void* xnext;
  long long* xtag;
  // this step's rows and labels as the forward read them ([B][784] in X's dtype, [B] int32,
  // -1 = no row): the backward reads them there instead of through the ctrl block's cursor
  // (both may be null = off; used together with xnext)
  void* xcur;
  int* ycur;
  // the step parity (ctrl.wpar) the host expects at this launch, or -1 = unknown: with it
  // the kernels address the parity buffers before the ctrl block arrives (a mismatch with
  // ctrl.wpar -- a host bookkeeping bug -- raises ctrl.bad: the loss reads NaN)
  int par_hint;
  // pooled positions per slice of the backward kernel (0: the forward's PP).  The forward
  // runs 4 image groups per slice (a 228-block grid at PP 3); the backward has one block per
  // slice, so a finer slicing spreads its dW1 / dP / conv-gradient work over more CUs
  int ppb;
};
constexpr int kConvNetNConv = 320;
constexpr int kConvNetNParam = 347146;
constexpr int kConvNetNGrad = 347152;
int convnet_num_slices(int PP);
long convnet_hacc_elems(int B);
int convnet_f1_lg(int B);
size_t convnet2_fwd_lds(int PP, int lg);
size_t convnet2_bwd_lds(int PP);
hipError_t convnet2_launch_step(const ConvNetBuffers& b, int B, int PP, hipStream_t st);
// the two launches separately (phase timing)
hipError_t convnet2_launch_fwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st);
hipError_t convnet2_launch_bwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st);
hipError_t convnet2_launch_flush(const ConvNetBuffers& b, int B, hipStream_t st);
// sharded step: gather the pending update's reduced small gradients (before flush / host reads)
hipError_t convnet2_launch_gather(const ConvNetBuffers& b, int PP, hipStream_t st);
hipError_t convnet2_set_lds_limits();
// elements of the all-reduced gradient buffer
size_t convnet_grad_count(int PP);
}  // namespace damd
