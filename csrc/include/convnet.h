// Host interface of the fused MNIST-CNN step kernels (csrc/kernels/convnet_step2.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace damd {
struct Ctrl;
// X / labels are the epoch-permuted copies of the dataset (row g = global sample g).
struct ConvNetBuffers {
  const void* X; const int* labels;  // X: fp32 [n][784], or uint8 [n][784] when x_u8
  int x_u8;
  float* P; float* G; float* V; Ctrl* ctrl;
  float* W1alt; float* V1alt; uint16_t* w1bf;  // W1 double buffer (fp32, velocity) + bf16 copy
  uint16_t* pooled /* [5408][BP] */; uint8_t* code /* [B][5408] */;
  unsigned long long* stamps;  // optional [3][256][16] phase stamps (diagnostics), may be null
  // fixed-point accumulators of the cross-block sums
  long long* hacc;   // [2][B][64] dense-1 pre-activations x 2^32, by step parity
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
};
constexpr int kConvNetNConv = 320;
constexpr int kConvNetNParam = 347146;
constexpr int kConvNetNGrad = 347152;
int convnet_num_slices(int PP);
int convnet_f1_lg(int B);
size_t convnet2_fwd_lds(int PP, int lg);
size_t convnet2_bwd_lds(int PP);
hipError_t convnet2_launch_step(const ConvNetBuffers& b, int B, int PP, hipStream_t st);
// the two launches separately (phase timing)
hipError_t convnet2_launch_fwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st);
hipError_t convnet2_launch_bwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st);
hipError_t convnet2_launch_flush(const ConvNetBuffers& b, int B, hipStream_t st);
hipError_t convnet2_set_lds_limits();
// elements of the all-reduced gradient buffer
size_t convnet_grad_count(int PP);
}  // namespace damd
