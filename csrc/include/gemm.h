// Generic bf16 MFMA GEMM / implicit-GEMM convolution (csrc/kernels/gemm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "layer_ops.h"

namespace damd {

enum GemmAMode { A_KC = 0, A_IM2COL = 1, A_DGRAD = 2, A_MC = 3, A_WGRAD = 4,
                 // glds-staged BK=64 conv kernels (csrc/kernels/conv_gemm.hip): gathered
                 // channel count % 64 == 0; A_DGRAD64 stride 1 only
                 A_CONV64 = 5, A_DGRAD64 = 6,
                 // weight gradient over "virtual rows" (conv_gemm.hip): K = virtual rows
                 A_WGRAD64 = 7,
                 // conv_wgrad3.hip: direct 3x3/s1/p1 weight gradient (all taps per block)
                 A_WGRAD3 = 8,
                 // conv3x3.hip: direct 3x3/s1/p1 forward / backprop-input (input halo in LDS)
                 A_CONV3 = 9, A_DGRAD3 = 10 };
enum GemmBMode { B_NC = 0, B_KC = 1 };
// E_SLAB: split-K partial of split z stored (plain fp32 stores) to C + z * M * ldc; a
// deterministic splitk_reduce then adds the slabs into the destination in fixed order.
// E_BNRED: the GEMM produces the gradient of a BN -> ReLU output (backprop-input of the
// conv that consumes it): the tile's BN-backward partials (sum of the ReLU-masked stored
// gradient, and of it times xhat, from bnx / bnst) go to `stats` as E_STATS would
// E_FIXUP (conv_gemm.hip, split-K): every split stores its fp32 partial to slab z, the
// tile's LAST-arriving split (per-tile ticket) sums slabs 0..S-1 in order and runs the
// epilogue of the other flags itself -- no separate splitk_finish launch
enum GemmEpi { E_BIAS = 1, E_RELU = 2, E_BF16 = 4, E_ATOMIC = 8, E_STATS = 16, E_ADD = 32, E_SLAB = 64, E_BNRED = 128,
               E_FIXUP = 256 };

struct GemmArgs {
  const void* A;       // bf16
  const void* B;       // bf16
  void* C;             // fp32 or bf16 (E_BF16)
  const float* bias;   // [N] (E_BIAS)
  float* stats;        // [M-tiles][splits][2][N] partial column sum / sumsq (E_STATS)
  const void* R;       // bf16 [M][ldc] added to the result (E_ADD; may alias C)
  int M, N, K;
  int lda, ldb, ldc;
  // convolution geometry (A_IM2COL / A_DGRAD / A_WGRAD):
  //   x [Nimg][H][W][Cin], y [Nimg][Ho][Wo][Cout], kernel KHxKW, stride, pad (top/left)
  //   A_DGRAD: Cin = Cout (the gathered tensor's channel count)
  int H, W, Cin, Ho, Wo, KH, KW, stride, pad;
  int kc;              // B_KC: inner k length per tap
  int k_per_split;     // multiple of 32
  int kstep;           // conv_gemm.hip k-step depth: 32 | 64 (0: DAMD_CONV_KB / 64)
  long long* stats_acc;  // E_STATS: non-null -> the tile's column sum / sumsq are added (bnacc_add
                       // atomics) into stats_acc[reps][2][N] (+ the sticky flag plane after the replicas) instead of stored to `stats`:
  int stats_reps;      //   M-tile tm into replica tm % reps (0 / 1: one), see layer_ops.h BNFin
  const uint16_t* bnx; // E_BNRED: the BN input x [M][ldc] bf16 and its st [4][N] (mean,
  const float* bnst;   //   invstd, scale, shift)
  // A_CONV3 forward, bnin.acc non-null: A is a BatchNorm's INPUT; the kernel finalizes its
  // statistics (bnin, as the apply kernels do: block (0, 0) publishes st / moving stats) and
  // normalises + ReLUs the staged halo in LDS (bitwise bn_apply's values); the blocks of
  // N-tile 0 also store that BN -> ReLU output to bnin_y (for the conv's weight gradient).
  BNFin bnin;
  uint16_t* bnin_y;
  // E_FIXUP: fp32 slabs [splits][M][N] and one arrival ticket per output tile (zero between
  // launches: the reducing split resets its tile's)
  float* slab;
  unsigned* tickets;
};

// tile: 0 -> 128x128 tiles, 1 -> 256x64 tiles (N <= 64 layers)
hipError_t gemm_launch(const GemmArgs& a, int amode, int bmode, int epi, int splits, int tile, hipStream_t s);
// conv_gemm.hip: A_CONV64 (with B_NC weights) / A_DGRAD64 (with B_KC weights) /
// A_WGRAD64 (B_NC = dy; K = wgrad64_rows, k_per_split a multiple of wgrad64_rows_per_step)
hipError_t conv_gemm_launch(const GemmArgs& a, int amode, int epi, int splits, int tile, hipStream_t s);
int wgrad64_rows(int N, int Ho, int Wo, int kstep);
// A_WGRAD3: K = wgrad3_rows (q space), k_per_split a multiple of 32, tiles 64x64 x 9 taps
hipError_t wgrad3_launch(const GemmArgs& a, int epi, int splits, hipStream_t s);
int wgrad3_rows(int N, int H, int W);
hipError_t wgrad3_stamps_enable(int on);                              // diagnostics
hipError_t wgrad3_stamps_read(unsigned long long* host, int blocks);  // [blocks][4]
// A_CONV3 / A_DGRAD3: tile 1 -> BN 64 (256 x 64), 0 -> BN 128 (128 x 128); output rows per
// block for an H x W image (0: not supported); stats partials = Nimg * ceil(H / rows)
hipError_t conv3_launch(const GemmArgs& a, int dgrad, int epi, int bn, hipStream_t s);
int conv3_rows(int H, int W, int bn);
// conv3r.hip: the persistent weight-stationary variant for 64 -> 64 channels (layer 1)
int conv3r_ok(const GemmArgs& a, int dgrad);
hipError_t conv3r_launch(const GemmArgs& a, int dgrad, int epi, hipStream_t s);
// conv_stem.hip: the direct packed-tap stem forward (A_CONV64 with Cin == 4; 0: not taken)
int stem_direct_ok(const GemmArgs& a, int epi, int splits);
hipError_t stem_direct_launch(const GemmArgs& a, int epi, hipStream_t s);
hipError_t stem_stamps_enable(int on);                              // diagnostics
hipError_t stem_stamps_read(unsigned long long* host, int blocks);  // [blocks][8]
hipError_t conv3_stamps_enable(int on);                              // diagnostics
hipError_t conv3_stamps_read(unsigned long long* host, int blocks);  // [blocks][4]
int wgrad64_rows_per_step(int Wo, int kstep);
// k-step depth of those kernels (32 or 64, env DAMD_CONV_KB): the gathered channel count
// must be a multiple of it for A_CONV64 / A_DGRAD64
int conv_gemm_kstep();
int gemm_stats_tile_rows(int tile);
// dst[i] (+)= sum_{s < splits} slab[s * n + i]  (fp32, n % 4 == 0, fixed summation order);
// accumulate = 0 overwrites dst (no zeroing pass before a first writer)
hipError_t splitk_reduce(const float* slab, int splits, long n, float* dst, hipStream_t s, int accumulate = 1);
// splitk_reduce from a padded [R][C1p][C2p] slab layout into dst [R][C1][C2] (junk dropped)
hipError_t splitk_reduce_unpad(const float* slab, int splits, int R, int C1, int C2, int C1p, int C2p, float* dst,
                               hipStream_t s, int accumulate);
// bf16 split-K epilogue: out = relu?(sum_s slab[s] + bias + R) (R bf16 [M][ldc], may alias
// out); stats (optional) = per-column sum / sumsq of the stored pre-ReLU values per block
// of rows_per_block rows: [ceil(M / rows_per_block)][2][N]
hipError_t splitk_finish(const float* slab, int splits, int M, int N, const float* bias, const uint16_t* R, int relu,
                         float* stats, int rows_per_block, uint16_t* out, int ldc, hipStream_t s,
                         long long* stats_acc = nullptr, int stats_reps = 1);
// fp32 split-K epilogue (dense logits): out[m][n] = relu?(sum_s slab[s][m][n] + bias[n]),
// slab [splits][M][N], out pitch ldc, fixed summation order
hipError_t splitk_finish_f32(const float* slab, int splits, int M, int N, const float* bias, int relu, float* out,
                             int ldc, hipStream_t s);

}  // namespace damd
