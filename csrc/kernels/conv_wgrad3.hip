// Direct 3x3 / stride-1 / pad-1 convolution weight gradient (gfx950 / MI355X): all nine
// filter taps of a 64(ci) x 64(co) tile from ONE pass over the block's pixels.
//
//   dW[kh][kw][ci][co] = sum_{n,oh,ow} x[n][oh+kh-1][ow+kw-1][ci] * dy[n][oh][ow][co]
//
// The implicit-GEMM weight gradient (conv_gemm.hip wgrad_kernel, gemm.hip A_WGRAD) treats
// (kh,kw,ci) as the GEMM's M: every M-tile re-reads dy and every tap re-gathers x, so the
// 3x3 layers ran at 200-300 TFLOP/s, bound by those re-reads (scripts/bench_gemm.py,
// profiles/r02_resnet18/conv_gemm_layers.txt).  Here a block keeps a sliding window of x
// rows in LDS and the nine taps are nine constant row shifts of that window:
//
//   "q space": virtual pixels q = ((n*(H+1) + r) * P + c), pitch P = W + 1, r in [0, H]
//   (r == H: a zero row shared by consecutive images), c in [0, P) (c == W: zero column).
//   x and dy are both laid out on q; for a dy pixel at q the tap (kh, kw) operand is the x
//   pixel at q + (kh-1)*P + (kw-1) -- the zero column/row supply the padding, for the left
//   and top edges through the previous row/image's zero column/row.  Junk q (c == W or
//   r == H) carry dy = 0.  MFMA work is (H+1)(W+1)/(HW) of the useful: 1.04x at 56x56.
//
// Block: a 64(ci) x 64(co) tile for all nine taps, 9 waves (below).  Per 32-pixel
// k-step the block DMAs (global_load_lds, lane-linear, source-side swizzle) one 32-row x
// block into a ring and one dy block into an S-stage buffer; one barrier per k-step.
// Both operands are read with ds_read_b64_tr_b16 at a row base that is NOT 32-aligned
// (the tap shift), so the swizzle is chosen to be conflict-free for every base: 16-byte
// chunk c of ring row R sits at c ^ swz(R), swz(R) = 2*(((R>>1)&1) | (((R>>3)&1)<<1)) -- within each 32-lane half of
// a transposed read (rows b+i and b+8+i, i < 4) the rows of equal parity get four
// distinct chunk pairs for any b (exhaustively checked offline for ring sizes that are
// multiples of 16).
// GemmArgs: A = x, B = dy, C = slab/out fp32 [9*Cin][Cout], M = 9*Cin, N = Cout,
// K = Q = Nimg*(H+1)*(W+1), k_per_split multiple of 32, Cin/H/W as the conv geometry.
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace damd {
namespace {

__device__ __attribute__((aligned(64))) uint4 w3_zero16[4];

__device__ __forceinline__ int w3_swz(int R) { return (((R >> 1) & 1) | (((R >> 3) & 1) << 1)) << 1; }

// the two transposed reads of one fragment (gemm_tile.h frag_mc register layout)
__device__ __forceinline__ bf16x8 w3_pair(const char* lo, const char* hi) {
  tile::s16x4 l = tile::ds_tr16(lo), h = tile::ds_tr16(hi);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  return __builtin_bit_cast(bf16x8, v);
}

struct QGeo {
  int P, H1, H, W, Q;
  float invP, invH1;
};

// source of one 16-byte chunk of q-row q (channel offset ch0 + 8*chunk): nullptr if zero
__device__ __forceinline__ const uint16_t* w3_src(const uint16_t* base, const QGeo& g, int q, int C, int ch0,
                                                  int chunk) {
  if ((unsigned)q >= (unsigned)g.Q) return nullptr;
  const int v = (int)(((float)q + 0.5f) * g.invP);  // exact for q < 2^21 (host-checked)
  const int c = q - v * g.P;
  const int n = (int)(((float)v + 0.5f) * g.invH1);
  const int r = v - n * g.H1;
  if (r >= g.H || c >= g.W) return nullptr;
  return base + ((long)(n * g.H + r) * g.W + c) * C + ch0 + 8 * chunk;
}

// s_waitcnt vmcnt(min(ahead, S - 2)): the DMA issues this wave may leave in flight
template <int S>
__device__ __forceinline__ void w3_wait_vm(int ahead) {
  if (S >= 8 && ahead >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (S >= 7 && ahead >= 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (S >= 6 && ahead >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (S >= 5 && ahead >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (S >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (S >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Wave t = tap t: the whole 64x64 tile, 16 MFMAs and 16 transposed reads per k-step.
// Every read address is a per-lane constant (set up once: the swizzle of a ring row depends
// on its row mod 16 only, and k-steps advance the ring by 32 rows) plus, for x, the ring
// offset of the k-step (2 VALU per row pair) and, for dy, the stage as an immediate (the
// loop is unrolled by S) -- the first version computed every address per read and issued
// ~5.6 VALU per MFMA (SQ_INSTS_VALU / SQ_INSTS_MFMA), which bound it.  Waves 0-3 DMA the
// x block, 4-7 the dy block (one 1-KB DMA each per k-step).  S-stage pipeline: issue(kt)
// = x block kt+2D + dy step kt, S-1 issues in flight, counted vmcnt.
// Diagnostics (wgrad3_stamps_enable): per block s_memrealtime at start, first k-step's
// operands landed, k-loop done, end -> g_w3_st[block][4]
constexpr int kW3StampBlocks = 4096;
__device__ int g_w3_on;
__device__ unsigned long long g_w3_st[kW3StampBlocks][4];

template <int S, int EPI>
__global__ __launch_bounds__(576) void wgrad3_kernel(GemmArgs a) {
  const bool stamps = g_w3_on != 0;
  unsigned long long st0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull, st1 = 0ull, st2 = 0ull;
  constexpr int XB = (S <= 4 ? 8 : 16) * 32 * 128, DB = S * 32 * 128;  // x ring: 2D + S blocks (power of 2)
  __shared__ __attribute__((aligned(1024))) char smem[XB + DB];
  char* xring = smem;
  char* dyb = smem + XB;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int Cin = a.Cin, Cout = a.N;
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64;

  QGeo g;
  g.P = a.W + 1;
  g.H1 = a.H + 1;
  g.H = a.H;
  g.W = a.W;
  g.Q = a.K;
  g.invP = 1.f / (float)g.P;
  g.invH1 = 1.f / (float)g.H1;
  const int qa = blockIdx.z * a.k_per_split;
  const int qb = min(g.Q, qa + a.k_per_split);
  const int nk = (qb - qa + 31) >> 5;
  const int D = (g.P + 1 + 31) >> 5;  // x blocks of look-back / look-ahead (<= 2)
  const int xq0 = qa - 32 * D;        // q of x block 0
  int nbx = 4;
  while (nbx < 2 * D + S) nbx <<= 1;
  const int xmask = nbx * 32 - 1, rbm = nbx * 4096 - 1;

  const uint16_t* xs = (const uint16_t*)a.A;
  const uint16_t* dys = (const uint16_t*)a.B;
  const int lrow = lane >> 3, lslot = lane & 7;
  const void* zero = tile::pinned_addr(w3_zero16);

  auto issue_x = [&](int j, int part) __attribute__((always_inline)) {
    const int R = ((j * 32) & xmask) + 8 * part + lrow;  // ring row
    const int q = xq0 + 32 * j + 8 * part + lrow;
    const uint16_t* p = w3_src(xs, g, q, Cin, ci0, lslot ^ w3_swz(R));
    tile::glds16(p ? (const void*)p : zero, xring + (R - lrow) * 128);
  };
  auto issue = [&](int kt, int stage) __attribute__((always_inline)) {
    if (wave < 4) {
      issue_x(kt + 2 * D, wave);
    } else if (wave < 8) {
      const int part = wave - 4, R = stage * 32 + 8 * part + lrow;
      const int q = qa + 32 * kt + 8 * part + lrow;
      const uint16_t* p = q < qb ? w3_src(dys, g, q, Cout, co0, lslot ^ w3_swz(R)) : nullptr;
      tile::glds16(p ? (const void*)p : zero, dyb + (R - lrow) * 128);
    }
  };
  if (wave < 8)
    for (int i = wave; i < 8 * D; i += 8) issue_x(i >> 2, i & 3);
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);

  // per-lane read offsets: lane (g4, qq, p) reads rows 8 g4 + qq (lo) and +4 (hi) of the
  // fragment, columns 16 f + 4p .. +3 (f = 16-column group: ci for x, co for dy)
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int kh = wave / 3, kw = wave - 3 * kh;
  const int xr = 32 * D + (kh - 1) * g.P + (kw - 1) + 8 * g4 + qq;  // >= 0: ring row at kt = 0
  const int xlo0 = xr * 128, xhi0 = (xr + 4) * 128;
  int xcl[4], xch[4], dl[4], dh[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int ch = 2 * f + (pp >> 1), half = 8 * (pp & 1);
    xcl[f] = 16 * (ch ^ w3_swz(xr)) + half;
    xch[f] = 16 * (ch ^ w3_swz(xr + 4)) + half;
    const int dr = 8 * g4 + qq;
    dl[f] = dr * 128 + 16 * (ch ^ w3_swz(dr)) + half;
    dh[f] = (dr + 4) * 128 + 16 * (ch ^ w3_swz(dr + 4)) + half;
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto step = [&](auto stg, int kt) __attribute__((always_inline)) {
    constexpr int ST = decltype(stg)::value;
    const int ahead = min(nk - 1 - kt, S - 2);  // issues in flight beyond kt (1 DMA each)
    w3_wait_vm<S>(ahead);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (stamps && kt == 0) st1 = __builtin_amdgcn_s_memrealtime();
    if (kt + S - 1 < nk) issue(kt + S - 1, (ST + S - 1) % S);
    const int blo = (kt * 4096 + xlo0) & rbm, bhi = (kt * 4096 + xhi0) & rbm;
    const char* dstg = dyb + ST * 4096;
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      af[f] = w3_pair(xring + blo + xcl[f], xring + bhi + xch[f]);
      bfr[f] = w3_pair(dstg + dl[f], dstg + dh[f]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
  };
  for (int kt = 0; kt < nk; kt += S) {
    step(std::integral_constant<int, 0>{}, kt);
    if constexpr (S > 1) if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
    if constexpr (S > 2) if (kt + 2 < nk) step(std::integral_constant<int, 2 % S>{}, kt + 2);
    if constexpr (S > 3) if (kt + 3 < nk) step(std::integral_constant<int, 3 % S>{}, kt + 3);
    if constexpr (S > 4) if (kt + 4 < nk) step(std::integral_constant<int, 4 % S>{}, kt + 4);
    if constexpr (S > 5) if (kt + 5 < nk) step(std::integral_constant<int, 5 % S>{}, kt + 5);
    if constexpr (S > 6) if (kt + 6 < nk) step(std::integral_constant<int, 6 % S>{}, kt + 6);
    if constexpr (S > 7) if (kt + 7 < nk) step(std::integral_constant<int, 7 % S>{}, kt + 7);
  }
  if (stamps) st2 = __builtin_amdgcn_s_memrealtime();
  // wave tile: rows m = tap*Cin + ci0 .. +63, columns co0 .. +63
  tile::epilogue<64, 64, EPI>(a, acc, wave * Cin + ci0, co0, 0, 0, 0, wave, lane, nullptr);
  if (stamps && threadIdx.x == 0) {
    const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (b < kW3StampBlocks) {
      g_w3_st[b][0] = st0;
      g_w3_st[b][1] = st1;
      g_w3_st[b][2] = st2;
      g_w3_st[b][3] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

int w3_env(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

}  // namespace

// pipeline depth (2..4): env DAMD_WGRAD3_STAGES.  3 measured best on the ResNet-18 step
// once the LDS-DMA issue moved to inline asm (2.85 vs 2.89 ms/step with 2, 2.85 with 4)
int w3_stages() { return std::min(8, std::max(2, w3_env("DAMD_WGRAD3_STAGES", 3))); }

hipError_t wgrad3_stamps_enable(int on) {
  if (on) {
    static unsigned long long zeros[kW3StampBlocks][4];
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_w3_st), zeros, sizeof(zeros));
    if (e != hipSuccess) return e;
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_w3_on), &on, sizeof(int));
}
hipError_t wgrad3_stamps_read(unsigned long long* host, int blocks) {
  if (blocks > kW3StampBlocks) blocks = kW3StampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w3_st), (size_t)blocks * 4 * sizeof(unsigned long long));
}
int wgrad3_rows(int N, int H, int W) { return N * (H + 1) * (W + 1); }

hipError_t wgrad3_launch(const GemmArgs& a, int epi, int splits, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 || a.Ho != a.H || a.Wo != a.W) return hipErrorInvalidValue;
  if (a.Cin % 64 || a.N % 64 || a.M != 9 * a.Cin || a.W + 1 > 63 || a.H < 1 || a.W < 1) return hipErrorInvalidValue;
  const int per_img = (a.H + 1) * (a.W + 1);
  if (a.K % per_img || a.K + 64 * 32 >= (1 << 21)) return hipErrorInvalidValue;
  if (splits < 1 || a.k_per_split < 32 || a.k_per_split % 32 || (long)splits * a.k_per_split < a.K ||
      (long)(splits - 1) * a.k_per_split >= a.K)
    return hipErrorInvalidValue;
  const int st = w3_stages();
  dim3 grid(a.N / 64, a.Cin / 64, splits);
  if (epi != E_SLAB && epi != E_ATOMIC) return hipErrorInvalidValue;
#define W3_LAUNCH(S_)                                                                             \
  hipLaunchKernelGGL((epi == E_SLAB ? wgrad3_kernel<S_, E_SLAB> : wgrad3_kernel<S_, E_ATOMIC>), grid, \
                     dim3(576), 0, s, a)
  switch (st) {
    case 2: W3_LAUNCH(2); break;
    case 3: W3_LAUNCH(3); break;
    case 4: W3_LAUNCH(4); break;
    case 5:
    case 6: W3_LAUNCH(6); break;
    default: W3_LAUNCH(8); break;
  }
#undef W3_LAUNCH
  return hipGetLastError();
}

}  // namespace damd
