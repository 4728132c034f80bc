// Persistent, weight-stationary direct 3x3 / stride-1 / pad-1 convolution for 64 -> 64
// channels (ResNet-18 layer 1: 56 x 56 x 64, forward and backprop-input) on gfx950.
//
// Why a second direct kernel (conv3x3.hip is the general one): its blocks run the three
// phases of a tile in lock step -- every resident block fetches its halo (HBM-bound, the
// MFMAs idle), runs the nine taps (memory idle), then stores (3.9 / 6.5 / 3.5 us per round
// on layer 1, BENCH.md round 4) -- and at 896 blocks over 512 slots the rounds quantise.
// Layer 1 was ~37 us per conv against ~9 us of HBM traffic and ~7 us of MFMA work.
//
// Here each block owns a horizontal STRIP of one image (a run of 4-row tiles, one block per
// CU, grid = images x strips) and keeps for its whole life:
//   * the full 3 x 3 x 64 x 64 filter in LDS (72 KiB, loaded once: weight-stationary), so
//     the 18 k-steps of a tile run back to back without a barrier, the fragment reads of
//     k-step s + 1 issued before the MFMAs of k-step s (software pipelined);
//   * a ring of 10 halo ROWS (8 KiB each: 64 pixels x 64 channels, 16-byte chunk c of
//     pixel q at slot c ^ (q & 7)): a tile needs its 6 halo rows, the next tile's 4 new
//     rows arrive in the other 4 slots while this tile computes -- every input row crosses
//     HBM -> LDS once, and vertically adjacent tiles share their 2 overlap rows.
// Four LOADER waves issue every row DMA after the prologue (one row each, four LDS-DMA
// streams) and wait on their own vmcnt, so the four compute waves' epilogue stores never
// sit in front of a halo wait (in-order vmcnt: the round-4 persistent attempt serialised
// the next halo behind the stores).
// Synchronisation is the workgroup barrier only (no flag polling): per tile A (rows of
// this tile landed -- and, forward with a BN input, transformed to relu(BN(x)) by the loader
// that fetched them, while the compute waves ran the previous tile's taps; the previous
// tile's taps done, so its exclusive rows are free) and the epilogue's statistics barrier
// -- every wave, loader included, passes each one the same number of times (trip counts
// depend on blockIdx only).
//
// Tiles are the 4-row tiles of conv3x3.hip (tile index img * tpi + row block), so the
// statistics partial rows (GemmArgs::stats, stats_T = n * tpi) and the epilogue are shared
// with it bitwise: same fragment layouts, same MFMA order per output element (taps
// ascending, 32-deep k-steps ascending), same tile::epilogue.
#include "bn_fin.h"
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

#include <cstdlib>
#include <type_traits>

namespace damd {
namespace {

constexpr int RNT = 512;               // 4 compute waves + 4 loader waves
constexpr int RR = 4;                  // output rows per tile
constexpr int RING = 10;               // halo row slots: 6 of the tile + 4 incoming
constexpr int SLOT_PX = 64;            // pixels per row slot (W + 2 <= 64)
constexpr int SLOT_B = SLOT_PX * 128;  // 8 KiB
constexpr int WTAP_B = 64 * 64 * 2;    // one tap's [64][64] bf16 weight image
constexpr int OFF_RING = 9 * WTAP_B;   // 72 KiB of weights first
constexpr int OFF_RED = OFF_RING + RING * SLOT_B;
constexpr int OFF_SFT = OFF_RED + 2 * 4 * 64 * 4;
constexpr int LDS_R = OFF_SFT + 2 * 64 * 4;  // 158,208 B: one block per CU
static_assert(LDS_R <= 160 * 1024, "LDS budget");

__device__ __attribute__((aligned(64))) uint4 g_zero16_r[4];

using tile::glds16;

__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool DGRAD, int EPI>
__global__ __launch_bounds__(RNT, 1) void conv3r_kernel(GemmArgs a, int tpi, int S) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int H = a.H, W = a.W;
  const int img = blockIdx.x / S, sidx = blockIdx.x - img * S;
  const int tk0 = sidx * tpi / S, tk1 = (sidx + 1) * tpi / S;  // this block's tiles [tk0, tk1)
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool loader = wave >= 4;
  const int ldr = wave - 4;  // loader index: rows ir with ir % 4 == ldr
  const uint16_t* src = (const uint16_t*)a.A + (long)img * H * W * 64;
  const uint16_t* wsrc = (const uint16_t*)a.B;
  const void* zero = tile::pinned_addr(g_zero16_r);
  char* wts = smem;
  char* ring = smem + OFF_RING;
  float* red = reinterpret_cast<float*>(smem + OFF_RED);
  float* sft = reinterpret_cast<float*>(smem + OFF_SFT);
  const int base = tk0 * RR - 1;  // input row held by ring slot 0 (slot = (row - base) mod RING)
  auto slot_of = [&](int ir) __attribute__((always_inline)) { return (ir - base) % RING; };
  // 1 KiB piece j (0..7) of input row ir: pixels 8j .. 8j + 7 of its slot (slot pixel 0 =
  // the left padding column, 1..W the row, the rest zero)
  auto row_piece = [&](int ir, int j) __attribute__((always_inline)) {
    const int qs = 8 * j + (lane >> 3), col = qs - 1;
    const bool ok = (unsigned)ir < (unsigned)H && (unsigned)col < (unsigned)W;
    const int cs = (lane & 7) ^ (lane >> 3);  // (q & 7) = (8j + lane / 8) & 7
    const void* p = ok ? (const void*)(src + ((long)ir * W + col) * 64 + 8 * cs) : zero;
    glds16(p, ring + slot_of(ir) * SLOT_B + j * 1024);
  };
  // weight piece j (0..71): tap j / 8, 1 KiB piece j % 8 of its [64][64] image (backprop-
  // input: W[tap][ci][co] is already the [n = ci][k = co] k-contiguous operand)
  auto w_piece = [&](int j) __attribute__((always_inline)) {
    const int tap = j >> 3, p = j & 7;
    const int n = 8 * p + (lane >> 3);
    const int ca = (lane & 7) ^ (n & 7);  // kc64 swizzle: chunk c of row n at slot c ^ (n & 7)
    glds16(wsrc + (long)tap * 4096 + n * 64 + 8 * ca, wts + tap * WTAP_B + p * 1024);
  };
  // forward: W[tap][ci][co] is [k][n]; the image is stored TRANSPOSED, [n = co][k = ci] with
  // the same kc64 swizzle, so both directions read B fragments as one ds_read_b128 (the
  // transpose reads of an MC image cost the compiler register copies and spills here).
  // Thread unit u: the 8 x 8 block (tap, ci0..+7, co0..+7): 8 global 16-B rows in, 8 LDS
  // 16-B rows out.
  auto w_transpose = [&](int u) __attribute__((always_inline)) {
    const int tap = u >> 6, ci0 = 8 * ((u >> 3) & 7), co0 = 8 * (u & 7);
    uint4 r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = *reinterpret_cast<const uint4*>(wsrc + (long)(tap * 64 + ci0 + i) * 64 + co0);
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // output row co0 + c: the 8 ci values of column c
      uint32_t w[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t* a0 = reinterpret_cast<const uint32_t*>(&r[2 * h]);
        const uint32_t* a1 = reinterpret_cast<const uint32_t*>(&r[2 * h + 1]);
        const uint32_t lo = (c & 1) ? (a0[c >> 1] >> 16) : (a0[c >> 1] & 0xffffu);
        const uint32_t hi = (c & 1) ? (a1[c >> 1] & 0xffff0000u) : (a1[c >> 1] << 16);
        w[h] = lo | hi;
      }
      const int n = co0 + c;
      *reinterpret_cast<uint4*>(wts + tap * WTAP_B + n * 128 + 16 * ((ci0 >> 3) ^ (n & 7))) =
          uint4{w[0], w[1], w[2], w[3]};
    }
  };
  auto tile_rows = [&](int k) __attribute__((always_inline)) { return min(RR, H - k * RR); };
  // ---- prologue: weights + the first tile's halo rows, spread over all five waves -----
  {
    const int r0 = tk0 * RR - 1, nr = tile_rows(tk0) + 2;
    const int nw = DGRAD ? 72 : 0;  // forward: the weights are transposed below
    const int npieces = nw + nr * 8;
    for (int j = wave; j < npieces; j += 8) {
      if (j < nw) w_piece(j);
      else row_piece(r0 + (j - nw) / 8, (j - nw) & 7);
    }
    if constexpr (!DGRAD)
      for (int u = t; u < 9 * 64; u += RNT) w_transpose(u);
  }
  // BatchNorm on the input (forward, a.bnin): scale / shift of the 64 channels once
  const bool bnin = !DGRAD && a.bnin.acc != nullptr;
  if (bnin && t < 64) {
    double s, q;
    float m, inv, sc, sh;
    acc_sums(a.bnin.acc, a.bnin.reps, 64, t, s, q);
    bn_fin_sums(a.bnin, 64, t, s, q, blockIdx.x == 0, m, inv, sc, sh);
    sft[t] = sc;
    sft[64 + t] = sh;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

  // BN input: y = bf16(relu(x * scale + shift)) in place over the in-image pixels of rows
  // [lo, hi] (the padding stays zero: it is y's padding), exactly bn_apply's arithmetic, by
  // threads tid0, tid0 + nth, ...; the transformed 16-byte units of rows inside this strip's
  // output rows [ylo, yhi) also go to y (the BN -> ReLU output, for the conv's weight
  // gradient): every y row is stored once, by the block and at the moment it is transformed
  const int ylo = tk0 * RR, yhi = min(tk1 * RR, H);
  auto transform_rows = [&](int lo, int hi, int tid0, int nth) __attribute__((always_inline)) {
    lo = max(lo, 0);
    hi = min(hi, H - 1);
    const int units = (hi - lo + 1) * W * 8;
    for (int u = tid0; u < units; u += nth) {
      const int sl = u & 7, px = u >> 3;
      const int r = lo + px / W, c = px - (px / W) * W;
      const int q = c + 1;  // pixel within the slot
      char* p = ring + slot_of(r) * SLOT_B + q * 128 + 16 * sl;
      const int ch = 8 * (sl ^ (q & 7));
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo_ = fmaxf(fmaf(__uint_as_float(w[k] << 16), sft[ch + 2 * k], sft[64 + ch + 2 * k]), 0.f);
        const float hi_ =
            fmaxf(fmaf(__uint_as_float(w[k] & 0xffff0000u), sft[ch + 2 * k + 1], sft[64 + ch + 2 * k + 1]), 0.f);
        o[k] = (uint32_t)f2bf(lo_) | ((uint32_t)f2bf(hi_) << 16);
      }
      const uint4 y = uint4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<uint4*>(p) = y;
      if (a.bnin_y && r >= ylo && r < yhi)
        *reinterpret_cast<uint4*>(a.bnin_y + ((long)(img * H + r) * W + c) * 64 + ch) = y;
    }
  };
  // the strip's first tile: its six rows landed in the prologue; every wave transforms
  if (bnin) {
    transform_rows(tk0 * RR - 1, tk0 * RR + tile_rows(tk0), t, RNT);
    bar();
  }

  for (int k = tk0; k < tk1; ++k) {
    const int rk = tile_rows(k), row0 = k * RR;
    // A(k): this tile's rows have landed and are transformed (the loaders did both before
    // this barrier), and every compute wave has finished the previous tile's taps
    bar();
    if (loader) {
      // the next tile's new halo rows (row0 + rk + 1 .. ) into the slots the previous tile
      // alone used
      if (k + 1 < tk1) {
        const int nlo = row0 + rk + 1, nhi = (k + 1) * RR + tile_rows(k + 1);
        // one row (8 pieces) per loader wave: four LDS-DMA streams, each landing in issue
        // order (~25 GB/s per wave) -- a single loader wave's 32 pieces outlasted a tile
        for (int ir = nlo; ir <= nhi; ++ir)
          if ((ir & 3) == ldr)
#pragma unroll
            for (int j = 0; j < 8; ++j) row_piece(ir, j);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's rows landed
        // BN input: the loader that fetched a row transforms it (and stores its y) while the
        // compute waves run this tile's taps -- they no longer stop for a transform pass and
        // a second barrier per tile
        if (bnin)
          for (int ir = nlo; ir <= nhi; ++ir)
            if ((ir & 3) == ldr) transform_rows(ir, ir, lane, 64);
      }
      if constexpr ((EPI & (E_STATS | E_BNRED)) != 0) __syncthreads();  // the epilogue's barrier
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // landed + transformed before A(k + 1)
      continue;
    }
    const int npx = rk * W;
    // groups of 16 output pixels this wave owns (wave-uniform; all-invalid groups skipped)
    const int ng = min(4, max(0, (npx - wave * 64 + 15) / 16));
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // per group: halo row slot byte offsets for the three row offsets d and the column
    // parts for the three column offsets e and both k-steps (swizzled chunk)
    int rbase[4][3], cpart[4][3][2];
    const int g = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = min(wave * 64 + i * 16 + (lane & 15), npx - 1);
      const int r = p / W, c = p - r * W;
#pragma unroll
      for (int d = 0; d < 3; ++d) rbase[i][d] = slot_of(row0 - 1 + r + d) * SLOT_B;
#pragma unroll
      for (int e = 0; e < 3; ++e)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) cpart[i][e][kk] = (c + e) * 128 + 16 * ((4 * kk + g) ^ ((c + e) & 7));
    }
    bf16x8 af[2][4], bfr[2][4];
    // fragments of k-step s (tap s / 2, 32-deep half s % 2) into register set s & 1
    auto load = [&](int s, int NG) __attribute__((always_inline)) {
      const int tap = s >> 1, kk = s & 1;
      const int kh = tap / 3, kw = tap - kh * 3;
      const int d = DGRAD ? 2 - kh : kh, e = DGRAD ? 2 - kw : kw;
      const char* ib = wts + tap * WTAP_B;
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // [n][k] image (both directions): row n, k chunk 4 kk + g
        const int rr = j * 16 + (lane & 15), c = 4 * kk + g;
        bfr[s & 1][j] = *reinterpret_cast<const bf16x8*>(ib + rr * 128 + 16 * (c ^ (rr & 7)));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < NG) af[s & 1][i] = *reinterpret_cast<const bf16x8*>(ring + rbase[i][d] + cpart[i][e][kk]);
    };
    auto mma = [&](int s, int NG) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < NG)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[s & 1][j], af[s & 1][i], acc[i][j]);
    };
    auto taps = [&](auto NGc) __attribute__((always_inline)) {
      constexpr int NG = decltype(NGc)::value;
      load(0, NG);
#pragma unroll
      for (int s = 0; s < 18; ++s) {
        // every read of k-step s + 1 is issued before the MFMAs of k-step s (left to
        // itself the scheduler sank the reads next to their uses: lgkmcnt(0) waits between
        // MFMAs, which one wave per SIMD cannot hide)
        if (s + 1 < 18) load(s + 1, NG);
        __builtin_amdgcn_sched_barrier(0);
        mma(s, NG);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    switch (ng) {
      case 4: taps(std::integral_constant<int, 4>{}); break;
      case 3: taps(std::integral_constant<int, 3>{}); break;
      case 2: taps(std::integral_constant<int, 2>{}); break;
      case 1: taps(std::integral_constant<int, 1>{}); break;
      default: break;
    }
    GemmArgs e = a;
    const int m0 = (img * H + row0) * W;
    e.M = m0 + npx;  // rows past the tile's pixels are masked
    tile::epilogue<256, 64, EPI>(e, acc, m0, 0, img * tpi + k, wave, 0, wave, lane, red);
  }
}

template <bool DG, int EPI>
hipError_t launch_r(const GemmArgs& a, int tpi, int S, int blocks, hipStream_t s) {
  auto k = conv3r_kernel<DG, EPI>;
  static bool attr = false;  // once per instantiation (host-side, before any capture)
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_R);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(RNT), LDS_R, s, a, tpi, S);
  return hipGetLastError();
}

template <bool DG>
hipError_t launch_r_epi(const GemmArgs& a, int epi, int tpi, int S, int blocks, hipStream_t s) {
  switch (epi) {
    case E_BF16: return launch_r<DG, E_BF16>(a, tpi, S, blocks, s);
    case E_BIAS | E_BF16: return launch_r<DG, E_BIAS | E_BF16>(a, tpi, S, blocks, s);
    case E_BIAS | E_RELU | E_BF16: return launch_r<DG, E_BIAS | E_RELU | E_BF16>(a, tpi, S, blocks, s);
    case E_RELU | E_BF16: return launch_r<DG, E_RELU | E_BF16>(a, tpi, S, blocks, s);
    case E_BF16 | E_STATS: return launch_r<DG, E_BF16 | E_STATS>(a, tpi, S, blocks, s);
    case E_BIAS | E_BF16 | E_STATS: return launch_r<DG, E_BIAS | E_BF16 | E_STATS>(a, tpi, S, blocks, s);
    case E_BF16 | E_ADD: return launch_r<DG, E_BF16 | E_ADD>(a, tpi, S, blocks, s);
    case E_BF16 | E_BNRED:
      if constexpr (DG) return launch_r<DG, E_BF16 | E_BNRED>(a, tpi, S, blocks, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// The shapes this kernel takes: 64 -> 64 channels, 3x3 / s1 / p1, W + 2 <= 64, the 4-row
// tiles of conv3x3.hip (R = 4: 256 / W rounded down), DAMD_CONV3R != 0.  (0: not taken.)
int conv3r_ok(const GemmArgs& a, int dgrad) {
  const char* ev = getenv("DAMD_CONV3R");
  if (ev && ev[0] == '0') return 0;
  if (a.Cin != 64 || a.N != 64 || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1) return 0;
  if (dgrad && (a.kc != 64 || a.bnin.acc)) return 0;
  if (a.W + 2 > SLOT_PX || a.H < 1 || a.M % (a.H * a.W)) return 0;
  if (conv3_rows(a.H, a.W, 64) != RR) return 0;  // the same tiles as the general kernel
  return 1;
}

hipError_t conv3r_launch(const GemmArgs& a, int dgrad, int epi, hipStream_t s) {
  if (!conv3r_ok(a, dgrad) || (epi & (E_SLAB | E_ATOMIC))) return hipErrorInvalidValue;
  const int nimg = a.M / (a.H * a.W);
  const int tpi = (a.H + RR - 1) / RR;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  // strips per image: enough blocks for every CU, each strip >= 1 tile
  const int S = max(1, min(tpi, (cus + nimg - 1) / nimg));
  const int blocks = nimg * S;
  return dgrad ? launch_r_epi<true>(a, epi, tpi, S, blocks, s) : launch_r_epi<false>(a, epi, tpi, S, blocks, s);
}

}  // namespace damd
