// Strip-resident direct 3x3 / stride-1 / pad-1 convolution with the weights streamed by a
// loader wave (gfx950): ResNet-18 layers 2 and 3 (28 x 28 x 128, 14 x 14 x 256), forward
// and backprop-input.
//
// The general direct kernel (conv3x3.hip) on these shapes is bound by its stage loop, not
// by the MFMAs (scripts/conv3_probe.py stamps, layer 3 forward: 36 weight stages in
// 25.9 us = 0.72 us per stage against 0.21 us of MFMA work per wave): every stage, each of
// its four waves issues its share of the next weight stage's LDS-DMA (~100-185 cycles per
// piece beside MFMAs), waits for the stage, meets the others at a barrier, then reads
// fragments and computes; and every block re-streams the weights for a 112-126 pixel tile.
//
// Here a block owns one image STRIP (R whole output rows: layer 2 a quarter image, layer 3
// a whole one) and one 64-channel N-tile, the whole strip's accumulators in registers (each
// compute wave up to G = 4 groups of 16 pixels x 64 channels):
//   * the strip's (R + 2) x (W + 2) input halo of one 64-channel chunk is resident in LDS,
//     double-buffered: chunk c + 1 is fetched (by the compute waves, once per chunk) while
//     chunk c is consumed;
//   * four WEIGHT LOADER waves stream the [64 k][64 n] weight stage of every (chunk, tap)
//     through a ring of D stages, D - 1 in flight, each waiting on its own vmcnt (an
//     LDS-DMA stream lands in issue order at ~25 GB/s per wave: a single loader wave
//     starved the stages, layer-3 backprop-input 50.7 vs 27.6 us for the general kernel);
//   * the four compute waves only read fragments and issue MFMAs: one barrier per stage,
//     both 32-deep k-steps' fragments read before the MFMAs.
// So the weights of a block are streamed once for R x W pixels (2-4x the tile of the
// general kernel) and every CU holds one block (grid = images x strips x N-tiles = 256).
// Barrier discipline: every wave passes every barrier (one per stage, one more per chunk
// with a BatchNorm input, the epilogue's); trip counts depend on blockIdx only.
//
// Numerics: same fragment layouts and per-element MFMA order (chunks, then taps, then
// 32-deep k-steps, ascending) as conv3x3.hip, so outputs are bitwise its outputs; the BN
// statistics of the epilogue go to fixed-point accumulators (order-independent), the only
// statistics form taken here.
#include "bn_fin.h"
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

#include <cstdlib>

namespace damd {
namespace {

constexpr int SNT = 512;       // 4 compute waves (+ the halo DMA) + 4 weight-loader waves
constexpr int WST_B = 64 * 64 * 2;  // one weight stage
__device__ __attribute__((aligned(64))) uint4 g_zero16_s[4];

using tile::glds16;

__device__ __forceinline__ void sbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// wait until at most `ahead` weight stages (2 DMA pieces per loader wave each) of this
// wave are outstanding
template <int A>
__device__ __forceinline__ void wait_stages(int ahead) {
  if constexpr (A > 0) {
    if (ahead >= A) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A * 2) : "memory");
      return;
    }
    wait_stages<A - 1>(ahead);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

struct SGeo {
  int R;       // output rows per strip
  int S;       // strips per image
  int NTL;     // N-tiles (N / 64)
  int hbytes;  // one halo buffer (1 KiB multiple)
  int ring;    // byte offset of the weight ring
  int red;     // byte offset of the epilogue's reduction scratch
  int sft;     // byte offset of the BN-input scale / shift
};

template <bool DGRAD, int EPI, int G, int D>
__global__ __launch_bounds__(SNT, 1) void conv3s_kernel(GemmArgs a, SGeo sg) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int H = a.H, W = a.W, SC = a.Cin, N = a.N;
  const int HW = W + 2;
  const int nt = blockIdx.x % sg.NTL;
  const int strip = (blockIdx.x / sg.NTL) % sg.S;
  const int img = blockIdx.x / (sg.NTL * sg.S);
  const int oh0 = strip * sg.R;
  const int reff = min(sg.R, H - oh0);
  const int npx = reff * W;
  const int hpix = (reff + 2) * HW;
  const int n0 = nt * 64;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nch = SC / 64, NS = 9 * nch;
  const uint16_t* src = (const uint16_t*)a.A + (long)img * H * W * SC;
  const uint16_t* wsrc = (const uint16_t*)a.B;
  const void* zero = tile::pinned_addr(g_zero16_s);
  char* ring = smem + sg.ring;
  float* red = reinterpret_cast<float*>(smem + sg.red);
  float* sft = reinterpret_cast<float*>(smem + sg.sft);
  const bool bnin = !DGRAD && a.bnin.acc != nullptr;

  // halo DMA piece j of chunk c: pixels 8j .. 8j + 7 (lane / 8), 16-byte slot lane & 7
  auto halo_piece = [&](int c, int j) __attribute__((always_inline)) {
    const int q = 8 * j + (lane >> 3);
    const int hr = q / HW, hc = q - hr * HW;
    const int ih = oh0 - 1 + hr, iw = hc - 1;
    const bool ok = q < hpix && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    const int cs = (lane & 7) ^ (q & 7);
    const void* p = ok ? (const void*)(src + ((long)ih * W + iw) * SC + c * 64 + 8 * cs) : zero;
    glds16(p, smem + (c & 1) * sg.hbytes + j * 1024);
  };
  // loader wave l's share of weight stage s = (chunk s / 9, tap s % 9): 1 KiB pieces 2l and
  // 2l + 1 of the stage's 8, into ring slot s % D (one LDS-DMA stream lands in issue order
  // at ~25 GB/s per wave: four loader waves, four streams)
  const int ldr = wave - 4;
  auto weight_part = [&](int s) __attribute__((always_inline)) {
    const int c = s / 9, tap = s - c * 9;
    char* dst = ring + (s % D) * WST_B;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = 2 * ldr + u;
      const uint16_t* ptr;
      if constexpr (DGRAD) {  // [n = ci][k = co]: W[tap][n0 + n][c * 64 + k], k-contiguous
        const int n = 8 * p + (lane >> 3);
        const int ca = (lane & 7) ^ (n & 7);
        ptr = wsrc + ((long)tap * N + n0 + n) * a.kc + c * 64 + 8 * ca;
      } else {  // [k = ci][n = co]: W[tap][c * 64 + k][n0 + n], mn-contiguous (MC swizzle)
        const int kr = 8 * p + (lane >> 3);
        const int ch = (lane & 7) ^ tile::mc_swz<64>(kr);
        ptr = wsrc + ((long)tap * SC + c * 64 + kr) * N + n0 + 8 * ch;
      }
      glds16(ptr, dst + p * 1024);
    }
  };
  const int nhp = sg.hbytes / 1024;  // halo pieces per chunk (1 KiB granules, padded)

  // ---- prologue ---------------------------------------------------------------------
  if (wave < 4) {
    for (int j = wave; j < nhp; j += 4) halo_piece(0, j);
  } else {
    for (int s = 0; s < min(D - 1, NS); ++s) weight_part(s);
  }
  if (bnin && t < SC) {  // BatchNorm input: scale / shift of every input channel
    double s, q;
    float m, inv, sc, sh;
    acc_sums(a.bnin.acc, a.bnin.reps, SC, t, s, q);
    bn_fin_sums(a.bnin, SC, t, s, q, blockIdx.x == 0, m, inv, sc, sh);
    sft[t] = sc;
    sft[SC + t] = sh;
  }
  if (wave < 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk 0's halo landed
  else wait_stages<D - 2>(min(D - 1, NS) - 1);                     // stage 0 landed

  // compute waves: per group, the halo pixel of its lanes' output pixel at tap offset 0
  int hbase[G];
  f32x4 acc[G][4];
  const int g = lane >> 4;
  const int ng = wave < 4 ? min(G, max(0, ((npx + 15) / 16) - wave * G)) : 0;  // wave-uniform
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int p = min((wave * G + i) * 16 + (lane & 15), npx - 1);
    const int r = p / W, c = p - r * W;
    hbase[i] = r * HW + c;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  for (int s = 0; s < NS; ++s) {
    const int c = s / 9, tap = s - c * 9;
    sbar();  // stage s (and at a chunk start its halo) landed; stage s - 1 fully consumed
    if (wave >= 4) {
      const int sn = s + D - 1;
      if (sn < NS) weight_part(sn);
      // stage s + 1 landed before the next barrier: leave the later ones in flight
      if (s + 1 < NS) wait_stages<D - 2>(min(sn, NS - 1) - (s + 1));
      if (bnin && tap == 0) sbar();
      continue;
    }
    // compute waves: chunk c + 1's halo into the other buffer (chunk c - 1, its last user,
    // is done), landed before the next chunk's first barrier
    if (tap == 0 && c + 1 < nch)
      for (int j = wave; j < nhp; j += 4) halo_piece(c + 1, j);
    char* hcur = smem + (c & 1) * sg.hbytes;
    if (bnin && tap == 0) {
      // y = bf16(relu(x * scale + shift)) in place over the chunk's in-image halo pixels
      // (exactly bn_apply's arithmetic; the padding stays zero: it is y's padding)
      for (int u = t; u < hpix * 8; u += 256) {
        const int q = u >> 3, sl = u & 7;
        const int hr = q / HW, hc = q - hr * HW;
        const int ih = oh0 - 1 + hr, iw = hc - 1;
        if ((unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)W) continue;
        char* p = hcur + q * 128 + 16 * sl;
        const int ch = c * 64 + 8 * (sl ^ (q & 7));
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = fmaxf(fmaf(__uint_as_float(w[k] << 16), sft[ch + 2 * k], sft[SC + ch + 2 * k]), 0.f);
          const float hi =
              fmaxf(fmaf(__uint_as_float(w[k] & 0xffff0000u), sft[ch + 2 * k + 1], sft[SC + ch + 2 * k + 1]), 0.f);
          o[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
        }
        *reinterpret_cast<uint4*>(p) = uint4{o[0], o[1], o[2], o[3]};
      }
      sbar();
      // the strip's output rows of y (this chunk's 64 channels), N-tile 0 only
      if (nt == 0 && a.bnin_y) {
        uint16_t* yb = a.bnin_y + (long)(img * H + oh0) * W * SC + c * 64;
        for (int u = t; u < npx * 8; u += 256) {
          const int px = u >> 3, cl = u & 7;
          const int r = px / W, cc = px - r * W;
          const int q = (r + 1) * HW + cc + 1;
          *reinterpret_cast<uint4*>(yb + (long)px * SC + 8 * cl) =
              *reinterpret_cast<const uint4*>(hcur + q * 128 + 16 * (cl ^ (q & 7)));
        }
      }
    }
    const char* ib = ring + (s % D) * WST_B;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = DGRAD ? (2 - kh) * HW + (2 - kw) : kh * HW + kw;
    // fragments: both k-steps' B (the stage's 64 columns), one A register per group,
    // refilled with the group's k-step-1 fragment right behind its k-step-0 MFMAs (4 G + 32
    // VGPRs instead of 8 G + 32: G = 7 groups of accumulators are already 112)
    bf16x8 af[G], bfr[2][4];
    auto loadb = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (DGRAD) {
          const int rr = j * 16 + (lane & 15), cc = 4 * kk + g;
          bfr[kk][j] = *reinterpret_cast<const bf16x8*>(ib + rr * 128 + 16 * (cc ^ (rr & 7)));
        } else {
          bfr[kk][j] = tile::frag_mc<64>(ib + kk * 32 * 128, j * 16, lane);
        }
      }
    };
    auto loada = [&](int kk, int i) __attribute__((always_inline)) {
      const int q = hbase[i] + toff, cc = 4 * kk + g;
      af[i] = *reinterpret_cast<const bf16x8*>(hcur + q * 128 + 16 * (cc ^ (q & 7)));
    };
    loadb(0);
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (i < ng) loada(0, i);
    loadb(1);
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (i < ng) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[0][j], af[i], acc[i][j]);
        loada(1, i);
      }
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (i < ng)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[1][j], af[i], acc[i][j]);
    // the next chunk's halo (issued at this chunk's first stage) landed before its barrier
    if (tap == 8 && c + 1 < nch) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  // ---- epilogue over the wave's G groups (rows m0s + wave * 16 G + 16 i + lane & 15) ----
  // bias / residual / ReLU / bf16 stores as tile::epilogue; BN statistics: per column over
  // the wave's rows (16-lane xor reduction), across the 4 waves through LDS, then into the
  // fixed-point accumulators (replica = strip)
  const int m0s = (img * H + oh0) * W;
  const int mend = m0s + npx;
  constexpr bool ST = (EPI & (E_STATS | E_BNRED)) != 0;
  if (wave < 4) {
    float csum[4][4], csq[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[j][e] = csq[j][e] = 0.f;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int m = m0s + (wave * G + i) * 16 + (lane & 15);
      const bool mok = i < ng && m < mend;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + j * 16 + 4 * (lane >> 4);
        f32x4 v = acc[i][j];
        if constexpr (EPI & E_BIAS) {
          const float4 b = *reinterpret_cast<const float4*>(a.bias + n);
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if constexpr (EPI & E_ADD) {
          if (mok) {
            const uint2 r = *reinterpret_cast<const uint2*>((const uint16_t*)a.R + (size_t)m * a.ldc + n);
            v[0] += __uint_as_float(r.x << 16);
            v[1] += __uint_as_float(r.x & 0xffff0000u);
            v[2] += __uint_as_float(r.y << 16);
            v[3] += __uint_as_float(r.y & 0xffff0000u);
          }
        }
        if constexpr (EPI & E_STATS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = mok ? v[e] : 0.f;
            if constexpr (EPI & E_BF16) x = bf2f(f2bf(x));
            csum[j][e] += x;
            csq[j][e] += x * x;
          }
        }
        if constexpr (EPI & E_BNRED) {
          if (mok) {
            const uint2 xr = *reinterpret_cast<const uint2*>(a.bnx + (size_t)m * a.ldc + n);
            const float xv[4] = {__uint_as_float(xr.x << 16), __uint_as_float(xr.x & 0xffff0000u),
                                 __uint_as_float(xr.y << 16), __uint_as_float(xr.y & 0xffff0000u)};
            const float4 mu = *reinterpret_cast<const float4*>(a.bnst + n);
            const float4 iv = *reinterpret_cast<const float4*>(a.bnst + a.N + n);
            const float4 sc = *reinterpret_cast<const float4*>(a.bnst + 2 * a.N + n);
            const float4 sh = *reinterpret_cast<const float4*>(a.bnst + 3 * a.N + n);
            const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, i4[4] = {iv.x, iv.y, iv.z, iv.w};
            const float s4[4] = {sc.x, sc.y, sc.z, sc.w}, h4[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float y = bf2f(f2bf(fmaxf(fmaf(xv[e], s4[e], h4[e]), 0.f)));
              const float d = y > 0.f ? bf2f(f2bf(v[e])) : 0.f;
              csum[j][e] += d;
              csq[j][e] += d * (xv[e] - m4[e]) * i4[e];
            }
          }
        }
        if constexpr (EPI & E_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (!mok) continue;
        uint2 pk;
        pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>((uint16_t*)a.C + (size_t)m * a.ldc + n) = pk;
      }
    }
    if constexpr (ST) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
        {
          csum[j][e] = row16_sum(csum[j][e]);
          csq[j][e] = row16_sum(csq[j][e]);
        }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int cidx = j * 16 + 4 * (lane >> 4) + e;
            red[(0 * 4 + wave) * 64 + cidx] = csum[j][e];
            red[(1 * 4 + wave) * 64 + cidx] = csq[j][e];
          }
      }
    }
  }
  if constexpr (ST) {
    __syncthreads();  // every wave, the loaders included
    if (t < 64) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        sm += red[(0 * 4 + w) * 64 + t];
        sq += red[(1 * 4 + w) * 64 + t];
      }
      const int n = n0 + t;
      const size_t reps = a.stats_reps > 1 ? a.stats_reps : 1;
      const size_t rep = (size_t)(img * sg.S + strip) % reps;
      if constexpr (EPI & E_BNRED) {
        long long* accp = a.stats_acc + rep * 4 * a.N;
        long long* flag = a.stats_acc + reps * 4 * a.N + n;
        bnacc_add2(accp + n, accp + a.N + n, flag, sm);
        bnacc_add2(accp + 2 * a.N + n, accp + 3 * a.N + n, flag, sq);
      } else {
        long long* accp = a.stats_acc + rep * 2 * a.N;
        long long* flag = a.stats_acc + reps * 2 * a.N + n;
        bnacc_add1(accp + n, flag, sm);
        bnacc_add1(accp + a.N + n, flag, sq);
      }
    }
  }
}

template <bool DG, int EPI, int G, int D>
hipError_t launch_s(const GemmArgs& a, const SGeo& sg, int blocks, size_t lds, hipStream_t s) {
  auto k = conv3s_kernel<DG, EPI, G, D>;
  static bool attr = false;  // once per instantiation (host-side, before any capture)
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(SNT), lds, s, a, sg);
  return hipGetLastError();
}

template <bool DG, int G, int D>
hipError_t launch_s_epi(const GemmArgs& a, int epi, const SGeo& sg, int blocks, size_t lds, hipStream_t s) {
  switch (epi) {
    case E_BF16: return launch_s<DG, E_BF16, G, D>(a, sg, blocks, lds, s);
    case E_BIAS | E_BF16: return launch_s<DG, E_BIAS | E_BF16, G, D>(a, sg, blocks, lds, s);
    case E_BIAS | E_RELU | E_BF16: return launch_s<DG, E_BIAS | E_RELU | E_BF16, G, D>(a, sg, blocks, lds, s);
    case E_RELU | E_BF16: return launch_s<DG, E_RELU | E_BF16, G, D>(a, sg, blocks, lds, s);
    case E_BF16 | E_STATS: return launch_s<DG, E_BF16 | E_STATS, G, D>(a, sg, blocks, lds, s);
    case E_BIAS | E_BF16 | E_STATS: return launch_s<DG, E_BIAS | E_BF16 | E_STATS, G, D>(a, sg, blocks, lds, s);
    case E_BF16 | E_ADD: return launch_s<DG, E_BF16 | E_ADD, G, D>(a, sg, blocks, lds, s);
    case E_BF16 | E_BNRED:
      if constexpr (DG) return launch_s<DG, E_BF16 | E_BNRED, G, D>(a, sg, blocks, lds, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// strip geometry of a shape, or false: strips of R rows with <= 7 groups of 16 pixels per
// compute wave, the (R + 2) x (W + 2) halo double-buffered + a weight ring of >= 4 stages
// in the CU's 160 KiB, images x strips x N-tiles <= 2 x CUs (one block per CU, at most
// two rounds)
bool strip_plan(const GemmArgs& a, int cus, SGeo& sg, int& G, int& D) {
  const int H = a.H, W = a.W;
  const int nimg = a.M / (H * W), ntl = a.N / 64;
  // the largest strip (fewest strips per image) whose groups fit G <= 7
  for (int S = 1; S <= H; ++S) {
    const int R = (H + S - 1) / S;
    const int groups = (R * W + 15) / 16;
    const int g = (groups + 3) / 4;
    if (g > 4) continue;  // (7 groups of accumulators spill: 112 of the 256 VGPRs a 6-wave block allows)
    const int hb = (((R + 2) * (W + 2)) * 128 + 1023) & ~1023;
    const int fixed = 2 * hb + 2048 + 2 * a.Cin * 4;
    const int d = min(8, (160 * 1024 - fixed) / WST_B);
    if (d < 4) continue;
    if ((long)nimg * S * ntl > 2L * cus) return false;  // too many blocks: the general kernel
    sg.R = R;
    sg.S = (H + R - 1) / R;
    sg.NTL = ntl;
    sg.hbytes = hb;
    sg.ring = 2 * hb;
    sg.red = sg.ring + d * WST_B;
    sg.sft = sg.red + 2048;
    // one instantiation: <= 4 groups per compute wave, an 8-stage weight ring
    G = 4;
    D = 8;
    if (d < D) return false;
    return true;
  }
  return false;
}

}  // namespace

int conv3s_ok(const GemmArgs& a, int dgrad, int epi) {
  // opt-in while it loses to the general kernel (round 6: a single weight-loader wave's
  // LDS-DMA stream could not keep the stages fed -- layer-3 backprop-input 50.7 vs 27.6 us)
  const char* ev = getenv("DAMD_CONV3S");
  if (!(ev && ev[0] == '1')) return 0;
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 || a.Cin % 64 || a.N % 64 || a.Cin < 128) return 0;
  if (a.H < 1 || a.M % (a.H * a.W)) return 0;
  if (dgrad && (a.kc != a.Cin || a.bnin.acc)) return 0;
  // statistics only into fixed-point accumulators (no per-tile partial rows here)
  if ((epi & (E_STATS | E_BNRED)) && !a.stats_acc) return 0;
  if ((epi & (E_SLAB | E_ATOMIC)) || !(epi & E_BF16)) return 0;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  SGeo sg;
  int G, D;
  return strip_plan(a, cus, sg, G, D) ? 1 : 0;
}

hipError_t conv3s_launch(const GemmArgs& a, int dgrad, int epi, hipStream_t s) {
  if (!conv3s_ok(a, dgrad, epi)) return hipErrorInvalidValue;
  SGeo sg;
  int G = 0, D = 0;
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  if (!strip_plan(a, cus, sg, G, D)) return hipErrorInvalidValue;
  const int nimg = a.M / (a.H * a.W);
  const int blocks = nimg * sg.S * sg.NTL;
  const size_t lds = (size_t)sg.sft + 2 * a.Cin * 4;
  (void)G;
  (void)D;
  return dgrad ? launch_s_epi<true, 4, 8>(a, epi, sg, blocks, lds, s) : launch_s_epi<false, 4, 8>(a, epi, sg, blocks, lds, s);
}

}  // namespace damd
