// Implicit-GEMM convolution on MFMA with direct global->LDS staging (gfx950 / MI355X):
// the hot conv GEMMs of the generic path (ResNet-18: SURVEY.md §2.9 R2-R4, R9).
//
//   A_CONV64  forward:          C[m = (n,oh,ow)][co] = sum_{kh,kw,ci} x[n][oh*s-p+kh][ow*s-p+kw][ci] W[kh][kw][ci][co]
//   A_DGRAD64 backprop-input:   C[m = (n,ih,iw)][ci] = sum_{kh,kw,co} dy[n][ih+p-kh][iw+p-kw][co] W[kh][kw][ci][co]
//             (stride 1: the transposed conv is an ordinary conv with flipped taps)
//
// Why a second conv kernel (csrc/kernels/gemm.hip keeps the general cases): when the
// gathered tensor has C % 64 == 0, a BK = 64 k-step is ONE filter tap and 64 contiguous
// channels, i.e. one 128-byte segment per output row.  That lets the tile be staged by
// the LDS-DMA path (global_load_lds_dwordx4: no staging VGPRs, no ds_write, no
// per-element masking -- the register-staged kernel spends ~7 VALU instructions per MFMA
// on exactly that), with a per-row base pointer computed once and one wave-uniform tap
// offset per k-step.  Rows that fall into the zero padding read a 16-byte zero block.
//
// Tile: BM x BN (128x128 or 256x64), 256 threads = 4 waves, each wave 64x64 as 4x4
// v_mfma_f32_16x16x32_bf16; BK = 64 (two MFMA k-substeps per barrier).  Two LDS stages:
// the DMA of k-step t+1 is in flight while the MFMAs of step t run; raw s_barrier with a
// counted vmcnt (a __syncthreads() would drain the in-flight DMA, cdna_hip_programming.md
// §5 "Pipelining across barriers"); all LDS in ONE __shared__ array (second-object trap).
// LDS images (lane-linear for the DMA; the XOR swizzle is applied to the SOURCE address
// and again on the read, rule 21):
//   A (and the dgrad weights, k-contiguous): [rows][64] bf16, 128-B rows, chunk c of row r
//     at slot c ^ (r & 7)  -> ds_read_b128 fragment reads hit 8 distinct 4-bank groups
//     per 8 lanes;
//   forward weights (n-contiguous): [64 k][BN] with tile::mc_swz, read transposed with
//     ds_read_b64_tr_b16 (no transposing stores).
// Epilogue: tile::epilogue (bias / residual / BN statistics / ReLU / bf16 / split-K slab).
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

namespace damd {
namespace {

constexpr int NT = 256;
constexpr int BK = 64;

// 16-byte zero block: the DMA source of every padding / out-of-range row
__device__ __attribute__((aligned(64))) uint4 g_zero16[4];

typedef const void __attribute__((address_space(1)))* gptr_t;
typedef void __attribute__((address_space(3)))* lptr_t;

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_wave_base, 16, 0, 0);
}

// KC image fragment: rows r0..r0+15 (lane & 15), k-substep kk (chunks 4kk + lane>>4)
__device__ __forceinline__ bf16x8 frag_kc64(const char* img, int r0, int kk, int lane) {
  const int r = r0 + (lane & 15), c = 4 * kk + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * 128 + 16 * (c ^ (r & 7)));
}

template <int BM, int BN, bool DGRAD, int EPI>
__global__ __launch_bounds__(NT, 2) void conv_gemm_kernel(GemmArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  static_assert(WM * 64 == BM, "tile shape");
  constexpr int A_ST = BM * BK * 2, B_ST = BN * BK * 2, ST = A_ST + B_ST;
  constexpr int NA = BM / 32;  // A DMA instructions per wave per stage (8 rows each)
  constexpr int NB = BN / 32;  // B DMA instructions per wave per stage (1 KB each)
  constexpr int NQ = NA + NB;
  __shared__ __attribute__((aligned(1024))) char smem[2 * ST];

  const int tiles_n = gridDim.x, tiles = gridDim.x * gridDim.y;
  const int lin = tile::xcd_tile(blockIdx.y * tiles_n + blockIdx.x, tiles);
  const int tn = lin % tiles_n, tm = lin / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * a.k_per_split;
  const int kend = min(a.K, kbeg + a.k_per_split);
  const int nk = (kend - kbeg) / BK;  // > 0 and exact: checked by the launcher

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // ---- geometry: rows of the output grid (RH x RW), gathered tensor (SH x SW x SC) ----
  const int SC = a.Cin;
  const int RH = DGRAD ? a.H : a.Ho, RW = DGRAD ? a.W : a.Wo;
  const int SH = DGRAD ? a.Ho : a.H, SW = DGRAD ? a.Wo : a.W;
  const uint16_t* src = (const uint16_t*)a.A;
  // A rows of this thread: r = 8 * (wave + 4j) + (lane >> 3), 16-B source chunk
  // (lane & 7) ^ (r & 7) (= (lane & 7) ^ (lane >> 3): r & 7 == lane >> 3)
  const int ca = (lane & 7) ^ (lane >> 3);
  const uint16_t* arow[NA];
  int ay[NA], ax[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int m = m0 + 8 * (wave + 4 * j) + (lane >> 3);
    const int mm = min(m, a.M - 1);
    const int ow = mm % RW, tmp = mm / RW, oh = tmp % RH, n = tmp / RH;
    const int y0 = DGRAD ? oh + a.pad : oh * a.stride - a.pad;
    const int x0 = DGRAD ? ow + a.pad : ow * a.stride - a.pad;
    ay[j] = m < a.M ? y0 : -(1 << 28);  // out-of-range rows: never in bounds
    ax[j] = x0;
    arow[j] = src + ((long)n * SH * SW + (long)y0 * SW + x0) * SC + 8 * ca;
  }
  // B: forward = W[k][N] rows of BN*2 bytes (CPR chunks, RPI k-rows per 1-KB DMA);
  //    dgrad   = W[tap][n][kc] rows n of 64 k (like A)
  const uint16_t* wsrc = (const uint16_t*)a.B;
  constexpr int CPR = BN / 8, RPI = 64 / CPR;
  const uint16_t* brow[NB];
  bool bval[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int q = wave + 4 * j;
    if constexpr (DGRAD) {
      const int n = n0 + 8 * q + (lane >> 3);
      bval[j] = n < a.N;
      brow[j] = wsrc + (long)min(n, a.N - 1) * a.kc + 8 * ca;
    } else {
      const int kr = q * RPI + lane / CPR;
      const int ch = (lane % CPR) ^ tile::mc_swz<BN>(kr);
      const int n = n0 + 8 * ch;
      bval[j] = n < a.N;
      brow[j] = wsrc + (long)(kbeg + kr) * a.ldb + min(n, a.N - 8);
    }
  }

  // k-step state (wave-uniform): tap (kh, kw) and channel offset c0 of k = kbeg + 64 kt
  int tap = kbeg / SC, c0 = kbeg - tap * SC;
  int kh = tap / a.KW, kw = tap - kh * a.KW;

  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    char* sa = smem + stage * ST;
    const int dy = DGRAD ? -kh : kh, dx = DGRAD ? -kw : kw;
    const long toff = ((long)dy * SW + dx) * SC + c0;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const bool ok = (unsigned)(ay[j] + dy) < (unsigned)SH && (unsigned)(ax[j] + dx) < (unsigned)SW;
      glds16(ok ? (const void*)(arow[j] + toff) : (const void*)g_zero16, sa + (wave + 4 * j) * 1024);
    }
    char* sb = sa + A_ST;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const void* p;
      if constexpr (DGRAD) p = brow[j] + ((long)tap * a.N) * a.kc + c0;
      else p = brow[j] + (long)kt * BK * a.ldb;
      glds16(bval[j] ? p : (const void*)g_zero16, sb + (wave + 4 * j) * 1024);
    }
    // advance to the next k-step
    c0 += BK;
    if (c0 >= SC) {
      c0 = 0;
      ++tap;
      if (++kw == a.KW) { kw = 0; ++kh; }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue(cur ^ 1, kt + 1);  // WAR: the barrier closing step kt-1 retired its reads
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQ) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMA of step kt has landed
    const char* ia = smem + cur * ST;
    const char* ib = ia + A_ST;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = frag_kc64(ia, wm * 64 + i * 16, kk, lane);
        if constexpr (DGRAD) bfr[i] = frag_kc64(ib, wn * 64 + i * 16, kk, lane);
        else bfr[i] = tile::frag_mc<BN>(ib + kk * 32 * BN * 2, wn * 64 + i * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // reads of stage `cur` done before it is refilled
  }
  tile::epilogue<BM, BN, EPI>(a, acc, m0, n0, tm, wm, wn, wave, lane, reinterpret_cast<float*>(smem));
}

template <int BM, int BN, bool DG, int EPI>
hipError_t launch_t(const GemmArgs& a, int splits, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, DG, EPI>), grid, dim3(NT), 0, s, a);
  return hipGetLastError();
}

template <int BM, int BN, bool DG>
hipError_t launch_epi(const GemmArgs& a, int epi, int splits, hipStream_t s) {
  switch (epi) {
    case E_BF16: return launch_t<BM, BN, DG, E_BF16>(a, splits, s);
    case E_BIAS | E_BF16: return launch_t<BM, BN, DG, E_BIAS | E_BF16>(a, splits, s);
    case E_BIAS | E_RELU | E_BF16: return launch_t<BM, BN, DG, E_BIAS | E_RELU | E_BF16>(a, splits, s);
    case E_SLAB: return launch_t<BM, BN, DG, E_SLAB>(a, splits, s);
    case E_BF16 | E_STATS: return launch_t<BM, BN, DG, E_BF16 | E_STATS>(a, splits, s);
    case E_BIAS | E_BF16 | E_STATS: return launch_t<BM, BN, DG, E_BIAS | E_BF16 | E_STATS>(a, splits, s);
    case E_BF16 | E_ADD: return launch_t<BM, BN, DG, E_BF16 | E_ADD>(a, splits, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t conv_gemm_launch(const GemmArgs& a, int amode, int epi, int splits, int tile, hipStream_t s) {
  const bool dg = amode == A_DGRAD64;
  if (a.Cin % BK || a.N % 8 || a.M < 1 || a.K % BK || a.K != a.KH * a.KW * a.Cin) return hipErrorInvalidValue;
  if (splits < 1 || a.k_per_split % BK || a.k_per_split < BK || (long)splits * a.k_per_split < a.K ||
      (long)(splits - 1) * a.k_per_split >= a.K)
    return hipErrorInvalidValue;
  if (dg && (a.stride != 1 || a.kc != a.Cin)) return hipErrorInvalidValue;
  if (!dg && a.ldb % 8) return hipErrorInvalidValue;
  if ((epi & E_SLAB) && (epi & ~E_SLAB)) return hipErrorInvalidValue;
  if (tile == 1) return dg ? launch_epi<256, 64, true>(a, epi, splits, s) : launch_epi<256, 64, false>(a, epi, splits, s);
  return dg ? launch_epi<128, 128, true>(a, epi, splits, s) : launch_epi<128, 128, false>(a, epi, splits, s);
}

}  // namespace damd
