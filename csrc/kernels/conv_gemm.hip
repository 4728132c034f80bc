// Implicit-GEMM convolution on MFMA with direct global->LDS staging (gfx950 / MI355X):
// the hot conv GEMMs of the generic path (ResNet-18: SURVEY.md §2.9 R2-R4, R9).
//
//   A_CONV64  forward:          C[m = (n,oh,ow)][co] = sum_{kh,kw,ci} x[n][oh*s-p+kh][ow*s-p+kw][ci] W[kh][kw][ci][co]
//   A_DGRAD64 backprop-input:   C[m = (n,ih,iw)][ci] = sum_{kh,kw,co} dy[n][ih+p-kh][iw+p-kw][co] W[kh][kw][ci][co]
//             (stride 1: the transposed conv is an ordinary conv with flipped taps)
//   A_WGRAD64 backprop-filter:  C[m = (kh,kw,ci)][co] = sum_{n,oh,ow} x[n][oh*s-p+kh][ow*s-p+kw][ci] dy[n][oh][ow][co]
//
// Why a second conv kernel family (csrc/kernels/gemm.hip keeps the general cases): when
// the gathered tensor has C % KB == 0, a KB-deep k-step (KB = 32 or 64) is ONE filter tap
// and KB contiguous channels, i.e. one 2*KB-byte segment per output row.  That lets the
// tile be staged by the LDS-DMA path (global_load_lds_dwordx4: no staging VGPRs, no
// ds_write, no per-element masking -- the register-staged kernel spends ~7 VALU
// instructions per MFMA on exactly that), with a per-row base pointer computed once and
// one wave-uniform tap offset per k-step.  Rows in the zero padding read a zero block.
//
// Tile: BM x BN (128x128 or 256x64), 256 threads = 4 waves, each wave 64x64 as 4x4
// v_mfma_f32_16x16x32_bf16.  LDS ring of STAGES stages, one barrier per k-step (kloop),
// counted vmcnt + raw s_barrier (a __syncthreads() would drain the in-flight DMA,
// cdna_hip_programming.md §5 "Pipelining across barriers"), all LDS in ONE __shared__
// array (second-object trap).  Measured on the ResNet-18 shapes (scripts/bench_gemm.py):
// occupancy beats ring depth -- 2 stages at 2 blocks/CU ran 1.3x the 3-/4-stage rings at
// 1 block/CU (step-weighted conv GEMM sum 2.78 vs 3.69 / 3.49 ms).  KB = 32 halves the LDS
// per stage (4 blocks/CU): slower for conv fwd/dgrad, faster for the weight gradient of
// the small-image layers (the planner picks it per layer, ops/hip.py conv_wgrad_plan).
// LDS images (lane-linear for the DMA; the XOR swizzle is applied to the SOURCE address
// and again on the read, rule 21):
//   k-contiguous operands (conv rows, dgrad weights): [rows][KB] bf16; chunk c of row r at
//     slot c ^ kc_swz(r), read with ds_read_b128 -- each 8-lane group of a fragment read
//     covers 8 distinct 4-bank groups;
//   mn-contiguous operands (forward weights, both wgrad operands): [KB k-rows][cols] with
//     tile::mc_swz, read transposed with ds_read_b64_tr_b16 (no transposing stores).
// Epilogue: tile::epilogue (bias / residual / BN statistics / ReLU / bf16 / split-K slab).
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

#include <cstdlib>

namespace damd {
namespace {

constexpr int NT = 256;

// 16-byte zero block: the DMA source of every padding / out-of-range row
__device__ __attribute__((aligned(64))) uint4 g_zero16[4];

using tile::glds16;  // inline-asm LDS-DMA (no compiler drain before the next ds_read)

// k-contiguous image [rows][KB]: swizzle of row r (KB/8 chunks of 16 B per row)
template <int KB>
__device__ __forceinline__ int kc_swz(int r) {
  if constexpr (KB == 64) return r & 7;
  else return (r >> 1) & 3;
}
// fragment rows r0..r0+15 (lane & 15), k-substep kk (chunks 4kk + (lane >> 4))
template <int KB>
__device__ __forceinline__ bf16x8 frag_kc(const char* img, int r0, int kk, int lane) {
  const int r = r0 + (lane & 15), c = 4 * kk + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * (KB * 2) + 16 * (c ^ kc_swz<KB>(r)));
}

// k-loop over STAGES LDS stages, ONE barrier per k-step: wait for this wave's DMA of
// step kt (counted vmcnt leaves the later steps in flight) -> lgkmcnt(0) (its reads of
// step kt-1 retired) -> s_barrier (every wave's DMA of kt landed AND every wave is done
// with stage (kt-1) % STAGES) -> refill that stage with step kt+STAGES-1 -> MFMAs on kt.
template <int STAGES, int NQ, class Issue, class Compute>
__device__ __forceinline__ void kloop(int nk, Issue& issue, Compute& compute) {
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, STAGES - 2);  // steps in flight beyond kt
    if constexpr (STAGES >= 4) {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NQ) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQ) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (STAGES == 3) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQ) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES, kt + STAGES - 1);
    compute(kt % STAGES);
  }
}

// blocks per CU the LDS ring allows (160 KiB per CU), capped at 4
constexpr int blocks_per_cu(int lds_bytes) {
  const int b = (160 * 1024) / lds_bytes;
  return b >= 4 ? 4 : (b < 1 ? 1 : b);
}

template <int BM, int BN, int KB, bool DGRAD, int EPI, int STAGES>
__global__ __launch_bounds__(NT, blocks_per_cu((BM + BN) * KB * 2 * STAGES)) void conv_gemm_kernel(GemmArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  static_assert(WM * 64 == BM, "tile shape");
  constexpr int CPK = KB / 8;                           // 16-B chunks per k-contiguous row
  constexpr int RPQ = 64 / CPK;                         // such rows per 1-KB DMA instruction
  constexpr int A_ST = BM * KB * 2, B_ST = BN * KB * 2, ST = A_ST + B_ST;
  constexpr int NA = A_ST / 4096;                       // A DMA instructions per wave per stage
  constexpr int NB = B_ST / 4096;
  constexpr int NQ = NA + NB;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * ST];

  const int tiles_n = gridDim.x, tiles = gridDim.x * gridDim.y;
  const int lin = tile::xcd_tile(blockIdx.y * tiles_n + blockIdx.x, tiles);
  const int tn = lin % tiles_n, tm = lin / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // Stride-2 backprop-input as four sub-pixel convolutions (blockIdx.z = parity class
  // (ra, rb) of the input pixel; no K split): input row ih = 2 i2 + ra receives dy row
  // oh = (ih + pad - kh) / 2 from the taps kh = kh0, kh0 + 2, .. (kh0 = (ra + pad) & 1)
  // only, so each class is a stride-1 conv over the (H/2 x W/2) class grid with
  // ceil((KH - kh0)/2) x ceil((KW - kw0)/2) taps -- 9 tap-products per 4 pixels instead
  // of 36 with the zero taps of the dilated formulation.
  const bool sp = DGRAD && a.stride == 2;
  const int ra = sp ? (int)(blockIdx.z >> 1) : 0, rb = sp ? (int)(blockIdx.z & 1) : 0;
  const int kh0 = sp ? (ra + a.pad) & 1 : 0, kw0 = sp ? (rb + a.pad) & 1 : 0;
  const int tstep = sp ? 2 : 1;
  const int nth = sp ? (a.KH - kh0 + 1) >> 1 : a.KH, ntw = sp ? (a.KW - kw0 + 1) >> 1 : a.KW;
  const int kbeg = sp ? 0 : blockIdx.z * a.k_per_split;
  const int kend = sp ? nth * ntw * a.Cin : min(a.K, kbeg + a.k_per_split);
  const int nk = (kend - kbeg) / KB;  // exact: checked by the launcher (0 for an empty class)
  if constexpr ((EPI & E_ADD) != 0) {
    if (nk == 0) return;  // accumulating: a class without taps adds nothing
  }

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // ---- geometry: rows of the output grid (RH x RW), gathered tensor (SH x SW x SC) ----
  const int SC = a.Cin;
  const int RH = DGRAD ? (sp ? a.H >> 1 : a.H) : a.Ho, RW = DGRAD ? (sp ? a.W >> 1 : a.W) : a.Wo;
  const int SH = DGRAD ? a.Ho : a.H, SW = DGRAD ? a.Wo : a.W;
  const uint16_t* src = (const uint16_t*)a.A;
  const void* zero = tile::pinned_addr(g_zero16);
  // A rows of this thread: r = RPQ * (wave + 4j) + lane / CPK; source chunk
  // (lane % CPK) ^ kc_swz(r), and kc_swz(r) depends on r mod 8 == (lane / CPK) mod 8
  const int rin = lane / CPK;
  const int ca = (lane % CPK) ^ kc_swz<KB>(rin);
  // Packed-tap stem (forward, Cin == 4, KB == 32): a k-step is one filter row kh and its
  // 32 elements are 8 consecutive input pixels x 4 channels (kw' = 0..7, the weights of
  // kw' >= KW_true and channel 3 are zero), so chunk ca = input pixels x0 + 2ca, +1 --
  // the 7x7x3 ResNet stem runs K = 224 instead of 7x7x8 = 392 with 8-padded channels.
  const bool stem = !DGRAD && a.Cin == 4;
  const int cpx = stem ? 2 * ca : 0;  // this lane's pixel offset within the row segment
  const uint16_t* arow[NA];
  int ay[NA], ax[NA];
  // Row -> (n, oh, ow) by a float reciprocal multiply: floor((q + 0.5) * fl(1/d)) is exact
  // for q < 2^21 (the product's error stays below 0.25/d, its distance to an integer is
  // >= 0.5/d).  The 2 x NA integer divisions it replaces were ~600 of the ~1900 VALU a
  // wave issued on the 9-k-step ResNet layer-1 tiles (more than the main loop's 740).
  const bool fdiv = a.M < (1 << 21);
  const float invRW = 1.f / (float)RW, invRH = 1.f / (float)RH;
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int m = m0 + RPQ * (wave + 4 * j) + rin;
    const int mm = min(m, a.M - 1);
    int ow, oh, n;
    if (fdiv) {
      const int tmp = (int)(((float)mm + 0.5f) * invRW);
      ow = mm - tmp * RW;
      n = (int)(((float)tmp + 0.5f) * invRH);
      oh = tmp - n * RH;
    } else {
      const int tmp = mm / RW;
      ow = mm - tmp * RW;
      n = tmp / RH;
      oh = tmp - n * RH;
    }
    const int y0 = DGRAD ? (sp ? oh + ((ra + a.pad - kh0) >> 1) : oh + a.pad) : oh * a.stride - a.pad;
    const int x0 = DGRAD ? (sp ? ow + ((rb + a.pad - kw0) >> 1) : ow + a.pad) : ow * a.stride - a.pad;
    ay[j] = m < a.M ? y0 : -(1 << 28);  // out-of-range rows: never in bounds
    ax[j] = x0;
    arow[j] = src + ((long)n * SH * SW + (long)y0 * SW + x0) * SC + 8 * ca;
  }
  // B: forward = W[k][N], k-rows of BN*2 bytes (CPR chunks, RPI k-rows per 1-KB DMA);
  //    dgrad   = W[tap][n][kc], rows n of KB k (like A)
  const uint16_t* wsrc = (const uint16_t*)a.B;
  constexpr int CPR = BN / 8, RPI = 64 / CPR;
  const uint16_t* brow[NB];
  bool bval[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int q = wave + 4 * j;
    if constexpr (DGRAD) {
      const int n = n0 + RPQ * q + rin;
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

  // k-step state (wave-uniform): tap (kh, kw) of the iteration space (class taps when
  // sp: weight tap (kh0 + 2 kh, kw0 + 2 kw)) and channel offset c0 of k = kbeg + KB kt
  int tap = kbeg / SC, c0 = kbeg - tap * SC;
  int kh = tap / ntw, kw = tap - kh * ntw;

  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    char* sa = smem + stage * ST;
    const int dy = DGRAD ? -kh : (stem ? kbeg / KB + kt : kh), dx = DGRAD ? -kw : (stem ? 0 : kw);
    const int wtap = sp ? (kh0 + tstep * kh) * a.KW + kw0 + tstep * kw : tap;
    const long toff = ((long)dy * SW + dx) * SC + (stem ? 0 : c0);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const bool ok = (unsigned)(ay[j] + dy) < (unsigned)SH && (unsigned)(ax[j] + dx + cpx) < (unsigned)SW;
      glds16(ok ? (const void*)(arow[j] + toff) : zero, sa + (wave + 4 * j) * 1024);
    }
    char* sb = sa + A_ST;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const void* p;
      if constexpr (DGRAD) p = brow[j] + ((long)wtap * a.N) * a.kc + c0;
      else p = brow[j] + (long)kt * KB * a.ldb;
      glds16(bval[j] ? p : zero, sb + (wave + 4 * j) * 1024);
    }
    // advance to the next k-step
    c0 += KB;
    if (c0 >= SC) {
      c0 = 0;
      ++tap;
      if (++kw == ntw) { kw = 0; ++kh; }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) __attribute__((always_inline)) {
    const char* ia = smem + stage * ST;
    const char* ib = ia + A_ST;
#pragma unroll
    for (int kk = 0; kk < KB / 32; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = frag_kc<KB>(ia, wm * 64 + i * 16, kk, lane);
        if constexpr (DGRAD) bfr[i] = frag_kc<KB>(ib, wn * 64 + i * 16, kk, lane);
        else bfr[i] = tile::frag_mc<BN>(ib + kk * 32 * BN * 2, wn * 64 + i * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
  };
  kloop<STAGES, NQ>(nk, issue, compute);
  if constexpr ((EPI & E_FIXUP) != 0) {
    // split-K finished in this launch (cdna_hip_programming.md, in-launch split-K reduction):
    // slab store -> drain -> agent release -> ticket; the split drawing S - 1 acquires, sums
    // the S slabs at its lanes' own positions in split order (the order of splitk_finish:
    // the same output bits) and runs the final epilogue.  Nothing waits on the ticket.
    constexpr int EF = EPI & ~E_FIXUP;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
        if (m < a.M && n < a.N)
          *reinterpret_cast<f32x4*>(a.slab + ((size_t)blockIdx.z * a.M + m) * a.N + n) = acc[i][j];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem);  // (the staging stages are free; one LDS array)
    const int tile_id = tm * tiles_n + tn;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(a.tickets + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last[0] = old == gridDim.z - 1;
    }
    __syncthreads();
    if (!last[0]) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.tickets + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int S = gridDim.z;
    for (int sp = 0; sp < S; ++sp) {
      f32x4 v[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = min(m0 + wm * 64 + i * 16 + (lane & 15), a.M - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = min(n0 + wn * 64 + j * 16 + 4 * (lane >> 4), a.N - 4);
          v[i][j] = *reinterpret_cast<const f32x4*>(a.slab + ((size_t)sp * a.M + m) * a.N + n);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = sp == 0 ? v[i][j] : acc[i][j] + v[i][j];
    }
    __syncthreads();  // `red` aliases the staging stages (the ticket flag included)
    tile::epilogue<BM, BN, EF>(a, acc, m0, n0, tm, wm, wn, wave, lane, reinterpret_cast<float*>(smem));
    return;
  }
  if constexpr ((EPI & E_STATS) != 0) __syncthreads();  // `red` aliases the staging stages
  if (sp) {
    // class-grid row (n, i2, j2) -> input pixel (n, 2 i2 + ra, 2 j2 + rb)
    const int H = a.H, W = a.W;
    auto row_of = [=](int m) -> size_t {
      const int j2 = m % RW, tmp = m / RW, i2 = tmp % RH, n = tmp / RH;
      return ((size_t)n * H + 2 * i2 + ra) * W + 2 * j2 + rb;
    };
    tile::epilogue<BM, BN, EPI>(a, acc, m0, n0, tm, wm, wn, wave, lane, reinterpret_cast<float*>(smem), row_of);
  } else {
    tile::epilogue<BM, BN, EPI>(a, acc, m0, n0, tm, wm, wn, wave, lane, reinterpret_cast<float*>(smem));
  }
}

// =====================================================================================
// Weight gradient: C[m = (kh,kw,ci)][co] (+)= sum over output pixels p of
//   x[n][oh*s-p+kh][ow*s-p+kw][ci] * dy[p][co]
// The reduction runs over "virtual rows": output row (n, oh) cut into nseg = ceil(Wo/KB)
// segments of Wv = ceil(Wo/nseg) <= KB pixels.  A KB-deep k-step holds G = KB/S virtual
// rows in slots of S = pow2ceil(Wv) (slot >= Wv: zero), so every k-row's pixel is
// (row base + g, slot): no per-element division by Wo -- the (n, oh) of a virtual row
// comes from one float reciprocal multiply (exact while the row index < 2^21).  The slot
// padding costs <= 12.5 % extra MFMA on the ResNet shapes (Wv = 56, 28, 14, 7).
// Both operands are mn-contiguous (x channels, dy channels): [KB][cols] images read with
// ds_read_b64_tr_b16, filled by LDS-DMA (source-side swizzle).
// GemmArgs: M = KH*KW*Cin, N = Cout, K = virtual rows, k_per_split = virtual rows per
// split (multiple of G), Cin/H/W/Ho/Wo/KH/KW/stride/pad = the conv geometry.
// =====================================================================================
struct VRow {
  int nseg, Wv, S, lgS, G;
  float invHo;
};
template <int KB>
__device__ __forceinline__ VRow vrow_geo(const GemmArgs& a) {
  VRow v;
  v.nseg = (a.Wo + KB - 1) / KB;
  v.Wv = (a.Wo + v.nseg - 1) / v.nseg;
  v.lgS = v.Wv <= 1 ? 0 : 32 - __builtin_clz((unsigned)(v.Wv - 1));  // pow2ceil exponent
  v.S = 1 << v.lgS;
  v.G = KB >> v.lgS;
  v.invHo = 1.f / (float)a.Ho;
  return v;
}

template <int BM, int BN, int KB, int EPI, int STAGES>
__global__ __launch_bounds__(NT, blocks_per_cu((BM + BN) * KB * 2 * STAGES)) void wgrad_kernel(GemmArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  static_assert(WM * 64 == BM, "tile shape");
  constexpr int A_ST = BM * KB * 2, B_ST = BN * KB * 2, ST = A_ST + B_ST;
  constexpr int NA = A_ST / 4096, NB = B_ST / 4096, NQ = NA + NB;
  constexpr int CPA = BM / 8, RPA = 64 / CPA;  // A: chunks per k-row, k-rows per 1-KB DMA
  constexpr int CPB = BN / 8, RPB = 64 / CPB;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * ST];

  const int tiles_n = gridDim.x, tiles = gridDim.x * gridDim.y;
  const int lin = tile::xcd_tile(blockIdx.y * tiles_n + blockIdx.x, tiles);
  const int tn = lin % tiles_n, tm = lin / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const VRow v = vrow_geo<KB>(a);
  const int rbeg = blockIdx.z * a.k_per_split;
  const int rend = min(a.K, rbeg + a.k_per_split);
  const int nk = (rend - rbeg + v.G - 1) / v.G;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const uint16_t* xs = (const uint16_t*)a.A;
  const uint16_t* dys = (const uint16_t*)a.B;
  const void* zero = tile::pinned_addr(g_zero16);
  const int Cin = a.Cin, Cout = a.N;

  // Per lane and DMA instruction j everything but the virtual row is fixed: the k-row
  // slot (-> pixel column), the row-in-step g and the column chunk (-> tap, channel).
  // Offsets split into a lane-constant part and a row part; the row state (image, oh,
  // segment) of the step's first virtual row is wave-uniform and advanced incrementally
  // (when nseg > 1, G == 1: the whole step is one virtual row).
  int a_off[NA], a_g[NA], a_khp[NA], a_iwrel[NA], a_slot[NA];
  bool a_ok[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int kr = (wave + 4 * j) * RPA + lane / CPA;
    a_slot[j] = kr & (v.S - 1);
    a_g[j] = kr >> v.lgS;
    const int ch = (lane % CPA) ^ tile::mc_swz<BM>(kr);
    const int m = m0 + 8 * ch;
    const int mm = min(m, a.M - 8);
    const int tap = mm / Cin, ci = mm - tap * Cin;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    a_iwrel[j] = a_slot[j] * a.stride - a.pad + kw;  // iw = ow0 * stride + iwrel
    a_khp[j] = kh - a.pad;                           // ih = oh * stride + khp
    a_off[j] = (a_khp[j] * a.W + a_iwrel[j]) * Cin + ci;
    a_ok[j] = m < a.M && a_slot[j] < v.Wv;
    // with one segment per row (ow0 == 0) the column checks are lane-constant
    if (v.nseg == 1) a_ok[j] = a_ok[j] && a_slot[j] < a.Wo && (unsigned)a_iwrel[j] < (unsigned)a.W;
  }
  int b_off[NB], b_g[NB], b_slot[NB];
  bool b_ok[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int kr = (wave + 4 * j) * RPB + lane / CPB;
    b_slot[j] = kr & (v.S - 1);
    b_g[j] = kr >> v.lgS;
    const int ch = (lane % CPB) ^ tile::mc_swz<BN>(kr);
    const int n = n0 + 8 * ch;
    b_ok[j] = n < Cout && b_slot[j] < v.Wv && (v.nseg > 1 || b_slot[j] < a.Wo);
    b_off[j] = b_slot[j] * Cout + min(n, Cout - 8);
  }
  // wave-uniform row state of virtual row R0 = rbeg + kt * G
  int q0 = v.nseg == 1 ? rbeg : rbeg / v.nseg;
  int seg0 = rbeg - q0 * v.nseg;
  int img0 = q0 / a.Ho, oh0 = q0 - img0 * a.Ho;
  const int HW_C = a.H * a.W * Cin, sW_C = a.stride * a.W * Cin, HoWo_C = a.Ho * a.Wo * Cout;

  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    char* sa = smem + stage * ST;
    const int R0 = rbeg + kt * v.G;
    const int ow0 = seg0 * v.Wv;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      int oh = oh0 + a_g[j];
      const int wrap = (int)(((float)oh + 0.5f) * v.invHo);  // exact: oh < 2^14
      oh -= wrap * a.Ho;
      const int img = img0 + wrap;
      const int ih = oh * a.stride + a_khp[j];
      bool ok = a_ok[j] && R0 + a_g[j] < rend && (unsigned)ih < (unsigned)a.H;
      if (v.nseg > 1)
        ok = ok && ow0 + a_slot[j] < a.Wo && (unsigned)(ow0 * a.stride + a_iwrel[j]) < (unsigned)a.W;
      const long off = (long)img * HW_C + (long)oh * sW_C + a_off[j] + (long)ow0 * a.stride * Cin;
      glds16(ok ? (const void*)(xs + off) : zero, sa + (wave + 4 * j) * 1024);
    }
    char* sb = sa + A_ST;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      int oh = oh0 + b_g[j];
      const int wrap = (int)(((float)oh + 0.5f) * v.invHo);
      oh -= wrap * a.Ho;
      const int img = img0 + wrap;
      bool ok = b_ok[j] && R0 + b_g[j] < rend;
      if (v.nseg > 1) ok = ok && ow0 + b_slot[j] < a.Wo;
      const long off = (long)img * HoWo_C + ((long)oh * a.Wo + ow0) * Cout + b_off[j];
      glds16(ok ? (const void*)(dys + off) : zero, sb + (wave + 4 * j) * 1024);
    }
    // advance the row state by G virtual rows (G == 1 whenever nseg > 1)
    if (v.nseg > 1) {
      if (++seg0 == v.nseg) { seg0 = 0; if (++oh0 == a.Ho) { oh0 = 0; ++img0; } }
    } else {
      oh0 += v.G;
      while (oh0 >= a.Ho) { oh0 -= a.Ho; ++img0; }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) __attribute__((always_inline)) {
    const char* ia = smem + stage * ST;
    const char* ib = ia + A_ST;
#pragma unroll
    for (int kk = 0; kk < KB / 32; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = tile::frag_mc<BM>(ia + kk * 32 * BM * 2, wm * 64 + i * 16, lane);
        bfr[i] = tile::frag_mc<BN>(ib + kk * 32 * BN * 2, wn * 64 + i * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
  };
  kloop<STAGES, NQ>(nk, issue, compute);
  tile::epilogue<BM, BN, EPI>(a, acc, m0, n0, tm, wm, wn, wave, lane, reinterpret_cast<float*>(smem));
}

// ---- launch configuration ------------------------------------------------------------
// k-step depth: per launch from the planner (GemmArgs::kstep), else DAMD_CONV_KB (32|64),
// default 64.  LDS stages: 2 (kloop supports 3-4; those measured slower, see the header).
constexpr int kStages = 2;
inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
inline int conv_kb() { return env_int("DAMD_CONV_KB", 64) == 32 ? 32 : 64; }

// DAMD_CONV_STAGES=3: a third LDS stage (A/B runs; 2 measured best, see the header)
inline int conv_stages() { return env_int("DAMD_CONV_STAGES", kStages) == 3 ? 3 : 2; }

template <int BM, int BN, int KB, bool DG, int EPI>
void launch_stages(dim3 grid, const GemmArgs& a, hipStream_t s) {
  if (conv_stages() == 3) hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, KB, DG, EPI, 3>), grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, KB, DG, EPI, 2>), grid, dim3(NT), 0, s, a);
}

template <int BM, int BN, bool DG, int EPI>
hipError_t launch_t(const GemmArgs& a, int splits, int kb, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  if (kb == 64) launch_stages<BM, BN, 64, DG, EPI>(grid, a, s);
  else launch_stages<BM, BN, 32, DG, EPI>(grid, a, s);
  return hipGetLastError();
}

template <int BM, int BN, bool DG>
hipError_t launch_epi(const GemmArgs& a, int epi, int splits, int kb, hipStream_t s) {
  switch (epi) {
    case E_BF16: return launch_t<BM, BN, DG, E_BF16>(a, splits, kb, s);
    case E_BIAS | E_BF16: return launch_t<BM, BN, DG, E_BIAS | E_BF16>(a, splits, kb, s);
    case E_BIAS | E_RELU | E_BF16: return launch_t<BM, BN, DG, E_BIAS | E_RELU | E_BF16>(a, splits, kb, s);
    case E_RELU | E_BF16: return launch_t<BM, BN, DG, E_RELU | E_BF16>(a, splits, kb, s);
    case E_SLAB: return launch_t<BM, BN, DG, E_SLAB>(a, splits, kb, s);
    case E_BF16 | E_STATS: return launch_t<BM, BN, DG, E_BF16 | E_STATS>(a, splits, kb, s);
    case E_BIAS | E_BF16 | E_STATS: return launch_t<BM, BN, DG, E_BIAS | E_BF16 | E_STATS>(a, splits, kb, s);
    case E_BF16 | E_ADD: return launch_t<BM, BN, DG, E_BF16 | E_ADD>(a, splits, kb, s);
    case E_FIXUP | E_BF16: return launch_t<BM, BN, DG, E_FIXUP | E_BF16>(a, splits, kb, s);
    case E_FIXUP | E_BF16 | E_STATS: return launch_t<BM, BN, DG, E_FIXUP | E_BF16 | E_STATS>(a, splits, kb, s);
    case E_FIXUP | E_BIAS | E_BF16: return launch_t<BM, BN, DG, E_FIXUP | E_BIAS | E_BF16>(a, splits, kb, s);
    case E_FIXUP | E_BIAS | E_BF16 | E_STATS:
      return launch_t<BM, BN, DG, E_FIXUP | E_BIAS | E_BF16 | E_STATS>(a, splits, kb, s);
    case E_FIXUP | E_RELU | E_BF16: return launch_t<BM, BN, DG, E_FIXUP | E_RELU | E_BF16>(a, splits, kb, s);
    case E_FIXUP | E_BIAS | E_RELU | E_BF16:
      return launch_t<BM, BN, DG, E_FIXUP | E_BIAS | E_RELU | E_BF16>(a, splits, kb, s);
    case E_FIXUP | E_BF16 | E_ADD: return launch_t<BM, BN, DG, E_FIXUP | E_BF16 | E_ADD>(a, splits, kb, s);
    default: return hipErrorInvalidValue;
  }
}

template <int BM, int BN, int KB, int EPI>
void launch_wgrad_stages(dim3 grid, const GemmArgs& a, hipStream_t s) {
  if (conv_stages() == 3) hipLaunchKernelGGL((wgrad_kernel<BM, BN, KB, EPI, 3>), grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((wgrad_kernel<BM, BN, KB, EPI, 2>), grid, dim3(NT), 0, s, a);
}

template <int BM, int BN>
hipError_t launch_wgrad(const GemmArgs& a, int epi, int splits, int kb, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  if (epi == E_SLAB) {
    if (kb == 64) launch_wgrad_stages<BM, BN, 64, E_SLAB>(grid, a, s);
    else launch_wgrad_stages<BM, BN, 32, E_SLAB>(grid, a, s);
  } else if (epi == E_ATOMIC) {
    if (kb == 64) launch_wgrad_stages<BM, BN, 64, E_ATOMIC>(grid, a, s);
    else launch_wgrad_stages<BM, BN, 32, E_ATOMIC>(grid, a, s);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

int conv_gemm_kstep() { return conv_kb(); }

int wgrad64_rows(int N, int Ho, int Wo, int kb) {
  return N * Ho * ((Wo + kb - 1) / kb);
}
int wgrad64_rows_per_step(int Wo, int kb) {
  const int nseg = (Wo + kb - 1) / kb, Wv = (Wo + nseg - 1) / nseg;
  int S = 1;
  while (S < Wv) S <<= 1;
  return kb / S;
}

hipError_t conv_gemm_launch(const GemmArgs& a, int amode, int epi, int splits, int tile, hipStream_t s) {
  if (a.kstep != 0 && a.kstep != 32 && a.kstep != 64) return hipErrorInvalidValue;
  const int kb = a.kstep ? a.kstep : conv_kb();
  if (amode == A_WGRAD64) {
    const int nseg = (a.Wo + kb - 1) / kb;
    // Cin == 4: the packed-tap stem (KW' = 8): each 8-element chunk is 2 input pixels whose
    // bounds agree (even stride, pad and width)
    const bool stem4 = a.Cin == 4 && a.KW % 2 == 0 && a.stride % 2 == 0 && a.pad % 2 == 0 && a.W % 2 == 0;
    if ((a.Cin % 8 && !stem4) || a.N % 8 || a.M != a.KH * a.KW * a.Cin || a.Ho < 1 || a.Wo < 1 ||
        a.K % (a.Ho * nseg))
      return hipErrorInvalidValue;
    if (a.K != wgrad64_rows(a.K / (a.Ho * nseg), a.Ho, a.Wo, kb) || a.K >= (1 << 21)) return hipErrorInvalidValue;
    const int G = wgrad64_rows_per_step(a.Wo, kb);
    if (splits < 1 || a.k_per_split < G || a.k_per_split % G || (long)splits * a.k_per_split < a.K ||
        (long)(splits - 1) * a.k_per_split >= a.K)
      return hipErrorInvalidValue;
    if (epi != E_SLAB && epi != E_ATOMIC) return hipErrorInvalidValue;
    return tile == 1 ? launch_wgrad<256, 64>(a, epi, splits, kb, s) : launch_wgrad<128, 128>(a, epi, splits, kb, s);
  }
  const bool dg = amode == A_DGRAD64;
  // packed-tap stem: 8 pixels x 4 channels per 32-deep k-step, pixel pairs never straddle
  // the image edge (even stride, pad and width)
  const bool stem = !dg && a.Cin == 4;
  if (stem && (kb != 32 || a.KW != 8 || a.stride % 2 || a.pad % 2 || a.W % 2)) return hipErrorInvalidValue;
  if ((!stem && a.Cin % kb) || a.N % 8 || a.M < 1 || a.K % kb || a.K != a.KH * a.KW * a.Cin)
    return hipErrorInvalidValue;
  if (splits < 1 || a.k_per_split % kb || a.k_per_split < kb || (long)splits * a.k_per_split < a.K ||
      (long)(splits - 1) * a.k_per_split >= a.K)
    return hipErrorInvalidValue;
  if (dg && a.kc != a.Cin) return hipErrorInvalidValue;
  if (dg && a.stride == 2) {
    // sub-pixel classes: even input extent, class-grid rows, no K split, no statistics
    if (a.H % 2 || a.W % 2 || a.M % ((a.H / 2) * (a.W / 2)) || splits != 1 || (epi & (E_SLAB | E_STATS)) ||
        a.pad < 0 || a.pad > 1)
      return hipErrorInvalidValue;
    splits = 4;  // grid z = the four parity classes
  } else if (dg && a.stride != 1) {
    return hipErrorInvalidValue;
  }
  if (!dg && a.ldb % 8) return hipErrorInvalidValue;
  if ((epi & E_SLAB) && (epi & ~E_SLAB)) return hipErrorInvalidValue;
  // E_FIXUP: a real K split over plain tiles (not the sub-pixel classes), slabs + tickets, a
  // statistics accumulator (per-tile partial rows would not match the finish's row blocks)
  if ((epi & E_FIXUP) && (splits < 2 || (dg && a.stride != 1) || !a.slab || !a.tickets || a.N % 4 ||
                          ((epi & E_STATS) && !a.stats_acc) || (epi & (E_SLAB | E_ATOMIC | E_BNRED))))
    return hipErrorInvalidValue;
  // the stem: input rows staged once per tile (conv_stem.hip; same tiles and bits)
  if (stem && stem_direct_ok(a, epi, splits)) return stem_direct_launch(a, epi, s);
  if (tile == 1)
    return dg ? launch_epi<256, 64, true>(a, epi, splits, kb, s) : launch_epi<256, 64, false>(a, epi, splits, kb, s);
  return dg ? launch_epi<128, 128, true>(a, epi, splits, kb, s) : launch_epi<128, 128, false>(a, epi, splits, kb, s);
}

}  // namespace damd
