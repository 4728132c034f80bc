// Device-side building blocks of the fused MNIST-CNN step kernels
// (csrc/kernels/convnet_step2.hip): model constants and flat-buffer layout, input-row
// staging, the conv 3x3 + bias + ReLU + 2x2 max-pool on MFMA, fixed-point sums.
#pragma once
#include "convnet.h"
#include "damd_common.h"

namespace damd {
namespace convnet {

constexpr int IMG = 28, NPIX = IMG * IMG;
constexpr int PO = 13, NPOS = PO * PO;      // pooled 13x13
constexpr int NF = 32;                       // conv filters
constexpr int FEAT = NPOS * NF;              // 5408
constexpr int HID = 64, NCLS = 10;
constexpr int OFF_WC = 0, OFF_BC = 288, NCONV = 320;
constexpr int OFF_W1 = NCONV, OFF_B1 = OFF_W1 + FEAT * HID;
constexpr int OFF_W2 = OFF_B1 + HID, OFF_B2 = OFF_W2 + HID * NCLS;
constexpr int NPARAM = OFF_B2 + NCLS;        // 347146
constexpr int OFF_LOSS = NPARAM, OFF_CORR = NPARAM + 1, OFF_CNT = NPARAM + 2;
constexpr int NGRAD = NPARAM + 6;            // padded to 16 B: 347152
constexpr int NSMALL = HID + HID * NCLS + NCLS;  // b1, W2, b2 contiguous: 714
constexpr int CH = 64;                       // images per chunk
constexpr int LG_CH = 6;                     // log2(CH)
// dense-1 accumulator row pitch (int64 elements): one 512-B row of 64 sums per image.
// Contiguous (64) is the default: rows 4 KB apart, to spread the forward's 57-deep
// same-address atomic chains over more memory channels, measured +1.1 us per step (the
// backward started 0.95 us later; same-box A/B, round 5)
#ifndef DAMD_HACC_PITCH
#define DAMD_HACC_PITCH 64
#endif
constexpr int HACC_PITCH = DAMD_HACC_PITCH;
constexpr int XR = 6;                        // staged input rows per image
constexpr int MAXPP = 4;                     // max pooled positions per fwd / bwd block
constexpr int XS_BYTES = CH * XR * IMG * 4;  // 43008
constexpr int HP = 72;                       // bf16 pitch of 64-wide tiles (conflict-free)
static_assert(CH == 1 << LG_CH, "chunk size");
static_assert(HACC_PITCH >= 64 && HACC_PITCH % 64 == 0, "hacc pitch");
static_assert(NPARAM == kConvNetNParam && NGRAD == kConvNetNGrad, "param count");

__host__ __device__ constexpr int kpitch(int pp) { return pp * 32 + 8; }
__host__ __device__ constexpr int nsp(int ns) { return (ns + 3) & ~3; }

typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint16_t bf16_lo(float v, uint16_t hi) { return f2bf(v - bf2f(hi)); }

// next step index (wraps for benchmark epochs)
__device__ __forceinline__ int next_cursor(const Ctrl& c, int cur) {
  return (c.wrap > 0 && cur + 1 >= c.wrap) ? 0 : cur + 1;
}

// ---- staged input rows: registers first (loads in flight early), LDS later ------------
// A block stages rows [r0, r0 + nrows) of nimg = 2^lgi images (16 or 64) into the
// [nimg][XR][28] LDS tile.  One unit = 4 pixels: 4 B (u8) or 16 B (fp32).  Thread t owns
// column unit q = t & 7 (q = 7: idle) of rows rg, rg + RG, ... of image t >> (9 - lgi),
// where 512 / nimg threads share an image in RG = 2^(6 - lgi) row groups (64 images: all 6
// rows per thread; 16: rows rg, rg + 4).  Shifts only: the former linear unit index took a
// division per unit -- ~20 VALU each, quarter-rate multiplies among them -- and the
// prologue of both step kernels is VALU-issue bound (two waves per SIMD, wave64 over 16
// lanes: 4 clocks per VALU instruction).
template <bool U8>
struct XStage;
template <>
struct XStage<true> {
  uint32_t w[XR];
  int off, rg;  // LDS float offset of (image, row rg, unit q), -1: idle lane; row group
};
template <>
struct XStage<false> {
  float4 v[XR];
  int off, rg;
};
// Images b < nvalid with row_base + b < nsamples are loaded, others staged as zeros.
// U8: the dataset is kept as uint8 (inputs that are exactly k/255, e.g. MNIST) -- 4x fewer
// bytes -- and k/255.f (correctly rounded, == float32(k/255.0)) is formed when staging;
// otherwise fp32 rows.  32-bit sample indices and byte offsets (the engine keeps the
// dataset below 2^31 bytes), so the loads take the scalar-base + 32-bit-offset form.
// t: the staging slot (thread index by default; a block may give one thread two slots)
template <bool U8>
__device__ __forceinline__ void x_load(XStage<U8>& st, const void* __restrict__ X, long row_base, int nsamples,
                                       int nvalid, int lgi, int r0, int nrows, int t = (int)threadIdx.x) {
  const int sh = 9 - lgi, b = t >> sh, rg = (t & ((1 << sh) - 1)) >> 3, q = t & 7;
  const int RG = 1 << (6 - lgi);
  const int g = (int)row_base + b;
  const bool ok = b < nvalid && g < nsamples && q < 7;
  st.off = q < 7 ? (b * XR + rg) * IMG + 4 * q : -1;
  st.rg = rg;
  // element offset of (row r0 + rg, unit q); rows advance by RG * IMG elements
  const unsigned eo = __umul24((unsigned)max(0, min(g, nsamples - 1)), (unsigned)NPIX) + (unsigned)((r0 + rg) * IMG + 4 * q);
  // one 64-bit base per thread, rows at a uniform byte stride (per-row 32-bit offsets became
  // a quarter-rate 64-bit multiply-add per row)
  constexpr int ES = U8 ? 1 : 4;
  const char* xb = static_cast<const char*>(X) + (size_t)eo * ES;
  const int rstride = RG * IMG * ES;
#pragma unroll
  for (int j = 0; j < XR; ++j) {
    if constexpr (U8) st.w[j] = 0u;
    else st.v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j * RG >= XR) continue;  // (uniform)
    if (ok && rg + j * RG < nrows) {
      const char* pj = xb + j * rstride;
      if constexpr (U8) st.w[j] = *reinterpret_cast<const uint32_t*>(pj);
      else st.v[j] = *reinterpret_cast<const float4*>(pj);
    }
  }
}

// k / 255 rounded to fp32 exactly as float32(k / 255.0) for every k < 256 (checked for all
// 256 with exact fma arithmetic): q = k * (1/255) plus one fma-residual correction -- three
// VALU ops instead of a correctly rounded division (~10) or an LDS table read (a serial
// LDS round trip per staged unit)
__device__ __forceinline__ float u8_over_255(uint32_t k) {
  const float r = 1.f / 255.f, x = (float)k, q = x * r;
  return fmaf(fmaf(-q, 255.f, x), r, q);
}
template <bool U8>
__device__ __forceinline__ void x_store(const XStage<U8>& st, float* xs, int lgi, int nrows) {
  const int RG = 1 << (6 - lgi);
  if (st.off < 0) return;
#pragma unroll
  for (int j = 0; j < XR; ++j) {
    if (j * RG >= XR) continue;  // (uniform)
    if (st.rg + j * RG < nrows) {
      float4 v;
      if constexpr (U8) {
        const uint32_t w = st.w[j];
        v = make_float4(u8_over_255(w & 0xff), u8_over_255((w >> 8) & 0xff), u8_over_255((w >> 16) & 0xff),
                        u8_over_255(w >> 24));
      } else {
        v = st.v[j];
      }
      *reinterpret_cast<float4*>(xs + st.off + j * RG * IMG) = v;
    }
  }
}

// ---- conv 3x3 + bias + ReLU + 2x2 max-pool of a slice on MFMA ----
// One 16x16x32 bf16 MFMA per tile with a split-precision K packing:
//   k in [0,9): x_hi*w_hi   [9,18): x_lo*w_hi   [18,27): x_hi*w_lo   [27,32): 0
// (x = hi + lo, w = hi + lo in bf16) -> ~16-bit-mantissa conv outputs, so the pool
// argmax / ReLU mask match an fp32 conv; the 23 spare K slots of a 9-tap conv pay it.
// Row tile rt = 4 pool windows x 4 sub-pixels (window wi = pl*64 + image), so the 4
// pixels of one window are the 4 accumulator rows of one lane: bias + ReLU + max +
// first-max argmax happen in registers.  Per-lane tap offsets / bit masks make the
// hi/lo selection branch-free (a ?: on the value turns into divergent control flow that
// serialises the LDS reads).
struct ConvFrag {
  bf16x8 w[2];
  float bias[2];
  int toff[8];
  uint32_t lomask[8], zmask[8];
};
__device__ __forceinline__ void conv_setup(ConvFrag& f, const float* cw, int lane) {
  const int kg = lane >> 4;
  // slot k = 8 kg + j: tap (8 kg + j) mod 9 = (j - kg) mod 9; the x-lo slots (part 1, k in
  // [9, 18)), w-lo slots (part 2, [18, 27)) and zero slots (k >= 27) of group kg as bit masks
  // over j -- shifts and selects, not the divisions by 9 and 3 (~10 VALU per slot, sunk by
  // hipcc into the conv loop)
  const unsigned xlo = (0x0003FE00u >> (8 * kg)) & 0xffu, wlo = (0x07FC0000u >> (8 * kg)) & 0xffu;
  const unsigned zer = kg == 3 ? 0xF8u : 0u;
  int tapj[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = j - kg;
    tapj[j] = t < 0 ? t + 9 : t;
    f.toff[j] = tapj[j] + (IMG - 3) * ((tapj[j] * 11) >> 5);  // (tap / 3) * IMG + tap % 3, tap < 9
    f.lomask[j] = (xlo >> j) & 1u ? 0xffffu : 0u;
    f.zmask[j] = (zer >> j) & 1u ? 0u : 0xffffu;
  }
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s16x8 t;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float w32 = cw[tapj[j] * NF + 16 * nt + (lane & 15)];
      const uint32_t hi = f2bf(w32), lo = bf16_lo(w32, (uint16_t)hi);
      const uint32_t wlomask = (wlo >> j) & 1u ? 0xffffu : 0u;
      t[j] = (short)((hi ^ ((hi ^ lo) & wlomask)) & f.zmask[j]);
    }
    f.w[nt] = __builtin_bit_cast(bf16x8, t);
    f.bias[nt] = cw[OFF_BC + 16 * nt + (lane & 15)];
  }
}
// emit(image, pl, channel, pooled_bf16, code) for every pooled output of the slice
template <class Emit>
__device__ __forceinline__ void conv_pool(const ConvFrag& f, const float* xs, int p0, int np, int r0, int lg,
                                          int wave, int lane, Emit&& emit) {
  const int nrt = (np << lg) >> 2;  // np positions x 2^lg images / 4 windows per tile
  for (int rt = wave; rt < nrt; rt += 8) {
    s16x8 at;
    {
      const int r = lane & 15, wi = 4 * rt + (r >> 2), sub = r & 3;
      const int pl = wi >> lg, b = wi & ((1 << lg) - 1), pos = p0 + pl, py = pos / PO, px = pos - py * PO;
      const float* base = xs + (b * XR + 2 * py - r0 + (sub >> 1)) * IMG + 2 * px + (sub & 1);
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = base[f.toff[j]];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t hi = f2bf(v[j]), lo = bf16_lo(v[j], (uint16_t)hi);
        at[j] = (short)((hi ^ ((hi ^ lo) & f.lomask[j])) & f.zmask[j]);
      }
    }
    const bf16x8 a = __builtin_bit_cast(bf16x8, at);
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    const f32x4 c0 = mfma16(a, f.w[0], zero);
    const f32x4 c1 = mfma16(a, f.w[1], zero);
    const int wo = 4 * rt + (lane >> 4), plo = wo >> lg, bo = wo & ((1 << lg) - 1);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const f32x4 cc = nt ? c1 : c0;
      float best = fmaxf(cc[0] + f.bias[nt], 0.f);
      int arg = 0;
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        const float v = fmaxf(cc[j] + f.bias[nt], 0.f);
        arg = v > best ? j : arg;
        best = fmaxf(best, v);
      }
      emit(bo, plo, 16 * nt + (lane & 15), f2bf(best), (uint8_t)(arg | (best > 0.f ? 4 : 0)));
    }
  }
}

// ---- fixed-point cross-block sums, DPP row reductions, small MFMA, SGD-or-keep ----------
constexpr float HSCALE = 4294967296.f;          // 2^32
constexpr double HINV = 1.0 / 4294967296.0;
constexpr float CSCALE = 1099511627776.f;       // 2^40
constexpr double CINV = 1.0 / 1099511627776.0;

// |v * scale| < 2^54: a sum of up to 512 such terms (57 slices x 8 ranks) stays inside int64.
// Anything else -- NaN, inf, a diverged partial -- is not representable: it is counted as 0
// and raises the sticky ctrl->bad flag, and the step reports loss = NaN from then on (the
// fp32 engines would show the NaN; a wrapped integer must not turn it into finite garbage)
constexpr float FIX_LIMIT = 18014398509481984.f;  // 2^54
__device__ __forceinline__ long long to_fix(float v, float scale, int* bad) {
  const float q = v * scale;
  if (!(fabsf(q) < FIX_LIMIT)) {
    __hip_atomic_fetch_or(bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  return (long long)__builtin_rintf(q);
}
// fixed point -> float as (q >> 24) * 2^24 + (q & (2^24 - 1)) in one fma: f32 only (the
// former (float)((double)q * inv) took ~6 half-rate f64 instructions per value, and the
// head converts 8 per thread).  Both parts are exact floats for |q| < 2^48 (the signed
// high part is arithmetic-shifted, the low part has 24 bits), so the fma rounds ONCE: the
// correctly rounded value, negative q included (round 5 split at 2^32 and rounded the
// unsigned low word first: q = -5 decoded to 0).  inv is a power of two.
__device__ __forceinline__ float from_fix(long long q, double inv) {
  const float fi = (float)inv;
  return fmaf((float)(q >> 24), fi * 16777216.f, (float)(int)(q & 0xFFFFFF) * fi);
}

__device__ __forceinline__ void atomic_add_i64(long long* p, long long v) {
  __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}

// Reductions over the 16 lanes of a DPP row (one MFMA output column group) on DPP moves:
// quad swaps, then half-row and row mirrors; every lane ends with the row's result, and
// the combination order is fixed (deterministic).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_QSWAP1 = 0xB1, DPP_QSWAP2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dppf<DPP_QSWAP1>(v));
  v = fmaxf(v, dppf<DPP_QSWAP2>(v));
  v = fmaxf(v, dppf<DPP_HMIRROR>(v));
  return fmaxf(v, dppf<DPP_MIRROR>(v));
}
// (row16_sum: damd_common.h, the same DPP sequence, shared with the GEMM epilogues)
__device__ __forceinline__ int row16_min(int v) {
  v = min(v, dppi<DPP_QSWAP1>(v));
  v = min(v, dppi<DPP_QSWAP2>(v));
  v = min(v, dppi<DPP_HMIRROR>(v));
  return min(v, dppi<DPP_MIRROR>(v));
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void sgd_or_keep(bool pend, float w, float g, float v, const Ctrl& c, float& wn,
                                            float& vn) {
  if (pend) {
    sgd_update(w, g, v, c.lr, c.momentum, c.nesterov, wn, vn);
  } else {
    wn = w;
    vn = v;
  }
}

}  // namespace convnet
}  // namespace damd
