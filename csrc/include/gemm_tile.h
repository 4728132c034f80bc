// Device-side building blocks shared by the MFMA GEMM kernels (csrc/kernels/gemm.hip,
// csrc/kernels/conv_gemm.hip): LDS image layouts, fragment reads and the common epilogue.
//
// Output layout: the MFMAs are issued with swapped operands (C^T = B^T A^T), so after a
// 16x16x32 MFMA lane l holds C[row 16i + (l & 15)][cols 16j + 4(l >> 4) .. +3] of the
// wave's 64x64 block -- 4 consecutive columns of one row: 8/16-byte epilogue stores.
#pragma once
#include "damd_common.h"
#include "gemm.h"

namespace damd {
namespace tile {

typedef short s16x4 __attribute__((ext_vector_type(4)));

// gfx950 transpose read ds_read_b64_tr_b16 (lane gets 4 bf16 of one column)
__device__ __forceinline__ s16x4 ds_tr16(const void* lds_byte_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)((__attribute__((address_space(3))) char*)(
          (uintptr_t)lds_byte_ptr)));
}

// LDS-DMA (global_load_lds_dwordx4: 16 B per lane to lds_wave_base + 16 * lane) issued
// from inline asm.  Through the builtin, hipcc treats the DMA as a pending LDS write of
// unknown extent and emits s_waitcnt vmcnt(0) before the next ds_read -- i.e. every k-step
// drains the stages just issued for later k-steps, and no load overlaps the MFMAs (seen in
// the .s of every LDS-DMA kernel here).  From asm the DMA is invisible to hipcc's
// bookkeeping: the kernel's own counted vmcnt + s_barrier order it (and it must be drained
// before any compiler-counted global load).  M0 is saved and restored inside the statement
// (cdna_hip_programming.md: the LDS-DMA recipe); the "memory" clobber keeps LDS reads from
// being cached across it.
__device__ __forceinline__ void glds16(const void* src, const void* lds_wave_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_wave_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// Address of a device symbol held in SGPRs for the whole kernel: an opaque copy, so the
// "memory" clobbers of the DMA statements do not make hipcc reload it from the GOT (an
// s_load + lgkmcnt(0) in front of every DMA issue).
template <class T>
__device__ __forceinline__ const void* pinned_addr(const T* sym) {
  uint64_t a = reinterpret_cast<uint64_t>(sym);
  asm volatile("" : "+s"(a));
  return reinterpret_cast<const void*>(a);
}

// MC image: [k rows][COLS] bf16 (mn-contiguous operand); the 16-byte chunk ch of row r is
// stored at chunk ch ^ mc_swz(r).  The swizzle depends on r mod 32 only (k-steps of 32
// rows are images of their own) and is an involution per row, so a lane-linear
// global->LDS DMA fills it by reading source chunk (slot ^ mc_swz(r)).
template <int COLS>
__device__ __forceinline__ int mc_swz(int r) {
  if constexpr (COLS == 64) return (r & 3) ^ ((r >> 1) & 7);
  else return (((r & 3) << 2) ^ ((r >> 2) & 3)) & (COLS / 8 - 1);
}
template <int COLS>
__device__ __forceinline__ int mc_off(int r, int ch) {
  return r * (COLS * 2) + 16 * (ch ^ mc_swz<COLS>(r));
}
// fragment of columns c0..c0+15, k rows 0..31 of an MC image (two transpose reads)
template <int COLS>
__device__ __forceinline__ bf16x8 frag_mc(const char* img, int c0, int lane) {
  int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  int ch = (c0 >> 3) + (p >> 1);
  s16x4 lo = ds_tr16(img + mc_off<COLS>(8 * g + q, ch) + 8 * (p & 1));
  s16x4 hi = ds_tr16(img + mc_off<COLS>(8 * g + 4 + q, ch) + 8 * (p & 1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// ---- epilogue --------------------------------------------------------------------------
// acc[i][j]: the wave's 64x64 block (wave grid position wm, wn) of the BMxBN tile at
// (m0, n0), M-tile index tm.  red: >= 2*4*64 floats of LDS, free to use (all staging reads
// done).  Flags (gemm.h): +bias[n], +R[m][n] (bf16), BatchNorm statistics of the stored
// pre-ReLU values per (M-tile, split), ReLU, and bf16 / fp32 / atomic / slab stores.
// GEMM row -> output row of C (and R): identity, or a scatter such as the parity classes
// of the sub-pixel backprop-input (conv_gemm.hip).  Slabs (E_SLAB) keep GEMM rows.
struct RowIdentity {
  __device__ __forceinline__ size_t operator()(int m) const { return (size_t)m; }
};
template <int BM, int BN, int EPI, class RowOf = RowIdentity>
__device__ __forceinline__ void epilogue(const GemmArgs& a, f32x4 (&acc)[4][4], int m0, int n0, int tm, int wm,
                                         int wn, int wave, int lane, float* red, RowOf row_of = RowOf{}) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  float csum[4][4], csq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[j][e] = csq[j][e] = 0.f;
  // The epilogue's global operands (the residual R, or the BN input x and its coefficients)
  // are ALL requested before the first store: interleaved with the stores, which may alias
  // them, every (i, j) fragment waited for its own load -- 16 dependent memory round trips
  // per tile (the layer-1 backprop-input + BN-partials launch ran ~17 us longer than the
  // forward).  Out-of-range fragments load a clamped in-range address and are skipped below.
  constexpr bool kPre = (EPI & (E_ADD | E_BNRED)) != 0;
  static_assert((EPI & E_ADD) == 0 || (EPI & E_BNRED) == 0, "one prefetched epilogue operand");
  uint2 pre[kPre ? 4 : 1][kPre ? 4 : 1];
  float4 bco[(EPI & E_BNRED) ? 4 : 1][4];
  if constexpr (kPre) {
    const uint16_t* pbase = (EPI & E_ADD) ? (const uint16_t*)a.R : a.bnx;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + (lane & 15);
      const size_t orow = row_of(m < a.M ? m : 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
        pre[i][j] = *reinterpret_cast<const uint2*>(pbase + orow * a.ldc + (n < a.N ? n : 0));
      }
    }
    if constexpr (EPI & E_BNRED) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4), nc = n < a.N ? n : 0;
#pragma unroll
        for (int p = 0; p < 4; ++p) bco[j][p] = *reinterpret_cast<const float4*>(a.bnst + p * a.N + nc);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    const bool mok = m < a.M;
    const size_t orow = row_of(mok ? m : 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      const bool ok = mok && n < a.N;
      f32x4 v = acc[i][j];
      if constexpr (EPI & E_BIAS) {
        if (n < a.N) {
          float4 b = *reinterpret_cast<const float4*>(a.bias + n);
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
      }
      if constexpr (EPI & E_ADD) {
        if (ok) {
          const uint2 r = pre[i][j];
          v[0] += __uint_as_float(r.x << 16);
          v[1] += __uint_as_float(r.x & 0xffff0000u);
          v[2] += __uint_as_float(r.y << 16);
          v[3] += __uint_as_float(r.y & 0xffff0000u);
        }
      }
      if constexpr (EPI & E_STATS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = ok ? v[e] : 0.f;
          if constexpr (EPI & E_BF16) x = bf2f(f2bf(x));  // statistics of the stored values
          csum[j][e] += x;
          csq[j][e] += x * x;
        }
      }
      if constexpr (EPI & E_BNRED) {
        // BN-backward partials of the stored gradient dy: dz = dy * [bf16(relu(x sc + sh)) > 0]
        // (the mask exactly as bn_apply stored the ReLU output), sum dz, sum dz * xhat
        if (ok) {
          const uint2 xr = pre[i][j];
          const float xv[4] = {__uint_as_float(xr.x << 16), __uint_as_float(xr.x & 0xffff0000u),
                               __uint_as_float(xr.y << 16), __uint_as_float(xr.y & 0xffff0000u)};
          const float4 mu = bco[j][0], iv = bco[j][1], sc = bco[j][2], sh = bco[j][3];
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
      if (!ok) continue;
      if constexpr (EPI & E_SLAB) {
        float* c = (float*)a.C + ((size_t)blockIdx.z * a.M + m) * a.ldc + n;
        *reinterpret_cast<float4*>(c) = float4{v[0], v[1], v[2], v[3]};
      } else if constexpr (EPI & E_ATOMIC) {
        float* c = (float*)a.C + orow * a.ldc + n;
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(c + e, v[e]);
      } else if constexpr (EPI & E_BF16) {
        uint2 pk;
        pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>((uint16_t*)a.C + orow * a.ldc + n) = pk;
      } else {
        *reinterpret_cast<float4*>((float*)a.C + orow * a.ldc + n) = float4{v[0], v[1], v[2], v[3]};
      }
    }
  }
  if constexpr ((EPI & (E_STATS | E_BNRED)) != 0) {
    // reduce over the 16 rows held by lanes l&15 (DPP row sum), then over the wave grid's
    // M direction through LDS; one partial per column per M-tile: stats[tm][z][2][N]
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        csum[j][e] = row16_sum(csum[j][e]);
        csq[j][e] = row16_sum(csq[j][e]);
      }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int c = j * 16 + 4 * (lane >> 4) + e;  // column within the wave's 64
          red[(0 * 4 + wave) * 64 + c] = csum[j][e];
          red[(1 * 4 + wave) * 64 + c] = csq[j][e];
        }
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < BN) {
      const int wnn = t / 64, c = t % 64;
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s += red[(0 * 4 + w * WN + wnn) * 64 + c];
        q += red[(1 * 4 + w * WN + wnn) * 64 + c];
      }
      const int n = n0 + t;
      if (n < a.N) {
        if (a.stats_acc) {
          const size_t reps = a.stats_reps > 1 ? a.stats_reps : 1;
          const size_t rep = a.stats_reps > 1 ? tm % a.stats_reps : 0;
          if constexpr (EPI & E_BNRED) {  // BN-backward sums: two words per value
            long long* acc = a.stats_acc + rep * 4 * a.N;  // hi / lo planes
            long long* flag = a.stats_acc + reps * 4 * a.N + n;  // sticky plane after the replicas
            bnacc_add2(acc + n, acc + a.N + n, flag, s);
            bnacc_add2(acc + 2 * a.N + n, acc + 3 * a.N + n, flag, q);
          } else {  // forward statistics: one word per value
            long long* acc = a.stats_acc + rep * 2 * a.N;
            long long* flag = a.stats_acc + reps * 2 * a.N + n;
            bnacc_add1(acc + n, flag, s);
            bnacc_add1(acc + a.N + n, flag, q);
          }
        } else {
          float* st = a.stats + ((size_t)tm * gridDim.z + blockIdx.z) * 2 * a.N;
          st[n] = s;
          st[a.N + n] = q;
        }
      }
    }
  }
}

// XCD-aware tile order: consecutive workgroups are dispatched round-robin over the 8
// XCDs; remap (bijectively, any tile count) so that the N-tiles of one M-panel -- which
// share the A rows -- run on the same XCD (same L2).  Returns the linear tile index.
__device__ __forceinline__ int xcd_tile(int lin, int tiles) {
  const int q = tiles >> 3, r = tiles & 7, xcd = lin & 7, idx = lin >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace tile
}  // namespace damd
