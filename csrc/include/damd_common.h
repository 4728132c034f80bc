// Common device helpers for distributed_amd HIP kernels (gfx950 / CDNA4 only).
//
// - bf16 <-> f32 conversion by bit manipulation (round-to-nearest-even),
// - MFMA fragment vector types for v_mfma_f32_16x16x32_bf16,
// - the in-launch "last arriver" hand-off (agent-scope release/acquire, see
//   cdna_hip_programming.md §6 Guideline 16 / §5 split-K counter recipe).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace damd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// f32 -> bf16 (RNE, NaN-preserving) on the gfx950 hardware converter (v_cvt_pk_bf16_f32).
// A software version with a NaN branch turns into divergent control flow that
// serialises the surrounding LDS reads (measured: 16 us vs ~1 us for the conv loop).
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not for its
// outstanding global stores.  Neither does __syncthreads() on gfx950: its workgroup-scope
// fence need not wait for vector-memory stores (the ISA shows a bare s_barrier after a
// store loop), so a cross-device publish drains explicitly -- see damd_publish_drain().

// Cross-device publish protocol (sharded exchange, peer all-reduce): the payload stores
// go to uncached (MTYPE UC) staging; before the flag store that announces them, EVERY wave
// that issued payload waits for its stores' acknowledgements (s_waitcnt vmcnt(0)).  The
// markers below are assembly comments (no code): scripts/check_publish_isa.py reads them
// from the device assembly to tell a workgroup publish (payload from all waves: the drain
// must precede the workgroup barrier ahead of the flag) from a per-wave publish (the
// wave's own drain must precede its flag).
__device__ __forceinline__ void damd_publish_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// ---- order-independent BatchNorm statistics accumulators (layer_ops.h BNFin) ----
// Producer blocks add fp32 partials into shared accumulators with atomics; with fp64
// atomics the rounding of each add depends on the arrival order.  Here every value is an
// int64 fixed-point number (wrapping integer adds are associative and commutative, so a
// sum is bitwise independent of the order in which the blocks arrive):
//  * forward statistics (sum x, sum x^2; BNFin): ONE word, v rounded to a multiple of
//    2^-24.  The rounding (<= 3e-8 per partial) is far below the fp32 partials' own and
//    is divided by the element count (>= 64 x 7 x 7) before it meets eps = 1e-3.
//    Range: |sum| < 2^35.
//  * backward sums (sum dz, sum dz xhat; BNBwdFin -- gradients, ~1e-9 per element): TWO
//    words, hi = floor(v 2^24), lo = floor((v 2^24 - hi) 2^40) in [0, 2^40): resolution
//    2^-64, exact for |v| >= 2^-40; < 2^23 addends per lo word.  Layout per replica:
//    [sum hi][sum lo][second hi][second lo], C words each.
// A non-finite or out-of-range partial (|v| >= 2^30) is NOT added: it sets a sticky flag
// word instead (atomicOr; one flag per channel, in a plane after the replicas:
// acc[reps][K] then flag[K]), and every consumer that sees a set flag decodes NaN.  (Round
// 5 added a +-2^58 poison into the sum word itself: N poisoned partials wrapped to 0 for N a
// multiple of 64, +inf and -inf cancelled, and finite sums >= 2^33 decoded as NaN.)
// Range of a decoded sum: the int64 word, |sum| < 2^39.
__device__ __forceinline__ bool bnacc_ok(float v) { return fabsf(v) < 1073741824.f; }  // 2^30 (false for NaN)
__device__ __forceinline__ void bnacc_flag(long long* flag) {
  atomicOr(reinterpret_cast<unsigned long long*>(flag), 1ull);
}
__device__ __forceinline__ void bnacc_add1(long long* p, long long* flag, float v) {
  if (!bnacc_ok(v)) {
    bnacc_flag(flag);
    return;
  }
  const long long w = __double2ll_rn((double)v * 16777216.0);  // 2^24: exact scaling
  atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)w);
}
// (hi and lo live in separate planes -- p_hi[c], p_lo[c] -- so that a wave's 64 channels add
// into 512 contiguous bytes per word: interleaved pairs doubled bn_bwd_reduce, 141 -> 277 us
// per ResNet-18 step)
__device__ __forceinline__ void bnacc_add2(long long* p_hi, long long* p_lo, long long* flag, float v) {
  if (!bnacc_ok(v)) {
    bnacc_flag(flag);
    return;
  }
  const double d = (double)v * 16777216.0;
  const double fh = floor(d);
  const long long hi = (long long)fh;
  const long long lo = (long long)((d - fh) * 1099511627776.0);  // [0, 1) x 2^40: exact, then floor
  atomicAdd(reinterpret_cast<unsigned long long*>(p_hi), (unsigned long long)hi);
  if (lo) atomicAdd(reinterpret_cast<unsigned long long*>(p_lo), (unsigned long long)lo);
}
__device__ __forceinline__ double bnacc_value1(long long w, long long flag = 0) {
  if (flag) return __builtin_nan("");
  return (double)w * 5.9604644775390625e-08;  // 2^-24
}
__device__ __forceinline__ double bnacc_value2(long long hi, long long lo, long long flag = 0) {
  if (flag) return __builtin_nan("");
  return (double)hi * 5.9604644775390625e-08 + (double)lo * 5.42101086242752217e-20;  // 2^-24, 2^-64
}

// Sum over the 16 lanes of a DPP row (lanes 16 r .. 16 r + 15), on DPP moves: quad swaps,
// then the half-row and row mirrors; every lane of the row ends with the same bits (each
// step adds two equal partial sums, in either order).  VALU only: the __shfl_xor butterfly
// it replaces in the GEMM epilogues' statistics was four ds_bpermute LDS round trips.
__device__ __forceinline__ float row16_sum(float v) {
  auto dpp = [](float x, auto ctrl) __attribute__((always_inline)) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xf, 0xf, false));
  };
  v += dpp(v, std::integral_constant<int, 0xB1>{});   // quad_perm [1, 0, 3, 2]
  v += dpp(v, std::integral_constant<int, 0x4E>{});   // quad_perm [2, 3, 0, 1]
  v += dpp(v, std::integral_constant<int, 0x141>{});  // row_half_mirror
  return v + dpp(v, std::integral_constant<int, 0x140>{});  // row_mirror
}

#define DAMD_PUBLISH_WG() asm volatile(";damd.publish wg")
#define DAMD_PUBLISH_WAVE() asm volatile(";damd.publish wave")
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Load 8 consecutive bf16 (16 B, must be 16-B aligned) from LDS / global as an MFMA fragment.
__device__ __forceinline__ bf16x8 ld_frag(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

// Control block shared by the fused trainer kernels and the host.  32 x 4 B.
// Written by the host only between graph replays (stream-ordered memcpy).
struct Ctrl {
  float lr;                 // 0  learning rate
  float momentum;           // 1  SGD momentum (0 = plain SGD)
  int   nesterov;           // 2
  int   nsamples;           // 3  dataset rows
  int   row0;               // 4  rank * per-replica batch (offset inside global batch)
  int   global_batch;       // 5
  int   cursor;             // 6  step index inside the epoch (advanced on device)
  int   iterations;         // 7  optimizer iterations (advanced on device)
  int   cnt_a;              // 8  arrival ticket of the 2-launch step's forward kernel (counts forever)
  int   cnt_b;              // 9  arrival ticket of its backward kernel
  float acc_loss;           // 10 epoch accumulators (sum of per-sample loss)
  float acc_correct;        // 11
  float acc_count;          // 12
  int   wrap;               // 13 if > 0: cursor wraps modulo `wrap` (benchmark epochs)
  int   cur2;               // 14 step index as seen by the 2nd kernel of a step (set by the 1st)
  int   cur3;               // 15 step index as seen by the 3rd kernel (set by the 2nd)
  int   wpar;               // 16 which W1 buffer is current (0: inside P, 1: the alternate)
  int   flush_ticket;       // 17 arrival counter of flush_pending (its last block resets wpar)
  int   pending;            // 18 1: the gradient buffers hold a step's gradient whose SGD update
                            //    is still to be applied (set by the last kernel of a step,
                            //    cleared by flush: the first step after a flush applies none)
  int   par2;               // 19 step parity as seen by the 2nd kernel of a 2-launch step (set by the 1st)
  int   bad;                // 20 sticky: a fixed-point conversion met a non-finite / out-of-range
                            //    value (the fused step reports loss = NaN from then on)
  int   xcnt;               // 21 gradient-exchange epoch of the sharded multi-rank step (counts forever)
  int   xcnt2;              // 22 xcnt as seen by the step's bwd (set by its fwd)
  int   ticket;             // 23 arrival ticket of the sharded bwd (its last block publishes the
                            //    rank's small-gradient message)
  int   pend2;              // 24 `pending` as seen by the step's fwd (set by it): bwd folds the
                            //    previous step's metric tail only when there was one
  int   xgen;               // 25 input-data generation: the host bumps it whenever it changes the
                            //    cursor or the epoch's rows (tags the prefetched next batch)
  int   pad[6];
};
static_assert(sizeof(Ctrl) == 128, "Ctrl must be 128 bytes");

// Keras tf.keras SGD update (optimizer_v2/gradient_descent.py semantics):
//   momentum == 0 : w -= lr * g
//   else          : v = m * v - lr * g ; w += v            (nesterov: w += m * v - lr * g)
__device__ __forceinline__ void sgd_update(float w, float g, float v, float lr, float mom, int nest,
                                           float& wn, float& vn) {
  if (mom == 0.f) {
    wn = w - lr * g;
    vn = v;
  } else {
    vn = mom * v - lr * g;
    wn = nest ? (w + mom * vn - lr * g) : (w + vn);
  }
}

// Last-arriver election across the workgroups of one launch.  Every thread of the
// block must call it (contains __syncthreads).  `flag` is one int in the block's LDS.
// Returns true in every thread of the last block to arrive; that block may then read
// every other block's plain-stored partials (agent-scope acquire done here).
__device__ __forceinline__ bool last_arriver(int* counter, int nblocks, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// Diagnostic phase stamps (s_memrealtime, 100 MHz).  Stamps are kept in registers
// and written once at kernel end (a mid-kernel store makes hipcc wait vmcnt(0) and
// distorts what it measures).  `st` is null unless DAMD_STAMPS is set on the host.
struct Stamps {
  unsigned long long t[13];
};
__device__ __forceinline__ void stamp(Stamps& s, unsigned long long* st, int idx) {
  if (st != nullptr) s.t[idx] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void stamp_flush(const Stamps& s, unsigned long long* st, int n) {
  if (st != nullptr && threadIdx.x == 0)
    for (int i = 0; i < n; ++i) st[blockIdx.x * 16 + i] = s.t[i];
}

}  // namespace damd
