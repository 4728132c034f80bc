// Two-launch data-parallel training step for the reference MNIST CNN (gfx950 / MI355X).
//
// Model (reference README.md:58-73): Conv2D(32,3x3,valid)+bias+ReLU
// -> MaxPool 2x2 -> Flatten(NHWC, 5408) -> Dense(64)+bias+ReLU -> Dense(10) ->
// SparseCategoricalCrossentropy(from_logits); SGD(lr, momentum, nesterov) on fp32 masters.
//
// Why two launches: at B = 64 the step is a chain of dependent memory round trips, and
// every launch costs ~2.5-3 us of prologue latency plus ~2.8 us of drain + dispatch
// (profiles/r02_mnist phase stamps).  The 3-launch step (convnet_fused.hip) needed its
// middle kernel only to combine the 57 dense-1 split-K slabs per row; here those partial
// sums, and the conv-gradient partials, are combined by integer atomics on fixed-point
// values, so the combine needs no extra launch and -- unlike fp32 atomics -- its result
// does not depend on arrival order: every step is bitwise reproducible.
//
//   fwd (grid NS slices x IG image groups, 512 thr): the pending SGD update of the W1
//       slice and of the conv parameters (both double-buffered by step parity: every
//       block updates in registers, one owner block writes the next buffer) and of
//       b1/W2/b2 (two owner blocks); conv + bias + ReLU + 2x2 max-pool on MFMA (pooled
//       tile + argmax codes stored for bwd); the dense-1 partial of the slice on MFMA,
//       added into hacc[par][row][n] as round(v * 2^32) with 64-bit atomics.
//   bwd (grid NS slices, 512 thr): every block converts hacc back, adds b1, and runs the
//       whole head redundantly: Dense(10) logits on f32 MFMA (16x16x4, exact fp32) with
//       softmax-xent / accuracy / dz by 16-lane shuffles in the same waves, dh as a bf16
//       hi+lo pair in both MFMA operand layouts in LDS (no global round trip for dh), its
//       share of the b1/W2/b2 gradient and of the metric tail (fixed row order);
//       dW1 = P^T dh and dP = dh W1^T on MFMA; MaxPool/ReLU backward through the stored
//       argmax codes fused into this slice's conv weight-gradient partial, added into
//       hconv[par] as round(v * 2^40) with 64-bit atomics; the dead parity of hacc is
//       zeroed for the next step.
//   No block waits on another: there is no ticket / last-arriver hand-off inside either
//   launch (a returning atomic on a contended counter stalled its wave ~1.5-2 us).
//
// Fixed point: h partials are fp32 MFMA sums of |v| < 2^31; x 2^32 keeps every bit a
// float carries down to 2^-32 (the sum of 57 roundings is < 1.4e-8 absolute); conv
// gradient partials x 2^40 (resolution 9e-13, range 8e6).  Integer addition is
// associative, so ranks and replays agree bitwise; the all-reduce sums both int64
// parities exactly too (the dead one is re-zeroed before its next use).
//
// Step counter / parity without intra-kernel races: fwd block 0 copies ctrl.cursor and
// ctrl.wpar to cur2 / par2; bwd reads those and its block 0 advances cursor / iterations,
// flips wpar and sets `pending`; no kernel uses a ctrl field that the same kernel writes.
#include "convnet_dev.h"

// Timing probes (wrong numerics, never in a product build): a probe build compiles this
// file with -DDAMD_PROBE_HACC=1|2 (skip all / half of the dense-1 atomics) or
// -DDAMD_PROBE_HCONV=1 (skip the conv-gradient atomics); scripts/probe_build.py makes one
// in a scratch directory.  The default build has both at 0, so the branches fold away.
#ifndef DAMD_PROBE_HACC
#define DAMD_PROBE_HACC 0
#endif
#ifndef DAMD_PROBE_HCONV
#define DAMD_PROBE_HCONV 0
#endif

namespace damd {
namespace convnet2 {
using namespace convnet;

constexpr int NAUX2 = NSMALL + 3;               // b1/W2/b2 gradients + [loss, correct, count]
constexpr int HPITCH = HID + 1;                 // fp32 pitch of the h tile in LDS
constexpr int ZP = 17;                          // pitch of the logit / dz rows (16 lanes store, odd: no conflicts)
constexpr int HEAD_FLOATS = CH * HPITCH + 716 + CH * ZP + 2 * CH + 16 * HID + CH;
constexpr int HEAD_BYTES = HEAD_FLOATS * 4;

// ---- sharded multi-rank exchange (XArgs, convnet.h) ----------------------------------
// Flag words live in every rank's uncached `out` staging; a flag holds the exchange epoch
// E (ctrl.xcnt after the step's bwd) of the last message it announces.  Publish: a wave
// drains its stores (s_waitcnt vmcnt(0): uncached stores are acknowledged by the owning
// device's memory) and one lane stores E with a relaxed system-scope atomic.  Consume: a
// lane polls with relaxed system-scope loads; the data loads follow in program order
// (uncached: nothing stale in any L1 / L2).  Every wait is bounded: on expiry the status
// word records which kind of wait expired and the kernel goes on (no GPU hang; the host
// raises on a non-zero status).
constexpr int SM_CONV = 0, SM_GRAD = 2 * NCONV, SM_MET = SM_GRAD + NSMALL;  // small-message fields
static_assert(SM_MET + 3 <= kXSmsg, "small message");
__device__ __forceinline__ unsigned* x_flags(float* out) { return reinterpret_cast<unsigned*>(out + kXFlags); }
__device__ __forceinline__ unsigned* x_pflag(float* out, int u, int slot) {
  return x_flags(out) + u * kXPFlagPitch + slot;
}
__device__ __forceinline__ unsigned* x_gflag(float* out, int nu, int u, int half) {
  return x_flags(out) + nu * kXPFlagPitch + u * 2 + half;
}
__device__ __forceinline__ unsigned* x_sflag(float* out, int nu, int par, int src) {
  return x_flags(out) + nu * (kXPFlagPitch + 2) + par * kXMaxRanks + src;
}
__device__ __forceinline__ float* x_small(float* out, int par, int src) {
  return out + kXSmall + ((long)par * kXMaxRanks + src) * kXSmsg;
}
__device__ __forceinline__ void x_signal(unsigned* f, unsigned e) {
  __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void x_wait(const XArgs& xa, unsigned* f, unsigned e, unsigned bit) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
    __builtin_amdgcn_s_sleep(1);
    const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
    if (dt > xa.timeout_ticks) {
      __hip_atomic_fetch_or(xa.status, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    // past 1 ms: give up at once when an earlier wait already expired (a broken exchange
    // costs one deadline, not one per wait of every later step; the host raises on status)
    if (dt > 100000ull && __hip_atomic_load(xa.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
  }
}
constexpr unsigned XW_SMALL = 1u << 8, XW_UNIT = 1u << 9, XW_PART = 1u << 10;  // status bits
__device__ __forceinline__ uint2 pack_bf16x4(const f32x4& v) {
  return make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                    (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
}
__device__ __forceinline__ float4 unpack_bf16x4(uint2 q) {
  return make_float4(bf2f((uint16_t)(q.x & 0xffffu)), bf2f((uint16_t)(q.x >> 16)), bf2f((uint16_t)(q.y & 0xffffu)),
                     bf2f((uint16_t)(q.y >> 16)));
}

// =================================================================================
// fwd: grid (NS slices, IG image groups of IB = 2^lg images)
// =================================================================================
template <bool U8>
// (ctrl and X lead the argument list: with kernarg preloading they arrive in SGPRs, so
// the first dependent loads -- the ctrl block, then the batch rows -- start at once)
// (the first 16 argument dwords arrive preloaded in SGPRs: the pointers of the prologue's
// first loads and the packed sizes their addresses need -- bpp = B | PP << 16, lge = lg |
// eager << 8; later arguments come from the kernarg segment, a scalar load's latency behind)
__global__ __launch_bounds__(512) void fwd(const void* __restrict__ xnext, uint16_t* __restrict__ w1bf,
                                           float* __restrict__ P, float* __restrict__ V,
                                           float* __restrict__ calt, const long long* __restrict__ hconv_r,
                                           const float* __restrict__ G, int bpp, int lge, Ctrl* __restrict__ ctrl,
                                           const void* __restrict__ X, float* __restrict__ W1alt,
                                           float* __restrict__ V1alt, uint16_t* __restrict__ pooled,
                                           uint8_t* __restrict__ code, long long* __restrict__ hacc,
                                           long long* __restrict__ hconv, unsigned long long* st, const XArgs xa,
                                           const long long* __restrict__ xtag, const int* __restrict__ labels,
                                           void* __restrict__ xcur, int* __restrict__ ycur, int phint) {
  const int B = bpp & 0xffff, PP = bpp >> 16, lg = lge & 0xff, eager = lge >> 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool sh = xa.world > 1;  // sharded multi-rank step: gradients from the exchange staging
  constexpr int hprobe = DAMD_PROBE_HACC;  // 0 in every product build (see the top of the file)
  const int nblk = gridDim.x * gridDim.y, lin = blockIdx.y * gridDim.x + s;
  Stamps sts;
  stamp(sts, st, 0);
  const int IB = 1 << lg, img0 = blockIdx.y * IB;
  const int BP = (B + CH - 1) / CH * CH;
  const int p0 = s * PP, p1 = min(NPOS, p0 + PP), np = p1 - p0, K = np * 32;
  const int KP = kpitch(PP);
  float* xs = reinterpret_cast<float*>(smem);                              // [IB][XR][28]; later [IB][64] partials
  uint16_t* as = reinterpret_cast<uint16_t*>(smem + IB * XR * IMG * 4);    // [IB][KP] pooled tile
  uint16_t* w1t = as + IB * KP;                                            // [HID][KP] W1 slice^T
  float* cw = reinterpret_cast<float*>(w1t + HID * KP);                    // [320] conv params
  const int n4 = K * HID / 4;  // <= 2048
  const int r0 = 2 * (p0 / PO);
  const int nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  // ---- the batch rows as the previous step's bwd prefetched them (xnext): issued first,
  // before the ctrl block is known; kept below if their tag names this step's rows ----
  XStage<U8> xst;
  long long xt = 0;
  if (xnext != nullptr) {
    x_load<U8>(xst, xnext, img0, B, B - img0, lg, r0, nrows);
    xt = *xtag;
  }
  // ---- first the loads whose addresses do not depend on the ctrl block: the bf16 W1 slice
  // (eager), both parities of the conv parameters, the b1/W2/b2 triplet; the scheduling
  // barrier keeps them ahead of the ctrl load (left alone, hipcc issued the ctrl load first
  // and waited for it with the kernel arguments, then sank these below further waits) ----
  uint4 bq[2];  // eager: the bf16 W1 slice (bwd already applied the update)
  if (eager) {
    // (lanes past the slice load nothing: at PP = 2 the second unit is all out of range, and
    // its clamped duplicate loads were 8 KB per block of wasted load bandwidth.  Written as a
    // conditional load, not a select between pointers: hipcc turns the latter into a flat
    // load from a zero vector in scratch)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bq[u] = make_uint4(0u, 0u, 0u, 0u);
      if (tid + u * 512 < n4 / 2) bq[u] = reinterpret_cast<const uint4*>(w1bf + p0 * 32 * HID)[tid + u * 512];
    }
  }
  // conv parameters: current buffer by parity; their gradient is the previous step's
  // (bwd added it into hconv[par ^ 1])
  const int tcl = min(tid, NCONV - 1);
  const float cp0 = P[tcl], cp1 = calt[tcl], cv0 = V[tcl], cv1 = calt[NCONV + tcl];
  const long long cq0 = sh ? 0 : hconv_r[NCONV + tcl], cq1 = sh ? 0 : hconv_r[tcl];
  // b1/W2/b2: the grid's last two blocks own their pending update (nobody else in this
  // launch reads them; bwd reads the updated values)
  const int si = (lin - (nblk - 2)) * 512 + tid;
  const bool small_on = lin >= nblk - 2 && si >= 0 && si < NSMALL;
  const int sic = OFF_B1 + max(0, min(si, NSMALL - 1));
  const float sp = P[sic], sg0 = sh ? 0.f : G[sic], sv = V[sic];
  __builtin_amdgcn_sched_barrier(0);

  const Ctrl c = *ctrl;
  const int par = phint >= 0 ? phint : c.wpar;
  if (phint >= 0 && phint != c.wpar && lin == 0 && tid == 0)
    __hip_atomic_fetch_or(&ctrl->bad, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned xe = (unsigned)c.xcnt;  // sharded: exchange epoch of the pending update
  if (lin == 0 && tid == 0) {
    ctrl->cur2 = c.cursor;
    ctrl->par2 = par;
    ctrl->xcnt2 = c.xcnt;
    ctrl->pend2 = c.pending;
  }
  const bool pend = c.pending != 0;
  const long row_base = (long)c.cursor * c.global_batch + c.row0 + img0;
  const bool mom = c.momentum != 0.f;

  // ---- then the ctrl-dependent loads: the batch rows unless prefetched (and, deferred
  // update, W1 by parity) ----
  const bool xhit = xnext != nullptr && xt == (((long long)c.xgen << 32) | (long long)(unsigned)(c.cursor + 1));
  if (!xhit) x_load<U8>(xst, X, row_base, c.nsamples, B - img0, lg, r0, nrows);
  // this step's rows and labels for the backward (xcur / ycur): a share per block, from the
  // prefetch when it hit (L2-hot), else from the dataset; stored at the end of the kernel
  constexpr int UPI = U8 ? NPIX / 16 : NPIX / 4;  // 16-byte units per image
  const int xcu = lin * 512 + tid;
  const bool xcp = xcur != nullptr && xcu < B * UPI;
  uint4 xcv = make_uint4(0u, 0u, 0u, 0u);
  int ycv = -1;
  {
    const long rb0 = (long)c.cursor * c.global_batch + c.row0;
    if (xcp) {
      const int b = xcu / UPI, q = xcu - b * UPI;
      if (xhit) xcv = reinterpret_cast<const uint4*>(xnext)[xcu];
      else if (rb0 + b < c.nsamples)
        xcv = reinterpret_cast<const uint4*>(static_cast<const char*>(X) +
                                             __umul24((unsigned)(rb0 + b), U8 ? NPIX : 4 * NPIX))[q];
    }
    if (xcur != nullptr && lin == 0 && tid < B && rb0 + tid < c.nsamples) ycv = labels[rb0 + tid];
  }
  float4 wv[4], gv[4], vv[4];
  const float* Wcur = par ? W1alt : P + OFF_W1;
  const float* Vcur = par ? V1alt : V + OFF_W1;
  float* Wnext = par ? P + OFF_W1 : W1alt;
  float* Vnext = par ? V + OFF_W1 : V1alt;
  const float4* P4 = reinterpret_cast<const float4*>(Wcur + p0 * 32 * HID);
  const float4* G4 = reinterpret_cast<const float4*>(G + OFF_W1 + p0 * 32 * HID);
  const float4* V4 = reinterpret_cast<const float4*>((mom ? Vcur : Wcur) + p0 * 32 * HID);
  const bool owner = blockIdx.y == 0;
  float4* Wn4 = reinterpret_cast<float4*>(Wnext + p0 * 32 * HID);
  float4* Vn4 = reinterpret_cast<float4*>(Vnext + p0 * 32 * HID);
  uint2* Wb = reinterpret_cast<uint2*>(w1bf + p0 * 32 * HID);
  if (!eager) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ic = min(tid + u * 512, n4 - 1);
      wv[u] = P4[ic];
      gv[u] = sh ? make_float4(0.f, 0.f, 0.f, 0.f) : G4[ic];  // sharded: after its unit flags
      vv[u] = V4[ic];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  const float cp = par ? cp1 : cp0, cv = par ? cv1 : cv0;
  long long cq = par ? cq1 : cq0;
  float sg = sg0;
  // sharded: the previous step's conv / b1 / W2 / b2 gradients and metric tail are the
  // rank-ordered sums of every rank's small message (published by each rank's last bwd block)
  if (sh && pend) {
    const int ps = xe & 1;
    float* xo = xa.out[xa.rank];
    if (tid < xa.world) x_wait(xa, x_sflag(xo, 4 * ((NPOS + xa.ppb - 1) / xa.ppb), ps, tid), xe, XW_SMALL);
    __syncthreads();
    long long q = 0;
    float g = 0.f;
    for (int r = 0; r < xa.world; ++r) {
      const float* m = x_small(xo, ps, r);
      q += reinterpret_cast<const long long*>(m + SM_CONV)[tcl];
      if (small_on) g += m[SM_GRAD + max(0, min(si, NSMALL - 1))];
    }
    cq = q;
    sg = g;
    if (lin == nblk - 1 && tid < 3) {  // fold the reduced metric tail into the epoch totals
      float a = 0.f;
      for (int r = 0; r < xa.world; ++r) a += x_small(xo, ps, r)[SM_MET + tid];
      float* accp = tid == 0 ? &ctrl->acc_loss : (tid == 1 ? &ctrl->acc_correct : &ctrl->acc_count);
      *accp = (tid == 0 ? c.acc_loss : (tid == 1 ? c.acc_correct : c.acc_count)) + a;
    }
  }

  // ---- pending SGD updates ----
  if (eager) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + u * 512;  // 8 consecutive n of row kr
      if (i < n4 / 2) {
        const int e = i * 8, kr = e >> 6, n = e & 63;
        const uint32_t w[4] = {bq[u].x, bq[u].y, bq[u].z, bq[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          w1t[(n + 2 * q) * KP + kr] = (uint16_t)(w[q] & 0xffffu);
          w1t[(n + 2 * q + 1) * KP + kr] = (uint16_t)(w[q] >> 16);
        }
      }
    }
  }
  // deferred W1 update of the slice (registers -> bf16 W1^T tile in LDS; the image group 0
  // block also writes the next fp32 buffer, velocity and bf16 copy)
  auto w1_update = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + u * 512;
      if (!eager && i < n4) {
        float4 wn, vn;
        sgd_or_keep(pend, wv[u].x, gv[u].x, vv[u].x, c, wn.x, vn.x);
        sgd_or_keep(pend, wv[u].y, gv[u].y, vv[u].y, c, wn.y, vn.y);
        sgd_or_keep(pend, wv[u].z, gv[u].z, vv[u].z, c, wn.z, vn.z);
        sgd_or_keep(pend, wv[u].w, gv[u].w, vv[u].w, c, wn.w, vn.w);
        const int e = i * 4, kr = e >> 6, n = e & 63;
        const uint16_t h0 = f2bf(wn.x), h1 = f2bf(wn.y), h2 = f2bf(wn.z), h3 = f2bf(wn.w);
        w1t[(n + 0) * KP + kr] = h0;
        w1t[(n + 1) * KP + kr] = h1;
        w1t[(n + 2) * KP + kr] = h2;
        w1t[(n + 3) * KP + kr] = h3;
        if (owner) {
          Wn4[i] = wn;
          if (mom) Vn4[i] = vn;
          Wb[i] = make_uint2((uint32_t)h0 | ((uint32_t)h1 << 16), (uint32_t)h2 | ((uint32_t)h3 << 16));
        }
      }
    }
  };
  if (!sh) w1_update();
  float cwn = 0.f, cvn = 0.f;
  if (tid < NCONV) {
    sgd_or_keep(pend, cp, from_fix(cq, CINV), cv, c, cwn, cvn);
    cw[tid] = cwn;
    // the conv epilogue's ReLU (fmaxf) and the head's would turn a NaN parameter into 0:
    // a non-finite conv / b1 / W2 / b2 value raises ctrl.bad (loss NaN) here instead
    if (!__builtin_isfinite(cwn)) __hip_atomic_fetch_or(&ctrl->bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (small_on) {
    float wn, vn;
    sgd_or_keep(pend, sp, sg, sv, c, wn, vn);
    P[sic] = wn;
    if (mom) V[sic] = vn;
    if (!__builtin_isfinite(wn)) __hip_atomic_fetch_or(&ctrl->bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the owner writes the next conv buffer and zeroes the hconv parity bwd adds into next
  if (lin == 0 && tid < NCONV) {
    (par ? P : calt)[tid] = cwn;
    if (mom) (par ? V : calt + NCONV)[tid] = cvn;
    hconv[par * NCONV + tid] = 0;
  }
  stamp(sts, st, 1);
  x_store<U8>(xst, xs, lg, nrows);
  lds_barrier();
  stamp(sts, st, 2);

  ConvFrag cf;
  conv_setup(cf, cw, lane);
  stamp(sts, st, 5);
  uint8_t* csl = reinterpret_cast<uint8_t*>(cw + NCONV);  // [IB][K] argmax codes
  conv_pool(cf, xs, p0, np, r0, lg, wave, lane, [&](int bo, int plo, int ch, uint16_t hb, uint8_t cd) {
    as[bo * KP + plo * 32 + ch] = hb;
    csl[bo * K + plo * 32 + ch] = cd;
  });
  stamp(sts, st, 6);
  lds_barrier();
  stamp(sts, st, 3);
  // pooled tile (feature-major [k][b]: bwd's dW1 operand) and argmax codes ([b][k]) for
  // bwd, from LDS as contiguous 8-byte / 4-byte stores instead of scattered 1-2 B stores
  // (IB / 4 = 2^(lg - 2) and K / 4 = 8 np: shifts and a multiply, not divisions)
  for (int i = tid; i < K * (IB / 4); i += 512) {
    const int kk = i >> (lg - 2), bo = 4 * (i & ((1 << (lg - 2)) - 1));
    uint16_t v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = as[(bo + e) * KP + kk];
    uint16_t* dst = pooled + (unsigned)((p0 * NF + kk) * BP + img0 + bo);
    if (img0 + bo + 3 < B) {
      *reinterpret_cast<uint2*>(dst) = make_uint2((uint32_t)v[0] | ((uint32_t)v[1] << 16),
                                                 (uint32_t)v[2] | ((uint32_t)v[3] << 16));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (img0 + bo + e < B) dst[e] = v[e];
    }
  }
  for (int i = tid; i < IB * (K / 4); i += 512) {
    const int i8 = i >> 3, bo = np == 3 ? (int)(((unsigned)i8 * 21846u) >> 16) : i8 >> (np >> 1), w = i - bo * (K / 4);
    if (img0 + bo < B)
      *reinterpret_cast<uint32_t*>(code + (unsigned)((img0 + bo) * FEAT + p0 * NF + 4 * w)) =
          reinterpret_cast<const uint32_t*>(csl + bo * K)[w];
  }
  stamp(sts, st, 7);
  if (sh) {
    // sharded: the slice's reduced dW1 arrives as 4 units (2 halves each) from their owners,
    // pushed at the end of every owner's bwd -- waited for only now, after the conv
    if (pend) {
      // units of the bwd slices covering this slice's rows, 2 halves each
      const int sb0 = p0 / xa.ppb, nunits = 4 * ((p1 - 1) / xa.ppb - sb0 + 1), NUb = 4 * ((NPOS + xa.ppb - 1) / xa.ppb);
      if (tid < 2 * nunits) x_wait(xa, x_gflag(xa.out[xa.rank], NUb, 4 * sb0 + (tid >> 1), tid & 1), xe, XW_UNIT);
      __syncthreads();
      if (xa.gbf16) {
        const uint2* R2 = reinterpret_cast<const uint2*>(xa.out[xa.rank] + kXG16) + p0 * 32 * HID / 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) gv[u] = unpack_bf16x4(R2[min(tid + u * 512, n4 - 1)]);
      } else {
        const float4* R4 = reinterpret_cast<const float4*>(xa.out[xa.rank] + kXGred + OFF_W1 + p0 * 32 * HID);
#pragma unroll
        for (int u = 0; u < 4; ++u) gv[u] = R4[min(tid + u * 512, n4 - 1)];
      }
    }
    w1_update();
    lds_barrier();
  }
  // ---- dense-1 partial of the slice: part[row][n] = sum_k pooled[row][k] W1[k][n] ----
  const int ko = 8 * (lane >> 4);
  const int ntiles = (IB >> 4) * 4;
  float* part = xs;  // [IB][64] (the staged rows are dead)
  for (int t = wave; t < ntiles; t += 8) {
    const int mt = t >> 2, nt = t & 3;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int ar = 16 * mt + (lane & 15), bn = 16 * nt + (lane & 15);
    for (int ks = 0; ks < np; ++ks) {
      const bf16x8 a = ld_frag(as + ar * KP + ks * 32 + ko);
      const bf16x8 bb = ld_frag(w1t + bn * KP + ks * 32 + ko);
      acc = mfma16(a, bb, acc);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) part[(16 * mt + 4 * (lane >> 4) + j) * HID + bn] = acc[j];
  }
  stamp(sts, st, 8);
  lds_barrier();
  stamp(sts, st, 9);
  // one wave instruction = one 512-B row of 64 int64 adds
  long long* hp = hacc + (long)par * B * HACC_PITCH;
  for (int r = wave; r < (hprobe == 1 ? 0 : hprobe == 2 ? IB / 2 : IB); r += 8)
    if (img0 + r < B) atomic_add_i64(hp + (unsigned)((img0 + r) * HACC_PITCH + lane), to_fix(part[r * HID + lane], HSCALE, &ctrl->bad));
  if (xcp) reinterpret_cast<uint4*>(xcur)[xcu] = xcv;
  if (xcur != nullptr && lin == 0 && tid < B) ycur[tid] = ycv;
  stamp(sts, st, 4);
  if (st != nullptr && tid == 0 && lin < 256)
    for (int i = 0; i < 10; ++i) st[lin * 16 + i] = sts.t[i];
}

// =================================================================================
// sharded exchange, end of bwd (every wave of every block calls it)
// =================================================================================
//  1. the partial pushes of this wave have drained (nothing else was issued since, so the
//     wait costs nothing): raise the partial flag at the owner
//  2. arrival ticket: the last block of the launch reads this rank's conv-gradient int64
//     sums, b1 / W2 / b2 gradient and metric tail (all complete: every block drained its
//     stores before its ticket) and publishes them as this rank's small message on every rank
//  3. owner waves: wait for the other ranks' halves of their unit, sum the world partials
//     in rank order (own from registers), push the reduced unit to every rank's gradient
//     staging, raise the unit flag there
__device__ __forceinline__ void exchange_tail(const XArgs& xa, Ctrl* ctrl, const float* G, const long long* hconv_p,
                                              const f32x4* accw, unsigned xe, int s, int NS, int np, int p0, int dn,
                                              int dm0, int lane, int tid, bool xown, int xo, int xu) {
  __shared__ int last_flag;
  const int NU = 4 * NS, W = xa.world, ps = xe & 1;
  damd_publish_drain();
  DAMD_PUBLISH_WAVE();
  if (!xown && lane == 0) x_signal(x_pflag(xa.out[xo], xu, xa.rank * 2 + dm0), xe);
  // 2. ticket (counts forever: NS arrivals per step)
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int t = __hip_atomic_fetch_add(&ctrl->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t % NS) == NS - 1;
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    last_flag = last;
  }
  __syncthreads();
  if (last_flag) {
    const float* hc = reinterpret_cast<const float*>(hconv_p);
    for (int i = tid; i < SM_MET + 3; i += 512) {
      const float v = i < SM_GRAD ? hc[i] : (i < SM_MET ? G[OFF_B1 + i - SM_GRAD] : G[OFF_LOSS + i - SM_MET]);
      for (int r = 0; r < W; ++r) x_small(xa.out[r], ps, xa.rank)[i] = v;
    }
    // publish: EVERY wave drains its own small-message stores before the barrier (a
    // workgroup barrier does not wait for outstanding vector-memory stores), then the
    // flag -- the order scripts/check_publish_isa.py verifies on the gfx950 code object
    damd_publish_drain();
    __syncthreads();
    DAMD_PUBLISH_WG();
    if (tid < W) x_signal(x_sflag(xa.out[tid], NU, ps, xa.rank), xe);
  }
  // 3. owners
  if (xown) {
    if (lane < W && lane != xa.rank) x_wait(xa, x_pflag(xa.out[xa.rank], xu, lane * 2 + dm0), xe, XW_PART);
    asm volatile("" ::: "memory");
    f32x4 g[MAXPP];
#pragma unroll
    for (int i = 0; i < MAXPP; ++i) g[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < W; ++r) {
      const float* slot = xa.in[xa.rank] + ((long)r * NU + xu) * kXPSlot;
#pragma unroll
      for (int i = 0; i < MAXPP; ++i) {
        if (i >= np) break;
        float4 v;
        if (xa.gbf16)  // own partial rounded like the others': the sum is symmetric in the ranks
          v = unpack_bf16x4(r == xa.rank ? pack_bf16x4(accw[i])
                                         : reinterpret_cast<const uint2*>(slot)[(dm0 * MAXPP + i) * 64 + lane]);
        else
          v = r == xa.rank ? make_float4(accw[i][0], accw[i][1], accw[i][2], accw[i][3])
                           : reinterpret_cast<const float4*>(slot)[(dm0 * MAXPP + i) * 64 + lane];
        g[i][0] += v.x;
        g[i][1] += v.y;
        g[i][2] += v.z;
        g[i][3] += v.w;
      }
    }
    const int lr16 = lane & 15;
    if (xa.gbf16) {
      // bf16 reduced unit, row-major [k][n]: column pairs packed into 32-bit words (the even
      // lane of each pair stores both), i.e. 16 lanes write one 32-byte row piece
      for (int r = 0; r < W; ++r) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(xa.out[r] + kXG16) + ((long)p0 * 32 * HID + 16 * dn + lr16) / 2;
#pragma unroll
        for (int i = 0; i < MAXPP; ++i) {
          if (i >= np) break;
          const int mt = dm0 + 2 * i;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t h = f2bf(g[i][j]);
            const uint32_t o = (uint32_t)__shfl_xor((int)h, 1);
            if (!(lr16 & 1)) dst[(16 * mt + 4 * (lane >> 4) + j) * (HID / 2)] = h | (o << 16);
          }
        }
      }
    } else {
      for (int r = 0; r < W; ++r) {
        float* dst = xa.out[r] + kXGred + OFF_W1 + (long)p0 * 32 * HID + 16 * dn + lr16;
#pragma unroll
        for (int i = 0; i < MAXPP; ++i) {
          if (i >= np) break;
          const int mt = dm0 + 2 * i;
#pragma unroll
          for (int j = 0; j < 4; ++j) dst[(16 * mt + 4 * (lane >> 4) + j) * HID] = g[i][j];
        }
      }
    }
    damd_publish_drain();
    DAMD_PUBLISH_WAVE();
    if (lane < W) x_signal(x_gflag(xa.out[lane], NU, xu, dm0), xe);
  }
}

// =================================================================================
// bwd: grid NS slices
// =================================================================================
// aux element e (parameter order at G + OFF_B1): [0,64) db1, [64,704) dW2
// (k = (e-64)/10, c = (e-64)%10), [704,714) db2, then 714 loss, 715 correct, 716 count.
template <bool U8, bool ONE>  // ONE: B <= 64, a single chunk (no loop-carried prefetch registers)
// (the first 16 argument dwords arrive preloaded in SGPRs: they are what the prologue's first
// loads address -- the dense-1 sums by the known parity, this step's staged labels / rows, b1 /
// W2 / b2, the bf16 W1 slice, the pooled tile and codes; later arguments come from the
// kernarg segment, a scalar load's latency behind)
__global__ __launch_bounds__(512) void bwd(long long* __restrict__ hacc, const int* __restrict__ ycur,
                                           const void* __restrict__ xcur, int phint, int bpp, const float* P,
                                           const uint16_t* w1bf, const uint16_t* __restrict__ pooled,
                                           const uint8_t* __restrict__ code, Ctrl* __restrict__ ctrl,
                                           const void* __restrict__ X, const int* __restrict__ labels,
                                           float* __restrict__ G, long long* __restrict__ hconv,
                                           int eager, float* Pw, float* Vw, uint16_t* w1bf_out,
                                           unsigned long long* st, const float* __restrict__ Gr, const XArgs xa,
                                           void* __restrict__ xnext, long long* __restrict__ xtag, int auxm) {
  const int B = bpp & 0xffff, PP = bpp >> 16;  // (packed: both preloaded)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bool sh = xa.world > 1;  // sharded multi-rank step (see the exchange at the end)
  constexpr int cprobe = DAMD_PROBE_HCONV;  // 0 in every product build (see the top of the file)
  Stamps sts;
  stamp(sts, st, 0);
  const int s = blockIdx.x, tid = threadIdx.x, NS = gridDim.x;
  const int p0 = s * PP, p1 = min(NPOS, p0 + PP), np = p1 - p0, K = np * 32;
  const int KD = PP * 32 + 4;   // dps pitch (f32)
  const int KC = PP * 32;       // code pitch (bytes)
  const int RB = max(CH * KD * 4, HEAD_BYTES);
  float* xs = reinterpret_cast<float*>(smem);                              // [CH][XR][28]
  float* dps = reinterpret_cast<float*>(smem + XS_BYTES);                  // [CH][KD] (after the head)
  uint16_t* pt = reinterpret_cast<uint16_t*>(smem + XS_BYTES + RB);        // [PP*32][HP]
  uint16_t* dht = pt + PP * 32 * HP;                                       // [2][HID][HP] dh^T hi, lo
  uint16_t* dhs = dht + 2 * HID * HP;                                      // [2][CH][HP]  dh hi, lo
  uint16_t* w1s = dhs + 2 * CH * HP;                                       // [PP*32][HP]
  uint8_t* cs = reinterpret_cast<uint8_t*>(w1s + PP * 32 * HP);            // [CH][KC] argmax codes
  float* red = reinterpret_cast<float*>(pt);  // [16][320] reduction scratch, after the MFMAs
  // head scratch (aliases dps: used before the dP MFMA of each chunk)
  float* hs = dps;                 // [CH][HPITCH] h = relu(dense-1)
  float* spl = hs + CH * HPITCH;   // [716] b1[64] W2[64][10] b2[10]
  float* zs = spl + 716;           // [CH][ZP] logits, then dz
  float* rl = zs + CH * ZP;        // [CH] per-row loss
  float* rc = rl + CH;             // [CH] per-row correct
  float* db1p = rc + CH;           // [16][64] db1 partials
  int* ylds = reinterpret_cast<int*>(db1p + 16 * HID);  // [CH] label of the row, -1 if invalid
  const int r0 = 2 * (p0 / PO);
  const int nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  const int wave = tid >> 6, lane = tid & 63;
  const int ko = 8 * (lane >> 4), lr16 = lane & 15;

  // ---- this block's aux elements ----
  // (auxm, from the host: chunk_aux | log2(threads per element) << 16 -- the divisions
  // that derive them from the grid cost ~40 VALU of the prologue on the device)
  const int chunk_aux = auxm & 0xffff, ltpe = auxm >> 16, tpe = 1 << ltpe;
  const int ae_local = tid >> ltpe, aq = tid & (tpe - 1);
  const int ae = s * chunk_aux + ae_local;
  const bool aux_on = ae_local < chunk_aux && ae < NAUX2;
  const int aec = min(ae, NAUX2 - 1);
  float arsum = 0.f;

  // ---- prologue: first the loads whose addresses do not depend on the ctrl block (the
  // previous metric, b1/W2/b2, the bf16 W1 slice, chunk 0's pooled tile and argmax codes),
  // kept ahead of the ctrl load by a scheduling barrier (as in fwd) ----
  // previous step's reduced metric (sharded: fwd folds it from the small messages)
  const float ag_old = sh ? 0.f : Gr[OFF_LOSS + max(0, min(aec - NSMALL, 2))];
  // small parameters (b1/W2/b2, updated by fwd): 2 per thread, re-staged every chunk
  const float spv0 = P[OFF_B1 + tid];
  float spv1 = 0.f;
  if (tid + 512 < NSMALL) spv1 = P[OFF_B1 + tid + 512];
  uint4 hq0, hq1, hq2, hq3;  // hacc row (tid >> 3), columns 8 (tid & 7) .. + 8
  // known parity (single chunk): the head's first operand -- this step's dense-1 sums --
  // right behind b1 / W2 / b2, before the ctrl block
  const bool hq_early = ONE && phint >= 0;
  auto load_hq = [&](int chunk, int p) __attribute__((always_inline)) {
    const int r = tid >> 3, q = tid & 7;
    const int row = min(chunk * CH + r, B - 1);
    const uint4* hp = reinterpret_cast<const uint4*>(hacc + (unsigned)((p * B + row) * HACC_PITCH + q * 8));
    hq0 = hp[0];
    hq1 = hp[1];
    hq2 = hp[2];
    hq3 = hp[3];
  };
  if (hq_early) load_hq(0, phint);
  const int n8 = K * HID / 8;
  uint4 wv0, wv1;
  // (only in-range units are loaded: clamped duplicates cost load bandwidth -- at PP = 2 the
  // whole second unit is out of range)
  // (conditional loads, not selects between pointers: see fwd's bq)
  wv0 = wv1 = make_uint4(0u, 0u, 0u, 0u);
  if (tid < n8) wv0 = reinterpret_cast<const uint4*>(w1bf + p0 * 32 * HID)[tid];
  if (tid + 512 < n8) wv1 = reinterpret_cast<const uint4*>(w1bf + p0 * 32 * HID)[tid + 512];
  // the body -- pooled tile, argmax codes, input rows, read only by the MFMAs and the conv
  // gradient -- is staged by NB threads with two slots each: all 512 when chunked; in the
  // single-chunk step only waves 4-7 (slots bt and bt + 256), which have no logits to
  // compute and store it while waves 0-3 run the logits / softmax (staged by waves 0-3 too,
  // it sat on the head's critical path)
  constexpr int NB = ONE ? 256 : 512;
  const int bt = ONE ? tid - 256 : tid;  // (< 0: no body slots)
  const bool bw = !ONE || bt >= 0;
  XStage<U8> xst, xst1;      // input rows: slot bt, and (single chunk) bt + 256
  uint4 pv0, pv1, pv2, pv3;  // pooled tile units bt + j NB (K * 8 <= 1024 units)
  uint4 cv, cv1;             // argmax codes, units bt (+ NB), zeroed at the LDS store unless cok
  bool cok = false, cok1 = false;
  int ylab = 0;
  bool yval = false;
  const int BP = (B + CH - 1) / CH * CH;
  const int kc = K / 16;  // = 2 np, np in 1..MAXPP
  // i / kc for i < 512 without a division sequence: (i / 2) / np, np = 3 by a multiply
  auto div_kc = [&](int i) __attribute__((always_inline)) {
    return np == 3 ? (int)(((unsigned)(i >> 1) * 21846u) >> 16) : (i >> 1) >> (np >> 1);
  };
  static_assert(MAXPP == 4, "div_kc covers np = 1..4");
  // (32-bit element offsets: the pooled tile is FEAT x BP bf16, far below 2^31; only
  // in-range units load -- conditional loads, not pointer selects, see fwd's bq)
  auto load_pv = [&](uint4& v, int i, int chunk) __attribute__((always_inline)) {
    v = make_uint4(0u, 0u, 0u, 0u);
    if (i < K * 8) v = *reinterpret_cast<const uint4*>(pooled + (__umul24(p0 * NF + (i >> 3), BP) + chunk * CH + (i & 7) * 8));
  };
  auto load_cv = [&](uint4& v, bool& ok, int i, int chunk) __attribute__((always_inline)) {
    const int bb = div_kc(i), q = i - bb * kc, lb = chunk * CH + bb;
    ok = i < CH * kc && lb < B;
    v = make_uint4(0u, 0u, 0u, 0u);
    if (i < CH * kc) v = *reinterpret_cast<const uint4*>(code + (__umul24(min(lb, B - 1), FEAT) + p0 * NF + q * 16));
  };
  auto load_indep = [&](int chunk) __attribute__((always_inline)) {
    if (bw) {
      load_pv(pv0, bt, chunk);
      load_pv(pv1, bt + NB, chunk);
      if (ONE) {
        load_pv(pv2, bt + 2 * NB, chunk);
        load_pv(pv3, bt + 3 * NB, chunk);
      }
      load_cv(cv, cok, bt, chunk);
      if (ONE) load_cv(cv1, cok1, bt + NB, chunk);
    }
    if (ycur != nullptr) {  // labels and rows as this step's fwd read them: no cursor needed
      const int b = chunk * CH + min(tid, CH - 1);
      ylab = ycur[min(b, B - 1)];
      yval = tid < CH && b < B && ylab >= 0;
      if (bw) {
        x_load<U8>(xst, xcur, chunk * CH, B, B - chunk * CH, LG_CH, r0, nrows, bt);
        if (ONE) x_load<U8>(xst1, xcur, chunk * CH, B, B - chunk * CH, LG_CH, r0, nrows, bt + NB);
      }
    }
  };
  load_indep(0);
  __builtin_amdgcn_sched_barrier(0);

  const Ctrl c = *ctrl;
  const int cur = c.cur2, par = phint >= 0 ? phint : c.par2;
  if (phint >= 0 && phint != c.par2 && s == 0 && tid == 0)
    __hip_atomic_fetch_or(&ctrl->bad, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned xe = (unsigned)c.xcnt2 + 1u;  // sharded: this step's exchange epoch
  if (s == 0 && tid == 0) {
    ctrl->cursor = next_cursor(c, cur);
    ctrl->iterations = c.iterations + 1;
    ctrl->wpar = c.wpar ^ 1;  // fwd of this step wrote the next W1 buffer
    ctrl->pending = 1;
    if (sh) ctrl->xcnt = (int)xe;
  }
  const long gstart = (long)cur * c.global_batch;
  const long row_base = gstart + c.row0;
  const int gcount = (int)min((long)c.global_batch, (long)c.nsamples - gstart);
  const float inv = gcount > 0 ? 1.f / (float)gcount : 0.f;
  // next-batch prefetch for the next fwd: this block's share of the next step's rows as
  // 16-byte units (stored at the end; the loads travel meanwhile)
  const int ncur = next_cursor(c, cur);
  constexpr int UPI = U8 ? NPIX / 16 : NPIX / 4;  // 16-byte units per image
  const int xpu = s * 512 + tid;
  const bool xpf = ONE && xnext != nullptr && xpu < B * UPI;
  uint4 xnv = make_uint4(0u, 0u, 0u, 0u);

  // then the ctrl-dependent ones: the dense-1 sums by parity (unless known), the labels and
  // the batch rows (unless the fwd staged them in ycur / xcur)
  auto load_dep = [&](int chunk) __attribute__((always_inline)) {
    if (!hq_early || chunk > 0) load_hq(chunk, par);
    if (ycur == nullptr) {
      {
        const int b = chunk * CH + min(tid, CH - 1);
        const long g = row_base + b;
        yval = tid < CH && b < B && g < c.nsamples;
        ylab = labels[max(0L, min(g, (long)c.nsamples - 1))];
      }
      if (bw) {
        x_load<U8>(xst, X, row_base + chunk * CH, c.nsamples, B - chunk * CH, LG_CH, r0, nrows, bt);
        if (ONE) x_load<U8>(xst1, X, row_base + chunk * CH, c.nsamples, B - chunk * CH, LG_CH, r0, nrows, bt + NB);
      }
    }
  };
  auto load_chunk = [&](int chunk) __attribute__((always_inline)) {
    load_indep(chunk);
    load_dep(chunk);
  };
  // what the head needs (b1 / W2 / b2, labels) and what only the MFMAs / conv gradient
  // need (pooled tile, argmax codes, input rows): the single-chunk backward stores the
  // latter while waves 0-3 run the logits / softmax, so the head does not wait for the
  // input rows (the largest, last-issued loads)
  auto store_head = [&]() __attribute__((always_inline)) {
    spl[tid] = spv0;
    if (tid + 512 < NSMALL) spl[tid + 512] = spv1;
    if (tid < CH) ylds[tid] = yval ? ylab : -1;
  };
  auto store_pv = [&](const uint4& v, int i) __attribute__((always_inline)) {
    if (i < K * 8) *reinterpret_cast<uint4*>(pt + (i >> 3) * HP + (i & 7) * 8) = v;
  };
  auto store_cv = [&](const uint4& v, bool ok, int i) __attribute__((always_inline)) {
    if (i < CH * kc) {
      const int bb = div_kc(i), q = i - bb * kc;
      *reinterpret_cast<uint4*>(cs + bb * KC + q * 16) = ok ? v : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store_body = [&]() __attribute__((always_inline)) {
    if (!bw) return;
    store_pv(pv0, bt);
    store_pv(pv1, bt + NB);
    if (ONE) {
      store_pv(pv2, bt + 2 * NB);
      store_pv(pv3, bt + 3 * NB);
    }
    store_cv(cv, cok, bt);
    if (ONE) store_cv(cv1, cok1, bt + NB);
    x_store<U8>(xst, xs, LG_CH, nrows);
    if (ONE) x_store<U8>(xst1, xs, LG_CH, nrows);
  };
  auto store_chunk = [&](int chunk) __attribute__((always_inline)) {
    store_body();
    store_head();
  };
  load_dep(0);
  // the next step's rows for its fwd (issued after this step's own loads: in-order vmcnt)
  if (xpf) {
    const int b = xpu / UPI, q = xpu - b * UPI;
    const int g = (int)((long)ncur * c.global_batch + c.row0) + b;  // (dataset < 2^31 bytes: 32-bit)
    if (g < c.nsamples)
      xnv = reinterpret_cast<const uint4*>(static_cast<const char*>(X) + __umul24((unsigned)g, U8 ? NPIX : 4 * NPIX))[q];
  }
  // (w1s is read only by the dP MFMAs, several barriers later)
  if (tid < n8) *reinterpret_cast<uint4*>(w1s + (tid >> 3) * HP + (tid & 7) * 8) = wv0;
  if (tid + 512 < n8) *reinterpret_cast<uint4*>(w1s + ((tid + 512) >> 3) * HP + (tid & 7) * 8) = wv1;

  const int dn = wave & 3, dm0 = wave >> 2;
  const bool mom = c.momentum != 0.f;
  float ew[ONE ? MAXPP : 1][4], ev[ONE ? MAXPP : 1][4];  // eager (single chunk only)
  f32x4 accw[MAXPP];
#pragma unroll
  for (int i = 0; i < MAXPP; ++i) accw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // ---- sharded exchange: this wave's dW1 tiles form half of unit u = 4 s + dn (rows of
  // tiles dm0 + 2 i, 16 columns), owned by rank u % world ----
  const int NU = 4 * NS, xu = 4 * s + dn;
  const int xo = !sh ? 0 : (xa.world & (xa.world - 1)) == 0 ? xu & (xa.world - 1) : xu % xa.world;
  const bool xown = sh && xo == xa.rank;
  auto push_partials = [&]() __attribute__((always_inline)) {
    if (!sh || xown) return;
    float* slot = xa.in[xo] + ((long)xa.rank * NU + xu) * kXPSlot;
    if (xa.gbf16) {  // bf16 partials: half the bytes (the owner accumulates in fp32)
      uint2* dst = reinterpret_cast<uint2*>(slot) + dm0 * MAXPP * 64 + lane;
#pragma unroll
      for (int i = 0; i < MAXPP; ++i)
        if (i < np) dst[i * 64] = pack_bf16x4(accw[i]);
    } else {
      float4* dst = reinterpret_cast<float4*>(slot) + dm0 * MAXPP * 64 + lane;
#pragma unroll
      for (int i = 0; i < MAXPP; ++i)
        if (i < np) dst[i * 64] = make_float4(accw[i][0], accw[i][1], accw[i][2], accw[i][3]);
    }
  };
  const int ch = tid & 31, grp = tid >> 5;
  float gw[9], gb = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) gw[t] = 0.f;
  const int nchunks = ONE ? 1 : (B + CH - 1) / CH;

  for (int chunk = 0; chunk < nchunks; ++chunk) {
    if (chunk) {
      lds_barrier();
      load_chunk(chunk);
    }
    if (ONE) store_head();
    else store_chunk(chunk);
    lds_barrier();
    stamp(sts, st, 1);
    // eager: the slice's fp32 masters / velocities for the update right after the dW1
    // MFMAs, issued once the staged operands have landed (in flight through the head)
    if (ONE && eager) {
#pragma unroll
      for (int i = 0; i < MAXPP; ++i) {
        if (i >= np) break;
        const int mt = dm0 + 2 * i;
        // (one address per tile, the 4 rows at immediate offsets)
        const unsigned e0 = OFF_W1 + (unsigned)((p0 * 32 + 16 * mt + 4 * (lane >> 4)) * HID + 16 * dn + lr16);
        const float* pw = Pw + e0;
        const float* vw = Vw + e0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ew[i][j] = pw[j * HID];
          ev[i][j] = mom ? vw[j * HID] : 0.f;
        }
      }
    }
    // ---- head (every block, redundantly): h = relu(hacc / 2^32 + b1) ----
    {
      const int r = tid >> 3, q = tid & 7;
      const bool rv = chunk * CH + r < B;
      const uint4 hq[4] = {hq0, hq1, hq2, hq3};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long a = (long long)(((unsigned long long)hq[u].y << 32) | hq[u].x);
        const long long b = (long long)(((unsigned long long)hq[u].w << 32) | hq[u].z);
        const int n = q * 8 + 2 * u;
        hs[r * HPITCH + n] = rv ? fmaxf(from_fix(a, HINV) + spl[n], 0.f) : 0.f;
        hs[r * HPITCH + n + 1] = rv ? fmaxf(from_fix(b, HINV) + spl[n + 1], 0.f) : 0.f;
      }
    }
    lds_barrier();
    stamp(sts, st, 6);
    if (ONE && wave >= 4) {  // (waves 4-7 stage the whole body: see NB above)
      store_body();
      stamp(sts, st, 12);
    }
    // logits on f32 MFMA (wave mt: rows 16 mt .. 16 mt + 15, 16 columns, 10 used), then
    // softmax-xent / accuracy / dz over each row's 16 lanes (DPP row reductions); the four
    // rows j of a lane are independent chains, interleaved
    if (wave < 4) {
      const int mt = wave, lr = lane & 15, kq = lane >> 4;
      float av[HID / 4], bv[HID / 4];  // all operands first: one LDS wait, then 16 MFMAs
#pragma unroll
      for (int ks = 0; ks < HID / 4; ++ks) {
        const int k = 4 * ks + kq;
        av[ks] = hs[(16 * mt + lr) * HPITCH + k];
        bv[ks] = spl[HID + k * NCLS + min(lr, NCLS - 1)];
      }
      // the labels of this lane's 4 rows, read with the operands (read after the softmax, they
      // were 4 serial LDS round trips on the critical path)
      int yv4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) yv4[j] = ylds[16 * mt + 4 * kq + j];
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (ONE) stamp(sts, st, 9);  // (sub-phase stamps, single chunk: wave 0's view)
#pragma unroll
      for (int ks = 0; ks < HID / 4; ++ks) acc = mfma4(av[ks], lr < NCLS ? bv[ks] : 0.f, acc);
      const float b2v = lr < NCLS ? spl[HID + HID * NCLS + lr] : 0.f;
      float v[4], m[4], e[4], lse[4];
      int am[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = lr < NCLS ? acc[j] + b2v : -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = row16_max(v[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = lr < NCLS ? __expf(v[j] - m[j]) : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] = row16_sum(e[j]);
      if (ONE) stamp(sts, st, 10);
      // log-sum-exp: the sum is in [1, 10], so the hardware log2 (v_log_f32) is accurate here;
      // __logf's denormal-safe expansion was ~15 instructions per row on the critical path
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lse[j] = m[j] + __builtin_amdgcn_logf(e[j]) * 0.693147180559945f;
        am[j] = row16_min(v[j] == m[j] ? lr : 16);
      }
      if (ONE) stamp(sts, st, 11);
      // dz for all 16 lanes of a row (lanes >= NCLS: v = -inf, so 0 -- the padding of the
      // zs row), no per-store exec masks; the label's lane writes the row's loss and hit
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * mt + 4 * kq + j;
        const int yv = yv4[j];
        const bool valid = yv >= 0;
        const int y = valid ? yv : 0;
        zs[r * ZP + lr] = valid ? (__expf(v[j] - lse[j]) - (lr == y ? 1.f : 0.f)) * inv : 0.f;
        if (lr == y) {
          rl[r] = valid ? (lse[j] - v[j]) : 0.f;
          rc[r] = (valid && am[j] == y) ? 1.f : 0.f;
        }
      }
    }
    if (ONE && wave < 4) stamp(sts, st, 12);
    lds_barrier();
    stamp(sts, st, 7);
    // dh = (dz W2^T) * [h > 0] on f32 MFMA: 16 tiles of 16x16, two per wave, K = 10 (three
    // k-steps of 4, zero-padded); a lane's 4 outputs are 4 consecutive rows of one column,
    // so dh^T is stored 8 bytes at a time.
    // Every LDS operand of both tiles first (dz, W2, the ReLU mask of h): one LDS wait
    // instead of three per tile -- hipcc cannot move reads above the tile's dh stores itself
    float za[2][3], wb[2][3], hm[2][4];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const int t = wave + 8 * ti, mt = t >> 2, nt = t & 3, lr = lane & 15, kq = lane >> 4;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int k = 4 * ks + kq;
        za[ti][ks] = k < NCLS ? zs[(16 * mt + lr) * ZP + k] : 0.f;
        wb[ti][ks] = k < NCLS ? spl[HID + (16 * nt + lr) * NCLS + k] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) hm[ti][j] = hs[(16 * mt + 4 * kq + j) * HPITCH + 16 * nt + lr];
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const int t = wave + 8 * ti, mt = t >> 2, nt = t & 3, lr = lane & 15, kq = lane >> 4;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) acc = mfma4(za[ti][ks], wb[ti][ks], acc);
      const int n = 16 * nt + lr, rb = 16 * mt + 4 * kq;
      uint16_t hi[4], lo[4];
      float dsum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = hm[ti][j] > 0.f ? acc[j] : 0.f;
        dsum += d;
        hi[j] = f2bf(d);
        lo[j] = bf16_lo(d, hi[j]);
        dhs[(rb + j) * HP + n] = hi[j];
        dhs[CH * HP + (rb + j) * HP + n] = lo[j];
      }
      *reinterpret_cast<uint2*>(dht + n * HP + rb) =
          make_uint2((uint32_t)hi[0] | ((uint32_t)hi[1] << 16), (uint32_t)hi[2] | ((uint32_t)hi[3] << 16));
      *reinterpret_cast<uint2*>(dht + HID * HP + n * HP + rb) =
          make_uint2((uint32_t)lo[0] | ((uint32_t)lo[1] << 16), (uint32_t)lo[2] | ((uint32_t)lo[3] << 16));
      db1p[(4 * mt + kq) * HID + n] = dsum;  // [16][64]: partial over rows rb .. rb + 3
    }
    lds_barrier();
    stamp(sts, st, 8);
    // this block's aux elements over the chunk's rows (fixed order: deterministic)
    if (aux_on) {
      // element order = parameter order of b1[64], W2[64][10], b2[10] (G + OFF_B1)
      float a = 0.f;
      if (aec < HID) {
        if (aq == 0)
#pragma unroll
          for (int q = 0; q < 16; ++q) a += db1p[q * HID + aec];
      } else if (aec < HID + HID * NCLS) {
        const int kk = (aec - HID) / NCLS, cc = aec - HID - kk * NCLS;
        for (int r = aq; r < CH; r += tpe) a = fmaf(hs[r * HPITCH + kk], zs[r * ZP + cc], a);
      } else if (aec < NSMALL) {
        const int cc = aec - HID - HID * NCLS;
        for (int r = aq; r < CH; r += tpe) a += zs[r * ZP + cc];
      } else if (aec < NSMALL + 2) {
        const float* src = aec == NSMALL ? rl : rc;
        for (int r = aq; r < CH; r += tpe) a += src[r];
      }
      arsum += a;
    }
    lds_barrier();  // the head scratch (dps) is overwritten by dP below
    stamp(sts, st, 2);
    // dW1[k][n] += sum_b P[b][k] (dh_hi + dh_lo)[b][n]
#pragma unroll
    for (int i = 0; i < MAXPP; ++i) {
      if (i >= np) break;
      const int mt = dm0 + 2 * i;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 a = ld_frag(pt + (16 * mt + lr16) * HP + kk * 32 + ko);
        const bf16x8 bh = ld_frag(dht + (16 * dn + lr16) * HP + kk * 32 + ko);
        const bf16x8 bl = ld_frag(dht + HID * HP + (16 * dn + lr16) * HP + kk * 32 + ko);
        accw[i] = mfma16(a, bh, accw[i]);
        accw[i] = mfma16(a, bl, accw[i]);
      }
    }
    // sharded: a unit owned by another rank leaves now (data only; its flag is raised once
    // the stores have drained, after the conv gradient) and travels during dP / conv grad
    if (ONE && sh) push_partials();
    // eager: the slice's SGD update now, its stores overlapping dP and the conv gradient
    // (fp32 master and velocity in place, bf16 copy for the next fwd; this block read its
    // old bf16 slice in the prologue and nobody else touches the slice in this launch)
    if (ONE && eager) {
#pragma unroll
      for (int i = 0; i < MAXPP; ++i) {
        if (i >= np) break;
        const int mt = dm0 + 2 * i;
        const unsigned e0 = OFF_W1 + (unsigned)((p0 * 32 + 16 * mt + 4 * (lane >> 4)) * HID + 16 * dn + lr16);
        float* pw = Pw + e0;
        float* vw = Vw + e0;
        uint16_t* bw = w1bf_out + (e0 - OFF_W1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float wn, vn;
          sgd_update(ew[i][j], accw[i][j], ev[i][j], c.lr, c.momentum, c.nesterov, wn, vn);
          pw[j * HID] = wn;
          if (mom) vw[j * HID] = vn;
          bw[j * HID] = f2bf(wn);
        }
      }
    }
    // dP[b][k] = sum_n (dh_hi + dh_lo)[b][n] W1[k][n]
    {
      const int pm = wave & 3;
#pragma unroll
      for (int i = 0; i < MAXPP; ++i) {
        if (i >= np) break;
        const int nt = (wave >> 2) + 2 * i;
        f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 ah = ld_frag(dhs + (16 * pm + lr16) * HP + kk * 32 + ko);
          const bf16x8 al = ld_frag(dhs + CH * HP + (16 * pm + lr16) * HP + kk * 32 + ko);
          const bf16x8 bb = ld_frag(w1s + (16 * nt + lr16) * HP + kk * 32 + ko);
          a4 = mfma16(ah, bb, a4);
          a4 = mfma16(al, bb, a4);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) dps[(16 * pm + 4 * (lane >> 4) + j) * KD + 16 * nt + lr16] = a4[j];
      }
    }
    lds_barrier();
    stamp(sts, st, 3);
    // MaxPool + ReLU backward fused into the conv weight-gradient accumulation
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int bb = grp * 4 + ii;
      for (int pl = 0; pl < np; ++pl) {
        const int cd = cs[bb * KC + pl * 32 + ch];
        const int pos = p0 + pl, py = pos / PO, px = pos - py * PO;
        const float dv0 = dps[bb * KD + pl * 32 + ch];
        const float d = (cd & 4) ? dv0 : 0.f;
        const int y0 = 2 * py + ((cd >> 1) & 1) - r0, x0 = 2 * px + (cd & 1);
        const float* xp = xs + (bb * XR + y0) * IMG + x0;
        float xv[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) xv[t] = xp[(t / 3) * IMG + (t % 3)];
#pragma unroll
        for (int t = 0; t < 9; ++t) gw[t] = fmaf(d, xv[t], gw[t]);
        gb += d;
      }
    }
  }
  stamp(sts, st, 4);
  if (!ONE && sh) push_partials();
  // ---- dW1 straight into the flat gradient buffer (this block owns these rows), unless
  // the update was applied eagerly above or the exchange carries it ----
#pragma unroll
  for (int i = 0; i < MAXPP; ++i) {
    if (i >= np || (ONE && eager) || sh) break;
    const int mt = dm0 + 2 * i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * mt + 4 * (lane >> 4) + j;
      G[OFF_W1 + (unsigned)((p0 * 32 + k) * HID + 16 * dn + lr16)] = accw[i][j];
    }
  }
  lds_barrier();  // pt/dht region becomes `red`, dps becomes `ared`
#pragma unroll
  for (int t = 0; t < 9; ++t) red[grp * NCONV + t * NF + ch] = gw[t];
  red[grp * NCONV + OFF_BC + ch] = gb;
  float* ared = dps;
  ared[tid] = arsum;
  lds_barrier();
  // this slice's conv-gradient partial, fixed order over the 16 thread groups, then a
  // 64-bit fixed-point atomic add (order-independent sum over the slices)
  for (int i = tid; i < (cprobe ? 0 : NCONV); i += 512) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) a += red[r * NCONV + i];
    atomic_add_i64(hconv + par * NCONV + i, to_fix(a, CSCALE, &ctrl->bad));
  }
  // ---- aux: new b1/W2/b2 gradient, metric tail ----
  if (aux_on && aq == 0) {
    float tot = 0.f;
    for (int q = 0; q < tpe; ++q) tot += ared[ae_local * tpe + q];
    if (ae < NSMALL) {
      G[OFF_B1 + ae] = tot;
    } else {
      const int m = ae - NSMALL;  // 0 loss, 1 correct, 2 count
      float* accp = m == 0 ? &ctrl->acc_loss : (m == 1 ? &ctrl->acc_correct : &ctrl->acc_count);
      const float old = m == 0 ? c.acc_loss : (m == 1 ? c.acc_correct : c.acc_count);
      // fold the previous step's all-reduced metric into the epoch total -- if there is one
      // not yet folded: none before the first step, none right after a flush (which folded
      // it), and the staging may hold anything then (the peer self-test's values)
      if (!sh) *accp = c.pend2 ? old + ag_old : old;
      // (a non-finite / out-of-range fixed-point input so far: the loss is NaN from now on)
      G[OFF_LOSS + m] = m == 0 && c.bad ? __builtin_nanf("") : m < 2 ? tot : (float)max(0, min(B, gcount - c.row0));
    }
  }
  // zero the dead hacc parity (read by the previous step's bwd) for the next fwd,
  // spread over the blocks
  {
    long long* hz = hacc + (long)(par ^ 1) * B * HACC_PITCH;
    for (int i = s * 512 + tid; i < B * HID / 2; i += NS * 512)  // (32 16-B units per row)
      *reinterpret_cast<uint4*>(hz + (i >> 5) * HACC_PITCH + (i & 31) * 2) = make_uint4(0u, 0u, 0u, 0u);
  }
  if (xpf) reinterpret_cast<uint4*>(xnext)[xpu] = xnv;
  if (ONE && xnext != nullptr && s == 0 && tid == 0) *xtag = ((long long)c.xgen << 32) | (long long)(unsigned)(ncur + 1);
  if (sh) exchange_tail(xa, ctrl, G, hconv + par * NCONV, accw, xe, s, NS, np, p0, dn, dm0, lane, tid, xown, xo, xu);
  stamp(sts, st, 5);
  stamp_flush(sts, st, 13);
  if (st != nullptr && tid == 256) st[blockIdx.x * 16 + 13] = sts.t[12];  // wave 4's view
}

// =================================================================================
// flush: apply the pending (deferred) update to every parameter, zero the gradient
// buffers, fold the pending metrics into the epoch accumulators, clear `pending`.
// =================================================================================
// G / hconv: the reduced gradient (the peer all-reduce's `out` when it is folded into the
// step, see ConvNetBuffers::Gr); hconv_w: the buffer bwd adds into (both parities cleared)
__global__ __launch_bounds__(1024) void flush(float* __restrict__ P, float* __restrict__ G, float* __restrict__ V,
                                             const float* __restrict__ W1alt, const float* __restrict__ V1alt,
                                             long long* __restrict__ hconv, const float* __restrict__ calt,
                                             long long* __restrict__ hacc, int B, int eager,
                                             uint16_t* __restrict__ w1bf, Ctrl* __restrict__ ctrl,
                                             long long* __restrict__ hconv_w) {
  const Ctrl c = *ctrl;
  const bool mom = c.momentum != 0.f, pend = c.pending != 0;
  // after a step's bwd: current W1 / conv parameters live in the alternates when wpar is
  // set; the pending conv gradient is in hconv[wpar ^ 1]
  const long long* hg = hconv + (c.wpar ^ 1) * NCONV;
  // eager: W1 is current and its gradient was never stored -- only the conv and
  // b1/W2/b2 parameters are visited
  const int nvisit = eager ? NPARAM - (OFF_B1 - OFF_W1) : NPARAM;
  for (int iv = blockIdx.x * blockDim.x + threadIdx.x; iv < nvisit; iv += gridDim.x * blockDim.x) {
    const int i = eager && iv >= OFF_W1 ? iv + (OFF_B1 - OFF_W1) : iv;
    const bool w1 = i >= OFF_W1 && i < OFF_B1;
    const bool alt1 = !eager && c.wpar && w1, altc = c.wpar && i < NCONV;
    const float w = alt1 ? W1alt[i - OFF_W1] : (altc ? calt[i] : P[i]);
    const float v = alt1 ? V1alt[i - OFF_W1] : (altc ? calt[NCONV + i] : V[i]);
    const float g = i < NCONV ? from_fix(hg[i], CINV) : G[i];
    float wn, vn;
    sgd_or_keep(pend && !(eager && w1), w, g, v, c, wn, vn);  // eager: W1 is already current
    P[i] = wn;
    if (mom) V[i] = vn;
    if (w1) w1bf[i - OFF_W1] = f2bf(wn);
  }
  // the fixed-point accumulators start the next step at zero -- except the conv-gradient
  // parity read above (hg): other threads / blocks of THIS launch may not have loaded it
  // yet, and zeroing it here raced with them (a lost conv gradient on one rank, seen as
  // replicas whose conv parameters differed after an epoch flush).  That parity needs no
  // zero: after the flush nothing pending reads it, and the step that next writes it
  // zeroes it first (fwd's owner block).
  const int rp = c.wpar ^ 1;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * NCONV + 2 * B * HID; i += gridDim.x * blockDim.x) {
    if (i < 2 * NCONV) {
      const bool read_parity = i / NCONV == rp;
      if (!read_parity) hconv[i] = 0;
      if (!read_parity || hconv_w != hconv) hconv_w[i] = 0;
    } else {
      const int j = i - 2 * NCONV;  // (row j / HID of both parities, column j % HID)
      hacc[(j >> 6) * HACC_PITCH + (j & 63)] = 0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && pend) {
    ctrl->acc_loss = c.acc_loss + G[OFF_LOSS];
    ctrl->acc_correct = c.acc_correct + G[OFF_CORR];
    ctrl->acc_count = c.acc_count + G[OFF_CNT];
    // the metric tail is folded: the next bwd's fold of "the previous step's metric" (world 1
    // / the standalone all-reduce) must add nothing (the gradient itself is never re-read:
    // the next fwd applies no update)
    G[OFF_LOSS] = G[OFF_CORR] = G[OFF_CNT] = 0.f;
  }
  __syncthreads();
  // one block (eager world 1: 1,034 parameters): every read of the ctrl block is behind the
  // barrier above, so no arrival ticket (a returning atomic costs the kernel ~1.5 us)
  if (threadIdx.x == 0) {
    if (gridDim.x == 1 ||
        __hip_atomic_fetch_add(&ctrl->flush_ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (int)gridDim.x - 1) {
      ctrl->wpar = 0;
      ctrl->pending = 0;
      ctrl->flush_ticket = 0;
      ctrl->ticket = 0;  // (the sharded bwd's arrival count: bounded between flushes)
    }
  }
}

// =================================================================================
// sharded step: the pending update's reduced gradient gathered for flush / the host
// (waits for every unit and every rank's small message of the last exchange epoch, then
// writes the small sums into the gradient staging's b1 / W2 / b2 / metric slots and the
// conv sum into hred[wpar ^ 1], where flush reads them).  One block; nothing pending: no-op.
// It depends only on every rank having run that step's bwd -- not on their calling it.
// =================================================================================
__global__ __launch_bounds__(512) void sh_gather(Ctrl* __restrict__ ctrl, const XArgs xa, long long* __restrict__ hred,
                                                 int NS, int PP) {
  const Ctrl c = *ctrl;
  if (!c.pending) return;
  const unsigned xe = (unsigned)c.xcnt;
  const int ps = xe & 1, NU = 4 * NS, tid = threadIdx.x;
  float* xo = xa.out[xa.rank];
  // every block: its units (u = block, block + grid, ...); bf16 exchange: expanded into the
  // fp32 staging that flush reads
  for (int u = blockIdx.x; u < NU; u += gridDim.x) {
    if (tid < 2) x_wait(xa, x_gflag(xo, NU, u, tid), xe, XW_UNIT);
    __syncthreads();
    if (xa.gbf16) {
      const int sl = u >> 2, q = u & 3, k0 = sl * PP * 32, k1 = min(FEAT, k0 + PP * 32);
      const uint16_t* g16 = reinterpret_cast<const uint16_t*>(xo + kXG16);
      for (int e = tid; e < (k1 - k0) * 16; e += 512) {
        const long idx = (long)(k0 + (e >> 4)) * HID + 16 * q + (e & 15);
        xo[kXGred + OFF_W1 + idx] = bf2f(g16[idx]);
      }
    }
  }
  if (blockIdx.x != 0) return;
  if (tid < xa.world) x_wait(xa, x_sflag(xo, NU, ps, tid), xe, XW_SMALL);
  __syncthreads();
  for (int i = tid; i < NSMALL + 3; i += 512) {
    float a = 0.f;
    for (int r = 0; r < xa.world; ++r) a += x_small(xo, ps, r)[SM_GRAD + i];
    xo[kXGred + (i < NSMALL ? OFF_B1 + i : OFF_LOSS + i - NSMALL)] = a;
  }
  for (int i = tid; i < NCONV; i += 512) {
    long long q = 0;
    for (int r = 0; r < xa.world; ++r) q += reinterpret_cast<const long long*>(x_small(xo, ps, r) + SM_CONV)[i];
    hred[(c.wpar ^ 1) * NCONV + i] = q;
  }
}

}  // namespace convnet2

// ---------------------------------------------------------------------------------
// Host-side launchers (no allocation / sync: capturable into a hipGraph).
// ---------------------------------------------------------------------------------
int convnet_num_slices(int PP) { return (convnet::NPOS + PP - 1) / PP; }
// int64 elements of the dense-1 accumulator (both parities, rows HACC_PITCH apart)
long convnet_hacc_elems(int B) { return 2L * B * convnet::HACC_PITCH; }
size_t convnet_grad_count(int) { return (size_t)convnet::NGRAD; }
// fwd images per block = 2^lg: 16 up to B = 256 (more blocks, shorter per-block chains),
// 64 beyond (bounded replication of the W1-slice / conv-parameter loads)
int convnet_f1_lg(int B) { return B <= 256 ? 4 : 6; }

size_t convnet2_fwd_lds(int PP, int lg) {
  using namespace convnet;
  const int KP = kpitch(PP), IB = 1 << lg;
  const size_t xsb = (size_t)IB * XR * IMG * 4, partb = (size_t)IB * HID * 4;
  return (xsb > partb ? xsb : partb) + (size_t)(IB + HID) * KP * 2 + NCONV * 4 + (size_t)IB * PP * 32 + 256 * 4;
}
size_t convnet2_bwd_lds(int PP) {
  using namespace convnet;
  const int KD = PP * 32 + 4;
  const size_t dpsb = (size_t)CH * KD * 4;
  const size_t rb = dpsb > (size_t)convnet2::HEAD_BYTES ? dpsb : (size_t)convnet2::HEAD_BYTES;
  const size_t redb = (size_t)16 * NCONV * 4;  // `red` spans pt + dht after the MFMAs
  const size_t ptdht = (size_t)PP * 32 * HP * 2 + (size_t)2 * HID * HP * 2;
  return XS_BYTES + rb + (ptdht > redb ? ptdht : redb) + (size_t)2 * CH * HP * 2 + (size_t)PP * 32 * HP * 2 +
         (size_t)CH * PP * 32 + 16 + 256 * 4;
}

// eager W1 update: world-1 runs with the single-chunk backward (B <= 64) only
static int eager2(const ConvNetBuffers& b, int B) { return b.eager_w1 && B <= convnet::CH ? 1 : 0; }

static XArgs xargs(const ConvNetBuffers& b) {
  if (b.xa) return *b.xa;
  XArgs a{};
  return a;  // world 0: not sharded
}

template <bool U8>
static void launch2_fwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  using namespace convnet;
  const int NS = convnet_num_slices(PP);
  const int lg = convnet_f1_lg(B);
  const dim3 g1(NS, (B + (1 << lg) - 1) >> lg);
  hipLaunchKernelGGL((convnet2::fwd<U8>), g1, dim3(512), convnet2_fwd_lds(PP, lg), st,
                     B <= CH ? b.xnext : nullptr, b.w1bf, b.P, b.V, b.calt, b.hconv_r ? b.hconv_r : b.hconv,
                     b.Gr ? b.Gr : b.G, B | (PP << 16), lg | (eager2(b, B) << 8), b.ctrl, b.X, b.W1alt, b.V1alt,
                     b.pooled, b.code, b.hacc, b.hconv, b.stamps, xargs(b), b.xtag, b.labels,
                     B <= CH ? b.xcur : nullptr, b.ycur, b.par_hint);
}

static int ppb_of(const ConvNetBuffers& b, int PP) { return b.ppb > 0 ? b.ppb : PP; }

template <bool U8>
static void launch2_bwd(const ConvNetBuffers& b, int B, int PPf, hipStream_t st) {
  using namespace convnet;
  const int PP = ppb_of(b, PPf);
  const int NS = convnet_num_slices(PP);
  // aux elements (b1/W2/b2 gradients + metric tail) per block, and a power-of-two thread
  // count per element (<= 64) that fits them in 512 threads
  const int chunk_aux = (convnet2::NAUX2 + NS - 1) / NS;
  int ltpe = 0;
  while (ltpe < 6 && (2 << ltpe) * chunk_aux <= 512) ++ltpe;
  const int auxm = chunk_aux | (ltpe << 16);
  if (B <= CH)
    hipLaunchKernelGGL((convnet2::bwd<U8, true>), dim3(NS), dim3(512), convnet2_bwd_lds(PP), st, b.hacc,
                       B <= CH ? b.ycur : nullptr, B <= CH ? b.xcur : nullptr, b.par_hint, B | (PP << 16), b.P,
                       b.w1bf, b.pooled, b.code, b.ctrl, b.X, b.labels, b.G, b.hconv, eager2(b, B), b.P, b.V, b.w1bf,
                       b.stamps ? b.stamps + 2 * 256 * 16 : nullptr, b.Gr ? b.Gr : b.G, xargs(b), b.xnext, b.xtag,
                       auxm);
  else
    hipLaunchKernelGGL((convnet2::bwd<U8, false>), dim3(NS), dim3(512), convnet2_bwd_lds(PP), st, b.hacc,
                       B <= CH ? b.ycur : nullptr, B <= CH ? b.xcur : nullptr, b.par_hint, B | (PP << 16), b.P,
                       b.w1bf, b.pooled, b.code, b.ctrl, b.X, b.labels, b.G, b.hconv, eager2(b, B), b.P, b.V, b.w1bf,
                       b.stamps ? b.stamps + 2 * 256 * 16 : nullptr, b.Gr ? b.Gr : b.G, xargs(b), b.xnext, b.xtag,
                       auxm);
}

hipError_t convnet2_launch_fwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  if (!b.hacc || !b.hconv || !b.calt || B > 0xffff) return hipErrorInvalidValue;
  if (b.x_u8) launch2_fwd<true>(b, B, PP, st);
  else launch2_fwd<false>(b, B, PP, st);
  return hipGetLastError();
}

hipError_t convnet2_launch_bwd(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  if (!b.hacc || !b.hconv || !b.calt || B > 0xffff) return hipErrorInvalidValue;
  if (convnet2_bwd_lds(ppb_of(b, PP)) > 160 * 1024) return hipErrorInvalidValue;
  if (b.xa && b.xa->ppb != ppb_of(b, PP)) return hipErrorInvalidValue;
  if (b.x_u8) launch2_bwd<true>(b, B, PP, st);
  else launch2_bwd<false>(b, B, PP, st);
  return hipGetLastError();
}

hipError_t convnet2_launch_step(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  hipError_t e = convnet2_launch_fwd(b, B, PP, st);
  return e != hipSuccess ? e : convnet2_launch_bwd(b, B, PP, st);
}

hipError_t convnet2_launch_gather(const ConvNetBuffers& b, int PP, hipStream_t st) {
  if (!b.xa || b.xa->world < 2 || !b.hconv_r) return hipErrorInvalidValue;
  const int ppb = ppb_of(b, PP);
  hipLaunchKernelGGL(convnet2::sh_gather, dim3(57), dim3(512), 0, st, b.ctrl, *b.xa, b.hconv_r, convnet_num_slices(ppb),
                     ppb);
  return hipGetLastError();
}

hipError_t convnet2_launch_flush(const ConvNetBuffers& b, int B, hipStream_t st) {
  hipLaunchKernelGGL(convnet2::flush, dim3(eager2(b, B) ? 1 : 340), dim3(eager2(b, B) ? 1024 : 256), 0, st, b.P, b.Gr ? b.Gr : b.G, b.V,
                     b.W1alt, b.V1alt, b.hconv_r ? b.hconv_r : b.hconv, b.calt, b.hacc, B, eager2(b, B), b.w1bf, b.ctrl,
                     b.hconv);
  return hipGetLastError();
}

hipError_t convnet2_set_lds_limits() {
  const void* fns[6] = {(const void*)convnet2::fwd<false>,        (const void*)convnet2::fwd<true>,
                        (const void*)convnet2::bwd<false, true>,  (const void*)convnet2::bwd<true, true>,
                        (const void*)convnet2::bwd<false, false>, (const void*)convnet2::bwd<true, false>};
  for (const void* f : fns) {
    hipFuncAttributes at;
    hipError_t e = hipFuncGetAttributes(&at, f);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - (int)at.sharedSizeBytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace damd
