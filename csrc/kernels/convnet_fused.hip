// Fused data-parallel training step for the reference MNIST CNN (gfx950 / MI355X).
//
// Model (reference README.md:58-73):
//   x[28,28,1] -> Conv2D(32,3x3,valid)+bias+ReLU -> MaxPool 2x2/2 -> Flatten(NHWC, 5408)
//   -> Dense(64)+bias+ReLU -> Dense(10) logits -> SparseCategoricalCrossentropy(from_logits)
//   optimizer: SGD(lr, momentum, nesterov) on fp32 master weights.
//
// One training step = 3 launches (+ one RCCL all-reduce of the flat gradient buffer
// between steps when world > 1).  At this size (183 MFLOP/step) every kernel is bound
// by its chain of dependent memory round trips, so each kernel issues all of its
// independent global loads up front, loads are unconditional (clamped index + value
// mask: a guarded load becomes a branch + vmcnt(0)), workgroup barriers are LDS-only
// (lds_barrier: no wait for outstanding global stores), and no kernel has a grid-wide
// reduction on its critical path.  The optimizer update of step t is *deferred* into
// the kernels of step t+1 that first consume each parameter, so there is no separate
// SGD launch (flush_pending applies the last pending update before the host reads
// weights):
//
//   F1 (grid NS slices of PP pooled positions, 512 thr): pending SGD update of this
//       slice's W1 rows (owned by exactly one block) and of the conv weights (in
//       registers), conv on MFMA
//       (16x16x32 bf16 with a split-precision K packing): the 4 pixels of one 2x2 pool
//       window are the 4 accumulator rows of one lane, so bias+ReLU+max+argmax happen
//       in registers; the pooled tile stays in LDS and is multiplied by the W1 K-slice
//       on MFMA (one pooled position == one K step) -> split-K slab.
//   F2 (grid B, 256 thr, one sample row per block): slab reduction (4 waves split the
//       slices) + b1 + ReLU, Dense(10), softmax-xent + accuracy, dz, dh, the row's
//       contributions to dW2/db2/db1/loss/correct (column-major records), and the
//       write-back of the conv parameters' pending update (spread over blocks).
//   F3 (grid NS, 512 thr): dW1 = P^T dh (MFMA, straight into the gradient buffer),
//       dP = dh W1^T (MFMA into LDS), MaxPool/ReLU backward through the stored argmax
//       code, this slice's conv weight/bias gradient partial (atomically added into
//       the gradient buffer); every block also applies the
//       pending update of a slice of b1/W2/b2 and reduces that slice's new gradient
//       from F2's records (fixed order: deterministic, no atomics).
//   dh enters both backward MFMAs as a hi+lo pair of bf16 (~16-bit mantissa) because
//   the conv weight gradient sums 43k terms with heavy cancellation.
//
// Step counter without intra-kernel races: F1 reads ctrl.cursor and its block 0 copies
// it to cur2, F2 reads cur2 and copies it to cur3, F3 reads cur3 and its block 0
// advances cursor / iterations -- no kernel writes a field it reads.
//
// Flat parameter / gradient layout = Keras weight order (views of the master buffer are
// the Keras variables): conv2d/kernel (3,3,1,32), conv2d/bias, dense/kernel (5408,64),
// dense/bias, dense_1/kernel (64,10), dense_1/bias; the gradient buffer tail carries
// [loss_sum, correct, count], so ONE all-reduce per step moves grads + metrics.  Inputs are epoch-permuted copies of
// the dataset (row g of the epoch = global sample g), read without an index gather.
#include "convnet_dev.h"

namespace damd {
namespace convnet {

// =================================================================================
// Head fused into F1 (opt-in, DAMD_CONVNET_FUSE_HEAD=1; measured 37.5 vs 30.0 us/step for the
// separate F2 launch at B=64, so F2 stays the default).
// Dense-1 split-K: every F1 block adds its [IB rows][64] partial into hacc (fp32 atomics,
// memory-side; 256 contiguous bytes per wave instruction) and draws a ticket from its
// image group's counter.  The block whose ticket completes the group (the last arriver,
// told by the returned count) runs F2's work for the group's rows: hacc + b1 + ReLU,
// Dense(10), softmax-xent, accuracy, dz, dh (bf16 hi/lo, both layouts), the per-row
// records, then re-zeroes hacc.  The block completing the whole grid writes back the
// conv parameters' pending update and zeroes their gradient (F2's other duty).  Hand-off
// per cdna_hip_programming.md §6 Guideline 16 (row 1 of the valid forms): every payload
// access is memory-side or sc1 (atomics; hacc loads/stores via relaxed agent-scope
// atomics), every storing wave drains vmcnt before the barrier that precedes the ticket.
// Counters count forever (ticket mod blocks per group), so no per-step reset.  Saves
// F2's launch and boundary (~9 us of a ~30 us step) for ~3 us of tail in F1.
// hacc = slabs[0 .. B*64), counters = slabs[B*64 ..) (as unsigned): per group, then one
// for the grid.
// =================================================================================
struct HeadIn {
  float sp[2], sg[2], sv[2];  // b1/W2/b2 (714 values): this thread's i = tid, tid + 512
  int y;                      // label of row (img0 + tid) for tid < IB
  bool yvalid;
};

__device__ __forceinline__ void head_prefetch(HeadIn& h, const float* P, const float* G, const float* V,
                                              const int* labels, const Ctrl& c, int img0, int B) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = min(tid + u * 512, NSMALL - 1);
    h.sp[u] = P[OFF_B1 + i];
    h.sg[u] = G[OFF_B1 + i];
    h.sv[u] = V[OFF_B1 + i];
  }
  const long g = (long)c.cursor * c.global_batch + c.row0 + img0 + min(tid, 63);
  h.yvalid = g < c.nsamples && img0 + tid < B;
  h.y = labels[max(0L, min(g, (long)c.nsamples - 1))];
}

__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void f1_head(const HeadIn& hin, float* xs, const float* cw, float* P, float* G, float* V,
                                     Ctrl* ctrl, const Ctrl& c, float* slabs, uint16_t* dhq, float* rec, float cp,
                                     float cg, float cv, int img0, int IB, int B, int tid, int wave, int lane) {
  __shared__ int flag[2];
  __shared__ float zsh[8][16];
  __shared__ float ysh[64];
  __shared__ unsigned char yok[64];
  float* hacc = slabs;
  unsigned* cnt = reinterpret_cast<unsigned*>(slabs + (long)B * HID);
  const int ngroups = gridDim.y, per_group = gridDim.x;
  // 1) this block's partial rows -> hacc (one wave instruction = one 256-B row)
  for (int r = wave; r < IB; r += 8)
    if (img0 + r < B) atomicAdd(hacc + (long)(img0 + r) * HID + lane, xs[r * HID + lane]);
  if (tid < IB) {
    ysh[tid] = __int_as_float(hin.y);
    yok[tid] = hin.yvalid ? 1 : 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every adding wave: its atomics acknowledged
  __syncthreads();
  if (tid == 0) {
    const unsigned tg = __hip_atomic_fetch_add(cnt + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned ta = __hip_atomic_fetch_add(cnt + ngroups, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = (tg % per_group) == (unsigned)(per_group - 1);
    flag[1] = (ta % (per_group * ngroups)) == (unsigned)(per_group * ngroups - 1);
  }
  __syncthreads();
  // 2) the grid's last block: conv parameters' pending update written back, gradient zeroed
  //    (every F1 block has read them by now -- it arrived)
  if (flag[1] && tid < NCONV) {
    float wn, vn;
    sgd_update(cp, cg, cv, c.lr, c.momentum, c.nesterov, wn, vn);
    P[tid] = wn;
    if (c.momentum != 0.f) V[tid] = vn;
    G[tid] = 0.f;
  }
  if (!flag[0]) return;
  // 3) the group's last block: the head of rows img0 .. img0 + IB
  float* sp = xs;                  // updated b1[64], W2[640], b2[10] (LDS, after the partial rows)
  float* hs = xs + NSMALL + 2;     // [8 waves][64] h of the wave's current row
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * 512;
    if (i < NSMALL) {
      float wn, vn;
      sgd_update(hin.sp[u], hin.sg[u], hin.sv[u], c.lr, c.momentum, c.nesterov, wn, vn);
      sp[i] = wn;
    }
  }
  __syncthreads();
  const float* b1n = sp;
  const float* w2n = sp + HID;
  const float* b2n = sp + HID + HID * NCLS;
  const long gstart = (long)c.cursor * c.global_batch;
  const int gcount = (int)min((long)c.global_batch, (long)c.nsamples - gstart);
  const float inv = gcount > 0 ? 1.f / (float)gcount : 0.f;
  const int BP = (B + CH - 1) / CH * CH;
  const long Q = (long)BP * HID;
  // one wave per row (rows are independent: no block barrier inside the loop)
  for (int r = wave; r < IB; r += 8) {
    const int b = img0 + r;
    if (b >= B) break;
    float* hacc_row = hacc + (long)b * HID;
    const float hv = ld_agent(hacc_row + lane);
    st_agent(hacc_row + lane, 0.f);  // consumed: zero for the next step
    const float h = fmaxf(hv + b1n[lane], 0.f);
    hs[wave * 64 + lane] = h;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < 16) {
      float z = -INFINITY;
      if (lane < NCLS) {
        z = b2n[lane];
#pragma unroll 8
        for (int k = 0; k < HID; ++k) z = fmaf(hs[wave * 64 + k], w2n[k * NCLS + lane], z);
      }
      zsh[wave][lane] = z;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool valid = yok[r] != 0;
    const int y = valid ? __float_as_int(ysh[r]) : 0;
    float z[NCLS];
    float m = -INFINITY;
    int am = 0;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) {
      z[k] = zsh[wave][k];
      am = z[k] > m ? k : am;
      m = fmaxf(m, z[k]);
    }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) se += __expf(z[k] - m);
    const float lse = m + __logf(se);
    float zy = z[0];
#pragma unroll
    for (int k = 1; k < NCLS; ++k) zy = (k == y) ? z[k] : zy;
    float dz[NCLS];
#pragma unroll
    for (int k = 0; k < NCLS; ++k) dz[k] = valid ? (__expf(z[k] - lse) - (k == y ? 1.f : 0.f)) * inv : 0.f;
    float dhl = 0.f;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) dhl = fmaf(dz[k], w2n[lane * NCLS + k], dhl);
    dhl = h > 0.f ? dhl : 0.f;
    const uint16_t hi = f2bf(dhl), lo = bf16_lo(dhl, hi);
    dhq[(long)b * HID + lane] = hi;
    dhq[Q + (long)b * HID + lane] = lo;
    dhq[2 * Q + (long)lane * BP + b] = hi;
    dhq[3 * Q + (long)lane * BP + b] = lo;
    rec[(long)(650 + lane) * B + b] = dhl;  // db1
#pragma unroll
    for (int k = 0; k < NCLS; ++k) rec[(long)(lane * NCLS + k) * B + b] = h * dz[k];  // dW2
    if (lane < NCLS) {
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < NCLS; ++q) d = (q == lane) ? dz[q] : d;
      rec[(long)(640 + lane) * B + b] = d;  // db2
    }
    if (lane == 0) {
      rec[(long)714 * B + b] = valid ? (lse - zy) : 0.f;
      rec[(long)715 * B + b] = (valid && am == y) ? 1.f : 0.f;
    }
  }
}

// =================================================================================
// F1: grid (NS slices, ISPLIT image groups of IB = 2^lg images)
// =================================================================================
template <bool U8, bool HEAD>
__global__ __launch_bounds__(512) void f1_forward(
    const void* __restrict__ X, float* __restrict__ P, float* __restrict__ G,
    float* __restrict__ V, float* __restrict__ W1alt, float* __restrict__ V1alt,
    uint16_t* __restrict__ w1bf, Ctrl* __restrict__ ctrl, uint16_t* __restrict__ pooled,
    uint8_t* __restrict__ code, float* __restrict__ slabs, const int* __restrict__ labels,
    uint16_t* __restrict__ dhq, float* __restrict__ rec, int B, int PP, int lg, unsigned long long* st) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  Stamps sts;
  stamp(sts, st, 0);
  const int IB = 1 << lg, img0 = blockIdx.y * IB;
  const int BP = (B + CH - 1) / CH * CH;  // padded batch pitch of the feature-major buffers
  const int p0 = s * PP, p1 = min(NPOS, p0 + PP), np = p1 - p0, K = np * 32;
  const int KP = kpitch(PP);
  float* xs = reinterpret_cast<float*>(smem);                              // [IB][XR][28]
  uint16_t* as = reinterpret_cast<uint16_t*>(smem + IB * XR * IMG * 4);    // [IB][KP] pooled tile
  uint16_t* w1t = as + IB * KP;                                            // [HID][KP] W1 slice^T
  float* cw = reinterpret_cast<float*>(w1t + HID * KP);                    // [320] conv params
  const Ctrl c = *ctrl;
  if (s == 0 && blockIdx.y == 0 && tid == 0) {
    ctrl->cur2 = c.cursor;
    if (HEAD) ctrl->cur3 = c.cursor;  // no F2 in between: F3 reads the step index directly
  }
  const long row_base = (long)c.cursor * c.global_batch + c.row0 + img0;
  const int r0 = 2 * (p0 / PO);
  const int nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  const bool mom = c.momentum != 0.f;
  stamp(sts, st, 1);

  // ---- issue every independent load of the prologue ----
  XStage<U8> xst;
  x_load<U8>(xst, X, row_base, c.nsamples, B - img0, IB, r0, nrows);
  const int n4 = K * HID / 4;  // <= 2048
  float4 wv[4], gv[4], vv[4];
  // W1 (and its velocity) are double-buffered by step parity: this step reads the
  // current buffer and the slice's first image-group block writes the updated rows into
  // the other one, so the four blocks sharing a slice never race on the master copy
  const float* Wcur = c.wpar ? W1alt : P + OFF_W1;
  const float* Vcur = c.wpar ? V1alt : V + OFF_W1;
  float* Wnext = c.wpar ? const_cast<float*>(P) + OFF_W1 : W1alt;
  float* Vnext = c.wpar ? const_cast<float*>(V) + OFF_W1 : V1alt;
  const float4* P4 = reinterpret_cast<const float4*>(Wcur + p0 * 32 * HID);
  const float4* G4 = reinterpret_cast<const float4*>(G + OFF_W1 + p0 * 32 * HID);
  // without momentum the velocity is never read: point its loads at W (cache hits)
  const float4* V4 = reinterpret_cast<const float4*>((mom ? Vcur : Wcur) + p0 * 32 * HID);
  const bool owner = blockIdx.y == 0;
  float4* Wn4 = reinterpret_cast<float4*>(Wnext + p0 * 32 * HID);
  float4* Vn4 = reinterpret_cast<float4*>(Vnext + p0 * 32 * HID);
  uint2* Wb = reinterpret_cast<uint2*>(w1bf + p0 * 32 * HID);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int ic = min(tid + u * 512, n4 - 1);
    wv[u] = P4[ic];
    gv[u] = G4[ic];
    vv[u] = V4[ic];
  }
  const int tcl = min(tid, NCONV - 1);
  const float cp = P[tcl], cv = V[tcl], cg = G[tcl];
  HeadIn hin;
  if constexpr (HEAD) head_prefetch(hin, P, G, V, labels, c, img0, B);

  // ---- pending SGD update of the W1 slice (the owner block writes the next buffer and
  //      a bf16 copy for F3) and of the conv weights (registers; F2 writes them back) ----
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + u * 512;
    if (i < n4) {
      float4 wn, vn;
      sgd_update(wv[u].x, gv[u].x, vv[u].x, c.lr, c.momentum, c.nesterov, wn.x, vn.x);
      sgd_update(wv[u].y, gv[u].y, vv[u].y, c.lr, c.momentum, c.nesterov, wn.y, vn.y);
      sgd_update(wv[u].z, gv[u].z, vv[u].z, c.lr, c.momentum, c.nesterov, wn.z, vn.z);
      sgd_update(wv[u].w, gv[u].w, vv[u].w, c.lr, c.momentum, c.nesterov, wn.w, vn.w);
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
  if (tid < NCONV) {
    float wn, vn;
    sgd_update(cp, cg, cv, c.lr, c.momentum, c.nesterov, wn, vn);
    cw[tid] = wn;
  }
  stamp(sts, st, 2);
  x_store<U8>(xst, xs);
  lds_barrier();
  stamp(sts, st, 3);

  ConvFrag cf;
  conv_setup(cf, cw, lane);
  conv_pool(cf, xs, p0, np, r0, lg, wave, lane, [&](int bo, int plo, int ch, uint16_t hb, uint8_t cd) {
    as[bo * KP + plo * 32 + ch] = hb;
    if (img0 + bo < B) {  // pooled tile + argmax codes for F3 (async stores, off the critical path)
      const int k = (p0 + plo) * NF + ch;
      pooled[(long)k * BP + img0 + bo] = hb;  // feature-major: F3's dW1 A operand, no transpose
      code[(long)(img0 + bo) * FEAT + k] = cd;
    }
  });
  lds_barrier();
  stamp(sts, st, 4);
  // ---- dense-1 split-K partial: slab[s][row][n] = sum_k pooled[row][k] * W1[k][n] ----
  const int ko = 8 * (lane >> 4);
  const int ntiles = (IB >> 4) * 4;  // (row tile, col tile) pairs
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
    for (int j = 0; j < 4; ++j) {
      const int row = 16 * mt + 4 * (lane >> 4) + j, lb = img0 + row;
      if constexpr (HEAD) xs[row * HID + bn] = acc[j];  // staged: one 256-B atomic row per wave op
      else if (lb < B) slabs[((long)s * B + lb) * HID + bn] = acc[j];
    }
  }
  stamp(sts, st, 5);
  if constexpr (HEAD) {
    lds_barrier();
    f1_head(hin, xs, cw, P, G, V, ctrl, c, slabs, dhq, rec, cp, cg, cv, img0, IB, B, tid, wave, lane);
  }
  stamp_flush(sts, st, 6);
}

// =================================================================================
// F2: one sample row per block
// =================================================================================
__global__ __launch_bounds__(256) void f2_head(
    const int* __restrict__ labels, float* __restrict__ P, float* __restrict__ G, float* __restrict__ V,
    Ctrl* __restrict__ ctrl, const float* __restrict__ slabs,
    uint16_t* __restrict__ dhq, float* __restrict__ rec, int B, int NS, unsigned long long* st) {
  Stamps sts;
  stamp(sts, st, 0);
  __shared__ __attribute__((aligned(16))) float lds[NSMALL + 2 + 4 * 64 + 64 + 16];
  float* sp = lds;                 // updated b1[64], W2[640], b2[10]
  float* hw = sp + NSMALL + 2;     // [4][64] per-wave partial slab sums
  float* hs = hw + 4 * 64;         // [64] h
  float* zs = hs + 64;             // [16] logits
  const Ctrl c = *ctrl;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, b = blockIdx.x;
  if (b == 0 && tid == 0) ctrl->cur3 = c.cur2;
  const long gstart = (long)c.cur2 * c.global_batch;
  const long g = gstart + c.row0 + b;
  const bool valid = g < c.nsamples;
  const int gcount = (int)min((long)c.global_batch, (long)c.nsamples - gstart);
  const float inv = gcount > 0 ? 1.f / (float)gcount : 0.f;

  // ---- issue: label, small params (3 per thread), slab slices, conv write-back inputs ----
  const int yl = labels[max(0L, min(g, (long)c.nsamples - 1))];
  const int y = valid ? yl : 0;
  float pv[3], gvv[3], vv[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int i = min(tid + u * 256, NSMALL - 1);
    pv[u] = P[OFF_B1 + i];
    gvv[u] = G[OFF_B1 + i];
    vv[u] = V[OFF_B1 + i];
  }
  // conv parameters' pending update is written back here, spread over the B blocks
  const int cpb = (NCONV + gridDim.x - 1) / gridDim.x;
  const int ci = min(b * cpb + tid, NCONV - 1);
  const bool c_on = tid < cpb && b * cpb + tid < NCONV;
  const float cpp = P[ci], cvv = V[ci], cgg = G[ci];
  float hsum = 0.f;
  {
    const float* src = slabs + (long)b * HID + l;
    const long stride = (long)B * HID;
    float t[16];
    for (int s0 = w; s0 < NS; s0 += 64) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int sj = s0 + 4 * j;
        const float v = src[min(sj, NS - 1) * stride];
        t[j] = sj < NS ? v : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) hsum += t[j];
    }
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int i = tid + u * 256;
    if (i < NSMALL) {
      float wn, vn;
      sgd_update(pv[u], gvv[u], vv[u], c.lr, c.momentum, c.nesterov, wn, vn);
      sp[i] = wn;
    }
  }
  if (c_on) {
    float wn, vn;
    sgd_update(cpp, cgg, cvv, c.lr, c.momentum, c.nesterov, wn, vn);
    P[ci] = wn;
    if (c.momentum != 0.f) V[ci] = vn;
    G[ci] = 0.f;  // consumed (F1 read it before this launch); F3 accumulates the new one
  }
  hw[w * 64 + l] = hsum;
  lds_barrier();
  stamp(sts, st, 1);
  const float* b1n = sp;
  const float* w2n = sp + HID;
  const float* b2n = sp + HID + HID * NCLS;
  const float h = fmaxf(((hw[l] + hw[64 + l]) + (hw[128 + l] + hw[192 + l])) + b1n[l], 0.f);
  if (w == 0) hs[l] = h;
  lds_barrier();
  if (tid < 16) {
    float z = -INFINITY;
    if (tid < NCLS) {
      z = b2n[tid];
#pragma unroll 8
      for (int k = 0; k < HID; ++k) z = fmaf(hs[k], w2n[k * NCLS + tid], z);
    }
    zs[tid] = z;
  }
  lds_barrier();
  float z[NCLS];
  float m = -INFINITY;
  int am = 0;
#pragma unroll
  for (int k = 0; k < NCLS; ++k) {
    z[k] = zs[k];
    am = z[k] > m ? k : am;
    m = fmaxf(m, z[k]);
  }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < NCLS; ++k) se += __expf(z[k] - m);
  const float lse = m + __logf(se);
  float zy = z[0];
#pragma unroll
  for (int k = 1; k < NCLS; ++k) zy = (k == y) ? z[k] : zy;
  float dz[NCLS];
#pragma unroll
  for (int k = 0; k < NCLS; ++k) dz[k] = valid ? (__expf(z[k] - lse) - (k == y ? 1.f : 0.f)) * inv : 0.f;
  if (w == 0) {
    float dhl = 0.f;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) dhl = fmaf(dz[k], w2n[l * NCLS + k], dhl);
    dhl = h > 0.f ? dhl : 0.f;
    // dh as a bf16 hi+lo pair, row-major [b][n] (dP's A operand) and feature-major [n][b]
    // (dW1's B operand), so F3 stages both with plain 16-byte copies
    const int BP = (B + CH - 1) / CH * CH;
    const long Q = (long)BP * HID;
    const uint16_t hi = f2bf(dhl), lo = bf16_lo(dhl, hi);
    dhq[(long)b * HID + l] = hi;
    dhq[Q + (long)b * HID + l] = lo;
    dhq[2 * Q + (long)l * BP + b] = hi;
    dhq[3 * Q + (long)l * BP + b] = lo;
    rec[(long)(650 + l) * B + b] = dhl;  // db1 contribution
  }
  // dW2[k][c] = h_k dz_c   (column-major records: rec[col][row])
  for (int i = tid; i < HID * NCLS; i += 256) {
    const int k = i / NCLS, cc = i - k * NCLS;
    float d = 0.f;
#pragma unroll
    for (int q = 0; q < NCLS; ++q) d = (q == cc) ? dz[q] : d;
    rec[(long)i * B + b] = hs[k] * d;
  }
  if (tid < NCLS) {
    float d = 0.f;
#pragma unroll
    for (int q = 0; q < NCLS; ++q) d = (q == tid) ? dz[q] : d;
    rec[(long)(640 + tid) * B + b] = d;
  }
  if (tid == 0) {
    rec[(long)714 * B + b] = valid ? (lse - zy) : 0.f;
    rec[(long)715 * B + b] = (valid && am == y) ? 1.f : 0.f;
  }
  stamp(sts, st, 2);
  stamp_flush(sts, st, 3);
}

// =================================================================================
// F3
// =================================================================================
// aux element e: [0,714) b1/W2/b2 (P index OFF_B1 + e), [714,717) metric tail.
__device__ __forceinline__ int aux_rec_col(int j) {  // record column of small param j
  if (j < HID) return 650 + j;                 // db1
  if (j < HID + HID * NCLS) return j - HID;    // dW2
  return 640 + (j - HID - HID * NCLS);         // db2
}

// sum of rc[r] for r = q, q + stride, ... < n with 8 independent loads in flight.
__device__ __forceinline__ float rec_sum(const float* __restrict__ rc, int q, int stride, int n) {
  float a = 0.f;
  for (int r0 = q; r0 < n; r0 += 8 * stride) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = rc[min(r0 + j * stride, n - 1)];
      t[j] = (r0 + j * stride < n) ? v : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) a += t[j];
  }
  return a;
}

template <bool U8>
__global__ __launch_bounds__(512) void f3_backward(
    const void* __restrict__ X, float* __restrict__ P, float* __restrict__ G, float* __restrict__ V,
    const uint16_t* __restrict__ w1bf, Ctrl* __restrict__ ctrl, const uint16_t* __restrict__ pooled,
    const uint8_t* __restrict__ code, const uint16_t* __restrict__ dhq, const float* __restrict__ rec, int B, int PP,
    unsigned long long* st) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Stamps sts;
  stamp(sts, st, 0);
  const int s = blockIdx.x, tid = threadIdx.x, NS = gridDim.x;
  const int p0 = s * PP, p1 = min(NPOS, p0 + PP), np = p1 - p0, K = np * 32;
  const int KD = PP * 32 + 4;   // dps pitch (f32)
  const int KC = PP * 32;       // code pitch (bytes)
  float* xs = reinterpret_cast<float*>(smem);                              // [CH][XR][28]
  float* dps = reinterpret_cast<float*>(smem + XS_BYTES);                  // [CH][KD]
  uint16_t* pt = reinterpret_cast<uint16_t*>(dps + CH * KD);               // [PP*32][HP]
  uint16_t* dht = pt + PP * 32 * HP;                                       // [2][HID][HP] hi, lo
  uint16_t* dhs = dht + 2 * HID * HP;                                      // [2][CH][HP]  hi, lo
  uint16_t* w1s = dhs + 2 * CH * HP;                                       // [PP*32][HP]
  uint8_t* cs = reinterpret_cast<uint8_t*>(w1s + PP * 32 * HP);            // [CH][KC] argmax codes
  float* red = reinterpret_cast<float*>(pt);  // [16][320] reduction scratch, after the MFMAs
  const Ctrl c = *ctrl;
  if (s == 0 && tid == 0) {
    ctrl->cursor = next_cursor(c, c.cur3);
    ctrl->iterations = c.iterations + 1;
    ctrl->wpar = c.wpar ^ 1;  // F1 of this step wrote the next W1 buffer
  }
  const long gstart = (long)c.cur3 * c.global_batch;
  const long row_base = gstart + c.row0;
  const int r0 = 2 * (p0 / PO);
  const int nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  const int wave = tid >> 6, lane = tid & 63;
  const int ko = 8 * (lane >> 4), lr16 = lane & 15;

  // ---- aux work of this block (loads issued now, consumed at the end) ----
  const int chunk_aux = (NAUX + NS - 1) / NS;
  const int tpe = max(1, min(512 / chunk_aux, 64));  // threads per aux element
  const int ae_local = tid / tpe, aq = tid - ae_local * tpe;
  const int ae = s * chunk_aux + ae_local;
  const bool aux_on = ae_local < chunk_aux && ae < NAUX;
  const int aec = min(ae, NAUX - 1);
  float ap, ag, av, arsum;
  if (aec < NSMALL) {
    ap = P[OFF_B1 + aec]; ag = G[OFF_B1 + aec]; av = V[OFF_B1 + aec];
    arsum = rec_sum(rec + (long)aux_rec_col(aec) * B, aq, tpe, B);
  } else {
    const int m = aec - NSMALL;  // 0 loss, 1 correct, 2 count
    ap = 0.f; av = 0.f;
    ag = G[OFF_LOSS + m];
    arsum = rec_sum(rec + (long)(714 + min(m, 1)) * B, aq, tpe, B);
  }

  // ---- prologue loads: W1 slice, dh, pooled slice, code slice, input rows ----
  // W1 slice of this step (bf16 copy written by F1's owner block) for dP
  const int n8 = K * HID / 8;  // uint4 of 8 bf16
  uint4 wv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
    wv[u] = reinterpret_cast<const uint4*>(w1bf + p0 * 32 * HID)[min(tid + u * 512, n8 - 1)];
  XStage<U8> xst;
  // named registers, not arrays: arrays captured by the lambdas below end up in scratch
  uint4 dq0, dq1, dq2, dq3;  // dh hi/lo [b][n] rows, dh hi/lo [n][b] rows
  uint4 pv0, pv1;            // pooled [k][b] rows of the slice
  uint4 cv;
  const int BP = (B + CH - 1) / CH * CH;
  const long Q = (long)BP * HID;
  const int kc = K / 16;  // uint4 of code bytes per image
  auto load_chunk = [&](int chunk) __attribute__((always_inline)) {
    {
      const int r = tid >> 3, q = tid & 7;  // 64 rows x 8 uint4
      const long rowo = (long)(chunk * CH + r) * HID + q * 8, colo = (long)r * BP + chunk * CH + q * 8;
      dq0 = *reinterpret_cast<const uint4*>(dhq + rowo);
      dq1 = *reinterpret_cast<const uint4*>(dhq + Q + rowo);
      dq2 = *reinterpret_cast<const uint4*>(dhq + 2 * Q + colo);
      dq3 = *reinterpret_cast<const uint4*>(dhq + 3 * Q + colo);
    }
    {
      const int i0 = min(tid, K * 8 - 1), i1 = min(tid + 512, K * 8 - 1);
      pv0 = *reinterpret_cast<const uint4*>(pooled + (long)(p0 * NF + (i0 >> 3)) * BP + chunk * CH + (i0 & 7) * 8);
      pv1 = *reinterpret_cast<const uint4*>(pooled + (long)(p0 * NF + (i1 >> 3)) * BP + chunk * CH + (i1 & 7) * 8);
    }
    {
      const int i = tid, bb = i / kc, q = i - bb * kc, lb = chunk * CH + bb;
      const bool ok = i < CH * kc && lb < B;
      const uint4 v = *reinterpret_cast<const uint4*>(code + (long)min(lb, B - 1) * FEAT + p0 * NF +
                                                      min(q, kc - 1) * 16);
      cv = ok ? v : make_uint4(0u, 0u, 0u, 0u);
    }
    x_load<U8>(xst, X, row_base + chunk * CH, c.nsamples, B - chunk * CH, CH, r0, nrows);
  };
  auto store_chunk = [&]() __attribute__((always_inline)) {
    {
      const int r = tid >> 3, q = tid & 7;
      *reinterpret_cast<uint4*>(dhs + r * HP + q * 8) = dq0;
      *reinterpret_cast<uint4*>(dhs + CH * HP + r * HP + q * 8) = dq1;
      *reinterpret_cast<uint4*>(dht + r * HP + q * 8) = dq2;
      *reinterpret_cast<uint4*>(dht + HID * HP + r * HP + q * 8) = dq3;
    }
    if (tid < K * 8) *reinterpret_cast<uint4*>(pt + (tid >> 3) * HP + (tid & 7) * 8) = pv0;
    if (tid + 512 < K * 8) *reinterpret_cast<uint4*>(pt + ((tid + 512) >> 3) * HP + (tid & 7) * 8) = pv1;
    if (tid < CH * kc) {
      const int bb = tid / kc, q = tid - bb * kc;
      *reinterpret_cast<uint4*>(cs + bb * KC + q * 16) = cv;
    }
    x_store<U8>(xst, xs);
  };
  load_chunk(0);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * 512;
    if (i < n8) *reinterpret_cast<uint4*>(w1s + (i >> 3) * HP + (i & 7) * 8) = wv[u];
  }

  const int dn = wave & 3, dm0 = wave >> 2;
  f32x4 accw[MAXPP];
#pragma unroll
  for (int i = 0; i < MAXPP; ++i) accw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ch = tid & 31, grp = tid >> 5;
  float gw[9], gb = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) gw[t] = 0.f;
  const int nchunks = (B + CH - 1) / CH;

  for (int chunk = 0; chunk < nchunks; ++chunk) {
    if (chunk) {
      lds_barrier();
      load_chunk(chunk);
    }
    store_chunk();
    lds_barrier();
    stamp(sts, st, 1);
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
    stamp(sts, st, 2);
    // MaxPool + ReLU backward fused into the conv weight-gradient accumulation
    // (branch-free: the gradient is masked, the reads always hit staged LDS rows)
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
  stamp(sts, st, 3);
  // ---- dW1 straight into the flat gradient buffer (this block owns these rows) ----
#pragma unroll
  for (int i = 0; i < MAXPP; ++i) {
    if (i >= np) break;
    const int mt = dm0 + 2 * i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * mt + 4 * (lane >> 4) + j;
      G[OFF_W1 + (long)(p0 * 32 + k) * HID + 16 * dn + lr16] = accw[i][j];
    }
  }
  lds_barrier();  // pt/dht region becomes `red`, dps becomes `ared`
#pragma unroll
  for (int t = 0; t < 9; ++t) red[grp * NCONV + t * NF + ch] = gw[t];
  red[grp * NCONV + OFF_BC + ch] = gb;
  float* ared = dps;
  ared[tid] = arsum;
  lds_barrier();
  // this slice's conv-gradient partial -> G[conv] (device-scope fp32 atomics: 320 per
  // block; the summation order over the 43 slices is not fixed, so the conv gradient is
  // reproducible to rounding, not bitwise -- ranks still agree after the all-reduce)
  for (int i = tid; i < NCONV; i += 512) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) a += red[r * NCONV + i];
    atomicAdd(&G[i], a);
  }
  // ---- aux: pending update of b1/W2/b2, their new gradients, metrics ----
  if (aux_on && aq == 0) {
    float tot = 0.f;
    for (int q = 0; q < tpe; ++q) tot += ared[ae_local * tpe + q];
    if (ae < NSMALL) {
      float wn, vn;
      sgd_update(ap, ag, av, c.lr, c.momentum, c.nesterov, wn, vn);
      P[OFF_B1 + ae] = wn;
      if (c.momentum != 0.f) V[OFF_B1 + ae] = vn;
      G[OFF_B1 + ae] = tot;  // new gradient (the old one was consumed above)
    } else {
      const int m = ae - NSMALL;
      float* accp = m == 0 ? &ctrl->acc_loss : (m == 1 ? &ctrl->acc_correct : &ctrl->acc_count);
      const float old = m == 0 ? c.acc_loss : (m == 1 ? c.acc_correct : c.acc_count);
      *accp = old + ag;  // fold the previous step's all-reduced metric into the epoch total
      const int gcount = (int)min((long)c.global_batch, (long)c.nsamples - gstart);
      G[OFF_LOSS + m] = m < 2 ? tot : (float)max(0, min(B, gcount - c.row0));
    }
  }
  stamp(sts, st, 4);
  stamp_flush(sts, st, 5);
}

// =================================================================================
// flush: apply the pending (deferred) update to every parameter, zero the gradient
// buffers and fold the pending metrics into the epoch accumulators.
// =================================================================================
__global__ __launch_bounds__(256) void flush_pending(float* __restrict__ P, float* __restrict__ G,
                                                     float* __restrict__ V, const float* __restrict__ W1alt,
                                                     const float* __restrict__ V1alt, Ctrl* __restrict__ ctrl) {
  const Ctrl c = *ctrl;
  const bool mom = c.momentum != 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < NPARAM; i += gridDim.x * blockDim.x) {
    const bool alt = c.wpar && i >= OFF_W1 && i < OFF_B1;  // current W1 lives in the alternate
    const float w = alt ? W1alt[i - OFF_W1] : P[i], v = alt ? V1alt[i - OFF_W1] : V[i];
    float wn, vn;
    sgd_update(w, G[i], v, c.lr, c.momentum, c.nesterov, wn, vn);
    P[i] = wn;
    if (mom) V[i] = vn;
    G[i] = 0.f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctrl->acc_loss = c.acc_loss + G[OFF_LOSS];
    ctrl->acc_correct = c.acc_correct + G[OFF_CORR];
    ctrl->acc_count = c.acc_count + G[OFF_CNT];
    for (int i = NPARAM; i < NGRAD; ++i) G[i] = 0.f;
  }
  // W1 is back inside P: the last block to arrive clears wpar, so the flush is one launch
  // instead of a follow-up fix-up kernel.  Every block's threads consumed their load of
  // ctrl (the loop above used c.wpar) before the barrier, so the ticket needs no fence --
  // an agent-scope fence per block (an L2 write-back on the multi-XCD part) made this
  // launch 13.8 us instead of ~5.
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(&ctrl->flush_ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        (int)gridDim.x - 1) {
      ctrl->wpar = 0;
      ctrl->flush_ticket = 0;
    }
  }
}

}  // namespace convnet

// ---------------------------------------------------------------------------------
// Host-side launchers (no allocation / sync: capturable into a hipGraph).
// ---------------------------------------------------------------------------------
int convnet_num_slices(int PP) { return (convnet::NPOS + PP - 1) / PP; }
size_t convnet_grad_count(int) { return (size_t)convnet::NGRAD; }

// F1 images per block = 2^lg: 16 up to B = 256 (more blocks, shorter per-block chains),
// 64 beyond (bounded replication of the W1-slice / conv-partial loads)
int convnet_f1_lg(int B) { return B <= 256 ? 4 : 6; }
size_t convnet_f1_lds(int PP, int lg) {
  using namespace convnet;
  const int KP = kpitch(PP), IB = 1 << lg;
  return (size_t)IB * XR * IMG * 4 + (size_t)(IB + HID) * KP * 2 + NCONV * 4;
}
size_t convnet_f3_lds(int PP) {
  using namespace convnet;
  const int KD = PP * 32 + 4;
  return XS_BYTES + (size_t)CH * KD * 4 + (size_t)PP * 32 * HP * 2 * 2 + (size_t)2 * (HID + CH) * HP * 2 +
         (size_t)CH * PP * 32 + 16;
}

template <bool U8>
static void launch_step_impl(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  using namespace convnet;
  const int NS = convnet_num_slices(PP);
  const int lg = convnet_f1_lg(B);
  const dim3 g1(NS, (B + (1 << lg) - 1) >> lg);
  if (b.fuse_head) {
    hipLaunchKernelGGL((f1_forward<U8, true>), g1, dim3(512), convnet_f1_lds(PP, lg), st, b.X, b.P, b.G, b.V,
                       b.W1alt, b.V1alt, b.w1bf, b.ctrl, b.pooled, b.code, b.slabs, b.labels, b.dhq, b.hpart, B, PP,
                       lg, b.stamps);
  } else {
    hipLaunchKernelGGL((f1_forward<U8, false>), g1, dim3(512), convnet_f1_lds(PP, lg), st, b.X, b.P, b.G, b.V,
                       b.W1alt, b.V1alt, b.w1bf, b.ctrl, b.pooled, b.code, b.slabs, b.labels, b.dhq, b.hpart, B, PP,
                       lg, b.stamps);
    hipLaunchKernelGGL(f2_head, dim3(B), dim3(256), 0, st, b.labels, b.P, b.G, b.V, b.ctrl, b.slabs, b.dhq,
                       b.hpart, B, NS, b.stamps ? b.stamps + 256 * 16 : nullptr);
  }
  hipLaunchKernelGGL(f3_backward<U8>, dim3(NS), dim3(512), convnet_f3_lds(PP), st, b.X, b.P, b.G, b.V, b.w1bf,
                     b.ctrl, b.pooled, b.code, b.dhq, b.hpart, B, PP, b.stamps ? b.stamps + 2 * 256 * 16 : nullptr);
}

hipError_t convnet_launch_step(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  if (b.x_u8) launch_step_impl<true>(b, B, PP, st);
  else launch_step_impl<false>(b, B, PP, st);
  return hipGetLastError();
}

hipError_t convnet_launch_flush(const ConvNetBuffers& b, int PP, hipStream_t st) {
  hipLaunchKernelGGL(convnet::flush_pending, dim3(340), dim3(256), 0, st, b.P, b.G, b.V, b.W1alt, b.V1alt, b.ctrl);
  return hipGetLastError();
}

hipError_t convnet_set_lds_limits() {
  const void* fns[6] = {(const void*)convnet::f3_backward<false>, (const void*)convnet::f3_backward<true>,
                        (const void*)convnet::f1_forward<false, false>, (const void*)convnet::f1_forward<true, false>,
                        (const void*)convnet::f1_forward<false, true>, (const void*)convnet::f1_forward<true, true>};
  for (const void* f : fns) {
    // the head variants hold a little static LDS (labels, ticket flags): the dynamic
    // limit is what is left of the CU's 160 KB
    hipFuncAttributes at;
    hipError_t e = hipFuncGetAttributes(&at, f);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024 - (int)at.sharedSizeBytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace damd
