// Non-GEMM layer kernels of the generic path: BatchNorm (train fwd/bwd, fused residual
// add + ReLU), max / global-average pooling, ReLU backward, sparse softmax
// cross-entropy (+accuracy), column sums (bias grads) and the flat multi-tensor SGD
// that also refreshes the bf16 weight shadow read by the MFMA GEMMs.
//
// Layout: NHWC bf16 activations, channel count C % 8 == 0, so every thread moves one
// 16-byte vector of 8 channels (global_load_dwordx4) and keeps the 8 per-channel
// parameters in registers.  Statistics are reduced in fp32 per block (LDS), then across
// blocks in double by a finalize kernel (deterministic, no atomics on the hot reductions).
#include <cstdlib>

#include "bn_fin.h"
#include "damd_common.h"
#include "layer_ops.h"

namespace damd {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return uint4{w[0], w[1], w[2], w[3]};
}
__device__ __forceinline__ void ld8f(const float* p, float* f) {
  float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

inline int grid_for(long work, int per_block = NT, int cap = 8192) {
  long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ---- BatchNorm -------------------------------------------------------------------------
// relu(BN(x)) rounded to bf16 exactly as bn_apply stores it: ReLU masks recomputed from
// the BN input (relu_mask == 2 below, the stem kernels) equal those of the stored output.
__device__ __forceinline__ void bn_relu8(const float* x, const float* sc, const float* sh, float* y) {
#pragma unroll
  for (int e = 0; e < 8; ++e) y[e] = bf2f(f2bf(fmaxf(fmaf(x[e], sc[e], sh[e]), 0.f)));
}
// Sum the partials [T][2][C] over T in fp64 for the 8 channels c0..c0+7 of this block
// (FT = 1024 threads).  Thread t owns value v = t % 16 of the 16-value record (8 sums, 8
// second statistics) and rows t / 16 + 64 k: 64 row slices with up to 16 loads each in
// flight, so the ResNet-18 partial counts (T = 784..1024; 3136 at the stem) take one
// batch of loads (four with the 256-thread version: ~1 us of latency each), then a
// three-level LDS tree (64 -> 16 -> 1 slices, fixed order: deterministic).
// On return sums[j] (j < 8) is the channel sum, sums[8 + j] the second statistic.
constexpr int FT = 1024, FSL = FT / 16;
__device__ __forceinline__ void reduce_partials8(const float* __restrict__ part, int T, int C, int c0,
                                                 double* sums) {
  __shared__ double red[FSL][17];
  __shared__ double red2[16][17];
  const int t = threadIdx.x, v = t & 15, sl = t >> 4;
  const float* p = part + (v < 8 ? c0 + v : C + c0 + (v - 8));
  const size_t row = (size_t)2 * C;
  double a = 0.0;
  for (int i0 = sl; i0 < T; i0 += FSL * 16) {
    float f[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = i0 + FSL * u;
      f[u] = p[(size_t)min(i, T - 1) * row];
      f[u] = i < T ? f[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) a += (double)f[u];
  }
  red[sl][v] = a;
  __syncthreads();
  if (t < 256) {
    const int g = t >> 4;
    double b = 0.0;
#pragma unroll
    for (int q = 0; q < FSL / 16; ++q) b += red[g * (FSL / 16) + q][v];
    red2[g][v] = b;
  }
  __syncthreads();
  if (t < 16) {
    double s2 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) s2 += red2[q][t];
    sums[t] = s2;
  }
  __syncthreads();
}

// ---- in-consumer finalize (BNFin / BNBwdFin, layer_ops.h) ----------------------------
// Every block derives the per-channel coefficients of all C channels from the fp64
// accumulators into LDS (s: [4][C] for the forward, [3][C] for the backward); block 0 also
// publishes them (st / co), updates the moving statistics and adds dgamma / dbeta.  The
// returned pointer replaces st / co in the kernel body (global when acc is null).
// backward coefficients of channel c: dx = a dz + b + cc xhat; pub: co, dgamma, dbeta
__device__ __forceinline__ void bn_bwd_fin_sums(const BNBwdFin& f, int C, int c, double s, double q,
                                                const float* st, bool pub, float& a, float& b, float& cc) {
  const float db = (float)s, dg = (float)q;
  a = st[2 * C + c];
  b = -a * db / f.count;
  cc = -a * dg / f.count;
  if (pub) {
    if (f.dbeta) f.dbeta[c] += db;
    if (f.dgamma) f.dgamma[c] += dg;
    f.co[c] = a;
    f.co[C + c] = b;
    f.co[2 * C + c] = cc;
  }
}
__device__ __forceinline__ const float* bn_fin_prologue(const BNFin& f, int C, float* s, const float* st) {
  if (f.acc == nullptr) return st;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double a, b;
    acc_sums(f.acc, f.reps, C, c, a, b);
    bn_fin_sums(f, C, c, a, b, blockIdx.x == 0, s[c], s[C + c], s[2 * C + c], s[3 * C + c]);
  }
  __syncthreads();
  return s;
}
__device__ __forceinline__ const float* bn_bwd_fin_prologue(const BNBwdFin& f, int C, const float* st, float* s,
                                                            const float* co) {
  if (f.acc == nullptr) return co;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double a, b;
    acc_sums2(f.acc, f.reps, C, c, a, b);
    bn_bwd_fin_sums(f, C, c, a, b, st, blockIdx.x == 0, s[c], s[C + c], s[2 * C + c]);
  }
  __syncthreads();
  return s;
}
// per-block (fp32, fixed order) partial of channel ch -> replica blockIdx.x % reps of the
// accumulator (order-independent fixed point), or the partials row of this block
__device__ __forceinline__ void put_partial(float* part, long long* acc, int reps, int C, int ch, float a, float b) {
  if (acc) {
    long long* r = acc + (size_t)(blockIdx.x % reps) * 4 * C;  // (backward sums: hi / lo planes)
    long long* flag = acc + (size_t)max(reps, 1) * 4 * C + ch;   // sticky plane
    bnacc_add2(r + ch, r + C + ch, flag, a);
    bnacc_add2(r + 2 * C + ch, r + 3 * C + ch, flag, b);
  } else {
    part[(size_t)blockIdx.x * 2 * C + ch] = a;
    part[(size_t)blockIdx.x * 2 * C + C + ch] = b;
  }
}

__global__ __launch_bounds__(FT) void bn_finalize_k(const float* part, int T, int C, float count,
                                                    const float* gamma, const float* beta, float eps, float mom,
                                                    float* rmean, float* rvar, float* st) {
  __shared__ double sums[16];
  const int c0 = blockIdx.x * 8;
  reduce_partials8(part, T, C, c0, sums);
  if (threadIdx.x >= 8) return;
  const int c = c0 + threadIdx.x;
  const double mean = sums[threadIdx.x] / count;
  double var = fma(-mean, mean, sums[8 + threadIdx.x] / count);  // (explicit fmas: as bn_fin.h)
  if (var < 0.0) var = 0.0;
  const float m = (float)mean, v = (float)var;
  const float inv = rsqrtf(v + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  const float sc = g * inv;
  st[c] = m;
  st[C + c] = inv;
  st[2 * C + c] = sc;
  st[3 * C + c] = fmaf(-m, sc, b);
  if (rmean) {
    rmean[c] = fmaf(rmean[c], mom, m * (1.f - mom));
    rvar[c] = fmaf(rvar[c], mom, v * (1.f - mom));
  }
}

__global__ __launch_bounds__(NT) void bn_apply_k(const uint16_t* __restrict__ x, const float* st_in,
                                                 const uint16_t* __restrict__ r, const float* st2_in,
                                                 int res_mode, int relu, uint16_t* __restrict__ y, long n8, int C,
                                                 BNFin f1, BNFin f2) {
  extern __shared__ float sfin[];  // [4][C] (f1), then [4][C] (f2)
  const float* st = bn_fin_prologue(f1, C, sfin, st_in);
  const float* st2 = res_mode == 2 ? bn_fin_prologue(f2, C, sfin + 4 * C, st2_in) : st2_in;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    const int c = (int)((i * 8) % C);
    float xv[8], sc[8], sh[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], xv);
    ld8f(st + 2 * C + c, sc);
    ld8f(st + 3 * C + c, sh);
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = fmaf(xv[e], sc[e], sh[e]);
    if (res_mode) {
      float rv[8];
      unpack8(reinterpret_cast<const uint4*>(r)[i], rv);
      if (res_mode == 2) {
        float sc2[8], sh2[8];
        ld8f(st2 + 2 * C + c, sc2);
        ld8f(st2 + 3 * C + c, sh2);
#pragma unroll
        for (int e = 0; e < 8; ++e) rv[e] = rv[e] * sc2[e] + sh2[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] += rv[e];
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = fmaxf(xv[e], 0.f);
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(xv);
  }
}

// Row-mapped apply kernels: thread t keeps channel group t % (C/8) for the whole launch,
// so its per-channel coefficients are loaded once into registers instead of once per
// 16-byte data vector (the flat kernels above fetched 2-7 coefficient vectors per data
// vector); BN_UNR rows per thread in flight.  Same arithmetic, bitwise equal output.
// Measured on ResNet-18: backward apply 9.9 -> 8.8 us per launch, forward apply unchanged
// (already at HBM rate); the same unrolling of bn_bwd_reduce_k's row loop was slower
// (8.6 -> 9.5 us) and is not used.  With the in-consumer finalize (BNFin / BNBwdFin) the
// first batch of rows is requested before the prologue, so the data fetch overlaps the
// accumulator read and the fp64 finalize instead of queueing behind them.
constexpr int BN_UNR = 4;
__global__ __launch_bounds__(NT) void bn_apply_rows_k(const uint16_t* __restrict__ x, const float* st,
                                                      const uint16_t* __restrict__ r, const float* st2,
                                                      int res_mode, int relu, uint16_t* __restrict__ y, long M, int C,
                                                      BNFin f1, BNFin f2) {
  extern __shared__ float sfin[];  // in-consumer finalize: [4][C] (f1), then [4][C] (f2)
  const int cg = C / 8, t = threadIdx.x, rpi = NT / cg;  // launcher: NT % cg == 0
  const int g = t % cg, rr = t / cg, c = g * 8;
  const long stride = (long)gridDim.x * rpi;
  const uint4* x4 = reinterpret_cast<const uint4*>(x);
  const uint4* r4 = reinterpret_cast<const uint4*>(r);
  uint4* y4 = reinterpret_cast<uint4*>(y);
  uint4 xq[BN_UNR], rq[BN_UNR];
  auto load = [&](long row0) {
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      const long row = min(row0 + u * stride, M - 1);
      xq[u] = x4[row * cg + g];
      if (res_mode) rq[u] = r4[row * cg + g];
    }
  };
  long row0 = (long)blockIdx.x * rpi + rr;
  load(row0);
  st = bn_fin_prologue(f1, C, sfin, st);
  if (res_mode == 2) st2 = bn_fin_prologue(f2, C, sfin + 4 * C, st2);
  float sc[8], sh[8], sc2[8], sh2[8];
  ld8f(st + 2 * C + c, sc);
  ld8f(st + 3 * C + c, sh);
  if (res_mode == 2) {
    ld8f(st2 + 2 * C + c, sc2);
    ld8f(st2 + 3 * C + c, sh2);
  }
  for (bool first = true; row0 < M; row0 += stride * BN_UNR, first = false) {
    if (!first) load(row0);
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      const long row = row0 + u * stride;
      if (row >= M) break;
      float xv[8];
      unpack8(xq[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = fmaf(xv[e], sc[e], sh[e]);
      if (res_mode) {
        float rv[8];
        unpack8(rq[u], rv);
        if (res_mode == 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) rv[e] = rv[e] * sc2[e] + sh2[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] += rv[e];
      }
      if (relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = fmaxf(xv[e], 0.f);
      }
      y4[row * cg + g] = pack8(xv);
    }
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_apply_rows_k(const uint16_t* __restrict__ dy,
                                                          const uint16_t* __restrict__ y, int relu_mask,
                                                          const uint16_t* __restrict__ x, const float* __restrict__ st,
                                                          const float* co, uint16_t* __restrict__ dx,
                                                          long M, int C, BNBwdFin bf) {
  extern __shared__ float sfin[];  // in-consumer finalize: [3][C]
  const int cg = C / 8, t = threadIdx.x, rpi = NT / cg;  // launcher: NT % cg == 0
  const int g = t % cg, rr = t / cg, c = g * 8;
  const long stride = (long)gridDim.x * rpi;
  const uint4* d4 = reinterpret_cast<const uint4*>(dy);
  const uint4* x4 = reinterpret_cast<const uint4*>(x);
  const uint4* y4 = reinterpret_cast<const uint4*>(y);
  uint4* o4 = reinterpret_cast<uint4*>(dx);
  uint4 dq[BN_UNR], xq[BN_UNR], yq[BN_UNR];
  auto load = [&](long row0) {
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      const long row = min(row0 + u * stride, M - 1);
      dq[u] = d4[row * cg + g];
      xq[u] = x4[row * cg + g];
      if (relu_mask == 1) yq[u] = y4[row * cg + g];
    }
  };
  long row0 = (long)blockIdx.x * rpi + rr;
  load(row0);
  co = bn_bwd_fin_prologue(bf, C, st, sfin, co);
  float mean[8], inv[8], a[8], b[8], cc[8], sc[8], sh[8];
  ld8f(st + c, mean);
  ld8f(st + C + c, inv);
  ld8f(co + c, a);
  ld8f(co + C + c, b);
  ld8f(co + 2 * C + c, cc);
  if (relu_mask == 2) {
    ld8f(st + 2 * C + c, sc);
    ld8f(st + 3 * C + c, sh);
  }
  for (bool first = true; row0 < M; row0 += stride * BN_UNR, first = false) {
    if (!first) load(row0);
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      const long row = row0 + u * stride;
      if (row >= M) break;
      float d[8], xv[8];
      unpack8(dq[u], d);
      unpack8(xq[u], xv);
      if (relu_mask) {
        float yv[8];
        if (relu_mask == 2)
          bn_relu8(xv, sc, sh, yv);
        else
          unpack8(yq[u], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = a[e] * d[e] + b[e] + cc[e] * (xv[e] - mean[e]) * inv[e];
      o4[row * cg + g] = pack8(d);
    }
  }
}

// dz = dy * [y>0]; partial sums of dz and dz*xhat per channel for a contiguous row range.
// MODE = relu_mask (0 none, 1 mask from the stored y, 2 recomputed from x): a template
// argument, so the loads of RU rows (dy, x, y) are issued together before the first use --
// with the mask source behind a runtime branch and the dz stores (which may alias the next
// rows' loads) between rows, every row cost its own two memory round trips.  Rows are
// still accumulated in ascending order: the partials are bitwise those of the row loop.
constexpr int RED_RU = 4;
template <int MODE>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_k(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                      const uint16_t* __restrict__ x,
                                                      const float* __restrict__ st, uint16_t* __restrict__ dz_out,
                                                      float* __restrict__ part, long M, int C, long rows_per_block,
                                                      long long* __restrict__ acc, int reps, int rev) {
  __shared__ float red[2][NT * 8];
  const int cg = C / 8, t = threadIdx.x;
  const int rpi = NT / cg;  // rows per iteration
  const int g = t % cg, rr = t / cg;
  const int c = g * 8;
  // rev (tests, bn_reduce_reverse): block b reduces the rows of block G-1-b -- the same
  // partials, produced in a different order and added into different replicas
  const long blk = rev ? (long)gridDim.x - 1 - blockIdx.x : blockIdx.x;
  float s0[8], s1[8], mean[8], inv[8], sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s0[e] = s1[e] = 0.f;
  ld8f(st + c, mean);
  ld8f(st + C + c, inv);
  if (MODE == 2) {
    ld8f(st + 2 * C + c, sc);
    ld8f(st + 3 * C + c, sh);
  }
  const long r0 = blk * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rr < rpi) {
    for (long row = r0 + rr; row < r1; row += (long)RED_RU * rpi) {
      uint4 dq[RED_RU], xq[RED_RU], yq[RED_RU];
#pragma unroll
      for (int u = 0; u < RED_RU; ++u) {
        const long off = (min(row + u * rpi, r1 - 1) * C + c) / 8;
        dq[u] = reinterpret_cast<const uint4*>(dy)[off];
        xq[u] = reinterpret_cast<const uint4*>(x)[off];
        if (MODE == 1) yq[u] = reinterpret_cast<const uint4*>(y)[off];
      }
#pragma unroll
      for (int u = 0; u < RED_RU; ++u) {
        const long rw = row + u * rpi;
        if (rw >= r1) break;
        const long off = (rw * C + c) / 8;
        float d[8], xv[8];
        unpack8(dq[u], d);
        unpack8(xq[u], xv);
        if (MODE) {
          float yv[8];
          if (MODE == 2)
            bn_relu8(xv, sc, sh, yv);
          else
            unpack8(yq[u], yv);
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
          if (dz_out) reinterpret_cast<uint4*>(dz_out)[off] = pack8(d);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s0[e] += d[e];
          s1[e] += d[e] * (xv[e] - mean[e]) * inv[e];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][t * 8 + e] = rr < rpi ? s0[e] : 0.f;
    red[1][t * 8 + e] = rr < rpi ? s1[e] : 0.f;
  }
  __syncthreads();
  // thread t < C sums channel t over the rpi row groups: element (rr*cg + g)*8 + e, c = 8g+e
  for (int ch = t; ch < C; ch += NT) {
    const int gg = ch / 8, e = ch % 8;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < rpi; ++q) {
      a += red[0][(q * cg + gg) * 8 + e];
      b += red[1][(q * cg + gg) * 8 + e];
    }
    put_partial(part, acc, reps, C, ch, a, b);
  }
}

// Two BatchNorms fed by the same masked gradient (a ResNet downsampling block's output
// relu(BN2(x2) + BNd(xd))): ONE pass over dy and the mask source y for both -- per
// channel sum dz (shared), sum dz * xhat2, sum dz * xhatd -- each BN's partials into its own
// accumulator.  The row ranges, the per-thread order and the LDS tree are those of
// bn_bwd_reduce_k, so each accumulator receives bitwise the partials the single-BN launch
// would add (relu_mask 0 / 1 only; fixed-point accumulators only).
__global__ __launch_bounds__(NT) void bn_bwd_reduce2_k(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                       int relu_mask, const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ x2, const float* __restrict__ st,
                                                       const float* __restrict__ st2, long M, int C,
                                                       long rows_per_block, long long* __restrict__ acc,
                                                       long long* __restrict__ acc2, int reps) {
  __shared__ float red[3][NT * 8];
  const int cg = C / 8, t = threadIdx.x;
  const int rpi = NT / cg;
  const int g = t % cg, rr = t / cg;
  const int c = g * 8;
  const long blk = blockIdx.x;
  float s0[8], s1[8], s2[8], mean[8], inv[8], mean2[8], inv2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s0[e] = s1[e] = s2[e] = 0.f;
  ld8f(st + c, mean);
  ld8f(st + C + c, inv);
  ld8f(st2 + c, mean2);
  ld8f(st2 + C + c, inv2);
  const long r0 = blk * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rr < rpi) {
    for (long row = r0 + rr; row < r1; row += rpi) {
      const long off = (row * C + c) / 8;
      float d[8], xv[8], xw[8];
      unpack8(reinterpret_cast<const uint4*>(dy)[off], d);
      unpack8(reinterpret_cast<const uint4*>(x)[off], xv);
      unpack8(reinterpret_cast<const uint4*>(x2)[off], xw);
      if (relu_mask) {
        float yv[8];
        unpack8(reinterpret_cast<const uint4*>(y)[off], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s0[e] += d[e];
        s1[e] += d[e] * (xv[e] - mean[e]) * inv[e];
        s2[e] += d[e] * (xw[e] - mean2[e]) * inv2[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][t * 8 + e] = rr < rpi ? s0[e] : 0.f;
    red[1][t * 8 + e] = rr < rpi ? s1[e] : 0.f;
    red[2][t * 8 + e] = rr < rpi ? s2[e] : 0.f;
  }
  __syncthreads();
  for (int ch = t; ch < C; ch += NT) {
    const int gg = ch / 8, e = ch % 8;
    float a = 0.f, b = 0.f, b2 = 0.f;
    for (int q = 0; q < rpi; ++q) {
      a += red[0][(q * cg + gg) * 8 + e];
      b += red[1][(q * cg + gg) * 8 + e];
      b2 += red[2][(q * cg + gg) * 8 + e];
    }
    put_partial(nullptr, acc, reps, C, ch, a, b);
    put_partial(nullptr, acc2, reps, C, ch, a, b2);
  }
}

// ... and the matching apply: both BNs' coefficients finalized in the prologue, dx and dx2
// from one read of dy / y (row mapping and arithmetic of bn_bwd_apply_rows_k)
__global__ __launch_bounds__(NT) void bn_bwd_apply2_rows_k(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ y, int relu_mask,
                                                           const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ x2,
                                                           const float* __restrict__ st,
                                                           const float* __restrict__ st2, uint16_t* __restrict__ dx,
                                                           uint16_t* __restrict__ dx2, long M, int C, BNBwdFin bf,
                                                           BNBwdFin bf2) {
  extern __shared__ float sfin[];  // [3][C] (bf), then [3][C] (bf2)
  const int cg = C / 8, t = threadIdx.x, rpi = NT / cg;
  const int g = t % cg, rr = t / cg, c = g * 8;
  const long stride = (long)gridDim.x * rpi;
  const uint4* d4 = reinterpret_cast<const uint4*>(dy);
  const uint4* x4 = reinterpret_cast<const uint4*>(x);
  const uint4* w4 = reinterpret_cast<const uint4*>(x2);
  const uint4* y4 = reinterpret_cast<const uint4*>(y);
  uint4* o4 = reinterpret_cast<uint4*>(dx);
  uint4* p4 = reinterpret_cast<uint4*>(dx2);
  uint4 dq[BN_UNR], xq[BN_UNR], wq[BN_UNR], yq[BN_UNR];
  auto load = [&](long row0) {
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      const long row = min(row0 + u * stride, M - 1);
      dq[u] = d4[row * cg + g];
      xq[u] = x4[row * cg + g];
      wq[u] = w4[row * cg + g];
      if (relu_mask) yq[u] = y4[row * cg + g];
    }
  };
  long row0 = (long)blockIdx.x * rpi + rr;
  load(row0);
  const float* co = bn_bwd_fin_prologue(bf, C, st, sfin, bf.co);
  const float* co2 = bn_bwd_fin_prologue(bf2, C, st2, sfin + 3 * C, bf2.co);
  float mean[8], inv[8], a[8], b[8], cc[8], mean2[8], inv2[8], a2[8], b2[8], cc2[8];
  ld8f(st + c, mean);
  ld8f(st + C + c, inv);
  ld8f(co + c, a);
  ld8f(co + C + c, b);
  ld8f(co + 2 * C + c, cc);
  ld8f(st2 + c, mean2);
  ld8f(st2 + C + c, inv2);
  ld8f(co2 + c, a2);
  ld8f(co2 + C + c, b2);
  ld8f(co2 + 2 * C + c, cc2);
  for (bool first = true; row0 < M; row0 += stride * BN_UNR, first = false) {
    if (!first) load(row0);
#pragma unroll
    for (int u = 0; u < BN_UNR; ++u) {
      const long row = row0 + u * stride;
      if (row >= M) break;
      float d[8], xv[8], xw[8], o[8], p[8];
      unpack8(dq[u], d);
      unpack8(xq[u], xv);
      unpack8(wq[u], xw);
      if (relu_mask) {
        float yv[8];
        unpack8(yq[u], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = a[e] * d[e] + b[e] + cc[e] * (xv[e] - mean[e]) * inv[e];
        p[e] = a2[e] * d[e] + b2[e] + cc2[e] * (xw[e] - mean2[e]) * inv2[e];
      }
      o4[row * cg + g] = pack8(o);
      p4[row * cg + g] = pack8(p);
    }
  }
}

__global__ __launch_bounds__(FT) void bn_bwd_finalize_k(const float* part, int T, int C, float count,
                                                        const float* st, float* dgamma, float* dbeta, float* co) {
  __shared__ double sums[16];
  const int c0 = blockIdx.x * 8;
  reduce_partials8(part, T, C, c0, sums);
  if (threadIdx.x >= 8) return;
  const int c = c0 + threadIdx.x;
  const float db = (float)sums[threadIdx.x], dg = (float)sums[8 + threadIdx.x];
  if (dbeta) dbeta[c] += db;
  if (dgamma) dgamma[c] += dg;
  const float a = st[2 * C + c];
  co[c] = a;
  co[C + c] = -a * db / count;
  co[2 * C + c] = -a * dg / count;
}

__global__ __launch_bounds__(NT) void bn_bwd_apply_k(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                     int relu_mask, const uint16_t* __restrict__ x,
                                                     const float* __restrict__ st, const float* co_in,
                                                     uint16_t* __restrict__ dx, long n8, int C, BNBwdFin bf) {
  extern __shared__ float sfin[];  // [3][C]
  const float* co = bn_bwd_fin_prologue(bf, C, st, sfin, co_in);
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    const int c = (int)((i * 8) % C);
    float d[8], xv[8], mean[8], inv[8], a[8], b[8], cc[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], d);
    unpack8(reinterpret_cast<const uint4*>(x)[i], xv);
    if (relu_mask) {
      float yv[8];
      if (relu_mask == 2) {
        float sc[8], sh[8];
        ld8f(st + 2 * C + c, sc);
        ld8f(st + 3 * C + c, sh);
        bn_relu8(xv, sc, sh, yv);
      } else {
        unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
    }
    ld8f(st + c, mean);
    ld8f(st + C + c, inv);
    ld8f(co + c, a);
    ld8f(co + C + c, b);
    ld8f(co + 2 * C + c, cc);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = a[e] * d[e] + b[e] + cc[e] * (xv[e] - mean[e]) * inv[e];
    reinterpret_cast<uint4*>(dx)[i] = pack8(d);
  }
}

// ---- pooling -----------------------------------------------------------------------------
struct PoolGeo {
  int N, H, W, C, ph, pw, sh, sw, pt, pl, Ho, Wo;
};

__global__ __launch_bounds__(NT) void maxpool_fwd_k(const uint16_t* __restrict__ x, PoolGeo g,
                                                    uint16_t* __restrict__ y, uint8_t* __restrict__ arg) {
  const int cg = g.C / 8;
  const long total = (long)g.N * g.Ho * g.Wo * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    long pix = i / cg;
    const int ow = (int)(pix % g.Wo);
    pix /= g.Wo;
    const int oh = (int)(pix % g.Ho);
    const int n = (int)(pix / g.Ho);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int kh = 0; kh < g.ph; ++kh) {
      const int ih = oh * g.sh - g.pt + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.pw; ++kw) {
        const int iw = ow * g.sw - g.pl + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float v[8];
        unpack8(reinterpret_cast<const uint4*>(x)[(((long)n * g.H + ih) * g.W + iw) * cg + c8], v);
        const uint8_t idx = (uint8_t)(kh * g.pw + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = idx; }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    reinterpret_cast<uint2*>(arg)[i] = a;
  }
}

__global__ __launch_bounds__(NT) void maxpool_bwd_k(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                    PoolGeo g, uint16_t* __restrict__ dx) {
  const int cg = g.C / 8;
  const long total = (long)g.N * g.H * g.W * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    long pix = i / cg;
    const int iw = (int)(pix % g.W);
    pix /= g.W;
    const int ih = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // output rows whose window covers ih: oh*sh - pt <= ih <= oh*sh - pt + ph - 1
    const int ohlo = max(0, (ih + g.pt - g.ph + g.sh) / g.sh), ohhi = min(g.Ho - 1, (ih + g.pt) / g.sh);
    const int owlo = max(0, (iw + g.pl - g.pw + g.sw) / g.sw), owhi = min(g.Wo - 1, (iw + g.pl) / g.sw);
    for (int oh = ohlo; oh <= ohhi; ++oh) {
      const int kh = ih - (oh * g.sh - g.pt);
      if (kh < 0 || kh >= g.ph) continue;
      for (int ow = owlo; ow <= owhi; ++ow) {
        const int kw = iw - (ow * g.sw - g.pl);
        if (kw < 0 || kw >= g.pw) continue;
        const long o = (((long)n * g.Ho + oh) * g.Wo + ow) * cg + c8;
        const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
        const uint8_t me = (uint8_t)(kh * g.pw + kw);
        float d[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], d);
        const uint32_t w[2] = {a.x, a.y};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (((w[e >> 2] >> (8 * (e & 3))) & 0xff) == me) acc[e] += d[e];
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
  }
}

// Average pooling (Keras AveragePooling2D): the divisor is the number of in-bounds taps, so
// 'same' windows that overhang the border average only real pixels (TF's avg_pool) and
// 'valid' windows divide by ph*pw.  The backward is a gather over the output windows that
// cover each input pixel (no atomics, every dx written once).
__device__ __forceinline__ float pool_inv_count(int oh, int ow, const PoolGeo& g) {
  const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
  const int nh = min(h0 + g.ph, g.H) - max(h0, 0), nw = min(w0 + g.pw, g.W) - max(w0, 0);
  return 1.f / (float)(nh * nw);
}

__global__ __launch_bounds__(NT) void avgpool_fwd_k(const uint16_t* __restrict__ x, PoolGeo g,
                                                    uint16_t* __restrict__ y) {
  const int cg = g.C / 8;
  const long total = (long)g.N * g.Ho * g.Wo * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    long pix = i / cg;
    const int ow = (int)(pix % g.Wo);
    pix /= g.Wo;
    const int oh = (int)(pix % g.Ho);
    const int n = (int)(pix / g.Ho);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int kh = 0; kh < g.ph; ++kh) {
      const int ih = oh * g.sh - g.pt + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.pw; ++kw) {
        const int iw = ow * g.sw - g.pl + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float v[8];
        unpack8(reinterpret_cast<const uint4*>(x)[(((long)n * g.H + ih) * g.W + iw) * cg + c8], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    }
    const float inv = pool_inv_count(oh, ow, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    reinterpret_cast<uint4*>(y)[i] = pack8(acc);
  }
}

__global__ __launch_bounds__(NT) void avgpool_bwd_k(const uint16_t* __restrict__ dy, PoolGeo g,
                                                    uint16_t* __restrict__ dx) {
  const int cg = g.C / 8;
  const long total = (long)g.N * g.H * g.W * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    long pix = i / cg;
    const int iw = (int)(pix % g.W);
    pix /= g.W;
    const int ih = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int ohlo = max(0, (ih + g.pt - g.ph + g.sh) / g.sh), ohhi = min(g.Ho - 1, (ih + g.pt) / g.sh);
    const int owlo = max(0, (iw + g.pl - g.pw + g.sw) / g.sw), owhi = min(g.Wo - 1, (iw + g.pl) / g.sw);
    for (int oh = ohlo; oh <= ohhi; ++oh) {
      const int kh = ih - (oh * g.sh - g.pt);
      if (kh < 0 || kh >= g.ph) continue;
      for (int ow = owlo; ow <= owhi; ++ow) {
        const int kw = iw - (ow * g.sw - g.pl);
        if (kw < 0 || kw >= g.pw) continue;
        float d[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[(((long)n * g.Ho + oh) * g.Wo + ow) * cg + c8], d);
        const float inv = pool_inv_count(oh, ow, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += d[e] * inv;
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
  }
}

// ---- stem fusion: BatchNorm -> ReLU -> MaxPool without the normalised tensor ----------
// Forward: the pool reads the conv output x and normalises on the fly (the BN+ReLU output
// is never stored); each candidate is rounded to bf16 exactly as bn_apply stores it, so
// max / argmax equal the unfused pair's.  Backward: the pool's gradient routing and the
// ReLU mask are recomputed from (dy_pool, argmax, x, BN scale/shift) in both BN-backward
// passes, so neither the 4x larger un-pooled gradient nor the ReLU output is stored.

__global__ __launch_bounds__(NT) void bn_relu_maxpool_fwd_k(const uint16_t* __restrict__ x,
                                                            const float* st_in, PoolGeo g,
                                                            uint16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                            BNFin f) {
  extern __shared__ float sfin[];
  const float* st = bn_fin_prologue(f, g.C, sfin, st_in);
  const int cg = g.C / 8;
  const long total = (long)g.N * g.Ho * g.Wo * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    long pix = i / cg;
    const int ow = (int)(pix % g.Wo);
    pix /= g.Wo;
    const int oh = (int)(pix % g.Ho);
    const int n = (int)(pix / g.Ho);
    float sc[8], sh[8];
    ld8f(st + 2 * g.C + c8 * 8, sc);
    ld8f(st + 3 * g.C + c8 * 8, sh);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int kh = 0; kh < g.ph; ++kh) {
      const int ih = oh * g.sh - g.pt + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.pw; ++kw) {
        const int iw = ow * g.sw - g.pl + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float xv[8], v[8];
        unpack8(reinterpret_cast<const uint4*>(x)[(((long)n * g.H + ih) * g.W + iw) * cg + c8], xv);
        bn_relu8(xv, sc, sh, v);
        const uint8_t idx = (uint8_t)(kh * g.pw + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = idx; }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    reinterpret_cast<uint2*>(arg)[i] = a;
  }
}

// 3x3/s2 pool, H = 2 Ho, W = 2 Wo, Ho and Wo even: one thread per 2x2 block of outputs.
// Its 5x5 input patch is walked row by row (5 loads + BN/ReLU each), and every row updates
// the outputs whose windows contain it, taps in ascending (kh, kw) order with the same
// strict '>' as bn_relu_maxpool_fwd_k, so values and argmax codes are bitwise equal; 25
// loads and normalisations per 4 outputs instead of 36.
template <int PT, int PL>
__global__ __launch_bounds__(NT) void bn_relu_maxpool_fwd_q_k(const uint16_t* __restrict__ x,
                                                              const float* st_in, PoolGeo g,
                                                              uint16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                              BNFin f) {
  extern __shared__ float sfin[];
  const float* st = bn_fin_prologue(f, g.C, sfin, st_in);
  const int cg = g.C / 8;
  const int Ho2 = g.Ho / 2, Wo2 = g.Wo / 2;
  const long total = (long)g.N * Ho2 * Wo2 * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    long q = i / cg;
    const int b2 = (int)(q % Wo2);
    q /= Wo2;
    const int a2 = (int)(q % Ho2);
    const int n = (int)(q / Ho2);
    float sc[8], sh[8];
    ld8f(st + 2 * g.C + c8 * 8, sc);
    ld8f(st + 3 * g.C + c8 * 8, sh);
    float best[4][8];
    uint32_t code[4][2];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
#pragma unroll
      for (int e = 0; e < 8; ++e) best[o][e] = -INFINITY;
      code[o][0] = code[o][1] = 0u;
    }
    const int ih0 = 4 * a2 - PT, iw0 = 4 * b2 - PL;
#pragma unroll
    for (int pr = 0; pr < 5; ++pr) {
      const int ih = ih0 + pr;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      float v[5][8];
      bool ok[5];
#pragma unroll
      for (int pc = 0; pc < 5; ++pc) {
        const int iw = iw0 + pc;
        ok[pc] = (unsigned)iw < (unsigned)g.W;
        float xv[8];
        unpack8(reinterpret_cast<const uint4*>(x)[(((long)n * g.H + ih) * g.W + (ok[pc] ? iw : 0)) * cg + c8], xv);
        bn_relu8(xv, sc, sh, v[pc]);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int kh = pr - 2 * r;
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int o = 2 * r + c;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int pc = 2 * c + kw;
            if (!ok[pc]) continue;
            const uint32_t idx = (uint32_t)(kh * 3 + kw);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (v[pc][e] > best[o][e]) {
                best[o][e] = v[pc][e];
                code[o][e >> 2] = (code[o][e >> 2] & ~(0xffu << (8 * (e & 3)))) | (idx << (8 * (e & 3)));
              }
          }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const long oi = (((long)n * g.Ho + 2 * a2 + (o >> 1)) * g.Wo + 2 * b2 + (o & 1)) * cg + c8;
      reinterpret_cast<uint4*>(y)[oi] = pack8(best[o]);
      reinterpret_cast<uint2*>(arg)[oi] = uint2{code[o][0], code[o][1]};
    }
  }
}

// gradient reaching input pixel (n, ih, iw), channels 8*c8.. through the max-pool windows
// (fp32 sum, then rounded to bf16 as maxpool_bwd stores it)
__device__ __forceinline__ void pool_grad8(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                           const PoolGeo& g, int n, int ih, int iw, int c8, float* acc) {
  const int cg = g.C / 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int ohlo = max(0, (ih + g.pt - g.ph + g.sh) / g.sh), ohhi = min(g.Ho - 1, (ih + g.pt) / g.sh);
  const int owlo = max(0, (iw + g.pl - g.pw + g.sw) / g.sw), owhi = min(g.Wo - 1, (iw + g.pl) / g.sw);
  for (int oh = ohlo; oh <= ohhi; ++oh) {
    const int kh = ih - (oh * g.sh - g.pt);
    if (kh < 0 || kh >= g.ph) continue;
    for (int ow = owlo; ow <= owhi; ++ow) {
      const int kw = iw - (ow * g.sw - g.pl);
      if (kw < 0 || kw >= g.pw) continue;
      const long o = (((long)n * g.Ho + oh) * g.Wo + ow) * cg + c8;
      const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
      const uint8_t me = (uint8_t)(kh * g.pw + kw);
      float d[8];
      unpack8(reinterpret_cast<const uint4*>(dy)[o], d);
      const uint32_t w[2] = {a.x, a.y};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (((w[e >> 2] >> (8 * (e & 3))) & 0xff) == me) acc[e] += d[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = bf2f(f2bf(acc[e]));
}

// masked upstream gradient of the BN output at input row `row` (flattened n, ih, iw)
__device__ __forceinline__ void stem_dy8(const uint16_t* __restrict__ dpool, const uint8_t* __restrict__ arg,
                                         const PoolGeo& g, long row, int c8, const float* xv, const float* sc,
                                         const float* sh, float* d) {
  const int iw = (int)(row % g.W);
  const long t = row / g.W;
  const int ih = (int)(t % g.H), n = (int)(t / g.H);
  pool_grad8(dpool, arg, g, n, ih, iw, c8, d);
  float yv[8];
  bn_relu8(xv, sc, sh, yv);
#pragma unroll
  for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
}

__global__ __launch_bounds__(NT) void pool_bn_bwd_reduce_k(const uint16_t* __restrict__ dpool,
                                                           const uint8_t* __restrict__ arg, PoolGeo g,
                                                           const uint16_t* __restrict__ x, const float* __restrict__ st,
                                                           float* __restrict__ part, long M, long rows_per_block,
                                                           long long* __restrict__ acc, int reps) {
  __shared__ float red[2][NT * 8];
  const int C = g.C, cg = C / 8, t = threadIdx.x;
  const int rpi = NT / cg;
  const int gq = t % cg, rr = t / cg;
  const int c = gq * 8;
  float s0[8], s1[8], mean[8], inv[8], sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s0[e] = s1[e] = 0.f;
  ld8f(st + c, mean);
  ld8f(st + C + c, inv);
  ld8f(st + 2 * C + c, sc);
  ld8f(st + 3 * C + c, sh);
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rr < rpi) {
    for (long row = r0 + rr; row < r1; row += rpi) {
      float xv[8], d[8];
      unpack8(reinterpret_cast<const uint4*>(x)[(row * C + c) / 8], xv);
      stem_dy8(dpool, arg, g, row, gq, xv, sc, sh, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s0[e] += d[e];
        s1[e] += d[e] * (xv[e] - mean[e]) * inv[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][t * 8 + e] = rr < rpi ? s0[e] : 0.f;
    red[1][t * 8 + e] = rr < rpi ? s1[e] : 0.f;
  }
  __syncthreads();
  for (int ch = t; ch < C; ch += NT) {
    const int gg = ch / 8, e = ch % 8;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < rpi; ++q) {
      a += red[0][(q * cg + gg) * 8 + e];
      b += red[1][(q * cg + gg) * 8 + e];
    }
    put_partial(part, acc, reps, C, ch, a, b);
  }
}

__global__ __launch_bounds__(NT) void pool_bn_bwd_apply_k(const uint16_t* __restrict__ dpool,
                                                          const uint8_t* __restrict__ arg, PoolGeo g,
                                                          const uint16_t* __restrict__ x, const float* __restrict__ st,
                                                          const float* co_in, uint16_t* __restrict__ dx,
                                                          long n8, BNBwdFin bf) {
  extern __shared__ float sfin[];
  const float* co = bn_bwd_fin_prologue(bf, g.C, st, sfin, co_in);
  const int C = g.C, cg = C / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg), c = c8 * 8;
    const long row = i / cg;
    float xv[8], d[8], mean[8], inv[8], sc[8], sh[8], a[8], b[8], cc[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], xv);
    ld8f(st + c, mean);
    ld8f(st + C + c, inv);
    ld8f(st + 2 * C + c, sc);
    ld8f(st + 3 * C + c, sh);
    stem_dy8(dpool, arg, g, row, c8, xv, sc, sh, d);
    ld8f(co + c, a);
    ld8f(co + C + c, b);
    ld8f(co + 2 * C + c, cc);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = a[e] * d[e] + b[e] + cc[e] * (xv[e] - mean[e]) * inv[e];
    reinterpret_cast<uint4*>(dx)[i] = pack8(d);
  }
}

// ---- stem backward, 3x3/s2 pool with H = 2 Ho, W = 2 Wo: one thread per 2x2 input quad --
// Pixel-centric gathers (above) load every covering pool window per input pixel: 2.25
// windows x (16 B gradient + 8 B argmax code) per pixel on average, each a dependent
// chain.  The 2x2 quad (2a..2a+1, 2b..2b+1) is covered by exactly the windows
// {a-1+PT, a+PT} x {b-1+PL, b+PL}: one thread loads those 4 windows once (8 independent
// loads) and routes them to its 4 pixels.  Window (wr, wc) reaches pixel (py, px) at tap
// kh = py + 2 - PT - 2 wr, kw = px + 2 - PL - 2 wc (valid when in [0, 2]); taps are
// accumulated in ascending (oh, ow) order exactly as pool_grad8 does, so the routed
// gradient and dx are bitwise those of the pixel-centric kernels for the same BN
// coefficients.
struct Quad8 {
  float d[4][8];  // routed (bf16-rounded) pool gradient of pixels (py, px) = (q >> 1, q & 1)
};

template <int PT, int PL>
__device__ __forceinline__ void quad_route8(const uint16_t* __restrict__ dpool, const uint8_t* __restrict__ arg,
                                            const PoolGeo& g, int n, int a, int b, int c8, Quad8& o) {
  const int cg = g.C / 8;
  float dw[2][2][8];
  uint32_t aw[2][2][2];
  // the four windows are loaded unconditionally at clamped coordinates and the out-of-range
  // ones neutralised after (a load under the edge branch cost its own round trip: the
  // ResNet-18 stem's backward apply 66 -> 59 us)
  uint4 dq[2][2];
  uint2 aq[2][2];
#pragma unroll
  for (int wr = 0; wr < 2; ++wr) {
#pragma unroll
    for (int wc = 0; wc < 2; ++wc) {
      const int oh = min(max(a - 1 + PT + wr, 0), g.Ho - 1), ow = min(max(b - 1 + PL + wc, 0), g.Wo - 1);
      const long w = (((long)n * g.Ho + oh) * g.Wo + ow) * cg + c8;
      dq[wr][wc] = reinterpret_cast<const uint4*>(dpool)[w];
      aq[wr][wc] = reinterpret_cast<const uint2*>(arg)[w];
    }
  }
#pragma unroll
  for (int wr = 0; wr < 2; ++wr) {
#pragma unroll
    for (int wc = 0; wc < 2; ++wc) {
      const int oh = a - 1 + PT + wr, ow = b - 1 + PL + wc;
      const bool ok = (unsigned)oh < (unsigned)g.Ho && (unsigned)ow < (unsigned)g.Wo;
      unpack8(dq[wr][wc], dw[wr][wc]);
      aw[wr][wc][0] = ok ? aq[wr][wc].x : 0xffffffffu;  // code 255 never matches a tap
      aw[wr][wc][1] = ok ? aq[wr][wc].y : 0xffffffffu;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int py = q >> 1, px = q & 1;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.d[q][e] = 0.f;
#pragma unroll
    for (int wr = 0; wr < 2; ++wr) {
      const int kh = py + 2 - PT - 2 * wr;
      if (kh < 0 || kh > 2) continue;
#pragma unroll
      for (int wc = 0; wc < 2; ++wc) {
        const int kw = px + 2 - PL - 2 * wc;
        if (kw < 0 || kw > 2) continue;
        const uint32_t me = (uint32_t)(kh * 3 + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (((aw[wr][wc][e >> 2] >> (8 * (e & 3))) & 0xffu) == me) o.d[q][e] += dw[wr][wc][e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o.d[q][e] = bf2f(f2bf(o.d[q][e]));
  }
}

template <int PT, int PL>
__global__ __launch_bounds__(NT) void pool_bn_bwd_reduce_q_k(const uint16_t* __restrict__ dpool,
                                                             const uint8_t* __restrict__ arg, PoolGeo g,
                                                             const uint16_t* __restrict__ x,
                                                             const float* __restrict__ st, float* __restrict__ part,
                                                             long nquad, long quads_per_block, long long* __restrict__ acc,
                                                             int reps) {
  __shared__ float red[2][NT * 8];
  const int C = g.C, cg = C / 8, t = threadIdx.x;
  const int rpi = NT / cg;
  const int gq = t % cg, rr = t / cg;
  const int c = gq * 8;
  float s0[8], s1[8], mean[8], inv[8], sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s0[e] = s1[e] = 0.f;
  ld8f(st + c, mean);
  ld8f(st + C + c, inv);
  ld8f(st + 2 * C + c, sc);
  ld8f(st + 3 * C + c, sh);
  const long q0 = blockIdx.x * quads_per_block, q1 = min(nquad, q0 + quads_per_block);
  if (rr < rpi) {
    for (long qd = q0 + rr; qd < q1; qd += rpi) {
      const int b = (int)(qd % g.Wo);
      const long tq = qd / g.Wo;
      const int a = (int)(tq % g.Ho), n = (int)(tq / g.Ho);
      float xv[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long pix = ((long)n * g.H + 2 * a + (q >> 1)) * g.W + 2 * b + (q & 1);
        unpack8(reinterpret_cast<const uint4*>(x)[pix * cg + gq], xv[q]);
      }
      Quad8 r;
      quad_route8<PT, PL>(dpool, arg, g, n, a, b, gq, r);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float yv[8];
        bn_relu8(xv[q], sc, sh, yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = yv[e] > 0.f ? r.d[q][e] : 0.f;
          s0[e] += d;
          s1[e] += d * (xv[q][e] - mean[e]) * inv[e];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][t * 8 + e] = rr < rpi ? s0[e] : 0.f;
    red[1][t * 8 + e] = rr < rpi ? s1[e] : 0.f;
  }
  __syncthreads();
  for (int ch = t; ch < C; ch += NT) {
    const int gg = ch / 8, e = ch % 8;
    float sa = 0.f, sb = 0.f;
    for (int q = 0; q < rpi; ++q) {
      sa += red[0][(q * cg + gg) * 8 + e];
      sb += red[1][(q * cg + gg) * 8 + e];
    }
    put_partial(part, acc, reps, C, ch, sa, sb);
  }
}

template <int PT, int PL>
__global__ __launch_bounds__(NT) void pool_bn_bwd_apply_q_k(const uint16_t* __restrict__ dpool,
                                                            const uint8_t* __restrict__ arg, PoolGeo g,
                                                            const uint16_t* __restrict__ x,
                                                            const float* __restrict__ st,
                                                            const float* co_in, uint16_t* __restrict__ dx,
                                                            long nq8, BNBwdFin bf) {
  extern __shared__ float sfin[];
  const float* co = bn_bwd_fin_prologue(bf, g.C, st, sfin, co_in);
  const int C = g.C, cg = C / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < nq8; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg), c = c8 * 8;
    const long qd = i / cg;
    const int b = (int)(qd % g.Wo);
    const long tq = qd / g.Wo;
    const int a = (int)(tq % g.Ho), n = (int)(tq / g.Ho);
    long pix[4];
    float xv[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pix[q] = ((long)n * g.H + 2 * a + (q >> 1)) * g.W + 2 * b + (q & 1);
      unpack8(reinterpret_cast<const uint4*>(x)[pix[q] * cg + c8], xv[q]);
    }
    Quad8 r;
    quad_route8<PT, PL>(dpool, arg, g, n, a, b, c8, r);
    float mean[8], inv[8], sc[8], sh[8], ca[8], cb[8], cc[8];
    ld8f(st + c, mean);
    ld8f(st + C + c, inv);
    ld8f(st + 2 * C + c, sc);
    ld8f(st + 3 * C + c, sh);
    ld8f(co + c, ca);
    ld8f(co + C + c, cb);
    ld8f(co + 2 * C + c, cc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float yv[8], d[8];
      bn_relu8(xv[q], sc, sh, yv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dm = yv[e] > 0.f ? r.d[q][e] : 0.f;
        d[e] = ca[e] * dm + cb[e] + cc[e] * (xv[q][e] - mean[e]) * inv[e];
      }
      reinterpret_cast<uint4*>(dx)[pix[q] * cg + c8] = pack8(d);
    }
  }
}

__host__ __forceinline__ bool quad_pool_geo(const PoolGeo& g) {
  return g.ph == 3 && g.pw == 3 && g.sh == 2 && g.sw == 2 && (g.pt == 0 || g.pt == 1) && (g.pl == 0 || g.pl == 1) &&
         g.H == 2 * g.Ho && g.W == 2 * g.Wo;
}

__global__ __launch_bounds__(NT) void gap_fwd_k(const uint16_t* __restrict__ x, int N, int HW, int C, void* y,
                                                int y_f32) {
  const int cg = C / 8;
  const long total = (long)N * cg;
  const float inv = 1.f / HW;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg), n = (int)(i / cg);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int p = 0; p < HW; ++p) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(x)[((long)n * HW + p) * cg + c8], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    if (y_f32) {
      float* o = (float*)y + (long)n * C + c8 * 8;
      *reinterpret_cast<float4*>(o) = float4{acc[0], acc[1], acc[2], acc[3]};
      *reinterpret_cast<float4*>(o + 4) = float4{acc[4], acc[5], acc[6], acc[7]};
    } else {
      reinterpret_cast<uint4*>(y)[i] = pack8(acc);
    }
  }
}

// One image per block, the pixels split over G = NT / cg thread groups (ResNet-18's 7x7x512
// head: 4 groups of ~12 pixels, 64 blocks) instead of one thread walking all HW pixels per
// channel group (16 blocks, a 49-long load chain each); partials combined in group order.
__global__ __launch_bounds__(NT) void gap_fwd_img_k(const uint16_t* __restrict__ x, int HW, int C, void* y,
                                                    int y_f32) {
  __shared__ float part[NT * 8];
  const int cg = C / 8, G = NT / cg, t = threadIdx.x, n = blockIdx.x;
  const int c8 = t % cg, g = t / cg;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if (g < G) {
    for (int p = g; p < HW; p += G) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(x)[((long)n * HW + p) * cg + c8], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[t * 8 + e] = acc[e];
  __syncthreads();
  if (t >= cg) return;
  float r[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = 0.f;
  for (int q = 0; q < G; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] += part[(q * cg + t) * 8 + e];
  const float inv = 1.f / HW;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] *= inv;
  if (y_f32) {
    float* o = (float*)y + (long)n * C + t * 8;
    *reinterpret_cast<float4*>(o) = float4{r[0], r[1], r[2], r[3]};
    *reinterpret_cast<float4*>(o + 4) = float4{r[4], r[5], r[6], r[7]};
  } else {
    reinterpret_cast<uint4*>(y)[(long)n * cg + t] = pack8(r);
  }
}

__global__ __launch_bounds__(NT) void gap_bwd_k(const void* dy, int dy_f32, int N, int HW, int C,
                                                uint16_t* __restrict__ dx) {
  const int cg = C / 8;
  const long total = (long)N * HW * cg;
  const float inv = 1.f / HW;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    const int n = (int)(i / ((long)cg * HW));
    float d[8];
    if (dy_f32) ld8f((const float*)dy + (long)n * C + c8 * 8, d);
    else unpack8(reinterpret_cast<const uint4*>(dy)[(long)n * cg + c8], d);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] *= inv;
    reinterpret_cast<uint4*>(dx)[i] = pack8(d);
  }
}

// ---- elementwise ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void relu_bwd_k(const uint16_t* dy, const uint16_t* y, uint16_t* dz, long n8) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float d[8], yv[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], d);
    unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = yv[e] > 0.f ? d[e] : 0.f;
    reinterpret_cast<uint4*>(dz)[i] = pack8(d);
  }
}

// Pointwise activations on bf16 tensors (kind 0 relu, 1 sigmoid, 2 tanh).  The backward
// reads the stored output y: relu' = [y > 0], sigmoid' = y (1 - y), tanh' = 1 - y^2.  A
// thread owns 8 elements (one 16-byte access); the last, partial group of a length that
// is not a multiple of 8 goes element by element.
__device__ __forceinline__ float act_f(float z, int kind) {
  if (kind == 1) return 1.f / (1.f + __expf(-z));
  if (kind == 2) return tanhf(z);
  return fmaxf(z, 0.f);
}
__device__ __forceinline__ float act_df(float y, int kind) {
  if (kind == 1) return y * (1.f - y);
  if (kind == 2) return 1.f - y * y;
  return y > 0.f ? 1.f : 0.f;
}

__global__ __launch_bounds__(NT) void act_fwd_k(const uint16_t* x, uint16_t* y, long n, int kind) {
  const long n8 = (n + 7) / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    if (8 * i + 8 <= n) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = act_f(v[e], kind);
      reinterpret_cast<uint4*>(y)[i] = pack8(v);
    } else {
      for (long j = 8 * i; j < n; ++j) y[j] = f2bf(act_f(bf2f(x[j]), kind));
    }
  }
}

__global__ __launch_bounds__(NT) void act_bwd_k(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n,
                                                int kind) {
  const long n8 = (n + 7) / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    if (8 * i + 8 <= n) {
      float d[8], yv[8];
      unpack8(reinterpret_cast<const uint4*>(dy)[i], d);
      unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] *= act_df(yv[e], kind);
      reinterpret_cast<uint4*>(dx)[i] = pack8(d);
    } else {
      for (long j = 8 * i; j < n; ++j) dx[j] = f2bf(bf2f(dy[j]) * act_df(bf2f(y[j]), kind));
    }
  }
}

// Dropout with a counter-based mask: element j of step t is kept iff
// drop_hash(key_t, j) >= rate * 2^32, key_t = mix32(seed + t * golden), t = ctrl->cur3 (the
// step's iteration, set by gather_batch).  No mask tensor and no RNG state: the backward
// regenerates the same mask from (seed, t, j), and a graph replay draws a fresh mask
// because t advances on the device.  Kept elements are scaled by 1 / (1 - rate).
// distributed_amd/engine/native_graph.py:dropout_mask_reference is the host oracle.
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__global__ __launch_bounds__(NT) void dropout_k(const uint16_t* x, uint16_t* y, long n, const Ctrl* ctrl,
                                                uint32_t seed, uint32_t thr, float scale) {
  const uint32_t key = mix32(seed + (uint32_t)ctrl->cur3 * 0x9e3779b9u);
  const long n8 = (n + 7) / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    if (8 * i + 8 <= n) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t h = mix32(mix32((uint32_t)(8 * i + e) ^ key) + key);
        v[e] = h >= thr ? v[e] * scale : 0.f;
      }
      reinterpret_cast<uint4*>(y)[i] = pack8(v);
    } else {
      for (long j = 8 * i; j < n; ++j) {
        const uint32_t h = mix32(mix32((uint32_t)j ^ key) + key);
        y[j] = f2bf(h >= thr ? bf2f(x[j]) * scale : 0.f);
      }
    }
  }
}

__global__ __launch_bounds__(NT) void add_bf16_k(const uint16_t* a, const uint16_t* b, uint16_t* o, long n8) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float x[8], y[8];
    unpack8(reinterpret_cast<const uint4*>(a)[i], x);
    unpack8(reinterpret_cast<const uint4*>(b)[i], y);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] += y[e];
    reinterpret_cast<uint4*>(o)[i] = pack8(x);
  }
}

__global__ __launch_bounds__(NT) void cast_f32_bf16_k(const float* x, uint16_t* y, long n) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) y[i] = f2bf(x[i]);
}

__global__ __launch_bounds__(NT) void cast_bf16_f32_k(const uint16_t* x, float* y, long n) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) y[i] = bf2f(x[i]);
}

__global__ __launch_bounds__(NT) void cast_u8_bf16_k(const uint8_t* x, float scale, uint16_t* y, long n) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT)
    y[i] = f2bf((float)x[i] * scale);
}

// Column sums in a fixed order (bias gradients; no float atomics).  grid (ceil(N/64),
// splits), 4 row phases per block: split y sums rows y*4+ph, y*4+ph + 4*splits, ...; one
// split adds straight into out[n], several write slab[y][n] and colsum_fin_k adds the
// slabs in split order.
__global__ __launch_bounds__(NT) void colsum_k(const void* x, int x_f32, int M, int N, int ld, float* out,
                                               float* slab) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + cl;
  float a = 0.f;
  if (n < N)
    for (int m = blockIdx.y * 4 + ph; m < M; m += gridDim.y * 4)
      a += x_f32 ? ((const float*)x)[(size_t)m * ld + n] : bf2f(((const uint16_t*)x)[(size_t)m * ld + n]);
  red[ph][cl] = a;
  __syncthreads();
  if (ph == 0 && n < N) {
    const float v = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    if (gridDim.y == 1) out[n] += v;
    else slab[(size_t)blockIdx.y * N + n] = v;
  }
}
__global__ __launch_bounds__(NT) void colsum_fin_k(const float* slab, int splits, int N, float* out) {
  const int n = blockIdx.x * NT + threadIdx.x;
  if (n >= N) return;
  float a = 0.f;
  for (int y = 0; y < splits; ++y) a += slab[(size_t)y * N + n];
  out[n] += a;
}

// ---- loss ------------------------------------------------------------------------------------
// Rows with label < 0 (past the end of the dataset in a short final batch) get a zero
// gradient and no loss / metric contribution.  With ctrl != nullptr the gradient scale is
// 1 / (rows of this global batch that exist): Keras' SUM_OVER_BATCH_SIZE on the real
// final batch; benchmark wrap mode (ctrl->wrap > 0) always has full batches.
// One block per row; the row is read from memory once (up to 4 values per thread held in
// registers) and reduced by wave shuffles plus one LDS exchange per quantity.  The first
// version re-read the row for the max, the exponent sum and the output, and reduced each
// by an 8-level LDS tree (17 barriers per row, 30 more in the last block): 9.8 us for the
// ResNet-18 head (64 x 1000) -- the 1000-class logits of 64 rows.
constexpr int SX_KPT = 4, SX_NW = NT / 64, SX_BK = 1024;
__device__ __forceinline__ void sx_better(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }  // max, ties -> smallest index
}
__device__ __forceinline__ float sx_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__global__ __launch_bounds__(NT) void softmax_xent_k(const float* __restrict__ logits, int ld,
                                                     const int32_t* __restrict__ labels, int K, float scale,
                                                     const Ctrl* __restrict__ ctrl, uint16_t* __restrict__ dl,
                                                     float* tail, float* rows, float* bias_grad) {
  __shared__ float wmax[SX_NW], wsum[SX_NW], wtail[3][SX_NW];
  __shared__ int widx[SX_NW];
  __shared__ int last;
  const int b = blockIdx.x, t = threadIdx.x, B = gridDim.x, lane = t & 63, w = t >> 6;
  const int y = labels[b];
  float row_loss = 0.f, row_corr = 0.f;
  if (y < 0) {
    for (int k = t; k < K; k += NT) dl[(size_t)b * ld + k] = 0;
  } else {
    if (ctrl) {
      const int gb = ctrl->global_batch;
      const int left = ctrl->nsamples - ctrl->cursor * gb;
      scale = 1.f / (float)(ctrl->wrap > 0 ? gb : max(1, min(gb, left)));
    }
    const float* z = logits + (size_t)b * ld;
    const bool reg = K <= SX_KPT * NT;  // the row fits the registers
    float zr[SX_KPT];
    float mx = -INFINITY;
    int mi = 0x7fffffff;
    if (reg) {
#pragma unroll
      for (int i = 0; i < SX_KPT; ++i) zr[i] = t + i * NT < K ? z[t + i * NT] : -INFINITY;
#pragma unroll
      for (int i = 0; i < SX_KPT; ++i)
        if (t + i * NT < K && zr[i] > mx) { mx = zr[i]; mi = t + i * NT; }
    } else {
      for (int k = t; k < K; k += NT) {
        const float v = z[k];
        if (v > mx) { mx = v; mi = k; }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sx_better(mx, mi, __shfl_xor(mx, o), __shfl_xor(mi, o));
    if (lane == 0) { wmax[w] = mx; widx[w] = mi; }
    __syncthreads();
    float zmax = wmax[0];
    int amax = widx[0];
#pragma unroll
    for (int v = 1; v < SX_NW; ++v) sx_better(zmax, amax, wmax[v], widx[v]);
    float se = 0.f;
    if (reg) {
#pragma unroll
      for (int i = 0; i < SX_KPT; ++i) {
        zr[i] = t + i * NT < K ? __expf(zr[i] - zmax) : 0.f;
        se += zr[i];
      }
    } else {
      for (int k = t; k < K; k += NT) se += __expf(z[k] - zmax);
    }
    se = sx_wave_sum(se);
    if (lane == 0) wsum[w] = se;
    __syncthreads();
    float sum = wsum[0];
#pragma unroll
    for (int v = 1; v < SX_NW; ++v) sum += wsum[v];
    const float inv = 1.f / sum;
    if (reg) {
#pragma unroll
      for (int i = 0; i < SX_KPT; ++i) {
        const int k = t + i * NT;
        if (k < K) dl[(size_t)b * ld + k] = f2bf((zr[i] * inv - (k == y ? 1.f : 0.f)) * scale);
      }
    } else {
      for (int k = t; k < K; k += NT) {
        const float p = __expf(z[k] - zmax) * inv;
        dl[(size_t)b * ld + k] = f2bf((p - (k == y ? 1.f : 0.f)) * scale);
      }
    }
    row_loss = logf(sum) + zmax - z[y];
    row_corr = amax == y ? 1.f : 0.f;
  }
  // the batch sums in a fixed order (no float atomics: replays and graph / eager runs give
  // the same bits): every row stores (loss, correct, valid), the last block to arrive adds
  // them up (fixed shuffle tree + fixed wave order) and re-arms the arrival counter rows[3 B]
  if (t == 0) {
    rows[3 * b] = row_loss;
    rows[3 * b + 1] = row_corr;
    rows[3 * b + 2] = y < 0 ? 0.f : 1.f;
  }
  int* counter = reinterpret_cast<int*>(rows + 3 * B);
  if (!last_arriver(counter, B, &last)) return;
  float a[3] = {0.f, 0.f, 0.f};
  for (int r = t; r < B; r += NT)
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] += rows[3 * r + q];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    a[q] = sx_wave_sum(a[q]);
    if (lane == 0) wtail[q][w] = a[q];
  }
  __syncthreads();
  if (t < 3) {
    float v = wtail[t][0];
#pragma unroll
    for (int u = 1; u < SX_NW; ++u) v += wtail[t][u];
    tail[t] += v;
  }
  if (t == 0) *counter = 0;
  if (bias_grad) {
    // the logits layer's bias gradient from the stored dl rows (every block's, acquired by
    // last_arriver), in colsum_k's one-split order: 4 row phases each summed in row order,
    // then (p0 + p1) + (p2 + p3), added to the gradient -- the same bits as its launch.
    // Work item = (phase, 8 columns): 16-byte loads of 8 rows in flight at a time, the
    // phase sums meet in LDS (a thread per column walking the rows one load at a time took
    // the launch from 7.5 to 66 us)
    __shared__ float bph[4][SX_BK];
    if (K <= SX_BK && ld % 8 == 0) {
      const int ng = (K + 7) / 8;
      for (int wi = t; wi < 4 * ng; wi += NT) {
        const int q = wi / ng, g = wi - q * ng;
        float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int m0 = q; m0 < B; m0 += 32) {
          uint4 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int m = m0 + 4 * u;
            v[u] = m < B ? *reinterpret_cast<const uint4*>(dl + (size_t)m * ld + 8 * g) : uint4{0u, 0u, 0u, 0u};
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (m0 + 4 * u >= B) break;
            const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              s8[2 * e] += __uint_as_float(w4[e] << 16);
              s8[2 * e + 1] += __uint_as_float(w4[e] & 0xffff0000u);
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) bph[q][8 * g + e] = s8[e];
      }
      __syncthreads();
      for (int k = t; k < K; k += NT) bias_grad[k] += (bph[0][k] + bph[1][k]) + (bph[2][k] + bph[3][k]);
    } else {
      for (int k = t; k < K; k += NT) {
        float ph[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          for (int m = q; m < B; m += 4) ph[q] += bf2f(dl[(size_t)m * ld + k]);
        bias_grad[k] += (ph[0] + ph[1]) + (ph[2] + ph[3]);
      }
    }
  }
}

// ---- inference (predict / evaluate through the native forward plan) ----------------------
// BatchNorm with the moving statistics: the same st rows bn_finalize writes from batch
// statistics (mean, 1/sqrt(var + eps), scale, shift), so every BN apply / fused residual /
// stem-pool kernel runs unchanged in inference mode.
__global__ __launch_bounds__(NT) void bn_infer_st_k(const float* __restrict__ rmean, const float* __restrict__ rvar,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float eps, int C, float* __restrict__ st) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  const float m = rmean[c], inv = rsqrtf(rvar[c] + eps);
  const float sc = (gamma ? gamma[c] : 1.f) * inv;
  st[c] = m;
  st[C + c] = inv;
  st[2 * C + c] = sc;
  st[3 * C + c] = fmaf(-m, sc, beta ? beta[c] : 0.f);
}

// logits rows of this step -> out[global row][K] (rows past the end of the data dropped);
// the row base comes from the device cursor, so a captured graph replays across batches
__global__ __launch_bounds__(NT) void logits_store_k(const float* __restrict__ logits, int ld, int K, int B,
                                                     const Ctrl* __restrict__ ctrl, float* __restrict__ out) {
  const long base = (long)ctrl->cursor * ctrl->global_batch + ctrl->row0;
  const long n = ctrl->nsamples;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < (long)B * K; i += (long)gridDim.x * NT) {
    const int r = (int)(i / K), k = (int)(i % K);
    if (base + r < n) out[(base + r) * K + k] = logits[(long)r * ld + k];
  }
}

// end of an inference step: fold the metric tail into the epoch accumulators (and clear
// it for the next step), advance the cursor
__global__ void step_fold_k(Ctrl* ctrl, float* tail) {
  if (threadIdx.x != 0) return;
  if (tail) {
    ctrl->acc_loss += tail[0];
    ctrl->acc_correct += tail[1];
    ctrl->acc_count += tail[2];
    tail[0] = tail[1] = tail[2] = 0.f;
  }
  int c = ctrl->cursor + 1;
  if (ctrl->wrap > 0 && c >= ctrl->wrap) c = 0;
  ctrl->cursor = c;
}

// ---- optimizer ------------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void sgd_flat_k(float* __restrict__ P, const float* __restrict__ G,
                                                 float* __restrict__ V, uint16_t* __restrict__ Pb, long n, float lr,
                                                 float mom, int nest) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    float wn, vn;
    sgd_update(P[i], G[i], V ? V[i] : 0.f, lr, mom, nest, wn, vn);
    P[i] = wn;
    if (V) V[i] = vn;
    if (Pb) Pb[i] = f2bf(wn);
  }
}

__global__ __launch_bounds__(NT) void sgd_step_k(float* __restrict__ P, const float* __restrict__ G,
                                                 float* __restrict__ V, uint16_t* __restrict__ Pb, long n,
                                                 Ctrl* ctrl, const float* tail) {
  const float lr = ctrl->lr, mom = ctrl->momentum;
  const int nest = ctrl->nesterov;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    float wn, vn;
    sgd_update(P[i], G[i], mom != 0.f ? V[i] : 0.f, lr, mom, nest, wn, vn);
    P[i] = wn;
    if (mom != 0.f) V[i] = vn;
    Pb[i] = f2bf(wn);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctrl->acc_loss += tail[0];
    ctrl->acc_correct += tail[1];
    ctrl->acc_count += tail[2];
    int c = ctrl->cursor + 1;
    if (ctrl->wrap > 0 && c >= ctrl->wrap) c = 0;
    ctrl->cursor = c;
    ctrl->iterations += 1;
  }
}

__global__ __launch_bounds__(NT) void gather_batch_k(const void* __restrict__ x, int x_u8, float scale,
                                                     const int32_t* __restrict__ labels, Ctrl* __restrict__ ctrl,
                                                     int per, int HW, int Cin, int Cp, uint16_t* __restrict__ xb,
                                                     int32_t* __restrict__ yb, uint4* __restrict__ zero, long nz16,
                                                     uint4* __restrict__ zero2, long nz16b, PadCastJob pc) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < nz16; i += (long)gridDim.x * NT) zero[i] = uint4{0u, 0u, 0u, 0u};
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < nz16b; i += (long)gridDim.x * NT) zero2[i] = uint4{0u, 0u, 0u, 0u};
  // a layer's padded bf16 weight copy, element for element as pad_cast_k: a thread's first
  // element is loaded here and stored when the thread's gather work is done (the load's
  // latency hides under it; loading and storing up front cost the launch ~2 us)
  const long pc_total = pc.src ? (long)pc.R * pc.C1p * pc.C2p : 0;
  const long gt = blockIdx.x * (long)NT + threadIdx.x;
  auto pc_src = [&](long i) -> const float* {
    const int c2 = (int)(i % pc.C2p);
    const long t = i / pc.C2p;
    const int c1 = (int)(t % pc.C1p), r = (int)(t / pc.C1p);
    return c1 < pc.C1 && c2 < pc.C2 ? pc.src + ((long)r * pc.C1 + c1) * pc.C2 + c2 : nullptr;
  };
  float pcf = 0.f;
  if (gt < pc_total) {
    const float* p = pc_src(gt);
    pcf = p ? *p : 0.f;
  }
  auto pc_finish = [&]() {
    if (gt >= pc_total) return;
    pc.dst[gt] = f2bf(pcf);
    for (long i = gt + (long)gridDim.x * NT; i < pc_total; i += (long)gridDim.x * NT) {
      const float* p = pc_src(i);
      pc.dst[i] = p ? f2bf(*p) : (uint16_t)0;
    }
  };
  const long base = (long)ctrl->cursor * ctrl->global_batch + ctrl->row0;
  const int n = ctrl->nsamples;
  const bool wrap = ctrl->wrap > 0;  // benchmark mode: the epoch wraps, every row is real
  if (blockIdx.x == 0 && threadIdx.x == 0) ctrl->cur3 = ctrl->iterations + 1;  // this step's t (opt_step)
  if (Cp == 4 && Cin == 3 && x_u8 && HW % 4 == 0) {
    // RGB uint8 rows -> packed 4-channel bf16: one thread per 4 pixels of one row, the 12
    // source bytes as three aligned dword loads (byte loads moved 64 B per wave
    // instruction), two 16-byte stores
    const long total = (long)per * HW / 4;
    for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
      const long pr = 4 * i;
      const int p = (int)(pr % HW), r = (int)(pr / HW);
      const bool valid = wrap || base + r < n;
      const long row = valid ? (base + r) % n : 0;
      uint32_t w[3] = {0u, 0u, 0u};
      if (valid) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>((const uint8_t*)x + (row * HW + p) * 3);
        w[0] = src[0];
        w[1] = src[1];
        w[2] = src[2];
      }
      float v[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int b = 3 * k + c;
          v[4 * k + c] = (float)((w[b >> 2] >> (8 * (b & 3))) & 0xffu) / scale;
        }
        v[4 * k + 3] = 0.f;
      }
      if (p == 0) yb[r] = valid ? labels[row] : -1;
      reinterpret_cast<uint4*>(xb)[2 * i] = pack8(v);
      reinterpret_cast<uint4*>(xb)[2 * i + 1] = pack8(v + 8);
    }
    pc_finish();
    return;
  }
  if (Cp == 4) {
    // packed-tap stem input (4 channels): one thread per 2 pixels, one 16-byte store
    const long total = (long)per * HW / 2;
    for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
      float v[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const long pr = 2 * i + h;
        const int p = (int)(pr % HW), r = (int)(pr / HW);
        const bool valid = wrap || base + r < n;
        const long row = valid ? (base + r) % n : 0;
        const long si = (row * HW + p) * Cin;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          v[4 * h + c] = 0.f;
          if (c < Cin && valid)
            v[4 * h + c] = x_u8 ? (float)((const uint8_t*)x)[si + c] / scale : ((const float*)x)[si + c];
        }
        if (p == 0) yb[r] = valid ? labels[row] : -1;
      }
      reinterpret_cast<uint4*>(xb)[i] = pack8(v);
    }
    pc_finish();
    return;
  }
  // one thread per 8 (padded) channels of one pixel: one 16-byte store
  const int cg = Cp / 8;
  const long total = (long)per * HW * cg;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % cg);
    const long pr = i / cg;
    const int p = (int)(pr % HW), r = (int)(pr / HW);
    // rows past the end of a short final batch: zero image, label -1 (masked downstream)
    const bool valid = wrap || base + r < n;
    const long row = valid ? (base + r) % n : 0;
    const long si = (row * HW + p) * Cin;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c8 * 8 + e;
      v[e] = 0.f;
      if (c < Cin && valid)
        v[e] = x_u8 ? (float)((const uint8_t*)x)[si + c] / scale : ((const float*)x)[si + c];
    }
    reinterpret_cast<uint4*>(xb)[i] = pack8(v);
    if (p == 0 && c8 == 0) yb[r] = valid ? labels[row] : -1;
  }
  pc_finish();
}

__global__ __launch_bounds__(NT) void pad_cast_k(const float* src, int R, int C1, int C2, int C1p, int C2p,
                                                 uint16_t* dst) {
  const long total = (long)R * C1p * C2p;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c2 = (int)(i % C2p);
    const long t = i / C2p;
    const int c1 = (int)(t % C1p), r = (int)(t / C1p);
    dst[i] = (c1 < C1 && c2 < C2) ? f2bf(src[((long)r * C1 + c1) * C2 + c2]) : (uint16_t)0;
  }
}

__global__ __launch_bounds__(NT) void unpad_add_k(const float* src, int R, int C1, int C2, int C1p, int C2p,
                                                  float* dst) {
  const long total = (long)R * C1 * C2;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c2 = (int)(i % C2);
    const long t = i / C2;
    const int c1 = (int)(t % C1), r = (int)(t / C1);
    dst[i] += src[((long)r * C1p + c1) * C2p + c2];
  }
}

}  // namespace

// Keras optimizer_v2 update rules on the flat fp32 master buffer (+ bf16 shadow): the
// native-engine counterpart of keras/optimizers.py apply_flat.  lr from ctrl (a schedule
// needs no re-capture); Adam's step t = ctrl->cur3, written by gather_batch at the start
// of the step (no block of this kernel reads a ctrl field this kernel writes).
__global__ __launch_bounds__(NT) void opt_step_k(float* __restrict__ P, const float* __restrict__ G,
                                                 float* __restrict__ S0, float* __restrict__ S1,
                                                 float* __restrict__ S2, uint16_t* __restrict__ Pb, long n,
                                                 Ctrl* ctrl, const float* tail, OptArgs o, int book) {
  const float lr = ctrl->lr;
  const int t = ctrl->cur3;
  float lr_t = lr;
  if (o.kind == 1) lr_t = lr * sqrtf(1.f - powf(o.b2, (float)t)) / (1.f - powf(o.b1, (float)t));
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const float g = G[i];
    float w = P[i];
    if (o.kind == 1) {  // Adam (S0 m, S1 v, S2 vhat)
      const float m = o.b1 * S0[i] + (1.f - o.b1) * g;
      const float v = o.b2 * S1[i] + (1.f - o.b2) * g * g;
      S0[i] = m;
      S1[i] = v;
      float d = v;
      if (o.flag) {
        d = fmaxf(S2[i], v);
        S2[i] = d;
      }
      w -= lr_t * (m / (sqrtf(d) + o.eps));
    } else if (o.kind == 2) {  // RMSprop (S0 rms, S1 momentum, S2 mg)
      const float ms = o.rho * S0[i] + (1.f - o.rho) * g * g;
      S0[i] = ms;
      float den = ms;
      if (o.flag) {
        const float mg = o.rho * S2[i] + (1.f - o.rho) * g;
        S2[i] = mg;
        den = ms - mg * mg;
      }
      const float upd = g / (sqrtf(den) + o.eps) * lr;
      if (o.mom != 0.f) {
        const float mo = o.mom * S1[i] + upd;
        S1[i] = mo;
        w -= mo;
      } else {
        w -= upd;
      }
    } else {  // SGD (S0 momentum)
      float wn, vn;
      sgd_update(w, g, o.mom != 0.f ? S0[i] : 0.f, lr, o.mom, o.flag, wn, vn);
      if (o.mom != 0.f) S0[i] = vn;
      w = wn;
    }
    P[i] = w;
    Pb[i] = f2bf(w);
  }
  // the step's bookkeeping, once per step: by the launch covering the metric tail's bucket
  // when the update is split per gradient bucket (native_graph bucket_opt), else by the
  // single launch.  (The per-bucket launches only READ ctrl's lr / cur3.)
  if (book && blockIdx.x == 0 && threadIdx.x == 0) {
    ctrl->acc_loss += tail[0];
    ctrl->acc_correct += tail[1];
    ctrl->acc_count += tail[2];
    int c = ctrl->cursor + 1;
    if (ctrl->wrap > 0 && c >= ctrl->wrap) c = 0;
    ctrl->cursor = c;
    ctrl->iterations = t;
  }
}

hipError_t opt_step(float* P, const float* G, float* S0, float* S1, float* S2, uint16_t* Pb, long n, Ctrl* ctrl,
                    const float* tail, const OptArgs& o, hipStream_t s, int book) {
  if (o.kind < 0 || o.kind > 2 || n < 0) return hipErrorInvalidValue;
  const int grid = n > 0 ? grid_for(n, NT, 4096) : 1;
  hipLaunchKernelGGL(opt_step_k, dim3(grid), dim3(NT), 0, s, P, G, S0, S1, S2, Pb, n, ctrl, tail, o, book);
  return hipGetLastError();
}

hipError_t bn_infer_st(const float* rmean, const float* rvar, const float* gamma, const float* beta, float eps, int C,
                       float* st, hipStream_t s) {
  hipLaunchKernelGGL(bn_infer_st_k, dim3((C + NT - 1) / NT), dim3(NT), 0, s, rmean, rvar, gamma, beta, eps, C, st);
  return hipGetLastError();
}

hipError_t logits_store(const float* logits, int ld, int K, int B, const Ctrl* ctrl, float* out, hipStream_t s) {
  if (K > ld) return hipErrorInvalidValue;
  hipLaunchKernelGGL(logits_store_k, dim3(grid_for((long)B * K)), dim3(NT), 0, s, logits, ld, K, B, ctrl, out);
  return hipGetLastError();
}

hipError_t step_fold(Ctrl* ctrl, float* tail, hipStream_t s) {
  hipLaunchKernelGGL(step_fold_k, dim3(1), dim3(64), 0, s, ctrl, tail);
  return hipGetLastError();
}

hipError_t sgd_step(float* P, const float* G, float* V, uint16_t* Pb, long n, Ctrl* ctrl, const float* tail,
                    hipStream_t s) {
  hipLaunchKernelGGL(sgd_step_k, dim3(grid_for(n, NT, 4096)), dim3(NT), 0, s, P, G, V, Pb, n, ctrl, tail);
  return hipGetLastError();
}

hipError_t gather_batch(const void* x, int x_u8, float scale, const int32_t* labels, Ctrl* ctrl, int per,
                        int HW, int Cin, int Cp, uint16_t* xb, int32_t* yb, hipStream_t s, void* zero, long zero_bytes,
                        void* zero2, long zero2_bytes, PadCastJob pc) {
  if (pc.src && (!pc.dst || pc.R < 1 || pc.C1 < 1 || pc.C2 < 1 || pc.C1p < pc.C1 || pc.C2p < pc.C2))
    return hipErrorInvalidValue;
  if (Cp % 8 && !(Cp == 4 && Cin <= 4 && HW % 2 == 0)) return hipErrorInvalidValue;
  for (int k = 0; k < 2; ++k) {
    const void* z = k ? zero2 : zero;
    const long nb = k ? zero2_bytes : zero_bytes;
    if (nb < 0 || nb % 16 || (nb > 0 && (z == nullptr || reinterpret_cast<uintptr_t>(z) % 16)))
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(gather_batch_k, dim3(grid_for((long)per * HW * Cp / 8)), dim3(NT), 0, s, x, x_u8, scale, labels,
                     ctrl, per, HW, Cin, Cp, xb, yb, static_cast<uint4*>(zero), zero_bytes / 16,
                     static_cast<uint4*>(zero2), zero2_bytes / 16, pc);
  return hipGetLastError();
}

hipError_t pad_cast(const float* src, int R, int C1, int C2, int C1p, int C2p, uint16_t* dst, hipStream_t s) {
  hipLaunchKernelGGL(pad_cast_k, dim3(grid_for((long)R * C1p * C2p)), dim3(NT), 0, s, src, R, C1, C2, C1p, C2p, dst);
  return hipGetLastError();
}

hipError_t unpad_add(const float* src, int R, int C1, int C2, int C1p, int C2p, float* dst, hipStream_t s) {
  hipLaunchKernelGGL(unpad_add_k, dim3(grid_for((long)R * C1 * C2)), dim3(NT), 0, s, src, R, C1, C2, C1p, C2p, dst);
  return hipGetLastError();
}

hipError_t bn_finalize(const float* part, int T, int C, float count, const float* gamma, const float* beta, float eps,
                       float momentum, float* rmean, float* rvar, float* st, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_finalize_k, dim3(C / 8), dim3(FT), 0, s, part, T, C, count, gamma, beta, eps,
                     momentum, rmean, rvar, st);
  return hipGetLastError();
}

// row-mapped apply kernels: about BN_UNR rows per thread (one batch of loads in flight)
static int rows_grid(long M, int C, int cap = 16384) {
  const long rpi = NT / (C / 8);
  long g = (M + rpi * BN_UNR - 1) / (rpi * BN_UNR);
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}
// grid cap of a row-mapped consumer that finalizes in its prologue (env DAMD_BN_FIN_GRID):
// every block pays the prologue, so fewer, longer-lived blocks.  ResNet-18 step: 2.707 ms
// uncapped (1568 blocks on layer 1), 2.671 at 512, 2.665 at 768.
static int fin_rows_cap() {
  static int cap = [] {
    const char* e = getenv("DAMD_BN_FIN_GRID");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 768;
  }();
  return cap;
}
// ... and at least DAMD_BN_FIN_MINKB KiB of each input tensor per block: every block reads
// all R x 4C accumulator words, which on the deep layers (C = 512: 128 KiB per block) was
// more than the block's share of the data
static int fin_rows_grid(long M, int C) {
  static long minb = -1;
  if (minb < 0) {
    const char* e = getenv("DAMD_BN_FIN_MINKB");
    minb = e ? atol(e) * 1024 : 0;
  }
  int g = rows_grid(M, C, fin_rows_cap());
  if (minb > 0) {
    const long cap = ((long)M * C * 2 + minb - 1) / minb;
    if (g > cap) g = (int)(cap < 1 ? 1 : cap);
  }
  return g;
}

// blocks of a consumer that finalizes in its prologue: every block pays one pass over the
// C channels, so the grid-stride kernels run at most 8 blocks per CU
constexpr int FIN_GRID_CAP = 2048;
constexpr int FIN_MAX_C = 4096;
static const BNFin kNoFin{};
static const BNBwdFin kNoBwdFin{};

hipError_t bn_apply(const uint16_t* x, const float* st, const uint16_t* r, const float* st2, int res_mode, int relu,
                    uint16_t* y, long M, int C, hipStream_t s, const BNFin* f1, const BNFin* f2) {
  const long n8 = M * C / 8;
  const BNFin a = f1 ? *f1 : kNoFin, b = (f2 && res_mode == 2) ? *f2 : kNoFin;
  if ((a.acc && !a.st) || (b.acc && !b.st) || ((a.acc || b.acc) && C > FIN_MAX_C)) return hipErrorInvalidValue;
  const size_t lds = (a.acc ? 4 * C * sizeof(float) : 0) + (b.acc ? 4 * C * sizeof(float) : 0);
  // (the f2 region starts at 4C: allocate it whenever f2 finalizes)
  const size_t lds2 = b.acc ? 8 * C * sizeof(float) : lds;
  if (NT % (C / 8) == 0) {
    hipLaunchKernelGGL(bn_apply_rows_k, dim3((a.acc || b.acc) ? fin_rows_grid(M, C) : rows_grid(M, C, 16384)), dim3(NT),
                       lds2, s, x, st, r, st2,
                       res_mode, relu, y, M, C, a, b);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(bn_apply_k, dim3(grid_for(n8, NT, (a.acc || b.acc) ? FIN_GRID_CAP : 8192)), dim3(NT), lds2, s,
                     x, st, r, st2, res_mode, relu, y, n8, C, a, b);
  return hipGetLastError();
}

int bn_bwd_blocks(long M, int C) {
  // target grid (DAMD_BN_BWD_BLOCKS, default 512): fewer blocks = fewer per-block partials
  // added into the fixed-point accumulators (4 atomics per channel and block).  ResNet-18
  // step, one box: 1024 blocks 2.736 ms, 512 2.718, 256 2.757
  static long target = 0;
  if (!target) {
    const char* e = getenv("DAMD_BN_BWD_BLOCKS");
    target = e ? atol(e) : 512;
    if (target < 64) target = 512;
  }
  const int rpi = NT / (C / 8);
  long rows = (M + target - 1) / target;
  if (rows < rpi) rows = rpi;
  // at least DAMD_BN_BWD_MINKB KiB of dy per block: on the small deep layers (M = 3136 rows
  // of 512 channels) the 512-block target gave 7 rows per block, and the 4C fixed-point
  // atomics of every block, not the 6 MB read, set the launch time
  static long minb = -1;
  if (minb < 0) {
    const char* e = getenv("DAMD_BN_BWD_MINKB");
    minb = e ? atol(e) * 1024 : 0;
  }
  const long row_bytes = (long)C * 2;
  if (minb > 0 && rows * row_bytes < minb) rows = (minb + row_bytes - 1) / row_bytes;
  return (int)((M + rows - 1) / rows);
}

bool g_bn_reduce_reverse = false;
void bn_reduce_reverse(bool on) { g_bn_reduce_reverse = on; }

hipError_t bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x, const float* st,
                         uint16_t* dz_out, float* part, int T, long M, int C, hipStream_t s, long long* acc,
                         int acc_reps) {
  if (C % 8 || C / 8 > NT || (!part && !acc) || acc_reps < 1) return hipErrorInvalidValue;
  const long rows = (M + T - 1) / T;
  if (relu_mask < 0 || relu_mask > 2) return hipErrorInvalidValue;
  auto k = relu_mask == 0 ? bn_bwd_reduce_k<0> : relu_mask == 1 ? bn_bwd_reduce_k<1> : bn_bwd_reduce_k<2>;
  hipLaunchKernelGGL(k, dim3(T), dim3(NT), 0, s, dy, y, x, st, dz_out, part, M, C, rows, acc, acc_reps,
                     g_bn_reduce_reverse ? 1 : 0);
  return hipGetLastError();
}

hipError_t bn_bwd_reduce_dual(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x,
                              const uint16_t* x2, const float* st, const float* st2, int T, long M, int C,
                              hipStream_t s, long long* acc, long long* acc2, int acc_reps) {
  if (C % 8 || C / 8 > NT || !acc || !acc2 || acc_reps < 1 || relu_mask < 0 || relu_mask > 1)
    return hipErrorInvalidValue;
  const long rows = (M + T - 1) / T;
  hipLaunchKernelGGL(bn_bwd_reduce2_k, dim3(T), dim3(NT), 0, s, dy, y, relu_mask, x, x2, st, st2, M, C, rows, acc,
                     acc2, acc_reps);
  return hipGetLastError();
}

hipError_t bn_bwd_apply_dual(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x,
                             const uint16_t* x2, const float* st, const float* st2, uint16_t* dx, uint16_t* dx2,
                             long M, int C, hipStream_t s, const BNBwdFin& bf, const BNBwdFin& bf2) {
  if (C % 8 || NT % (C / 8) || !bf.acc || !bf2.acc || !bf.co || !bf2.co || C > FIN_MAX_C || relu_mask < 0 ||
      relu_mask > 1)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_apply2_rows_k, dim3(fin_rows_grid(M, C)), dim3(NT), 6 * C * sizeof(float), s, dy, y,
                     relu_mask, x, x2, st, st2, dx, dx2, M, C, bf, bf2);
  return hipGetLastError();
}

hipError_t bn_bwd_finalize(const float* part, int T, int C, float count, const float* st, const float* gamma,
                           float* dgamma, float* dbeta, float* co, hipStream_t s) {
  (void)gamma;
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_finalize_k, dim3(C / 8), dim3(FT), 0, s, part, T, C, count, st, dgamma, dbeta,
                     co);
  return hipGetLastError();
}

hipError_t bn_bwd_apply(const uint16_t* dy, const uint16_t* y, int relu_mask, const uint16_t* x, const float* st,
                        const float* co, uint16_t* dx, long M, int C, hipStream_t s, const BNBwdFin* bf) {
  const long n8 = M * C / 8;
  const BNBwdFin f = bf ? *bf : kNoBwdFin;
  if (f.acc && (!f.co || C > FIN_MAX_C)) return hipErrorInvalidValue;
  if (NT % (C / 8) == 0) {
    hipLaunchKernelGGL(bn_bwd_apply_rows_k, dim3(f.acc ? fin_rows_grid(M, C) : rows_grid(M, C, 16384)), dim3(NT),
                       f.acc ? 3 * C * sizeof(float) : 0, s, dy, y,
                       relu_mask, x, st, co, dx, M, C, f);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(bn_bwd_apply_k, dim3(grid_for(n8, NT, f.acc ? FIN_GRID_CAP : 8192)), dim3(NT),
                     f.acc ? 3 * C * sizeof(float) : 0, s, dy, y, relu_mask, x, st, co, dx, n8, C, f);
  return hipGetLastError();
}

hipError_t maxpool_fwd(const uint16_t* x, int N, int H, int W, int C, int ph, int pw, int sh, int sw, int pad_t,
                       int pad_l, int Ho, int Wo, uint16_t* y, uint8_t* arg, hipStream_t s) {
  if (C % 8 || ph * pw > 255) return hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  hipLaunchKernelGGL(maxpool_fwd_k, dim3(grid_for((long)N * Ho * Wo * C / 8)), dim3(NT), 0, s, x, g, y, arg);
  return hipGetLastError();
}

hipError_t maxpool_bwd(const uint16_t* dy, const uint8_t* arg, int N, int H, int W, int C, int ph, int pw, int sh,
                       int sw, int pad_t, int pad_l, int Ho, int Wo, uint16_t* dx, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  hipLaunchKernelGGL(maxpool_bwd_k, dim3(grid_for((long)N * H * W * C / 8)), dim3(NT), 0, s, dy, arg, g, dx);
  return hipGetLastError();
}

hipError_t bn_relu_maxpool_fwd(const uint16_t* x, const float* st, int N, int H, int W, int C, int ph, int pw, int sh,
                               int sw, int pad_t, int pad_l, int Ho, int Wo, uint16_t* y, uint8_t* arg, hipStream_t s,
                               const BNFin* fp) {
  if (C % 8 || ph * pw > 255) return hipErrorInvalidValue;
  const BNFin f = fp ? *fp : kNoFin;
  if (f.acc && (!f.st || C > FIN_MAX_C)) return hipErrorInvalidValue;
  const int cap = f.acc ? FIN_GRID_CAP : 8192;
  const size_t lds = f.acc ? 4 * C * sizeof(float) : 0;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  if (quad_pool_geo(g) && Ho % 2 == 0 && Wo % 2 == 0) {
    auto k = g.pt ? (g.pl ? bn_relu_maxpool_fwd_q_k<1, 1> : bn_relu_maxpool_fwd_q_k<1, 0>)
                  : (g.pl ? bn_relu_maxpool_fwd_q_k<0, 1> : bn_relu_maxpool_fwd_q_k<0, 0>);
    hipLaunchKernelGGL(k, dim3(grid_for((long)N * Ho * Wo * C / 32, NT, cap)), dim3(NT), lds, s, x, st, g, y, arg, f);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(bn_relu_maxpool_fwd_k, dim3(grid_for((long)N * Ho * Wo * C / 8, NT, cap)), dim3(NT), lds, s, x,
                     st, g, y, arg, f);
  return hipGetLastError();
}

hipError_t pool_bn_bwd_reduce(const uint16_t* dpool, const uint8_t* arg, int N, int H, int W, int C, int ph, int pw,
                              int sh, int sw, int pad_t, int pad_l, int Ho, int Wo, const uint16_t* x, const float* st,
                              float* part, int T, hipStream_t s, long long* acc, int acc_reps) {
  if (C % 8 || C / 8 > NT || (!part && !acc) || acc_reps < 1) return hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  const long M = (long)N * H * W, rows = (M + T - 1) / T;
  if (quad_pool_geo(g)) {
    const long nq = (long)N * Ho * Wo, qpb = (nq + T - 1) / T;
    auto k = g.pt ? (g.pl ? pool_bn_bwd_reduce_q_k<1, 1> : pool_bn_bwd_reduce_q_k<1, 0>)
                  : (g.pl ? pool_bn_bwd_reduce_q_k<0, 1> : pool_bn_bwd_reduce_q_k<0, 0>);
    hipLaunchKernelGGL(k, dim3(T), dim3(NT), 0, s, dpool, arg, g, x, st, part, nq, qpb, acc, acc_reps);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pool_bn_bwd_reduce_k, dim3(T), dim3(NT), 0, s, dpool, arg, g, x, st, part, M, rows, acc,
                     acc_reps);
  return hipGetLastError();
}

hipError_t pool_bn_bwd_apply(const uint16_t* dpool, const uint8_t* arg, int N, int H, int W, int C, int ph, int pw,
                             int sh, int sw, int pad_t, int pad_l, int Ho, int Wo, const uint16_t* x, const float* st,
                             const float* co, uint16_t* dx, hipStream_t s, const BNBwdFin* bfp) {
  if (C % 8) return hipErrorInvalidValue;
  const BNBwdFin f = bfp ? *bfp : kNoBwdFin;
  if (f.acc && (!f.co || C > FIN_MAX_C)) return hipErrorInvalidValue;
  const int cap = f.acc ? FIN_GRID_CAP : 8192;
  const size_t lds = f.acc ? 3 * C * sizeof(float) : 0;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  const long n8 = (long)N * H * W * C / 8;
  if (quad_pool_geo(g)) {
    const long nq8 = (long)N * Ho * Wo * C / 8;
    auto k = g.pt ? (g.pl ? pool_bn_bwd_apply_q_k<1, 1> : pool_bn_bwd_apply_q_k<1, 0>)
                  : (g.pl ? pool_bn_bwd_apply_q_k<0, 1> : pool_bn_bwd_apply_q_k<0, 0>);
    hipLaunchKernelGGL(k, dim3(grid_for(nq8, NT, cap)), dim3(NT), lds, s, dpool, arg, g, x, st, co, dx, nq8, f);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pool_bn_bwd_apply_k, dim3(grid_for(n8, NT, cap)), dim3(NT), lds, s, dpool, arg, g, x, st, co, dx,
                     n8, f);
  return hipGetLastError();
}

hipError_t gap_fwd(const uint16_t* x, int N, int HW, int C, void* y, int y_f32, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  if (C / 8 <= NT / 2 && HW >= 8) {
    hipLaunchKernelGGL(gap_fwd_img_k, dim3(N), dim3(NT), 0, s, x, HW, C, y, y_f32);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(gap_fwd_k, dim3(grid_for((long)N * C / 8)), dim3(NT), 0, s, x, N, HW, C, y, y_f32);
  return hipGetLastError();
}

hipError_t gap_bwd(const void* dy, int dy_f32, int N, int HW, int C, uint16_t* dx, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gap_bwd_k, dim3(grid_for((long)N * HW * C / 8)), dim3(NT), 0, s, dy, dy_f32, N, HW, C, dx);
  return hipGetLastError();
}

hipError_t relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dz, long n, hipStream_t s) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(relu_bwd_k, dim3(grid_for(n / 8)), dim3(NT), 0, s, dy, y, dz, n / 8);
  return hipGetLastError();
}

hipError_t act_fwd(const uint16_t* x, uint16_t* y, long n, int kind, hipStream_t s) {
  if (kind < 0 || kind > 2 || n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(act_fwd_k, dim3(grid_for((n + 7) / 8)), dim3(NT), 0, s, x, y, n, kind);
  return hipGetLastError();
}

hipError_t act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, int kind, hipStream_t s) {
  if (kind < 0 || kind > 2 || n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(act_bwd_k, dim3(grid_for((n + 7) / 8)), dim3(NT), 0, s, dy, y, dx, n, kind);
  return hipGetLastError();
}

hipError_t dropout(const uint16_t* x, uint16_t* y, long n, const Ctrl* ctrl, uint32_t seed, float rate,
                   hipStream_t s) {
  if (!(rate >= 0.f && rate < 1.f) || n <= 0) return hipErrorInvalidValue;
  const uint32_t thr = (uint32_t)fmin((double)rate * 4294967296.0, 4294967295.0);
  hipLaunchKernelGGL(dropout_k, dim3(grid_for((n + 7) / 8)), dim3(NT), 0, s, x, y, n, ctrl, seed, thr,
                     1.f / (1.f - rate));
  return hipGetLastError();
}

hipError_t avgpool_fwd(const uint16_t* x, int N, int H, int W, int C, int ph, int pw, int sh, int sw, int pad_t,
                       int pad_l, int Ho, int Wo, uint16_t* y, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  hipLaunchKernelGGL(avgpool_fwd_k, dim3(grid_for((long)N * Ho * Wo * C / 8)), dim3(NT), 0, s, x, g, y);
  return hipGetLastError();
}

hipError_t avgpool_bwd(const uint16_t* dy, int N, int H, int W, int C, int ph, int pw, int sh, int sw, int pad_t,
                       int pad_l, int Ho, int Wo, uint16_t* dx, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, ph, pw, sh, sw, pad_t, pad_l, Ho, Wo};
  hipLaunchKernelGGL(avgpool_bwd_k, dim3(grid_for((long)N * H * W * C / 8)), dim3(NT), 0, s, dy, g, dx);
  return hipGetLastError();
}

hipError_t add_bf16(const uint16_t* a, const uint16_t* b, uint16_t* out, long n, hipStream_t s) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(add_bf16_k, dim3(grid_for(n / 8)), dim3(NT), 0, s, a, b, out, n / 8);
  return hipGetLastError();
}

hipError_t cast_f32_bf16(const float* x, uint16_t* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_k, dim3(grid_for(n)), dim3(NT), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t cast_bf16_f32(const uint16_t* x, float* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_k, dim3(grid_for(n)), dim3(NT), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t cast_u8_bf16(const uint8_t* x, float scale, uint16_t* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_u8_bf16_k, dim3(grid_for(n)), dim3(NT), 0, s, x, scale, y, n);
  return hipGetLastError();
}

int colsum_splits(int M, int N) {
  // one pass while the column tiles alone give the chip enough blocks or M is short
  if (M <= 4096 || (N + 63) / 64 >= 64) return 1;
  int splits = (M + 1023) / 1024;
  return splits > 64 ? 64 : splits;
}
hipError_t colsum(const void* x, int x_f32, int M, int N, int ld, float* out, float* ws, hipStream_t s) {
  const int splits = colsum_splits(M, N);
  if (splits > 1 && !ws) return hipErrorInvalidValue;
  hipLaunchKernelGGL(colsum_k, dim3((N + 63) / 64, splits), dim3(NT), 0, s, x, x_f32, M, N, ld, out, ws);
  if (splits > 1) hipLaunchKernelGGL(colsum_fin_k, dim3((N + NT - 1) / NT), dim3(NT), 0, s, ws, splits, N, out);
  return hipGetLastError();
}

hipError_t softmax_xent(const float* logits, int ld, const int32_t* labels, int B, int K, float scale, const Ctrl* ctrl,
                        uint16_t* dlogits, float* tail, float* rows, hipStream_t s, float* bias_grad) {
  if (!rows || B < 1) return hipErrorInvalidValue;
  if (bias_grad && colsum_splits(B, K) != 1) return hipErrorInvalidValue;  // the fold keeps colsum's order
  hipLaunchKernelGGL(softmax_xent_k, dim3(B), dim3(NT), 0, s, logits, ld, labels, K, scale, ctrl, dlogits, tail, rows,
                     bias_grad);
  return hipGetLastError();
}

hipError_t sgd_flat(float* P, const float* G, float* V, uint16_t* Pb, long n, float lr, float momentum, int nesterov,
                    hipStream_t s) {
  hipLaunchKernelGGL(sgd_flat_k, dim3(grid_for(n, NT, 4096)), dim3(NT), 0, s, P, G, momentum != 0.f ? V : nullptr,
                     Pb, n, lr, momentum, nesterov);
  return hipGetLastError();
}

}  // namespace damd
