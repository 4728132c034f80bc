// BatchNorm statistics finalize from the fp64 accumulators (layer_ops.h BNFin), shared by
// the consumers that finalize in their prologue: the apply kernels (layer_ops.hip) and the
// direct conv that normalises its input on load (conv3x3.hip, GemmArgs::bnin).  One
// definition, so every consumer derives bitwise the same coefficients.
#pragma once
#include <hip/hip_runtime.h>

#include "damd_common.h"
#include "layer_ops.h"

namespace damd {

// Forward statistics: the replicas acc[r][2][C] (one word per value) summed as integers
// (exact, any order), then decoded; the sticky flag plane after the replicas
// (damd_common.h bnacc_flag) turns a channel's statistics into NaN.
// The replicas are read ACC_U at a time with every load issued before the first add: the
// words were just written by memory-side atomics, so each dependent round trip costs a
// memory latency -- a rolled loop (one wait per replica) made the finalize of every
// consumer prologue 8 + 2 serialised round trips.  (Clamped indices: the loads past reps
// re-read the last replica and are not added.)
constexpr int ACC_U = 8;
__device__ inline void acc_sums(const long long* acc, int reps, int C, int c, double& s, double& q) {
  long long ws = 0, wq = 0;
  reps = max(reps, 1);
  const long long f = acc[(size_t)reps * 2 * C + c];
  for (int r0 = 0; r0 < reps; r0 += ACC_U) {
    long long vs[ACC_U], vq[ACC_U];
#pragma unroll
    for (int u = 0; u < ACC_U; ++u) {
      const size_t r = (size_t)min(r0 + u, reps - 1);
      vs[u] = acc[r * 2 * C + c];
      vq[u] = acc[r * 2 * C + C + c];
    }
#pragma unroll
    for (int u = 0; u < ACC_U; ++u) {
      ws += r0 + u < reps ? vs[u] : 0ll;
      wq += r0 + u < reps ? vq[u] : 0ll;
    }
  }
  s = bnacc_value1(ws, f);
  q = bnacc_value1(wq, f);
}
// Backward sums: acc[r][4][C] (planes: sum hi, sum lo, second hi, second lo), the same way.
__device__ inline void acc_sums2(const long long* acc, int reps, int C, int c, double& s, double& q) {
  long long sh = 0, sl = 0, qh = 0, ql = 0;
  reps = max(reps, 1);
  const long long f = acc[(size_t)reps * 4 * C + c];
  for (int r0 = 0; r0 < reps; r0 += ACC_U) {
    long long v[ACC_U][4];
#pragma unroll
    for (int u = 0; u < ACC_U; ++u) {
      const long long* a = acc + (size_t)min(r0 + u, reps - 1) * 4 * C;
#pragma unroll
      for (int p = 0; p < 4; ++p) v[u][p] = a[p * C + c];
    }
#pragma unroll
    for (int u = 0; u < ACC_U; ++u) {
      const bool in = r0 + u < reps;
      sh += in ? v[u][0] : 0ll;
      sl += in ? v[u][1] : 0ll;
      qh += in ? v[u][2] : 0ll;
      ql += in ? v[u][3] : 0ll;
    }
  }
  s = bnacc_value2(sh, sl, f);
  q = bnacc_value2(qh, ql, f);
}
// coefficients of channel c (mean, invstd, scale, shift); pub: also published to st and
// the moving statistics (one thread per channel of the whole grid)
// (g, b: gamma[c] / beta[c], or 1 / 0 -- loaded by the caller, possibly early)
__device__ inline void bn_fin_sums_gb(const BNFin& f, int C, int c, double s, double q, float g, float b, bool pub,
                                      float& m, float& inv, float& sc, float& sh) {
  const double mean = s / (double)f.count;
  // (every multiply-add written as an explicit fma: the compiler's contraction choices may
  // differ between the kernels that inline this, and the moving statistics must not)
  double var = fma(-mean, mean, q / (double)f.count);
  if (var < 0.0) var = 0.0;
  m = (float)mean;
  const float v = (float)var;
  inv = rsqrtf(v + f.eps);
  sc = g * inv;
  sh = fmaf(-m, sc, b);
  if (pub) {
    f.st[c] = m;
    f.st[C + c] = inv;
    f.st[2 * C + c] = sc;
    f.st[3 * C + c] = sh;
    if (f.rmean) {
      f.rmean[c] = fmaf(f.rmean[c], f.mom, m * (1.f - f.mom));
      f.rvar[c] = fmaf(f.rvar[c], f.mom, v * (1.f - f.mom));
    }
  }
}
__device__ inline void bn_fin_sums(const BNFin& f, int C, int c, double s, double q, bool pub, float& m,
                                   float& inv, float& sc, float& sh) {
  bn_fin_sums_gb(f, C, c, s, q, f.gamma ? f.gamma[c] : 1.f, f.beta ? f.beta[c] : 0.f, pub, m, inv, sc, sh);
}

}  // namespace damd
