// Fused data-parallel training step for the reference MNIST CNN (gfx950 / MI355X).
//
// Model (reference README.md:58-73):
//   x[28,28,1] -> Conv2D(32,3x3,valid)+bias+ReLU -> MaxPool 2x2/2 -> Flatten(NHWC, 5408)
//   -> Dense(64)+bias+ReLU -> Dense(10) logits -> SparseCategoricalCrossentropy(from_logits)
//   optimizer: SGD(lr, momentum, nesterov) on fp32 master weights.
//
// One training step = 3 launches (+ one RCCL all-reduce of the flat gradient between
// steps when world > 1).  The optimizer update of step t is *deferred* into the kernels of
// step t+1 that first consume each parameter, so no separate SGD launch exists in the
// steady state (mnist_flush applies the last pending update before weights are read by
// the host):
//
//   F1 (grid NS, 512 thr): W1-slice SGD apply, conv SGD apply (registers), gather batch
//       rows from the device-resident dataset, conv+bias+ReLU+maxpool on VALU, keep the
//       pooled tile in LDS and multiply it by the matching W1 K-slice on MFMA
//       (16x16x32 bf16, one pooled position == one K step) -> split-K slab.
//   F2 (grid B/4, 256 thr, one wave per sample row, lane == hidden unit): split-K slab
//       reduction + b1 + ReLU, Dense(10), softmax-xent + accuracy, dz, dh, per-block
//       partials of dW2/db2/db1/metrics.  Last arriving block writes back the small
//       parameters (applying their deferred update) and reduces the partials into the
//       flat gradient buffer in a fixed order (deterministic).
//   F3 (grid NS, 512 thr): dW1 = P^T dh (MFMA, written straight into the gradient
//       buffer), dP = dh W1^T (MFMA, kept in LDS), MaxPool/ReLU backward via the stored
//       argmax code, conv weight/bias gradient partials; last arriver reduces them.
//
// Flat parameter / gradient layout = Keras weight order (so views of the master buffer
// are the Keras variables): conv2d/kernel (3,3,1,32), conv2d/bias, dense/kernel
// (5408,64), dense/bias, dense_1/kernel (64,10), dense_1/bias; gradient buffer tail
// carries [loss_sum, correct, count] so one all-reduce per step moves grads + metrics
// (SURVEY.md D5/D6).
#include "damd_common.h"
#include "convnet.h"

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
constexpr int REC = NSMALL + 2;              // F2 partial record: dW2, db2, db1 order below
constexpr int CH = 64;                       // images per chunk
constexpr int XR = 6;                        // staged input rows per image
constexpr int MAXPP = 4;                     // max pooled positions per F1/F3 block
static_assert(NPARAM == kConvNetNParam && NGRAD == kConvNetNGrad, "param count");

// ---------------------------------------------------------------------------------
// LDS budgets (bytes)
constexpr int XS_BYTES = CH * XR * IMG * 4;  // 43008
__host__ __device__ constexpr int kpitch(int pp) { return pp * 32 + 8; }

// Stage input rows [r0, r0+nrows) of the CH images of chunk `chunk` into xs[b][r][28].
__device__ __forceinline__ void stage_rows(float* xs, const float* __restrict__ X,
                                           const int* __restrict__ perm, const Ctrl& c,
                                           int B, int chunk, int r0, int nrows) {
  const long gstart = (long)c.cursor * c.global_batch + c.row0;
  const int per_img = nrows * 7;  // float4 per image
  for (int i = threadIdx.x; i < CH * per_img; i += blockDim.x) {
    const int b = i / per_img, rem = i - b * per_img, r = rem / 7, q = rem - r * 7;
    const int lb = chunk * CH + b;
    const long g = gstart + lb;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lb < B && g < c.nsamples) {
      const int sidx = perm[g];
      v = reinterpret_cast<const float4*>(X + (long)sidx * NPIX + (r0 + r) * IMG)[q];
    }
    reinterpret_cast<float4*>(xs + (b * XR + r) * IMG)[q] = v;
  }
}

// =================================================================================
// F1: deferred SGD on W1 slice + conv, conv/ReLU/pool fwd, dense-1 split-K partial.
// =================================================================================
__global__ __launch_bounds__(512) void f1_forward(
    const float* __restrict__ X, const int* __restrict__ perm, float* __restrict__ P,
    const float* __restrict__ G, float* __restrict__ V, const Ctrl* __restrict__ ctrl,
    uint16_t* __restrict__ pooled, uint8_t* __restrict__ code, float* __restrict__ slabs,
    int B, int PP) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int p0 = s * PP, p1 = min(NPOS, p0 + PP), np = p1 - p0, K = np * 32;
  const int KP = kpitch(PP);
  float* xs = reinterpret_cast<float*>(smem);
  uint16_t* as = reinterpret_cast<uint16_t*>(smem + XS_BYTES);   // [CH][KP]
  uint16_t* w1t = as + CH * KP;                                    // [HID][KP]
  float* cw = reinterpret_cast<float*>(w1t + HID * KP);            // [320]
  const Ctrl c = *ctrl;

  // 1. deferred SGD of this block's W1 rows (each row owned by exactly one block).
  {
    const int n4 = K * HID / 4;
    float4* P4 = reinterpret_cast<float4*>(P + OFF_W1 + p0 * 32 * HID);
    const float4* G4 = reinterpret_cast<const float4*>(G + OFF_W1 + p0 * 32 * HID);
    float4* V4 = reinterpret_cast<float4*>(V + OFF_W1 + p0 * 32 * HID);
    const bool mom = c.momentum != 0.f;
    for (int i = tid; i < n4; i += blockDim.x) {
      float4 w = P4[i], g = G4[i], v = mom ? V4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 wn, vn;
      sgd_update(w.x, g.x, v.x, c.lr, c.momentum, c.nesterov, wn.x, vn.x);
      sgd_update(w.y, g.y, v.y, c.lr, c.momentum, c.nesterov, wn.y, vn.y);
      sgd_update(w.z, g.z, v.z, c.lr, c.momentum, c.nesterov, wn.z, vn.z);
      sgd_update(w.w, g.w, v.w, c.lr, c.momentum, c.nesterov, wn.w, vn.w);
      P4[i] = wn;
      if (mom) V4[i] = vn;
      const int e = i * 4, kr = e >> 6, n = e & 63;
      w1t[(n + 0) * KP + kr] = f2bf(wn.x);
      w1t[(n + 1) * KP + kr] = f2bf(wn.y);
      w1t[(n + 2) * KP + kr] = f2bf(wn.z);
      w1t[(n + 3) * KP + kr] = f2bf(wn.w);
    }
  }
  // 2. conv parameters after their deferred update (not written back here: F2 does it).
  for (int i = tid; i < NCONV; i += blockDim.x) {
    float wn, vn;
    sgd_update(P[i], G[i], V[i], c.lr, c.momentum, c.nesterov, wn, vn);
    cw[i] = wn;
  }
  __syncthreads();

  const int cb = tid >> 3, cg = tid & 7;  // conv mapping: image, 4-channel group
  float wr[9][4], br[4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[t][j] = cw[t * NF + cg * 4 + j];
#pragma unroll
  for (int j = 0; j < 4; ++j) br[j] = cw[OFF_BC + cg * 4 + j];

  const int r0 = 2 * (p0 / PO);
  const int nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  const int wave = tid >> 6, lane = tid & 63;
  const int mt = wave & 3, nt0 = (wave >> 2) * 2;
  const int nchunks = (B + CH - 1) / CH;

  for (int chunk = 0; chunk < nchunks; ++chunk) {
    if (chunk) __syncthreads();
    stage_rows(xs, X, perm, c, B, chunk, r0, nrows);
    __syncthreads();
    // conv 3x3 + bias + ReLU + 2x2 max-pool for (image cb, channels 4cg..4cg+3)
    {
      const float* xb = xs + cb * XR * IMG;
      const int lb = chunk * CH + cb;
      for (int pl = 0; pl < np; ++pl) {
        const int pos = p0 + pl, py = pos / PO, px = pos - py * PO;
        const int ry = 2 * py - r0, cx = 2 * px;
        float pt[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) pt[i][j] = xb[(ry + i) * IMG + cx + j];
        float best[4];
        int arg[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int dy = q >> 1, dx = q & 1;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float a = br[j];
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx) a = fmaf(pt[dy + ky][dx + kx], wr[ky * 3 + kx][j], a);
            a = fmaxf(a, 0.f);
            if (q == 0 || a > best[j]) { best[j] = a; arg[j] = q; }
          }
        }
        uint16_t hb[4];
        uint32_t cd = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hb[j] = f2bf(best[j]);
          cd |= (uint32_t)(arg[j] | ((best[j] > 0.f) ? 4 : 0)) << (8 * j);
        }
        uint2 packed = make_uint2((uint32_t)hb[0] | ((uint32_t)hb[1] << 16),
                                  (uint32_t)hb[2] | ((uint32_t)hb[3] << 16));
        *reinterpret_cast<uint2*>(as + cb * KP + pl * 32 + cg * 4) = packed;
        if (lb < B) {
          *reinterpret_cast<uint2*>(pooled + (long)lb * FEAT + pos * NF + cg * 4) = packed;
          *reinterpret_cast<uint32_t*>(code + (long)lb * FEAT + pos * NF + cg * 4) = cd;
        }
      }
    }
    __syncthreads();
    // dense-1 split-K partial: slab[s][row][n] = sum_k pooled[row][k] * W1[k][n]
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int ar = 16 * mt + (lane & 15), ko = 8 * (lane >> 4);
    const int bn0 = 16 * nt0 + (lane & 15), bn1 = bn0 + 16;
    for (int ks = 0; ks < np; ++ks) {
      const bf16x8 a = ld_frag(as + ar * KP + ks * 32 + ko);
      const bf16x8 b0 = ld_frag(w1t + bn0 * KP + ks * 32 + ko);
      const bf16x8 b1 = ld_frag(w1t + bn1 * KP + ks * 32 + ko);
      acc0 = mfma16(a, b0, acc0);
      acc1 = mfma16(a, b1, acc1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 16 * mt + 4 * (lane >> 4) + j, lb = chunk * CH + row;
      if (lb < B) {
        float* dst = slabs + ((long)s * B + lb) * HID;
        dst[bn0] = acc0[j];
        dst[bn1] = acc1[j];
      }
    }
  }
}

// =================================================================================
// F2: dense-1 epilogue, dense-2, softmax-xent, dz / dh, small-param partials.
// =================================================================================
__global__ __launch_bounds__(256) void f2_head(
    const int* __restrict__ perm, const int* __restrict__ labels, float* __restrict__ P,
    float* __restrict__ G, float* __restrict__ V, Ctrl* __restrict__ ctrl,
    const float* __restrict__ slabs, float* __restrict__ dh, float* __restrict__ hpart, int B,
    int NS) {
  __shared__ __attribute__((aligned(16))) float lds[NSMALL + 2 + 4 * 64 + 4 * 16 + 4 * REC + 4];
  float* sp = lds;                      // updated b1[64], W2[640], b2[10]
  float* hs = sp + NSMALL + 2;          // [4][64]
  float* zs = hs + 4 * 64;              // [4][16]
  float* part = zs + 4 * 16;            // [4][REC]
  int* flag = reinterpret_cast<int*>(part + 4 * REC);
  const Ctrl c = *ctrl;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;

  for (int i = tid; i < NSMALL; i += blockDim.x) {
    float wn, vn;
    sgd_update(P[OFF_B1 + i], G[OFF_B1 + i], V[OFF_B1 + i], c.lr, c.momentum, c.nesterov, wn, vn);
    sp[i] = wn;
  }
  __syncthreads();
  const float* b1n = sp;
  const float* w2n = sp + HID;
  const float* b2n = sp + HID + HID * NCLS;

  const long gstart = (long)c.cursor * c.global_batch;
  const int gcount = (int)min((long)c.global_batch, (long)c.nsamples - gstart);
  const float inv = gcount > 0 ? 1.f / (float)gcount : 0.f;
  const int b = blockIdx.x * 4 + w;
  const long g = gstart + c.row0 + b;
  const bool valid = (b < B) && (g < c.nsamples);

  float h = 0.f;
  if (b < B) {
    const float* src = slabs + (long)b * HID + l;
    const long stride = (long)B * HID;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int sidx = 0;
    for (; sidx + 4 <= NS; sidx += 4) {
      a0 += src[(sidx + 0) * stride];
      a1 += src[(sidx + 1) * stride];
      a2 += src[(sidx + 2) * stride];
      a3 += src[(sidx + 3) * stride];
    }
    for (; sidx < NS; ++sidx) a0 += src[sidx * stride];
    h = (a0 + a1) + (a2 + a3);
  }
  h = fmaxf(h + b1n[l], 0.f);
  hs[w * 64 + l] = h;
  __syncthreads();
  if (l < 16) {
    float z = -INFINITY;
    if (l < NCLS) {
      z = b2n[l];
      for (int k = 0; k < HID; ++k) z = fmaf(hs[w * 64 + k], w2n[k * NCLS + l], z);
    }
    zs[w * 16 + l] = z;
  }
  __syncthreads();
  const int y = valid ? labels[perm[g]] : 0;
  float z[NCLS];
  float m = -INFINITY;
  int am = 0;
#pragma unroll
  for (int k = 0; k < NCLS; ++k) {
    z[k] = zs[w * 16 + k];
    if (z[k] > m) { m = z[k]; am = k; }
  }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < NCLS; ++k) se += __expf(z[k] - m);
  const float lse = m + __logf(se);
  float zy = z[0];
#pragma unroll
  for (int k = 1; k < NCLS; ++k) zy = (k == y) ? z[k] : zy;
  const float loss = lse - zy;
  float dz[NCLS];
#pragma unroll
  for (int k = 0; k < NCLS; ++k)
    dz[k] = valid ? (__expf(z[k] - lse) - (k == y ? 1.f : 0.f)) * inv : 0.f;
  float dhl = 0.f;
  if (h > 0.f) {
#pragma unroll
    for (int k = 0; k < NCLS; ++k) dhl = fmaf(dz[k], w2n[l * NCLS + k], dhl);
  }
  if (b < B) dh[(long)b * HID + l] = dhl;
  // per-row partial record: [0,640) dW2 (row-major [64][10]), [640,650) db2, [650,714) db1,
  // 714 loss, 715 correct
  float* pr = part + w * REC;
#pragma unroll
  for (int k = 0; k < NCLS; ++k) pr[l * NCLS + k] = h * dz[k];
  if (l < NCLS) {
    float d = 0.f;
#pragma unroll
    for (int k = 0; k < NCLS; ++k) d = (k == l) ? dz[k] : d;
    pr[640 + l] = d;
  }
  pr[650 + l] = dhl;
  if (l == 0) {
    pr[714] = valid ? loss : 0.f;
    pr[715] = (valid && am == y) ? 1.f : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < REC; i += blockDim.x)
    hpart[(long)blockIdx.x * REC + i] = (part[i] + part[REC + i]) + (part[2 * REC + i] + part[3 * REC + i]);

  if (!last_arriver(&ctrl->cnt_a, gridDim.x, flag)) return;

  // ---- last arriving block: write back deferred updates of small + conv params ----
  const bool mom = c.momentum != 0.f;
  for (int i = tid; i < NSMALL + NCONV; i += blockDim.x) {
    const int idx = i < NSMALL ? OFF_B1 + i : i - NSMALL;
    float wn, vn;
    sgd_update(P[idx], G[idx], V[idx], c.lr, c.momentum, c.nesterov, wn, vn);
    P[idx] = wn;
    if (mom) V[idx] = vn;
  }
  if (tid == 0) {  // fold previous step's all-reduced metrics into the epoch accumulators
    ctrl->acc_loss = c.acc_loss + G[OFF_LOSS];
    ctrl->acc_correct = c.acc_correct + G[OFF_CORR];
    ctrl->acc_count = c.acc_count + G[OFF_CNT];
  }
  __syncthreads();
  const int nb = gridDim.x;
  for (int i = tid; i < REC; i += blockDim.x) {
    float a = 0.f;
    for (int r = 0; r < nb; ++r) a += hpart[(long)r * REC + i];
    int dst;
    if (i < 640) dst = OFF_W2 + i;
    else if (i < 650) dst = OFF_B2 + (i - 640);
    else if (i < 714) dst = OFF_B1 + (i - 650);
    else dst = (i == 714) ? OFF_LOSS : OFF_CORR;
    G[dst] = a;
  }
  if (tid == 0) {
    const int nv = max(0, min(B, gcount - c.row0));
    G[OFF_CNT] = (float)nv;
    __hip_atomic_store(&ctrl->cnt_a, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// =================================================================================
// F3: dense-1 backward (dW1, dP), maxpool/ReLU backward, conv weight gradient.
// =================================================================================
__global__ __launch_bounds__(512) void f3_backward(
    const float* __restrict__ X, const int* __restrict__ perm, const float* __restrict__ P,
    float* __restrict__ G, Ctrl* __restrict__ ctrl, const uint16_t* __restrict__ pooled,
    const uint8_t* __restrict__ code, const float* __restrict__ dh, float* __restrict__ cpart,
    int B, int PP) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int p0 = s * PP, p1 = min(NPOS, p0 + PP), np = p1 - p0, K = np * 32;
  const int KD = PP * 32 + 4;      // dps pitch (f32)
  constexpr int HP = 72;           // bf16 pitch of 64-wide tiles
  float* xs = reinterpret_cast<float*>(smem);                              // [CH][XR][28]
  float* dps = reinterpret_cast<float*>(smem + XS_BYTES);                  // [CH][KD]
  uint16_t* pt = reinterpret_cast<uint16_t*>(dps + CH * KD);               // [PP*32][HP]
  uint16_t* dht = pt + PP * 32 * HP;                                       // [HID][HP]
  uint16_t* dhs = dht + HID * HP;                                          // [CH][HP]
  uint16_t* w1s = dhs + CH * HP;                                           // [PP*32][HP]
  float* red = reinterpret_cast<float*>(w1s + PP * 32 * HP);               // [16][320]
  int* flag = reinterpret_cast<int*>(red + 16 * NCONV);
  const Ctrl c = *ctrl;

  // W1 rows of this slice (already updated by F1 of this step) -> bf16 [k][n]
  for (int i = tid; i < K * HID / 4; i += blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(P + OFF_W1 + p0 * 32 * HID)[i];
    const int e = i * 4, kr = e >> 6, n = e & 63;
    uint2 pk = make_uint2((uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16),
                          (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16));
    *reinterpret_cast<uint2*>(w1s + kr * HP + n) = pk;
  }

  const int wave = tid >> 6, lane = tid & 63;
  const int ko = 8 * (lane >> 4), lr16 = lane & 15;
  // dW1 tiles: rows (k) 16*mt, cols (n) 16*nt; wave owns nt = wave&3, mt = (wave>>2) + 2i
  const int dn = wave & 3, dm0 = wave >> 2;
  f32x4 accw[MAXPP];
#pragma unroll
  for (int i = 0; i < MAXPP; ++i) accw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // conv-grad mapping: channel ch, image group grp (4 images)
  const int ch = tid & 31, grp = tid >> 5;
  float gw[9], gb = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) gw[t] = 0.f;
  const int r0 = 2 * (p0 / PO);
  const int nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  const int nchunks = (B + CH - 1) / CH;

  for (int chunk = 0; chunk < nchunks; ++chunk) {
    if (chunk) __syncthreads();
    // dh chunk -> dhs [b][n] and dht [n][b] (bf16)
    for (int i = tid; i < CH * HID; i += blockDim.x) {
      const int bb = i >> 6, n = i & 63, lb = chunk * CH + bb;
      const float v = lb < B ? dh[(long)lb * HID + n] : 0.f;
      const uint16_t hv = f2bf(v);
      dhs[bb * HP + n] = hv;
      dht[n * HP + bb] = hv;
    }
    // pooled slice -> pt [k][b]
    for (int i = tid; i < CH * K / 4; i += blockDim.x) {
      const int bb = i / (K / 4), kq = i - bb * (K / 4), lb = chunk * CH + bb;
      uint2 v = make_uint2(0u, 0u);
      if (lb < B) v = *reinterpret_cast<const uint2*>(pooled + (long)lb * FEAT + p0 * NF + kq * 4);
      pt[(kq * 4 + 0) * HP + bb] = (uint16_t)(v.x & 0xffff);
      pt[(kq * 4 + 1) * HP + bb] = (uint16_t)(v.x >> 16);
      pt[(kq * 4 + 2) * HP + bb] = (uint16_t)(v.y & 0xffff);
      pt[(kq * 4 + 3) * HP + bb] = (uint16_t)(v.y >> 16);
    }
    stage_rows(xs, X, perm, c, B, chunk, r0, nrows);
    __syncthreads();
    // dW1[k][n] += sum_b P[b][k] dh[b][n]   (static accumulator indices: no scratch)
#pragma unroll
    for (int i = 0; i < MAXPP; ++i) {
      if (i >= np) break;
      const int mt = dm0 + 2 * i;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 a = ld_frag(pt + (16 * mt + lr16) * HP + kk * 32 + ko);
        const bf16x8 bb = ld_frag(dht + (16 * dn + lr16) * HP + kk * 32 + ko);
        accw[i] = mfma16(a, bb, accw[i]);
      }
    }
    // dP[b][k] = sum_n dh[b][n] W1[k][n]   (row tile = wave&3, col tiles (wave>>2)+2i)
    {
      const int pm = wave & 3;
#pragma unroll
      for (int i = 0; i < MAXPP; ++i) {
        if (i >= np) break;
        const int nt = (wave >> 2) + 2 * i;
        f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 a = ld_frag(dhs + (16 * pm + lr16) * HP + kk * 32 + ko);
          const bf16x8 bb = ld_frag(w1s + (16 * nt + lr16) * HP + kk * 32 + ko);
          a4 = mfma16(a, bb, a4);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) dps[(16 * pm + 4 * (lane >> 4) + j) * KD + 16 * nt + lr16] = a4[j];
      }
    }
    __syncthreads();
    // maxpool + ReLU backward fused into the conv weight-gradient accumulation
    for (int ii = 0; ii < 4; ++ii) {
      const int bb = grp * 4 + ii, lb = chunk * CH + bb;
      if (lb >= B) break;
      for (int pl = 0; pl < np; ++pl) {
        const int pos = p0 + pl, py = pos / PO, px = pos - py * PO;
        const int cd = code[(long)lb * FEAT + pos * NF + ch];
        if (cd & 4) {
          const float d = dps[bb * KD + pl * 32 + ch];
          const int y0 = 2 * py + ((cd >> 1) & 1) - r0, x0 = 2 * px + (cd & 1);
          const float* xp = xs + (bb * XR + y0) * IMG + x0;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) gw[ky * 3 + kx] = fmaf(d, xp[ky * IMG + kx], gw[ky * 3 + kx]);
          gb += d;
        }
      }
    }
  }
  // dW1 straight into the flat gradient buffer (this block owns these rows)
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
  // conv partial: reduce 16 image groups in LDS
#pragma unroll
  for (int t = 0; t < 9; ++t) red[grp * NCONV + t * NF + ch] = gw[t];
  red[grp * NCONV + OFF_BC + ch] = gb;
  __syncthreads();
  for (int i = tid; i < NCONV; i += blockDim.x) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) a += red[r * NCONV + i];
    cpart[(long)s * NCONV + i] = a;
  }
  if (!last_arriver(&ctrl->cnt_b, gridDim.x, flag)) return;
  const int nb = gridDim.x;
  for (int i = tid; i < NCONV; i += blockDim.x) {
    float a = 0.f;
    for (int r = 0; r < nb; ++r) a += cpart[(long)r * NCONV + i];
    G[i] = a;
  }
  if (tid == 0) {
    ctrl->iterations = c.iterations + 1;
    ctrl->cursor = (c.wrap > 0 && c.cursor + 1 >= c.wrap) ? 0 : c.cursor + 1;
    __hip_atomic_store(&ctrl->cnt_b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// =================================================================================
// flush: apply the pending (deferred) update to every parameter, zero the gradient
// buffer and fold the pending metrics into the epoch accumulators.
// =================================================================================
__global__ __launch_bounds__(256) void flush_pending(float* __restrict__ P, float* __restrict__ G,
                                                     float* __restrict__ V, Ctrl* __restrict__ ctrl) {
  const Ctrl c = *ctrl;
  const bool mom = c.momentum != 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < NPARAM; i += gridDim.x * blockDim.x) {
    float wn, vn;
    sgd_update(P[i], G[i], V[i], c.lr, c.momentum, c.nesterov, wn, vn);
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
}

}  // namespace convnet

// ---------------------------------------------------------------------------------
// Host-side launchers (called from the C++ runtime; never allocate / sync here so the
// sequence can be captured into a hipGraph).
// ---------------------------------------------------------------------------------
int convnet_num_slices(int PP) { return (convnet::NPOS + PP - 1) / PP; }

size_t convnet_f1_lds(int PP) {
  const int KP = convnet::kpitch(PP);
  return convnet::XS_BYTES + (size_t)(convnet::CH + convnet::HID) * KP * 2 + convnet::NCONV * 4;
}
size_t convnet_f3_lds(int PP) {
  const int KD = PP * 32 + 4, HP = 72;
  return convnet::XS_BYTES + (size_t)convnet::CH * KD * 4 + (size_t)PP * 32 * HP * 2 * 2 +
         (size_t)(convnet::HID + convnet::CH) * HP * 2 + 16 * convnet::NCONV * 4 + 16;
}

hipError_t convnet_launch_step(const ConvNetBuffers& b, int B, int PP, hipStream_t st) {
  using namespace convnet;
  const int NS = convnet_num_slices(PP);
  hipLaunchKernelGGL(f1_forward, dim3(NS), dim3(512), convnet_f1_lds(PP), st, b.X, b.perm, b.P, b.G,
                     b.V, b.ctrl, b.pooled, b.code, b.slabs, B, PP);
  hipLaunchKernelGGL(f2_head, dim3((B + 3) / 4), dim3(256), 0, st, b.perm, b.labels, b.P, b.G, b.V,
                     b.ctrl, b.slabs, b.dh, b.hpart, B, NS);
  hipLaunchKernelGGL(f3_backward, dim3(NS), dim3(512), convnet_f3_lds(PP), st, b.X, b.perm, b.P, b.G,
                     b.ctrl, b.pooled, b.code, b.dh, b.cpart, B, PP);
  return hipGetLastError();
}

hipError_t convnet_launch_flush(const ConvNetBuffers& b, hipStream_t st) {
  hipLaunchKernelGGL(convnet::flush_pending, dim3(340), dim3(256), 0, st, b.P, b.G, b.V, b.ctrl);
  return hipGetLastError();
}

hipError_t convnet_set_lds_limits() {
  // F3 needs > 64 KiB of dynamic LDS.
  hipError_t e = hipFuncSetAttribute((const void*)convnet::f3_backward,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)convnet::f1_forward,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

}  // namespace damd
