// Persistent multi-step training kernel for the reference MNIST CNN (gfx950 / MI355X),
// one replica (world 1).  Model / optimizer as convnet_step2.hip (reference
// README.md:58-73): Conv2D(32,3x3)+ReLU -> MaxPool 2x2 -> Dense(64)+ReLU -> Dense(10) ->
// sparse softmax cross-entropy, SGD(lr, momentum, nesterov) on fp32 masters.
//
// Why: at B = 64 a launch-per-phase step is bound by launch boundaries and the memory
// round trips of every kernel prologue (the 2-launch step: ~24 us, of which ~13 us are
// boundaries and prologues).  Here ONE launch runs k training steps.  Each of the 57
// workgroups owns one slice of 3 pooled positions (96 rows of W1) for the whole launch:
//
//   * its W1 slice (fp32 master + velocity) lives in registers, laid out like the dW1
//     MFMA accumulators, so the SGD update is register-local and W1 never goes through
//     memory between steps; the bf16 operand copies are rebuilt in LDS;
//   * conv parameters and b1/W2/b2 are replicated: every workgroup applies the same
//     update to the same exactly-reduced gradient, so every copy stays bitwise identical;
//   * the next step's input rows are prefetched into registers during the current step.
//
// Per step, two grid-wide hand-offs (workgroups are co-resident: one per CU, 57 of the
// 256 CUs), each an int64 fixed-point sum with memory-side atomics (order independent:
// every copy and every replay gets the same bits) + a monotonic arrival counter:
//   B1  dense-1 partial sums of the 57 slices -> h for every workgroup (then the whole head
//       runs redundantly in every workgroup, as in convnet_step2.hip's backward kernel);
//   B2  conv weight/bias gradient partials -> the replicated conv update (a 57 x 320 fp32
//       slab written through (sc1) and summed in slice order by every workgroup: 320
//       addresses x 57 atomic adds serialised at the memory side cost more).
// Accumulators rotate over 3 buffers by global step: a buffer is zeroed (atomic exchange)
// after the barrier that retires its last reader and before the barrier that precedes its
// next adds.  Measured on MI355X (scripts/probe_grid_barrier.hip): one such hand-off of
// 4096 int64 per workgroup costs ~4 us; the bare counter barrier 1.35 us.
//
// Safety: every wait is bounded (s_memrealtime deadline); on expiry the workgroup sets
// ctrl->err and leaves the step loop, so a non-resident grid can never hang the GPU.  The
// host launches only when every workgroup fits on its own CU.
#include "convnet_dev.h"

namespace damd {
namespace convnet_p {
using namespace convnet;

constexpr int NT = 512;
constexpr int PPC = 3;              // pooled positions per slice
constexpr int KPC = PPC * 32 + 8;   // 104: bf16 pitch of as / w1t rows
constexpr int KDC = PPC * 32 + 4;   // 100: fp32 pitch of dps rows
constexpr int KCC = PPC * 32;       // 96: code bytes per image
constexpr int HPITCH = HID + 1;
constexpr int ZP = 11;

// LDS layout (bytes)
constexpr int L_XS = 0;                                   // [64][6][28] f32
constexpr int L_CS = L_XS + XS_BYTES;                     // [64][96] u8 argmax codes
constexpr int L_W1T = L_CS + CH * KCC;                    // [64][104] bf16 W1 slice^T (dense-1 B)
constexpr int L_W1S = L_W1T + HID * KPC * 2;              // [96][72] bf16 W1 slice (dP B)
constexpr int L_PT = L_W1S + PPC * 32 * HP * 2;           // [96][72] bf16 pooled^T (dW1 A)
constexpr int L_DHT = L_PT + PPC * 32 * HP * 2;           // [2][64][72] bf16 dh^T hi/lo
constexpr int L_DHS = L_DHT + 2 * HID * HP * 2;           // [2][64][72] bf16 dh hi/lo
constexpr int L_U = L_DHS + 2 * CH * HP * 2;              // union: as | head scratch | dps
constexpr int U_BYTES = CH * KDC * 4;                     // 25600 (the largest member)
constexpr int L_SPL = L_U + U_BYTES;                      // [716] f32 b1, W2, b2 (replicated)
constexpr int L_CW = L_SPL + 716 * 4;                     // [320] f32 conv params (replicated)
constexpr int L_LUT = L_CW + NCONV * 4;                   // [256] f32 k / 255
constexpr int L_Y = L_LUT + 256 * 4;                      // [64] int labels of the step (-1: none)
constexpr int LDS_BYTES = L_Y + CH * 4;
static_assert(CH * KPC * 2 <= U_BYTES, "as fits the union");
static_assert((CH * HPITCH + CH * ZP + 2 * CH + 16 * HID) * 4 <= U_BYTES, "head scratch fits the union");
static_assert(16 * NCONV * 4 <= PPC * 32 * HP * 2 + 2 * HID * HP * 2, "red fits pt + dht");
static_assert(LDS_BYTES <= 160 * 1024 - 64, "LDS budget");

struct PArgs {
  const void* X;
  const int* labels;
  float* P;
  float* V;
  Ctrl* ctrl;
  long long* hacc;    // [3][64][64]
  long long* hconv;   // [3][320] (unused: the conv gradient goes through cslab)
  float* cslab;       // [57][320] per-slice conv-gradient partials
  unsigned* sync;     // [2] monotonic arrival counters (B1, B2)
  int B, nsteps;
  unsigned long long timeout_ticks;
  unsigned long long* stamps;  // optional [256][16]
};

__device__ __forceinline__ bool grid_sync(unsigned* ctr, unsigned target, unsigned long long timeout, Ctrl* ctrl,
                                          int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics / stores performed
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long dl = __builtin_amdgcn_s_memrealtime() + timeout;
    int ok = 1;
    while ((int)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() > dl) {
        ok = 0;
        __hip_atomic_fetch_or(&ctrl->pad[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // error word
        break;
      }
    }
    *flag = ok;
  }
  __syncthreads();
  return *flag != 0;
}

__device__ __forceinline__ long long ld_i64(const long long* p) {
  return (long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void zero_i64(long long* p) {
  __hip_atomic_exchange(reinterpret_cast<unsigned long long*>(p), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool U8>
__global__ __launch_bounds__(NT) void persist(PArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int flag;
  const int s = blockIdx.x, NS = gridDim.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr16 = lane & 15, ko = 8 * (lane >> 4);
  const int B = a.B;
  const int p0 = s * PPC, p1 = min(NPOS, p0 + PPC), np = p1 - p0, K = np * 32;
  const int r0 = 2 * (p0 / PO), nrows = 2 * ((p1 - 1) / PO) + 4 - r0;
  float* xs = reinterpret_cast<float*>(smem + L_XS);
  uint8_t* cs = reinterpret_cast<uint8_t*>(smem + L_CS);
  uint16_t* w1t = reinterpret_cast<uint16_t*>(smem + L_W1T);
  uint16_t* w1s = reinterpret_cast<uint16_t*>(smem + L_W1S);
  uint16_t* pt = reinterpret_cast<uint16_t*>(smem + L_PT);
  uint16_t* dht = reinterpret_cast<uint16_t*>(smem + L_DHT);
  uint16_t* dhs = reinterpret_cast<uint16_t*>(smem + L_DHS);
  uint16_t* as = reinterpret_cast<uint16_t*>(smem + L_U);   // conv -> dense-1
  float* hs = reinterpret_cast<float*>(smem + L_U);          // head (after B1)
  float* zs = hs + CH * HPITCH;
  float* rl = zs + CH * ZP;
  float* rc = rl + CH;
  float* db1p = rc + CH;
  float* dps = reinterpret_cast<float*>(smem + L_U);          // dP -> conv gradient
  float* red = reinterpret_cast<float*>(smem + L_PT);         // conv-gradient partials (after dW1)
  float* spl = reinterpret_cast<float*>(smem + L_SPL);
  float* cw = reinterpret_cast<float*>(smem + L_CW);
  float* lut = reinterpret_cast<float*>(smem + L_LUT);
  int* ylds = reinterpret_cast<int*>(smem + L_Y);
  Ctrl* ctrl = a.ctrl;
  const Ctrl c = *ctrl;
  const bool mom = c.momentum != 0.f;
  const int dn = wave & 3, dm0 = wave >> 2;
  const unsigned g0 = (unsigned)c.pad[0];  // global persistent-step counter (buffer rotation, barrier targets)

  // ---- resident state ----
  float wr[MAXPP - 1][4], vr[MAXPP - 1][4];  // W1 slice (master, velocity) in the dW1 accumulator layout
#pragma unroll
  for (int i = 0; i < PPC; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * (dm0 + 2 * i) + 4 * (lane >> 4) + j, n = 16 * dn + lr16;
      const long idx = OFF_W1 + (long)(p0 * 32 + min(k, K - 1)) * HID + n;
      wr[i][j] = a.P[idx];
      vr[i][j] = mom ? a.V[idx] : 0.f;
    }
  const int tcl = min(tid, NCONV - 1);
  float cpv = a.P[tcl], cvv = a.V[tcl];
  const int e0 = tid, e1 = min(tid + NT, NSMALL - 1);
  float sv0 = a.V[OFF_B1 + e0], sv1 = a.V[OFF_B1 + e1];
  spl[e0] = a.P[OFF_B1 + e0];
  if (tid + NT < NSMALL) spl[tid + NT] = a.P[OFF_B1 + tid + NT];
  if (tid < NCONV) cw[tid] = cpv;
  if (U8 && tid < 256) lut[tid] = (float)tid / 255.f;
  // bf16 operand copies of the W1 slice
  auto write_w1_bf16 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPC; ++i) {
      if (i >= np) break;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 16 * (dm0 + 2 * i) + 4 * (lane >> 4) + j, n = 16 * dn + lr16;
        const uint16_t h = f2bf(wr[i][j]);
        w1t[n * KPC + k] = h;
        w1s[k * HP + n] = h;
      }
    }
  };
  write_w1_bf16();

  int cur = c.cursor;
  const long GB = c.global_batch;
  XStage<U8> xst;
  int ylab = 0;
  bool yval = false;
  auto load_x = [&](int cursor) __attribute__((always_inline)) {
    const long rb = (long)cursor * GB + c.row0;
    x_load<U8>(xst, a.X, rb, c.nsamples, B, CH, r0, nrows);
    const long g = rb + min(tid, CH - 1);
    yval = tid < CH && tid < B && g < c.nsamples;
    ylab = a.labels[max(0L, min(g, (long)c.nsamples - 1))];
  };
  load_x(cur);
  lds_barrier();  // lut
  x_store<U8>(xst, xs, lut);
  if (tid < CH) ylds[tid] = yval ? ylab : -1;
  lds_barrier();

  float L = 0.f, Cn = 0.f, Nn = 0.f;  // metric sums of this launch (workgroup 0)
  int steps_done = 0;
  Stamps sts;
  for (int it = 0; it < a.nsteps; ++it) {
    // lane / wave indices laundered through an empty asm once per step: the compiler cannot
    // hoist the hundreds of LDS / global addresses derived from them out of the step loop
    // (it did, and spilled them to scratch); recomputing them is a few VALU per use
    int tid_o = threadIdx.x;
    asm volatile("" : "+v"(tid_o));
    const int tid = tid_o, lane = tid & 63, lr16 = lane & 15, ko = 8 * (lane >> 4);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int dn = wave & 3, dm0 = wave >> 2;
    unsigned long long* st = (a.stamps != nullptr && it == a.nsteps - 1) ? a.stamps : nullptr;
    stamp(sts, st, 0);
    const unsigned g = g0 + (unsigned)it;
    long long* hacc = a.hacc + (long)(g % 3) * CH * HID;
    const long gstart = (long)cur * GB;
    const int gcount = (int)min(GB, (long)c.nsamples - gstart);
    const float inv = gcount > 0 ? 1.f / (float)gcount : 0.f;
    const int nxt = next_cursor(c, cur);

    // ---- conv + bias + ReLU + max-pool of 64 images on MFMA ----
    ConvFrag cf;
    conv_setup(cf, cw, lane);
    conv_pool(cf, xs, p0, np, r0, 6, wave, lane, [&](int bo, int plo, int ch, uint16_t hb, uint8_t cd) {
      as[bo * KPC + plo * 32 + ch] = hb;
      pt[(plo * 32 + ch) * HP + bo] = hb;
      cs[bo * KCC + plo * 32 + ch] = cd;
    });
    lds_barrier();
    stamp(sts, st, 1);
    // ---- dense-1 partial of the slice -> hacc (int64, x 2^32) ----
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const int t = wave + 8 * ti, mt = t >> 2, nt = t & 3;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < np; ++ks) {
        const bf16x8 av = ld_frag(as + (16 * mt + lr16) * KPC + ks * 32 + ko);
        const bf16x8 bv = ld_frag(w1t + (16 * nt + lr16) * KPC + ks * 32 + ko);
        acc = mfma16(av, bv, acc);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 16 * mt + 4 * (lane >> 4) + j;
        if (row < B) atomic_add_i64(hacc + row * HID + 16 * nt + lr16, to_fix(acc[j], HSCALE));
      }
    }
    // ---- B1: every slice's partial is in ----
    stamp(sts, st, 2);
    if (!grid_sync(a.sync, (unsigned)NS * (g + 1), a.timeout_ticks, ctrl, &flag)) break;
    stamp(sts, st, 3);
    // next step's rows: loads in flight across the whole backward half
    if (it + 1 < a.nsteps) load_x(nxt);
    // retire the buffer two steps back (its last reader passed B1 of this step)
    for (int i = s * NT + tid; i < CH * HID; i += NS * NT) zero_i64(a.hacc + (long)((g + 2) % 3) * CH * HID + i);
    // h = relu(hacc / 2^32 + b1)
    {
      const int r = tid >> 3, q = tid & 7;
      const bool rv = r < B;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = q * 8 + e;
        const long long v = rv ? ld_i64(hacc + r * HID + n) : 0;
        hs[r * HPITCH + n] = rv ? fmaxf(from_fix(v, HINV) + spl[n], 0.f) : 0.f;
      }
    }
    lds_barrier();
    stamp(sts, st, 4);
    // ---- head: logits (f32 MFMA) + softmax-xent / accuracy / dz (DPP row reductions) ----
    if (wave < 4) {
      const int mt = wave, kq = lane >> 4;
      float av[HID / 4], bv[HID / 4];
#pragma unroll
      for (int ks = 0; ks < HID / 4; ++ks) {
        const int k = 4 * ks + kq;
        av[ks] = hs[(16 * mt + lr16) * HPITCH + k];
        bv[ks] = spl[HID + k * NCLS + min(lr16, NCLS - 1)];
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < HID / 4; ++ks) acc = mfma4(av[ks], lr16 < NCLS ? bv[ks] : 0.f, acc);
      const float b2v = lr16 < NCLS ? spl[HID + HID * NCLS + lr16] : 0.f;
      float v[4], m[4], ex[4], lse[4];
      int am[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = lr16 < NCLS ? acc[j] + b2v : -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = row16_max(v[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) ex[j] = lr16 < NCLS ? __expf(v[j] - m[j]) : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) ex[j] = row16_sum(ex[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lse[j] = m[j] + __logf(ex[j]);
        am[j] = row16_min(v[j] == m[j] ? lr16 : 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * mt + 4 * kq + j;
        const int yv = ylds[r];
        const bool valid = yv >= 0;
        const int y = valid ? yv : 0;
        if (lr16 < NCLS) zs[r * ZP + lr16] = valid ? (__expf(v[j] - lse[j]) - (lr16 == y ? 1.f : 0.f)) * inv : 0.f;
        if (lr16 == y) rl[r] = valid ? (lse[j] - v[j]) : 0.f;
        if (lr16 == 0) rc[r] = (valid && am[j] == y) ? 1.f : 0.f;
      }
    }
    lds_barrier();
    // dh = (dz W2^T) * [h > 0] on f32 MFMA -> bf16 hi/lo in both operand layouts
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const int t = wave + 8 * ti, mt = t >> 2, nt = t & 3, kq = lane >> 4;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int k = 4 * ks + kq;
        const float av = k < NCLS ? zs[(16 * mt + lr16) * ZP + k] : 0.f;
        const float bv = k < NCLS ? spl[HID + (16 * nt + lr16) * NCLS + k] : 0.f;
        acc = mfma4(av, bv, acc);
      }
      const int n = 16 * nt + lr16, rb = 16 * mt + 4 * kq;
      uint16_t hi[4], lo[4];
      float dsum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = hs[(rb + j) * HPITCH + n] > 0.f ? acc[j] : 0.f;
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
      db1p[(4 * mt + kq) * HID + n] = dsum;
    }
    lds_barrier();
    stamp(sts, st, 5);
    // ---- b1/W2/b2: full gradient (fixed order, identical in every workgroup) into gsl
    //      (the w1t region: dense-1 is done, w1t is rebuilt after the update); metrics ----
    float* gsl = reinterpret_cast<float*>(w1t);  // [714] b1, W2, b2 gradients
    {
      if (wave < 4) {
        // dW2[k][c] = sum_r h[r][k] dz[r][c] on f32 MFMA: rows k = 16 wave .., K = rows r
        const int kq = lane >> 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int ks = 0; ks < CH / 4; ++ks) {
          const int r = 4 * ks + kq;
          const float av = hs[r * HPITCH + 16 * wave + lr16];
          const float bv = lr16 < NCLS ? zs[r * ZP + lr16] : 0.f;
          acc = mfma4(av, bv, acc);
        }
        if (lr16 < NCLS)
#pragma unroll
          for (int j = 0; j < 4; ++j) gsl[HID + (16 * wave + 4 * kq + j) * NCLS + lr16] = acc[j];
      } else if (wave == 4) {
        if (lane < NCLS) {  // db2
          float gg = 0.f;
          const float* zp = zs + lane;
#pragma unroll 4
          for (int r = 0; r < CH; ++r, zp += ZP) gg += *zp;
          gsl[HID + HID * NCLS + lane] = gg;
        }
      } else if (wave == 5) {  // db1
        float gg = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) gg += db1p[q * HID + lane];
        gsl[lane] = gg;
      } else if (wave == 6 && s == 0 && lane == 0) {
        float ls = 0.f, cr = 0.f;
#pragma unroll 4
        for (int r = 0; r < CH; ++r) {
          ls += rl[r];
          cr += rc[r];
        }
        L += ls;
        Cn += cr;
        Nn += (float)max(0, min(B, gcount - c.row0));
      }
      // dW1 = P^T dh: the slice's gradient straight into registers
      f32x4 accw[PPC];
#pragma unroll
      for (int i = 0; i < PPC; ++i) accw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < PPC; ++i) {
        if (i >= np) break;
        const int mt = dm0 + 2 * i;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 av = ld_frag(pt + (16 * mt + lr16) * HP + kk * 32 + ko);
          const bf16x8 bh = ld_frag(dht + (16 * dn + lr16) * HP + kk * 32 + ko);
          const bf16x8 bl = ld_frag(dht + HID * HP + (16 * dn + lr16) * HP + kk * 32 + ko);
          accw[i] = mfma16(av, bh, accw[i]);
          accw[i] = mfma16(av, bl, accw[i]);
        }
      }
      lds_barrier();  // spl reads of this step are done; the head scratch becomes dps
      stamp(sts, st, 6);
      {
        float wn, vn;
        sgd_update(spl[e0], gsl[e0], sv0, c.lr, c.momentum, c.nesterov, wn, vn);
        spl[e0] = wn;
        sv0 = vn;
        if (tid + NT < NSMALL) {
          sgd_update(spl[e1], gsl[e1], sv1, c.lr, c.momentum, c.nesterov, wn, vn);
          spl[e1] = wn;
          sv1 = vn;
        }
      }
      // dP[b][k] = sum_n (dh_hi + dh_lo)[b][n] W1[k][n]
      {
        const int pm = wave & 3;
#pragma unroll
        for (int i = 0; i < PPC; ++i) {
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
          for (int j = 0; j < 4; ++j) dps[(16 * pm + 4 * (lane >> 4) + j) * KDC + 16 * nt + lr16] = a4[j];
        }
      }
      // W1 slice update (registers), then its bf16 copies (w1t / w1s reads are done)
#pragma unroll
      for (int i = 0; i < PPC; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float wn, vn;
          sgd_update(wr[i][j], accw[i][j], vr[i][j], c.lr, c.momentum, c.nesterov, wn, vn);
          wr[i][j] = wn;
          vr[i][j] = vn;
        }
    }
    lds_barrier();
    stamp(sts, st, 7);
    write_w1_bf16();
    // ---- MaxPool + ReLU backward fused into the conv weight-gradient partial ----
    const int ch = tid & 31, grp = tid >> 5;
    float gw[9], gb = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) gw[t] = 0.f;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int bb = grp * 4 + ii;
      for (int pl = 0; pl < np; ++pl) {
        const int cd = cs[bb * KCC + pl * 32 + ch];
        const int pos = p0 + pl, py = pos / PO, px = pos - py * PO;
        const float dv0 = dps[bb * KDC + pl * 32 + ch];
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
#pragma unroll
    for (int t = 0; t < 9; ++t) red[grp * NCONV + t * NF + ch] = gw[t];
    red[grp * NCONV + OFF_BC + ch] = gb;
    lds_barrier();
    // this slice's conv-gradient partial -> its row of the slab (write-through sc1 stores)
    for (int i = tid; i < NCONV; i += NT) {
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc += red[r * NCONV + i];
      __hip_atomic_store(a.cslab + s * NCONV + i, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- B2: every slice's conv-gradient partial is in ----
    stamp(sts, st, 8);
    if (!grid_sync(a.sync + 1, (unsigned)NS * (g + 1), a.timeout_ticks, ctrl, &flag)) break;
    stamp(sts, st, 9);
    if (tid < NCONV) {
      // the 57 slice partials in slice order (sc1 loads, all issued before the sum): the
      // same sum in every workgroup.  The slab is rewritten only after B1 of the next step,
      // which no workgroup passes before every workgroup has finished these reads.
      float part[19], gsum = 0.f;
      for (int q0 = 0; q0 < NS; q0 += 19) {
#pragma unroll
        for (int q = 0; q < 19; ++q)
          part[q] = q0 + q < NS ? __hip_atomic_load(a.cslab + (q0 + q) * NCONV + tid, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : 0.f;
#pragma unroll
        for (int q = 0; q < 19; ++q) gsum += part[q];
      }
      float wn, vn;
      sgd_update(cpv, gsum, cvv, c.lr, c.momentum, c.nesterov, wn, vn);
      cpv = wn;
      cvv = vn;
      cw[tid] = wn;
    }
    // next step's input rows (prefetched since B1) and labels
    if (it + 1 < a.nsteps) {
      x_store<U8>(xst, xs, lut);
      if (tid < CH) ylds[tid] = yval ? ylab : -1;
    }
    cur = nxt;
    ++steps_done;
    lds_barrier();
    stamp(sts, st, 10);
    if (st != nullptr && tid == 0)
      for (int i = 0; i < 11; ++i) st[s * 16 + i] = sts.t[i];
  }

  // ---- write back the resident state (a complete, applied update: nothing pending) ----
#pragma unroll
  for (int i = 0; i < PPC; ++i) {
    if (i >= np) break;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * (dm0 + 2 * i) + 4 * (lane >> 4) + j, n = 16 * dn + lr16;
      const long idx = OFF_W1 + (long)(p0 * 32 + k) * HID + n;
      a.P[idx] = wr[i][j];
      if (mom) a.V[idx] = vr[i][j];
    }
  }
  if (s == 0) {
    if (tid < NCONV) {
      a.P[tid] = cpv;
      if (mom) a.V[tid] = cvv;
    }
    a.P[OFF_B1 + e0] = spl[e0];
    if (mom) a.V[OFF_B1 + e0] = sv0;
    if (tid + NT < NSMALL) {
      a.P[OFF_B1 + e1] = spl[e1];
      if (mom) a.V[OFF_B1 + e1] = sv1;
    }
    if (tid == 6 * 64) {  // the lane that kept the metric sums (wave 6, lane 0)
      ctrl->cursor = cur;
      ctrl->iterations = c.iterations + steps_done;
      ctrl->acc_loss = c.acc_loss + L;
      ctrl->acc_correct = c.acc_correct + Cn;
      ctrl->acc_count = c.acc_count + Nn;
      ctrl->pad[0] = (int)(g0 + (unsigned)steps_done);
      ctrl->pending = 0;
      ctrl->wpar = 0;
    }
  }
}

}  // namespace convnet_p

// ---------------------------------------------------------------------------------
size_t convnet_persist_lds() { return (size_t)convnet_p::LDS_BYTES; }

hipError_t convnet_persist_launch(const ConvNetBuffers& b, int B, int nsteps, long long* hacc3, long long* hconv3,
                                  unsigned* sync, double timeout_s, hipStream_t st) {
  // (phase stamps of the launch's last step go to b.stamps when the host asked for them)
  using namespace convnet;
  if (B < 1 || B > CH || nsteps < 1 || !hacc3 || !hconv3 || !sync) return hipErrorInvalidValue;
  int dev = 0, ncu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const int NS = convnet_num_slices(convnet_p::PPC);
  if (NS > ncu) return hipErrorInvalidConfiguration;  // workgroups must be co-resident
  convnet_p::PArgs a;
  a.X = b.X;
  a.labels = b.labels;
  a.P = b.P;
  a.V = b.V;
  a.ctrl = b.ctrl;
  a.hacc = hacc3;
  a.hconv = hconv3;
  a.cslab = reinterpret_cast<float*>(hconv3);  // host sizes the buffer for 57 x 320 floats
  a.sync = sync;
  a.B = B;
  a.nsteps = nsteps;
  a.timeout_ticks = (unsigned long long)(timeout_s * 1e8);
  a.stamps = b.stamps;
  if (b.x_u8)
    hipLaunchKernelGGL(convnet_p::persist<true>, dim3(NS), dim3(convnet_p::NT), convnet_p::LDS_BYTES, st, a);
  else
    hipLaunchKernelGGL(convnet_p::persist<false>, dim3(NS), dim3(convnet_p::NT), convnet_p::LDS_BYTES, st, a);
  return hipGetLastError();
}

hipError_t convnet_persist_set_lds_limits() {
  const void* fns[2] = {(const void*)convnet_p::persist<false>, (const void*)convnet_p::persist<true>};
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
