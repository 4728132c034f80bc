// Direct 3x3 / stride-1 / pad-1 convolution on MFMA with the input halo resident in LDS
// (gfx950 / MI355X): the ResNet-18 layer-1 / layer-2 convolutions,
// forward and backprop-input.
//
//   forward:         y[n][oh][ow][co] = sum_{kh,kw,ci} x[n][oh+kh-1][ow+kw-1][ci] W[kh][kw][ci][co]
//   backprop-input:  dx[n][ih][iw][ci] = sum_{kh,kw,co} dy[n][ih+1-kh][iw+1-kw][co] W[kh][kw][ci][co]
//                    (the same convolution of dy with the flipped taps)
//
// Why (rocprofv3 PMC, scripts/pmc_l2.sh): the implicit-GEMM conv kernels (conv_gemm.hip)
// stage one filter tap per k-step, so every input pixel crosses L2 -> LDS nine times:
// ~300 MB of L2 -> LDS traffic for a 25 MB layer-1 activation, 86-90 % L2 hits, ~10 TB/s
// achieved -- the kernels are bound by the LDS fill rate, not by the MFMAs (16-22 % of
// peak).  Here a block owns R whole output rows of one image and stages the (R+2) x (W+2)
// input halo of a 64-channel chunk ONCE; the nine taps read shifted windows of it, and only
// the weights stream through the LDS ring (one 64 x BN tile per tap and chunk).  A-side
// traffic drops ~9x (layer 1: BN = 64 tile, 256 output pixels per block).
//
// LDS images (all filled by LDS-DMA, swizzle applied to the source address, rule 21):
//   halo [pixel q][64 ch] bf16, 128 B per pixel; 16-byte chunk c of pixel q at slot
//     c ^ (q & 7): the 16 lanes of a fragment read (16 consecutive output pixels = 16
//     consecutive halo pixels at any tap) hit 8 distinct 16-B bank groups per 8 lanes;
//   weights: forward [64 k][BN] (mn-contiguous, tile::frag_mc transpose reads), backprop-
//     input [BN rows][64 k] (k-contiguous, as conv_gemm.hip's DGRAD operand).
// Tile: 256 threads = 4 waves, BN = 64 -> 256 x 64 (4 x 1 waves), BN = 128 -> 128 x 128
// (2 x 2), each wave 64 x 64 as 4 x 4 v_mfma_f32_16x16x32_bf16.  Rows of the tile beyond
// the block's R x W pixels read a clamped halo pixel and are masked in the epilogue.
// Epilogue: tile::epilogue (bias / residual add / BN statistics per tile / ReLU / bf16).
#include "bn_fin.h"
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

#include <cstdlib>

namespace damd {
namespace {

constexpr int NT = 256;

__device__ __attribute__((aligned(64))) uint4 g_zero16_c3[4];

// Diagnostics (conv3_stamps_enable): per block s_memrealtime at kernel start, after the
// first tap's operands landed, after the taps, after the epilogue -> g_c3_st[block][4]
constexpr int kC3StampBlocks = 4096;
__device__ int g_c3_on;
__device__ unsigned long long g_c3_st[kC3StampBlocks][4];

using tile::glds16;

// k-contiguous [rows][64] image swizzle (conv_gemm.hip kc_swz<64>)
__device__ __forceinline__ int kc64_swz(int r) { return r & 7; }

// halo prefetch of the next 64-channel chunk (double-buffered halo): LDS-DMA instructions
// per wave, uniform so that the stage waits can count them
constexpr int C3_HQ = 6;

// pf: issue prefetch() after tap KH's weight stage; the stage waits of the later taps then
// leave those C3_HQ newer DMA instructions in flight
// pre(): once, after the first tap's operands (and so the chunk's halo) have landed, before
// any tap reads the halo (the BN-input transform; it ends with its own barrier)
// wait until at most ahead x NQ + EXTRA DMA instructions of this wave are outstanding (the
// stage this tap reads has landed; `ahead` later stages -- and EXTRA halo-prefetch pieces --
// stay in flight); vmcnt takes an immediate, so one branch per possible `ahead`
template <int NQ, int EXTRA, int A>
__device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (A > 0) {
    if (ahead >= A) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A * NQ + EXTRA) : "memory");
      return;
    }
    wait_ahead<NQ, EXTRA, A - 1>(ahead);
  } else {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EXTRA) : "memory");
  }
}

template <int STAGES, int NQ, class Issue, class Compute, class Prefetch, class Pre>
__device__ __forceinline__ void tap_loop(Issue& issue, Compute& compute, Prefetch& prefetch, bool pf, Pre& pre) {
  constexpr int NK = 9, KH = NK - STAGES;
  static_assert(STAGES >= 2 && STAGES <= 8 && (STAGES - 2) * NQ + C3_HQ <= 63, "vmcnt range");
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue(s, s);
  for (int kt = 0; kt < NK; ++kt) {
    const int ahead = min(NK - 1 - kt, STAGES - 2);
    if (pf && kt > KH) wait_ahead<NQ, C3_HQ, STAGES - 2>(ahead);
    else wait_ahead<NQ, 0, STAGES - 2>(ahead);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < NK) issue((kt + STAGES - 1) % STAGES, kt + STAGES - 1);
    if (pf && kt == KH) prefetch();
    if (kt == 0) pre();
    compute(kt % STAGES, kt);
  }
}

// GemmArgs: A = gathered tensor (x, or dy for DGRAD) [Nimg][H][W][Cin] bf16, B = weights
// [3][3][.][.] bf16, C = output [Nimg][H][W][N]; M = Nimg*H*W; Cin = gathered channels
// (% 64), N = output channels (% BN); H, W the (shared) image size.  R output rows per
// block, tpi = ceil(H / R) row blocks per image; grid (N / BN, Nimg * tpi).
template <int BN, bool DGRAD, int EPI, int STAGES>
__global__ __launch_bounds__(NT, 2) void conv3_kernel(GemmArgs a, int R, int tpi, int hb2, int sft_off) {
  const bool stamps = g_c3_on != 0;
  unsigned long long st0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull, st1 = 0ull, st2 = 0ull;
  constexpr int WN = BN / 64, WM = 4 / WN, BM = WM * 64;
  constexpr int B_ST = BN * 64 * 2;
  constexpr int NB = B_ST / 4096;  // weight DMA instructions per wave per stage
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int H = a.H, W = a.W, SC = a.Cin, N = a.N;
  const int HW = W + 2;
  const int hpix = (R + 2) * HW;
  const int halo_bytes = (hpix * 128 + 1023) & ~1023;
  // hb2: two halo buffers (+ a 1 KiB sink for the padding DMA instructions): the next
  // chunk's halo is fetched by LDS-DMA during the current chunk's last taps
  char* halo = smem;
  char* sink = smem + 2 * halo_bytes;
  char* ring = smem + (hb2 ? 2 * halo_bytes + 1024 : halo_bytes);

  const int tn = blockIdx.x, tm = blockIdx.y;
  const int img = tm / tpi, oh0 = (tm - img * tpi) * R;
  const int reff = min(R, H - oh0);
  const int npx = reff * W;  // valid output pixels of this block
  const int n0 = tn * BN;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const uint16_t* src = (const uint16_t*)a.A;
  const uint16_t* wsrc = (const uint16_t*)a.B;
  const void* zero = tile::pinned_addr(g_zero16_c3);

  // halo pixel of output pixel p (row-major over the block's R x W) at tap offset 0
  int hbase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = min(wm * 64 + i * 16 + (lane & 15), npx - 1);
    const int r = p / W, c = p - r * W;
    hbase[i] = r * HW + c;
  }
  // weight DMA: forward rows k of BN*2 bytes (CPR chunks, RPI k-rows per 1-KB instruction);
  // backprop-input rows n of 64 k (8 chunks, 8 rows per instruction)
  constexpr int CPR = BN / 8, RPI = 64 / CPR;
  const int ca = (lane & 7) ^ kc64_swz(lane >> 3);
  const uint16_t* brow[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int q = wave + 4 * j;
    if constexpr (DGRAD) {
      const int n = n0 + 8 * q + (lane >> 3);  // row of the [BN][64] image
      brow[j] = wsrc + (long)n * a.kc + 8 * ca;
    } else {
      const int kr = q * RPI + lane / CPR;
      const int ch = (lane % CPR) ^ tile::mc_swz<BN>(kr);
      brow[j] = wsrc + (long)kr * N + n0 + 8 * ch;
    }
  }
  // halo DMA: instruction j covers halo pixels 8j .. 8j+7 (lane / 8), slot lane & 7
  const int nhi = halo_bytes / 1024;
  const uint16_t* img_base = src + (long)img * H * W * SC;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // BatchNorm on the input (a.bnin): thread t < SC requests channel t's accumulator
  // replicas now (in flight with the first halo / weight DMA); the first chunk's pre()
  // finalizes them into LDS (sft: [2][SC] floats past the halo / ring)
  const bool bnin = !DGRAD && a.bnin.acc != nullptr;
  float* sft = reinterpret_cast<float*>(smem + sft_off);
  constexpr int FR = 8;  // replicas held in registers (more: summed in pre())
  long long fs[FR], fq[FR];  // fixed-point words (damd_common.h bnacc_add1)
  long long ff = 0;          // the channel's sticky non-finite flag (plane after the replicas)
  float fg = 1.f, fb = 0.f;
  if (bnin && t < SC) {
    if (a.bnin.gamma) fg = a.bnin.gamma[t];
    if (a.bnin.beta) fb = a.bnin.beta[t];
    ff = a.bnin.acc[(size_t)max(a.bnin.reps, 1) * 2 * SC + t];
#pragma unroll
    for (int r = 0; r < FR; ++r) {
      const int rr = min(r, max(a.bnin.reps, 1) - 1);
      fs[r] = a.bnin.acc[(size_t)rr * 2 * SC + t];
      fq[r] = a.bnin.acc[(size_t)rr * 2 * SC + SC + t];
    }
  }

  const int nchunks = SC / 64;
  // halo instruction j (all 64 lanes): pixel q = 8j + lane / 8, 16-byte slot lane & 7 of
  // the swizzled image -> source (zeros outside the image / past the halo)
  auto halo_src = [&](int j, int c0) __attribute__((always_inline)) -> const void* {
    const int q = 8 * j + (lane >> 3);
    const int hr = q / HW, hc = q - hr * HW;
    const int ih = oh0 - 1 + hr, iw = hc - 1;
    const bool ok = q < hpix && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    const int cs = (lane & 7) ^ (q & 7);
    return ok ? (const void*)(img_base + ((long)ih * W + iw) * SC + c0 + 8 * cs) : zero;
  };
  const bool pf_on = hb2 && nchunks > 1 && nhi <= 4 * C3_HQ;
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    const int c0 = chunk * 64;
    char* hcur = halo + (pf_on ? (chunk & 1) * halo_bytes : 0);
    if (chunk) {  // every wave is done with the previous halo and weight stages
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    if (chunk == 0 || !pf_on)
      for (int j = wave; j < nhi; j += 4) glds16(halo_src(j, c0), hcur + j * 1024);
    // the next chunk's halo into the other buffer, from tap KH on
    auto prefetch = [&]() __attribute__((always_inline)) {
      char* nb = halo + ((chunk + 1) & 1) * halo_bytes;
#pragma unroll
      for (int u = 0; u < C3_HQ; ++u) {
        const int j = wave + 4 * u;
        glds16(halo_src(j, c0 + 64), j < nhi ? nb + j * 1024 : sink);
      }
    };
    auto issue = [&](int stage, int tap) __attribute__((always_inline)) {
      char* sb = ring + stage * B_ST;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const void* p;
        if constexpr (DGRAD) p = brow[j] + (long)tap * N * a.kc + c0;  // W[tap][n][co0 ..]
        else p = brow[j] + (long)(tap * SC + c0) * N;                    // W[tap][c0 + k][n0 ..]
        glds16(p, sb + (wave + 4 * j) * 1024);
      }
    };
    auto compute = [&](int stage, int tap) __attribute__((always_inline)) {
      if (stamps && chunk == 0 && tap == 0) st1 = __builtin_amdgcn_s_memrealtime();
      const char* ib = ring + stage * B_ST;
      const int kh = tap / 3, kw = tap - kh * 3;
      const int toff = DGRAD ? (2 - kh) * HW + (2 - kw) : kh * HW + kw;
      // both 32-deep k-steps' fragments in distinct registers: all of k-step 0's LDS reads
      // are issued before its MFMAs, k-step 1's overlap them (left to itself the scheduler
      // reused one A register quad, i.e. one LDS round trip per 4 MFMAs)
      bf16x8 af[2][4], bfr[2][4];
      auto load = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = hbase[i] + toff, c = 4 * kk + (lane >> 4);
          af[kk][i] = *reinterpret_cast<const bf16x8*>(hcur + q * 128 + 16 * (c ^ (q & 7)));
          if constexpr (DGRAD) {
            const int r = wn * 64 + i * 16 + (lane & 15);
            bfr[kk][i] = *reinterpret_cast<const bf16x8*>(ib + r * 128 + 16 * (c ^ kc64_swz(r)));
          } else {
            bfr[kk][i] = tile::frag_mc<BN>(ib + kk * 32 * BN * 2, wn * 64 + i * 16, lane);
          }
        }
      };
      auto mma = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[kk][j], af[kk][i], acc[i][j]);
      };
      load(0);
      __builtin_amdgcn_sched_barrier(0);
      load(1);
      mma(0);
      __builtin_amdgcn_sched_barrier(0);
      mma(1);
    };
    // BN input: y = bf16(relu(x * scale + shift)) in place over the chunk's halo (in-image
    // pixels only: the zero padding is the padding of y), exactly bn_apply's arithmetic
    auto pre = [&]() __attribute__((always_inline)) {
      if (!bnin) return;
      if (chunk == 0) {  // the statistics -> scale / shift of all SC channels
        const bool pub = tn == 0 && tm == 0;
        for (int c = t; c < SC; c += NT) {
          double s, q;
          float m, inv, sc, sh;
          if (c == t && a.bnin.reps <= FR) {  // requested at kernel start
            long long ws = fs[0], wq = fq[0];
#pragma unroll
            for (int r = 1; r < FR; ++r)
              if (r < a.bnin.reps) {
                ws += fs[r];
                wq += fq[r];
              }
            s = bnacc_value1(ws, ff);
            q = bnacc_value1(wq, ff);
            bn_fin_sums_gb(a.bnin, SC, c, s, q, fg, fb, pub, m, inv, sc, sh);
          } else {
            acc_sums(a.bnin.acc, a.bnin.reps, SC, c, s, q);
            bn_fin_sums(a.bnin, SC, c, s, q, pub, m, inv, sc, sh);
          }
          sft[c] = sc;
          sft[SC + c] = sh;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      // thread t: 16-byte slot t & 7 of pixels q = t / 8 + 32 k; that slot holds the same
      // 8 channels in every one of them (the swizzle c ^ (q & 7) is fixed: 32 k = 0 mod 8)
      int q = t >> 3;
      const int sl = t & 7, ch = c0 + 8 * (sl ^ (q & 7));
      float sc[8], sh[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc[e] = sft[ch + e];
        sh[e] = sft[SC + ch + e];
      }
      int hr = q / HW, hc = q - hr * HW;
      // TU pixels per pass: all their LDS reads issued before the first transform
      constexpr int TU = 4;
      for (; q < hpix; q += TU * (NT / 8)) {
        uint4 v[TU];
        bool ok[TU];
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          const int qu = q + u * (NT / 8);
          const int ih = oh0 - 1 + hr, iw = hc - 1;
          ok[u] = qu < hpix && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
          v[u] = *reinterpret_cast<const uint4*>(hcur + min(qu, hpix - 1) * 128 + 16 * sl);
          hc += NT / 8;
          while (hc >= HW) {
            hc -= HW;
            ++hr;
          }
        }
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          if (!ok[u]) continue;
          const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float lo = fmaxf(fmaf(__uint_as_float(w[k] << 16), sc[2 * k], sh[2 * k]), 0.f);
            const float hi = fmaxf(fmaf(__uint_as_float(w[k] & 0xffff0000u), sc[2 * k + 1], sh[2 * k + 1]), 0.f);
            o[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
          }
          *reinterpret_cast<uint4*>(hcur + (q + u * (NT / 8)) * 128 + 16 * sl) = uint4{o[0], o[1], o[2], o[3]};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    tap_loop<STAGES, NB>(issue, compute, prefetch, pf_on && chunk + 1 < nchunks, pre);
    // BN input: the block's output rows of y (this chunk's 64 channels) back to memory, from
    // the transformed halo interior (N-tile 0 only; the halo stays intact until the next
    // chunk's barrier)
    if (bnin && tn == 0 && a.bnin_y) {
      const int cl = t & 7;
      int p = t >> 3, r = p / W, c = p - r * W;
      uint16_t* yb = a.bnin_y + (long)(img * H + oh0) * W * SC + c0 + 8 * cl;
      for (; p < npx; p += NT / 8) {
        const int q = (r + 1) * HW + c + 1;
        *reinterpret_cast<uint4*>(yb + (long)p * SC) =
            *reinterpret_cast<const uint4*>(hcur + q * 128 + 16 * (cl ^ (q & 7)));
        c += NT / 8;
        while (c >= W) {
          c -= W;
          ++r;
        }
      }
    }
  }
  if (stamps) st2 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();  // `red` of the epilogue aliases the halo
  GemmArgs e = a;
  const int m0 = (img * H + oh0) * W;
  e.M = m0 + npx;  // rows past the block's pixels are masked
  tile::epilogue<BM, BN, EPI>(e, acc, m0, n0, tm, wm, wn, wave, lane, reinterpret_cast<float*>(smem));
  if (stamps && threadIdx.x == 0) {
    const int b = blockIdx.y * gridDim.x + blockIdx.x;
    if (b < kC3StampBlocks) {
      g_c3_st[b][0] = st0;
      g_c3_st[b][1] = st1;
      g_c3_st[b][2] = st2;
      g_c3_st[b][3] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

template <int BN>
constexpr int conv3_stages() { return BN == 64 ? 4 : 3; }
int halo_bytes_of(int R, int W) { return (((R + 2) * (W + 2)) * 128 + 1023) & ~1023; }

template <int BN, bool DG, int EPI, int ST>
hipError_t launch3_st(const GemmArgs& a, int R, hipStream_t s) {
  const int tpi = (a.H + R - 1) / R;
  const size_t hb = (size_t)halo_bytes_of(R, a.W), ring = (size_t)ST * BN * 64 * 2;
  auto k = conv3_kernel<BN, DG, EPI, ST>;
  static bool attr = false;  // once per instantiation (host-side, before any capture)
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nimg = a.M / (a.H * a.W);
  const long grid = (long)(a.N / BN) * nimg * tpi;
  // double-buffered halo: several chunks, the padded DMA count fits C3_HQ per wave, and no
  // residency lost -- the grid fits one block per CU anyway, or two blocks still fit a CU's
  // LDS (DAMD_CONV3_HB2=0: single buffer)
  const size_t sft = (!DG && a.bnin.acc) ? (size_t)2 * a.Cin * sizeof(float) : 0;  // BN-input scale / shift
  const size_t lds2 = 2 * hb + 1024 + ring + sft;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  const char* ev = getenv("DAMD_CONV3_HB2");
  const int hb2 = !(ev && ev[0] == '0') && a.Cin / 64 > 1 && (int)(hb / 1024) <= 4 * C3_HQ && lds2 <= 160 * 1024 &&
                  (grid <= cus || lds2 <= 80 * 1024);
  const size_t lds = hb2 ? lds2 : hb + ring + sft;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k, dim3(a.N / BN, nimg * tpi), dim3(NT), lds, s, a, R, tpi, hb2, (int)(lds - sft));
  return hipGetLastError();
}

// (two more weight stages -- a deeper ring, one block per CU where two no longer fit --
// measured slower in round 5: layer-3 forward 39.1 -> 40.2 us, backprop-input 27.8 -> 29.9
// us; scripts/conv3_probe.py)
template <int BN, bool DG, int EPI>
hipError_t launch3(const GemmArgs& a, int R, hipStream_t s) {
  return launch3_st<BN, DG, EPI, conv3_stages<BN>()>(a, R, s);
}

template <int BN, bool DG>
hipError_t launch3_epi(const GemmArgs& a, int epi, int R, hipStream_t s) {
  switch (epi) {
    case E_BF16: return launch3<BN, DG, E_BF16>(a, R, s);
    case E_BIAS | E_BF16: return launch3<BN, DG, E_BIAS | E_BF16>(a, R, s);
    case E_BIAS | E_RELU | E_BF16: return launch3<BN, DG, E_BIAS | E_RELU | E_BF16>(a, R, s);
    case E_RELU | E_BF16: return launch3<BN, DG, E_RELU | E_BF16>(a, R, s);
    case E_BF16 | E_STATS: return launch3<BN, DG, E_BF16 | E_STATS>(a, R, s);
    case E_BIAS | E_BF16 | E_STATS: return launch3<BN, DG, E_BIAS | E_BF16 | E_STATS>(a, R, s);
    case E_BF16 | E_ADD: return launch3<BN, DG, E_BF16 | E_ADD>(a, R, s);
    case E_BF16 | E_BNRED:
      if constexpr (DG) return launch3<BN, DG, E_BF16 | E_BNRED>(a, R, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t conv3_stamps_enable(int on) {
  if (on) {  // clear the previous launch's stamps (a smaller grid leaves stale rows otherwise)
    static unsigned long long zeros[kC3StampBlocks][4];
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_c3_st), zeros, sizeof(zeros));
    if (e != hipSuccess) return e;
  }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_c3_on), &on, sizeof(int));
}
// [blocks][4] stamps of the last conv3_kernel launch (host copy; synchronizes)
hipError_t conv3_stamps_read(unsigned long long* host, int blocks) {
  if (blocks > kC3StampBlocks) blocks = kC3StampBlocks;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_c3_st), (size_t)blocks * 4 * sizeof(unsigned long long));
}

// Output rows per block of the direct 3x3 kernel for an image of width W and tile width bn
// (0: the shape is not taken): the block's pixels R x W fill its BM = 64 * 4 / (bn / 64)
// MFMA rows, R <= H, and the halo + weight ring fit 80 KiB (two blocks per CU).
int conv3_rows(int H, int W, int bn) {
  if (bn != 64 && bn != 128) return 0;
  const int bm = bn == 64 ? 256 : 128;
  int R = bm / W;
  if (R < 1) return 0;
  if (R > H) R = H;
  const int st = bn == 64 ? conv3_stages<64>() : conv3_stages<128>();
  if (halo_bytes_of(R, W) + st * bn * 64 * 2 > 80 * 1024) return 0;
  return R;
}

// a.kc: the backprop-input weight row length (= the gathered channel count Cout), as for
// A_DGRAD64; geometry in a.H / a.W (input = output size), a.Cin = gathered channels
hipError_t conv3_launch(const GemmArgs& a, int dgrad, int epi, int bn, hipStream_t s) {
  const int R = conv3_rows(a.H, a.W, bn);
  if (R == 0 || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 || a.Cin % 64 || a.N % bn || a.M % (a.H * a.W))
    return hipErrorInvalidValue;
  if (dgrad && (a.kc != a.Cin || a.bnin.acc)) return hipErrorInvalidValue;
  if (epi & (E_SLAB | E_ATOMIC)) return hipErrorInvalidValue;
  // 64 -> 64 channels: the persistent weight-stationary strip kernel (conv3r.hip), the same
  // tiles / numerics
  if (bn == 64 && conv3r_ok(a, dgrad)) return conv3r_launch(a, dgrad, epi, s);
  // (>= 128 channels, measured and removed in round 6: one image strip per CU with the
  // halo resident and the weights streamed by 1 or 4 loader waves -- layer 2 forward 49 vs
  // 30 us, backprop-input 40 vs 24 us; layer 3 42 vs 36 / 36 vs 28 us against this kernel)
  // (a weight-stationary persistent variant for 64 -> 64 channels -- 72 KiB of weights +
  // two halos = the CU's 160 KiB -- measured slower on ResNet layer 1, forward 42 vs 33 us,
  // backprop-input 37 vs 29 us: one 4-wave block per CU cannot hide the LDS / MFMA
  // latencies that two streamed-weight blocks per CU overlap; removed in round 4)
  if (bn == 64) return dgrad ? launch3_epi<64, true>(a, epi, R, s) : launch3_epi<64, false>(a, epi, R, s);
  return dgrad ? launch3_epi<128, true>(a, epi, R, s) : launch3_epi<128, false>(a, epi, R, s);
}

}  // namespace damd
