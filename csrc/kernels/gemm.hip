// Generic bf16 MFMA GEMM / implicit-GEMM convolution for the per-layer (generic) path:
// Dense fwd/bwd, Conv2D fwd / backprop-input / backprop-filter for any Keras model
// (ResNet-18 in particular), NHWC activations, Keras weight
// layouts ([KH][KW][Cin][Cout], [in][out]).
//
//   C[M,N] (op)= sum_k A(m,k) * B(k,n)      bf16 operands, fp32 accumulation
//
// One kernel template, specialised by how the two operands are addressed:
//   A_KC     A stored [M][lda], k contiguous              (Dense fwd x, Dense dgrad dy)
//   A_IM2COL implicit im2col of an NHWC image, k=(kh,kw,ci) (Conv fwd)
//   A_DGRAD  implicit gather of dy for backprop-input, k=(kh,kw,co), stride 1|2
//   A_MC     A stored [K][lda], m contiguous (A^T)        (Dense wgrad: x^T)
//   A_WGRAD  implicit im2col^T, m=(kh,kw,ci), k=output pixel (Conv backprop-filter)
//   B_NC     B stored [K][ldb], n contiguous              (weights [K][N], dy for wgrad)
//   B_KC     B(k,n) = Bt[((k/kc)*N + n)*kc + k%kc]         (W^T per tap for dgrads)
//
// CDNA4 mapping: 256-thread workgroups (4 waves), every wave owns a 64x64 block of C as
// 4x4 v_mfma_f32_16x16x32_bf16 tiles, BK = 32.  Operands are staged global->registers->
// LDS with a register prefetch of tile k+1 during the MFMAs of tile k (double-buffered
// LDS, one LDS-only barrier per k-step).  k-contiguous sources land in a [rows][32] LDS
// image read with ds_read_b128; mn-contiguous sources land untransposed in a [32][cols]
// image and are read with the gfx950 transpose read ds_read_b64_tr_b16 (no transposing
// stores).  Both images are XOR-swizzled so every fragment read is bank-conflict free
// (swizzles checked exhaustively against the MI355X LDS lane groups).  The MFMA is issued
// with swapped operands (C^T = B^T A^T) so each lane ends up with 4 consecutive columns
// of one row: 8/16-byte vector stores in the epilogue.
//
// Epilogue (flags): +bias[n], ReLU, bf16 or fp32 output, fp32 atomic accumulation
// (split-K), and per-column partial sum / sum of squares of the (pre-ReLU) output per
// M-block (BatchNorm batch statistics without re-reading the activation).
#include "damd_common.h"
#include "gemm.h"
#include "gemm_tile.h"

namespace damd {
namespace {

constexpr int BK = 32;
constexpr int NT = 256;

using tile::ds_tr16;
using tile::frag_mc;
using tile::mc_off;

// ---- LDS images --------------------------------------------------------------------
// KC image: [rows][32] bf16, 64-B rows; 16-B chunk c of row r stored at chunk c^((r>>1)&3).
__device__ __forceinline__ int kc_off(int r, int c) { return r * 64 + 16 * (c ^ ((r >> 1) & 3)); }
// ---- per-thread operand loaders ----------------------------------------------------
// Each loader owns CH chunks (16 B each) of the tile; `load(kt)` fills registers for
// k-tile starting at k0, `store(lds)` writes them into the LDS image.

// KC-image chunk assignment: chunk c = t&3 of rows (t>>2) + 64*i.
// MC-image chunk assignment: chunk ch = t % CPR of rows t / CPR + (256/CPR)*i.

struct Geo {
  int H, W, C, Ho, Wo, KH, KW, stride, pad;
};

__device__ __forceinline__ uint4 ld16(const uint16_t* p, bool ok, const uint16_t* safe) {
  uint4 v = *reinterpret_cast<const uint4*>(ok ? p : safe);
  uint32_t m = ok ? 0xffffffffu : 0u;
  v.x &= m; v.y &= m; v.z &= m; v.w &= m;
  return v;
}

template <int MODE, int ROWS>
struct ALoader;

// A stored [M][lda], k contiguous
template <int ROWS>
struct ALoader<A_KC, ROWS> {
  static constexpr int CH = ROWS / 64;
  const uint16_t* base;
  const uint16_t* p[CH];
  bool rv[CH];
  int k;  // this thread's k within the matrix
  int K;
  __device__ void init(const GemmArgs& a, int m0, int kbeg) {
    base = (const uint16_t*)a.A;
    K = a.K;
    int t = threadIdx.x;
    k = kbeg + 8 * (t & 3);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int m = m0 + (t >> 2) + 64 * i;
      rv[i] = m < a.M;
      p[i] = base + (size_t)(rv[i] ? m : 0) * a.lda;
    }
  }
  __device__ void load(uint4* r, int kend) {
#pragma unroll
    for (int i = 0; i < CH; ++i) r[i] = ld16(p[i] + k, rv[i] && k < kend, base);
  }
  __device__ void advance() { k += BK; }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + kc_off((t >> 2) + 64 * i, t & 3)) = r[i];
  }
};

// implicit im2col of NHWC x: m = (n, oh, ow), k = (kh, kw, ci), C % 8 == 0
template <int ROWS>
struct ALoader<A_IM2COL, ROWS> {
  static constexpr int CH = ROWS / 64;
  const uint16_t* base;
  const uint16_t* img[CH];
  int ih0[CH], iw0[CH];
  bool rv[CH];
  int k, kh, kw, ci;
  Geo g;
  __device__ void init(const GemmArgs& a, int m0, int kbeg) {
    base = (const uint16_t*)a.A;
    g = Geo{a.H, a.W, a.Cin, a.Ho, a.Wo, a.KH, a.KW, a.stride, a.pad};
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int m = m0 + (t >> 2) + 64 * i;
      rv[i] = m < a.M;
      int mm = rv[i] ? m : 0;
      int ow = mm % g.Wo, tmp = mm / g.Wo, oh = tmp % g.Ho, n = tmp / g.Ho;
      img[i] = base + (size_t)n * g.H * g.W * g.C;
      ih0[i] = oh * g.stride - g.pad;
      iw0[i] = ow * g.stride - g.pad;
    }
    k = kbeg + 8 * (t & 3);
    int tap = k / g.C;
    ci = k - tap * g.C;
    kh = tap / g.KW;
    kw = tap - kh * g.KW;
  }
  __device__ void load(uint4* r, int kend) {
    bool kv = k < kend;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int ih = ih0[i] + kh, iw = iw0[i] + kw;
      bool ok = kv && rv[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      r[i] = ld16(img[i] + ((size_t)ih * g.W + iw) * g.C + ci, ok, base);
    }
  }
  __device__ void advance() {
    k += BK;
    ci += BK;
    while (ci >= g.C) {
      ci -= g.C;
      if (++kw == g.KW) { kw = 0; ++kh; }
    }
  }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + kc_off((t >> 2) + 64 * i, t & 3)) = r[i];
  }
};

// backprop-input gather of dy [N][Ho][Wo][Cout]: m = (n, ih, iw) of dx, k = (kh, kw, co)
// dy index oh = (ih + pad - kh) / stride when divisible and in range (stride 1 or 2).
template <int ROWS>
struct ALoader<A_DGRAD, ROWS> {
  static constexpr int CH = ROWS / 64;
  const uint16_t* base;
  const uint16_t* img[CH];
  int ihp[CH], iwp[CH];
  bool rv[CH];
  int k, kh, kw, co;
  Geo g;  // C here = Cout (the k-inner length)
  __device__ void init(const GemmArgs& a, int m0, int kbeg) {
    base = (const uint16_t*)a.A;
    g = Geo{a.H, a.W, a.Cin, a.Ho, a.Wo, a.KH, a.KW, a.stride, a.pad};
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int m = m0 + (t >> 2) + 64 * i;
      rv[i] = m < a.M;
      int mm = rv[i] ? m : 0;
      int iw = mm % g.W, tmp = mm / g.W, ih = tmp % g.H, n = tmp / g.H;
      img[i] = base + (size_t)n * g.Ho * g.Wo * g.C;
      ihp[i] = ih + g.pad;
      iwp[i] = iw + g.pad;
    }
    k = kbeg + 8 * (t & 3);
    int tap = k / g.C;
    co = k - tap * g.C;
    kh = tap / g.KW;
    kw = tap - kh * g.KW;
  }
  __device__ void load(uint4* r, int kend) {
    bool kv = k < kend;
    int sm = g.stride - 1, sh = g.stride >> 1;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int ohn = ihp[i] - kh, own = iwp[i] - kw;
      int oh = ohn >> sh, ow = own >> sh;
      bool ok = kv && rv[i] && ohn >= 0 && own >= 0 && !(ohn & sm) && !(own & sm) && oh < g.Ho && ow < g.Wo;
      r[i] = ld16(img[i] + ((size_t)oh * g.Wo + ow) * g.C + co, ok, base);
    }
  }
  __device__ void advance() {
    k += BK;
    co += BK;
    while (co >= g.C) {
      co -= g.C;
      if (++kw == g.KW) { kw = 0; ++kh; }
    }
  }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + kc_off((t >> 2) + 64 * i, t & 3)) = r[i];
  }
};

// A stored [K][lda] (m contiguous): MC image [32][ROWS]
template <int ROWS>
struct ALoader<A_MC, ROWS> {
  static constexpr int CPR = ROWS / 8;          // chunks per k-row
  static constexpr int RPP = NT / CPR;          // k-rows per pass
  static constexpr int CH = BK / RPP;
  const uint16_t* base;
  const uint16_t* p;
  bool mv;
  int k, lda;
  __device__ void init(const GemmArgs& a, int m0, int kbeg) {
    base = (const uint16_t*)a.A;
    lda = a.lda;
    int t = threadIdx.x;
    int m = m0 + 8 * (t % CPR);
    mv = m < a.M;
    p = base + (mv ? m : 0);
    k = kbeg + t / CPR;
  }
  __device__ void load(uint4* r, int kend) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int kk = k + RPP * i;
      r[i] = ld16(p + (size_t)kk * lda, mv && kk < kend, base);
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + mc_off<ROWS>(t / CPR + RPP * i, t % CPR)) = r[i];
  }
};

// backprop-filter: A(m = (kh,kw,ci), k = output pixel p = (n,oh,ow)) = x[n][oh*s-pad+kh][ow*s-pad+kw][ci]
template <int ROWS>
struct ALoader<A_WGRAD, ROWS> {
  static constexpr int CPR = ROWS / 8;
  static constexpr int RPP = NT / CPR;
  static constexpr int CH = BK / RPP;
  const uint16_t* base;
  bool mv;
  int kh, kw, ci;
  int pn[CH], poh[CH], pow_[CH], pk[CH];
  Geo g;
  __device__ void init(const GemmArgs& a, int m0, int kbeg) {
    base = (const uint16_t*)a.A;
    g = Geo{a.H, a.W, a.Cin, a.Ho, a.Wo, a.KH, a.KW, a.stride, a.pad};
    int t = threadIdx.x;
    int m = m0 + 8 * (t % CPR);
    mv = m < a.M;
    int mm = mv ? m : 0;
    int tap = mm / g.C;
    ci = mm - tap * g.C;
    kh = tap / g.KW;
    kw = tap - kh * g.KW;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int p = kbeg + t / CPR + RPP * i;
      pk[i] = p;
      pow_[i] = p % g.Wo;
      int tmp = p / g.Wo;
      poh[i] = tmp % g.Ho;
      pn[i] = tmp / g.Ho;
    }
  }
  __device__ void load(uint4* r, int kend) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int ih = poh[i] * g.stride - g.pad + kh, iw = pow_[i] * g.stride - g.pad + kw;
      bool ok = mv && pk[i] < kend && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      r[i] = ld16(base + (((size_t)pn[i] * g.H + ih) * g.W + iw) * g.C + ci, ok, base);
    }
  }
  __device__ void advance() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      pk[i] += BK;
      pow_[i] += BK;
      while (pow_[i] >= g.Wo) {
        pow_[i] -= g.Wo;
        if (++poh[i] == g.Ho) { poh[i] = 0; ++pn[i]; }
      }
    }
  }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + mc_off<ROWS>(t / CPR + RPP * i, t % CPR)) = r[i];
  }
};

template <int MODE, int COLS>
struct BLoader;

// B stored [K][ldb], n contiguous: MC image [32][COLS]
template <int COLS>
struct BLoader<B_NC, COLS> {
  static constexpr int CPR = COLS / 8;
  static constexpr int RPP = NT / CPR;
  static constexpr int CH = BK / RPP;
  const uint16_t* base;
  const uint16_t* p;
  bool nv;
  int k, ldb;
  __device__ void init(const GemmArgs& a, int n0, int kbeg) {
    base = (const uint16_t*)a.B;
    ldb = a.ldb;
    int t = threadIdx.x;
    int n = n0 + 8 * (t % CPR);
    nv = n < a.N;
    p = base + (nv ? n : 0);
    k = kbeg + t / CPR;
  }
  __device__ void load(uint4* r, int kend) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int kk = k + RPP * i;
      r[i] = ld16(p + (size_t)kk * ldb, nv && kk < kend, base);
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + mc_off<COLS>(t / CPR + RPP * i, t % CPR)) = r[i];
  }
};

// B(k, n) = Bt[((k / kc) * N + n) * kc + k % kc]: KC image [COLS][32]
template <int COLS>
struct BLoader<B_KC, COLS> {
  static constexpr int CH = COLS / 64;
  const uint16_t* base;
  bool nv[CH];
  int nn[CH];
  int k, tap, kk, kc, N;
  __device__ void init(const GemmArgs& a, int n0, int kbeg) {
    base = (const uint16_t*)a.B;
    kc = a.kc;
    N = a.N;
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int n = n0 + (t >> 2) + 64 * i;
      nv[i] = n < a.N;
      nn[i] = nv[i] ? n : 0;
    }
    k = kbeg + 8 * (t & 3);
    tap = k / kc;
    kk = k - tap * kc;
  }
  __device__ void load(uint4* r, int kend) {
    bool kv = k < kend;
#pragma unroll
    for (int i = 0; i < CH; ++i)
      r[i] = ld16(base + ((size_t)tap * N + nn[i]) * kc + kk, kv && nv[i], base);
  }
  __device__ void advance() {
    k += BK;
    kk += BK;
    while (kk >= kc) { kk -= kc; ++tap; }
  }
  __device__ void store(char* lds, const uint4* r) {
    int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) *reinterpret_cast<uint4*>(lds + kc_off((t >> 2) + 64 * i, t & 3)) = r[i];
  }
};

template <int MODE> struct IsKC { static constexpr bool v = (MODE == A_KC || MODE == A_IM2COL || MODE == A_DGRAD); };

// fragment for 16 rows/cols starting at r0 of a KC image: lane gets row r0+(l&15), k 8(l>>4)..+7
__device__ __forceinline__ bf16x8 frag_kc(const char* img, int r0, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + kc_off(r0 + (lane & 15), lane >> 4));
}
template <int BM, int BN, int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;  // wave grid (each wave 64x64)
  static_assert(WM * 64 == BM, "tile shape");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];
  __shared__ float red[2][4][64];

  // XCD-aware tile order: consecutive workgroups are dispatched round-robin over the 8
  // XCDs; remap so that the N-tiles of one M-panel (which share the A rows) run on the
  // same XCD (same L2).
  const int tiles_n = gridDim.x, tiles = gridDim.x * gridDim.y;
  int lin = blockIdx.y * tiles_n + blockIdx.x;
  if ((tiles & 7) == 0) lin = (lin & 7) * (tiles >> 3) + (lin >> 3);
  const int tn = lin % tiles_n, tm = lin / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // split-K range
  const int kbeg = blockIdx.z * a.k_per_split;
  const int kend = min(a.K, kbeg + a.k_per_split);
  if (kbeg >= kend) return;
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;

  ALoader<AMODE, BM> al;
  BLoader<BMODE, BN> bl;
  al.init(a, m0, kbeg);
  bl.init(a, n0, kbeg);
  uint4 ra[ALoader<AMODE, BM>::CH], rb[BLoader<BMODE, BN>::CH];

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  al.load(ra, kend);
  bl.load(rb, kend);
  al.store(smem, ra);
  bl.store(smem + A_BYTES, rb);
  lds_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * (A_BYTES + B_BYTES);
    char* nxt = smem + ((kt + 1) & 1) * (A_BYTES + B_BYTES);
    const bool more = kt + 1 < nk;
    if (more) {
      al.advance();
      bl.advance();
      al.load(ra, kend);
      bl.load(rb, kend);
    }
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (IsKC<AMODE>::v) af[i] = frag_kc(cur, wm * 64 + i * 16, lane);
      else af[i] = frag_mc<BM>(cur, wm * 64 + i * 16, lane);
      if constexpr (BMODE == B_KC) bfr[i] = frag_kc(cur + A_BYTES, wn * 64 + i * 16, lane);
      else bfr[i] = frag_mc<BN>(cur + A_BYTES, wn * 64 + i * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    if (more) {
      al.store(nxt, ra);
      bl.store(nxt + A_BYTES, rb);
    }
    lds_barrier();
  }

  tile::epilogue<BM, BN, EPI>(a, acc, m0, n0, tm, wm, wn, wave, lane, &red[0][0][0]);
}

template <int BM, int BN, int AM, int BMo, int EPI>
hipError_t launch_t(const GemmArgs& a, int splits, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AM, BMo, EPI>), grid, dim3(NT), 0, s, a);
  return hipGetLastError();
}

template <int BM, int BN, int AM, int BMo>
hipError_t launch_epi(const GemmArgs& a, int epi, int splits, hipStream_t s) {
  switch (epi) {
    case 0: return launch_t<BM, BN, AM, BMo, 0>(a, splits, s);
    case E_BF16: return launch_t<BM, BN, AM, BMo, E_BF16>(a, splits, s);
    case E_BIAS: return launch_t<BM, BN, AM, BMo, E_BIAS>(a, splits, s);
    case E_BIAS | E_RELU: return launch_t<BM, BN, AM, BMo, E_BIAS | E_RELU>(a, splits, s);
    case E_BIAS | E_BF16: return launch_t<BM, BN, AM, BMo, E_BIAS | E_BF16>(a, splits, s);
    case E_BIAS | E_RELU | E_BF16: return launch_t<BM, BN, AM, BMo, E_BIAS | E_RELU | E_BF16>(a, splits, s);
    case E_RELU: return launch_t<BM, BN, AM, BMo, E_RELU>(a, splits, s);
    case E_RELU | E_BF16: return launch_t<BM, BN, AM, BMo, E_RELU | E_BF16>(a, splits, s);
    case E_ATOMIC: return launch_t<BM, BN, AM, BMo, E_ATOMIC>(a, splits, s);
    case E_SLAB: return launch_t<BM, BN, AM, BMo, E_SLAB>(a, splits, s);
    case E_BF16 | E_STATS: return launch_t<BM, BN, AM, BMo, E_BF16 | E_STATS>(a, splits, s);
    case E_BIAS | E_BF16 | E_STATS: return launch_t<BM, BN, AM, BMo, E_BIAS | E_BF16 | E_STATS>(a, splits, s);
    case E_BF16 | E_ADD: return launch_t<BM, BN, AM, BMo, E_BF16 | E_ADD>(a, splits, s);
    default: return hipErrorInvalidValue;
  }
}

template <int AM, int BMo>
hipError_t launch_tile(const GemmArgs& a, int epi, int splits, int tile, hipStream_t s) {
  if (tile == 1) return launch_epi<256, 64, AM, BMo>(a, epi, splits, s);
  return launch_epi<128, 128, AM, BMo>(a, epi, splits, s);
}

// dst[i] += sum_s slab[s][i].  Block = 16 float4 columns x 16 split groups: thread
// (g, e) sums splits g, g+16, ... of element e, then the 16 partials are combined in LDS
// in fixed order (deterministic), so even a 9k-float4 gradient with 170 splits keeps
// ~600 blocks streaming the slabs.
constexpr int RED_E = 16, RED_G = NT / RED_E;
// Unpad mode (c1p > 0): the slab rows are a padded [R][c1p][c2p4] float4 layout whose
// entries with c1 >= u_c1 or c2 >= u_c24 are junk; the rest land at [R][u_c1][u_c24] in dst
// (the packed-tap stem's weight gradient straight into the gradient buffer: no unpad_add
// launch after the reduce).
__global__ __launch_bounds__(NT) void splitk_reduce_k(const float4* __restrict__ slab, int splits, long n4,
                                                     float4* __restrict__ dst, int accumulate, int u_c1 = 0,
                                                     int u_c24 = 0, int u_c1p = 0, int u_c2p4 = 0) {
  __shared__ float4 part[RED_G][RED_E];
  const int e = threadIdx.x % RED_E, g = threadIdx.x / RED_E;
  const long i = blockIdx.x * (long)RED_E + e;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
#pragma unroll 4
    for (int sp = g; sp < splits; sp += RED_G) {
      const float4 v = slab[(size_t)sp * n4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  part[g][e] = acc;
  __syncthreads();
  long di = i;
  if (u_c1p > 0) {
    const int c2 = (int)(i % u_c2p4);
    const long t = i / u_c2p4;
    const int c1 = (int)(t % u_c1p);
    di = c1 < u_c1 && c2 < u_c24 ? (t / u_c1p * u_c1 + c1) * u_c24 + c2 : -1;
  }
  if (g == 0 && i < n4 && di >= 0) {
    const long i = di;
    float4 d = accumulate ? dst[i] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < RED_G; ++q) {
      d.x += part[q][e].x; d.y += part[q][e].y; d.z += part[q][e].z; d.w += part[q][e].w;
    }
    dst[i] = d;
  }
}

// Split-K epilogue for the bf16-output GEMMs (conv fwd, conv dgrad): out[m][n] =
// relu?( sum_s slab[s][m][n] + bias[n] + R[m][n] ) as bf16, plus per-column sum / sum of
// squares of the stored (pre-ReLU, bf16-rounded) values per block of `rb` rows
// (BatchNorm batch statistics: stats[blk][2][N]).  Thread = 8 columns of one row.
__global__ __launch_bounds__(NT) void splitk_finish_k(const float* __restrict__ slab, int S, int M, int N,
                                                      const float* __restrict__ bias, const uint16_t* R, int relu,
                                                      float* __restrict__ stats, int rb, uint16_t* out, int ldc,
                                                      long long* __restrict__ stats_acc, int reps) {
  __shared__ float red[2][NT * 8];
  // blockIdx.y: band of up to NT x 8 columns (wide layers: N > 2048)
  const int c0 = blockIdx.y * NT * 8, Nb = min(N - c0, NT * 8);
  const int cg = Nb / 8, rp = NT / cg;  // column groups, rows per pass
  const int t = threadIdx.x, g = t % cg, r0 = t / cg;
  const int n = c0 + 8 * g;
  const long row0 = (long)blockIdx.x * rb, row1 = min((long)M, row0 + rb);
  float cs[8], cq[8], bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] = cq[e] = 0.f;
    bv[e] = 0.f;
  }
  if (bias && r0 < rp) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = bias[n + e];
  }
  const size_t plane = (size_t)M * N;
  if (r0 < rp) {
    // FR rows per pass and the first FS splits of each requested together, before the
    // pass's stores (R may alias `out`, so the compiler kept every load behind the previous
    // row's store: rows x splits dependent round trips per thread); splits summed in
    // ascending order as before, so the bits are unchanged
    constexpr int FR = 2, FS = 4;
    for (long mb = row0 + r0; mb < row1; mb += FR * rp) {
      float4 la[FR][FS], lb[FR][FS];
      uint4 rq[FR];
#pragma unroll
      for (int f = 0; f < FR; ++f) {
        const long m = min(mb + f * rp, row1 - 1);
        const float* p = slab + (size_t)m * N + n;
#pragma unroll
        for (int u = 0; u < FS; ++u) {
          const float* q = p + (size_t)min(u, S - 1) * plane;
          la[f][u] = *reinterpret_cast<const float4*>(q);
          lb[f][u] = *reinterpret_cast<const float4*>(q + 4);
        }
        if (R) rq[f] = *reinterpret_cast<const uint4*>(R + (size_t)m * ldc + n);
      }
#pragma unroll
      for (int f = 0; f < FR; ++f) {
        const long m = mb + f * rp;
        if (m >= row1) break;
        float v[8];
        const float* p = slab + (size_t)m * N + n;
        float4 a = la[f][0], b = lb[f][0];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
        for (int u = 1; u < FS; ++u) {
          if (u >= S) break;
          a = la[f][u];
          b = lb[f][u];
          v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
        }
        for (int sp = FS; sp < S; ++sp) {
          const float* q = p + sp * plane;
          a = *reinterpret_cast<const float4*>(q);
          b = *reinterpret_cast<const float4*>(q + 4);
          v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
        }
        if (R) {
          const uint4 r = rq[f];
          const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[2 * k] += __uint_as_float(w[k] << 16);
            v[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
          }
        }
        uint32_t pk[4];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint16_t h = f2bf(v[e] + bv[e]);
          const float x = bf2f(h);  // statistics of the stored value
          cs[e] += x;
          cq[e] += x * x;
          const uint16_t o = relu ? f2bf(fmaxf(x, 0.f)) : h;
          if (e & 1) pk[e >> 1] |= (uint32_t)o << 16;
          else pk[e >> 1] = o;
        }
        *reinterpret_cast<uint4*>(out + (size_t)m * ldc + n) = uint4{pk[0], pk[1], pk[2], pk[3]};
      }
    }
  }
  if (!stats && !stats_acc) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][t * 8 + e] = r0 < rp ? cs[e] : 0.f;
    red[1][t * 8 + e] = r0 < rp ? cq[e] : 0.f;
  }
  __syncthreads();
  for (int c = t; c < Nb; c += NT) {
    const int gg = c / 8, e = c % 8;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < rp; ++q) {
      a += red[0][(q * cg + gg) * 8 + e];
      b += red[1][(q * cg + gg) * 8 + e];
    }
    if (stats_acc) {
      long long* acc = stats_acc + (size_t)(blockIdx.x % reps) * 2 * N;  // forward statistics
      long long* flag = stats_acc + (size_t)reps * 2 * N + c0 + c;       // sticky plane
      bnacc_add1(acc + c0 + c, flag, a);
      bnacc_add1(acc + N + c0 + c, flag, b);
    } else {
      stats[(size_t)blockIdx.x * 2 * N + c0 + c] = a;
      stats[(size_t)blockIdx.x * 2 * N + N + c0 + c] = b;
    }
  }
}

// Few splits over a large gradient (the ResNet weight gradients: 2-16 slabs of 0.15-2.4 M
// floats): one float4 per thread, all slab loads issued before the first add (up to 16
// independent 16-byte loads in flight), summed in split order after dst -- the same order
// (and so the same bits) as splitk_reduce_k, whose 16 split groups each hold <= 1 slab here.
// splitk_reduce_k would leave 16 - S of every 16 threads idle and run ~n4/16 tiny blocks.
constexpr int FLAT_MAX_SPLITS = 16;
__global__ __launch_bounds__(NT) void splitk_reduce_flat_k(const float4* __restrict__ slab, int splits, long n4,
                                                          float4* __restrict__ dst, int accumulate) {
  const long i = blockIdx.x * (long)NT + threadIdx.x;
  if (i >= n4) return;
  float4 v[FLAT_MAX_SPLITS];
#pragma unroll
  for (int sp = 0; sp < FLAT_MAX_SPLITS; ++sp)
    if (sp < splits) v[sp] = slab[(size_t)sp * n4 + i];
  float4 d = accumulate ? dst[i] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sp = 0; sp < FLAT_MAX_SPLITS; ++sp)
    if (sp < splits) {
      d.x += v[sp].x; d.y += v[sp].y; d.z += v[sp].z; d.w += v[sp].w;
    }
  dst[i] = d;
}

// fp32-output split-K epilogue: one thread per 4 columns of one row, splits summed in
// order, then bias / ReLU (the small-M dense GEMMs: logits of a 64-row batch)
__global__ __launch_bounds__(NT) void splitk_finish_f32_k(const float* __restrict__ slab, int S, int M, int N,
                                                         const float* __restrict__ bias, int relu,
                                                         float* __restrict__ out, int ldc) {
  const int n4 = N / 4;
  const long i = blockIdx.x * (long)NT + threadIdx.x;
  if (i >= (long)M * n4) return;
  const int m = (int)(i / n4), n = 4 * (int)(i % n4);
  const size_t plane = (size_t)M * N;
  float4 v = *reinterpret_cast<const float4*>(slab + (size_t)m * N + n);
  for (int sp = 1; sp < S; ++sp) {
    const float4 q = *reinterpret_cast<const float4*>(slab + sp * plane + (size_t)m * N + n);
    v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
  }
  if (bias) {
    v.x += bias[n]; v.y += bias[n + 1]; v.z += bias[n + 2]; v.w += bias[n + 3];
  }
  if (relu) {
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
  }
  *reinterpret_cast<float4*>(out + (size_t)m * ldc + n) = v;
}

}  // namespace

hipError_t splitk_finish_f32(const float* slab, int splits, int M, int N, const float* bias, int relu, float* out,
                             int ldc, hipStream_t s) {
  if (splits < 1 || N % 4 || ldc % 4) return hipErrorInvalidValue;
  const long n = (long)M * (N / 4);
  hipLaunchKernelGGL(splitk_finish_f32_k, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, s, slab, splits, M, N,
                     bias, relu, out, ldc);
  return hipGetLastError();
}

hipError_t splitk_reduce(const float* slab, int splits, long n, float* dst, hipStream_t s, int accumulate) {
  if (n % 4 || splits < 1) return hipErrorInvalidValue;
  const long n4 = n / 4;
  if (splits <= FLAT_MAX_SPLITS && n4 >= 32 * NT) {
    hipLaunchKernelGGL(splitk_reduce_flat_k, dim3((unsigned)((n4 + NT - 1) / NT)), dim3(NT), 0, s,
                       reinterpret_cast<const float4*>(slab), splits, n4, reinterpret_cast<float4*>(dst), accumulate);
    return hipGetLastError();
  }
  const long g = (n4 + RED_E - 1) / RED_E;
  hipLaunchKernelGGL(splitk_reduce_k, dim3((unsigned)g), dim3(NT), 0, s, reinterpret_cast<const float4*>(slab),
                     splits, n4, reinterpret_cast<float4*>(dst), accumulate, 0, 0, 0, 0);
  return hipGetLastError();
}

hipError_t splitk_reduce_unpad(const float* slab, int splits, int R, int C1, int C2, int C1p, int C2p, float* dst,
                               hipStream_t s, int accumulate) {
  if (splits < 1 || R < 1 || C2 % 4 || C2p % 4 || C1 > C1p || C2 > C2p || C1 < 1 || C2 < 4) return hipErrorInvalidValue;
  const long n4 = (long)R * C1p * (C2p / 4);
  const long g = (n4 + RED_E - 1) / RED_E;
  hipLaunchKernelGGL(splitk_reduce_k, dim3((unsigned)g), dim3(NT), 0, s, reinterpret_cast<const float4*>(slab),
                     splits, n4, reinterpret_cast<float4*>(dst), accumulate, C1, C2 / 4, C1p, C2p / 4);
  return hipGetLastError();
}

hipError_t splitk_finish(const float* slab, int splits, int M, int N, const float* bias, const uint16_t* R, int relu,
                         float* stats, int rows_per_block, uint16_t* out, int ldc, hipStream_t s, long long* stats_acc,
                         int stats_reps) {
  if (splits < 1 || N % 8 || ldc % 8 || rows_per_block < 1 || stats_reps < 1) return hipErrorInvalidValue;
  const int grid = (M + rows_per_block - 1) / rows_per_block;
  const int bands = (N / 8 + NT - 1) / NT;
  hipLaunchKernelGGL(splitk_finish_k, dim3(grid, bands), dim3(NT), 0, s, slab, splits, M, N, bias, R, relu, stats,
                     rows_per_block, out, ldc, stats_acc, stats_reps);
  return hipGetLastError();
}

int gemm_stats_tile_rows(int tile) { return tile == 1 ? 256 : 128; }

hipError_t gemm_launch(const GemmArgs& a, int amode, int bmode, int epi, int splits, int tile, hipStream_t s) {
  if (splits < 1) return hipErrorInvalidValue;
  if ((epi & E_ATOMIC) && (epi & ~E_ATOMIC)) return hipErrorInvalidValue;
  if ((epi & E_SLAB) && (epi & ~E_SLAB)) return hipErrorInvalidValue;
  if (amode == A_CONV3 || amode == A_DGRAD3) {
    if (bmode != (amode == A_DGRAD3 ? B_KC : B_NC) || splits != 1) return hipErrorInvalidValue;
    return conv3_launch(a, amode == A_DGRAD3, epi, tile == 1 ? 64 : 128, s);
  }
  if (amode == A_WGRAD3) {
    if (bmode != B_NC) return hipErrorInvalidValue;
    return wgrad3_launch(a, epi, splits, s);
  }
  if (amode == A_CONV64 || amode == A_DGRAD64 || amode == A_WGRAD64) {
    if (bmode != (amode == A_DGRAD64 ? B_KC : B_NC)) return hipErrorInvalidValue;
    return conv_gemm_launch(a, amode, epi, splits, tile, s);
  }
  const int key = amode * 2 + bmode;
  switch (key) {
    case A_KC * 2 + B_NC: return launch_tile<A_KC, B_NC>(a, epi, splits, tile, s);
    case A_KC * 2 + B_KC: return launch_tile<A_KC, B_KC>(a, epi, splits, tile, s);
    case A_IM2COL * 2 + B_NC: return launch_tile<A_IM2COL, B_NC>(a, epi, splits, tile, s);
    case A_DGRAD * 2 + B_KC: return launch_tile<A_DGRAD, B_KC>(a, epi, splits, tile, s);
    case A_MC * 2 + B_NC: return launch_tile<A_MC, B_NC>(a, epi, splits, tile, s);
    case A_WGRAD * 2 + B_NC: return launch_tile<A_WGRAD, B_NC>(a, epi, splits, tile, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace damd
