"""Python launchers for the generic-path HIP kernels (csrc/kernels/gemm.hip,
csrc/kernels/layer_ops.hip).

These are thin, validating wrappers: they check dtypes, shapes, contiguity and the
16-byte alignment the kernels' vector accesses assume, pick the tile shape and split-K
factor, and enqueue on torch's current stream (so everything is captured by a
``torch.cuda.CUDAGraph``).  Activations are NHWC bf16, parameters fp32 masters with
bf16 shadows.  There is no silent fallback: a call that does not meet a kernel's
contract raises.

Keras conventions (reference README.md:58-73): conv kernels ``[kh, kw, cin, cout]``,
dense kernels ``[in, out]``, TF 'same' padding (the extra pixel at bottom/right).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from ..native import require_C

A_KC, A_IM2COL, A_DGRAD, A_MC, A_WGRAD, A_CONV64, A_DGRAD64, A_WGRAD64, A_WGRAD3, A_CONV3, A_DGRAD3 = range(11)
B_NC, B_KC = 0, 1
E_BIAS, E_RELU, E_BF16, E_ATOMIC, E_STATS, E_ADD, E_SLAB, E_BNRED, E_FIXUP = 1, 2, 4, 8, 16, 32, 64, 128, 256
BK = 32


def conv_kstep() -> int:
    """k-step depth of the LDS-DMA conv kernels (csrc/kernels/conv_gemm.hip): 64 (default)
    or 32 (DAMD_CONV_KB=32); the same rule as the C++ side."""
    return 32 if os.environ.get("DAMD_CONV_KB") == "32" else 64


def use_glds(gathered_channels: int) -> bool:
    """The LDS-DMA conv kernels take a conv whose gathered tensor has C % kstep == 0 (one
    filter tap x kstep channels per k-step); DAMD_CONV_GLDS=0 forces the register-staged
    kernel (A/B comparisons)."""
    return gathered_channels % conv_kstep() == 0 and os.environ.get("DAMD_CONV_GLDS", "1") != "0"


def _C():
    return require_C()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _chk(t: torch.Tensor, dtype, name: str):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.data_ptr() % 16:
        raise ValueError(f"{name}: must be 16-byte aligned")


def same_pad(in_size: int, k: int, s: int) -> Tuple[int, int, int]:
    """TF 'same': (out, pad_before, pad_after)."""
    out = math.ceil(in_size / s)
    total = max((out - 1) * s + k - in_size, 0)
    return out, total // 2, total - total // 2


def conv_out(in_size: int, k: int, s: int, padding: str) -> Tuple[int, int]:
    if padding == "same":
        o, pb, _ = same_pad(in_size, k, s)
        return o, pb
    return (in_size - k) // s + 1, 0


def pick_tile(N: int) -> int:
    """1 -> 256x64 tiles (narrow layers, no wasted MFMA columns), 0 -> 128x128."""
    return 1 if N <= 64 else 0


def tile_rows(tile: int) -> int:
    return 256 if tile == 1 else 128


def pick_splits(M: int, N: int, K: int, tile: int, target_wg: int = 1024) -> Tuple[int, int]:
    """Split-K factor so a long-K product still launches >> 256 workgroups (256 CUs)."""
    bm, bn = (256, 64) if tile == 1 else (128, 128)
    tiles = -(-M // bm) * -(-N // bn)
    splits = max(1, min(-(-target_wg // tiles), max(1, K // 256)))
    kps = -(-K // splits)
    kps = -(-kps // BK) * BK
    splits = -(-K // kps)
    return splits, kps


# weight-gradient split-K: every split stores its fp32 partial tile to a slab and one
# reduce kernel adds the slabs into the gradient in fixed order (deterministic; fp32
# atomics from hundreds of blocks on the same addresses serialise at the memory side)
WGRAD_TARGET_WG = int(os.environ.get("DAMD_WGRAD_TARGET_WG", 512))  # 2 workgroups per CU
WGRAD_SLAB_MAX = 64 << 20      # bytes of slab per GEMM


def wgrad_plan(M: int, N: int, K: int) -> Tuple[int, int, int]:
    """(tile, splits, k_per_split) of a weight-gradient GEMM [M,N] summed over K."""
    t = pick_tile(N)
    bm, bn = (256, 64) if t == 1 else (128, 128)
    tiles = -(-M // bm) * -(-N // bn)
    cap = max(1, WGRAD_SLAB_MAX // (M * N * 4))
    splits = max(1, min(-(-WGRAD_TARGET_WG // tiles), max(1, K // 256), cap))
    kps = -(-K // splits)
    kps = -(-kps // BK) * BK
    return t, -(-K // kps), kps


# bf16-output GEMMs (conv fwd / dgrad) whose tile count leaves CUs idle are split over K
# into fp32 slabs; splitk_finish then applies the epilogue (bias, residual, ReLU, BN
# statistics per FINISH_RB rows, bf16 store)
SPLIT_MIN_TILES = int(os.environ.get("DAMD_SPLIT_MIN_TILES", 320))
SPLIT_TARGET_WG = int(os.environ.get("DAMD_SPLIT_TARGET_WG", 384))
FINISH_RB = 16


def split_plan(M: int, N: int, K: int, tile: int, bk: int = BK) -> Tuple[int, int]:
    """(splits, k_per_split) for a bf16-output GEMM; splits == 1: the fused epilogue.
    k_per_split is a multiple of the kernel's k-step ``bk``."""
    bm, bn = (256, 64) if tile == 1 else (128, 128)
    tiles = -(-M // bm) * -(-N // bn)
    kfull = -(-K // bk) * bk
    if tiles >= SPLIT_MIN_TILES:
        return 1, kfull
    cap = max(1, WGRAD_SLAB_MAX // (M * N * 4))
    splits = max(1, min(-(-SPLIT_TARGET_WG // tiles), K // (BK * 8), cap))
    if splits == 1:
        return 1, kfull
    kps = -(-K // splits)
    kps = -(-kps // bk) * bk
    return -(-K // kps), kps


def _wgrad_slab1(M: int, N: int, K: int) -> bool:
    """An unsplit weight-gradient GEMM over few tiles (the classifier's dW: 32 tiles, K =
    batch): plain stores to one slab + the flat reduce beat the atomic epilogue there
    (fp32 atomics measured 19 us for the 512 x 1000 dW)."""
    t, splits, _ = wgrad_plan(M, N, K)
    bm, bn = (256, 64) if t == 1 else (128, 128)
    return splits == 1 and -(-M // bm) * -(-N // bn) <= 64 and (M * N) % 4 == 0 and M * N >= 4 * 8192


def wgrad_workspace_elems(M: int, N: int, K: int) -> int:
    _, splits, _ = wgrad_plan(M, N, K)
    if splits == 1 and _wgrad_slab1(M, N, K):
        return M * N
    return splits * M * N if splits > 1 else 0


def wgrad64_geo(n: int, ho: int, wo: int, kb: int) -> Tuple[int, int]:
    """(virtual rows, virtual rows per k-step) of the LDS-DMA weight-gradient kernel at
    k-step depth kb (mirror of csrc/kernels/conv_gemm.hip wgrad64_rows / _rows_per_step)."""
    nseg = -(-wo // kb)
    wv = -(-wo // nseg)
    s = 1
    while s < wv:
        s <<= 1
    return n * ho * nseg, kb // s


def wgrad3_ok(n, h, w, cin, cout, k, s, pad) -> bool:
    """Shapes the direct 3x3 weight-gradient kernel takes (mirror of wgrad3_launch)."""
    return (k == 3 and s == 1 and pad == 1 and cin % 64 == 0 and cout % 64 == 0 and w + 1 <= 63
            and n * (h + 1) * (w + 1) + 2048 < (1 << 21))


def conv_wgrad_plan(x_shape, w_shape, strides=(1, 1), padding="valid") -> dict:
    """Launch plan of conv_wgrad.  3x3/stride-1/pad-1 layers with channels % 64 == 0: the
    direct kernel (conv_wgrad3.hip, all nine taps per block).  Otherwise the LDS-DMA
    kernel over virtual rows (conv_gemm.hip) for layers with N = Cout > 64, k-step 32 for images of <= 16 columns (4 blocks/CU:
    the small-image layers are bound by per-block overheads) else 64; the register-staged
    kernel over pixels for N <= 64 (measured faster there: scripts/bench_gemm.py)."""
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x_shape, w_shape, strides, padding)
    M, N = kh * kw * cin, cout
    kb = int(os.environ.get("DAMD_CONV_KB", "0")) or (32 if wo <= 16 else 64)
    vr, g = wgrad64_geo(n, ho, wo, kb)
    if stem4_ok(x_shape, w_shape, strides, padding):
        # packed-tap stem: M = KH x 8 x 4 rows of the stem4_weight_shape layout
        M = kh * 32
        t = pick_tile(N)
        bm, bn = (256, 64) if t == 1 else (128, 128)
        tiles = -(-M // bm) * -(-N // bn)
        steps = -(-vr // g)
        cap = max(1, WGRAD_SLAB_MAX // (M * N * 4))
        splits = max(1, min(-(-WGRAD_TARGET_WG // tiles), max(1, steps // 4), cap))
        kps = -(-steps // splits) * g
        splits = -(-vr // kps)
        return {"amode": A_WGRAD64, "M": M, "N": N, "K": vr, "tile": t, "splits": splits, "kps": kps, "kstep": kb,
                "ws": splits * M * N if splits > 1 else 0}
    pick = os.environ.get("DAMD_WGRAD_KERNEL", "auto")  # auto | direct | glds | reg (tests, A/B runs)
    dma = os.environ.get("DAMD_CONV_GLDS", "1") != "0"
    if dma and pick in ("auto", "direct") and wgrad3_ok(n, h, wd, cin, cout, kh, s, pad):
        # direct 3x3 kernel (csrc/kernels/conv_wgrad3.hip): 64x64 (ci, co) tiles x all 9 taps
        Q = n * (h + 1) * (wd + 1)
        tiles = (cin // 64) * (cout // 64)
        steps = -(-Q // 32)
        cap = max(1, WGRAD_SLAB_MAX // (M * N * 4))
        target = int(os.environ.get("DAMD_WGRAD3_WG", "256"))  # 8-9-wave blocks, 1 per CU
        splits = max(1, min(-(-target // tiles), max(1, steps // 8), cap))
        kps = -(-steps // splits) * 32
        splits = -(-Q // kps)
        return {"amode": A_WGRAD3, "M": M, "N": N, "K": Q, "tile": 0, "splits": splits, "kps": kps, "kstep": 0,
                "ws": splits * M * N if splits > 1 else 0}
    glds = N > 64 if pick == "auto" else pick == "glds"
    if os.environ.get("DAMD_CONV_GLDS", "1") != "0" and glds and vr < (1 << 21):
        t = pick_tile(N)
        bm, bn = (256, 64) if t == 1 else (128, 128)
        tiles = -(-M // bm) * -(-N // bn)
        steps = -(-vr // g)
        cap = max(1, WGRAD_SLAB_MAX // (M * N * 4))
        splits = max(1, min(-(-WGRAD_TARGET_WG // tiles), max(1, steps // 4), cap))
        kps = -(-steps // splits) * g
        splits = -(-vr // kps)
        return {"amode": A_WGRAD64, "M": M, "N": N, "K": vr, "tile": t, "splits": splits, "kps": kps, "kstep": kb,
                "ws": splits * M * N if splits > 1 else 0}
    K = n * ho * wo
    t, splits, kps = wgrad_plan(M, N, K)
    return {"amode": A_WGRAD, "M": M, "N": N, "K": K, "tile": t, "splits": splits, "kps": kps, "kstep": 0,
            "ws": splits * M * N if splits > 1 else 0}


def _wgrad_gemm(A, B, dw, workspace, *, amode, M, N, K, lda=0, ldb=0, geo=(), accumulate=True):
    t, splits, kps = wgrad_plan(M, N, K)
    if splits == 1 and not (_wgrad_slab1(M, N, K) and workspace is not None and workspace.numel() >= M * N):
        # one writer per element: the atomic epilogue is an uncontended add
        if not accumulate:
            dw.zero_()
        gemm(A, B, dw, amode=amode, bmode=B_NC, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=N, epi=E_ATOMIC, geo=geo,
             tile=t)
        return
    need = splits * M * N
    if workspace is None or workspace.numel() < need or workspace.dtype != torch.float32:
        raise ValueError(f"weight-gradient GEMM needs an fp32 workspace of {need} elements")
    gemm(A, B, workspace, amode=amode, bmode=B_NC, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=N, epi=E_SLAB,
         splits=splits, k_per_split=kps, tile=t, geo=geo)
    _C().splitk_reduce(_ptr(workspace), splits, M * N, _ptr(dw), stream_handle(), accumulate=int(accumulate))


def acc_reps(acc):
    """Replica count of a BatchNorm statistics accumulator (int64 fixed point, layer_ops.h
    BNFin): [reps + 1, 2C] forward / [reps + 1, 4C] backward (2-D: the last row is the sticky
    non-finite flag plane, damd_common.h bnacc_flag) or one replica + its flag plane (1-D,
    [2 x K]).  Producer block b adds into replica b % reps."""
    if acc is None or acc.dim() != 2:
        return 1
    if acc.shape[0] < 2:
        raise ValueError("a BatchNorm accumulator needs >= 1 replica row + the flag row")
    return int(acc.shape[0]) - 1


def acc_zeros(reps: int, K: int, device) -> torch.Tensor:
    """A cleared accumulator of ``reps`` replicas of K words + the flag plane."""
    return torch.zeros(reps + 1, K, dtype=torch.int64, device=device)


# Fixed-point BatchNorm accumulators (csrc/include/damd_common.h bnacc_add1 / bnacc_add2):
# integer atomics, so the statistics are bitwise independent of the producer blocks'
# arrival order.  Forward sums: one int64 word per value (unit 2^-24); backward sums: two
# (hi = floor(v 2^24), lo = floor((v 2^24 - hi) 2^40)) in planes [s hi | s lo | q hi | q lo].
ACC_UNIT = 2.0 ** -24


def bn_acc_encode(values: torch.Tensor, words: int = 1) -> torch.Tensor:
    """Host encoding of fp64 sums into accumulator words (tests / diagnostics): [..., 2C]
    doubles (sums, second statistics) -> [..., 2C] (words 1) or [..., 4C] (words 2: planes
    s hi | s lo | q hi | q lo) int64."""
    v = values.double().cpu()
    if words == 1:
        return torch.round(v * 2.0 ** 24).to(torch.int64)
    d = v * 2.0 ** 24
    hi = torch.floor(d)
    lo = torch.floor((d - hi) * 2.0 ** 40)
    C = v.shape[-1] // 2
    parts = [hi[..., :C], lo[..., :C], hi[..., C:], lo[..., C:]]
    return torch.cat([p.to(torch.int64) for p in parts], -1)


def bn_acc_decode(acc: torch.Tensor, words: int = 1) -> torch.Tensor:
    """Replica-summed values of an accumulator ([reps + 1, K] or [2K]: replicas then the flag
    plane) as fp64; NaN where a channel's flag is set."""
    a = acc.cpu()
    if a.dim() == 1:
        a = a.view(2, -1)
    flag = a[-1]
    a = a[:-1].sum(0)
    if words == 1:
        C = a.numel() // 2
        out = a.double() * ACC_UNIT
        bad = torch.cat([flag[:C] != 0] * 2)
    else:
        C = a.numel() // 4
        s = a[:C].double() * ACC_UNIT + a[C:2 * C].double() * 2.0 ** -64
        q = a[2 * C:3 * C].double() * ACC_UNIT + a[3 * C:].double() * 2.0 ** -64
        out = torch.cat([s, q])
        bad = torch.cat([flag[:C] != 0] * 2)
    out[bad] = float("nan")
    return out


def _stats_ptrs(stats):
    """(partials pointer, accumulator pointer, replicas) of a stats argument: an fp32
    [T][2][N] partials tensor, or an int64 fixed-point accumulator [2N] / [reps, 2N]
    (forward) or [reps, 4N] (backward, E_BNRED) (BNFin: producers add, the consumer
    finalizes)."""
    if stats is None:
        return 0, 0, 1
    if stats.dtype == torch.int64:
        return 0, _ptr(stats), acc_reps(stats)
    return _ptr(stats), 0, 1


def gemm(A, B, C, *, amode, bmode, M, N, K, lda=0, ldb=0, ldc=0, epi=0, bias=None, stats=None, R=None,
         geo: Sequence[int] = (), kc=0, splits=1, k_per_split=None, tile=None, kstep=0, bnx=None, bnst=None,
         bnin=None, slab=None):
    t = pick_tile(N) if tile is None else tile
    kps = k_per_split if k_per_split is not None else -(-K // BK) * BK
    sp, sa, reps = _stats_ptrs(stats)
    bp, bv = bnin[0].args() if bnin is not None else ([], [])
    _C().gemm(amode, bmode, epi, splits, t, _ptr(A), _ptr(B), _ptr(C), _ptr(bias), sp, _ptr(R), M, N, K,
              lda, ldb, ldc, list(geo), kc, kps, stream_handle(), kstep, stats_acc=sa, bnx=_ptr(bnx), bnst=_ptr(bnst),
              stats_reps=reps, bnin_p=bp, bnin_v=bv, bnin_y=_ptr(bnin[1]) if bnin is not None else 0,
              slab=_ptr(slab), tickets=_ptr(_tickets(A.device)) if epi & E_FIXUP else 0)


_TICKETS = {}


def _tickets(device) -> torch.Tensor:
    """The per-tile arrival tickets of the in-launch split-K finish (E_FIXUP): zero between
    launches (each tile's reducing split resets its own), shared by the launches of one
    stream in order."""
    t = _TICKETS.get(device)
    if t is None:
        t = _TICKETS[device] = torch.zeros(1 << 16, dtype=torch.int32, device=device)
    return t


def splitk_fixup_on(stats) -> bool:
    """Split-K GEMMs finish inside the launch (E_FIXUP) with DAMD_SPLITK_FIXUP=1 when the BN
    statistics (if any) go to a fixed-point accumulator.  Off by default: measured on the
    ResNet-18 step, 2.704 vs 2.587 ms -- the last split of a 128 x 128 tile re-reads S x 64 KB
    of slabs serially (layer-4 forward 26 -> 48 us per conv against the 8 us finish launch
    it replaces); the in-launch reduction pays only for slabs of a few tens of KB per tile."""
    return os.environ.get("DAMD_SPLITK_FIXUP", "0") == "1" and (stats is None or stats.dtype == torch.int64)


# ---- dense -------------------------------------------------------------------------------
# Small-M dense GEMMs (a 64-row batch against a 512 x 1000 classifier) give 4-8 output
# tiles: 4-8 busy CUs walking 8-16 serial k-steps (23-32 us on MI355X for <= 66 MFLOP).
# They are split over K into fp32 slabs (one k-step or two per workgroup) and finished by
# a fixed-order reduction kernel with the bias / ReLU / accumulate epilogue.
DENSE_SPLIT_MAX_TILES = 32
DENSE_SPLIT_TARGET_WG = int(os.environ.get("DAMD_DENSE_SPLIT_WG", "128"))  # 1: no split-K (A/B runs)


def dense_split_plan(M: int, N: int, K: int) -> Tuple[int, int]:
    """(splits, k_per_split) of a dense forward / backprop-input GEMM [M,N] over K."""
    t = pick_tile(N)
    bm, bn = (256, 64) if t == 1 else (128, 128)
    tiles = -(-M // bm) * -(-N // bn)
    kfull = -(-K // BK) * BK
    if tiles > DENSE_SPLIT_MAX_TILES or K < 2 * BK:
        return 1, kfull
    splits = max(1, min(-(-DENSE_SPLIT_TARGET_WG // tiles), K // BK))
    kps = -(-(-(-K // splits)) // BK) * BK
    return -(-K // kps), kps


def dense_workspace_elems(M: int, N: int, K: int) -> int:
    """fp32 workspace of the split forward (x[M,K] @ w[K,N]) and backprop-input GEMMs."""
    s1, _ = dense_split_plan(M, N, K)
    s2, _ = dense_split_plan(M, K, N)
    return max(s1 * M * N if s1 > 1 else 0, s2 * M * K if s2 > 1 else 0)


def dense_fwd(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, bias=None, relu=False, stats=None,
              workspace: Optional[torch.Tensor] = None):
    """out[M,N] = x[M,K] @ w[K,N] (+bias)(relu); x, w bf16; out bf16 or fp32.  With a
    workspace, under-filled shapes run split-K (dense_split_plan)."""
    M, K = x.shape
    K2, N = w.shape
    assert K == K2 and tuple(out.shape) == (M, N)
    _chk(x, torch.bfloat16, "x")
    _chk(w, torch.bfloat16, "w")
    if K % 8 or N % 8:
        raise ValueError("dense_fwd: K and N must be multiples of 8 (pad the layer)")
    splits, kps = dense_split_plan(M, N, K)
    if splits > 1 and stats is None and workspace is not None and workspace.numel() >= splits * M * N:
        gemm(x, w, workspace, amode=A_KC, bmode=B_NC, M=M, N=N, K=K, lda=K, ldb=N, ldc=N, epi=E_SLAB,
             splits=splits, k_per_split=kps)
        if out.dtype == torch.float32:
            _C().splitk_finish_f32(_ptr(workspace), splits, M, N, _ptr(bias), int(relu), _ptr(out), N,
                                   stream_handle())
        else:
            _C().splitk_finish(_ptr(workspace), splits, M, N, _ptr(bias), 0, int(relu), 0, FINISH_RB, _ptr(out), N,
                               stream_handle())
        return
    epi = (E_BIAS if bias is not None else 0) | (E_RELU if relu else 0)
    epi |= E_BF16 if out.dtype == torch.bfloat16 else 0
    if stats is not None:
        epi |= E_STATS
    gemm(x, w, out, amode=A_KC, bmode=B_NC, M=M, N=N, K=K, lda=K, ldb=N, ldc=N, epi=epi, bias=bias, stats=stats)


def dense_dgrad(dy: torch.Tensor, w: torch.Tensor, dx: torch.Tensor, accumulate=False,
                workspace: Optional[torch.Tensor] = None):
    """dx[M,K] (+)= dy[M,N] @ w[K,N]^T (bf16 out); split-K with a workspace like dense_fwd."""
    M, N = dy.shape
    K, N2 = w.shape
    assert N == N2 and tuple(dx.shape) == (M, K)
    _chk(dy, torch.bfloat16, "dy")
    _chk(w, torch.bfloat16, "w")
    _chk(dx, torch.bfloat16, "dx")
    splits, kps = dense_split_plan(M, K, N)
    if splits > 1 and workspace is not None and workspace.numel() >= splits * M * K:
        gemm(dy, w, workspace, amode=A_KC, bmode=B_KC, M=M, N=K, K=N, lda=N, ldc=K, epi=E_SLAB, kc=N,
             splits=splits, k_per_split=kps)
        _C().splitk_finish(_ptr(workspace), splits, M, K, 0, _ptr(dx) if accumulate else 0, 0, 0, FINISH_RB,
                           _ptr(dx), K, stream_handle())
        return
    epi = E_BF16 | (E_ADD if accumulate else 0)
    gemm(dy, w, dx, amode=A_KC, bmode=B_KC, M=M, N=K, K=N, lda=N, ldc=K, epi=epi, kc=N,
         R=dx if accumulate else None)


def dense_wgrad(x: torch.Tensor, dy: torch.Tensor, dw: torch.Tensor, workspace: Optional[torch.Tensor] = None,
                accumulate: bool = True):
    """dw[K,N] (+)= x[M,K]^T @ dy[M,N] (fp32; split over M, slabs reduced in fixed order);
    accumulate=False overwrites dw."""
    M, K = x.shape
    M2, N = dy.shape
    assert M == M2 and tuple(dw.shape) == (K, N)
    _chk(x, torch.bfloat16, "x")
    _chk(dy, torch.bfloat16, "dy")
    _chk(dw, torch.float32, "dw")
    if workspace is None and wgrad_workspace_elems(K, N, M):
        workspace = torch.empty(wgrad_workspace_elems(K, N, M), device=x.device)
    _wgrad_gemm(x, dy, dw, workspace, amode=A_MC, M=K, N=N, K=M, lda=K, ldb=N, accumulate=accumulate)


# ---- conv ---------------------------------------------------------------------------------
def conv_geo(x_shape, w_shape, strides, padding):
    n, h, w_, c = x_shape
    kh, kw, cin, cout = w_shape
    if strides[0] != strides[1] or kh != kw or h != w_:
        raise ValueError("HIP conv path: square kernels/images and equal strides only")
    ho, pad = conv_out(h, kh, strides[0], padding)
    wo, pad2 = conv_out(w_, kw, strides[1], padding)
    assert pad == pad2
    return n, h, w_, cin, ho, wo, kh, kw, strides[0], pad, cout


def stem4_ok(x_shape, w_shape, strides, padding) -> bool:
    """A conv the packed-tap stem kernels take (conv_gemm.hip): a 4-channel input (e.g.
    RGB + one zero channel), a square kernel of <= 8 columns, even stride, even top/left
    padding and an even image width.  Its weights are laid out [KH][8][4][Cout] (zero
    beyond the true KW columns / Cin channels): stem4_weight_layout."""
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x_shape, w_shape, strides, padding)
    return (cin == 4 and kw <= 8 and s % 2 == 0 and pad % 2 == 0 and wd % 2 == 0 and cout % 8 == 0
            and os.environ.get("DAMD_CONV_GLDS", "1") != "0")


def stem4_weight_shape(w_shape):
    kh, kw, cin, cout = w_shape
    return (kh, 8, 4, cout)


def conv_fwd_stem4(x, w8, out, kernel_size, strides=(2, 2), padding="same", bias=None, relu=False, stats=None,
                   workspace: Optional[torch.Tensor] = None):
    """Packed-tap stem forward: out = conv(x [N,H,W,4], true kernel kernel_size x
    kernel_size) with w8 = the weights in stem4_weight_shape layout (bf16)."""
    k = kernel_size
    cout = w8.shape[-1]
    wshape = (k, k, 4, cout)
    if not stem4_ok(x.shape, wshape, strides, padding) or tuple(w8.shape) != stem4_weight_shape(wshape):
        raise ValueError("conv_fwd_stem4: not a packed-tap stem conv")
    _chk(x, torch.bfloat16, "x")
    _chk(w8, torch.bfloat16, "w8")
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x.shape, wshape, strides, padding)
    assert tuple(out.shape) == (n, ho, wo, cout)
    plan = conv_fwd_plan(x.shape, wshape, strides, padding)
    _check_stats(stats, plan, cout, "conv_fwd_stem4")
    M, K = plan["M"], plan["K"]
    geo = (h, wd, 4, ho, wo, kh, 8, s, pad)
    if plan["splits"] == 1:
        epi = (E_BIAS if bias is not None else 0) | (E_RELU if relu else 0) | E_BF16 | \
            (E_STATS if stats is not None else 0)
        gemm(x, w8, out, amode=A_CONV64, bmode=B_NC, M=M, N=cout, K=K, ldb=cout, ldc=cout, epi=epi, bias=bias,
             stats=stats, geo=geo, tile=plan["tile"], kstep=32)
        return
    ws = _workspace(workspace, plan["ws"], x.device)
    gemm(x, w8, ws, amode=A_CONV64, bmode=B_NC, M=M, N=cout, K=K, ldb=cout, ldc=cout, epi=E_SLAB,
         splits=plan["splits"], k_per_split=plan["kps"], tile=plan["tile"], geo=geo, kstep=32)
    sp, sa, reps = _stats_ptrs(stats)
    _C().splitk_finish(_ptr(ws), plan["splits"], M, cout, _ptr(bias), 0, int(relu), sp, FINISH_RB,
                       _ptr(out), cout, stream_handle(), stats_acc=sa, stats_reps=reps)


def _check_stats(stats, plan, cout, who):
    if stats is None:
        return
    if stats.dtype == torch.int64:
        ok = (stats.numel() == 4 * cout if stats.dim() == 1 else
              (stats.dim() == 2 and stats.shape[0] >= 2 and stats.shape[-1] == 2 * cout))
        if not ok:
            raise ValueError(f"{who}: a statistics accumulator is int64 [reps + 1][2 x {cout}], "
                             f"got {tuple(stats.shape)}")
    elif stats.shape[0] != plan["stats_T"]:
        raise ValueError(f"{who}: stats needs {plan['stats_T']} partial rows, got {stats.shape[0]}")


def conv_wgrad_stem4(x, dy, dw8, kernel_size, strides=(2, 2), padding="same",
                     workspace: Optional[torch.Tensor] = None, accumulate: bool = True,
                     dw: Optional[torch.Tensor] = None) -> bool:
    """Packed-tap stem weight gradient: dw8 [KH][8][4][Cout] (fp32) += the gradient in the
    stem4_weight_shape layout (entries beyond the true kernel are junk to drop).  With
    ``dw`` (the true [KH][KW][Cin][Cout] fp32 gradient) and a split-K plan, the split-K
    reduce drops the junk and ADDS straight into ``dw`` (dw8 untouched; ``accumulate``
    applies to dw8 only); returns True then, else False (the caller unpads dw8 itself)."""
    k = kernel_size
    cout = dw8.shape[-1]
    wshape = (k, k, 4, cout)
    if not stem4_ok(x.shape, wshape, strides, padding) or tuple(dw8.shape) != stem4_weight_shape(wshape):
        raise ValueError("conv_wgrad_stem4: not a packed-tap stem conv")
    _chk(x, torch.bfloat16, "x")
    _chk(dy, torch.bfloat16, "dy")
    _chk(dw8, torch.float32, "dw8")
    plan = conv_wgrad_plan(x.shape, wshape, strides, padding)
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x.shape, wshape, strides, padding)
    geo = (h, wd, 4, ho, wo, kh, 8, s, pad)
    M, N, K, splits = plan["M"], plan["N"], plan["K"], plan["splits"]
    if splits == 1:
        if not accumulate:
            dw8.zero_()
        gemm(x, dy, dw8, amode=A_WGRAD64, bmode=B_NC, M=M, N=N, K=K, ldb=cout, ldc=N, epi=E_ATOMIC, geo=geo,
             k_per_split=plan["kps"], tile=plan["tile"], kstep=plan["kstep"])
        return False
    workspace = _workspace(workspace, plan["ws"], x.device)
    gemm(x, dy, workspace, amode=A_WGRAD64, bmode=B_NC, M=M, N=N, K=K, ldb=cout, ldc=N, epi=E_SLAB,
         splits=splits, k_per_split=plan["kps"], tile=plan["tile"], geo=geo, kstep=plan["kstep"])
    if dw is not None:
        _chk(dw, torch.float32, "dw")
        ci = dw.shape[2] if dw.dim() == 4 else 0
        if tuple(dw.shape) != (k, k, ci, cout) or not 1 <= ci <= 4:
            raise ValueError(f"conv_wgrad_stem4: dw shape {tuple(dw.shape)} is not [{k}][{k}][<=4][{cout}]")
        # the reduce's rows [KH][8][4 x Cout] -> [KH][KW][Cin x Cout]
        _C().splitk_reduce_unpad(_ptr(workspace), splits, k, k, ci * cout, 8, 4 * cout, _ptr(dw), stream_handle(), 1)
        return True
    _C().splitk_reduce(_ptr(workspace), splits, M * N, _ptr(dw8), stream_handle(), accumulate=int(accumulate))
    return False


# ---- direct 3x3 / stride-1 / pad-1 convolution (csrc/kernels/conv3x3.hip) ---------------


def conv3_rows(h: int, w: int, bn: int) -> int:
    """Output rows per block of the direct 3x3 kernel (mirror of conv3x3.hip conv3_rows):
    the block's R x W pixels fill its 256 (BN 64) / 128 (BN 128) MFMA rows and the input
    halo + weight ring fit 80 KiB (two blocks per CU); 0 = shape not taken."""
    bm = 256 if bn == 64 else 128
    r = min(bm // w, h)
    if r < 1:
        return 0
    halo = (((r + 2) * (w + 2)) * 128 + 1023) & ~1023
    return r if halo + (4 if bn == 64 else 3) * bn * 128 <= 80 * 1024 else 0


def conv3_tile(n: int, h: int, w: int, gathered: int, out_ch: int):
    """(tile, rows, row blocks per image) when the direct kernel takes a 3x3/s1/p1 conv of
    ``gathered`` input channels into ``out_ch`` on n x h x w images, else None: channels %
    64, the block's pixels fill >= 3/4 of its MFMA rows, and the grid has >= CONV3_MIN_WG
    blocks (DAMD_CONV3_MIN_WG, default 256: ResNet layers 1-3; smaller grids keep the split-K implicit GEMM)."""
    if os.environ.get("DAMD_CONV3", "1") == "0" or os.environ.get("DAMD_CONV_GLDS", "1") == "0":
        return None
    if gathered % 64 or out_ch % 64:
        return None
    bn = 64 if out_ch % 128 else 128
    r = conv3_rows(h, w, bn)
    if r == 0 or r * w < 0.75 * (256 if bn == 64 else 128):
        return None
    tpi = -(-h // r)
    if (out_ch // bn) * n * tpi < int(os.environ.get("DAMD_CONV3_MIN_WG", 256)):
        return None
    return (1 if bn == 64 else 0), r, tpi


def conv_fwd_plan(x_shape, w_shape, strides=(1, 1), padding="valid") -> dict:
    """Launch plan of conv_fwd: tile, split-K, number of BN-statistics partials and the
    fp32 workspace it needs (0 when not split)."""
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x_shape, w_shape, strides, padding)
    if stem4_ok(x_shape, w_shape, strides, padding):
        # packed-tap stem: K = KH x (8 pixels x 4 channels), k-step 32 (conv_gemm.hip)
        M, N, K = n * ho * wo, cout, kh * 32
        t = pick_tile(N)
        splits, kps = split_plan(M, N, K, t, 32)
        return {"M": M, "N": N, "K": K, "tile": t, "splits": splits, "kps": kps, "amode": A_CONV64,
                "kstep": 32, "stats_T": -(-M // (FINISH_RB if splits > 1 else tile_rows(t))),
                "ws": splits * M * N if splits > 1 else 0}
    M, N, K = n * ho * wo, cout, kh * kw * cin
    c3 = conv3_tile(n, h, wd, cin, cout) if (kh == kw == 3 and s == 1 and pad == 1 and ho == h) else None
    if c3 is not None:
        return {"M": M, "N": N, "K": K, "tile": c3[0], "splits": 1, "kps": K, "amode": A_CONV3,
                "stats_T": n * c3[2], "ws": 0}
    t = pick_tile(N)
    glds = use_glds(cin)
    splits, kps = split_plan(M, N, K, t, conv_kstep() if glds else BK)
    return {"M": M, "N": N, "K": K, "tile": t, "splits": splits, "kps": kps,
            "amode": A_CONV64 if glds else A_IM2COL,
            "stats_T": -(-M // (FINISH_RB if splits > 1 else tile_rows(t))),
            "ws": splits * M * N if splits > 1 else 0}


def conv_fwd(x, w, out, strides=(1, 1), padding="valid", bias=None, relu=False, stats=None,
             workspace: Optional[torch.Tensor] = None, bnin=None):
    """out [N,Ho,Wo,Cout] = conv(x [N,H,W,Cin], w [KH,KW,Cin,Cout]); bf16 in/out.  stats
    (BN batch statistics partials) must have conv_fwd_plan(...)["stats_T"] rows.
    bnin = (fin: BNFin, y): x is a BatchNorm's input and the conv runs on y = relu(BN(x)),
    finalized and applied on load by the direct kernel (A_CONV3 plans only), which also
    stores y (bitwise bn_apply_fin(x, y, fin, relu=True)) and publishes fin's st / moving
    statistics."""
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x.shape, w.shape, strides, padding)
    _chk(x, torch.bfloat16, "x")
    _chk(w, torch.bfloat16, "w")
    if cin % 8 or cout % 8:
        raise ValueError("conv_fwd: Cin and Cout must be multiples of 8 (pad the channels)")
    assert tuple(out.shape) == (n, ho, wo, cout)
    plan = conv_fwd_plan(x.shape, w.shape, strides, padding)
    M, K = plan["M"], plan["K"]
    _check_stats(stats, plan, cout, "conv_fwd")
    geo = (h, wd, cin, ho, wo, kh, kw, s, pad)
    if bnin is not None and (plan["amode"] != A_CONV3 or plan["splits"] != 1 or bnin[0].acc is None
                             or tuple(bnin[1].shape) != tuple(x.shape)):
        raise ValueError("conv_fwd: a BN input needs a direct 3x3 plan and y of x's shape")
    if plan["splits"] == 1:
        epi = (E_BIAS if bias is not None else 0) | (E_RELU if relu else 0) | E_BF16 | \
            (E_STATS if stats is not None else 0)
        gemm(x, w, out, amode=plan["amode"], bmode=B_NC, M=M, N=cout, K=K, ldb=cout, ldc=cout, epi=epi,
             bias=bias, stats=stats, geo=geo, tile=plan["tile"], bnin=bnin)
        return
    ws = _workspace(workspace, plan["ws"], x.device)
    if plan["amode"] in (A_CONV64,) and splitk_fixup_on(stats) and cout % 4 == 0:
        epi = E_FIXUP | (E_BIAS if bias is not None else 0) | (E_RELU if relu else 0) | E_BF16 | \
            (E_STATS if stats is not None else 0)
        if not (relu and stats is not None):  # (no kernel instantiates both)
            gemm(x, w, out, amode=plan["amode"], bmode=B_NC, M=M, N=cout, K=K, ldb=cout, ldc=cout, epi=epi,
                 bias=bias, stats=stats, splits=plan["splits"], k_per_split=plan["kps"], tile=plan["tile"], geo=geo,
                 slab=ws)
            return
    gemm(x, w, ws, amode=plan["amode"], bmode=B_NC, M=M, N=cout, K=K, ldb=cout, ldc=cout, epi=E_SLAB,
         splits=plan["splits"], k_per_split=plan["kps"], tile=plan["tile"], geo=geo)
    sp, sa, reps = _stats_ptrs(stats)
    _C().splitk_finish(_ptr(ws), plan["splits"], M, cout, _ptr(bias), 0, int(relu), sp, FINISH_RB,
                       _ptr(out), cout, stream_handle(), stats_acc=sa, stats_reps=reps)


def _workspace(ws, need, device):
    if need == 0:
        return None
    if ws is None:
        return torch.empty(need, device=device)
    if ws.dtype != torch.float32 or ws.numel() < need:
        raise ValueError(f"split-K GEMM needs an fp32 workspace of {need} elements")
    return ws


def conv_dgrad_plan(dx_shape, w_shape, strides=(1, 1), padding="valid") -> dict:
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(dx_shape, w_shape, strides, padding)
    M, N, K = n * h * wd, cin, kh * kw * cout
    c3 = conv3_tile(n, h, wd, cout, cin) if (kh == kw == 3 and s == 1 and pad == 1 and ho == h) else None
    if c3 is not None:
        return {"M": M, "N": N, "K": K, "tile": c3[0], "splits": 1, "kps": K, "amode": A_DGRAD3, "ws": 0,
                "stats_T": n * c3[2]}
    t = pick_tile(N)
    if (s == 2 and use_glds(cout) and h % 2 == 0 and wd % 2 == 0 and pad == 0
            and os.environ.get("DAMD_DGRAD_SUBPIX", "1") != "0"):
        # stride 2: four sub-pixel classes (conv_gemm.hip), rows = one class grid, no K split
        return {"M": n * (h // 2) * (wd // 2), "N": N, "K": K, "tile": t, "splits": 1, "kps": K,
                "amode": A_DGRAD64, "ws": 0}
    glds = s == 1 and use_glds(cout)
    splits, kps = split_plan(M, N, K, t, conv_kstep() if glds else BK)
    return {"M": M, "N": N, "K": K, "tile": t, "splits": splits, "kps": kps,
            "amode": A_DGRAD64 if glds else A_DGRAD,
            "ws": splits * M * N if splits > 1 else 0}


def conv_dgrad(dy, w, dx, strides=(1, 1), padding="valid", accumulate=False,
               workspace: Optional[torch.Tensor] = None, bnred=None) -> bool:
    """dx [N,H,W,Cin] (+)= backprop-input of dy [N,Ho,Wo,Cout] through w.  ``bnred`` =
    (x, st, part): dx is the gradient of relu(BN(x)) (BN coefficients st [4][Cin]); when the
    direct kernel runs (conv_dgrad_plan stats_T rows) it also writes the BN-backward
    partials (sum dz, sum dz * xhat per tile) into part [stats_T][2][Cin] (or adds them into
    an int64 fixed-point accumulator [reps][4 Cin]: two words per value), replacing
    bn_bwd_reduce.  Returns True when it did."""
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(dx.shape, w.shape, strides, padding)
    if s not in (1, 2):
        raise ValueError("conv_dgrad: stride 1 or 2")
    _chk(dy, torch.bfloat16, "dy")
    _chk(w, torch.bfloat16, "w")
    _chk(dx, torch.bfloat16, "dx")
    if cin % 8 or cout % 8:
        raise ValueError("conv_dgrad: Cin and Cout must be multiples of 8")
    plan = conv_dgrad_plan(dx.shape, w.shape, strides, padding)
    M, K = plan["M"], plan["K"]
    geo = (h, wd, cout, ho, wo, kh, kw, s, pad)
    if bnred is not None and plan["amode"] == A_DGRAD3 and not accumulate:
        bx, bst, part = bnred
        is_acc = part.dtype == torch.int64  # a fixed-point accumulator [reps][4 Cin] (BNBwdFin)
        if ((part.shape[-1] != 4 * cin if is_acc else part.shape[0] != plan["stats_T"])
                or tuple(bx.shape) != tuple(dx.shape)):
            raise ValueError("conv_dgrad: bnred partials / BN input do not match the plan")
        gemm(dy, w, dx, amode=A_DGRAD3, bmode=B_KC, M=M, N=cin, K=K, ldc=cin, epi=E_BF16 | E_BNRED, kc=cout,
             geo=geo, stats=part, tile=plan["tile"], bnx=bx, bnst=bst)
        return True
    if plan["splits"] == 1:
        epi = E_BF16 | (E_ADD if accumulate else 0)
        gemm(dy, w, dx, amode=plan["amode"], bmode=B_KC, M=M, N=cin, K=K, ldc=cin, epi=epi, kc=cout, geo=geo,
             R=dx if accumulate else None, tile=plan["tile"])
        return False
    ws = _workspace(workspace, plan["ws"], dx.device)
    if plan["amode"] == A_DGRAD64 and splitk_fixup_on(None) and cin % 4 == 0:
        gemm(dy, w, dx, amode=plan["amode"], bmode=B_KC, M=M, N=cin, K=K, ldc=cin,
             epi=E_FIXUP | E_BF16 | (E_ADD if accumulate else 0), kc=cout, geo=geo, R=dx if accumulate else None,
             splits=plan["splits"], k_per_split=plan["kps"], tile=plan["tile"], slab=ws)
        return False
    gemm(dy, w, ws, amode=plan["amode"], bmode=B_KC, M=M, N=cin, K=K, ldc=cin, epi=E_SLAB, kc=cout, geo=geo,
         splits=plan["splits"], k_per_split=plan["kps"], tile=plan["tile"])
    _C().splitk_finish(_ptr(ws), plan["splits"], M, cin, 0, _ptr(dx) if accumulate else 0, 0, 0, FINISH_RB,
                       _ptr(dx), cin, stream_handle())
    return False


def conv_wgrad_workspace_elems(x_shape, w_shape, strides=(1, 1), padding="valid") -> int:
    return conv_wgrad_plan(x_shape, w_shape, strides, padding)["ws"]


def conv_wgrad(x, dy, dw, strides=(1, 1), padding="valid", workspace: Optional[torch.Tensor] = None,
               accumulate: bool = True):
    """dw [KH,KW,Cin,Cout] (+)= sum over pixels of im2col(x)^T dy (split-K over pixels, fp32
    slabs in ``workspace`` (conv_wgrad_workspace_elems) reduced in fixed order);
    accumulate=False overwrites dw (no zeroing pass)."""
    n, h, wd, cin, ho, wo, kh, kw, s, pad, cout = conv_geo(x.shape, dw.shape, strides, padding)
    _chk(x, torch.bfloat16, "x")
    _chk(dy, torch.bfloat16, "dy")
    _chk(dw, torch.float32, "dw")
    if cin % 8 or cout % 8:
        raise ValueError("conv_wgrad: Cin and Cout must be multiples of 8")
    plan = conv_wgrad_plan(x.shape, dw.shape, strides, padding)
    M, N, K, splits = plan["M"], plan["N"], plan["K"], plan["splits"]
    geo = (h, wd, cin, ho, wo, kh, kw, s, pad)
    if splits == 1:  # one writer per element: the atomic epilogue is an uncontended add
        if not accumulate:
            dw.zero_()
        gemm(x, dy, dw, amode=plan["amode"], bmode=B_NC, M=M, N=N, K=K, ldb=cout, ldc=N, epi=E_ATOMIC, geo=geo,
             k_per_split=plan["kps"], tile=plan["tile"], kstep=plan["kstep"])
        return
    workspace = _workspace(workspace, plan["ws"], x.device)
    gemm(x, dy, workspace, amode=plan["amode"], bmode=B_NC, M=M, N=N, K=K, ldb=cout, ldc=N, epi=E_SLAB,
         splits=splits, k_per_split=plan["kps"], tile=plan["tile"], geo=geo, kstep=plan["kstep"])
    _C().splitk_reduce(_ptr(workspace), splits, M * N, _ptr(dw), stream_handle(), accumulate=int(accumulate))


# ---- BN / pooling / loss / optimizer -------------------------------------------------------------
def bn_finalize(part, T, C, count, gamma, beta, eps, momentum, rmean, rvar, st):
    _C().bn_finalize(_ptr(part), T, C, float(count), _ptr(gamma), _ptr(beta), float(eps), float(momentum),
                     _ptr(rmean), _ptr(rvar), _ptr(st), stream_handle())


def bn_apply(x, st, y, relu=False, r=None, st2=None):
    C = x.shape[-1]
    M = x.numel() // C
    mode = 0 if r is None else (1 if st2 is None else 2)
    _C().bn_apply(_ptr(x), _ptr(st), _ptr(r), _ptr(st2), mode, int(relu), _ptr(y), M, C, stream_handle())


def bn_bwd(dy, y, relu_mask, x, st, part, co, dx, dgamma=None, dbeta=None, dz_out=None):
    """Full BN backward (reduce, finalize, apply); part must hold bn_bwd_blocks(M, C) x 2C."""
    C = x.shape[-1]
    M = x.numel() // C
    T = _C().bn_bwd_blocks(M, C)
    assert part.numel() >= T * 2 * C
    s = stream_handle()
    _C().bn_bwd_reduce(_ptr(dy), _ptr(y), int(relu_mask), _ptr(x), _ptr(st), _ptr(dz_out), _ptr(part), T, M, C, s)
    _C().bn_bwd_finalize(_ptr(part), T, C, float(M), _ptr(st), 0, _ptr(dgamma), _ptr(dbeta), _ptr(co), s)
    _C().bn_bwd_apply(_ptr(dy), _ptr(y), int(relu_mask), _ptr(x), _ptr(st), _ptr(co), _ptr(dx), M, C, s)


def pool_geo(x_shape, pool, strides, padding):
    n, h, w, c = x_shape
    if padding == "same":
        ho, pt, _ = same_pad(h, pool[0], strides[0])
        wo, pl, _ = same_pad(w, pool[1], strides[1])
    else:
        ho, pt = (h - pool[0]) // strides[0] + 1, 0
        wo, pl = (w - pool[1]) // strides[1] + 1, 0
    return [n, h, w, c, pool[0], pool[1], strides[0], strides[1], pt, pl, ho, wo]


def maxpool_fwd(x, y, arg, pool, strides, padding):
    g = pool_geo(x.shape, pool, strides, padding)
    _C().maxpool_fwd(_ptr(x), g, _ptr(y), _ptr(arg), stream_handle())


def maxpool_bwd(dy, arg, dx, pool, strides, padding):
    g = pool_geo(dx.shape, pool, strides, padding)
    _C().maxpool_bwd(_ptr(dy), _ptr(arg), g, _ptr(dx), stream_handle())


def bn_relu_maxpool_fwd(x, st, y, arg, pool, strides, padding):
    """y, arg = maxpool(relu(BN_st(x))) without materialising the BN output (stem fusion)."""
    g = pool_geo(x.shape, pool, strides, padding)
    _C().bn_relu_maxpool_fwd(_ptr(x), _ptr(st), g, _ptr(y), _ptr(arg), stream_handle())


def pool_bn_bwd(dpool, arg, x, st, part, co, dx, pool, strides, padding, dgamma=None, dbeta=None):
    """Backward of bn_relu_maxpool_fwd: BN batch-statistics backward with the pool routing
    and ReLU mask recomputed (reduce -> finalize (dgamma/dbeta) -> apply into dx)."""
    g = pool_geo(x.shape, pool, strides, padding)
    C = x.shape[-1]
    M = x.numel() // C
    T = _C().bn_bwd_blocks(M, C)
    assert part.numel() >= T * 2 * C
    s = stream_handle()
    _C().pool_bn_bwd_reduce(_ptr(dpool), _ptr(arg), g, _ptr(x), _ptr(st), _ptr(part), T, s)
    _C().bn_bwd_finalize(_ptr(part), T, C, float(M), _ptr(st), 0, _ptr(dgamma), _ptr(dbeta), _ptr(co), s)
    if dx is not None:
        _C().pool_bn_bwd_apply(_ptr(dpool), _ptr(arg), g, _ptr(x), _ptr(st), _ptr(co), _ptr(dx), s)


# ---- BatchNorm with the finalize folded into the consumer kernel (layer_ops.h BNFin) ------
# The producers (conv / dense GEMM epilogue with an int64 `stats` accumulator, split-K
# finish, bn_bwd_reduce with `acc`) add their per-block partials into an int64 fixed-point
# accumulator ([2C] / [reps, 2C] forward, [reps, 4C] backward: block b into replica
# b % reps; integer sums, so the statistics do not depend on the blocks' arrival order);
# the consumer derives the coefficients in its prologue, so neither bn_finalize nor
# bn_bwd_finalize is launched.  The accumulators must be zero before the producers run
# (the native graph engine clears them all in the step's gather_batch launch).
FIN_MAX_C = 4096


class BNFin:
    """Forward finalize parameters of one BatchNorm: int64 accumulator acc [2][C] (sum,
    sum of squares of the BN input), gamma / beta (None: 1 / 0), st [4][C] written by the
    consumer's block 0 (mean, invstd, scale, shift), moving statistics (None: not
    updated), the element count per channel, epsilon and the moving-average momentum."""

    def __init__(self, acc, gamma, beta, st, rmean, rvar, count, eps, momentum):
        self.acc, self.st = acc, st
        self._p = [_ptr(acc), _ptr(gamma), _ptr(beta), _ptr(st), _ptr(rmean), _ptr(rvar)]
        self._v = [float(count), float(eps), float(momentum), float(acc_reps(acc))]

    def args(self):
        return self._p, self._v


_NOFIN = ([], [])


def bn_apply_fin(x, y, fin: BNFin, relu=False, r=None, fin2: Optional[BNFin] = None):
    """bn_apply with its statistics finalized in the kernel: y = act(BN(x) [+ r | + BN2(r)])."""
    C = x.shape[-1]
    M = x.numel() // C
    mode = 0 if r is None else (1 if fin2 is None else 2)
    p1, v1 = fin.args()
    p2, v2 = fin2.args() if fin2 is not None else _NOFIN
    _C().bn_apply_fin(_ptr(x), _ptr(r), mode, int(relu), _ptr(y), M, C, p1, v1, p2, v2, stream_handle())


def bn_bwd_fin(dy, y, relu_mask, x, st, acc, co, dx, dgamma=None, dbeta=None, dz_out=None, reduce=True):
    """BN backward in two launches: bn_bwd_reduce adds sum(dz), sum(dz * xhat) into the int64
    accumulator acc [reps][4C] (two words per value; reduce=False: a conv epilogue, E_BNRED, already did); bn_bwd_apply
    derives co, adds dgamma / dbeta (block 0) and writes dx."""
    C = x.shape[-1]
    M = x.numel() // C
    T = _C().bn_bwd_blocks(M, C)
    s = stream_handle()
    r = acc_reps(acc)
    if reduce:
        _C().bn_bwd_reduce_acc(_ptr(dy), _ptr(y), int(relu_mask), _ptr(x), _ptr(st), _ptr(dz_out), _ptr(acc), T, M, C,
                               s, r)
        if dz_out is not None and relu_mask:
            # the reduce just wrote the masked gradient: the apply reads it instead of dy and
            # the mask source (one input tensor less, the same values)
            dy, y, relu_mask = dz_out, None, 0
    _C().bn_bwd_apply_fin(_ptr(dy), _ptr(y), int(relu_mask), _ptr(x), _ptr(st), _ptr(dx), M, C,
                          [_ptr(acc), _ptr(dgamma), _ptr(dbeta), _ptr(co)], float(M), s, r)


def bn_bwd_fin_dual(dy, y, relu_mask, bns):
    """Backward of two BatchNorms fed by the same (masked) gradient dy -- the two BN inputs
    of relu(BN(x) + BN(xd)) -- in two launches instead of four (bn_bwd_reduce_dual /
    bn_bwd_apply_dual: one read of dy and the mask source y for both, bitwise the single-BN
    launches).  bns: two dicts x, st, acc, co, dx, dgamma, dbeta."""
    a, b = bns
    C = a["x"].shape[-1]
    M = a["x"].numel() // C
    if b["x"].shape != a["x"].shape or acc_reps(a["acc"]) != acc_reps(b["acc"]) or relu_mask not in (0, 1):
        raise ValueError("bn_bwd_fin_dual: the two BatchNorms must match in shape and replicas")
    T = _C().bn_bwd_blocks(M, C)
    s = stream_handle()
    r = acc_reps(a["acc"])
    _C().bn_bwd_reduce_dual_acc(_ptr(dy), _ptr(y), int(relu_mask), _ptr(a["x"]), _ptr(b["x"]), _ptr(a["st"]),
                                _ptr(b["st"]), _ptr(a["acc"]), _ptr(b["acc"]), T, M, C, s, r)
    _C().bn_bwd_apply_dual_fin(_ptr(dy), _ptr(y), int(relu_mask), _ptr(a["x"]), _ptr(b["x"]), _ptr(a["st"]),
                               _ptr(b["st"]), _ptr(a["dx"]), _ptr(b["dx"]), M, C,
                               [_ptr(a["acc"]), _ptr(a.get("dgamma")), _ptr(a.get("dbeta")), _ptr(a["co"])],
                               [_ptr(b["acc"]), _ptr(b.get("dgamma")), _ptr(b.get("dbeta")), _ptr(b["co"])],
                               float(M), s, r)


def bn_relu_maxpool_fwd_fin(x, y, arg, pool, strides, padding, fin: BNFin):
    g = pool_geo(x.shape, pool, strides, padding)
    p, v = fin.args()
    _C().bn_relu_maxpool_fwd_fin(_ptr(x), g, _ptr(y), _ptr(arg), p, v, stream_handle())


def pool_bn_bwd_fin(dpool, arg, x, st, acc, co, dx, pool, strides, padding, dgamma=None, dbeta=None):
    g = pool_geo(x.shape, pool, strides, padding)
    C = x.shape[-1]
    M = x.numel() // C
    T = _C().bn_bwd_blocks(M, C)
    s = stream_handle()
    r = acc_reps(acc)
    _C().pool_bn_bwd_reduce_acc(_ptr(dpool), _ptr(arg), g, _ptr(x), _ptr(st), _ptr(acc), T, s, r)
    _C().pool_bn_bwd_apply_fin(_ptr(dpool), _ptr(arg), g, _ptr(x), _ptr(st), _ptr(dx),
                               [_ptr(acc), _ptr(dgamma), _ptr(dbeta), _ptr(co)], float(M), s, r)


def gap_fwd(x, y):
    n, h, w, c = x.shape
    _C().gap_fwd(_ptr(x), n, h * w, c, _ptr(y), int(y.dtype == torch.float32), stream_handle())


def gap_bwd(dy, dx):
    n, h, w, c = dx.shape
    _C().gap_bwd(_ptr(dy), int(dy.dtype == torch.float32), n, h * w, c, _ptr(dx), stream_handle())


def relu_bwd(dy, y, dz):
    _C().relu_bwd(_ptr(dy), _ptr(y), _ptr(dz), dy.numel(), stream_handle())


ACT_KINDS = {"relu": 0, "sigmoid": 1, "tanh": 2}


def act_fwd(x, y, kind: str):
    """y = act(x) on bf16 tensors (in place allowed); kind relu / sigmoid / tanh."""
    _C().act_fwd(_ptr(x), _ptr(y), x.numel(), ACT_KINDS[kind], stream_handle())


def act_bwd(dy, y, dx, kind: str):
    """dx = dy * act'(y) from the stored activation output y."""
    _C().act_bwd(_ptr(dy), _ptr(y), _ptr(dx), dy.numel(), ACT_KINDS[kind], stream_handle())


def dropout(x, y, ctrl, seed: int, rate: float):
    """y = x * keep / (1 - rate); keep from (seed, ctrl step t, element) -- the same call on
    dy is the backward (see dropout_mask_reference)."""
    _C().dropout(_ptr(x), _ptr(y), x.numel(), _ptr(ctrl), int(seed) & 0xFFFFFFFF, float(rate), stream_handle())


def _mix32(h):
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x85EBCA6B)
    h ^= h >> np.uint32(13)
    h *= np.uint32(0xC2B2AE35)
    h ^= h >> np.uint32(16)
    return h


def dropout_mask_reference(n: int, seed: int, t: int, rate: float) -> np.ndarray:
    """Host oracle of the dropout kernel's keep mask (bool [n]) at step t."""
    with np.errstate(over="ignore"):
        key = _mix32(np.array([(int(seed) + int(t) * 0x9E3779B9) & 0xFFFFFFFF], dtype=np.uint64))[0]
        j = np.arange(n, dtype=np.uint64).astype(np.uint32)
        h = _mix32((_mix32(j ^ key).astype(np.uint64) + int(key)) & 0xFFFFFFFF)
    thr = min(int(rate * 4294967296.0), 4294967295)
    return h >= np.uint32(thr)


def avgpool_fwd(x, y, pool, strides, padding):
    g = pool_geo(x.shape, pool, strides, padding)
    _C().avgpool_fwd(_ptr(x), g, _ptr(y), stream_handle())


def avgpool_bwd(dy, dx, pool, strides, padding):
    g = pool_geo(dx.shape, pool, strides, padding)
    _C().avgpool_bwd(_ptr(dy), g, _ptr(dx), stream_handle())


def add_bf16(a, b, out):
    _C().add_bf16(_ptr(a), _ptr(b), _ptr(out), a.numel(), stream_handle())


def colsum_workspace_elems(M: int, N: int) -> int:
    """fp32 workspace floats colsum needs for an [M][N] input (0: one pass, no workspace)."""
    sp = _C().colsum_splits(M, N)
    return sp * N if sp > 1 else 0


def colsum(x, out, workspace=None, M=None, N=None, ld=None):
    """out[n] += sum over rows of x (bf16 or fp32) in a fixed order (no float atomics)."""
    N = N or x.shape[-1]
    ld = ld or N
    M = M or x.numel() // ld
    need = colsum_workspace_elems(M, N)
    if need and (workspace is None or workspace.numel() < need):
        workspace = torch.empty(need, dtype=torch.float32, device=x.device)  # (eager callers only)
    _C().colsum(_ptr(x), int(x.dtype == torch.float32), M, N, ld, _ptr(out), stream_handle(),
                _ptr(workspace) if need else 0)


def xent_rows(B: int, device) -> torch.Tensor:
    """softmax_xent's per-row scratch: 3 B floats + the arrival counter (zeroed once)."""
    return torch.zeros(3 * B + 1, dtype=torch.float32, device=device)


def softmax_xent(logits, labels, K, scale, dlogits, tail, ctrl=None, rows=None, bias_grad=None):
    """ctrl (the engine's device control block) makes the scale 1 / real rows of the global
    batch; labels < 0 mark padding rows of a short final batch.  The loss / correct / count
    sums are formed in a fixed row order (``rows``: :func:`xent_rows` scratch).
    ``bias_grad`` (fp32 [K], optional; needs :func:`softmax_bias_fold_ok`): += the column
    sums of dlogits, bitwise as :func:`colsum` would add them."""
    B, ld = logits.shape
    if rows is None:
        rows = xent_rows(B, logits.device)  # (eager callers only: engines pass their own)
    if bias_grad is not None:
        _chk(bias_grad, torch.float32, "bias_grad")
        if bias_grad.numel() < K or not softmax_bias_fold_ok(B, K):
            raise ValueError("softmax_xent: bias_grad needs >= K floats and a one-split colsum shape")
    _C().softmax_xent(_ptr(logits), ld, _ptr(labels), B, K, float(scale), _ptr(ctrl), _ptr(dlogits), _ptr(tail),
                      _ptr(rows), stream_handle(), bias_grad=_ptr(bias_grad))


def softmax_bias_fold_ok(B: int, K: int) -> bool:
    """colsum of a [B][K] gradient runs as one split (the order softmax_xent reproduces)."""
    return _C().colsum_splits(B, K) == 1


def sgd_flat(P, G, V, Pb, lr, momentum=0.0, nesterov=False):
    _C().sgd_flat(_ptr(P), _ptr(G), _ptr(V), _ptr(Pb), P.numel(), float(lr), float(momentum), int(nesterov),
                  stream_handle())


def cast_bf16(x, y):
    _C().cast_f32_bf16(_ptr(x), _ptr(y), x.numel(), stream_handle())


def pad_cast(src, R, C1, C2, C1p, C2p, dst):
    _C().pad_cast(_ptr(src), R, C1, C2, C1p, C2p, _ptr(dst), stream_handle())


def unpad_add(src, R, C1, C2, C1p, C2p, dst):
    _C().unpad_add(_ptr(src), R, C1, C2, C1p, C2p, _ptr(dst), stream_handle())
