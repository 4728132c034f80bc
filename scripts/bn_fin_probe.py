"""BatchNorm finalize folded into the consumer (layer_ops.h BNFin): time of the producer
(bn_bwd_reduce adding into `reps` fp64 replicas) and of the row-mapped consumers (bn_apply /
bn_bwd_apply finalizing in their prologue) on the ResNet-18 layer shapes, against the
partials + finalize + apply launches.  GPU box:
    python scripts/bn_fin_probe.py [reps ...]      (env DAMD_BN_FIN_GRID caps the grid)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.native import require_C  # noqa: E402
from distributed_amd.ops import hip as H  # noqa: E402

dev = torch.device("cuda:0")
C_ = require_C()
REPS = [int(a) for a in sys.argv[1:]] or [1, 8]


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for (hw, c) in [(56, 64), (28, 128), (14, 256), (7, 512)]:
    M = 64 * hw * hw
    x = torch.randn(M, c, device=dev).bfloat16()
    dy = torch.randn(M, c, device=dev).bfloat16()
    out = torch.empty_like(x)
    st = torch.zeros(4, c, device=dev)
    co = torch.zeros(3, c, device=dev)
    gamma, beta = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
    T = C_.bn_bwd_blocks(M, c)
    part = torch.zeros(T, 2, c, device=dev)
    s = H.stream_handle()
    ident = torch.zeros(4, c, device=dev)
    ident[1] = 1.0

    def base():
        C_.bn_bwd_reduce(x.data_ptr(), 0, 0, x.data_ptr(), ident.data_ptr(), 0, part.data_ptr(), T, M, c, s)
        H.bn_finalize(part, T, c, M, gamma, beta, 1e-3, 0.99, rm, rv, st)
        H.bn_apply(x, st, out, relu=True)

    def bwd_base():
        C_.bn_bwd_reduce(dy.data_ptr(), 0, 2, x.data_ptr(), st.data_ptr(), 0, part.data_ptr(), T, M, c, s)
        C_.bn_bwd_finalize(part.data_ptr(), T, c, float(M), st.data_ptr(), 0, 0, 0, co.data_ptr(), s)
        C_.bn_bwd_apply(dy.data_ptr(), 0, 2, x.data_ptr(), st.data_ptr(), co.data_ptr(), out.data_ptr(), M, c, s)

    tb, tbb = timeit(base), timeit(bwd_base)
    print(f"{hw}x{hw}x{c} (M {M}, T {T}): partials+finalize+apply fwd {tb:6.2f} us  bwd {tbb:6.2f} us")
    for r in REPS:
        acc = torch.zeros(r + 1, 4 * c, dtype=torch.int64, device=dev)  # (backward layout: 2 words / value; + flag plane)
        fin = H.BNFin(acc, gamma, beta, st, rm, rv, M, 1e-3, 0.99)
        red = lambda: C_.bn_bwd_reduce_acc(x.data_ptr(), 0, 0, x.data_ptr(), ident.data_ptr(), 0, acc.data_ptr(),
                                           T, M, c, s, r)
        app = lambda: H.bn_apply_fin(x, out, fin, relu=True)
        bapp = lambda: C_.bn_bwd_apply_fin(dy.data_ptr(), 0, 2, x.data_ptr(), st.data_ptr(), out.data_ptr(), M, c,
                                           [acc.data_ptr(), 0, 0, co.data_ptr()], float(M), s, r)
        tr, ta, tba = timeit(red), timeit(app), timeit(bapp)
        both = timeit(lambda: (red(), app()))
        print(f"   reps {r:2d}: reduce(acc) {tr:6.2f}  apply(fin) {ta:6.2f}  bwd apply(fin) {tba:6.2f}  "
              f"reduce+apply {both:6.2f} us")
