"""Diagnostics of the sharded exchange with W in-process ranks on one GPU: one step (+flush)
with a short in-kernel wait deadline; prints every rank's status word (which kind of wait
expired: 256 small message, 512 reduced unit, 1024 partial) and the flag arrays."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_sharded_inproc_gpu as T  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    nocu = os.environ.get("DIAG_NOCU") == "1"
    from distributed_amd.native import require_C

    C = require_C()
    dev = torch.device("cuda", 0)
    import distributed_amd as tf

    tf.set_seed(21)
    m = tf.models.mnist_cnn()
    P0 = torch.cat([torch.as_tensor(w).reshape(-1) for w in m.get_weights()]).float()
    P0 = torch.cat([P0, torch.zeros(T.NGRAD - T.NPARAM)]).cuda()
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.integers(0, 256, size=(1024, 784), dtype=np.uint8)).cuda()
    Y = torch.from_numpy(rng.integers(0, 10, size=1024).astype(np.int32)).cuda()
    B = 64 // W
    ranks = [T.Rank(C, dev, B, 64, r, P0, X, Y, 0.1, 0.9, 1) for r in range(W)]
    NU = 4 * C.convnet_num_slices(1)
    cap = max(W * NU * 2048, 347648 + 2 * 8 * 1408 + 16384 + T.FEAT * T.HID // 2)
    peers = [C.PeerAllreduce(W, r, 0, cap, 16, 3.0) for r in range(W)]
    for p in peers:
        p.link_local(peers)
    for r, rk in enumerate(ranks):
        rk.t.set_sharded(peers[r], rk.hred.data_ptr(), 0)
        if not nocu:
            rk.t.restrict_cus(r, W)
    torch.cuda.synchronize(dev)
    for rk in ranks:
        rk.t.step(steps)
    ok = [rk.t.sync(60.0) for rk in ranks]
    print("synced", ok, flush=True)
    for r, p in enumerate(peers):
        print("rank", r, "status", p.status(), "iters", int(ranks[r].ctrl[7]), "xcnt", int(ranks[r].ctrl[21]),
              "ticket", int(ranks[r].ctrl[23]), flush=True)
    kx = 347648 + 2 * 8 * 1408
    for r, p in enumerate(peers):
        f = np.array(p.peek_out(kx, NU * 18 + 16), dtype=np.int64)
        pf = f[:NU * 16].reshape(NU, 16)[:, :2 * W]
        gf = f[NU * 16:NU * 18].reshape(NU, 2)
        sf = f[NU * 18:].reshape(2, 8)[:, :W]
        print(f"rank {r}: partial flags (units owned: {NU // W}) min/max per src-half:",
              [(int(pf[:, k].min()), int(pf[:, k].max())) for k in range(2 * W)], flush=True)
        own = [u for u in range(NU) if u % W == r]
        print(f"rank {r}: partial flags on owned units min:", pf[own].min(0).tolist(),
              "units missing:", [u for u in own if pf[u][[k for k in range(2 * W) if k // 2 != r]].min() < steps][:10])
        print(f"rank {r}: unit flags min/max:", int(gf.min()), int(gf.max()),
              "missing:", [u for u in range(NU) if gf[u].min() < steps][:12], flush=True)
        print(f"rank {r}: small flags:", sf.tolist(), flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
