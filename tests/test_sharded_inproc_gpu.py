"""The sharded multi-rank MNIST step (convnet.h XArgs; csrc/kernels/convnet_step2.hip) with
W "ranks" inside ONE process on one GPU: W ConvNetTrainers, each on its own HIP stream
restricted to its own CUs, their exchange staging linked without IPC
(PeerAllreduce.link_local).  This isolates the exchange protocol from the multi-process
scheduling of a shared GPU (the process-per-rank path is covered by
test_peer_allreduce_gpu.py): every rank's steps are enqueued before any rank is waited
for, so the in-kernel cross-rank waits run concurrently, as on W GPUs.

Checks, for W = 2 and 3 and both exchange dtypes: bitwise-identical parameters on every
rank after several steps and a flush (deferred update, gather), the same metric sums on
every rank, and agreement with ONE rank over the whole global batch (fp32: within the
summation-order tolerance; bf16 exchange: within the stated bf16 bound)."""
import os
import struct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NPARAM, NGRAD, NCONV, FEAT, HID = 347146, 347152, 320, 5408, 64
C_LR, C_MOM, C_NEST, C_NS, C_ROW0, C_GB, C_CUR, C_IT = 0, 1, 2, 3, 4, 5, 6, 7
C_AL, C_AC, C_AN, C_WRAP = 10, 11, 12, 13


def _f2i(f):
    return struct.unpack("<i", struct.pack("<f", float(f)))[0]


def _i2f(i):
    return struct.unpack("<f", struct.pack("<i", int(i)))[0]


class Rank:
    """One rank's buffers + trainer (what FusedConvNetEngine allocates)."""

    def __init__(self, C, dev, B, GB, r, P0, X, Y, lr, mom, ppb):
        f32 = dict(dtype=torch.float32, device=dev)
        BP = (B + 63) // 64 * 64
        self.P = P0.clone()
        self.G = torch.zeros(NGRAD, **f32)
        self.V = torch.zeros(NGRAD, **f32)
        self.ctrl = torch.zeros(32, dtype=torch.int32, device=dev)
        self.w1alt = torch.zeros(FEAT * HID, **f32)
        self.v1alt = torch.zeros(FEAT * HID, **f32)
        self.w1bf = self.P[NCONV:NCONV + FEAT * HID].to(torch.bfloat16)
        self.pooled = torch.zeros(FEAT, BP, dtype=torch.bfloat16, device=dev)
        self.code = torch.zeros(B, FEAT, dtype=torch.uint8, device=dev)
        self.hacc = torch.zeros(C.convnet_hacc_elems(B), dtype=torch.int64, device=dev)
        self.hconv = torch.zeros(2 * NCONV, dtype=torch.int64, device=dev)
        self.calt = torch.zeros(2 * NCONV, **f32)
        self.hred = torch.zeros(2 * NCONV, dtype=torch.int64, device=dev)
        c = torch.zeros(32, dtype=torch.int32)
        c[C_LR], c[C_MOM], c[C_NEST] = _f2i(lr), _f2i(mom), 0
        c[C_NS], c[C_ROW0], c[C_GB], c[C_WRAP] = X.shape[0], r * B, GB, 0
        self.ctrl.copy_(c.to(dev))
        bufs = dict(params=self.P.data_ptr(), grads=self.G.data_ptr(), velocity=self.V.data_ptr(),
                    ctrl=self.ctrl.data_ptr(), pooled=self.pooled.data_ptr(), code=self.code.data_ptr(),
                    w1alt=self.w1alt.data_ptr(), v1alt=self.v1alt.data_ptr(), w1bf=self.w1bf.data_ptr(),
                    hacc=self.hacc.data_ptr(), hconv=self.hconv.data_ptr(), calt=self.calt.data_ptr(),
                    eager_w1=0, ppb=ppb)
        torch.cuda.synchronize(dev)
        self.t = C.ConvNetTrainer(dev.index or 0, bufs, B, 3, 1)
        self.t.set_data(X.data_ptr(), Y.data_ptr(), 1)

    def metrics(self):
        c = self.ctrl.cpu().tolist()
        return _i2f(c[C_AL]), _i2f(c[C_AC]), _i2f(c[C_AN])


def _run(W, B, steps, gbf16, ppb, P0, X, Y, lr=0.1, mom=0.9):
    from distributed_amd.native import require_C

    C = require_C()
    dev = torch.device("cuda", 0)
    GB = B * W
    ranks = [Rank(C, dev, B, GB, r, P0, X, Y, lr, mom, ppb) for r in range(W)]
    if W > 1:
        NU = 4 * C.convnet_num_slices(ppb)
        cap = max(W * NU * 2048, 347648 + 2 * 8 * 1408 + 16384 + FEAT * HID // 2)
        peers = [C.PeerAllreduce(W, r, 0, cap, 16, 20.0) for r in range(W)]
        for p in peers:
            p.link_local(peers)
        for r, rk in enumerate(ranks):
            rk.t.set_sharded(peers[r], rk.hred.data_ptr(), int(gbf16))
            rk.t.restrict_cus(r, W)  # each rank's own CUs (as one GPU per rank would have)
        torch.cuda.synchronize(dev)
    for rk in ranks:  # the launch contract: two kernels per step at every world size, no
        # all-reduce launch (the exchange runs inside them), no copy / memset nodes
        assert tuple(rk.t.step_graph_nodes(4)) == (8, 8), rk.t.step_graph_nodes(4)
    for _ in range(2):  # two epochs of `steps` steps, each ended by the flush
        for rk in ranks:
            rk.t.step(steps)  # enqueue only: every rank's step is in flight before any wait
        for rk in ranks:
            assert rk.t.sync(30.0)
        for rk in ranks:
            rk.t.flush()
        for rk in ranks:
            assert rk.t.sync(30.0)
    torch.cuda.synchronize(dev)
    if W > 1:
        assert all(p.status() == 0 for p in peers), [p.status() for p in peers]
    return [rk.P[:NPARAM].cpu() for rk in ranks], [rk.metrics() for rk in ranks], [int(rk.ctrl[C_IT]) for rk in ranks]


def _case(W, gbf16, ppb):
    """One case in this process (GPU_MAX_HW_QUEUES must cover the W rank streams)."""
    import distributed_amd as tf

    tf.set_seed(21)
    m = tf.models.mnist_cnn()
    P0 = torch.cat([torch.as_tensor(w).reshape(-1) for w in m.get_weights()]).float()
    P0 = torch.cat([P0, torch.zeros(NGRAD - NPARAM)]).cuda()
    rng = np.random.default_rng(3)
    n = 1024
    X = torch.from_numpy(rng.integers(0, 256, size=(n, 784), dtype=np.uint8)).cuda()
    Y = torch.from_numpy(rng.integers(0, 10, size=n).astype(np.int32)).cuda()
    B = 64 // W
    Ps, mets, its = _run(W, B, 3, gbf16, ppb, P0, X, Y)
    P1, met1, _ = _run(1, B * W, 3, 0, ppb, P0, X, Y)  # one rank over the same global batch
    return {"its": its, "replicas_equal": all(torch.equal(p, Ps[0]) for p in Ps[1:]),
            "metrics": mets, "metrics1": met1[0], "maxdiff": (Ps[0] - P1[0]).abs().max().item(),
            "maxupd": (P1[0] - P0[:NPARAM].cpu()).abs().max().item(), "gb": B * W}


# W <= 3: a process gets at most 4 concurrently scheduled hardware queues on this pool
# (measured: with 4 or 8 rank streams in one process, whatever GPU_MAX_HW_QUEUES and CU
# masks, only ~4 streams' kernels run at once, so a rank's in-kernel wait for a rank whose
# stream is not scheduled expires; scripts/diag_sharded.py shows every flag of W = 4 and 8
# arriving, late).  One process per GPU -- the deployment -- has no such limit.
@pytest.mark.parametrize("W,gbf16,ppb", [(2, 0, 1), (3, 0, 1), (3, 1, 1), (2, 0, 3), (2, 1, 3)])
@pytest.mark.timeout(300)
def test_sharded_exchange_in_process(W, gbf16, ppb, tmp_path):
    # a child process: one HIP hardware queue per rank stream (GPU_MAX_HW_QUEUES), else two
    # ranks' kernels could share a queue and one would wait behind the other's spin
    import json
    import subprocess
    import sys

    out = tmp_path / "r.json"
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), str(W), str(gbf16), str(ppb), str(out)], env=env,
                       timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.load(open(out))
    assert j["its"] == [6] * W
    assert j["replicas_equal"], "replicas diverged"
    mets, met1 = j["metrics"], j["metrics1"]
    assert all(mt == mets[0] for mt in mets), mets
    # fp32 exchange: summation order only (<= 0.2 % of the largest update after 6 momentum
    # steps at lr 0.1).  bf16 exchange: every exchanged gradient rounded to bf16 (relative
    # 2^-9); the bf16 forward of later steps amplifies that (ReLU / max-pool decisions near
    # ties): measured 1-3.3 % of the largest update -- the stated bound is 5 %
    d, upd = j["maxdiff"], j["maxupd"]
    assert d <= (5e-2 if gbf16 else 2e-3) * upd + 1e-6, (d, upd)
    assert abs(mets[0][0] - met1[0]) <= 1e-3 * abs(met1[0]), (mets[0], met1)
    assert mets[0][2] == met1[2] == 2 * 3 * j["gb"] and abs(mets[0][1] - met1[1]) <= 2


if __name__ == "__main__":
    import json
    import sys

    W, gbf16, ppb, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    with open(out, "w") as f:
        json.dump(_case(W, gbf16, ppb), f)
