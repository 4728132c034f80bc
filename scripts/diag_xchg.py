#!/usr/bin/env python
"""Diagnostics: run the fused MNIST trainer at W = 2 (ranks sharing cuda:0) under several
gradient-exchange settings, several times each, and print per-tensor replica / vs-host
differences (tests/helpers/dist_worker.py; the same runs as
test_fused_exchanges_bitwise_equal_host_rank_order_reduction)."""
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from distributed_amd import launch  # noqa: E402

WORKER = str(ROOT / "tests" / "helpers" / "dist_worker.py")


def run(d, **kw):
    d.mkdir()
    env = {"DAMD_DEVICE": "cuda:0", "DAMD_COMM": "gloo", "DAMD_TEST_OUT": str(d), "PYTHONPATH": str(ROOT),
           "OMP_NUM_THREADS": "2", "DAMD_LOG_LEVEL": "WARNING", "DAMD_WATCHDOG_S": "20",
           "DAMD_TEST_PER_REPLICA": "32", "DAMD_TEST_STEPS": "8", "DAMD_GRAPH_STEPS": "5"}
    env.update({k: str(v) for k, v in kw.items()})
    res = launch.launch_script([WORKER], nproc=2, env=env, timeout=300)
    if not res.ok:
        return None
    return [([a for a in np.load(d / f"rank{r}.npz").values()], json.load(open(d / f"rank{r}.json"))) for r in range(2)]


def main():
    cases = [c for c in (sys.argv[1:] or ["xgmi", "injected", "xgmi", "injected"])]
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        host = run(td / "host", DAMD_ALLREDUCE="off")
        init = td / "host" / "init0.npz"
        wh = host[0][0]
        for i, c in enumerate(cases):
            kw = {"xgmi": dict(DAMD_ALLREDUCE="xgmi"), "sharded": dict(DAMD_ALLREDUCE="sharded"),
                  "injected": dict(DAMD_ALLREDUCE="auto", DAMD_XCHG_SELFTEST_INJECT="xgmi-sharded:1"),
                  "noselftest": dict(DAMD_ALLREDUCE="xgmi", DAMD_XCHG_SELFTEST="0"),
                  "nofold": dict(DAMD_ALLREDUCE="xgmi", DAMD_PEER_FOLD="0"),
                  "sharded_nopf": dict(DAMD_ALLREDUCE="sharded", DAMD_XPREFETCH="0"),
                  "sharded_nohint": dict(DAMD_ALLREDUCE="sharded", DAMD_PAR_HINT="0"),
                  "sharded_plain": dict(DAMD_ALLREDUCE="sharded", DAMD_PAR_HINT="0", DAMD_XPREFETCH="0"),
                  "xgmi_plain": dict(DAMD_ALLREDUCE="xgmi", DAMD_PAR_HINT="0", DAMD_XPREFETCH="0"),
                  "sharded_nograph": dict(DAMD_ALLREDUCE="sharded", DAMD_GRAPH="0"),
                  "xgmi_nograph": dict(DAMD_ALLREDUCE="xgmi", DAMD_GRAPH="0"),
                  "sharded_nopc": dict(DAMD_ALLREDUCE="sharded", DEBUG_CLR_GRAPH_PACKET_CAPTURE="0"),
                  "xgmi_nopc": dict(DAMD_ALLREDUCE="xgmi", DEBUG_CLR_GRAPH_PACKET_CAPTURE="0")}[c]
            r = run(td / f"{c}{i}", DAMD_TEST_INIT_FROM=init, **kw)
            if r is None:
                print(c, "FAILED to run", flush=True)
                continue
            (w0, j0), (w1, j1) = r
            rep = [float(np.abs(a - b).max()) for a, b in zip(w0, w1)]
            vsh = [float(np.abs(a - b).max()) for a, b in zip(w0, wh)]
            vsh1 = [float(np.abs(a - b).max()) for a, b in zip(w1, wh)]
            print(f"{c}: exchange {j0['exchange']} fb {j0['fallback_from']} | replica diff {rep} | "
                  f"r0 vs host {vsh} | r1 vs host {vsh1} | hist eq {j0['history'] == j1['history']}", flush=True)


if __name__ == "__main__":
    main()
