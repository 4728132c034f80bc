"""The start-up self-test's set-up vote (engine/xchg_selftest.py) on CPU, with the native
set-up stubbed: every rank gets the set-up's result or every rank gets None (a
rank whose restrict_cus / set_sharded raised must not fall out of step with the others),
and the arguments reach _setup unchanged (a round-6 regression passed `kind` twice)."""
from distributed_amd.engine import xchg_selftest as X


class _Comm:
    def __init__(self, others):
        self.others = others  # what the other ranks report
        self.barriers = 0

    def allgather_object(self, obj):
        return [obj] + list(self.others)

    def barrier(self):
        self.barriers += 1


def test_voted_setup_passes_arguments_through(monkeypatch):
    seen = []
    monkeypatch.setattr(X, "_setup", lambda *a: seen.append(a) or "scratch")
    comm = _Comm([""])
    s, why = X._voted_setup("xgmi-peer", comm, "xgmi-peer", "C", comm, "peer", None, "dev", 64, 128, 0,
                            "P0", "X", "Y", 2, 3, False, None)
    assert s == "scratch" and why == ""
    assert seen == [("xgmi-peer", "C", comm, "peer", None, "dev", 64, 128, 0, "P0", "X", "Y", 2, 3, False, None)]
    assert comm.barriers == 0  # the barrier belongs to the sharded exchange only
    X._voted_setup("xgmi-sharded", comm, "xgmi-sharded", "C", comm, "peer", None, "dev", 64, 128, 0,
                   "P0", "X", "Y", 2, 3, False, None)
    assert comm.barriers == 1


def test_voted_setup_failure_on_another_rank_fails_every_rank(monkeypatch):
    monkeypatch.setattr(X, "_setup", lambda *a: "scratch")
    comm = _Comm(["set-up raised RuntimeError('restrict_cus')"])
    s, why = X._voted_setup("xgmi-sharded", comm, "xgmi-sharded", "C", comm, "peer", None, "dev", 64, 128, 0,
                            "P0", "X", "Y", 2, 3, False, None)
    assert s is None and "rank 1" in why and "restrict_cus" in why
    assert comm.barriers == 0  # no rank enters the sharded barrier after a failed set-up


def test_voted_setup_local_failure(monkeypatch):
    def boom(*a):
        raise RuntimeError("set_sharded")

    monkeypatch.setattr(X, "_setup", boom)
    s, why = X._voted_setup("xgmi-peer", _Comm([""]), "xgmi-peer")
    assert s is None and "rank 0" in why and "set_sharded" in why
