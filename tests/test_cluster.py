import json

import pytest

from distributed_amd.parallel import cluster


def test_python_form():
    raw = json.dumps({"cluster": {"worker": ["172.17.0.6:10090", "172.17.0.3:10088", "172.17.0.4:10087",
                                             "172.17.0.5:10089"]}, "task": {"type": "worker", "index": 2}})
    s = cluster.parse_tf_config(raw)
    assert s.num_workers == 4 and s.task_id == 2 and not s.is_chief
    assert s.chief_address == "172.17.0.6:10090"


def test_r_auto_unbox_scalar_worker_and_list_index():
    # jsonlite::toJSON(auto_unbox=TRUE) of a length-1 vector gives a bare string
    s = cluster.parse_tf_config('{"cluster":{"worker":"10.0.0.1:8001"},"task":{"type":"worker","index":[0]}}')
    assert s.workers == ["10.0.0.1:8001"] and s.task_id == 0 and s.is_chief


def test_spark_form_ports():
    # README.md:180-183: paste(gsub(":[0-9]+$", "", address), 8000 + seq_along(address), sep=":")
    addrs = ["h1:4040", "h2:4041", "h3:4042"]
    import re

    workers = [f"{re.sub(r':[0-9]+$', '', a)}:{8000 + i + 1}" for i, a in enumerate(addrs)]
    s = cluster.parse_tf_config(cluster.tf_config_json(workers, 1))
    assert s.workers == ["h1:8001", "h2:8002", "h3:8003"] and s.rank == 1


@pytest.mark.parametrize("raw", [
    "not json",
    '{"cluster":{"ps":["a:1"]},"task":{"type":"ps","index":0}}',
    '{"cluster":{"worker":["a:1"]},"task":{"type":"evaluator","index":0}}',
    '{"cluster":{"worker":["a:1"]},"task":{"type":"worker","index":3}}',
    '{"cluster":{"worker":["nohostport"]},"task":{"type":"worker","index":0}}',
    '{"cluster":{"worker":["a:99999"]},"task":{"type":"worker","index":0}}',
])
def test_rejects(raw):
    with pytest.raises(cluster.ClusterConfigError):
        cluster.parse_tf_config(raw)


def test_resolve_precedence():
    env = {"TF_CONFIG": cluster.tf_config_json(["127.0.0.1:5000", "127.0.0.1:5001"], 1),
           "WORLD_SIZE": "8", "RANK": "3"}
    s = cluster.resolve(env)
    assert s.source == "tf_config" and s.num_workers == 2 and s.rank == 1
    s = cluster.resolve({"WORLD_SIZE": "4", "RANK": "3", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1234",
                         "LOCAL_RANK": "3"})
    assert s.source == "torchrun" and s.num_workers == 4 and s.rank == 3 and s.local_rank == 3
    s = cluster.resolve({})
    assert s.num_workers == 1 and s.is_chief


def test_tf_config_roundtrip_property():
    """Any worker list (list or R's auto-unboxed scalar for one worker) and any valid index
    (int or R's length-1 vector) parses back to the same cluster (hypothesis-drawn)."""
    hyp = pytest.importorskip("hypothesis")
    from hypothesis import given, settings
    from hypothesis import strategies as st

    host = st.from_regex(r"[a-z][a-z0-9\-]{0,14}(\.[a-z0-9]{1,8}){0,2}", fullmatch=True)
    port = st.integers(1, 65535)

    @settings(max_examples=150, deadline=None, derandomize=True, database=None)
    @given(hosts=st.lists(st.tuples(host, port), min_size=1, max_size=8), data=st.data(),
           boxed=st.booleans(), scalar=st.booleans())
    def check(hosts, data, boxed, scalar):
        workers = [f"{h}:{p}" for h, p in hosts]
        idx = data.draw(st.integers(0, len(workers) - 1))
        w = workers[0] if (scalar and len(workers) == 1) else workers
        raw = json.dumps({"cluster": {"worker": w}, "task": {"type": "worker", "index": [idx] if boxed else idx}})
        s = cluster.parse_tf_config(raw)
        assert s.workers == workers and s.num_workers == len(workers)
        assert s.task_id == idx and s.is_chief == (idx == 0)
        assert s.chief_address == workers[0]
        assert cluster.parse_tf_config(cluster.tf_config_json(workers, idx)).workers == workers

    check()
