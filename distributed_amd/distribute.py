"""``tf.distribute`` facade (reference README.md:122, 187, 364)."""
from __future__ import annotations

from .parallel.strategy import (  # noqa: F401
    CollectiveCommunication,
    MultiWorkerMirroredStrategy,
    ReduceOp,
    Strategy,
    get_strategy,
    has_strategy,
)
from .parallel.cluster import ClusterSpec, parse_tf_config, resolve as resolve_cluster  # noqa: F401


class experimental:  # noqa: N801 - mirrors tf.distribute.experimental
    MultiWorkerMirroredStrategy = MultiWorkerMirroredStrategy
    CollectiveCommunication = CollectiveCommunication


class cluster_resolver:  # noqa: N801
    @staticmethod
    def TFConfigClusterResolver():  # noqa: N802
        return resolve_cluster()
