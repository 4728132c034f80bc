"""Device-resident input pipeline.

The whole training set lives in device memory (MNIST: 60000x784 fp32 = 188 MB of
288 GB HBM), a per-epoch permutation is generated from a seed shared by all ranks,
and each rank reads its rows of global batch ``s`` as
``perm[s*global_batch + rank*per_replica : ... + per_replica]`` — deterministic,
disjoint per-rank sharding of every global batch (the reference lets tf.distribute
auto-shard, README.md:127-132; progbar counts global samples, README.md:413).
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils.random import _GLOBAL_SEED  # noqa: F401

_BASE_SEED = 0x5EED


class DataFeed:
    def __init__(self, x, y, device: torch.device, flatten: bool = False, label_dtype=torch.int32):
        x = np.asarray(x)
        y = np.asarray(y)
        if len(x) != len(y):
            raise ValueError(f"x has {len(x)} rows but y has {len(y)}")
        self.n = int(len(x))
        self.sample_shape = tuple(x.shape[1:])
        xt = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
        if flatten:
            xt = xt.reshape(self.n, -1)
        self.x = xt.to(device)
        if y.ndim > 1 and y.shape[-1] > 1:  # one-hot / dense targets
            self.y = torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).to(device)
        elif np.issubdtype(y.dtype, np.integer) or label_dtype == torch.int32:
            self.y = torch.from_numpy(np.ascontiguousarray(y.reshape(self.n), dtype=np.int64)).to(device).to(
                torch.int32)
        else:
            self.y = torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).to(device)
        self.perm = torch.arange(self.n, dtype=torch.int32, device=device)
        self.device = device

    def set_epoch(self, epoch: int, shuffle: bool = True, seed: int = None) -> None:
        from ..utils import random as _r

        if not shuffle:
            p = torch.arange(self.n, dtype=torch.int32)
        else:
            g = torch.Generator()
            base = _r._GLOBAL_SEED if _r._GLOBAL_SEED is not None else _BASE_SEED
            g.manual_seed(int(seed if seed is not None else base) * 7919 + int(epoch))
            p = torch.randperm(self.n, generator=g).to(torch.int32)
        self.perm.copy_(p.to(self.device))

    def batch_indices(self, step: int, global_batch: int, row0: int, per_replica: int) -> torch.Tensor:
        lo = step * global_batch + row0
        hi = min(lo + per_replica, self.n)
        lo = min(lo, self.n)
        return self.perm[lo:hi].long()
