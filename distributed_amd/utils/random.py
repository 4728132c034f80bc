"""Global seeding (tf.random.set_seed analogue)."""
from __future__ import annotations

import random as _py_random

import numpy as np
import torch

_GLOBAL_SEED = None
_OP_COUNTER = 0


def set_seed(seed: int) -> None:
    global _GLOBAL_SEED, _OP_COUNTER
    _GLOBAL_SEED = int(seed)
    _OP_COUNTER = 0
    _py_random.seed(seed)
    np.random.seed(seed % (2**32))
    torch.manual_seed(seed)


def next_generator() -> torch.Generator:
    """CPU generator for one initializer call: deterministic if a global seed is set."""
    global _OP_COUNTER
    g = torch.Generator()
    if _GLOBAL_SEED is None:
        g.seed()
    else:
        _OP_COUNTER += 1
        g.manual_seed(_GLOBAL_SEED * 1000003 + _OP_COUNTER)
    return g
