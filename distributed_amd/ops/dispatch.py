"""Device dispatch for the per-layer ops: HIP kernels for device tensors where the
native module implements them, the torch reference otherwise (CPU path)."""
from __future__ import annotations

from . import reference as _ref

conv2d = _ref.conv2d
dense = _ref.dense
maxpool2d = _ref.maxpool2d
avgpool2d = _ref.avgpool2d
batchnorm = _ref.batchnorm
sparse_softmax_xent = _ref.sparse_softmax_xent
