"""Tensor ops used by the Keras layers.

``reference`` holds the plain-PyTorch fp32 definitions: they are the CPU compute path
and the numerics oracle every HIP kernel is tested against.
``hip`` holds the launchers of the hand-written gfx950 kernels (``csrc/kernels``); on a
GPU the engines (``distributed_amd.engine``) call them directly -- there is no per-op
dispatch layer between the two.
"""
from . import reference  # noqa: F401
from .reference import (  # noqa: F401
    conv2d,
    dense,
    maxpool2d,
    avgpool2d,
    batchnorm,
    sparse_softmax_xent,
)
