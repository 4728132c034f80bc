"""Tensor ops used by the Keras layers.

``reference`` holds the plain-PyTorch fp32 definitions: they are the CPU compute path
and the numerics oracle every HIP kernel is tested against.
``dispatch`` picks the HIP kernel for device tensors when one exists.
"""
from . import reference  # noqa: F401
from .dispatch import (  # noqa: F401
    conv2d,
    dense,
    maxpool2d,
    avgpool2d,
    batchnorm,
    sparse_softmax_xent,
)
