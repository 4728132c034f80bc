"""distributed_amd — an MI355X-native multi-worker data-parallel training framework.

It offers the capabilities of the Mrhs121/distributed reference (a TF 2.0 / Keras
tutorial, reference README.md) re-designed for AMD MI355X (gfx950):

* ``import distributed_amd as tf`` exposes the ``tf.keras`` surface the reference uses
  (``Sequential``, ``layers.Conv2D/MaxPooling2D/Flatten/Dense``, ``losses``,
  ``optimizers.SGD``, ``compile``/``fit``/``History``/``Progbar``, ``datasets.mnist``)
  and ``tf.distribute.experimental.MultiWorkerMirroredStrategy`` driven by ``TF_CONFIG``.
* Compute: PyTorch-ROCm tensors + hand-written CDNA4 HIP kernels (``csrc/kernels``);
  the reference CNN trains through a fused 3-launch step captured in a hipGraph.
* Communication: RCCL all-reduce over xGMI from a native communicator (one process
  per GPU); gloo on CPU.
* Launch: ``python -m distributed_amd.launch`` / ``barrier_apply`` (Spark-barrier
  gang semantics); checkpoints: Keras-layout HDF5 via libhdf5 (``csrc/io``).
"""
from __future__ import annotations

import torch  # noqa: F401  (must be imported before the native module: shared HIP/RCCL libs)

# ``tf.__version__`` reports the API level of the TF surface this framework reproduces
# (reference README.md:263-266 prints ``2.0.0``); the framework's own release is
# ``FRAMEWORK_VERSION``.
API_VERSION = "2.0.0"
__version__ = API_VERSION
FRAMEWORK_VERSION = "0.3.0"

from . import utils  # noqa: E402
from . import parallel  # noqa: E402
from . import keras  # noqa: E402
from . import distribute  # noqa: E402
from . import models  # noqa: E402
from .utils.random import set_seed  # noqa: E402


class _RandomNS:
    set_seed = staticmethod(set_seed)


random = _RandomNS()


def tf_version() -> str:
    """R ``tensorflow::tf_version()`` analogue (reference README.md:35-40): API level."""
    return ".".join(API_VERSION.split(".")[:2])


def install_tensorflow(*args, **kwargs) -> None:
    """R ``install_tensorflow()`` analogue: nothing to install (validates the runtime)."""
    from .native import native_status

    native_status()


__all__ = ["keras", "distribute", "parallel", "models", "utils", "random", "tf_version", "__version__"]
