"""``tf.keras`` surface used by the reference (README.md:58-75, 282-304, 363-392)."""
from __future__ import annotations

from . import activations, backend, callbacks, datasets, initializers, layers, losses, metrics, optimizers  # noqa
from . import utils  # noqa: F401
from .layers import Input  # noqa: F401
from .models import Model, Sequential  # noqa: F401
from . import models  # noqa: F401

__version__ = "2.2.4-tf"
