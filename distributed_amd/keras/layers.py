"""Keras layers (tf.keras 2.0 semantics) over torch tensors.

Layers used by the reference model (reference README.md:58-68, 292-298):
``Conv2D``, ``MaxPooling2D``, ``Flatten``, ``Dense`` — with Keras default arguments,
initializers, NHWC layout and auto-naming (``conv2d``, ``max_pooling2d``, ``flatten``,
``dense``, ``dense_1``).  The extra layers (BatchNormalization, Add, pooling variants,
ZeroPadding2D, Activation, Dropout, Reshape, Input) support the functional API and
ResNet-18 (BASELINE.json:10).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from . import activations as _act
from . import backend as K
from . import initializers as _init


def _pair(v):
    if isinstance(v, (list, tuple)):
        return tuple(int(a) for a in v)
    return (int(v), int(v))


def _current_device() -> torch.device:
    from ..parallel.strategy import get_strategy

    return get_strategy().device


class Variable:
    """A named model variable; storage may be relocated into a flat engine buffer."""

    def __init__(self, name: str, value: torch.Tensor, trainable: bool = True, aggregation: str = "none"):
        self.name = name
        self._t = value
        self.trainable = trainable
        # tf.VariableAggregation of a mirrored variable read across replicas: "mean" marks
        # the SyncOnRead BN moving statistics (each replica updates its own copy, readers
        # see the replica mean), "none" variables are kept identical by construction
        self.aggregation = aggregation
        # weakref to the engine whose flat buffer holds this variable: host writes go
        # through its before/after hooks (flush a deferred update, refresh bf16 shadows)
        self._engine_ref = None

    @property
    def value(self) -> torch.Tensor:
        return self._t

    @property
    def shape(self):
        return tuple(self._t.shape)

    @property
    def dtype(self):
        return self._t.dtype

    def numpy(self) -> np.ndarray:
        return self._t.detach().to("cpu", torch.float32).numpy().copy()

    def assign(self, v) -> None:
        t = torch.as_tensor(np.asarray(v), dtype=self._t.dtype)
        if tuple(t.shape) != self.shape:
            raise ValueError(f"assign shape {tuple(t.shape)} != {self.shape} for {self.name}")
        eng = self._engine_ref() if self._engine_ref is not None else None
        if eng is not None:
            eng.before_external_write()
        with torch.no_grad():
            self._t.copy_(t.to(self._t.device))
        if eng is not None:
            eng.after_external_write()

    def _rebind(self, storage: torch.Tensor) -> None:
        """Point this variable at ``storage`` (same shape), copying the current value."""
        with torch.no_grad():
            storage.copy_(self._t.to(storage.device))
        self._t = storage

    def __repr__(self):
        return f"<Variable '{self.name}' shape={self.shape} dtype={self.dtype}>"


class KerasTensor:
    """Symbolic tensor of the functional API (shape excludes nothing: batch is None).

    ``node_index`` numbers the calls of ``layer`` (a layer applied twice owns two nodes):
    Keras' ``inbound_nodes`` / ``input_layers`` entries are ``[layer_name, node_index,
    tensor_index]``."""

    def __init__(self, shape, layer=None, inputs=None, node_index=0):
        self.shape = tuple(shape)
        self.layer = layer
        self.inputs = inputs or []
        self.node_index = node_index

    def __repr__(self):
        return f"<KerasTensor shape={self.shape}>"


class Layer:
    def __init__(self, name: Optional[str] = None, input_shape=None, batch_input_shape=None, trainable=True,
                 dtype=None, **kwargs):
        self.name = name or K.unique_name(K.to_snake_case(type(self).__name__))
        self.trainable = trainable
        self.built = False
        self._weights: List[Variable] = []
        if batch_input_shape is not None:
            self._batch_input_shape = tuple(batch_input_shape)
        elif input_shape is not None:
            self._batch_input_shape = (None,) + tuple(int(d) for d in input_shape)
        else:
            self._batch_input_shape = None
        self.input_shape = None
        self.output_shape = None

    # --- weights -------------------------------------------------------------
    def add_weight(self, name, shape, initializer="zeros", trainable=True, aggregation="none") -> Variable:
        init = _init.get(initializer)
        val = init(tuple(shape)).to(torch.float32).to(_current_device())
        v = Variable(f"{self.name}/{name}:0", val, trainable, aggregation)
        self._weights.append(v)
        return v

    @property
    def weights(self) -> List[Variable]:
        return self.trainable_weights + self.non_trainable_weights

    @property
    def trainable_weights(self) -> List[Variable]:
        return [w for w in self._weights if w.trainable and self.trainable]

    @property
    def non_trainable_weights(self) -> List[Variable]:
        return [w for w in self._weights if not (w.trainable and self.trainable)]

    def get_weights(self):
        return [w.numpy() for w in self.weights]

    def set_weights(self, values):
        ws = self.weights
        if len(values) != len(ws):
            raise ValueError(f"layer {self.name} expects {len(ws)} weights, got {len(values)}")
        for w, v in zip(ws, values):
            w.assign(v)

    def count_params(self) -> int:
        return int(sum(int(np.prod(w.shape)) for w in self.weights))

    # --- build / call ----------------------------------------------------------
    def build(self, input_shape):
        self.built = True

    def _maybe_build(self, input_shape):
        if not self.built:
            self.input_shape = tuple(input_shape)
            self.build(tuple(input_shape))
            self.built = True
            self.output_shape = self.compute_output_shape(tuple(input_shape))

    def compute_output_shape(self, input_shape):
        return input_shape

    def call(self, x, training=False):
        raise NotImplementedError

    def __call__(self, x, training=False):
        if isinstance(x, KerasTensor) or (isinstance(x, (list, tuple)) and x and isinstance(x[0], KerasTensor)):
            ins = list(x) if isinstance(x, (list, tuple)) else [x]
            shp = [t.shape for t in ins] if isinstance(x, (list, tuple)) else x.shape
            self._maybe_build(shp)
            self._n_nodes = getattr(self, "_n_nodes", 0) + 1
            return KerasTensor(self.compute_output_shape(shp), self, ins, node_index=self._n_nodes - 1)
        shp = [tuple(t.shape) for t in x] if isinstance(x, (list, tuple)) else tuple(x.shape)
        self._maybe_build(shp)
        return self.call(x, training=training)

    def get_config(self) -> dict:
        cfg = {"name": self.name, "trainable": self.trainable, "dtype": "float32"}
        if self._batch_input_shape is not None:
            cfg["batch_input_shape"] = list(self._batch_input_shape)
        return cfg

    @classmethod
    def from_config(cls, config):
        return cls(**config)


class InputLayer(Layer):
    def __init__(self, input_shape=None, batch_size=None, name=None, sparse=False, **kw):
        super().__init__(name=name or K.unique_name("input"), input_shape=input_shape, **kw)

    def call(self, x, training=False):
        return x

    def get_config(self):
        return {"batch_input_shape": list(self._batch_input_shape), "dtype": "float32", "sparse": False,
                "name": self.name}


def Input(shape, batch_size=None, name=None):  # noqa: N802
    lyr = InputLayer(input_shape=tuple(shape), name=name)
    lyr._n_nodes = 1
    t = KerasTensor((batch_size,) + tuple(shape), lyr, [], node_index=0)
    lyr.built = True
    lyr.output_shape = t.shape
    return t


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", data_format=None, dilation_rate=(1, 1),
                 activation=None, use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 **kw):
        super().__init__(**kw)
        if data_format not in (None, "channels_last"):
            raise ValueError("only channels_last (NHWC) is supported, as in the reference")
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        self.dilation_rate = _pair(dilation_rate)
        self.activation = _act.get(activation)
        self.use_bias = use_bias
        self.kernel_initializer = _init.get(kernel_initializer)
        self.bias_initializer = _init.get(bias_initializer)
        if self._batch_input_shape is not None:
            self._maybe_build(self._batch_input_shape)

    def build(self, input_shape):
        cin = int(input_shape[-1])
        self.kernel = self.add_weight("kernel", self.kernel_size + (cin, self.filters), self.kernel_initializer)
        self.bias = self.add_weight("bias", (self.filters,), self.bias_initializer) if self.use_bias else None

    def compute_output_shape(self, s):
        n, h, w, _ = s
        out = []
        for size, k, st, d in zip((h, w), self.kernel_size, self.strides, self.dilation_rate):
            eff = (k - 1) * d + 1
            out.append(None if size is None else
                       (math.ceil(size / st) if self.padding == "same" else (size - eff) // st + 1))
        return (n, out[0], out[1], self.filters)

    def call(self, x, training=False):
        y = ops.conv2d(x, self.kernel.value, self.bias.value if self.bias is not None else None,
                       self.strides, self.padding, self.dilation_rate)
        return self.activation(y)

    def get_config(self):
        c = super().get_config()
        c.update(filters=self.filters, kernel_size=list(self.kernel_size), strides=list(self.strides),
                 padding=self.padding, data_format="channels_last", dilation_rate=list(self.dilation_rate),
                 activation=_act.serialize(self.activation), use_bias=self.use_bias,
                 kernel_initializer=_init.serialize(self.kernel_initializer),
                 bias_initializer=_init.serialize(self.bias_initializer),
                 kernel_regularizer=None, bias_regularizer=None, activity_regularizer=None,
                 kernel_constraint=None, bias_constraint=None)
        return c


class _Pool2D(Layer):
    _op = None

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", data_format=None, **kw):
        super().__init__(**kw)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding.lower()

    def compute_output_shape(self, s):
        n, h, w, c = s
        out = []
        for size, k, st in zip((h, w), self.pool_size, self.strides):
            out.append(None if size is None else
                       (math.ceil(size / st) if self.padding == "same" else (size - k) // st + 1))
        return (n, out[0], out[1], c)

    def get_config(self):
        c = super().get_config()
        c.update(pool_size=list(self.pool_size), padding=self.padding, strides=list(self.strides),
                 data_format="channels_last")
        return c


class MaxPooling2D(_Pool2D):
    def call(self, x, training=False):
        return ops.maxpool2d(x, self.pool_size, self.strides, self.padding)


class AveragePooling2D(_Pool2D):
    def call(self, x, training=False):
        return ops.avgpool2d(x, self.pool_size, self.strides, self.padding)


MaxPool2D = MaxPooling2D
AvgPool2D = AveragePooling2D


class GlobalAveragePooling2D(Layer):
    def compute_output_shape(self, s):
        return (s[0], s[-1])

    def call(self, x, training=False):
        return x.mean(dim=(1, 2))

    def get_config(self):
        c = super().get_config()
        c["data_format"] = "channels_last"
        return c


class GlobalMaxPooling2D(GlobalAveragePooling2D):
    def call(self, x, training=False):
        return x.amax(dim=(1, 2))


class Flatten(Layer):
    def compute_output_shape(self, s):
        rest = s[1:]
        return (s[0], None if any(d is None for d in rest) else int(np.prod(rest)))

    def call(self, x, training=False):
        return x.reshape(x.shape[0], -1)  # NHWC row-major: Keras-compatible feature order

    def get_config(self):
        c = super().get_config()
        c["data_format"] = "channels_last"
        return c


class Reshape(Layer):
    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(target_shape)

    def compute_output_shape(self, s):
        return (s[0],) + self.target_shape

    def call(self, x, training=False):
        return x.reshape((x.shape[0],) + self.target_shape)

    def get_config(self):
        c = super().get_config()
        c["target_shape"] = list(self.target_shape)
        return c


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = _act.get(activation)
        self.use_bias = use_bias
        self.kernel_initializer = _init.get(kernel_initializer)
        self.bias_initializer = _init.get(bias_initializer)
        if self._batch_input_shape is not None:
            self._maybe_build(self._batch_input_shape)

    def build(self, input_shape):
        fin = int(input_shape[-1])
        self.kernel = self.add_weight("kernel", (fin, self.units), self.kernel_initializer)
        self.bias = self.add_weight("bias", (self.units,), self.bias_initializer) if self.use_bias else None

    def compute_output_shape(self, s):
        return tuple(s[:-1]) + (self.units,)

    def call(self, x, training=False):
        y = ops.dense(x, self.kernel.value, self.bias.value if self.bias is not None else None)
        return self.activation(y)

    def get_config(self):
        c = super().get_config()
        c.update(units=self.units, activation=_act.serialize(self.activation), use_bias=self.use_bias,
                 kernel_initializer=_init.serialize(self.kernel_initializer),
                 bias_initializer=_init.serialize(self.bias_initializer),
                 kernel_regularizer=None, bias_regularizer=None, activity_regularizer=None,
                 kernel_constraint=None, bias_constraint=None)
        return c


class Activation(Layer):
    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation = _act.get(activation)

    def call(self, x, training=False):
        return self.activation(x)

    def get_config(self):
        c = super().get_config()
        c["activation"] = _act.serialize(self.activation)
        return c


class ReLU(Layer):
    def call(self, x, training=False):
        return torch.relu(x)


class Softmax(Layer):
    def call(self, x, training=False):
        return torch.softmax(x, dim=-1)


class Dropout(Layer):
    def __init__(self, rate, noise_shape=None, seed=None, **kw):
        super().__init__(**kw)
        self.rate = float(rate)
        self.seed = seed

    def call(self, x, training=False):
        if not training or self.rate == 0.0:
            return x
        return torch.nn.functional.dropout(x, self.rate, training=True)

    def get_config(self):
        c = super().get_config()
        c.update(rate=self.rate, noise_shape=None, seed=self.seed)
        return c


class ZeroPadding2D(Layer):
    def __init__(self, padding=(1, 1), **kw):
        super().__init__(**kw)
        if isinstance(padding, int):
            padding = ((padding, padding), (padding, padding))
        elif isinstance(padding[0], int):
            padding = ((padding[0], padding[0]), (padding[1], padding[1]))
        self.padding = tuple(tuple(p) for p in padding)

    def compute_output_shape(self, s):
        (t, b), (l, r) = self.padding
        return (s[0], None if s[1] is None else s[1] + t + b, None if s[2] is None else s[2] + l + r, s[3])

    def call(self, x, training=False):
        (t, b), (l, r) = self.padding
        return torch.nn.functional.pad(x, (0, 0, l, r, t, b))

    def get_config(self):
        c = super().get_config()
        c["padding"] = [list(p) for p in self.padding]
        return c


class BatchNormalization(Layer):
    """Keras BN over channels (axis=-1).  Under MWMS the batch statistics are per
    replica, as tf.keras 2.0's (non-synced) BatchNormalization; the moving
    statistics are SyncOnRead variables with MEAN aggregation (created inside
    ``strategy.scope()``, reference README.md:134-151): every replica updates its own
    copy and the model averages them across replicas at each epoch end (before
    validation, callbacks and checkpoints read them), so every worker holds, saves and
    evaluates with the replica mean."""

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        self.axis, self.momentum, self.epsilon, self.center, self.scale = axis, momentum, epsilon, center, scale

    def build(self, input_shape):
        c = int(input_shape[-1])
        self.gamma = self.add_weight("gamma", (c,), "ones") if self.scale else None
        self.beta = self.add_weight("beta", (c,), "zeros") if self.center else None
        self.moving_mean = self.add_weight("moving_mean", (c,), "zeros", trainable=False, aggregation="mean")
        self.moving_variance = self.add_weight("moving_variance", (c,), "ones", trainable=False,
                                               aggregation="mean")

    def call(self, x, training=False):
        g = self.gamma.value if self.gamma is not None else torch.ones(x.shape[-1], device=x.device)
        b = self.beta.value if self.beta is not None else torch.zeros(x.shape[-1], device=x.device)
        return ops.batchnorm(x, g, b, self.moving_mean.value, self.moving_variance.value,
                             training and self.trainable, self.momentum, self.epsilon)

    def get_config(self):
        c = super().get_config()
        c.update(axis=self.axis, momentum=self.momentum, epsilon=self.epsilon, center=self.center,
                 scale=self.scale)
        return c


class Add(Layer):
    def compute_output_shape(self, shapes):
        return tuple(shapes[0])

    def call(self, xs, training=False):
        out = xs[0]
        for t in xs[1:]:
            out = out + t
        return out


def add(inputs):
    return Add()(inputs)


LAYER_CLASSES = {c.__name__: c for c in (
    InputLayer, Conv2D, MaxPooling2D, AveragePooling2D, GlobalAveragePooling2D, GlobalMaxPooling2D, Flatten,
    Reshape, Dense, Activation, ReLU, Softmax, Dropout, ZeroPadding2D, BatchNormalization, Add)}
