"""Python mirror of the R keras/tensorflow/sparklyr verbs used by the reference.

R is not installed in this image, so the R package under ``R/`` (which calls these
functions through reticulate) is covered by testing this module instead.  Verb names
and argument names follow the reference R code (README.md:28-75, 119-153, 171-247):

    model <- keras_model_sequential() %>%
      layer_conv_2d(filters = 32, kernel_size = 3, activation = 'relu', input_shape = c(28, 28, 1)) %>%
      layer_max_pooling_2d() %>% layer_flatten() %>%
      layer_dense(units = 64, activation = 'relu') %>% layer_dense(units = 10)
    model %>% compile(loss = ..., optimizer = ..., metrics = 'accuracy')
    result <- model %>% fit(x_train, y_train, batch_size = 64L, epochs = 3, steps_per_epoch = 5)
    result$metrics$accuracy

``pipe(x, f1, f2, ...)`` stands in for ``%>%``.
"""
from __future__ import annotations

import base64
import json
import os
from typing import Any, Callable

import numpy as np

from . import keras as _keras
from .launch import collect, sdf_len, spark_apply  # noqa: F401  (sparklyr verbs)


def c(*xs):
    """R ``c()`` for shapes."""
    return tuple(int(x) if float(x).is_integer() else x for x in xs)


def pipe(x, *fns: Callable):
    for f in fns:
        x = f(x)
    return x


# ---- tensorflow package -------------------------------------------------------------
def tf_version():
    from . import tf_version as v

    return v()


def install_tensorflow(*a, **k):
    from . import install_tensorflow as it

    return it()


# ---- data helpers --------------------------------------------------------------------
def dataset_mnist(path: str = "mnist.npz") -> dict:
    """``dataset_mnist()`` -> ``mnist$train$x`` / ``$y``, ``mnist$test$x`` / ``$y``."""
    (xt, yt), (xv, yv) = _keras.datasets.mnist.load_data(path)
    return {"train": {"x": xt, "y": yt}, "test": {"x": xv, "y": yv}}


def array_reshape(x, dim, order: str = "C"):
    """R keras ``array_reshape``: row-major (C order) reshape, unlike R's ``dim<-``."""
    return np.reshape(np.asarray(x), tuple(int(d) for d in dim), order=order)


# ---- model construction ----------------------------------------------------------------
def keras_model_sequential(layers=None, name=None):
    return _keras.Sequential(layers, name=name)


def _add(model, layer):
    if model is None:
        return layer
    model.add(layer)
    return model


def _shape(input_shape):
    return None if input_shape is None else tuple(int(d) for d in input_shape)


def layer_conv_2d(object=None, filters=None, kernel_size=None, strides=(1, 1), padding="valid",
                  activation=None, use_bias=True, input_shape=None, name=None, **kw):
    kwargs = dict(strides=strides, padding=padding, activation=activation, use_bias=use_bias, name=name, **kw)
    if input_shape is not None:
        kwargs["input_shape"] = _shape(input_shape)
    return _add(object, _keras.layers.Conv2D(int(filters), kernel_size, **kwargs))


def layer_max_pooling_2d(object=None, pool_size=(2, 2), strides=None, padding="valid", name=None):
    return _add(object, _keras.layers.MaxPooling2D(pool_size, strides, padding, name=name))


def layer_average_pooling_2d(object=None, pool_size=(2, 2), strides=None, padding="valid", name=None):
    return _add(object, _keras.layers.AveragePooling2D(pool_size, strides, padding, name=name))


def layer_flatten(object=None, name=None, input_shape=None):
    kwargs = {"name": name}
    if input_shape is not None:
        kwargs["input_shape"] = _shape(input_shape)
    return _add(object, _keras.layers.Flatten(**kwargs))


def layer_dense(object=None, units=None, activation=None, use_bias=True, input_shape=None, name=None, **kw):
    kwargs = dict(activation=activation, use_bias=use_bias, name=name, **kw)
    if input_shape is not None:
        kwargs["input_shape"] = _shape(input_shape)
    return _add(object, _keras.layers.Dense(int(units), **kwargs))


def layer_dropout(object=None, rate=0.5, name=None):
    return _add(object, _keras.layers.Dropout(rate, name=name))


def layer_batch_normalization(object=None, name=None, **kw):
    return _add(object, _keras.layers.BatchNormalization(name=name, **kw))


def layer_activation(object=None, activation=None, name=None):
    return _add(object, _keras.layers.Activation(activation, name=name))


# ---- compile / fit / evaluate ---------------------------------------------------------------
def compile(object, optimizer=None, loss=None, metrics=None, **kw):  # noqa: A001  (R verb name)
    object.compile(optimizer=optimizer if optimizer is not None else "rmsprop", loss=loss, metrics=metrics, **kw)
    return object


def fit(object, x=None, y=None, batch_size=None, epochs=10, verbose=1, callbacks=None, steps_per_epoch=None,
        validation_split=0.0, validation_data=None, shuffle=True, initial_epoch=0, **kw):
    """R ``fit`` (note: R keras defaults epochs = 10).  Returns the History; the R
    accessor ``result$metrics$accuracy`` is ``History.metrics['accuracy']``."""
    return object.fit(x, y, batch_size=None if batch_size is None else int(batch_size), epochs=int(epochs),
                      verbose=verbose, callbacks=callbacks, steps_per_epoch=steps_per_epoch,
                      validation_split=validation_split, validation_data=validation_data, shuffle=shuffle,
                      initial_epoch=initial_epoch, **kw)


def evaluate(object, x, y, batch_size=None, verbose=1):
    return object.evaluate(x, y, batch_size=batch_size, verbose=verbose)


def predict(object, x, batch_size=None):
    return object.predict(x, batch_size=batch_size)


# ---- persistence (README.md:234-247) --------------------------------------------------------
def save_model_hdf5(object, filepath, overwrite=True, include_optimizer=True):
    object.save(filepath, overwrite=overwrite, include_optimizer=include_optimizer)
    return filepath


def load_model_hdf5(filepath, compile=True):  # noqa: A002
    return _keras.models.load_model(filepath, compile=compile)


def save_model_weights_hdf5(object, filepath):
    object.save_weights(filepath)


def load_model_weights_hdf5(object, filepath):
    object.load_weights(filepath)
    return object


def base64encode(path: str) -> str:
    """``base64enc::base64encode(file)``."""
    with open(path, "rb") as f:
        return base64.b64encode(f.read()).decode("ascii")


def base64decode(s: str) -> bytes:
    return base64.b64decode(s.encode("ascii"))


def write_bytes(data: bytes, path: str) -> str:
    """``write(base64decode(...), "model.hdf5")``."""
    with open(path, "wb") as f:
        f.write(data)
    return path


def save_from_result(results, path: str = "model.hdf5") -> str:
    """Driver side of README.md:240-247: take the per-partition results of a barrier
    apply (a list of strings / rows, or one string), find the chief's non-empty base64
    payload and write it to ``path``."""
    if isinstance(results, str):
        results = [results]
    for r in results:
        if isinstance(r, dict):
            r = next(iter(r.values()), "")
        if r:
            return write_bytes(base64decode(r), path)
    raise ValueError("no partition returned a model payload")


# ---- TF_CONFIG helpers (README.md:84-113, 180-183) ---------------------------------------------
def tf_config(workers, index) -> str:
    """``jsonlite::toJSON(list(cluster = list(worker = ...), task = list(type = 'worker', index = i)),
    auto_unbox = TRUE)`` — a length-1 worker vector is unboxed to a bare string like jsonlite."""
    w = list(workers)
    return json.dumps({"cluster": {"worker": w[0] if len(w) == 1 else w},
                       "task": {"type": "worker", "index": int(index)}})


def sys_setenv(**kv):
    for k, v in kv.items():
        os.environ[k] = str(v)


def barrier_tf_config(barrier: dict, base_port: int = 8000) -> str:
    """The Spark closure's TF_CONFIG: strip executor ports, assign base_port + seq_along
    (README.md:181: ``paste(gsub(":[0-9]+$", "", barrier$address), 8000 + seq_along(...))``)."""
    import re

    hosts = [re.sub(r":[0-9]+$", "", a) for a in barrier["address"]]
    return tf_config([f"{h}:{base_port + i + 1}" for i, h in enumerate(hosts)], barrier["partition"])
