"""Keras-HDF5 model files (save_model_hdf5 / model.save('x.h5')) — see csrc/io/keras_h5.cpp."""
from __future__ import annotations


def save_model(model, path, include_optimizer=True):
    raise NotImplementedError("HDF5 saving: native _h5 module pending")


def save_weights(model, path):
    raise NotImplementedError


def load_weights_into(model, path, with_optimizer=False):
    raise NotImplementedError


def load_model(path, compile=True):
    raise NotImplementedError
