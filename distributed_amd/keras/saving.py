"""Keras-compatible HDF5 model files (``model.save('x.h5')`` / ``save_model_hdf5``).

Reference: ``save_model_hdf5(model, model_file)`` on every Spark partition, the chief
returning the file base64-encoded (README.md:234-247).  Layout written (tf.keras 2.0
``hdf5_format``; strings as fixed-length byte strings like h5py writes numpy ``S``):

    /                       attrs keras_version, backend, model_config (JSON), training_config (JSON)
    /model_weights          attrs layer_names, backend, keras_version
    /model_weights/<layer>  attrs weight_names; datasets <layer>/<var>:0 (e.g. conv2d/kernel:0)
    /optimizer_weights      attrs weight_names; datasets SGD/iter:0, SGD/<layer>/<var>/momentum:0

``save_weights`` writes the ``model_weights`` content at the file root (Keras h5 weights).
I/O is native (``distributed_amd._h5`` over the libhdf5 C API); no h5py needed.
"""
from __future__ import annotations

import json

import numpy as np

from . import losses as _losses
from . import optimizers as _opts

KERAS_VERSION = "2.2.4-tf"
BACKEND = "tensorflow"


def _h5():
    from ..native import load_h5

    return load_h5()


def _weights_group(model) -> dict:
    layers = model.layers
    groups = {}
    for l in layers:
        ws = l.weights
        groups[l.name] = {
            "attrs": {"weight_names": [w.name for w in ws]},
            "datasets": {w.name: w.numpy() for w in ws},
        }
    return {
        "attrs": {"layer_names": [l.name for l in layers], "backend": BACKEND, "keras_version": KERAS_VERSION},
        "groups": groups,
    }


def _optimizer_weights(model):
    opt = model.optimizer
    if opt is None:
        return None
    names, vals = optimizer_weight_list(model)
    if not names:
        return None
    return {"attrs": {"weight_names": names}, "datasets": dict(zip(names, vals))}


def optimizer_weight_list(model):
    """(names, arrays) of the optimizer state in tf.keras optimizer_v2 naming."""
    opt = model.optimizer
    names = [f"{opt.name}/iter:0"]
    vals = [np.asarray(opt.iterations, dtype=np.int64)]
    tws = model.trainable_weights
    sizes = [int(np.prod(w.shape)) for w in tws]
    for slot in opt.slot_names():
        buf = opt.slots.get(slot)
        if buf is None:
            continue
        flat = buf.detach().float().cpu().numpy()
        off = 0
        for w, n in zip(tws, sizes):
            base = w.name[:-2] if w.name.endswith(":0") else w.name
            names.append(f"{opt.name}/{base}/{slot}:0")
            vals.append(flat[off:off + n].reshape(w.shape).astype(np.float32))
            off += n
    return names, vals


def _training_config(model) -> str:
    metrics = []
    for m in model.compiled_metrics:
        metrics.append(m.name)
    cfg = {
        "loss": _losses.serialize(model.loss),
        "metrics": metrics,
        "weighted_metrics": None,
        "sample_weight_mode": None,
        "loss_weights": None,
        "optimizer_config": _opts.serialize(model.optimizer),
    }
    return json.dumps(cfg)


def save_model(model, path: str, include_optimizer: bool = True) -> None:
    root = {
        "attrs": {"keras_version": KERAS_VERSION, "backend": BACKEND, "model_config": model.to_json()},
        "groups": {"model_weights": _weights_group(model)},
    }
    if include_optimizer and model.optimizer is not None and model.loss is not None:
        root["attrs"]["training_config"] = _training_config(model)
        ow = _optimizer_weights(model)
        if ow is not None:
            root["groups"]["optimizer_weights"] = ow
    _h5().write(path, root)


def save_weights(model, path: str) -> None:
    _h5().write(path, _weights_group(model))


def _flatten_datasets(tree: dict, prefix: str = "") -> dict:
    out = {}
    for k, v in tree.get("datasets", {}).items():
        out[prefix + k] = v
    for g, sub in tree.get("groups", {}).items():
        out.update(_flatten_datasets(sub, prefix + g + "/"))
    return out


def _apply_weights(model, wtree: dict) -> None:
    layer_names = wtree["attrs"]["layer_names"]
    if isinstance(layer_names, str):
        layer_names = [layer_names]
    by_name = {l.name: l for l in model.layers}
    if len(layer_names) == len(model.layers) and set(layer_names) != set(by_name):
        # different auto-names (e.g. dense_3 vs dense): match topologically like Keras
        pairs = list(zip(layer_names, model.layers))
    else:
        pairs = [(n, by_name[n]) for n in layer_names if n in by_name]
    for name, layer in pairs:
        g = wtree["groups"].get(name, {"attrs": {"weight_names": []}})
        wn = g["attrs"].get("weight_names", [])
        if isinstance(wn, str):
            wn = [wn]
        flat = _flatten_datasets(g)
        vals = [flat[n] for n in wn]
        if len(vals) != len(layer.weights):
            raise ValueError(f"layer {layer.name}: file has {len(vals)} weights, model has {len(layer.weights)}")
        layer.set_weights(vals)


def _apply_optimizer(model, otree: dict) -> None:
    opt = model.optimizer
    names = otree["attrs"].get("weight_names", [])
    if isinstance(names, str):
        names = [names]
    flat = _flatten_datasets(otree)
    import torch

    tws = model.trainable_weights
    sizes = [int(np.prod(w.shape)) for w in tws]
    n = int(sum(sizes))
    dev = tws[0].value.device if tws else "cpu"
    for nm in names:
        v = flat.get(nm)
        if v is None:
            continue
        if nm.endswith("/iter:0"):
            opt.iterations = int(np.asarray(v).reshape(-1)[0])
    # slot tensors are matched by position (like Keras' optimizer.set_weights), so a model
    # rebuilt in another session with different auto-names still restores correctly
    slot_vals = [flat[nm] for nm in names if not nm.endswith("/iter:0") and nm in flat]
    nslots = len(opt.slot_names())
    if nslots and len(slot_vals) == nslots * len(tws):
        for si, slot in enumerate(opt.slot_names()):
            parts = [np.asarray(v, dtype=np.float32).reshape(-1) for v in slot_vals[si * len(tws):(si + 1) * len(tws)]]
            if [p.size for p in parts] != sizes:
                raise ValueError(f"optimizer slot '{slot}' shapes do not match the model")
            opt.ensure_slots(n, dev)
            opt.slots[slot].copy_(torch.from_numpy(np.concatenate(parts)).to(opt.slots[slot].device))
    elif slot_vals:
        raise ValueError("optimizer weights in the file do not match this optimizer/model")
    if getattr(model, "_engine", None) is not None:
        model._engine.reload_optimizer_state()


def load_weights_into(model, path: str, with_optimizer: bool = False) -> None:
    tree = _h5().read(path)
    wtree = tree["groups"].get("model_weights", tree)
    _apply_weights(model, wtree)
    if with_optimizer and "optimizer_weights" in tree["groups"] and model.optimizer is not None:
        _apply_optimizer(model, tree["groups"]["optimizer_weights"])


def load_model(path: str, compile: bool = True):  # noqa: A002
    from .models import model_from_config

    tree = _h5().read(path)
    attrs = tree["attrs"]
    model = model_from_config(json.loads(attrs["model_config"]))
    _apply_weights(model, tree["groups"]["model_weights"])
    if compile and "training_config" in attrs:
        tc = json.loads(attrs["training_config"])
        model.compile(optimizer=_opts.get(tc["optimizer_config"]), loss=_losses.get(tc["loss"]),
                      metrics=tc.get("metrics") or None)
        if "optimizer_weights" in tree["groups"]:
            _apply_optimizer(model, tree["groups"]["optimizer_weights"])
    return model
