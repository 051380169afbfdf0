"""Keras-compatible ``.h5`` checkpoints on top of the native HDF5 codec (``streamml._io``).

Reference behaviour: ``model.save(path)`` / ``tf.keras.models.load_model(path)``
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:227,261; LSTM-.../cardata-v2.py:214,245)
write/read Keras 2.2.4-tf HDF5 files whose layout is pinned in SURVEY.md 5.4:

    /                  @keras_version @backend @model_config(JSON) @training_config(JSON)
    /model_weights     @layer_names @backend @keras_version
    /model_weights/<layer>            @weight_names  (e.g. 'dense/kernel:0')
    /model_weights/<layer>/<weight path>   float32 datasets ([in, out] kernels)
    /optimizer_weights @weight_names ('training/Adam/iter:0', .../m:0 ..., .../v:0 ...)

Weights are always resolved through the ``weight_names`` attributes, never by
layer name (the 100-epoch reference file stores layer ``dense_4``'s weights under
``dense_4_1/`` -- SURVEY.md 5.4 quirk).
"""
from __future__ import annotations

import json
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..ops._ext import load_io

KERAS_VERSION = "2.2.4-tf"
BACKEND = "tensorflow"


# ---------------------------------------------------------------------------
# generic tree <-> native dict conversion
# ---------------------------------------------------------------------------
def _value_from_native(v: dict) -> Any:
    kind = v["kind"]
    shape = tuple(v["shape"])
    if kind == "numeric":
        arr = np.frombuffer(v["data"], dtype=np.dtype(v["dtype"])).copy()
        return arr.reshape(shape) if shape else arr.reshape(())
    if kind == "fixed_str":
        arr = np.frombuffer(v["data"], dtype=f"S{v['size']}").copy()
        return arr.reshape(shape) if shape else arr.reshape(())
    vals = [b.decode("utf-8", errors="replace") for b in v["values"]]
    if not shape:
        return vals[0]
    return np.array(vals, dtype=object).reshape(shape)


def _value_to_native(x: Any) -> dict:
    if isinstance(x, bytes):
        x = x.decode("utf-8")
    if isinstance(x, str):
        return {"kind": "vlen_str", "shape": [], "values": [x.encode("utf-8")], "cset": 0}
    arr = np.asarray(x)
    if arr.dtype.kind == "S":
        size = max(1, arr.dtype.itemsize)
        return {"kind": "fixed_str", "shape": list(arr.shape), "size": size, "pad": 1, "cset": 0,
                "data": arr.copy(order="C").tobytes()}
    if arr.dtype.kind == "O" or arr.dtype.kind == "U":
        vals = [str(s).encode("utf-8") for s in arr.ravel()]
        return {"kind": "vlen_str", "shape": list(arr.shape), "values": vals, "cset": 0}
    if arr.dtype.kind not in "fiub":
        raise TypeError(f"unsupported dtype {arr.dtype}")
    if arr.dtype.kind == "b":
        arr = arr.astype(np.uint8)
    arr = arr.astype(arr.dtype.newbyteorder("<")).copy(order="C")  # keeps 0-d shape
    return {"kind": "numeric", "shape": list(arr.shape), "dtype": "<" + arr.dtype.kind + str(arr.dtype.itemsize),
            "data": arr.tobytes()}


@dataclass
class Group:
    attrs: Dict[str, Any] = field(default_factory=OrderedDict)
    children: Dict[str, Any] = field(default_factory=OrderedDict)   # name -> Group | Dataset

    def require_group(self, path: str) -> "Group":
        g = self
        for part in [p for p in path.split("/") if p]:
            nxt = g.children.get(part)
            if nxt is None:
                nxt = Group()
                g.children[part] = nxt
            if not isinstance(nxt, Group):
                raise ValueError(f"{part} is a dataset, not a group")
            g = nxt
        return g

    def __getitem__(self, path: str):
        node: Any = self
        for part in [p for p in path.split("/") if p]:
            node = node.children[part]
        return node

    def __contains__(self, path: str) -> bool:
        try:
            self[path]
            return True
        except (KeyError, AttributeError):
            return False

    def create_dataset(self, path: str, data) -> "Dataset":
        parts = [p for p in path.split("/") if p]
        g = self.require_group("/".join(parts[:-1]))
        ds = Dataset(np.asarray(data))
        g.children[parts[-1]] = ds
        return ds


@dataclass
class Dataset:
    value: np.ndarray
    attrs: Dict[str, Any] = field(default_factory=OrderedDict)


def _from_native(n: dict):
    attrs = OrderedDict((k, _value_from_native(v)) for k, v in n["attrs"].items())
    if n["type"] == "group":
        return Group(attrs, OrderedDict((k, _from_native(c)) for k, c in n["children"].items()))
    return Dataset(_value_from_native(n["value"]), attrs)


def _to_native(node) -> dict:
    attrs = {k: _value_to_native(v) for k, v in node.attrs.items()}
    if isinstance(node, Group):
        return {"type": "group", "attrs": attrs, "children": {k: _to_native(c) for k, c in node.children.items()}}
    return {"type": "dataset", "attrs": attrs, "value": _value_to_native(node.value)}


def read(path: str) -> Group:
    """Read an HDF5 file (superblock v0/v1 subset) into a :class:`Group` tree."""
    return _from_native(load_io().h5_read(path))


def write(path: str, root: Group) -> None:
    load_io().h5_write(path, _to_native(root))


def _fixed_strings(names: Sequence[str]) -> np.ndarray:
    enc = [n.encode("utf-8") for n in names]
    width = max([len(e) for e in enc] + [1])
    return np.array(enc, dtype=f"S{width}")


def _decode_names(arr) -> List[str]:
    if isinstance(arr, np.ndarray) and arr.dtype.kind == "S":
        return [b.decode("utf-8") for b in arr.ravel()]
    if isinstance(arr, np.ndarray) and arr.dtype.kind == "O":
        return [str(s) for s in arr.ravel()]
    if isinstance(arr, np.ndarray) and arr.size == 0:
        return []
    if isinstance(arr, (list, tuple)):
        return [a.decode() if isinstance(a, bytes) else str(a) for a in arr]
    return []


# ---------------------------------------------------------------------------
# Keras model files
# ---------------------------------------------------------------------------
@dataclass
class KerasCheckpoint:
    model_config: Optional[dict]
    training_config: Optional[dict]
    layer_names: List[str]
    weights: "OrderedDict[str, List[Tuple[str, np.ndarray]]]"    # layer -> [(weight name, array)]
    optimizer_weights: List[Tuple[str, np.ndarray]]
    keras_version: str = KERAS_VERSION

    def flat_weights(self) -> List[np.ndarray]:
        return [a for ws in self.weights.values() for _, a in ws]

    @property
    def optimizer_iterations(self) -> Optional[int]:
        for name, a in self.optimizer_weights:
            if name.endswith("iter:0") or name.endswith("iterations:0"):
                return int(np.asarray(a).reshape(-1)[0])
        return None


def save_keras_h5(path: str, model_config: dict, layers: Sequence[Tuple[str, Sequence[Tuple[str, np.ndarray]]]],
                  training_config: Optional[dict] = None,
                  optimizer_weights: Optional[Sequence[Tuple[str, np.ndarray]]] = None) -> None:
    """Write a Keras 2.2.4-tf style model file.

    ``layers``: ``[(layer_name, [(weight_name e.g. 'dense/kernel:0', array), ...]), ...]``
    in model order (input layers with no weights included).
    """
    root = Group()
    root.attrs["keras_version"] = KERAS_VERSION
    root.attrs["backend"] = BACKEND
    root.attrs["model_config"] = json.dumps(model_config)
    if training_config is not None:
        root.attrs["training_config"] = json.dumps(training_config)
    mw = root.require_group("model_weights")
    mw.attrs["layer_names"] = _fixed_strings([n for n, _ in layers])
    mw.attrs["backend"] = BACKEND
    mw.attrs["keras_version"] = KERAS_VERSION
    for lname, ws in layers:
        g = mw.require_group(lname)
        if ws:
            g.attrs["weight_names"] = _fixed_strings([w for w, _ in ws])
        else:
            g.attrs["weight_names"] = np.zeros((0,), dtype=np.float64)   # h5py's empty list encoding
        for wname, arr in ws:
            g.create_dataset(wname, np.asarray(arr))
    if optimizer_weights:
        ow = root.require_group("optimizer_weights")
        ow.attrs["weight_names"] = _fixed_strings([n for n, _ in optimizer_weights])
        for name, arr in optimizer_weights:
            ow.create_dataset(name, np.asarray(arr))
    write(path, root)


def load_keras_h5(path: str) -> KerasCheckpoint:
    root = read(path)
    mc = root.attrs.get("model_config")
    tc = root.attrs.get("training_config")
    mw = root["model_weights"] if "model_weights" in root else root
    layer_names = _decode_names(mw.attrs.get("layer_names", np.zeros(0)))
    weights: "OrderedDict[str, List[Tuple[str, np.ndarray]]]" = OrderedDict()
    for ln in layer_names:
        g = mw[ln]
        names = _decode_names(g.attrs.get("weight_names", np.zeros(0)))
        weights[ln] = [(wn, np.asarray(g[wn].value)) for wn in names]
    opt: List[Tuple[str, np.ndarray]] = []
    if "optimizer_weights" in root:
        ow = root["optimizer_weights"]
        for name in _decode_names(ow.attrs.get("weight_names", np.zeros(0))):
            opt.append((name, np.asarray(ow[name].value)))
    return KerasCheckpoint(
        model_config=json.loads(mc) if isinstance(mc, str) else None,
        training_config=json.loads(tc) if isinstance(tc, str) else None,
        layer_names=layer_names, weights=weights, optimizer_weights=opt,
        keras_version=root.attrs.get("keras_version", KERAS_VERSION) if isinstance(root.attrs.get("keras_version"), str)
        else KERAS_VERSION)


def adam_weight_names(layer_weight_names: Sequence[str], prefix: str = "training/Adam") -> List[str]:
    """TF-2.0 Keras optimizer weight names: iter, then every m, then every v."""
    stems = [w.rsplit(":", 1)[0] for w in layer_weight_names]
    return ([f"{prefix}/iter:0"] + [f"{prefix}/{s}/m:0" for s in stems] + [f"{prefix}/{s}/v:0" for s in stems])
