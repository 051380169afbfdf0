"""Keras-style layers for the generic model builder (:mod:`streamml.nn.model`).

The reference builds every model with ``tf.keras.layers``:
``Input``, ``Dense`` (with ``activity_regularizer=l1``), ``LSTM``,
``RepeatVector``, ``TimeDistributed(Dense)``, ``Flatten`` and ``Dropout``.  These
classes hold only configuration; parameters live in the owning model's single
flat fp32 buffer (one Adam launch, one DP all-reduce per step) and the compute
goes to the HIP ops -- ``ops.dense`` (K1/K2 tall-skinny MFMA kernels),
``ops.lstm`` (fused recurrence), the fused softmax-CE head -- on ROCm devices and
to the torch reference ops on CPU.

Parameter init follows Keras: GlorotUniform kernels, Orthogonal recurrent
kernels, zero biases, LSTM ``unit_forget_bias``.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import keras_config as kc


# ---------------------------------------------------------------------------
# regularizers / initializers
# ---------------------------------------------------------------------------
class L1L2:
    def __init__(self, l1: float = 0.0, l2: float = 0.0):
        self.l1, self.l2 = float(l1), float(l2)

    def get_config(self):
        return {"class_name": "L1L2", "config": {"l1": self.l1, "l2": self.l2}}


class regularizers:  # noqa: N801  (keras namespace spelling)
    L1L2 = L1L2

    @staticmethod
    def l1(l=0.01):  # noqa: E741
        return L1L2(l1=l)

    @staticmethod
    def l2(l=0.01):  # noqa: E741
        return L1L2(l2=l)


def glorot_uniform(fan_in: int, fan_out: int, rng: np.random.Generator, shape=None) -> np.ndarray:
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape or (fan_in, fan_out)).astype(np.float32)


def orthogonal(rows: int, cols: int, rng: np.random.Generator) -> np.ndarray:
    a = rng.standard_normal((max(rows, cols), min(rows, cols)))
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    return (q if rows >= cols else q.T)[:rows, :cols].astype(np.float32)


# ---------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------
class Layer:
    class_name = "Layer"
    prefix = "layer"

    def __init__(self, name: Optional[str] = None, input_shape=None, **_ignored):
        self.name = name
        self.input_shape = tuple(input_shape) if input_shape is not None else None
        self.built = False
        self.param_slots: List[int] = []       # indices into the model's FlatParams
        self.inbound: List["Layer"] = []       # functional graph edges
        self.out_shape: Optional[Tuple] = None

    # functional API: layer(tensor_spec) records the edge
    def __call__(self, inbound: "Layer") -> "Layer":
        self.inbound = [inbound]
        return self

    def weight_specs(self, in_shape) -> List[Tuple[str, tuple]]:
        return []

    def init_weights(self, in_shape, rng) -> List[np.ndarray]:
        return []

    def output_shape(self, in_shape):
        return in_shape

    def forward(self, params: Sequence[torch.Tensor], x: torch.Tensor, training: bool) -> torch.Tensor:
        return x

    def get_config(self) -> dict:
        return {"name": self.name, "trainable": True, "dtype": "float32"}

    def activity_penalty(self) -> float:
        return 0.0


class InputLayer(Layer):
    class_name = "InputLayer"
    prefix = "input"

    def __init__(self, shape=None, name=None, batch_input_shape=None, **kw):
        if shape is None and batch_input_shape is not None:
            shape = tuple(batch_input_shape[1:])
        super().__init__(name=name, input_shape=shape)
        self.shape = tuple(shape)

    def get_config(self):
        return {"batch_input_shape": [None, *self.shape], "dtype": "float32", "sparse": False, "name": self.name}


def Input(shape=None, name=None, **kw) -> InputLayer:  # noqa: N802 (keras spelling)
    return InputLayer(shape=shape, name=name, **kw)


class Dense(Layer):
    class_name = "Dense"
    prefix = "dense"

    def __init__(self, units: int, activation: Optional[str] = None, use_bias: bool = True,
                 activity_regularizer: Optional[L1L2] = None, name=None, input_shape=None, input_dim=None, **kw):
        if input_shape is None and input_dim is not None:
            input_shape = (input_dim,)
        super().__init__(name=name, input_shape=input_shape)
        self.units = int(units)
        self.activation = activation or "linear"
        if callable(self.activation):
            self.activation = getattr(self.activation, "__name__", "linear")
        self.use_bias = use_bias
        self.activity_regularizer = activity_regularizer
        self._penalty = None

    def weight_specs(self, in_shape):
        ws = [("kernel", (int(in_shape[-1]), self.units))]
        if self.use_bias:
            ws.append(("bias", (self.units,)))
        return ws

    def init_weights(self, in_shape, rng):
        out = [glorot_uniform(int(in_shape[-1]), self.units, rng)]
        if self.use_bias:
            out.append(np.zeros(self.units, np.float32))
        return out

    def output_shape(self, in_shape):
        return (*in_shape[:-1], self.units)

    def forward(self, params, x, training, logits_only: bool = False):
        from ..ops.dense import dense as dense_op
        W = params[0]
        b = params[1] if self.use_bias else None
        act = self.activation
        if act == "softmax":
            z = dense_op(x, W, b, "linear")
            return z if logits_only else torch.softmax(z, dim=-1)
        if act not in ("linear", "relu", "tanh", "sigmoid"):
            raise ValueError(f"unsupported activation {act!r}")
        y = dense_op(x, W, b, act)
        if self.activity_regularizer is not None and training:
            r = self.activity_regularizer
            pen = 0.0
            if r.l1:
                pen = pen + r.l1 * y.abs().sum()
            if r.l2:
                pen = pen + r.l2 * (y * y).sum()
            self._penalty = pen / max(y.shape[0], 1)      # Keras divides by the batch size
        return y

    def get_config(self):
        l1 = self.activity_regularizer.l1 if self.activity_regularizer is not None else None
        cfg = kc.dense_config(self.name, self.units, self.activation, l1, self.use_bias)
        if self.activity_regularizer is not None and self.activity_regularizer.l2:
            cfg["activity_regularizer"] = self.activity_regularizer.get_config()
        if self.input_shape is not None:
            cfg["batch_input_shape"] = [None, *self.input_shape]
        return cfg


class LSTM(Layer):
    class_name = "LSTM"
    prefix = "lstm"

    def __init__(self, units: int, activation: str = "tanh", return_sequences: bool = False,
                 recurrent_activation: str = "sigmoid", unit_forget_bias: bool = True, name=None, input_shape=None,
                 **kw):
        super().__init__(name=name, input_shape=input_shape)
        if recurrent_activation != "sigmoid":
            raise ValueError("LSTM recurrent_activation must be sigmoid")
        if activation not in ("relu", "tanh"):
            raise ValueError("LSTM activation must be relu or tanh")
        self.units = int(units)
        self.activation = activation
        self.return_sequences = bool(return_sequences)
        self.unit_forget_bias = unit_forget_bias

    def weight_specs(self, in_shape):
        u = self.units
        return [("kernel", (int(in_shape[-1]), 4 * u)), ("recurrent_kernel", (u, 4 * u)), ("bias", (4 * u,))]

    def init_weights(self, in_shape, rng):
        u = self.units
        fi = int(in_shape[-1])
        W = glorot_uniform(fi, 4 * u, rng)
        U = np.concatenate([orthogonal(u, u, rng) for _ in range(4)], axis=1)
        b = np.zeros(4 * u, np.float32)
        if self.unit_forget_bias:
            b[u:2 * u] = 1.0
        return [W, U, b]

    def output_shape(self, in_shape):
        return (in_shape[0], self.units) if self.return_sequences else (self.units,)

    def forward(self, params, x, training):
        from ..ops.lstm import lstm as lstm_op
        W, U, b = params
        return lstm_op(x, W, U, b, self.activation, return_sequences=self.return_sequences)

    def get_config(self):
        return kc.lstm_config(self.name, self.units, self.activation, self.return_sequences,
                              [None, *self.input_shape] if self.input_shape is not None else None)


class RepeatVector(Layer):
    class_name = "RepeatVector"
    prefix = "repeat_vector"

    def __init__(self, n: int, name=None, **kw):
        super().__init__(name=name)
        self.n = int(n)

    def output_shape(self, in_shape):
        return (self.n, *in_shape)

    def forward(self, params, x, training):
        return x.unsqueeze(1).expand(x.shape[0], self.n, *x.shape[1:]).contiguous()

    def get_config(self):
        return {**super().get_config(), "n": self.n}


class TimeDistributed(Layer):
    class_name = "TimeDistributed"
    prefix = "time_distributed"

    def __init__(self, layer: Layer, name=None, **kw):
        super().__init__(name=name)
        self.layer = layer

    def weight_specs(self, in_shape):
        return self.layer.weight_specs(in_shape[1:])

    def init_weights(self, in_shape, rng):
        return self.layer.init_weights(in_shape[1:], rng)

    def output_shape(self, in_shape):
        return (in_shape[0], *self.layer.output_shape(in_shape[1:]))

    def forward(self, params, x, training):
        # Dense over the last axis already treats leading axes as rows: one launch over B*T rows
        return self.layer.forward(params, x, training)

    def get_config(self):
        inner = self.layer.get_config()
        return {**super().get_config(), "layer": {"class_name": self.layer.class_name, "config": inner}}


class Flatten(Layer):
    class_name = "Flatten"
    prefix = "flatten"

    def output_shape(self, in_shape):
        return (int(np.prod(in_shape)),)

    def forward(self, params, x, training):
        return x.reshape(x.shape[0], -1)

    def get_config(self):
        cfg = {**super().get_config(), "data_format": "channels_last"}
        if self.input_shape is not None:
            cfg["batch_input_shape"] = [None, *self.input_shape]
        return cfg


class Dropout(Layer):
    class_name = "Dropout"
    prefix = "dropout"

    def __init__(self, rate: float, name=None, seed: Optional[int] = None, **kw):
        super().__init__(name=name)
        self.rate = float(rate)
        self.seed = seed
        self._gen = None

    def forward(self, params, x, training):
        if not training or self.rate <= 0:
            return x
        if self._gen is None or self._gen.device != x.device:
            self._gen = torch.Generator(device=x.device)
            self._gen.manual_seed(self.seed if self.seed is not None else 0)
        keep = 1.0 - self.rate
        mask = (torch.rand(x.shape, device=x.device, generator=self._gen) < keep).to(x.dtype)
        return x * mask * (1.0 / keep)

    def get_config(self):
        return {**super().get_config(), "rate": self.rate, "noise_shape": None, "seed": self.seed}


LAYER_CLASSES = {c.class_name: c for c in (InputLayer, Dense, LSTM, RepeatVector, TimeDistributed, Flatten, Dropout)}


def layer_from_config(class_name: str, cfg: dict) -> Layer:
    """Rebuild a layer from its Keras config (``load_model``)."""
    if class_name not in LAYER_CLASSES:
        raise ValueError(f"unsupported layer class {class_name}")
    c = dict(cfg)
    name = c.get("name")
    bis = c.get("batch_input_shape")
    if class_name == "InputLayer":
        return InputLayer(batch_input_shape=bis, name=name)
    if class_name == "Dense":
        ar = c.get("activity_regularizer")
        reg = None
        if ar:
            rc = ar.get("config", {})
            reg = L1L2(rc.get("l1", 0.0), rc.get("l2", 0.0))
        return Dense(c["units"], c.get("activation", "linear"), c.get("use_bias", True), reg, name=name,
                     input_shape=tuple(bis[1:]) if bis else None)
    if class_name == "LSTM":
        return LSTM(c["units"], c.get("activation", "tanh"), c.get("return_sequences", False),
                    c.get("recurrent_activation", "sigmoid"), c.get("unit_forget_bias", True), name=name,
                    input_shape=tuple(bis[1:]) if bis else None)
    if class_name == "RepeatVector":
        return RepeatVector(c["n"], name=name)
    if class_name == "TimeDistributed":
        inner = c["layer"]
        return TimeDistributed(layer_from_config(inner["class_name"], inner["config"]), name=name)
    if class_name == "Flatten":
        return Flatten(name=name, input_shape=tuple(bis[1:]) if bis else None)
    return Dropout(c.get("rate", 0.0), name=name, seed=c.get("seed"))
