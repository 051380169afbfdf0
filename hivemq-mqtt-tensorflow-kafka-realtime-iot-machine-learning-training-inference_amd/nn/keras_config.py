"""Keras 2.2.4-tf ``model_config`` / ``training_config`` JSON builders and parsers.

Shapes follow the configs stored in the reference's ``models/*.h5``
(SURVEY.md 5.4): a functional ``Model`` of ``InputLayer`` + ``Dense`` layers for
the autoencoder, and a ``Sequential`` of ``LSTM`` / ``RepeatVector`` /
``TimeDistributed(Dense)`` for the LSTM predictor (LSTM-.../cardata-v2.py:177-183).
"""
from __future__ import annotations

from typing import List, Optional, Sequence


def _init(name: str) -> dict:
    return {"class_name": name, "config": {"seed": None} if name in ("GlorotUniform", "Orthogonal") else {}}


def dense_config(name: str, units: int, activation: str, activity_l1: Optional[float] = None,
                 use_bias: bool = True) -> dict:
    return {
        "name": name, "trainable": True, "dtype": "float32", "units": int(units), "activation": activation,
        "use_bias": use_bias, "kernel_initializer": _init("GlorotUniform"), "bias_initializer": _init("Zeros"),
        "kernel_regularizer": None, "bias_regularizer": None,
        "activity_regularizer": ({"class_name": "L1L2", "config": {"l1": float(activity_l1), "l2": 0.0}}
                                 if activity_l1 else None),
        "kernel_constraint": None, "bias_constraint": None,
    }


def functional_dense_model(name: str, input_name: str, input_dim: int,
                           layers: Sequence[dict]) -> dict:
    """``Input -> Dense -> ... -> Dense`` as a functional Model config (node / layer
    list nesting exactly as stored in the reference models/*.h5)."""
    out = [{"name": input_name, "class_name": "InputLayer",
            "config": {"batch_input_shape": [None, int(input_dim)], "dtype": "float32", "sparse": False,
                       "name": input_name}, "inbound_nodes": []}]
    prev = input_name
    for cfg in layers:
        out.append({"name": cfg["name"], "class_name": "Dense", "config": cfg,
                    "inbound_nodes": [[prev, 0, 0, {}]]})
        prev = cfg["name"]
    return {"class_name": "Model", "config": {"name": name, "layers": out,
                                              "input_layers": [input_name, 0, 0],
                                              "output_layers": [prev, 0, 0]}}


def lstm_config(name: str, units: int, activation: str = "relu", return_sequences: bool = False,
                batch_input_shape: Optional[list] = None) -> dict:
    cfg = {
        "name": name, "trainable": True, "dtype": "float32", "return_sequences": return_sequences,
        "return_state": False, "go_backwards": False, "stateful": False, "unroll": False, "time_major": False,
        "units": int(units), "activation": activation, "recurrent_activation": "sigmoid", "use_bias": True,
        "kernel_initializer": _init("GlorotUniform"), "recurrent_initializer": _init("Orthogonal"),
        "bias_initializer": _init("Zeros"), "unit_forget_bias": True, "kernel_regularizer": None,
        "recurrent_regularizer": None, "bias_regularizer": None, "activity_regularizer": None,
        "kernel_constraint": None, "recurrent_constraint": None, "bias_constraint": None, "dropout": 0.0,
        "recurrent_dropout": 0.0, "implementation": 2,
    }
    if batch_input_shape is not None:
        cfg["batch_input_shape"] = batch_input_shape
    return cfg


def sequential(name: str, layers: List[dict]) -> dict:
    return {"class_name": "Sequential", "config": {"name": name, "layers": layers}}


def training_config(lr: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999, epsilon: float = 1e-7,
                    loss: str = "mean_squared_error", metrics=("accuracy",)) -> dict:
    return {"optimizer_config": {"class_name": "Adam", "config": {
        "name": "Adam", "learning_rate": lr, "decay": 0.0, "beta_1": beta_1, "beta_2": beta_2, "epsilon": epsilon,
        "amsgrad": False}}, "loss": loss, "metrics": list(metrics), "weighted_metrics": None,
        "sample_weight_mode": None, "loss_weights": None}


def parse_dense_model(model_config: dict):
    """Return (input_name, input_dim, [dense layer configs]) of a Dense-only model."""
    cfg = model_config["config"]
    layers = cfg["layers"]
    input_name, input_dim, dense = None, None, []
    for lyr in layers:
        cn = lyr["class_name"]
        c = lyr["config"]
        if cn == "InputLayer":
            input_name = c["name"]
            input_dim = int(c["batch_input_shape"][-1])
        elif cn == "Dense":
            dense.append(c)
            if input_dim is None and "batch_input_shape" in c:   # Sequential form
                input_dim = int(c["batch_input_shape"][-1])
        else:
            raise ValueError(f"not a dense model: layer class {cn}")
    return input_name, input_dim, dense


def optimizer_hparams(training_cfg: Optional[dict]) -> dict:
    if not training_cfg:
        return {}
    c = training_cfg.get("optimizer_config", {}).get("config", {})
    out = {}
    for k_src, k_dst in (("learning_rate", "lr"), ("lr", "lr"), ("beta_1", "beta_1"), ("beta_2", "beta_2"),
                         ("epsilon", "epsilon")):
        if k_src in c:
            out[k_dst] = float(c[k_src])
    return out
