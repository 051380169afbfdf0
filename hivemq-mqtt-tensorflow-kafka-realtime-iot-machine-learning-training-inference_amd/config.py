"""Single configuration object for every entry point.

The reference hard-codes hyper-parameters as module constants
(``AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:176-183``,
``LSTM-TensorFlow-IO-Kafka/cardata-v2.py:172-174``) and passes librdkafka
options as ``key=value`` strings (``cardata-v3.py:7-15``).  Here one dataclass
carries all of it; defaults reproduce the reference constants.

Precedence (lowest -> highest): dataclass defaults, YAML/JSON file,
``SML_<FIELD>`` environment variables, ``--field=value`` CLI overrides.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

# librdkafka-style options used by every reference script (cardata-v3.py:7-15).
REFERENCE_KAFKA_CONFIG = [
    "broker.version.fallback=0.10.0.0",
    "security.protocol=sasl_plaintext",
    "sasl.username=test",
    "sasl.password=test123",
    "sasl.mechanisms=PLAIN",
]


@dataclass
class Config:
    # --- source / sink -------------------------------------------------------
    servers: str = "synthetic://"          # kafka host:port list | fake:// | synthetic:// | csv:<path>
    topic: str = "SENSOR_DATA_S_AVRO"
    partition: int = 0                      # reference hard-codes partition 0 (cardata-v3.py:46); -1 = all
    offset: int = 0
    assign: str = "auto"                    # DP share of the partitions: split | partitions | keys (kafka/assign.py)
    native_feed: bool = True                # ROCm: the C++ partition-parallel feed (kafka/feed.py)
    feed_workers: int = 4                   # its fetch + decode threads per rank
    result_topic: str = "model-predictions"
    group: str = "cardata-autoencoder"
    kafka_config: List[str] = field(default_factory=lambda: list(REFERENCE_KAFKA_CONFIG))
    eof: bool = True                        # bounded read to partition end (cardata-v3.py:47)
    schema: str = "cardata-v1"              # name of a bundled .avsc or a path

    # --- model ---------------------------------------------------------------
    model: str = "autoencoder"              # autoencoder | lstm | mnist
    input_dim: int = 18
    encoding_dim: int = 14
    hidden_dim: int = 7
    activity_l1: float = 1e-7               # cardata-v3.py:183 (named learning_rate there)
    lstm_units: List[int] = field(default_factory=lambda: [32, 16, 16, 32])
    look_back: int = 1                      # LSTM-.../cardata-v2.py:173

    # --- training ------------------------------------------------------------
    mode: str = "train"
    epochs: int = 20                        # cardata-v3.py:176
    batch_size: int = 100                   # cardata-v3.py:177
    take: Optional[int] = 100               # .take(100) epoch cap (cardata-v3.py:218)
    learning_rate: float = 1e-3             # Keras Adam defaults (models/*.h5 training_config)
    beta_1: float = 0.9
    beta_2: float = 0.999
    epsilon: float = 1e-7
    seed: int = 0
    dtype: str = "bf16"                     # compute dtype of the HIP path
    device: str = "auto"                    # auto | cuda | cpu

    # --- inference -----------------------------------------------------------
    predict_skip: int = 100                 # .skip(100) (cardata-v3.py:274)
    predict_take: int = 100
    threshold: float = 5.0                  # notebook threshold_fixed (Fraud-Detection ipynb:1129)

    # --- artefacts -----------------------------------------------------------
    model_file: str = "model1.h5"
    model_store: str = "local:./model-store"  # local:<dir> | gcs:<bucket>
    log_dir: Optional[str] = None           # tfevents output (TensorBoard-compatible)

    # ------------------------------------------------------------------------
    @classmethod
    def fields(cls) -> Dict[str, dataclasses.Field]:
        return {f.name: f for f in dataclasses.fields(cls)}

    def update(self, values: Dict[str, Any]) -> "Config":
        flds = self.fields()
        for k, v in values.items():
            k = k.replace("-", "_")
            if k not in flds:
                raise KeyError(f"unknown config key {k!r}")
            setattr(self, k, _coerce(getattr(self, k), v, flds[k]))
        return self

    @classmethod
    def load(cls, path: Optional[str] = None, env: bool = True,
             argv: Optional[List[str]] = None) -> "Config":
        cfg = cls()
        if path:
            with open(path) as f:
                text = f.read()
            if path.endswith((".yaml", ".yml")):
                import yaml
                data = yaml.safe_load(text) or {}
            else:
                data = json.loads(text)
            cfg.update(data)
        if env:
            envvals = {}
            for name in cls.fields():
                key = "SML_" + name.upper()
                if key in os.environ:
                    envvals[name] = os.environ[key]
            cfg.update(envvals)
        if argv:
            cfg.update(parse_overrides(argv))
        return cfg

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def parse_overrides(argv: List[str]) -> Dict[str, str]:
    """Parse ``--key=value`` / ``--key value`` tokens into a dict of strings."""
    out: Dict[str, str] = {}
    i = 0
    while i < len(argv):
        tok = argv[i]
        if not tok.startswith("--"):
            raise ValueError(f"expected --key=value, got {tok!r}")
        body = tok[2:]
        if "=" in body:
            k, v = body.split("=", 1)
        elif i + 1 < len(argv) and not argv[i + 1].startswith("--"):
            k, v = body, argv[i + 1]
            i += 1
        else:
            k, v = body, "true"
        out[k.replace("-", "_")] = v
        i += 1
    return out


def _coerce(current: Any, value: Any, fld: dataclasses.Field) -> Any:
    if not isinstance(value, str):
        return value
    typ = fld.type if isinstance(fld.type, str) else getattr(fld.type, "__name__", "")
    if isinstance(current, bool) or "bool" in typ:
        return value.strip().lower() in ("1", "true", "yes", "on")
    if isinstance(current, int) and not isinstance(current, bool):
        return int(value)
    if isinstance(current, float):
        return float(value)
    if isinstance(current, list) or "List" in typ:
        if value.strip().startswith("["):
            return json.loads(value)
        items = [s for s in value.split(",") if s]
        if current and isinstance(current[0], int):
            return [int(s) for s in items]
        return items
    if "Optional[int]" in typ:
        return None if value.lower() in ("none", "null", "") else int(value)
    if value.lower() in ("none", "null") and current is None:
        return None
    return value
