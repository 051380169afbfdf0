"""Car-sensor schema facts, the reference normalisation, and a synthetic source.

* Column order follows the KSQL Avro record ``KsqlDataSourceSchema``
  (``AUTOENCODER-TensorFlow-IO-Kafka/cardata-v1.avsc``) which is also the argument
  order of ``normalize_fn`` (``cardata-v3.py:78-97``).
* ``normalize_fn`` (``cardata-v3.py:99-168``) is an affine map per column:
  ``scale_fn(v, lo, hi) = (v - lo) / (hi - lo) * 2 - 1``; four columns are
  replaced by the constant 0.0 (reference TODOs, ``:109, :115, :121, :124``).
  We express it as ``x * SCALE + SHIFT`` so the GPU kernels can fuse it into
  their first load; the zeroed columns have SCALE = SHIFT = 0 (quirk preserved).
* The synthetic generator reproduces the value ranges observed in
  ``testdata/car-sensor-data.csv`` and the device/rate parameters of the HiveMQ
  device-simulator scenarios (``infrastructure/test-generator/scenario.xml:13,48``:
  100 000 cars x 1 msg / 10 s; ``scenario_evaluation.xml``: 25 cars x 1 / 5 s).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

# canonical (snake_case) feature names, 18 sensors + label
FEATURES: List[str] = [
    "coolant_temp",
    "intake_air_temp",
    "intake_air_flow_speed",
    "battery_percentage",
    "battery_voltage",
    "current_draw",
    "speed",
    "engine_vibration_amplitude",
    "throttle_pos",
    "tire_pressure_11",
    "tire_pressure_12",
    "tire_pressure_21",
    "tire_pressure_22",
    "accelerometer_11_value",
    "accelerometer_12_value",
    "accelerometer_21_value",
    "accelerometer_22_value",
    "control_unit_firmware",
]
LABEL = "failure_occurred"
NUM_FEATURES = len(FEATURES)
INT_FEATURES = {"tire_pressure_11", "tire_pressure_12", "tire_pressure_21", "tire_pressure_22",
                "control_unit_firmware"}

# normalize_fn ranges (cardata-v3.py:105-148); None = replaced by 0.0
NORMALIZE_RANGES: Dict[str, Optional[Tuple[float, float]]] = {
    "coolant_temp": None,
    "intake_air_temp": (15.0, 40.0),
    "intake_air_flow_speed": None,
    "battery_percentage": (0.0, 100.0),
    "battery_voltage": None,
    "current_draw": None,
    "speed": (0.0, 50.0),
    "engine_vibration_amplitude": (0.0, 7500.0),
    "throttle_pos": (0.0, 1.0),
    "tire_pressure_11": (20.0, 35.0),
    "tire_pressure_12": (20.0, 35.0),
    "tire_pressure_21": (20.0, 35.0),
    "tire_pressure_22": (20.0, 35.0),
    "accelerometer_11_value": (0.0, 7.0),
    "accelerometer_12_value": (0.0, 7.0),
    "accelerometer_21_value": (0.0, 7.0),
    "accelerometer_22_value": (0.0, 7.0),
    "control_unit_firmware": (1000.0, 2000.0),
}


def normalize_affine() -> Tuple[np.ndarray, np.ndarray]:
    """(scale, shift) float64 arrays so that ``normalize_fn(x) = x * scale + shift``."""
    scale = np.zeros(NUM_FEATURES, dtype=np.float64)
    shift = np.zeros(NUM_FEATURES, dtype=np.float64)
    for i, name in enumerate(FEATURES):
        rng = NORMALIZE_RANGES[name]
        if rng is None:
            continue
        lo, hi = rng
        scale[i] = 2.0 / (hi - lo)
        shift[i] = -2.0 * lo / (hi - lo) - 1.0
    return scale, shift


def normalize_np(raw: np.ndarray) -> np.ndarray:
    """Reference ``normalize_fn`` applied row-wise (numpy oracle)."""
    out = np.zeros(raw.shape, dtype=np.float64)
    for i, name in enumerate(FEATURES):
        rng = NORMALIZE_RANGES[name]
        if rng is None:
            continue
        lo, hi = rng
        out[:, i] = (raw[:, i].astype(np.float64) - lo) / (hi - lo) * 2.0 - 1.0
    return out


# alias map: KSQL UPPERCASE, CSV (tire_pressure_1_1) and camelCase JSON keys
def _aliases() -> Dict[str, str]:
    al: Dict[str, str] = {}
    for name in FEATURES + [LABEL]:
        al[name] = name
        al[name.upper()] = name
    extra = {
        "tire_pressure_1_1": "tire_pressure_11", "tire_pressure_1_2": "tire_pressure_12",
        "tire_pressure_2_1": "tire_pressure_21", "tire_pressure_2_2": "tire_pressure_22",
        "accelerometer_1_1_value": "accelerometer_11_value", "accelerometer_1_2_value": "accelerometer_12_value",
        "accelerometer_2_1_value": "accelerometer_21_value", "accelerometer_2_2_value": "accelerometer_22_value",
        "TIRE_PRESSURE11": "tire_pressure_11", "TIRE_PRESSURE12": "tire_pressure_12",
        "TIRE_PRESSURE21": "tire_pressure_21", "TIRE_PRESSURE22": "tire_pressure_22",
        "ACCELEROMETER11_VALUE": "accelerometer_11_value", "ACCELEROMETER12_VALUE": "accelerometer_12_value",
        "ACCELEROMETER21_VALUE": "accelerometer_21_value", "ACCELEROMETER22_VALUE": "accelerometer_22_value",
        "coolantTemp": "coolant_temp", "intakeAirTemp": "intake_air_temp",
        "intakeAirFlowSpeed": "intake_air_flow_speed", "batteryPercentage": "battery_percentage",
        "batteryVoltage": "battery_voltage", "currentDraw": "current_draw", "speed": "speed",
        "engineVibrationAmplitude": "engine_vibration_amplitude", "throttlePos": "throttle_pos",
        "tirePressure11": "tire_pressure_11", "tirePressure12": "tire_pressure_12",
        "tirePressure21": "tire_pressure_21", "tirePressure22": "tire_pressure_22",
        "accelerometer11Value": "accelerometer_11_value", "accelerometer12Value": "accelerometer_12_value",
        "accelerometer21Value": "accelerometer_21_value", "accelerometer22Value": "accelerometer_22_value",
        "controlUnitFirmware": "control_unit_firmware", "failureOccurred": "failure_occurred",
    }
    al.update(extra)
    # lower-case KSQL DDL column names (CREATE STREAM SENSOR_DATA_S (... tire_pressure11 INT,
    # accelerometer11_value DOUBLE ...), 01_installConfluentPlatform.sh:235)
    for k, v in extra.items():
        if k.isupper():
            al[k.lower()] = v
    return al


ALIASES = _aliases()


def canonical(name: str) -> Optional[str]:
    return ALIASES.get(name)


# ---------------------------------------------------------------------------
# synthetic source
# ---------------------------------------------------------------------------
# (low, high) generation ranges matched to testdata/car-sensor-data.csv stats
#  and to the normalisation ranges.
SYNTH_RANGES: Dict[str, Tuple[float, float]] = {
    "coolant_temp": (18.5, 1977.0),
    "intake_air_temp": (15.0, 40.0),
    "intake_air_flow_speed": (0.0, 200.0),
    "battery_percentage": (0.0, 100.0),
    "battery_voltage": (205.0, 260.0),
    "current_draw": (0.03, 57.9),
    "speed": (0.0, 50.0),
    "engine_vibration_amplitude": (0.0, 7500.0),   # ~ speed * 100..150 in the simulator
    "throttle_pos": (0.0, 1.0),
    "tire_pressure_11": (20.0, 35.0),
    "tire_pressure_12": (20.0, 35.0),
    "tire_pressure_21": (20.0, 35.0),
    "tire_pressure_22": (20.0, 35.0),
    "accelerometer_11_value": (0.0, 7.0),
    "accelerometer_12_value": (0.0, 7.0),
    "accelerometer_21_value": (0.0, 7.0),
    "accelerometer_22_value": (0.0, 7.0),
    "control_unit_firmware": (1000.0, 2000.0),
}

SCENARIOS = {
    # scenario.xml: 100 000 clients, publish every 10 s, QoS 0, 3 000 msgs each
    "full": dict(n_devices=100_000, interval_s=10.0, msgs_per_device=3000, qos=0),
    # scenario_evaluation.xml: 25 clients, every 5 s, QoS 1, 40 msgs each
    "evaluation": dict(n_devices=25, interval_s=5.0, msgs_per_device=40, qos=1),
}


@dataclass
class SyntheticCarSource:
    """Deterministic synthetic car-sensor event generator.

    Each device ("electric-vehicle-NNNNN", the MQTT topic suffix of
    ``scenario.xml:22-27``) has a smooth per-device operating point plus noise;
    a ``failure_rate`` fraction of events is drawn off-distribution and labelled
    ``failure_occurred="true"`` so the anomaly path has something to find.
    """

    n_devices: int = 100_000
    interval_s: float = 10.0
    failure_rate: float = 0.01
    seed: int = 0
    start_time: int = 1567606196   # first timestamp of testdata/car-sensor-data.csv

    @classmethod
    def scenario(cls, name: str, **kw) -> "SyntheticCarSource":
        sc = dict(SCENARIOS[name])
        return cls(n_devices=sc["n_devices"], interval_s=sc["interval_s"], **kw)

    @property
    def rate_msgs_per_s(self) -> float:
        return self.n_devices / self.interval_s

    def generate(self, n: int, start: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """Return (raw[n,18] float32, failure[n] bool, device_id[n] int64, timestamp[n] int64).

        Event ``k`` (global index ``start + k``) comes from device
        ``k % n_devices`` at time ``start_time + (k // n_devices) * interval_s``.
        """
        idx = np.arange(start, start + n, dtype=np.int64)
        dev = idx % self.n_devices
        tick = idx // self.n_devices
        rng = np.random.default_rng(self.seed * 1_000_003 + start)
        # per-device operating point (stable across ticks)
        drng = np.random.default_rng(self.seed + 17)
        dev_bias = drng.random((min(self.n_devices, 1 << 20), NUM_FEATURES))
        base = dev_bias[dev % dev_bias.shape[0]]
        noise = rng.standard_normal((n, NUM_FEATURES)) * 0.05
        u = np.clip(base * 0.7 + 0.15 + noise, 0.0, 1.0)
        fail = rng.random(n) < self.failure_rate
        if fail.any():
            u[fail] = np.clip(u[fail] + rng.choice([-1.0, 1.0], size=(int(fail.sum()), NUM_FEATURES)) * 0.6, 0, 1)
        raw = np.empty((n, NUM_FEATURES), dtype=np.float32)
        for i, name in enumerate(FEATURES):
            lo, hi = SYNTH_RANGES[name]
            col = lo + u[:, i] * (hi - lo)
            if name == "control_unit_firmware":
                col = np.where(u[:, i] > 0.5, 2000.0, 1000.0)
            elif name in INT_FEATURES:
                col = np.rint(col)
            raw[:, i] = col
        # vibration tracks speed (simulator: speed * 100..150)
        raw[:, 7] = np.where(fail, raw[:, 7], raw[:, 6] * (100.0 + 50.0 * u[:, 7]))
        ts = self.start_time + (tick * self.interval_s).astype(np.int64)
        return raw, fail, dev, ts


def synthetic_device_tensor(n: int, device, seed: int = 0, dtype=None, n_devices: int = 100_000,
                            shard: int = 0, n_shards: int = 1):
    """Generate ``n`` raw car-sensor rows directly on ``device`` (torch).

    Row ``i`` is an event of car ``(i * n_shards + shard) % n_devices`` so that
    ``n_shards`` ranks own disjoint car-key sets (shard-by-key, the KSQL
    ``PARTITION BY CAR`` of 01_installConfluentPlatform.sh:249).  Each car has a
    stable operating point plus per-event noise.  Used by the benchmark to build
    per-GPU datasets larger than the Infinity Cache without a host round trip;
    value ranges follow :data:`SYNTH_RANGES`.
    """
    import torch

    dtype = dtype or torch.float32
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    car_point = torch.rand((n_devices, NUM_FEATURES), generator=g, device=device)
    g.manual_seed(seed * 7919 + shard + 1)
    cars = (torch.arange(n, device=device, dtype=torch.int64) * n_shards + shard) % n_devices
    noise = torch.randn((n, NUM_FEATURES), generator=g, device=device) * 0.05
    u = (car_point[cars] * 0.7 + 0.15 + noise).clamp_(0.0, 1.0)
    del noise, cars
    lo = torch.tensor([SYNTH_RANGES[f][0] for f in FEATURES], device=device)
    hi = torch.tensor([SYNTH_RANGES[f][1] for f in FEATURES], device=device)
    raw = lo + u * (hi - lo)
    for i, name in enumerate(FEATURES):
        if name == "control_unit_firmware":
            raw[:, i] = torch.where(u[:, i] > 0.5, 2000.0, 1000.0)
        elif name in INT_FEATURES:
            raw[:, i] = torch.round(raw[:, i])
    raw[:, 7] = raw[:, 6] * (100.0 + 50.0 * u[:, 7])
    return raw.to(dtype)


def load_csv(path: str) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Read ``testdata/car-sensor-data.csv`` -> (raw[n,18] float32, time[n], car[n] str).

    The CSV has no ``failure_occurred`` column, so
    callers treat every row as normal.
    """
    import csv

    with open(path, newline="") as f:
        rd = csv.reader(f)
        header = next(rd)
        cols = [canonical(h) for h in header]
        idx = [cols.index(name) for name in FEATURES]
        t_idx = header.index("time") if "time" in header else None
        c_idx = header.index("car") if "car" in header else None
        rows, times, cars = [], [], []
        for rec in rd:
            if not rec:
                continue
            rows.append([float(rec[i]) for i in idx])
            times.append(int(rec[t_idx]) if t_idx is not None else 0)
            cars.append(rec[c_idx] if c_idx is not None else "")
    return np.asarray(rows, dtype=np.float32), np.asarray(times, dtype=np.int64), np.asarray(cars)
