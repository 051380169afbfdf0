"""Observability: Prometheus metrics, TensorBoard event files, rocprofv3 helpers."""
from .metrics import REGISTRY, Counter, Gauge, Registry, Summary  # noqa: F401
from .tfevents import EventFileWriter, read_scalars  # noqa: F401
