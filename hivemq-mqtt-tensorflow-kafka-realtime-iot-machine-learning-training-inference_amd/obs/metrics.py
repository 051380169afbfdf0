"""Prometheus text-exposition metrics for the streaming engine.

The reference's observability is platform-level Prometheus + Grafana (HiveMQ /
device-simulator dashboards, hivemq/hivemq.json, test-generator/devsim.json;
ServiceMonitor at 5 s, kube-cli.sh:272-288).  The ML engine exports analogous
counters: ingest_records_total, ingest_bytes_total,
h2d_bytes_total, train_rows_total, train_step_latency_us{quantile},
allreduce_us, infer_event_latency_us{quantile}, anomaly_events_total,
ring_buffer_occupancy ...  ``serve(port)`` exposes them at /metrics.
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, HTTPServer
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


class _Metric:
    kind = "untyped"

    def __init__(self, name: str, help: str = "", labels: Sequence[str] = ()):
        self.name, self.help, self.labelnames = name, help, tuple(labels)
        self._lock = threading.Lock()

    def _key(self, labels: Dict[str, str]) -> Tuple[str, ...]:
        return tuple(str(labels.get(n, "")) for n in self.labelnames)

    def _fmt_labels(self, key: Tuple[str, ...], extra: Optional[Dict[str, str]] = None) -> str:
        items = list(zip(self.labelnames, key)) + list((extra or {}).items())
        if not items:
            return ""
        return "{" + ",".join(f'{k}="{v}"' for k, v in items) + "}"


class Counter(_Metric):
    kind = "counter"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._v: Dict[Tuple[str, ...], float] = {}

    def inc(self, amount: float = 1.0, **labels) -> None:
        if amount < 0:
            raise ValueError("counters only increase")
        k = self._key(labels)
        with self._lock:
            self._v[k] = self._v.get(k, 0.0) + amount

    def value(self, **labels) -> float:
        return self._v.get(self._key(labels), 0.0)

    def expose(self) -> List[str]:
        return [f"{self.name}{self._fmt_labels(k)} {v:.17g}" for k, v in sorted(self._v.items())]


class Gauge(Counter):
    kind = "gauge"

    def set(self, value: float, **labels) -> None:
        with self._lock:
            self._v[self._key(labels)] = float(value)

    def inc(self, amount: float = 1.0, **labels) -> None:
        k = self._key(labels)
        with self._lock:
            self._v[k] = self._v.get(k, 0.0) + amount


class Summary(_Metric):
    """Sliding-window quantiles (p50/p90/p99) + _sum/_count."""

    kind = "summary"

    def __init__(self, name, help="", labels=(), window: int = 10000,
                 quantiles: Sequence[float] = (0.5, 0.9, 0.99)):
        super().__init__(name, help, labels)
        self.window, self.quantiles = int(window), tuple(quantiles)
        self._obs: Dict[Tuple[str, ...], List[float]] = {}
        self._sum: Dict[Tuple[str, ...], float] = {}
        self._count: Dict[Tuple[str, ...], int] = {}

    def observe(self, value: float, **labels) -> None:
        k = self._key(labels)
        with self._lock:
            buf = self._obs.setdefault(k, [])
            buf.append(float(value))
            if len(buf) > self.window:
                del buf[: len(buf) - self.window]
            self._sum[k] = self._sum.get(k, 0.0) + value
            self._count[k] = self._count.get(k, 0) + 1

    def quantile(self, q: float, **labels) -> float:
        buf = self._obs.get(self._key(labels), [])
        return float(np.percentile(buf, 100 * q)) if buf else float("nan")

    def expose(self) -> List[str]:
        out = []
        for k, buf in sorted(self._obs.items()):
            for q in self.quantiles:
                v = float(np.percentile(buf, 100 * q)) if buf else float("nan")
                out.append(f"{self.name}{self._fmt_labels(k, {'quantile': str(q)})} {v:.17g}")
            out.append(f"{self.name}_sum{self._fmt_labels(k)} {self._sum[k]:.17g}")
            out.append(f"{self.name}_count{self._fmt_labels(k)} {self._count[k]}")
        return out


class Registry:
    def __init__(self):
        self._m: Dict[str, _Metric] = {}
        self._collectors: Dict[str, object] = {}
        self._lock = threading.Lock()

    def add_collector(self, key: str, fn) -> None:
        """``fn() -> [(name, kind, value, labels_dict)]`` sampled at every scrape (native
        components -- the MQTT broker's counters -- are read, not mirrored)."""
        with self._lock:
            self._collectors[key] = fn

    def remove_collector(self, key: str) -> None:
        with self._lock:
            self._collectors.pop(key, None)

    def _get(self, cls, name, help, labels, **kw):
        with self._lock:
            m = self._m.get(name)
            if m is None:
                m = cls(name, help, labels, **kw)
                self._m[name] = m
            elif not isinstance(m, cls):
                raise TypeError(f"metric {name} already registered as {type(m).__name__}")
            return m

    def counter(self, name, help="", labels=()) -> Counter:
        return self._get(Counter, name, help, labels)

    def gauge(self, name, help="", labels=()) -> Gauge:
        return self._get(Gauge, name, help, labels)

    def summary(self, name, help="", labels=(), **kw) -> Summary:
        return self._get(Summary, name, help, labels, **kw)

    def exposition(self) -> str:
        lines = []
        for name, m in sorted(self._m.items()):
            if m.help:
                lines.append(f"# HELP {name} {m.help}")
            lines.append(f"# TYPE {name} {m.kind}")
            lines += m.expose()
        with self._lock:
            collectors = list(self._collectors.values())
        sampled: Dict[str, Tuple[str, List[str]]] = {}
        for fn in collectors:
            try:
                samples = fn()
            except Exception:  # noqa: BLE001 - a stopped component drops out of the scrape
                continue
            for name, kind, value, labels in samples:
                lab = "{" + ",".join(f'{k}="{v}"' for k, v in sorted(labels.items())) + "}" if labels else ""
                sampled.setdefault(name, (kind, []))[1].append(f"{name}{lab} {float(value):.17g}")
        for name, (kind, rows) in sorted(sampled.items()):
            lines.append(f"# TYPE {name} {kind}")
            lines += rows
        return "\n".join(lines) + "\n"

    def serve(self, port: int = 0, addr: str = "127.0.0.1") -> HTTPServer:
        reg = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if self.path.rstrip("/") not in ("/metrics", ""):
                    self.send_response(404)
                    self.end_headers()
                    return
                body = reg.exposition().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        srv = HTTPServer((addr, port), H)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        return srv


REGISTRY = Registry()


# ---------------------------------------------------------------------------
# the engine's standard metrics, registered once on REGISTRY
# ---------------------------------------------------------------------------
class EngineMetrics:
    """Handles to the engine metrics; hot paths touch these at batch / epoch
    granularity only (never per event, never with a device sync)."""

    def __init__(self, reg: Registry):
        self.ingest_records = reg.counter("ingest_records_total", "records fetched from Kafka", ("topic",))
        self.ingest_bytes = reg.counter("ingest_bytes_total", "record bytes fetched from Kafka", ("topic",))
        self.ingest_skipped = reg.counter("ingest_skipped_records_total",
                                          "records a consumer jumped over after OFFSET_OUT_OF_RANGE "
                                          "(deleted by retention; auto.offset.reset)", ("topic",))
        self.decode_seconds = reg.counter("decode_seconds_total", "host time in fetch + Avro decode", ("topic",))
        self.decode_errors = reg.counter("decode_errors_total", "records that failed Avro decoding", ("topic",))
        self.h2d_bytes = reg.counter("h2d_bytes_total", "bytes staged host->device through the pinned ring")
        self.ring_occupancy = reg.gauge("ring_buffer_occupancy", "filled pinned-ring slots awaiting the consumer")
        self.train_rows = reg.counter("train_rows_total", "rows consumed by optimizer steps", ("model",))
        self.train_steps = reg.counter("train_steps_total", "optimizer steps", ("model",))
        self.train_step_latency = reg.summary("train_step_latency_us", "mean step time per epoch (us)", ("model",))
        self.epoch_loss = reg.gauge("train_epoch_loss", "last epoch loss", ("model",))
        self.allreduce_bytes = reg.counter("allreduce_bytes_total", "bytes all-reduced across replicas")
        self.allreduce_calls = reg.counter("allreduce_calls_total", "all-reduce launches")
        self.infer_rows = reg.counter("infer_rows_total", "rows scored / reconstructed", ("model",))
        self.infer_latency = reg.summary("infer_event_latency_us", "per-event inference latency (us)")
        self.anomaly_events = reg.counter("anomaly_events_total", "events flagged anomalous", ("model",))
        self.produced_records = reg.counter("produced_records_total", "records produced to Kafka", ("topic",))


ENGINE = EngineMetrics(REGISTRY)
