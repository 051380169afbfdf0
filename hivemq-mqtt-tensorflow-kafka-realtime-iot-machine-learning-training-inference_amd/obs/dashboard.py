"""Grafana dashboard for the engine's Prometheus metrics.

The reference ships its dashboards through the Prometheus Operator on GKE
(infrastructure/hivemq/README.md:23, infrastructure/confluent/README.md): HiveMQ
broker panels, Kafka-extension throughput and the device simulator. Here the
dashboard is generated from the metric names this package actually exports
(``obs.metrics.ENGINE`` and the MQTT broker collector in ``mqtt/__init__.py``), so
a renamed metric breaks ``tests/test_obs.py`` instead of silently emptying a panel.

``python -m streamml.obs.dashboard > deploy/grafana/streamml.json`` regenerates
the committed copy.
"""
from __future__ import annotations

import json
import sys
from typing import Dict, List, Tuple

# (title, unit, [(promql, legend)]) per panel, grouped by row
_ROWS: List[Tuple[str, List[Tuple[str, str, List[Tuple[str, str]]]]]] = [
    ("MQTT broker (HiveMQ counterpart)", [
        ("Inbound / outbound PUBLISH rate", "ops", [
            ("sum(rate(com_hivemq_messages_incoming_publish_count[1m]))", "incoming"),
            ("sum(rate(com_hivemq_messages_outgoing_publish_count[1m]))", "outgoing")]),
        ("Connections", "short", [
            ("sum(com_hivemq_networking_connections_current)", "current"),
            ("sum(rate(com_hivemq_networking_connections_total_count[1m]))", "new / s")]),
        ("Kafka bridge", "ops", [
            ("sum(rate(kafka_extension_total_success_count[1m]))", "sent / s"),
            ("sum(rate(kafka_extension_total_failure_count[1m]))", "failed / s"),
            ("sum(kafka_extension_queue_current)", "queued")]),
        ("Retained messages", "short", [
            ("sum(com_hivemq_messages_retained_current)", "retained")]),
    ]),
    ("Ingest (Kafka -> Avro -> pinned ring -> HBM)", [
        ("Records fetched", "ops", [
            ("sum by (topic) (rate(ingest_records_total[1m]))", "{{topic}}")]),
        ("Fetch bandwidth", "Bps", [
            ("sum by (topic) (rate(ingest_bytes_total[1m]))", "{{topic}}"),
            ("rate(h2d_bytes_total[1m])", "H2D")]),
        ("Host decode time share", "percentunit", [
            ("sum by (topic) (rate(decode_seconds_total[1m]))", "{{topic}}")]),
        ("Decode errors", "ops", [
            ("sum by (topic) (rate(decode_errors_total[1m]))", "{{topic}}")]),
        ("Pinned ring occupancy", "short", [
            ("ring_buffer_occupancy", "{{instance}}")]),
    ]),
    ("Training (MI355X)", [
        ("Train rows / s", "ops", [
            ("sum by (model) (rate(train_rows_total[1m]))", "{{model}}")]),
        ("Optimizer steps / s", "ops", [
            ("sum by (model) (rate(train_steps_total[1m]))", "{{model}}")]),
        ("Step latency", "µs", [
            ("train_step_latency_us{quantile=\"0.5\"}", "p50 {{model}}"),
            ("train_step_latency_us{quantile=\"0.99\"}", "p99 {{model}}")]),
        ("Epoch loss", "short", [
            ("train_epoch_loss", "{{model}}")]),
        ("Gradient all-reduce (RCCL)", "Bps", [
            ("rate(allreduce_bytes_total[1m])", "bytes / s"),
            ("rate(allreduce_calls_total[1m])", "calls / s")]),
    ]),
    ("Scoring", [
        ("Scored events / s", "ops", [
            ("sum by (model) (rate(infer_rows_total[1m]))", "{{model}}")]),
        ("Per-event latency", "µs", [
            ("infer_event_latency_us{quantile=\"0.5\"}", "p50"),
            ("infer_event_latency_us{quantile=\"0.99\"}", "p99")]),
        ("Anomalies flagged / s", "ops", [
            ("sum by (model) (rate(anomaly_events_total[1m]))", "{{model}}")]),
        ("Records produced", "ops", [
            ("sum by (topic) (rate(produced_records_total[1m]))", "{{topic}}")]),
    ]),
]


def metric_names() -> List[str]:
    """Every metric name a panel query references (for the sync test)."""
    import re
    names = set()
    for _, panels in _ROWS:
        for _, _, targets in panels:
            for expr, _ in targets:
                # identifiers followed by '[' (range), '{' (selector), ')' or end: metric names
                for m in re.finditer(r"([a-z_][a-z0-9_]*)\s*(?=\[|\{|\)|$)", expr):
                    if m.group(1) not in ("sum", "rate", "by", "topic", "model"):
                        names.add(m.group(1))
    return sorted(names)


def build(datasource: str = "Prometheus", title: str = "streamml - MI355X streaming ML") -> Dict:
    panels, pid, y = [], 1, 0
    for row_title, row_panels in _ROWS:
        panels.append({"id": pid, "type": "row", "title": row_title, "collapsed": False,
                       "gridPos": {"h": 1, "w": 24, "x": 0, "y": y}})
        pid, y = pid + 1, y + 1
        for i, (ptitle, unit, targets) in enumerate(row_panels):
            panels.append({
                "id": pid, "type": "timeseries", "title": ptitle,
                "datasource": {"type": "prometheus", "uid": datasource},
                "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
                "gridPos": {"h": 8, "w": 8, "x": (i % 3) * 8, "y": y + (i // 3) * 8},
                "targets": [{"expr": e, "legendFormat": lg, "refId": chr(ord("A") + k)}
                            for k, (e, lg) in enumerate(targets)],
            })
            pid += 1
        y += ((len(row_panels) + 2) // 3) * 8
    return {"title": title, "uid": "streamml-mi355x", "schemaVersion": 39, "version": 1,
            "time": {"from": "now-30m", "to": "now"}, "refresh": "10s", "tags": ["streamml", "mi355x"],
            "templating": {"list": []}, "panels": panels}


def main() -> None:
    json.dump(build(), sys.stdout, indent=1)
    sys.stdout.write("\n")


if __name__ == "__main__":
    main()
