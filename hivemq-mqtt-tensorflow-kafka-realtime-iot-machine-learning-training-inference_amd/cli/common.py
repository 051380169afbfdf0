"""Shared plumbing for the reference-compatible command-line front ends.

The reference scripts take positional ``sys.argv`` only and print
``Options: <argv>`` first (e.g. AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:22-37).
Every front end here accepts the same positional form and exits 1 with the same
usage line on a wrong count; extra knobs are ``--flags``.

``<servers>`` may be

* a Kafka bootstrap list ``host:port[,host:port]`` (SASL PLAIN with the
  reference's ``test/test123`` credentials by default, cardata-v3.py:7-15),
* ``fake://name`` -- an in-process broker (same wire protocol),
* ``synthetic://[rows]`` -- an in-process broker pre-filled with ``rows``
  synthetic car events (the simulator fleet of scenario.xml) on ``<topic>``,
  so a front end can run end to end on a machine without Kafka.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import List, Optional, Sequence

from ..config import REFERENCE_KAFKA_CONFIG

SYNTHETIC_DEFAULT_ROWS = 20000


class UsageError(SystemExit):
    pass


def print_options(argv: Sequence[str]) -> None:
    print("Options: ", list(argv), flush=True)


def parse(argv: Sequence[str], usage: str, positionals: Sequence[str], n_optional: int = 0,
          add_flags=None) -> argparse.Namespace:
    """Positional parse with the reference's exact arity check + usage message."""
    p = argparse.ArgumentParser(usage=usage, add_help=True)
    p.add_argument("args", nargs="*")
    p.add_argument("--device", default="auto", help="cuda:N | cpu | auto")
    p.add_argument("--kafka-config", default="auto",
                   help="'auto' (reference SASL config for real brokers, none for fake://), 'none', "
                        "or comma-separated key=value librdkafka entries")
    p.add_argument("--workdir", default=".", help="where model files are written / downloaded "
                                                   "(the reference uses '/')")
    p.add_argument("--store", default=None, help="model store URL (file://dir | gs://); default $SML_MODEL_STORE")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--synthetic-seed", type=int, default=0)
    if add_flags:
        add_flags(p)
    ns = p.parse_args(list(argv))
    lo, hi = len(positionals) - n_optional, len(positionals)
    if not lo <= len(ns.args) <= hi:
        print(usage)
        raise UsageError(1)
    for i, name in enumerate(positionals):
        setattr(ns, name, ns.args[i] if i < len(ns.args) else None)
    return ns


def kafka_config(servers: str, choice: str) -> Optional[List[str]]:
    if choice == "none":
        return None
    if choice == "auto":
        if servers.startswith(("fake://", "synthetic://")):
            return None
        return list(REFERENCE_KAFKA_CONFIG)
    return [s for s in choice.split(",") if s]


def prepare_servers(servers: str, topic: str, seed: int = 0, schema: str = "cardata-v1",
                    rows: Optional[int] = None, partitions: int = 1) -> str:
    """Resolve ``synthetic://[rows]`` into a pre-filled in-process broker (records keyed by
    car and spread over ``partitions`` with the Kafka murmur2 partitioner); others pass through."""
    if not servers.startswith("synthetic://"):
        return servers
    from ..data import produce as prod
    from ..data import stream as st
    from ..kafka import fake_broker

    rest = servers[len("synthetic://"):]
    n = int(rest) if rest else (rows or SYNTHETIC_DEFAULT_ROWS)
    name = f"synthetic-{topic}"
    b = fake_broker(name)
    if _has_topic(b, topic) and b.end_offset(topic, 0) > 0:   # already filled in this process
        return f"fake://{name}"
    b.create_topic(topic, max(1, int(partitions)))
    prod.produce(st.synthetic(n, chunk=8192, seed=seed), f"fake://{name}", topic, schema=schema, create=False,
                 partitions=max(1, int(partitions)))
    return f"fake://{name}"


def _has_topic(b, topic: str) -> bool:
    try:
        b.end_offset(topic, 0)
        return True
    except Exception:
        return False


def model_path(workdir: str, model_file: str) -> str:
    """Reference writes to ``"/" + model_file``; we write under ``--workdir``."""
    path = os.path.join(workdir, model_file.lstrip("/"))
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    return path


def run(main, argv: Optional[Sequence[str]] = None) -> int:
    """Entry wrapper: UsageError -> exit code, everything else propagates."""
    try:
        return int(main(list(sys.argv[1:] if argv is None else argv)) or 0)
    except UsageError as e:
        return int(e.code or 1)
