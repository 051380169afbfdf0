"""Fault injection and failure detection for data-parallel jobs.

The reference has no ML-level fault tolerance (K8s ``restartPolicy: Never`` +
``kubectl wait --timeout=5m``, model-training.yaml:6, run.sh:47).  Here:

* **detection**: every collective runs under the process-group timeout set in
  :func:`streamml.parallel.dp.init_from_env` (``SML_PG_TIMEOUT_S``), so a dead or
  hung peer turns into an exception on the survivors instead of a hang; the
  launcher (``torchrun --max-restarts N``) then tears the group down and
  restarts every rank;
* **recovery**: restarted ranks resume from the newest complete checkpoint
  (:mod:`streamml.ckpt.resume`), rank 0's weights are broadcast;
* **injection** for tests: ``SML_FAULT_RANK=k SML_FAULT_STEP=s`` makes rank k
  exit hard (``os._exit``) when it reaches global step s, on the first attempt
  only (``TORCHELASTIC_RESTART_COUNT`` = 0) -- i.e. a process crash mid-epoch.
  ``SML_FAULT_MODE=hang`` sleeps instead, to exercise the collective timeout.
"""
from __future__ import annotations

import os
import sys
import time


def _attempt() -> int:
    return int(os.environ.get("TORCHELASTIC_RESTART_COUNT", os.environ.get("SML_ATTEMPT", "0")) or 0)


def maybe_inject(step: int, rank: int) -> None:
    """Call once per optimizer step; no-op unless the SML_FAULT_* variables select this rank/step."""
    fr = os.environ.get("SML_FAULT_RANK")
    fs = os.environ.get("SML_FAULT_STEP")
    if fr is None or fs is None:
        return
    if int(fr) != rank or int(fs) != step or _attempt() != 0:
        return
    mode = os.environ.get("SML_FAULT_MODE", "crash")
    sys.stderr.write(f"[fault-injection] rank {rank} {mode} at step {step}\n")
    sys.stderr.flush()
    if mode == "hang":
        time.sleep(float(os.environ.get("SML_FAULT_HANG_S", "3600")))
    os._exit(17)


def maybe_inject_range(start: int, stop: int, rank: int) -> None:
    """``maybe_inject`` for every step in ``[start, stop)`` -- the injection points of a
    whole persistent-kernel launch -- at O(1) cost (an epoch is ~10^4-10^5 steps)."""
    fs = os.environ.get("SML_FAULT_STEP")
    if fs is None or os.environ.get("SML_FAULT_RANK") is None:
        return
    if start <= int(fs) < stop:
        maybe_inject(int(fs), rank)
