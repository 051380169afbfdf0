"""Checkpoint / resume for streaming training jobs.

The reference never resumes: every K8s run rebuilds and recompiles a fresh model
(cardata-v3.py:187-205) and re-reads the topic from the given offset; the Keras
``.h5`` it saves nevertheless carries the optimizer state.  Here a checkpoint is

* ``<dir>/ckpt-<epoch>.h5``   -- the Keras-layout model file (weights + Adam
  moments + ``iterations``), readable by ``load_model``;
* ``<dir>/ckpt-<epoch>.h5.state.json`` -- sidecar with the training position:
  completed epochs / steps, Kafka offsets per ``topic:partition`` (committed to
  the consumer group as well when a group is configured), world size, config.

A sidecar (not an extra HDF5 attribute) keeps strict Keras readers happy.  Both
files are written atomically (temp file + ``os.replace``) and only by rank 0
under data parallelism; the others wait at a barrier.  On restart every rank
reads the newest complete checkpoint, rank 0's weights are broadcast (RCCL /
gloo) so replicas start bit-identical, and training continues at the next
epoch -- the same run as without the failure (tests/test_resume.py).
"""
from __future__ import annotations

import glob
import json
import os
import re
import tempfile
import time
from typing import Dict, Optional, Tuple

SIDE = ".state.json"


def _rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _atomic_json(path: str, obj: dict) -> None:
    d = os.path.dirname(os.path.abspath(path))
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp-")
    with os.fdopen(fd, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    os.replace(tmp, path)


def checkpoint_path(ckpt_dir: str, epoch: int) -> str:
    return os.path.join(ckpt_dir, f"ckpt-{epoch:05d}.h5")


def save_checkpoint(model, ckpt_dir: str, epoch: int, step: int = 0, offsets: Optional[Dict[str, int]] = None,
                    extra: Optional[dict] = None, keep: int = 3) -> Optional[str]:
    """Rank 0 writes ``ckpt-<epoch>.h5`` + sidecar; all ranks synchronise. Returns the path (rank 0)."""
    from ..parallel.dp import barrier
    rank, world = _rank_world()
    path = checkpoint_path(ckpt_dir, epoch)
    if rank == 0:
        os.makedirs(ckpt_dir, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=ckpt_dir, prefix=".tmp-", suffix=".h5")
        os.close(fd)
        model.save(tmp)
        os.replace(tmp, path)
        state = {"epoch": int(epoch), "step": int(step), "offsets": dict(offsets or {}), "world_size": world,
                 "time": time.time(), **(extra or {})}
        _atomic_json(path + SIDE, state)   # the sidecar is written last: it marks the checkpoint complete
        for old in list_checkpoints(ckpt_dir)[:-keep] if keep > 0 else []:
            for p in (old, old + SIDE):
                if os.path.exists(p):
                    os.unlink(p)
    barrier(getattr(model, "device", None))
    return path if rank == 0 else None


def list_checkpoints(ckpt_dir: str):
    """Complete checkpoints (model + sidecar) in epoch order."""
    out = []
    for p in glob.glob(os.path.join(ckpt_dir, "ckpt-*.h5")):
        if os.path.exists(p + SIDE) and re.search(r"ckpt-(\d+)\.h5$", p):
            out.append(p)
    return sorted(out, key=lambda p: int(re.search(r"ckpt-(\d+)\.h5$", p).group(1)))


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    cks = list_checkpoints(ckpt_dir)
    return cks[-1] if cks else None


def read_state(path: str) -> dict:
    with open(path + SIDE) as f:
        return json.load(f)


def load_latest(ckpt_dir: str, loader, **kw) -> Tuple[Optional[object], Optional[dict]]:
    """(model, state) from the newest complete checkpoint, or (None, None)."""
    p = latest_checkpoint(ckpt_dir)
    if p is None:
        return None, None
    return loader(p, **kw), read_state(p)
