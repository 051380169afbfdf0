"""Data parallelism over RCCL (torch.distributed backend ``nccl`` on ROCm).

The reference has no ML-level parallelism at all; its only
scale-out axis is Kafka partitions / consumer groups.  Here one process drives
one GPU, every replica consumes a disjoint car-key shard of the stream
(shard-by-key), and the whole per-step gradient -- 1536 gradient sums plus the 4
metric sums of the fused AE step, 6 KB -- travels in ONE flat all-reduce.
At that size a ring all-reduce over xGMI is latency-bound (~2(N-1) hops of a
few microseconds), so the design lever is the per-GPU micro-batch size (work per
collective), not bucketing.

On CPU (tests) the same code runs over ``gloo``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..obs.metrics import ENGINE


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None

    @property
    def is_dist(self) -> bool:
        return self.world_size > 1 or self.backend is not None

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_from_env(device_type: Optional[str] = None, timeout_s: Optional[int] = None) -> DistEnv:
    """Initialise the process group from torchrun's RANK/WORLD_SIZE/LOCAL_RANK.

    Single-process runs (no WORLD_SIZE or WORLD_SIZE=1) do not create a group, unless
    ``SML_FORCE_PG=1`` asks for one at world 1 (TCP rendezvous on MASTER_ADDR/PORT,
    defaulting to 127.0.0.1 and a free port).
    ``device_type`` defaults to ``cuda`` (ROCm) when available, else ``cpu``.
    """
    if timeout_s is None:   # collective watchdog: a dead / hung peer raises instead of hanging
        timeout_s = int(os.environ.get("SML_PG_TIMEOUT_S", "600"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # SML_SHARE_GPU0=1 maps every rank onto GPU 0 (multi-rank rehearsal on a
        # one-GPU box; RCCL refuses two ranks on one device, so that mode uses gloo)
        shared = os.environ.get("SML_SHARE_GPU0") == "1"
        local_dev = 0 if shared else local
        torch.cuda.set_device(local_dev)
        device = torch.device("cuda", local_dev)
        backend = os.environ.get("SML_DIST_BACKEND", "gloo" if shared else "nccl")   # nccl = RCCL on ROCm
    else:
        device = torch.device("cpu")
        backend = "gloo"
    force = os.environ.get("SML_FORCE_PG") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(free_port())
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if restart is not None and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
            # torchrun keeps one store across restarts: key this attempt's rendezvous by the
            # restart count so a restarted group never reads the dead attempt's addresses
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, False,
                                 timeout=datetime.timedelta(seconds=timeout_s))
            kw["store"] = dist.PrefixStore(f"/sml/attempt_{restart}", base)
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return DistEnv(rank=rank, world_size=world, local_rank=local, device=device,
                   backend=backend if (world > 1 or force) else None)


def free_port() -> int:
    """An unused TCP port on 127.0.0.1 (rendezvous for a self-launched or forced group)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _pg_active() -> bool:
    """A process group exists: torchrun with WORLD_SIZE > 1, or one forced at world 1
    (``SML_FORCE_PG=1``: the whole DP path -- RCCL communicator, collectives, P2P
    exchange -- on a single GPU, so it is exercised even where only one device exists)."""
    return dist.is_available() and dist.is_initialized()


def allreduce_sum_(t: torch.Tensor) -> torch.Tensor:
    """In-place SUM all-reduce of one flat bucket (no-op without a process group)."""
    if _pg_active():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        ENGINE.allreduce_calls.inc()
        ENGINE.allreduce_bytes.inc(t.numel() * t.element_size())
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _pg_active():
        dist.broadcast(t, src=src)
    return t


def sync_model_from_rank0(model) -> None:
    """Broadcast rank 0's parameters AND optimizer state to every replica (after init / load)."""
    if not (_pg_active()):
        return
    fp = getattr(model, "fp", None)
    if fp is not None and getattr(model, "_fused", None) is None:
        for t in (fp.flat, fp.m, fp.v, fp.iter):
            dist.broadcast(t, src=0)
        return
    inner = getattr(model, "_fused", None) or model
    import numpy as np
    dev = inner.device
    ws = inner.get_weights()
    flat = torch.as_tensor(np.concatenate([w.ravel() for w in ws]), device=dev)
    dist.broadcast(flat, src=0)
    out, o = [], 0
    for w in ws:
        out.append(flat[o:o + w.size].cpu().numpy().reshape(w.shape))
        o += w.size
    inner.set_weights(out)
    be = getattr(inner, "backend", None)
    if be is not None and hasattr(be, "get_optimizer_state"):
        it, m, v = be.get_optimizer_state()
        st = torch.as_tensor(np.concatenate([np.array([it], np.float64)] + [a.ravel().astype(np.float64) for a in m + v]),
                             device=dev)
        dist.broadcast(st, src=0)
        st = st.cpu().numpy()
        it2, o = int(st[0]), 1
        mm, vv = [], []
        for a in m:
            mm.append(st[o:o + a.size].reshape(a.shape).astype(np.float32))
            o += a.size
        for a in v:
            vv.append(st[o:o + a.size].reshape(a.shape).astype(np.float32))
            o += a.size
        be.set_optimizer_state(it2, mm, vv)


_REDUCE_OPS = {"min": "MIN", "max": "MAX", "sum": "SUM"}


def collective_device() -> torch.device:
    """Where a small host-side collective's tensor must live: the current GPU under RCCL
    (``nccl``), the CPU under gloo."""
    if _pg_active() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def agree(values, device: Optional[torch.device] = None, ops=None):
    """Element-wise collective agreement on small ints (``ops`` per element: ``"min"``
    (default), ``"max"`` or ``"sum"``): every rank returns the same list.  One all-reduce
    per distinct op (no-op without a process group)."""
    vals = [int(v) for v in values]
    if not (_pg_active()):
        return vals
    ops = ops or ["min"] * len(vals)
    if device is None:
        device = collective_device()
    out = []
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    for op in sorted(set(ops)):
        u = t.clone()
        dist.all_reduce(u, op=getattr(dist.ReduceOp, _REDUCE_OPS[op]))
        out.append((op, u.cpu().tolist()))
    res = dict(out)
    return [res[o][i] for i, o in enumerate(ops)]


def allreduce_max(value: float, device: torch.device) -> float:
    if _pg_active():
        t = torch.tensor([value], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return value


def reduce_metrics(metrics: dict, device: torch.device, weight_key: str = "rows") -> dict:
    """Row-weighted average of per-replica epoch metrics (one small all-reduce per epoch)."""
    if not (_pg_active()):
        return dict(metrics)
    keys = [k for k in metrics if k != weight_key]
    w = float(metrics.get(weight_key, 1.0))
    t = torch.tensor([float(metrics[k]) * w for k in keys] + [w], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    tot = float(t[-1].item())
    out = {k: float(t[i].item()) / max(tot, 1e-30) for i, k in enumerate(keys)}
    out[weight_key] = tot
    return out


def barrier(device: Optional[torch.device] = None) -> None:
    if _pg_active():
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def rccl_version() -> Optional[str]:
    """The collective library's version as torch reports it (RCCL on ROCm), or None."""
    try:
        v = torch.cuda.nccl.version()
    except Exception:  # noqa: BLE001 - no RCCL in this build / no GPU
        return None
    return ".".join(str(x) for x in v) if isinstance(v, (tuple, list)) else str(v)


def device_identity(device: torch.device) -> dict:
    """Who this rank is and which physical device it drives: host, pid, device index, PCI bus id,
    UUID and name -- so a multi-GPU record can show that N distinct GPUs took part."""
    import socket
    ident = {"host": socket.gethostname(), "pid": os.getpid(), "device": str(device)}
    if device.type == "cuda":
        p = torch.cuda.get_device_properties(device)
        ident.update(
            name=p.name,
            index=device.index if device.index is not None else torch.cuda.current_device(),
            pci_bus_id="%04x:%02x:%02x.0" % (int(getattr(p, "pci_domain_id", 0)), int(getattr(p, "pci_bus_id", 0)),
                                             int(getattr(p, "pci_device_id", 0))),
            uuid=str(getattr(p, "uuid", "") or ""),
            arch=str(getattr(p, "gcnArchName", "") or ""))
    return ident


def device_key(ident: dict) -> tuple:
    """What makes two ranks' devices the same physical device: host + UUID (or PCI bus id)."""
    return (ident.get("host"), ident.get("uuid") or ident.get("pci_bus_id") or ident.get("device"))


def check_distinct_devices(idents, world: int, rehearsal: bool) -> dict:
    """Decide whether a ``world``-rank measurement may be reported as ``n_gpus = world``: it needs
    ``world`` distinct devices (by :func:`device_key`), unless it is a labelled rehearsal
    (``SML_SHARE_GPU0=1``: every rank on GPU 0).  Returns ``{"ok", "n_distinct_devices",
    "rehearsal", "reason"}``; a pure function, so the refusal logic is unit-tested on CPU."""
    keys = [device_key(i) for i in idents]
    n = len(set(keys))
    ok = len(idents) == world and (n == world or rehearsal)
    reason = ""
    if len(idents) != world:
        reason = f"{len(idents)} identities for world {world}"
    elif n != world and not rehearsal:
        reason = f"only {n} distinct device(s) among {world} ranks: {sorted(set(keys))}"
    return {"ok": ok, "n_distinct_devices": n, "rehearsal": bool(rehearsal), "reason": reason}


def peer_access(device: torch.device, peers) -> dict:
    """``can_device_access_peer`` from this rank's device to each other local device index."""
    out = {}
    if device.type != "cuda":
        return out
    me = device.index if device.index is not None else torch.cuda.current_device()
    for d in sorted(set(int(x) for x in peers)):
        if d != me:
            try:
                out[str(d)] = bool(torch.cuda.can_device_access_peer(me, d))
            except Exception as e:  # noqa: BLE001
                out[str(d)] = repr(e)[:80]
    return out


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def shard_range(n: int, rank: int, world: int):
    """Contiguous [start, stop) of ``n`` items owned by ``rank``."""
    per = n // world
    rem = n % world
    start = rank * per + min(rank, rem)
    return start, start + per + (1 if rank < rem else 0)


def shard_by_key(keys, rank: int, world: int):
    """Boolean mask of records whose key hashes to ``rank`` (stable FNV-1a)."""
    import numpy as np

    out = np.zeros(len(keys), dtype=bool)
    for i, k in enumerate(keys):
        b = k.encode() if isinstance(k, str) else bytes(k)
        h = 0xCBF29CE484222325
        for c in b:
            h ^= c
            h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
        out[i] = (h % world) == rank
    return out
