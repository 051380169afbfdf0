"""Keras-granularity data parallelism over xGMI without a collective library call per step.

The reference trains one model in one process (no DP anywhere).  The
BASELINE adds DP on 8 MI355X.  At the reference's own optimizer granularity -- one Adam
step per 32 (cardata-v1) or 100 (cardata-v3, AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:
176-177) rows -- a step is 2-4 us of GPU work, while an RCCL all-reduce of even a 6 KB
bucket costs ~10-30 us plus a launch.  So the gradient exchange is built
into the persistent trainer (``csrc/kernels/ae_minibatch.hip``): every rank pushes its
partial gradient tile straight into every peer's receive buffer over the point-to-point
xGMI links (HIP IPC-mapped, uncached memory), polls its own buffer and sums the world's
partials in rank order -- bit-identical replicas, one hop, no launch, no host.

:class:`P2PGroup` sets the buffers up (one ``hipIpcMemHandle`` per rank, exchanged over the
process group, each mapping validated by a DMA read of the peer's magic word before any
kernel touches it).  ``P2PGroup.local(device, world)`` puts every rank's buffer in one
process: the ranks are then the workgroups of ONE launch (``AEFleet`` replicas) -- the
same kernel path, used by the tests and on a single GPU.  ``allreduce_`` is a
host-callable one-launch small all-reduce over the same buffers (the launch-per-step
path's replacement for an RCCL call on <= 64 KB buckets).

Every device-side spin is bounded (``timeout_s``): a missing peer turns into
:class:`P2PTimeout` on the host, never a hung GPU.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops._ext import load_c

NSLOTS = 1540   # the AE's padded 1536-float gradient image (+ 4 metric sums for allreduce_)


class P2PTimeout(RuntimeError):
    pass


class P2PGroup:
    def __init__(self, device, slots: int = NSLOTS, group=None, timeout_s: float = 10.0, _local_world: int = 0):
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        C = load_c()
        self.timeout_s = float(timeout_s)
        self._last_iter = -1
        if _local_world:
            self.x = C.P2PExchange.local(self.device.index, int(_local_world), int(slots))
            self.rank, self.world, self.group, self.in_launch = 0, int(_local_world), None, True
            return
        import torch.distributed as dist
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.in_launch = False
        self.x = C.P2PExchange(self.device.index, self.rank, self.world, int(slots))
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(self.x.handle()), group=group)
        self.x.open(list(handles))          # maps + validates every peer buffer
        dist.barrier(group=group)

    @classmethod
    def try_create(cls, device, slots: int = NSLOTS, group=None, timeout_s: float = 10.0):
        """Collective: every rank gets a group, or every rank gets ``None`` (e.g. no IPC /
        peer access on this platform) -- never a mix that would strand a peer's kernel."""
        import torch.distributed as dist

        from .dp import agree
        ok, err, g = 1, None, None
        C = load_c()
        dev = torch.device(device)
        # every rank must reach every other rank's GPU directly (xGMI peer access);
        # ranks that share a GPU (tests) need no peer mapping
        my_idx = dev.index if dev.index is not None else torch.cuda.current_device()
        idxs = [None] * dist.get_world_size(group)
        dist.all_gather_object(idxs, int(my_idx), group=group)
        for j in set(idxs):
            if j != my_idx and not torch.cuda.can_device_access_peer(my_idx, j):
                ok, err = 0, RuntimeError(f"GPU {my_idx} has no peer access to GPU {j}")
        try:
            if not ok:
                raise err
            x = C.P2PExchange(dev.index if dev.index is not None else torch.cuda.current_device(),
                              dist.get_rank(group), dist.get_world_size(group), int(slots))
            h = bytes(x.handle())
        except Exception as e:  # noqa: BLE001 - agreed on below
            ok, err, h, x = 0, e, b"", None
        handles = [None] * dist.get_world_size(group)
        dist.all_gather_object(handles, h, group=group)
        if agree([ok], dev)[0]:
            try:
                x.open(list(handles))
            except Exception as e:  # noqa: BLE001
                ok, err = 0, e
        if not agree([ok], dev)[0]:
            return None, err
        g = cls.__new__(cls)
        g.device = dev if dev.index is not None else torch.device("cuda", torch.cuda.current_device())
        g.timeout_s, g._last_iter, g.x = float(timeout_s), -1, x
        g.rank, g.world, g.group, g.in_launch = dist.get_rank(group), dist.get_world_size(group), group, False
        dist.barrier(group=group)
        # self-test before any persistent kernel relies on the exchange: one small all-reduce
        # of exact integers (bounded device-side polls; a failure disables P2P on every rank)
        try:
            t = torch.arange(64, dtype=torch.float32, device=g.device) + float(g.rank)
            g.allreduce_(t)
            g.check()
            want = torch.arange(64, dtype=torch.float32, device=g.device) * g.world + float(sum(range(g.world)))
            ok = int(bool(torch.equal(t, want)))
            err = None if ok else RuntimeError("P2P self-test sum mismatch")
        except Exception as e:  # noqa: BLE001 - agreed on below
            ok, err = 0, e
        if not agree([ok], dev)[0]:
            return None, err or RuntimeError("P2P self-test failed on a peer")
        return g, None

    @classmethod
    def local(cls, device, world: int, slots: int = NSLOTS, timeout_s: float = 10.0) -> "P2PGroup":
        """Every rank's buffer in this process: ranks = workgroups of one launch."""
        return cls(device, slots, timeout_s=timeout_s, _local_world=int(world))

    # ------------------------------------------------------------------ kernel hook
    def kernel_args(self, start_iter: int) -> dict:
        """Arguments for ``ae_train_minibatches``: the gradient tiles of optimizer iteration
        ``it`` carry tag ``it + 1``.  Iterations must keep increasing across launches; a
        restart from an older iteration (new model, restored checkpoint) re-zeroes the
        receive buffers first, behind a barrier on both sides, so no stale granule of the
        earlier run can match a new tag."""
        from ..ops.ae import NPARAM
        if int(self.x.slots) < NPARAM:   # the trainer strides peer buffers by NPARAM floats
            raise ValueError(f"P2P exchange built with {int(self.x.slots)} slots; the persistent trainer needs "
                             f">= {NPARAM}")
        if start_iter <= self._last_iter:
            self._reset()
        return dict(dp_peers=int(self.x.peers_ptr), dp_ranks=self.world, dp_rank0=0 if self.in_launch else self.rank,
                    dp_status=int(self.x.status_ptr), dp_timeout_ticks=int(self.timeout_s * 1e8))

    def note_iter(self, last_iter: int) -> None:
        self._last_iter = max(self._last_iter, int(last_iter))

    def _reset(self) -> None:
        torch.cuda.synchronize(self.device)
        if not self.in_launch:
            import torch.distributed as dist
            dist.barrier(group=self.group)
        self.x.clear()
        if not self.in_launch:
            import torch.distributed as dist
            dist.barrier(group=self.group)
        self._last_iter = -1

    def check(self) -> None:
        """Raise if a device-side poll gave up (synchronises the device)."""
        torch.cuda.synchronize(self.device)
        if self.x.status():
            self.x.reset_status()
            raise P2PTimeout(f"rank {self.rank}: a peer's gradient never arrived within {self.timeout_s} s")

    # ------------------------------------------------------------------ host collective
    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group (rank order): one launch, one xGMI hop."""
        if self.in_launch:
            raise RuntimeError("allreduce_ needs one process per rank")
        load_c().p2p_allreduce(t, self.x, self.timeout_s)
        return t
