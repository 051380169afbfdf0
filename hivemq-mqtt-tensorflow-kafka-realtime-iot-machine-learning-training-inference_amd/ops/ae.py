"""Device runtime for the fused dense-autoencoder kernels (``csrc/kernels/ae_fused.hip``).

One optimizer step on ``n`` rows is two launches (plus one all-reduce under DP):

1. ``ae_train_partials``: fwd + bwd of every 16-row tile on MFMA, weight
   gradients accumulated in registers, one fp32 slab per workgroup;
2. ``reduce_adam``: slab reduction and the Keras/TF Adam update applied to the
   padded parameter image (``iterations`` counter lives on device).

With data parallelism the reduction writes the flat gradient bucket
(1536 gradient sums + 4 metric sums = 6160 bytes), which is all-reduced once per
step over RCCL, then a second ``reduce_adam`` (G = 1) applies Adam.  Metrics are
accumulated on device and read once per epoch, never per step.
"""
from __future__ import annotations


import os

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._ext import load_c

ACT_CODES = {"linear": 0, None: 0, "relu": 1, "tanh": 2, "sigmoid": 3}
NPARAM = 1536
NSLOT = 1540
# offsets / shapes of the padded image [in_pad][out_pad] and the bias row
LAYOUT = [(0, 32, 16, 31), (512, 16, 16, 15), (768, 16, 16, 15), (1024, 16, 32, 15)]

RA_WRITE_GRAD, RA_ADAM, RA_METRICS, RA_ADVANCE = 1, 2, 4, 8
# ae_train_kernel keeps 3 (<= 168 VGPRs) or 4 (<= 128 VGPRs, SML_AE_OCC=4) four-wave
# workgroups resident per CU.  A grid of exactly the resident capacity gives every wave
# the same tile count with no second dispatch round (sweep on MI355X, B = 4M rows:
# 768 blocks 176.6 us vs 1024 blocks 180.9 us at 3/CU; profiles/r01_v4/).


def default_train_blocks(device) -> int:
    """Host partials capacity: 2 x ae_train_blocks_per_cu() (5) workgroups per CU; the launcher
    trims each launch to its variant's own rounds x residency (one-tile: 2 x 4, packed pairs:
    3 x 3).  Two rounds of the resident capacity: each workgroup's share halves, so CUs that
    finish early pick up second-round workgroups (B = 8M rows: 2048 blocks 304 us vs
    1024 blocks 310 us at 4/CU; profiles/r01_v4/sweep_occ4.log)."""
    try:
        cus = torch.cuda.get_device_properties(torch.device(device)).multi_processor_count
    except Exception:  # noqa: BLE001 - no device properties (CPU build): MI355X has 256 CUs
        cus = 256
    return 2 * int(load_c().ae_train_blocks_per_cu()) * int(cus)


@dataclass
class AESpec:
    """Dense autoencoder D -> n1 -> n2 -> n3 -> D (reference cardata-v3.py:187-194)."""

    input_dim: int = 18
    encoding_dim: int = 14
    hidden_dim: int = 7
    activations: Tuple[str, str, str, str] = ("tanh", "relu", "tanh", "relu")
    activity_l1: float = 1e-7

    @property
    def dims(self) -> List[int]:
        return [self.input_dim, self.encoding_dim, self.hidden_dim, self.hidden_dim]

    @property
    def layer_sizes(self) -> List[Tuple[int, int]]:
        d, e, h = self.input_dim, self.encoding_dim, self.hidden_dim
        return [(d, e), (e, h), (h, h), (h, d)]

    @property
    def act_codes(self) -> List[int]:
        return [ACT_CODES[a] for a in self.activations]

    @property
    def n_params(self) -> int:
        return sum(i * o + o for i, o in self.layer_sizes)

    def check_fused(self) -> None:
        if not (1 <= self.input_dim <= 31 and 1 <= self.encoding_dim <= 15 and 1 <= self.hidden_dim <= 15):
            raise ValueError("fused AE kernel supports input_dim <= 31 and hidden sizes <= 15, got "
                             f"{self.layer_sizes}; wider autoencoders: streamml.nn.Sequential of Dense layers "
                             "(layer-by-layer engine on the K1/K2 and general GEMM kernels)")


def pack_image(weights: Sequence[np.ndarray]) -> np.ndarray:
    """Keras ``[k0, b0, k1, b1, k2, b2, k3, b3]`` (kernel [in, out]) -> padded 1536 image."""
    img = np.zeros(NPARAM, dtype=np.float32)
    for li, (off, ip, op, brow) in enumerate(LAYOUT):
        k = np.asarray(weights[2 * li], dtype=np.float32)
        b = np.asarray(weights[2 * li + 1], dtype=np.float32)
        i, o = k.shape
        view = img[off:off + ip * op].reshape(ip, op)
        view[:i, :o] = k
        view[brow, :o] = b
    return img


def unpack_image(img: np.ndarray, spec: AESpec) -> List[np.ndarray]:
    """Padded image -> Keras weight list ``[k0, b0, ..., k3, b3]``."""
    img = np.asarray(img, dtype=np.float32).reshape(-1)
    out: List[np.ndarray] = []
    for (off, ip, op, brow), (i, o) in zip(LAYOUT, spec.layer_sizes):
        view = img[off:off + ip * op].reshape(ip, op)
        out.append(view[:i, :o].copy())
        out.append(view[brow, :o].copy())
    return out


class FusedAE:
    """Holds the on-device state of one autoencoder replica and runs fused steps."""

    def __init__(self, spec: AESpec, weights: Sequence[np.ndarray], device,
                 lr: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999, epsilon: float = 1e-7,
                 max_blocks: Optional[int] = None, want_acc: bool = True,
                 scale: Optional[np.ndarray] = None, shift: Optional[np.ndarray] = None):
        spec.check_fused()
        self.C = load_c()
        self.spec = spec
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("FusedAE runs on a ROCm device only")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.lr, self.beta_1, self.beta_2, self.epsilon = lr, beta_1, beta_2, epsilon
        self.max_blocks = int(max_blocks) if max_blocks else default_train_blocks(self.device)
        self.want_acc = want_acc
        dev = self.device
        self.params = torch.from_numpy(pack_image(weights)).to(dev)
        self.m = torch.zeros(NPARAM, device=dev)
        self.v = torch.zeros(NPARAM, device=dev)
        self.iter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.partials = torch.zeros(self.max_blocks * NSLOT, device=dev)
        self.reduce_scratch = torch.zeros(((self.max_blocks + 31) // 32) * NSLOT, device=dev)
        # per-column arrival counters of the one-launch wide reduction (zero; re-armed by the kernel)
        self.reduce_counters = torch.zeros(64, dtype=torch.int32, device=dev)
        self.grad = torch.zeros(NSLOT, device=dev)
        self.metrics = torch.zeros(NSLOT - NPARAM, device=dev)   # epoch accumulators
        self.cursor = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ring: Optional[torch.Tensor] = None
        self.ring_xpack: Optional[torch.Tensor] = None
        self.ring_batch = 0
        self.set_normalizer(scale, shift)

    # -- normalisation fused into the first load ------------------------------------
    def set_normalizer(self, scale: Optional[np.ndarray], shift: Optional[np.ndarray]) -> None:
        if scale is None:
            self.scale = self.shift = None
        else:
            self.scale = torch.as_tensor(np.asarray(scale, dtype=np.float32), device=self.device)
            self.shift = torch.as_tensor(np.asarray(shift, dtype=np.float32), device=self.device)

    # -- state -------------------------------------------------------------------------
    def get_weights(self) -> List[np.ndarray]:
        return unpack_image(self.params.detach().cpu().numpy(), self.spec)

    def set_weights(self, weights: Sequence[np.ndarray]) -> None:
        self.params.copy_(torch.from_numpy(pack_image(weights)))

    def get_optimizer_state(self) -> Tuple[int, List[np.ndarray], List[np.ndarray]]:
        it = int(self.iter.item())
        return (it, unpack_image(self.m.cpu().numpy(), self.spec), unpack_image(self.v.cpu().numpy(), self.spec))

    def set_optimizer_state(self, it: int, m: Sequence[np.ndarray], v: Sequence[np.ndarray]) -> None:
        self.iter.fill_(int(it))
        self.m.copy_(torch.from_numpy(pack_image(m)))
        self.v.copy_(torch.from_numpy(pack_image(v)))

    # -- kernels ---------------------------------------------------------------------
    def _check_x(self, x: torch.Tensor) -> None:
        if x.device != self.device or x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1:
            raise ValueError("x must be a float32 [n, >=D] tensor with unit column stride on "
                             f"{self.device}, got {x.dtype} {tuple(x.shape)} on {x.device}")
        if x.size(1) < self.spec.input_dim:
            raise ValueError("x has too few columns")

    def grad_partials(self, x: torch.Tensor, bump_iter: bool = True) -> int:
        """Launch 1: fwd+bwd -> per-workgroup slabs; returns the grid size G."""
        self._check_x(x)
        return self.C.ae_train_partials(x, self.scale, self.shift, self.params, self.partials,
                                        self.iter if bump_iter else None, self.spec.dims, self.spec.act_codes,
                                        float(self.spec.activity_l1), bool(self.want_acc), self.max_blocks)

    def reduce(self, G: int, flags: int, gscale: float = 1.0, partials: Optional[torch.Tensor] = None) -> None:
        src = self.partials if partials is None else partials
        ring = self.ring.size(0) if self.ring is not None else 0
        self.C.reduce_adam(src, int(G), NSLOT, NPARAM, self.grad, self.params, self.m, self.v, self.iter,
                           self.lr, self.beta_1, self.beta_2, self.epsilon, float(gscale), self.metrics, int(flags),
                           self.cursor, int(self.ring_batch), int(ring),
                           self.reduce_scratch if partials is None else None,
                           self.reduce_counters if partials is None else None)

    # -- streaming ring consumption (device cursor; graph-capturable) ------------
    def attach_ring(self, ring: torch.Tensor, batch: int) -> None:
        """Consume ``batch`` rows per step from a device-resident ring of raw rows.

        The read position lives on the device (``self.cursor``) and is advanced by
        the Adam kernel, so a whole step -- launches and the all-reduce -- can be
        captured once in a hipGraph and replayed with no host work per step.
        """
        self._check_x(ring)
        if batch <= 0 or ring.size(0) % batch:
            raise ValueError("ring rows must be a positive multiple of the batch")
        self.ring, self.ring_batch = ring, int(batch)
        self.cursor.zero_()
        # Ingest-time tile packing (SML_AE_XPACK=0 disables): a copy of the ring laid out
        # per 16-row tile as [rows | 16 argmax(normalised x) bytes], so the training kernel
        # gets x's half of the accuracy metric with the tile's own two DMAs and skips the
        # 8-feature x 4-lane argmax of x per tile (profiles/r02/SUMMARY.md).
        self.ring_xpack = None
        if self._xpack_ok(ring.size(0), batch) and ring.size(1) == self.spec.input_dim:
            self.ring_xpack = self.C.pack_tiles_argmax(ring, self.spec.input_dim, self.scale, self.shift)

    def _xpack_ok(self, rows: int, batch: int) -> bool:
        """The tile-packed ring applies: the reference model (D = 18, reference activations,
        accuracy metric) and whole 16-row tiles -- the train kernels that read it."""
        return (self.want_acc and os.environ.get("SML_AE_XPACK", "1") != "0" and rows % 16 == 0
                and batch % 16 == 0 and self.spec.input_dim == 18
                and tuple(self.spec.activations) == ("tanh", "relu", "tanh", "relu"))

    def pack_ring(self, x: torch.Tensor, batch: int, index: Optional[torch.Tensor] = None,
                  perm_key: Optional[int] = None, reuse: bool = True) -> int:
        """Throughput-mode ring for ``step_ring``: the rows of ``x`` -- in order, through an
        explicit ``index``, or shuffled by the keyed bijection ``perm_key`` over all of ``x``
        (:meth:`perm_indices`) -- cut to whole batches and packed ONCE into the tile layout
        (normalize_fn + argmax(x), K8).  The shuffle is evaluated inside the pack kernel, so a
        shuffled epoch costs one gather pass over the rows: no permutation array, no copy.
        Returns the number of ring rows (full batches); the caller trains ``rows // batch``
        steps with ``step_ring`` and Keras' short last batch with ``step``."""
        self._check_x(x)
        B = int(batch)
        n = int(index.numel()) if index is not None else int(x.size(0))
        rows = (n // B) * B
        if rows == 0:
            raise ValueError(f"fewer rows ({n}) than one batch ({B})")
        if not (self._xpack_ok(rows, B) and x.size(1) == self.spec.input_dim):
            # no packed kernel for this model: materialise the epoch's rows, plain ring
            if perm_key is not None:
                index = self.perm_indices(int(x.size(0)), perm_key)
            src = x[index[:rows]] if index is not None else x[:rows]
            self.attach_ring(src.contiguous(), B)
            return rows
        nbytes = rows // 16 * (64 * self.spec.input_dim + 16)
        buf = getattr(self, "_pack_buf", None)
        if not reuse or buf is None or buf.numel() < nbytes:
            buf = self._pack_buf = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        if perm_key is not None:
            self.C.pack_tiles_argmax(x, self.spec.input_dim, self.scale, self.shift, None, buf,
                                     perm_key=int(perm_key) & ((1 << 64) - 1), perm_n=int(x.size(0)), n_rows=rows)
        else:
            idx = index[:rows].contiguous() if index is not None else None
            self.C.pack_tiles_argmax(x if idx is not None else x[:rows], self.spec.input_dim, self.scale, self.shift,
                                     idx, buf)
        # the ring tensor only carries the geometry (rows, stride): with a packed ring the
        # launcher reads the rows from the pack alone and refuses any variant that would not
        self.ring, self.ring_batch = x[:rows], B
        self.ring_xpack = buf[:nbytes]
        self.cursor.zero_()
        return rows

    def perm_indices(self, n: int, perm_key: int, start: int = 0, count: Optional[int] = None) -> torch.Tensor:
        """Rows ``start .. start + count`` of the keyed shuffle of [0, n) that ``pack_ring``
        evaluates in-kernel (int64 device tensor)."""
        return self.C.perm_indices(self.params, int(n), int(perm_key) & ((1 << 64) - 1), int(start),
                                   -1 if count is None else int(count))

    def step_ring(self, global_batch: Optional[int] = None, allreduce=None) -> None:
        if self.ring is None:
            raise RuntimeError("attach_ring() first")
        B = self.ring_batch
        gb = B if global_batch is None else int(global_batch)
        G = self.C.ae_train_partials(self.ring, self.scale, self.shift, self.params, self.partials, self.iter,
                                     self.spec.dims, self.spec.act_codes, float(self.spec.activity_l1),
                                     bool(self.want_acc), self.max_blocks, B, self.cursor, self.ring_xpack)
        if allreduce is None:
            self.reduce(G, RA_ADAM | RA_METRICS | RA_ADVANCE, gscale=1.0 / gb)
        else:
            # this replica's metric sums are accumulated BEFORE the all-reduce: every replica
            # keeps its own (``dp.reduce_metrics`` forms the global epoch values), as the
            # persistent kernel's in-kernel exchange and the CPU trainer do
            self.reduce(G, RA_WRITE_GRAD | RA_METRICS)
            allreduce(self.grad)
            self.reduce(1, RA_ADAM | RA_ADVANCE, gscale=1.0 / gb, partials=self.grad)

    def train_minibatches(self, nsteps: int, prof: Optional[torch.Tensor] = None, dp=None) -> None:
        """``nsteps`` sequential optimizer steps of ``ring_batch`` rows each, in ONE launch.

        Keras ``fit(batch_size=32)`` semantics (one Adam update per small batch, the
        reference's setting: cardata-v3.py:187-203) without a launch per step: the
        persistent kernel in ``csrc/kernels/ae_minibatch.hip`` keeps parameters, Adam
        moments and activations on chip and consumes the attached ring from the device
        cursor.  fp32 arithmetic.  ``dp`` (a process-group ``P2PGroup``): every step's
        gradient is summed over the ranks inside the kernel (global batch = world x batch).
        ``prof`` (int64 [11], optional) accumulates per-phase shader cycles of wave 0.
        """
        if self.ring is None:
            raise RuntimeError("attach_ring() first")
        B = self.ring_batch
        if B > self.max_minibatch():
            raise ValueError(f"batch {B} > {self.max_minibatch()}: use step_ring()")
        self._launch_minibatch(self.ring, self.cursor, B, int(nsteps), prof, dp=dp)

    def max_minibatch(self) -> int:
        """Largest batch the persistent small-batch trainer takes (128: cardata-v3's 100 fits)."""
        return int(self.C.ae_minibatch_max_batch())

    def train_rows(self, x: torch.Tensor, batch: int, max_steps: Optional[int] = None,
                   chunk_steps: int = 1 << 14, dp=None) -> Tuple[int, int]:
        """Keras ``fit`` over the rows of ``x`` in order: one Adam update per ``batch`` rows,
        the last batch short if ``len(x)`` is not a multiple (Keras' partial final batch),
        all on the persistent kernel (``csrc/kernels/ae_minibatch.hip``).

        Launches: ``ceil(full_batches / chunk_steps)`` for the full batches (each launch
        runs ``chunk_steps`` sequential steps with parameters, moments and activations on
        chip) plus one for the partial batch.  Returns ``(steps, rows)`` consumed, capped
        by ``max_steps`` (the reference's ``take(100)``, cardata-v3.py:218).

        ``dp`` (:class:`~streamml.parallel.p2p.P2PGroup`, one process per GPU): every step's
        gradient is summed over the ranks inside the kernel (xGMI push + rank-order sum);
        every rank must run the same number of full batches (the caller agrees on it, see
        ``Autoencoder.fit``), and the partial batch is dropped.
        """
        self._check_x(x)
        B = int(batch)
        if not 1 <= B <= self.max_minibatch():
            raise ValueError(f"batch {B} outside [1, {self.max_minibatch()}]")
        n = int(x.size(0))
        nfull, rem = divmod(n, B)
        if max_steps is not None:
            if nfull >= max_steps:
                nfull, rem = int(max_steps), 0
            elif nfull + (1 if rem else 0) > max_steps:
                rem = 0
        if not hasattr(self, "_tcur"):
            self._tcur = torch.zeros(1, dtype=torch.int64, device=self.device)
        if dp is not None:
            rem = 0
        steps = 0
        if nfull:
            ring = x[:nfull * B]
            self._tcur.zero_()
            while steps < nfull:
                k = min(int(chunk_steps), nfull - steps)
                self._launch_minibatch(ring, self._tcur, B, k, dp=dp)
                steps += k
        if rem:
            self._tcur.zero_()
            self._launch_minibatch(x[nfull * B:nfull * B + rem], self._tcur, rem, 1)
            steps += 1
        return steps, nfull * B + rem

    def train_stream(self, chunks, batch: int, max_steps: Optional[int] = None, ring_rows: Optional[int] = None,
                     timeout_s: float = 60.0) -> Tuple[int, int]:
        """Keras ``fit`` over a stream of device row chunks on ONE persistent-kernel launch.

        The kernel (``ae_minibatch.hip`` streaming mode) starts before the first chunk and
        stays resident for the whole epoch; ``push`` copies each chunk into a device ring
        and rings a doorbell (a host-mapped row count written by the copy stream after the
        copy), the kernel waits only when its next batch has not landed yet, and reports the
        rows it no longer needs (back-pressure).  Batches straddle chunk boundaries inside
        the ring, so there is no carry copy and no launch per chunk.  The stream's last
        ``n % batch`` rows are Keras' short final batch (one plain launch).  Returns
        ``(steps, rows)``; ``max_steps`` = the reference's ``take(n)`` (cardata-v3.py:218).
        """
        B = int(batch)
        if not 1 <= B <= self.max_minibatch():
            raise ValueError(f"batch {B} outside [1, {self.max_minibatch()}]")
        D = self.spec.input_dim
        if ring_rows is None:
            ring_rows = 1 << 20
        # the kernel reports consumed rows every 8 steps and prefetches one batch ahead, so
        # back-pressure needs room for >= 10 batches beyond the consumed mark
        rows = max(32 * B, (int(ring_rows) // B) * B)
        sr = getattr(self, "_sring", None)
        if sr is None or sr.rows != rows or getattr(self, "_sring_b", None) != B:
            sr = self.C.StreamRing(self.device.index or 0, rows, D)
            self._sring, self._sring_b = sr, B
        if not hasattr(self, "_tcur"):
            self._tcur = torch.zeros(1, dtype=torch.int64, device=self.device)
        sr.reset()
        self._tcur.zero_()
        it0 = int(self.iter.item())
        nmax = (1 << 30) if max_steps is None else int(max_steps)
        if nmax <= 0:
            return 0, 0
        limit = None if max_steps is None else nmax * B
        # Set the producer up BEFORE the kernel starts: building a loader allocates pinned
        # memory and starts threads, and no runtime call that may synchronise the device may
        # run while the resident kernel waits for the rows it produces.
        it = iter(chunks)
        xd = next(it, None)
        sr.train(self._tcur, self.scale, self.shift, self.params, self.m, self.v, self.iter, self.metrics, B,
                 nmax, self.spec.dims, self.spec.act_codes, float(self.spec.activity_l1), self.lr, self.beta_1,
                 self.beta_2, self.epsilon, 1.0 / B, bool(self.want_acc), float(timeout_s),
                 precision=self._mb_precision())
        pushed = 0
        try:
            while xd is not None and (limit is None or pushed < limit):
                if xd.dim() != 2 or xd.size(1) < D:
                    raise ValueError(f"stream chunks must be [n, >= {D}] rows")
                if limit is not None and pushed + xd.size(0) > limit:
                    xd = xd[:limit - pushed]
                sr.push(xd, float(timeout_s))
                pushed += int(xd.size(0))
                xd = next(it, None)
        finally:
            sr.finish()
            sr.join()
            sr.synchronize()
            close = getattr(it, "close", None)
            if close is not None:   # a partly consumed producer cleans up now, not mid next epoch
                close()
        if sr.status:
            raise RuntimeError(f"streaming fit: the training kernel waited {timeout_s:.0f} s for rows")
        steps = int(self.iter.item()) - it0
        rem = pushed - steps * B
        if steps < pushed // B:
            raise RuntimeError(f"streaming fit: kernel trained {steps} of {pushed // B} full batches")
        if 0 < rem < B and steps < nmax:
            start = (steps * B) % rows      # a multiple of B: the short batch never wraps
            self._tcur.zero_()
            self._launch_minibatch(sr.ring()[start:start + rem], self._tcur, rem, 1)
            steps += 1
        else:
            rem = 0
        return steps, (steps - (1 if rem else 0)) * B + rem

    # Small-batch trainer precision.  False: fp32 end to end (the Keras-exact path).  True: the
    # forward / activation-gradient contractions of each step on bf16 MFMAs (fp32 accumulation,
    # fp32 weight gradients, fp32 master weights and Adam): Autoencoder.fit(batch_size=100)
    # 27.3 -> 33.3 M rows/s, parameters within 0.4-1.5 % of the fp32 run after 400 steps
    # (profiles/r05 SUMMARY §9).  Passed to every launch of this model as an explicit argument
    # (SML_MB_BF16=1 stays a process-wide default for models that leave it unset); the in-kernel
    # DP exchange always runs fp32.
    minibatch_bf16 = None

    def _mb_precision(self) -> int:
        return -1 if self.minibatch_bf16 is None else int(bool(self.minibatch_bf16))

    def _launch_minibatch(self, ring: torch.Tensor, cursor: torch.Tensor, B: int, nsteps: int,
                          prof: Optional[torch.Tensor] = None, dp=None) -> None:
        kw, gscale = {}, 1.0 / B
        if dp is not None:
            if dp.in_launch:
                raise ValueError("a single FusedAE replica needs a process-group P2PGroup (one rank per process)")
            it0 = int(self.iter.item())
            kw = dp.kernel_args(it0)
            gscale = 1.0 / (B * dp.world)
        self.C.ae_train_minibatches(ring, cursor, self.scale, self.shift, self.params, self.m, self.v,
                                    self.iter, self.metrics, int(B), int(nsteps), self.spec.dims,
                                    self.spec.act_codes, float(self.spec.activity_l1), self.lr, self.beta_1,
                                    self.beta_2, self.epsilon, gscale, bool(self.want_acc), prof, None,
                                    precision=self._mb_precision(), **kw)
        if dp is not None:
            dp.note_iter(it0 + int(nsteps) - 1)
            dp.check()

    def step(self, x: torch.Tensor, global_batch: Optional[int] = None, allreduce=None) -> None:
        """One full optimizer step on ``x`` (all rows of the local micro-batch).

        ``global_batch`` defaults to ``len(x)``; under DP pass the global batch and
        an ``allreduce(tensor)`` callable (sum over replicas, in place).
        """
        n = x.size(0)
        gb = n if global_batch is None else int(global_batch)
        G = self.grad_partials(x)
        if allreduce is None:
            self.reduce(G, RA_ADAM | RA_METRICS, gscale=1.0 / gb)
        else:
            self.reduce(G, RA_WRITE_GRAD | RA_METRICS)   # local metric sums (see step_ring)
            allreduce(self.grad)
            self.reduce(1, RA_ADAM, gscale=1.0 / gb, partials=self.grad)

    def step_empty(self, global_batch: int, allreduce) -> None:
        """This replica has no rows in a data-parallel step (the uneven tail of a sharded
        streaming epoch): a zero gradient bucket into the all-reduce, then the same Adam
        update (and iteration count) as every replica that had rows."""
        self.grad.zero_()
        self.iter.add_(1)   # what the train kernel's first workgroup does for a step with rows
        allreduce(self.grad)
        self.reduce(1, RA_ADAM, gscale=1.0 / int(global_batch), partials=self.grad)

    def gradients(self, x: torch.Tensor, global_batch: Optional[int] = None) -> Tuple[List[np.ndarray], np.ndarray]:
        """Mean-over-batch gradients (Keras weight order) + raw metric sums; no update."""
        G = self.grad_partials(x, bump_iter=False)
        self.reduce(G, RA_WRITE_GRAD)
        gb = x.size(0) if global_batch is None else global_batch
        g = self.grad.detach().cpu().numpy()
        return unpack_image(g[:NPARAM] / gb, self.spec), g[NPARAM:].copy()

    def reset_metrics(self) -> None:
        self.metrics.zero_()

    def read_metrics(self) -> dict:
        """Epoch metrics in Keras terms from the device accumulators (one host sync)."""
        return self.metrics_from(self.metrics.cpu())

    def metrics_from(self, acc) -> dict:
        """Keras metrics from a host copy of the 4 accumulators (sum sq err, sum |h1|, correct, rows)."""
        sq, ab, corr, rows = [float(v) for v in acc.tolist()]
        D = self.spec.input_dim
        rows = max(rows, 1.0)
        loss = (sq / D + self.spec.activity_l1 * ab) / rows
        return {"loss": loss, "mse": sq / (D * rows), "accuracy": corr / rows, "rows": rows}

    def forward(self, x: torch.Tensor, recon: bool = True, score: bool = True,
                threshold: Optional[float] = None, metrics: Optional[torch.Tensor] = None):
        """Inference: reconstruction [n, D], per-row MSE score [n], anomaly flag [n].
        ``metrics`` (float32 [4] on the device): += (sum squared error, sum |h1|, correct
        argmax, rows) -- Keras ``evaluate`` from the forward pass alone."""
        self._check_x(x)
        n = x.size(0)
        D = self.spec.input_dim
        r = torch.empty((n, D), device=self.device) if recon else None
        s = torch.empty(n, device=self.device) if score else None
        f = torch.empty(n, dtype=torch.uint8, device=self.device) if threshold is not None else None
        self.C.ae_forward(x, self.scale, self.shift, self.params, r, s, f,
                          float(threshold if threshold is not None else 0.0), self.spec.dims,
                          self.spec.act_codes, self.max_blocks, metrics)
        return r, s, f

    def evaluate_sums(self, x: torch.Tensor, batch: int = 1 << 22) -> np.ndarray:
        """(sum squared error, sum |h1|, correct, rows) over x: forward kernel only."""
        acc = torch.zeros(4, device=self.device)
        for s0 in range(0, x.size(0), batch):
            self.forward(x[s0:s0 + batch], recon=False, score=False, metrics=acc)
        return acc.double().cpu().numpy()
