"""Fleet training: many independent small autoencoders on one GPU, Keras batch semantics.

The reference trains ONE dense autoencoder with ``fit(batch_size=32)``
(``python-scripts/AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:187-203``), streaming
from one topic.  In an IoT deployment the natural scale-out of that workload is many
models at once: one anomaly model per car / device group (a "digital twin" per
partition, as the MongoDB sink of the reference's Connect setup keys documents by car),
an ensemble, or a learning-rate sweep.  Each such model is far too small to use a GPU
on its own (one batch-32 step is ~1 MFLOP), so the fleet runs them side by side:

* ``csrc/kernels/ae_minibatch.hip`` in fleet mode -- workgroup ``b`` trains model ``b``
  for ``nsteps`` sequential Keras steps with its parameters, Adam moments and
  activations resident in LDS / VGPRs; a grid of M >= 256 workgroups fills the 256
  CUs.  The latency-optimal single-model build (~160 VGPRs) fits one 8-wave model per
  CU; fleets larger than the CU count switch to a 128-VGPR build that fits two
  (1 MI355X: 2.19 G rows/s at M = 256, 2.81 G rows/s at M = 1024; profiles/r01_v7);
* state is stacked: ``params/m/v [M, 1536]`` (the padded image of ``ops/ae.py``),
  ``iter/cursor [M]``, ``metrics [M, 4]``; model ``b`` reads either its own ring
  ``rings[b]`` (per-device streams) or one shared ring from its own cursor;
* optional per-model learning rates (``lrs``) for sweeps.

Every model follows the single-model path (``FusedAE.train_minibatches``): for
M <= #CUs the fleet kernel is the same instantiation with a per-workgroup pointer
rebase, so a model trained in a fleet is bit-identical to the same model trained
alone; the two-per-CU build agrees to fp32 rounding (<= 3e-8 measured) and with the
torch Keras-Adam oracle (``tests/test_ae_fleet_gpu.py``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from ._ext import load_c
from .ae import NPARAM, AESpec, FusedAE, pack_image, unpack_image


def _fnv1a(key) -> int:
    b = key.encode() if isinstance(key, str) else bytes(key)
    h = 0xCBF29CE484222325
    for c in b:
        h ^= c
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _groups_by_key(keys, n_models):
    keys = np.asarray(keys)
    uniq, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    order = np.argsort(first)
    if n_models is None:
        rank = np.empty(len(uniq), np.int64)
        rank[order] = np.arange(len(uniq))
        model_of_row = rank[inv]
        members = [[uniq[j].item()] for j in order]
    else:
        if n_models < 1:
            raise ValueError("n_models must be >= 1")
        mk = np.array([_fnv1a(str(k)) % n_models for k in uniq], np.int64)
        model_of_row = mk[inv]
        members = [[uniq[j].item() for j in order if mk[j] == b] for b in range(n_models)]
        empty = [b for b in range(n_models) if not members[b]]
        if empty:
            raise ValueError(f"models {empty[:8]} receive no keys: use fewer models or n_models=None")
    return [np.flatnonzero(model_of_row == b) for b in range(len(members))], members


def rings_by_key(raw: np.ndarray, keys, batch: int = 32, n_models: Optional[int] = None):
    """Route a keyed stream to per-model rings: ``(rings [M, R, D] float32, members)``.

    ``n_models=None``: one model per distinct key (``members[b] = [key]``, keys in order
    of first appearance -- e.g. one anomaly model per car of the reference's
    ``testdata/car-sensor-data.csv``).  Otherwise key -> model ``fnv1a(key) % n_models``
    (the same stable hash as ``parallel.dp.shard_by_key`` for ``str`` keys; other keys
    are hashed as ``str(key)``), so a key always lands on the same model across restarts
    and hosts.  Each model's rows keep stream order; a ring is the longest group rounded
    up to a multiple of ``batch``, and shorter groups are repeated cyclically to fill it,
    so every model takes the same number of steps per pass.  Memory is therefore
    ``M x longest group`` and small groups are replayed (oversampled) -- use
    :func:`ragged_rings_by_key` + ``AEFleet.attach_ragged`` when group sizes differ a lot.
    """
    raw = np.asarray(raw, dtype=np.float32)
    keys = np.asarray(keys)
    if raw.ndim != 2 or len(keys) != raw.shape[0]:
        raise ValueError("raw must be [n, D] with one key per row")
    groups, members = _groups_by_key(keys, n_models)
    M = len(members)
    R = -(-max(len(g) for g in groups) // batch) * batch
    rings = np.empty((M, R, raw.shape[1]), np.float32)
    for b, g in enumerate(groups):
        rings[b] = raw[np.resize(g, R)]          # cyclic repeat of the group's rows
    return rings, members


def ragged_rings_by_key(raw: np.ndarray, keys, batch: int = 32, n_models: Optional[int] = None):
    """Like :func:`rings_by_key`, without padding every model to the largest group:
    ``(flat [sum R_b, D] float32, table [M, 2] int64 {first row, ring rows R_b}, members)``.
    ``R_b`` is model b's row count rounded up to a multiple of ``batch`` (at most
    ``batch - 1`` rows repeated), so memory is the stream's size and one epoch of model b
    is ``R_b / batch`` steps -- no model replays its rows more often than another."""
    raw = np.asarray(raw, dtype=np.float32)
    if raw.ndim != 2 or len(np.asarray(keys)) != raw.shape[0]:
        raise ValueError("raw must be [n, D] with one key per row")
    groups, members = _groups_by_key(keys, n_models)
    lens = [-(-len(g) // batch) * batch for g in groups]
    table = np.zeros((len(groups), 2), np.int64)
    table[:, 1] = lens
    table[1:, 0] = np.cumsum(lens)[:-1]
    flat = np.empty((int(sum(lens)), raw.shape[1]), np.float32)
    for b, g in enumerate(groups):
        flat[table[b, 0]:table[b, 0] + lens[b]] = raw[np.resize(g, lens[b])]
    return flat, table, members


class AEFleet:
    """M independent autoencoders of one architecture, trained concurrently."""

    def __init__(self, spec: AESpec, weights: Sequence[Sequence[np.ndarray]], device,
                 lr=1e-3, beta_1: float = 0.9, beta_2: float = 0.999, epsilon: float = 1e-7,
                 want_acc: bool = True, scale: Optional[np.ndarray] = None, shift: Optional[np.ndarray] = None):
        spec.check_fused()
        if len(weights) == 0:
            raise ValueError("a fleet needs at least one model")
        self.C = load_c()
        self.spec = spec
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("AEFleet runs on a ROCm device only")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.n_models = M = len(weights)
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon
        self.want_acc = want_acc
        dev = self.device
        self.params = torch.from_numpy(np.stack([pack_image(w) for w in weights])).to(dev)
        self.m = torch.zeros(M, NPARAM, device=dev)
        self.v = torch.zeros(M, NPARAM, device=dev)
        self.iter = torch.zeros(M, dtype=torch.int64, device=dev)
        self.cursor = torch.zeros(M, dtype=torch.int64, device=dev)
        self.metrics = torch.zeros(M, 4, device=dev)
        if np.ndim(lr) == 0:
            self.lr, self.lrs = float(lr), None
        else:
            lrs = np.asarray(lr, dtype=np.float32)
            if lrs.shape != (M,):
                raise ValueError(f"lr must be a scalar or [{M}] per-model rates")
            self.lr, self.lrs = float(lrs[0]), torch.from_numpy(lrs).to(dev)
        if scale is None:
            self.scale = self.shift = None
        else:
            self.scale = torch.as_tensor(np.asarray(scale, dtype=np.float32), device=dev)
            self.shift = torch.as_tensor(np.asarray(shift, dtype=np.float32), device=dev)
        self.ring: Optional[torch.Tensor] = None
        self.ring_batch = 0
        self.ragged: Optional[torch.Tensor] = None

    @classmethod
    def from_seeds(cls, spec: AESpec, seeds: Sequence[int], device, **kw) -> "AEFleet":
        from ..models.reference import init_dense_weights
        return cls(spec, [init_dense_weights(spec.layer_sizes, seed=int(s)) for s in seeds], device, **kw)

    # -- data ------------------------------------------------------------------------
    def attach_rings(self, rings: torch.Tensor, batch: int, offsets: Optional[Sequence[int]] = None) -> None:
        """``rings``: ``[M, ring, ld]`` (model ``b`` consumes ``rings[b]``) or ``[ring, ld]``
        shared by every model, each from its own start row ``offsets[b]`` (multiples of
        ``batch``; default 0)."""
        M, D = self.n_models, self.spec.input_dim
        if rings.device != self.device or rings.dtype != torch.float32 or rings.stride(-1) != 1:
            raise ValueError("rings must be float32 with unit column stride on " + str(self.device))
        if rings.dim() == 3:
            if rings.size(0) != M:
                raise ValueError(f"per-model rings need a leading dim of {M}")
        elif rings.dim() != 2:
            raise ValueError("rings must be [M, ring, ld] or [ring, ld]")
        n = rings.size(-2)
        if rings.size(-1) < D:
            raise ValueError("rings have too few columns")
        if batch <= 0 or batch > self.C.ae_minibatch_max_batch() or n % batch:
            raise ValueError(f"batch must be in [1, {self.C.ae_minibatch_max_batch()}] and divide the ring rows")
        offs = np.zeros(M, np.int64) if offsets is None else np.asarray(offsets, dtype=np.int64)
        if offs.shape != (M,) or (offs % batch).any() or (offs < 0).any() or (offs >= n).any():
            raise ValueError("offsets must be [M] multiples of the batch inside the ring")
        self.ring, self.ring_batch = rings, int(batch)
        self.ragged = None
        self.cursor.copy_(torch.from_numpy(offs))

    def attach_ragged(self, flat: torch.Tensor, batch: int, table) -> None:
        """Models of different sizes in one flat row array (:func:`ragged_rings_by_key`):
        model b's ring is ``flat[table[b, 0] : table[b, 0] + table[b, 1]]``."""
        M = self.n_models
        table = np.asarray(table, dtype=np.int64)
        if table.shape != (M, 2) or (table[:, 1] % batch).any() or (table[:, 1] < batch).any():
            raise ValueError(f"table must be [{M}, 2] {{first row, ring rows (multiple of the batch)}}")
        if flat.dim() != 2 or table[:, 0].min() < 0 or (table[:, 0] + table[:, 1]).max() > flat.size(0):
            raise ValueError("table rows outside the flat array")
        if batch <= 0 or batch > self.C.ae_minibatch_max_batch():
            raise ValueError(f"batch must be in [1, {self.C.ae_minibatch_max_batch()}]")
        self.ring, self.ring_batch = flat, int(batch)
        self._ragged_table = table
        self.ragged = torch.zeros((M, 3), dtype=torch.int64, device=self.device)
        self.cursor.zero_()

    def epoch_steps(self) -> np.ndarray:
        """Steps of one pass over each model's own rows (ragged) or the shared ring length."""
        if self.ragged is not None:
            return self._ragged_table[:, 1] // self.ring_batch
        return np.full(self.n_models, self.ring.size(-2) // self.ring_batch)

    def train_epoch(self, epochs: int = 1) -> None:
        """Every model passes ``epochs`` times over its OWN rows (ragged: own step count)."""
        steps = self.epoch_steps() * int(epochs)
        if self.ragged is None:
            self.train_minibatches(int(steps[0]))
            return
        t = np.concatenate([self._ragged_table, steps[:, None]], axis=1)
        self.ragged.copy_(torch.from_numpy(np.ascontiguousarray(t)))
        self._launch(max(int(steps.max()), 1), ragged=self.ragged)

    # -- training ----------------------------------------------------------------------
    def train_minibatches(self, nsteps: int, dp=None) -> None:
        """``nsteps`` Keras steps of ``ring_batch`` rows for EVERY model, in one launch.

        ``dp``: a :meth:`~streamml.parallel.p2p.P2PGroup.local` group of ``n_models`` ranks --
        the models are then data-parallel REPLICAS of one model (workgroup b = rank b, each
        on its own data): every step's gradient is summed over the replicas on chip before
        Adam (global batch = models x batch), and the replicas stay bit-identical."""
        if self.ring is None:
            raise RuntimeError("attach_rings() first")
        B = self.ring_batch
        kw, gscale = {}, 1.0 / B
        if dp is not None:
            if not dp.in_launch or dp.world != self.n_models:
                raise ValueError("in-launch data parallelism needs P2PGroup.local(device, n_models)")
            # the replicas spin-wait for each other inside ONE launch: every workgroup must be
            # resident at once, or the resident ones wait for ones that never start.  One
            # workgroup per CU is always resident (the kernel's LDS/VGPR budget admits >= 1),
            # so cap the replicas at the CU count rather than trusting the occupancy query.
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            if dp.world > cus:
                raise ValueError(f"in-launch DP with {dp.world} replicas > {cus} CUs: not all replicas can be "
                                 "resident at once (use one process per GPU for more ranks)")
            it0 = int(self.iter[0].item())
            kw = dp.kernel_args(it0)
            gscale = 1.0 / (B * dp.world)
        if self.ragged is not None:
            if dp is not None:
                raise ValueError("ragged fleets are independent models (no data parallelism)")
            t = self._ragged_table
            self.ragged.copy_(torch.from_numpy(np.concatenate(
                [t, np.full((self.n_models, 1), int(nsteps), np.int64)], axis=1)))
            self._launch(int(nsteps), ragged=self.ragged)
            return
        self._launch(int(nsteps), gscale=gscale, **kw)
        if dp is not None:
            dp.note_iter(it0 + int(nsteps) - 1)
            dp.check()

    def _launch(self, nsteps: int, gscale: Optional[float] = None, ragged=None, **kw) -> None:
        B = self.ring_batch
        self.C.ae_train_minibatches(self.ring, self.cursor, self.scale, self.shift, self.params, self.m, self.v,
                                    self.iter, self.metrics, B, int(nsteps), self.spec.dims, self.spec.act_codes,
                                    float(self.spec.activity_l1), self.lr, self.beta_1, self.beta_2, self.epsilon,
                                    1.0 / B if gscale is None else gscale, bool(self.want_acc), None, self.lrs,
                                    ragged=ragged, **kw)

    # -- state -------------------------------------------------------------------------
    def get_weights(self, i: int) -> List[np.ndarray]:
        return unpack_image(self.params[i].detach().cpu().numpy(), self.spec)

    def set_weights(self, i: int, weights: Sequence[np.ndarray]) -> None:
        self.params[i].copy_(torch.from_numpy(pack_image(weights)))

    def model(self, i: int, **kw) -> FusedAE:
        """Model ``i`` as a standalone ``FusedAE`` (weights, Adam state and iteration
        copied), e.g. to score a car's events with ``forward`` / the serving path."""
        ae = FusedAE(self.spec, self.get_weights(i), self.device, lr=float(self.lrs[i]) if self.lrs is not None
                     else self.lr, beta_1=self.beta_1, beta_2=self.beta_2, epsilon=self.epsilon,
                     want_acc=self.want_acc, scale=None if self.scale is None else self.scale.cpu().numpy(),
                     shift=None if self.shift is None else self.shift.cpu().numpy(), **kw)
        ae.m.copy_(self.m[i])
        ae.v.copy_(self.v[i])
        ae.iter.copy_(self.iter[i:i + 1])
        return ae

    def reset_metrics(self) -> None:
        self.metrics.zero_()

    def read_metrics(self) -> List[dict]:
        """Per-model epoch metrics in Keras terms (one host sync for the whole fleet)."""
        D, l1 = self.spec.input_dim, self.spec.activity_l1
        out = []
        for sq, ab, corr, rows in self.metrics.cpu().tolist():
            rows = max(rows, 1.0)
            out.append({"loss": (sq / D + l1 * ab) / rows, "mse": sq / (D * rows), "accuracy": corr / rows,
                        "rows": rows})
        return out
