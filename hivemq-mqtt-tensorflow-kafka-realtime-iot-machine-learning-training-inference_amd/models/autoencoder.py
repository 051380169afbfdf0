"""Dense autoencoder with a Keras-like API (compile / fit / predict / evaluate / save / load).

Reference model (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:176-222):

    Input(18) -> Dense(14, tanh, activity_regularizer=L1(1e-7)) -> Dense(7, relu)
              -> Dense(7, tanh) -> Dense(18, relu)
    compile(metrics=['accuracy'], loss='mean_squared_error', optimizer='adam')
    fit(zip((x, x)).batch(100).take(100), epochs=20, verbose=2); save('model1.h5')

(the creditcard notebooks use the same stack with D = 30).  On a ROCm device
every step runs the fused HIP train kernel (:mod:`streamml.ops.ae`); on CPU the
torch reference (:mod:`streamml.models.reference`) with identical semantics.
Raw sensor rows can be fed directly: ``input_normalizer="cardata"`` applies the
reference ``normalize_fn`` inside the kernel's first load.
"""
from __future__ import annotations

import math
import os
import sys
import time
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..ckpt import h5 as ckh5
from ..data.cardata import normalize_affine
from ..nn import keras_config as kc
from ..nn.callbacks import Callback, History
from ..obs.metrics import ENGINE
from ..ops.ae import AESpec, FusedAE
from .reference import TorchAE, init_dense_weights


class _RowStage:
    """Rows of a stream staged for whole batches: a preallocated [cap, D] buffer on the
    training device (grown geometrically; no per-chunk concatenation), consumed from the
    front."""

    def __init__(self, D: int, device: torch.device, cap: int):
        self.buf = torch.empty((int(cap), D), dtype=torch.float32, device=device)
        self.n = 0

    def push(self, x: torch.Tensor) -> None:
        k = int(x.size(0))
        if self.n + k > self.buf.size(0):
            bigger = torch.empty((max(2 * self.buf.size(0), self.n + k), self.buf.size(1)), dtype=torch.float32,
                                 device=self.buf.device)
            bigger[:self.n].copy_(self.buf[:self.n])
            self.buf = bigger
        self.buf[self.n:self.n + k].copy_(x[:, :self.buf.size(1)])
        self.n += k

    def rows(self, k: int) -> torch.Tensor:
        return self.buf[:k]

    def drop(self, k: int) -> None:
        rest = self.n - k
        if rest > 0:
            self.buf[:rest].copy_(self.buf[k:self.n].clone())
        self.n = max(rest, 0)


def _resolve_device(device) -> torch.device:
    if device in (None, "auto"):
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(device)


class Autoencoder:
    def __init__(self, input_dim: int = 18, encoding_dim: int = 14, hidden_dim: int = 7,
                 activations: Sequence[str] = ("tanh", "relu", "tanh", "relu"), activity_l1: float = 1e-7,
                 device="auto", seed: int = 0, layer_names: Optional[Sequence[str]] = None,
                 input_normalizer: Optional[str] = None, name: str = "model", max_blocks: Optional[int] = None):
        self.spec = AESpec(input_dim, encoding_dim, hidden_dim, tuple(activations), activity_l1)
        self.device = _resolve_device(device)
        self.name = name
        self.layer_names = list(layer_names or ["input_1", "dense", "dense_1", "dense_2", "dense_3"])
        self.weight_names = [f"{n}/{w}:0" for n in self.layer_names[1:] for w in ("kernel", "bias")]
        self.input_normalizer = input_normalizer
        self.max_blocks = max_blocks
        self.hp = dict(lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7)
        self.loss, self.metrics = "mean_squared_error", ["accuracy"]
        self._weights = init_dense_weights(self.spec.layer_sizes, seed=seed)
        self._backend = None
        self._opt_state = None
        self.stop_training = False
        self.compiled = False

    # ------------------------------------------------------------------ setup
    def _normalizer(self):
        if self.input_normalizer in (None, "none"):
            return None, None
        if self.input_normalizer == "cardata":
            if self.spec.input_dim != 18:
                raise ValueError("cardata normaliser needs input_dim 18")
            return normalize_affine()
        raise ValueError(f"unknown input_normalizer {self.input_normalizer!r}")

    def compile(self, optimizer="adam", loss="mean_squared_error", metrics=("accuracy",), learning_rate=None,
                minibatch_precision: Optional[str] = None, **adam_kw) -> "Autoencoder":
        """Keras ``compile``.  ``minibatch_precision`` picks the small-batch (Keras batch <= 128)
        trainer's contraction precision: ``"fp32"`` (Keras-exact) or ``"bf16"`` (bf16 MFMA forward /
        activation gradients, fp32 weight gradients, master weights and Adam); None (default) takes
        the process default (``SML_MB_BF16=1``: bf16, else fp32).  The choice is passed to this
        model's launches as an argument, so models of different precision can share a process."""
        if minibatch_precision not in (None, "fp32", "bf16"):
            raise ValueError("minibatch_precision must be 'fp32', 'bf16' or None")
        self.minibatch_precision = minibatch_precision
        if str(optimizer).lower() != "adam":
            raise ValueError("only the Adam optimizer is implemented (the reference uses 'adam')")
        if loss not in ("mean_squared_error", "mse"):
            raise ValueError("only mean_squared_error is implemented (the reference loss)")
        self.loss, self.metrics = "mean_squared_error", list(metrics)
        if learning_rate is not None:
            self.hp["lr"] = float(learning_rate)
        self.hp.update({k: float(v) for k, v in adam_kw.items() if k in ("beta_1", "beta_2", "epsilon")})
        self._build()
        self.compiled = True
        return self

    def _build(self) -> None:
        weights = self.get_weights() if self._backend is not None else self._weights
        opt = self._backend.get_optimizer_state() if self._backend is not None else self._opt_state
        sc, sh = self._normalizer()
        if self.device.type == "cuda":
            self._backend = FusedAE(self.spec, weights, self.device, max_blocks=self.max_blocks,
                                    want_acc="accuracy" in self.metrics, scale=sc, shift=sh, **self.hp)
            prec = getattr(self, "minibatch_precision", None)
            self._backend.minibatch_bf16 = None if prec is None else prec == "bf16"
        else:
            self._backend = TorchAE(self.spec.layer_sizes, self.spec.activations, self.spec.activity_l1, weights,
                                    device=self.device, **self.hp)
            self._cpu_norm = (sc, sh)
        if opt is not None:
            self._backend.set_optimizer_state(*opt)

    @property
    def backend(self):
        if self._backend is None:
            self._build()
        return self._backend

    # ------------------------------------------------------------------ weights
    def get_weights(self) -> List[np.ndarray]:
        return self._backend.get_weights() if self._backend is not None else [w.copy() for w in self._weights]

    def set_weights(self, weights: Sequence[np.ndarray]) -> None:
        self._weights = [np.asarray(w, np.float32).copy() for w in weights]
        if self._backend is not None:
            self._backend.set_weights(self._weights)

    @property
    def iterations(self) -> int:
        if self._backend is None:
            return int(self._opt_state[0]) if self._opt_state else 0
        return int(self._backend.get_optimizer_state()[0])

    def count_params(self) -> int:
        return self.spec.n_params

    def summary(self, print_fn=print) -> str:
        lines = [f'Model: "{self.name}"', "_" * 65, f"{'Layer (type)':<29}{'Output Shape':<22}{'Param #':>10}",
                 "=" * 65, f"{self.layer_names[0] + ' (InputLayer)':<29}{str((None, self.spec.input_dim)):<22}{0:>10}"]
        for n, (i, o) in zip(self.layer_names[1:], self.spec.layer_sizes):
            lines.append(f"{n + ' (Dense)':<29}{str((None, o)):<22}{i * o + o:>10}")
        lines += ["=" * 65, f"Total params: {self.count_params():,}", f"Trainable params: {self.count_params():,}",
                  "Non-trainable params: 0", "_" * 65]
        text = "\n".join(lines)
        if print_fn:
            print_fn(text)
        return text

    # ------------------------------------------------------------------ data helpers
    def _to_device(self, x) -> torch.Tensor:
        if isinstance(x, torch.Tensor):
            t = x.to(self.device, torch.float32)
        else:
            t = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32), device=self.device)
        return t.contiguous()

    def _cpu_x(self, x) -> torch.Tensor:
        x = x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x, np.float32)
        sc, sh = self._cpu_norm
        if sc is not None:
            x = x * sc + sh
        return torch.as_tensor(np.asarray(x, np.float32))

    def _dist(self):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return dist.get_rank(), dist.get_world_size()
        return 0, 1

    # ------------------------------------------------------------------ training
    def fit(self, x=None, y=None, epochs: int = 1, batch_size: int = 32, verbose: int = 1,
            callbacks: Optional[Sequence[Callback]] = None, validation_data=None, shuffle: bool = True,
            steps_per_epoch: Optional[int] = None, seed: int = 0, initial_epoch: int = 0,
            engine: str = "auto", dp: str = "auto") -> History:
        """Train on an array (``y`` must be ``x`` or None: autoencoder) or a Stream.

        ``engine``: ``"persistent"`` runs every Keras step of an epoch on the persistent
        small-batch kernel (``ae_minibatch.hip``: one launch per up to 16k steps, fp32,
        batch <= 128 -- the reference's batch 32 and cardata-v3's batch 100,
        cardata-v3.py:176-177, 212-222); ``"throughput"`` is the large-batch mode (SURVEY.md
        7.3 step 7): each epoch's rows -- shuffled by a device permutation fused into the
        pack -- are tile-packed once (K8: normalize_fn + argmax(x)) and every full batch runs
        the headline kernel (packed-pair bf16 MFMA train + slab-reduce/Adam, ``step_ring``),
        the short last batch the plain fused step; ``"launch"`` issues the two-launch fused
        step per batch with in-kernel normalisation, for any batch size; ``"auto"`` picks
        ``persistent`` on a single ROCm replica when the batch fits, else ``throughput``.

        Under ``torch.distributed`` every rank trains on its own shard: arrays are split
        contiguously by rank; a Stream must be rank-sharded already -- ``data.stream.kafka(...,
        shard="auto")`` gives every rank its own offset ranges of the topic's partitions
        (:mod:`streamml.kafka.assign`) -- and every row of every rank's share is trained exactly
        once (:meth:`_fit_stream_dp`); the global batch is ``batch_size * world_size``.  ``dp``
        picks the gradient exchange:

        * ``"p2p"`` -- inside the persistent kernel, every Keras step (xGMI push of the
          gradient tile to every peer + rank-order sum, :mod:`streamml.parallel.p2p`);
          ranks agree on the step count per launch (full batches only);
        * ``"rccl"`` -- the launch-per-step path with one flat RCCL all-reduce per step;
        * ``"local_sgd:K"`` -- documented semantics change: K
          independent persistent-kernel steps per rank, then the parameters are averaged;
        * ``"auto"`` -- ``p2p`` when the persistent kernel applies and the IPC exchange can
          be set up on every rank, else ``rccl``;
        * ``"none"`` -- this process trains alone on all of ``x`` even inside a process group
          (no collective is called: e.g. a measurement on one rank while the others idle).
        """
        from ..data.stream import Stream
        from ..parallel.dp import allreduce_sum_

        if not self.compiled:
            self.compile()
        if y is not None and y is not x:
            raise ValueError("autoencoder fit expects y == x (or y=None)")
        rank, world = (0, 1) if dp == "none" else self._dist()
        allreduce = allreduce_sum_ if world > 1 else None
        hist = History()
        cbs = [hist] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
        self.stop_training = False
        be = self.backend
        for cb in cbs:
            cb.on_train_begin()
        is_stream = isinstance(x, Stream)
        if is_stream and world > 1 and x.shard is None:
            import warnings
            warnings.warn("fit(stream) under data parallelism with a stream that is not rank-sharded: every rank "
                          "trains on the same records (build it with data.stream.kafka(..., shard='auto'))")
        if not is_stream:
            on_dev = isinstance(x, torch.Tensor) and x.device == self.device and self.device.type == "cuda"
            arr = x.detach() if on_dev else (x.detach().cpu().numpy() if isinstance(x, torch.Tensor)
                                              else np.asarray(x, np.float32))
            if world > 1:
                from ..parallel.dp import shard_range
                s0, s1 = shard_range(len(arr), rank, world)
                arr = arr[s0:s1]
            # device arrays stay on the device (no host round trip)
            xd = self._to_device(arr) if self.device.type == "cuda" else self._cpu_x(arr)
        from ..parallel.fault import maybe_inject, maybe_inject_range
        persistent = self._use_persistent(engine, batch_size, world, dp)
        throughput = not persistent and self._use_throughput(engine, batch_size)
        exch, local_k = None, 0
        if persistent and world > 1:
            exch, local_k = self._dp_setup(dp)
            if exch is None and not local_k:
                persistent = False   # p2p unavailable on some rank: RCCL launch path
        self.last_fit_engine = ("persistent" if persistent else "throughput" if throughput else
                                ("launch" if self.device.type == "cuda" else "torch-cpu"))
        if persistent and world > 1:
            self.last_fit_engine += "+p2p" if exch is not None else f"+local_sgd:{local_k}"
        gstep = int(getattr(self, "_global_step", 0))
        # Nothing reads an epoch's logs before the fit returns (no progress output, no user
        # callback, no validation, one replica): snapshot the device metric accumulators per
        # epoch and read them all once at the end, so consecutive epochs queue back to back
        # instead of draining the GPU for a host read after each one.
        defer = (verbose == 0 and not callbacks and validation_data is None and world == 1
                 and self.device.type == "cuda" and hasattr(be, "metrics_from"))
        pending = []
        for epoch in range(initial_epoch, epochs):
            rng = np.random.default_rng([seed, rank, epoch])   # epoch-keyed: a resumed run reshuffles identically
            t0 = time.perf_counter()
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            be.reset_metrics()
            steps = 0
            if is_stream and world > 1:
                steps = self._fit_stream_dp(x, batch_size, steps_per_epoch, exch, local_k, persistent=persistent,
                                            world=world, allreduce=allreduce, gstep=gstep, rank=rank)
                gstep += steps
            elif persistent and is_stream:
                steps = self._fit_stream_persistent(x, batch_size, steps_per_epoch, gstep, rank)
                gstep += steps
            elif persistent:
                n = len(xd)
                nb = math.ceil(n / batch_size)
                if world > 1:   # every rank runs the same number of full batches
                    from ..parallel.dp import agree
                    nb = agree([n // batch_size], self.device)[0]
                if steps_per_epoch is not None:
                    nb = min(nb, steps_per_epoch)
                xs = xd[self._device_perm(n, seed, rank, epoch)] if shuffle else xd
                maybe_inject_range(gstep, gstep + nb, rank)   # injection points, before the epoch's launches
                if world > 1:
                    steps = self._dp_train(xs[:nb * batch_size], batch_size, exch, local_k)
                else:
                    steps, _ = be.train_rows(xs[:min(n, nb * batch_size)], batch_size)
                gstep += steps
            elif throughput and is_stream:
                steps = self._fit_stream_throughput(x, batch_size, steps_per_epoch, world, allreduce, gstep, rank)
                gstep += steps
            elif throughput:
                steps = self._fit_array_throughput(xd, batch_size, steps_per_epoch, shuffle, seed, rank, epoch, world,
                                                   allreduce, gstep, epochs_left=epochs - epoch)
                gstep += steps
            elif is_stream:
                for xb in self._stream_batches(x, batch_size):
                    if steps_per_epoch is not None and steps >= steps_per_epoch:
                        break
                    maybe_inject(gstep, rank)
                    be.step(xb, global_batch=len(xb) * world, allreduce=allreduce)
                    steps += 1
                    gstep += 1
            else:
                n = len(xd)
                order = None
                if shuffle:
                    order = (self._device_perm(n, seed, rank, epoch) if xd.device.type == "cuda"
                             else torch.as_tensor(rng.permutation(n), device=xd.device))
                nb = math.ceil(n / batch_size)
                if steps_per_epoch is not None:
                    nb = min(nb, steps_per_epoch)
                xs = xd[order] if order is not None else xd
                for b in range(nb):
                    xb = xs[b * batch_size:(b + 1) * batch_size]
                    maybe_inject(gstep, rank)
                    be.step(xb, global_batch=len(xb) * world, allreduce=allreduce)
                    steps += 1
                    gstep += 1
            self._global_step = gstep
            if defer:
                pending.append((epoch, steps, time.perf_counter() - t0, be.metrics.clone()))
                continue
            m = be.read_metrics()
            if world > 1:
                from ..parallel.dp import reduce_metrics
                m = reduce_metrics(m, self.device)
            logs = {"loss": m["loss"]}
            if "accuracy" in self.metrics:
                logs["accuracy"] = m["accuracy"]
            if validation_data is not None:
                vx = validation_data[0] if isinstance(validation_data, (tuple, list)) else validation_data
                vl, va = self.evaluate(vx, batch_size=max(batch_size, 65536), verbose=0)
                logs["val_loss"] = vl
                if "accuracy" in self.metrics:
                    logs["val_accuracy"] = va
            dt = time.perf_counter() - t0
            logs["_seconds"] = dt
            logs["_rows"] = m["rows"]
            ENGINE.train_rows.inc(m["rows"], model=self.name)
            ENGINE.train_steps.inc(steps, model=self.name)
            if steps:
                ENGINE.train_step_latency.observe(dt / steps * 1e6, model=self.name)
            ENGINE.epoch_loss.set(m["loss"], model=self.name)
            if verbose and rank == 0:
                shown = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items() if not k.startswith("_"))
                if verbose == 2:
                    print(f"Epoch {epoch + 1}/{epochs}\n{steps} steps - {dt:.2f}s - {shown}", flush=True)
                else:
                    print(f"Epoch {epoch + 1}/{epochs} - {shown}", flush=True)
            for cb in cbs:
                cb.on_epoch_end(epoch, {k: v for k, v in logs.items()})
            if self.stop_training:
                break
        if pending:   # one host read for every deferred epoch
            snaps = torch.stack([p[3] for p in pending]).cpu()
            for (epoch, steps, dt, _), row in zip(pending, snaps):
                m = be.metrics_from(row)
                logs = {"loss": m["loss"]}
                if "accuracy" in self.metrics:
                    logs["accuracy"] = m["accuracy"]
                logs["_seconds"] = dt   # enqueue time of the epoch (its kernels ran asynchronously)
                logs["_rows"] = m["rows"]
                ENGINE.train_rows.inc(m["rows"], model=self.name)
                ENGINE.train_steps.inc(steps, model=self.name)
                ENGINE.epoch_loss.set(m["loss"], model=self.name)
                for cb in cbs:
                    cb.on_epoch_end(epoch, dict(logs))
        for cb in cbs:
            cb.on_train_end()
        return hist

    def _device_perm(self, n: int, seed: int, rank: int, epoch: int) -> torch.Tensor:
        """Epoch shuffle generated on the device (deterministic in (seed, rank, epoch), so a
        resumed run reshuffles identically) -- no host permutation, no H2D of indices."""
        g = torch.Generator(device=self.device)
        g.manual_seed((int(seed) * 1_000_003 + int(rank) * 7_919 + int(epoch)) & 0x7FFFFFFFFFFF)
        return torch.randperm(n, generator=g, device=self.device)

    def _use_throughput(self, engine: str, batch_size: int) -> bool:
        if self.device.type != "cuda":
            if engine == "throughput":
                raise ValueError("engine='throughput' needs a ROCm device")
            return False
        if engine == "throughput":
            return True
        return engine == "auto" and batch_size > self.backend.max_minibatch()

    # rows trained once: the direct fused step (packed pairs straight from the raw rows,
    # normalize_fn + argmax(x) in registers) takes 0.75 ms per 33.5 M rows against 1.04 (K8
    # pack) + 0.695 (packed-pair kernel on the packed ring) -- the pack pays off only from
    # ~19 passes over the same rows (profiles/r05/SUMMARY.md; with r03's one-tile direct
    # loop, 0.97 ms, it was 3)
    PACK_MIN_PASSES = 18
    # ... but the direct step only runs on packed pairs when the launcher's predicate holds
    # (ae_fused.hip: the reference model at D = 18, a batch of whole 32-row pairs, the default
    # loop); otherwise it is the one-tile direct loop (0.97 ms), whose break-even is ~3 passes
    PACK_MIN_PASSES_ONE_TILE = 3

    def _direct_pairs(self, B: int) -> bool:
        sp = self.spec
        return (sp.input_dim == 18 and sp.encoding_dim <= 15 and sp.hidden_dim <= 7 and B % 32 == 0
                and tuple(sp.activations) == ("tanh", "relu", "tanh", "relu")
                and os.environ.get("SML_AE_DIRECT_PAIRS", "1") != "0"
                and os.environ.get("SML_AE_ILP", "3") not in ("1", "2"))

    def pack_min_passes(self, B: int) -> int:
        """Passes over the same rows from which packing them once beats the direct step."""
        return self.PACK_MIN_PASSES if self._direct_pairs(B) else self.PACK_MIN_PASSES_ONE_TILE

    def _fit_array_throughput(self, xd: torch.Tensor, B: int, steps_per_epoch: Optional[int], shuffle: bool,
                              seed: int, rank: int, epoch: int, world: int, allreduce, gstep: int,
                              epochs_left: int = 1) -> int:
        """One epoch of the throughput engine over a device array: every full batch on the
        headline kernel from the epoch's tile-packed ring (shuffled epochs: the permutation
        is evaluated inside the pack kernel; unshuffled epochs reuse the packed ring of the
        previous one), or -- unshuffled, fewer than PACK_MIN_PASSES epochs left and no packed
        ring yet -- on the direct fused step over the rows in place; the last short batch
        (Keras) on the plain fused step."""
        from ..parallel.fault import maybe_inject_range
        be = self.backend
        n = xd.size(0)
        nfull = n // B
        if world > 1:   # every rank runs the same number of full batches; no short batch
            from ..parallel.dp import agree
            nfull = agree([nfull], self.device)[0]
        if steps_per_epoch is not None:
            nfull = min(nfull, steps_per_epoch)
        pkey = self.shuffle_key(seed, rank, epoch) if shuffle else None
        maybe_inject_range(gstep, gstep + nfull + 1, rank)
        steps = 0
        if nfull:
            key = self.pack_key(xd, B, nfull)
            packed = pkey is None and getattr(self, "_tp_key", None) == key and be.ring_xpack is not None
            if pkey is None and not packed and epochs_left < self.pack_min_passes(B):
                for i in range(nfull):   # rows in place, normalised inside the kernel
                    be.step(xd[i * B:(i + 1) * B], global_batch=B * world, allreduce=allreduce)
            else:
                if pkey is not None:   # the epoch's shuffle evaluated inside the pack kernel
                    be.pack_ring(xd, B, perm_key=pkey) if nfull * B == (n // B) * B else \
                        be.pack_ring(xd, B, index=be.perm_indices(n, pkey, 0, nfull * B))
                    self._tp_key = None
                elif not packed:
                    be.pack_ring(xd[:nfull * B], B)
                    self._tp_key = key
                else:
                    be.cursor.zero_()
                for _ in range(nfull):
                    be.step_ring(global_batch=B * world, allreduce=allreduce)
            steps = nfull
        rem = n - nfull * B
        if rem and world == 1 and (steps_per_epoch is None or steps < steps_per_epoch) and n // B == nfull:
            tail = xd[be.perm_indices(n, pkey, nfull * B, rem)] if pkey is not None else xd[nfull * B:]
            be.step(tail.contiguous())
            steps += 1
        return steps

    @staticmethod
    def pack_key(xd: torch.Tensor, B: int, nfull: int) -> tuple:
        """Identity of the rows a tile-packed ring was built from: storage, extent, batch AND
        the tensor's version counter, so an in-place update of the same device array between
        two ``fit`` calls re-packs instead of training on the stale packed rows."""
        return (xd.data_ptr(), int(xd.size(0)), int(B), int(nfull), int(xd._version))

    @staticmethod
    def shuffle_key(seed: int, rank: int, epoch: int) -> int:
        """64-bit key of an epoch's throughput-mode shuffle (a keyed bijection evaluated in the
        pack kernel; deterministic in (seed, rank, epoch), so a resumed run reshuffles alike)."""
        import hashlib
        h = hashlib.blake2b(f"{int(seed)}:{int(rank)}:{int(epoch)}".encode(), digest_size=8).digest()
        return int.from_bytes(h, "little")

    def _fit_stream_throughput(self, stream, B: int, max_steps: Optional[int], world: int, allreduce,
                               gstep: int, rank: int, round_batches: int = 8) -> int:
        """A streaming epoch on the throughput engine.  Streamed rows are trained once, so
        every batch runs the direct fused step (normalize_fn + argmax inside the unpacked
        kernel: faster than K8 pack + packed kernel for single-pass rows, PACK_MIN_PASSES).
        One replica: a batch that lies inside one device chunk is trained in place; only a
        batch straddling chunks is assembled in a B-row carry buffer.  Under DP the ranks
        agree, per round of ``round_batches`` staged batches, on how many to train, and the
        epoch ends for everyone when any rank's stream is exhausted.  Batches are exactly
        ``batch(B)`` over the stream; the final partial batch is Keras' short batch."""
        be = self.backend
        D = self.spec.input_dim
        steps = 0

        def left():
            return None if max_steps is None else max_steps - steps

        if world == 1:
            carry = torch.empty((B, D), dtype=torch.float32, device=self.device)
            have = 0
            for xd in self._stream_device_chunks(stream):
                if max_steps is not None and steps >= max_steps:
                    break
                k, pos = xd.size(0), 0
                if have:   # complete the batch straddling the previous chunk
                    t = min(B - have, k)
                    carry[have:have + t].copy_(xd[:t])
                    have += t
                    pos = t
                    if have < B:
                        continue
                    be.step(carry, global_batch=B)
                    steps += 1
                    have = 0
                nfull = (k - pos) // B
                if left() is not None:
                    nfull = min(nfull, left())
                for i in range(nfull):
                    be.step(xd[pos + i * B:pos + (i + 1) * B], global_batch=B)
                steps += nfull
                pos += nfull * B
                if k > pos and (max_steps is None or steps < max_steps):
                    carry[:k - pos].copy_(xd[pos:])
                    have = k - pos
            if have and (max_steps is None or steps < max_steps):
                be.step(carry[:have].contiguous())   # Keras' short final batch
                steps += 1
            return steps
        # several replicas: the sharded epoch (every rank its own partitions' rows)
        return self._fit_stream_dp(stream, B, max_steps, None, 0, persistent=False, world=world,
                                   allreduce=allreduce, gstep=gstep, rank=rank, round_batches=round_batches)

    def _use_persistent(self, engine: str, batch_size: int, world: int, dp: str = "auto") -> bool:
        if engine not in ("auto", "persistent", "launch", "throughput"):
            raise ValueError(f"engine must be auto / persistent / throughput / launch, got {engine!r}")
        if engine == "throughput":
            return False
        if not (dp in ("auto", "p2p", "rccl", "none") or dp.startswith("local_sgd:")):
            raise ValueError(f"dp must be auto / p2p / rccl / local_sgd:K / none, got {dp!r}")
        if engine == "launch" or self.device.type != "cuda":
            if engine == "persistent" and self.device.type != "cuda":
                raise ValueError("engine='persistent' needs a ROCm device")
            return False
        fits = 1 <= batch_size <= self.backend.max_minibatch() and (world == 1 or dp != "rccl")
        if engine == "persistent" and not fits:
            raise ValueError(f"engine='persistent' needs batch_size <= {self.backend.max_minibatch()} and, "
                             f"under DP, dp='p2p' / 'local_sgd:K' (got batch {batch_size}, dp {dp!r})")
        return fits

    def _dp_setup(self, dp: str):
        """(P2PGroup or None, local-SGD period or 0); collective over the process group."""
        if dp.startswith("local_sgd:"):
            k = int(dp.split(":", 1)[1])
            if k < 1:
                raise ValueError("local_sgd:K needs K >= 1")
            return None, k
        if getattr(self, "_p2p", None) is None:
            from ..parallel.p2p import P2PGroup
            self._p2p, err = P2PGroup.try_create(self.device)
            if self._p2p is None:
                if dp == "p2p":
                    raise RuntimeError(f"dp='p2p': the IPC exchange could not be set up ({err!r})")
                import warnings
                warnings.warn(f"P2P exchange unavailable ({err!r}); falling back to RCCL per step")
        return self._p2p, 0

    def _dp_train(self, rows: torch.Tensor, B: int, exch, local_k: int) -> int:
        """Train ``len(rows) // B`` steps (the same count on every rank) under DP."""
        be = self.backend
        n = rows.size(0) // B
        if exch is not None:
            steps, _ = be.train_rows(rows[:n * B], B, dp=exch)
            return steps
        import torch.distributed as dist
        world = dist.get_world_size()
        done = 0
        while done < n:   # local SGD: K independent steps, then average the parameters
            k = min(local_k, n - done)
            be.train_rows(rows[done * B:(done + k) * B], B)
            dist.all_reduce(be.params, op=dist.ReduceOp.SUM)
            be.params.div_(world)
            done += k
        return n

    def _fit_stream_dp(self, stream, B: int, max_steps: Optional[int], exch, local_k: int, persistent: bool = True,
                       world: int = 2, allreduce=None, gstep: int = 0, rank: int = 0,
                       round_batches: int = 8) -> int:
        """One streaming epoch under data parallelism, every rank on its own share of the
        stream (``kafka(..., shard="auto")``: its own partitions' offset ranges).  Every row of
        every share is trained exactly once and every rank runs the same number of optimizer
        steps -- the contract a DP all-reduce needs, without dropping a rank's leftovers.

        Phase 1 (lockstep): each rank stages rows from its stream; per round the ranks agree
        (one all-reduce of two ints) on the full batches every rank can run, and run them --
        on the persistent kernel with the in-kernel xGMI exchange (``persistent``:
        ``_dp_train``), or one fused step + one flat all-reduce per batch (throughput /
        launch engines, and the CPU path).  Global batch ``B x world``.

        Phase 2 (tail, once any rank's stream is exhausted): the remaining rows, < B on the
        exhausted ranks and whatever is left on the others, go in steps where each rank
        contributes ``min(B, rows left)`` rows -- possibly none -- and the step's global batch
        is the agreed sum, so the update is the mean over exactly the rows trained (Keras' short
        final batch, spread over the ranks).  With ``assign="split"`` shares differ by at most a
        record (plus the label filter), so the tail is a step or two.

        ``max_steps`` (``take(n)``) caps the steps of the epoch on every rank alike."""
        from ..parallel.dp import agree
        from ..parallel.fault import maybe_inject
        be = self.backend
        D = self.spec.input_dim
        gb = B * world
        cuda = self.device.type == "cuda"

        def chunks():
            if cuda:
                yield from self._stream_device_chunks(stream)
            else:   # CPU path: the host stream (filtered there), normalised as the CPU trainer expects
                for c in stream:
                    if len(c):
                        yield self._cpu_x(c.x)

        stage = _RowStage(D, self.device, max(round_batches * B, 1 << 16))
        it = iter(chunks())
        exhausted = False
        steps = 0

        def fill(target: int) -> None:
            nonlocal exhausted
            while not exhausted and stage.n < target:
                try:
                    stage.push(next(it))
                except StopIteration:
                    exhausted = True

        def full(nb: int) -> None:   # nb full batches of B rows on every rank
            rows = stage.rows(nb * B)
            if persistent:
                self._dp_train(rows, B, exch, local_k)
                return
            for i in range(nb):
                maybe_inject(gstep + steps + i, rank)
                be.step(rows[i * B:(i + 1) * B], global_batch=gb, allreduce=allreduce)

        try:
            while True:   # phase 1
                fill(round_batches * B)
                left = None if max_steps is None else max_steps - steps
                # a rank whose stream has ended with < B rows staged can run no more full batches
                nb, any_done = agree([stage.n // B, int(exhausted and stage.n < B)], self.device, ["min", "max"])
                if left is not None:
                    nb = min(nb, left)
                if nb > 0:
                    full(nb)
                    stage.drop(nb * B)
                    steps += nb
                if any_done or (max_steps is not None and steps >= max_steps):
                    break
            while max_steps is None or steps < max_steps:   # phase 2: uneven tail
                fill(B)
                k = min(B, stage.n)
                tot = agree([k], self.device, ["sum"])[0]
                if tot == 0:
                    break
                maybe_inject(gstep + steps, rank)
                if k:
                    be.step(stage.rows(k), global_batch=tot, allreduce=allreduce)
                    stage.drop(k)
                else:
                    be.step_empty(global_batch=tot, allreduce=allreduce)
                steps += 1
        finally:
            close = getattr(it, "close", None)
            if close is not None:
                close()
        return steps

    def _stream_device_chunks(self, stream, chunk_rows: int = 1 << 16):
        """Device chunks of raw rows from a Stream (no host re-batching): the pinned ring
        moves whole chunks, a deferred ``filter_normal(device=True)`` runs as K8 on them."""
        from ..data.loader import DeviceLoader
        deferred = getattr(stream, "device_filter", None)
        base, keep = deferred if deferred is not None else (stream, None)
        feed = getattr(base, "native_feed", None)
        if feed is not None and feed.features == self.spec.input_dim:
            # native Kafka feed: decode-time label filter, slabs straight to the device
            yield from feed.device_chunks(self.device, keep_label=keep)
            return
        if deferred is not None:
            parent, keep = deferred
            yield from DeviceLoader(parent, self.device, max_rows=chunk_rows, features=self.spec.input_dim,
                                    keep_label=keep).chunks()
            return
        yield from DeviceLoader(stream, self.device, max_rows=chunk_rows, features=self.spec.input_dim).chunks()

    def _fit_stream_persistent(self, stream, B: int, max_steps: Optional[int], gstep: int, rank: int) -> int:
        """One streaming epoch on the persistent kernel.  Default: ONE launch for the whole
        epoch fed through the device ring's doorbell (``FusedAE.train_stream``: batches
        straddle chunk boundaries inside the ring, no carry copy, no launch per chunk).
        With fault injection armed (SML_FAULT_STEP) or SML_STREAM_DOORBELL=0, whole device
        chunks go to ``train_rows`` instead and the < B rows left at a chunk boundary are
        carried to the next chunk (injection needs a host point between steps).  Both give
        exactly the reference's ``batch(B)`` over the (filtered) stream; ``max_steps`` =
        ``take(n)``."""
        from ..parallel.fault import maybe_inject, maybe_inject_range
        be = self.backend
        if os.environ.get("SML_FAULT_STEP") is None and os.environ.get("SML_STREAM_DOORBELL", "1") != "0":
            maybe_inject(gstep, rank)
            steps, _ = be.train_stream(self._stream_device_chunks(stream), B, max_steps)
            return steps
        D = self.spec.input_dim
        carry = torch.empty((B, D), dtype=torch.float32, device=self.device)
        have, steps = 0, 0

        def budget():
            return None if max_steps is None else max_steps - steps

        for xd in self._stream_device_chunks(stream):
            if max_steps is not None and steps >= max_steps:
                break
            k, pos = xd.size(0), 0
            if have:   # complete the carried batch first
                t = min(B - have, k)
                carry[have:have + t].copy_(xd[:t])
                have += t
                pos = t
                if have < B:
                    continue
                maybe_inject(gstep + steps, rank)
                s, _ = be.train_rows(carry, B, max_steps=budget())
                steps += s
                have = 0
            nfull = (k - pos) // B
            if max_steps is not None:
                nfull = min(nfull, max_steps - steps)
            if nfull:
                maybe_inject_range(gstep + steps, gstep + steps + nfull, rank)
                s, _ = be.train_rows(xd[pos:pos + nfull * B], B)
                steps += s
                pos += nfull * B
            rest = k - pos
            if rest and (max_steps is None or steps < max_steps):
                carry[:rest].copy_(xd[pos:])
                have = rest
        if have and (max_steps is None or steps < max_steps):
            maybe_inject(gstep + steps, rank)
            s, _ = be.train_rows(carry[:have], B)   # Keras' short final batch
            steps += s
        return steps

    def _stream_batches(self, stream, batch_size: int):
        """Yield device (or CPU) batches of raw rows from a Stream."""
        deferred = getattr(stream, "device_filter", None)
        if deferred is not None and self.device.type == "cuda":
            # K8 on the device: unfiltered rows + labels through the ring, compaction
            # and exact re-batching on the GPU (same batches as filter -> batch(B))
            from ..data.loader import DeviceLoader
            parent, keep = deferred
            for xb, _ in DeviceLoader(parent.batch(batch_size), self.device, max_rows=batch_size,
                                      features=self.spec.input_dim, keep_label=keep, batch_rows=batch_size):
                yield xb
            return
        st = stream.batch(batch_size)
        if self.device.type == "cuda":
            from ..data.loader import DeviceLoader
            for xb, _ in DeviceLoader(st, self.device, max_rows=batch_size, features=self.spec.input_dim):
                yield xb
        else:
            for c in st:
                yield self._cpu_x(c.x)

    # ------------------------------------------------------------------ inference
    def _forward_batches(self, x, batch_size: int):
        """(first row, reconstruction, score) per batch: device tensors on ROCm (the input
        goes to the device once, outputs stay there), numpy on CPU."""
        if self.device.type == "cuda":
            xd = self._to_device(x)
            for s in range(0, xd.size(0), batch_size):
                r, sc, _ = self.backend.forward(xd[s:s + batch_size])
                yield s, r, sc
            return
        arr = x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x, np.float32)
        for s in range(0, len(arr), batch_size):
            xn = self._cpu_x(arr[s:s + batch_size])
            y = self.backend.forward(xn)
            yield s, y.numpy(), ((y - xn) ** 2).mean(dim=1).numpy()

    @staticmethod
    def _np(t):
        return t.cpu().numpy() if isinstance(t, torch.Tensor) else t

    def _collect(self, parts):
        if not parts:
            return None
        if isinstance(parts[0], torch.Tensor):
            return torch.cat(parts).cpu().numpy()   # one device -> host copy
        return np.concatenate(parts)

    def predict(self, x, batch_size: int = 32, callbacks: Optional[Sequence[Callback]] = None,
                verbose: int = 0) -> np.ndarray:
        """Reconstructions (what the reference streams to Kafka, cardata-v3.py:243-249)."""
        from ..data.stream import Stream
        if not self.compiled:
            self.compile()
        cbs = list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
        outs = []
        if isinstance(x, Stream):
            gen = (r for c in x.batch(batch_size) for r in self._forward_batches(c.x, batch_size))
        else:
            gen = self._forward_batches(x, batch_size if cbs else max(batch_size, 1 << 20))
        for bi, (_, rec, sc) in enumerate(gen):
            outs.append(rec)
            ENGINE.infer_rows.inc(len(rec), model=self.name)
            if cbs:   # the callbacks see host arrays per batch, as Keras' on_predict_batch_end
                logs = {"outputs": self._np(rec), "scores": self._np(sc)}
                for cb in cbs:
                    cb.on_predict_batch_end(bi, logs)
        for cb in cbs:
            cb.on_predict_end()
        out = self._collect(outs)
        return out if out is not None else np.zeros((0, self.spec.input_dim), np.float32)

    def score(self, x, batch_size: int = 1 << 20) -> np.ndarray:
        """Per-row reconstruction MSE = anomaly score (notebook ...ipynb:1014-1015)."""
        if not self.compiled:
            self.compile()
        return self._collect([sc for _, _, sc in self._forward_batches(x, batch_size)])

    def reconstruct_and_score(self, x, batch_size: int = 1 << 20) -> Tuple[np.ndarray, np.ndarray]:
        """Reconstructions and anomaly scores from one device pass (K12)."""
        if not self.compiled:
            self.compile()
        parts = list(self._forward_batches(x, batch_size))
        return self._collect([r for _, r, _ in parts]), self._collect([sc for _, _, sc in parts])

    def detect(self, x, threshold: float = 5.0, batch_size: int = 1 << 20) -> np.ndarray:
        """Anomaly flags with the notebook's fixed threshold (``threshold_fixed = 5``)."""
        flags = self.score(x, batch_size) > threshold
        ENGINE.anomaly_events.inc(int(flags.sum()), model=self.name)
        return flags

    def evaluate(self, x, y=None, batch_size: int = 65536, verbose: int = 0) -> Tuple[float, float]:
        """Keras ``evaluate``: (loss, accuracy) without updating weights."""
        if not self.compiled:
            self.compile()
        D = self.spec.input_dim
        if self.device.type == "cuda":
            # forward kernel with on-device metric sums: no backward, one host read
            sq, ab, corr, rows = self.backend.evaluate_sums(self._to_device(x), max(int(batch_size), 1))
            rows = max(rows, 1.0)
            return float((sq / D + self.spec.activity_l1 * ab) / rows), float(corr / rows)
        arr = x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x, np.float32)
        from .reference import ae_loss_torch
        xn = self._cpu_x(arr)
        with torch.no_grad():
            loss, _, acc = ae_loss_torch(xn, self.backend.w, self.spec.activations, self.spec.activity_l1)
        return float(loss), float(acc)

    # ------------------------------------------------------------------ persistence
    def model_config(self) -> dict:
        dense = []
        for li, (n, (_, o)) in enumerate(zip(self.layer_names[1:], self.spec.layer_sizes)):
            dense.append(kc.dense_config(n, o, self.spec.activations[li],
                                         self.spec.activity_l1 if li == 0 else None))
        return kc.functional_dense_model(self.name, self.layer_names[0], self.spec.input_dim, dense)

    def save(self, path: str, include_optimizer: bool = True) -> None:
        """Keras-compatible ``.h5`` (cardata-v3.py:227 ``autoencoder.save``)."""
        w = self.get_weights()
        layers = [(self.layer_names[0], [])]
        for li, n in enumerate(self.layer_names[1:]):
            layers.append((n, [(self.weight_names[2 * li], w[2 * li]), (self.weight_names[2 * li + 1], w[2 * li + 1])]))
        opt = None
        if include_optimizer and self._backend is not None:
            it, m, v = self._backend.get_optimizer_state()
            names = ckh5.adam_weight_names(self.weight_names)
            opt = list(zip(names, [np.array(it, dtype=np.int64)] + list(m) + list(v)))
        ckh5.save_keras_h5(path, self.model_config(),
                           layers, kc.training_config(self.hp["lr"], self.hp["beta_1"], self.hp["beta_2"],
                                                      self.hp["epsilon"], metrics=self.metrics), opt)

    @classmethod
    def load(cls, path: str, device="auto", input_normalizer: Optional[str] = None, compile: bool = True,
             **kw) -> "Autoencoder":
        """``tf.keras.models.load_model`` equivalent (cardata-v3.py:261)."""
        ck = ckh5.load_keras_h5(path)
        in_name, in_dim, dense = kc.parse_dense_model(ck.model_config)
        if len(dense) != 4:
            raise ValueError(f"expected a 4-Dense autoencoder, found {len(dense)} Dense layers")
        acts = tuple(d["activation"] for d in dense)
        l1 = 0.0
        ar = dense[0].get("activity_regularizer")
        if ar:
            l1 = float(ar["config"].get("l1", 0.0))
        units = [int(d["units"]) for d in dense]
        if units[3] != in_dim or units[1] != units[2]:
            raise ValueError(f"unsupported autoencoder shape {in_dim}->{units}")
        m = cls(in_dim, units[0], units[1], acts, l1, device=device,
                layer_names=[in_name or "input_1"] + [d["name"] for d in dense],
                input_normalizer=input_normalizer, name=ck.model_config["config"].get("name", "model"), **kw)
        # weight dataset names come from the file (quirk: dense_4 -> dense_4_1/...)
        m.weight_names = [wn for ln in m.layer_names[1:] for wn, _ in ck.weights[ln]]
        m.set_weights(ck.flat_weights())
        hp = kc.optimizer_hparams(ck.training_config)
        m.hp.update(hp)
        if ck.optimizer_weights:
            arrays = [a for _, a in ck.optimizer_weights]
            k = len(m.weight_names)
            if len(arrays) == 1 + 2 * k:
                m._opt_state = (int(np.asarray(arrays[0]).reshape(-1)[0]), arrays[1:1 + k], arrays[1 + k:])
        if compile:
            metrics = (ck.training_config or {}).get("metrics", ["accuracy"]) or []
            m.compile(metrics=metrics)
        return m


def load_model(path: str, **kw) -> Autoencoder:
    return Autoencoder.load(path, **kw)
