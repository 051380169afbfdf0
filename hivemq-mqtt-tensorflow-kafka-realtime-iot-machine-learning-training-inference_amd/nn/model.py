"""Generic Keras-style model builder: ``Sequential`` / functional ``Model`` with
compile / fit / predict / evaluate / summary / save and ``load_model``.

Reference usage: every script builds a ``tf.keras`` model,
``compile(loss=..., optimizer='adam', metrics=['accuracy'])``, ``fit`` on a
dataset, ``save('x.h5')`` and ``tf.keras.models.load_model``.  A user of the
reference can write the same code against ``streamml.nn``.

MI355X-first execution:

* all parameters of a model live in ONE flat fp32 buffer (``ops.adam.FlatParams``)
  whose ``.grad`` is one flat buffer too, so the optimizer step is a single
  ``reduce_adam`` HIP launch and data parallelism is a single RCCL all-reduce
  per step (``parallel.dp``);
* layers dispatch to the HIP ops (K1/K2 dense, fused LSTM recurrence, fused
  softmax + sparse-CE head, K13);
* **graph selection at compile time**: a dense autoencoder chain
  ``D -> a -> b -> c -> D`` (<= 31 / 15 / 15 / 15 units, MSE loss) is recognised
  and compiled onto the persistent fused AE train kernel (``ops.ae.FusedAE``:
  normalise + fwd + bwd + Adam in two launches per step) -- the same path the
  headline benchmark measures.  ``compile(fused=False)`` keeps the layer-by-layer
  engine.
* metrics accumulate on the device and are read once per epoch.
"""
from __future__ import annotations

import math
import sys
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..ckpt import h5 as ckh5
from ..nn import keras_config as kc
from ..nn.callbacks import Callback, History
from ..ops.adam import FlatAdam, FlatParams
from .layers import (LSTM, Dense, Dropout, Flatten, InputLayer, Layer, RepeatVector, TimeDistributed,
                     layer_from_config)

LOSS_ALIASES = {"mse": "mean_squared_error", "mae": "mean_absolute_error",
                "mean_squared_error": "mean_squared_error", "mean_absolute_error": "mean_absolute_error",
                "sparse_categorical_crossentropy": "sparse_categorical_crossentropy",
                "categorical_crossentropy": "categorical_crossentropy",
                "binary_crossentropy": "binary_crossentropy"}


def _resolve_device(device) -> torch.device:
    if device in (None, "auto"):
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(device)


class Adam:
    """``tf.keras.optimizers.Adam`` hyper-parameters (epsilon 1e-7 as in the reference .h5)."""

    def __init__(self, learning_rate: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, lr: Optional[float] = None):
        self.lr = float(lr if lr is not None else learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)


class optimizers:  # noqa: N801 (keras namespace spelling)
    Adam = Adam


class _SparseXent(torch.autograd.Function):
    """Fused softmax + sparse CE on the device: forward writes dlogits in the same pass."""

    @staticmethod
    def forward(ctx, logits, labels, metric_acc):
        from ..ops._ext import load_c
        B = logits.shape[0]
        d = torch.empty_like(logits)
        acc = torch.zeros(2, device=logits.device)
        load_c().softmax_xent(logits.contiguous(), labels.contiguous(), 1.0 / max(B, 1), d, None, acc)
        metric_acc[1] += acc[1]
        ctx.save_for_backward(d)
        return acc[0] / max(B, 1)

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d * g, None, None


class Model:
    """Chain model (the reference only builds chains); ``Sequential`` and the functional form share it."""

    def __init__(self, inputs: Optional[Layer] = None, outputs: Optional[Layer] = None, name: str = "model",
                 layers: Optional[Sequence[Layer]] = None, device="auto", seed: int = 0):
        self.name = name
        self.device = _resolve_device(device)
        self.seed = seed
        self.functional = layers is None
        if layers is None:
            chain = []
            node = outputs
            while node is not None:
                chain.append(node)
                node = node.inbound[0] if node.inbound else None
            chain.reverse()
            if not chain or chain[0] is not inputs:
                raise ValueError("outputs are not connected to inputs")
            layers = chain
        self.layers: List[Layer] = list(layers)
        self.fp: Optional[FlatParams] = None
        self.opt: Optional[FlatAdam] = None
        self.compiled = False
        self.stop_training = False
        self.loss = "mean_squared_error"
        self.metrics: List[str] = []
        self.hp = dict(lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7)
        self._fused = None
        self._acc = None
        self._pending_opt_state = None

    # ------------------------------------------------------------------ build
    def add(self, layer: Layer) -> None:
        if self.fp is not None:
            raise RuntimeError("cannot add layers after the model is built")
        self.layers.append(layer)

    def _input_shape(self):
        first = self.layers[0]
        if isinstance(first, InputLayer):
            return first.shape
        if first.input_shape is None:
            raise ValueError("the first layer needs input_shape=")
        return first.input_shape

    def build(self) -> None:
        if self.fp is not None:
            return
        counters: Dict[str, int] = {}

        def auto(prefix):
            k = counters.get(prefix, 0)
            counters[prefix] = k + 1
            return prefix if k == 0 else f"{prefix}_{k}"

        if self.functional and not isinstance(self.layers[0], InputLayer):
            raise ValueError("functional models start with Input()")
        shape = tuple(self._input_shape())
        rng = np.random.default_rng(self.seed)
        shapes, inits = [], []
        for lyr in self.layers:
            if lyr.name is None:
                if isinstance(lyr, InputLayer):      # Keras numbers inputs from 1: input_1
                    counters["input"] = counters.get("input", 0) + 1
                    lyr.name = f"input_{counters['input']}"
                else:
                    lyr.name = auto(lyr.prefix)
            if isinstance(lyr, TimeDistributed) and lyr.layer.name is None:
                lyr.layer.name = auto(lyr.layer.prefix)
            lyr.param_slots = []
            in_shape = shape
            if not isinstance(lyr, InputLayer):
                for (_, wshape), arr in zip(lyr.weight_specs(in_shape), lyr.init_weights(in_shape, rng)):
                    lyr.param_slots.append(len(shapes))
                    shapes.append(wshape)
                    inits.append(arr)
                shape = tuple(lyr.output_shape(in_shape))
            lyr.out_shape = shape
        self.output_shape = shape
        self.fp = FlatParams(shapes, self.device, inits)

    # ------------------------------------------------------------------ compile
    def compile(self, optimizer="adam", loss="mean_squared_error", metrics=None, fused: Optional[bool] = None,
                **kw) -> "Model":
        self.build()
        if isinstance(optimizer, Adam):
            self.hp = dict(lr=optimizer.lr, beta_1=optimizer.beta_1, beta_2=optimizer.beta_2,
                           epsilon=optimizer.epsilon)
        elif str(optimizer).lower() != "adam":
            raise ValueError("only the Adam optimizer is implemented (the reference uses 'adam')")
        if callable(loss):
            loss = getattr(loss, "__name__", "mean_squared_error")
        if loss not in LOSS_ALIASES:
            raise ValueError(f"unsupported loss {loss!r}")
        self.loss = LOSS_ALIASES[loss]
        self.metrics = list(metrics or [])
        self.opt = FlatAdam(self.fp, **self.hp)
        if self._pending_opt_state is not None:
            self.opt.load_state(*self._pending_opt_state)
            self._pending_opt_state = None
        self._acc = torch.zeros(3, device=self.device, dtype=torch.float64 if self.device.type == "cpu"
                                else torch.float32)
        self._fused = None
        if fused is None:
            fused = self.device.type == "cuda"
        if fused:
            self._fused = self._try_fuse()
        self.compiled = True
        return self

    def _ae_pattern(self):
        """Return an AESpec when the model is a 4-Dense autoencoder the fused kernel implements."""
        from ..ops.ae import AESpec
        ls = [l for l in self.layers if not isinstance(l, InputLayer)]
        if len(ls) != 4 or not all(isinstance(l, Dense) and l.use_bias for l in ls):
            return None
        if self.loss != "mean_squared_error" or len(self._input_shape()) != 1:
            return None
        D = int(self._input_shape()[0])
        n1, n2, n3, n4 = (l.units for l in ls)
        if n4 != D or n2 != n3:
            return None
        if any(l.activation not in ("linear", "relu", "tanh", "sigmoid") for l in ls):
            return None
        if any(l.activity_regularizer is not None for l in ls[1:]):
            return None
        r = ls[0].activity_regularizer
        if r is not None and r.l2:
            return None
        spec = AESpec(D, n1, n2, tuple(l.activation for l in ls), r.l1 if r is not None else 0.0)
        try:
            spec.check_fused()
        except ValueError:
            return None
        return spec

    def _try_fuse(self):
        spec = self._ae_pattern()
        if spec is None:
            return None
        from ..models.autoencoder import Autoencoder
        names = [l.name for l in self.layers]
        if not isinstance(self.layers[0], InputLayer):
            names = ["input_1"] + names
        ae = Autoencoder(spec.input_dim, spec.encoding_dim, spec.hidden_dim, spec.activations, spec.activity_l1,
                         device=self.device, layer_names=names, name=self.name)
        ae.hp = dict(self.hp)
        ae.set_weights(self.fp.get())
        ae.compile(metrics=self.metrics or (), learning_rate=self.hp["lr"])
        it, m, v = self.opt.state()
        if it:
            ae.backend.set_optimizer_state(it, m, v)
        return ae

    @property
    def fused(self) -> bool:
        return self._fused is not None

    def _sync_from_fused(self) -> None:
        if self._fused is not None:
            self.fp.set(self._fused.get_weights())
            it, m, v = self._fused.backend.get_optimizer_state()
            self.opt.load_state(it, m, v)

    # ------------------------------------------------------------------ forward / loss
    def _forward(self, x: torch.Tensor, training: bool, logits_only: bool = False) -> torch.Tensor:
        P = self.fp.params
        h = x
        last = len(self.layers) - 1
        for i, lyr in enumerate(self.layers):
            if isinstance(lyr, InputLayer):
                continue
            params = [P[s] for s in lyr.param_slots]
            if i == last and logits_only and isinstance(lyr, Dense):
                h = lyr.forward(params, h, training, logits_only=True)
            else:
                h = lyr.forward(params, h, training)
        return h

    def __call__(self, x) -> torch.Tensor:
        with torch.no_grad():
            return self._forward(self._prep_x(x), False)

    def _head_is_softmax(self) -> bool:
        last = self.layers[-1]
        return isinstance(last, Dense) and last.activation == "softmax"

    def _loss_and_metric(self, x: torch.Tensor, y: torch.Tensor, training: bool):
        """(mean loss incl. activity penalties, #correct) for one batch."""
        B = x.shape[0]
        if self.loss == "sparse_categorical_crossentropy" and self._head_is_softmax():
            z = self._forward(x, training, logits_only=True)
            yl = y.reshape(-1).long()
            if z.is_cuda and z.shape[-1] in (2, 10, 16, 32) and z.dim() == 2:
                corr = torch.zeros(2, device=z.device)
                loss = _SparseXent.apply(z.float(), yl, corr)
                correct = corr[1]
            else:
                lsm = torch.log_softmax(z.float(), -1)
                loss = -lsm.gather(-1, yl[:, None]).mean()
                correct = (z.argmax(-1) == yl).sum()
        else:
            yp = self._forward(x, training)
            yt = y.to(yp.dtype)
            if yp.dim() == 3 and yt.dim() == 2:
                yt = yt.unsqueeze(1)
            if self.loss == "sparse_categorical_crossentropy":
                yl = y.reshape(-1).long()
                loss = -torch.log(yp.clamp(1e-7, 1 - 1e-7)).gather(-1, yl[:, None]).mean()
                correct = (yp.argmax(-1) == yl).sum()
            elif self.loss == "mean_squared_error":
                from ..ops.loss import mse_accuracy          # fused K3 + K6 on ROCm
                loss, correct = mse_accuracy(yp, y.to(yp.dtype))
            else:
                yt = torch.broadcast_to(yt, yp.shape)
                if self.loss == "mean_squared_error":
                    loss = ((yp - yt) ** 2).mean()
                elif self.loss == "mean_absolute_error":
                    loss = (yp - yt).abs().mean()
                elif self.loss == "categorical_crossentropy":
                    p = yp / yp.sum(-1, keepdim=True)
                    loss = -(yt * torch.log(p.clamp(1e-7, 1 - 1e-7))).sum(-1).mean()
                else:  # binary_crossentropy
                    p = yp.clamp(1e-7, 1 - 1e-7)
                    loss = -(yt * torch.log(p) + (1 - yt) * torch.log(1 - p)).mean()
                if self.loss == "binary_crossentropy":
                    eq = ((yp > 0.5) == (yt > 0.5)).float().mean(dim=tuple(range(1, yp.dim())) or None)
                else:
                    eq = (yp.argmax(-1) == yt.argmax(-1)).float()
                    if eq.dim() > 1:
                        eq = eq.mean(dim=tuple(range(1, eq.dim())))
                correct = eq.sum()
        if training:
            for lyr in self.layers:
                pen = getattr(lyr, "_penalty", None)
                if pen is not None:
                    loss = loss + pen
                    lyr._penalty = None
        return loss, correct

    # ------------------------------------------------------------------ data
    def _prep_x(self, x) -> torch.Tensor:
        t = torch.as_tensor(x)
        if t.device != self.device:
            t = t.to(self.device, non_blocking=True)
        if t.dtype == torch.uint8:
            return t.float()
        if t.dtype not in (torch.float32, torch.bfloat16):
            t = t.float()
        return t

    def _prep_y(self, y) -> torch.Tensor:
        t = torch.as_tensor(y)
        if t.device != self.device:
            t = t.to(self.device, non_blocking=True)
        if self.loss == "sparse_categorical_crossentropy":
            return t.long()
        return t.float()

    def _batches(self, x, y, batch_size, shuffle, rng, world, rank):
        """Yield (xb, yb) device batches from arrays, an iterable of batches, or a Stream."""
        from ..data.stream import Stream
        if isinstance(x, Stream):
            for c in x.batch(batch_size):
                xb = self._prep_x(c.x)
                yield xb, xb
            return
        if callable(x) and y is None:       # factory of (xb, yb) batches, re-read each epoch
            for xb, yb in x():
                yield self._prep_x(xb), self._prep_y(yb)
            return
        xs = np.asarray(x) if not isinstance(x, torch.Tensor) else x
        ys = xs if y is None else (np.asarray(y) if not isinstance(y, torch.Tensor) else y)
        if world > 1:
            from ..parallel.dp import shard_range
            s0, s1 = shard_range(len(xs), rank, world)
            xs, ys = xs[s0:s1], ys[s0:s1]
        n = len(xs)
        order = rng.permutation(n) if shuffle else None
        for s in range(0, n, batch_size):
            idx = order[s:s + batch_size] if order is not None else slice(s, s + batch_size)
            yield self._prep_x(xs[idx]), self._prep_y(ys[idx])

    # ------------------------------------------------------------------ training
    def train_on_batch(self, x, y, global_batch: Optional[int] = None, allreduce=None):
        xb, yb = self._prep_x(x), self._prep_y(y)
        self.fp.zero_grad()
        loss, correct = self._loss_and_metric(xb, yb, True)
        n = xb.shape[0]
        scale = n / float(global_batch or n)
        (loss * scale).backward()
        self.opt.step(allreduce=allreduce)
        with torch.no_grad():
            self._acc[0] += loss.detach().to(self._acc.dtype) * n
            self._acc[1] += correct.detach().to(self._acc.dtype)
            self._acc[2] += n
        return loss

    def fit(self, x=None, y=None, batch_size: int = 32, epochs: int = 1, verbose: int = 1,
            callbacks: Optional[Sequence[Callback]] = None, validation_data=None, shuffle: bool = True,
            steps_per_epoch: Optional[int] = None, seed: int = 0, initial_epoch: int = 0) -> History:
        if not self.compiled:
            self.compile()
        if self._fused is not None:
            if y is not None and y is not x:
                raise ValueError("autoencoder fit expects y == x")
            hist = self._fused.fit(x, epochs=epochs, batch_size=batch_size, verbose=verbose, callbacks=callbacks,
                                   validation_data=validation_data, shuffle=shuffle,
                                   steps_per_epoch=steps_per_epoch, seed=seed, initial_epoch=initial_epoch)
            self._sync_from_fused()
            return hist
        import torch.distributed as dist
        from ..parallel.dp import allreduce_sum_, reduce_metrics
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        rank = dist.get_rank() if world > 1 else 0
        allreduce = allreduce_sum_ if world > 1 else None
        hist = History()
        cbs = [hist] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
            cb.on_train_begin()
        from ..parallel.fault import maybe_inject
        gstep = int(getattr(self, "_global_step", 0))
        self.stop_training = False
        for epoch in range(initial_epoch, epochs):
            rng = np.random.default_rng([seed, rank, epoch])   # epoch-keyed shuffles: resumable
            t0 = time.perf_counter()
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            self._acc.zero_()
            steps = 0
            for xb, yb in self._batches(x, y, batch_size, shuffle, rng, world, rank):
                if steps_per_epoch is not None and steps >= steps_per_epoch:
                    break
                maybe_inject(gstep, rank)
                self.train_on_batch(xb, yb, global_batch=xb.shape[0] * world, allreduce=allreduce)
                steps += 1
                gstep += 1
            self._global_step = gstep
            a = self._acc.double().cpu().numpy()
            m = {"loss": a[0] / max(a[2], 1), "accuracy": a[1] / max(a[2], 1), "rows": a[2]}
            if world > 1:
                m = reduce_metrics(m, self.device)
            logs = {"loss": float(m["loss"])}
            if "accuracy" in self.metrics or "acc" in self.metrics:
                logs["accuracy"] = float(m["accuracy"])
            if validation_data is not None:
                vx = validation_data[0]
                vy = validation_data[1] if len(validation_data) > 1 else None
                vl, va = self.evaluate(vx, vy, batch_size=max(batch_size, 1024))
                logs["val_loss"] = vl
                if "accuracy" in logs:
                    logs["val_accuracy"] = va
            logs["_seconds"] = time.perf_counter() - t0
            logs["_rows"] = float(m["rows"])
            if verbose and rank == 0:
                shown = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items() if not k.startswith("_"))
                print(f"Epoch {epoch + 1}/{epochs}\n{steps} steps - {logs['_seconds']:.2f}s - {shown}", flush=True)
            for cb in cbs:
                cb.on_epoch_end(epoch, dict(logs))
            if self.stop_training:
                break
        for cb in cbs:
            cb.on_train_end()
        return hist

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def predict(self, x, batch_size: int = 32, callbacks: Optional[Sequence[Callback]] = None,
                verbose: int = 0) -> np.ndarray:
        if not self.compiled:
            self.compile()
        if self._fused is not None:
            return self._fused.predict(x, batch_size=batch_size, callbacks=callbacks)
        from ..data.stream import Stream
        cbs = list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
        outs = []
        if isinstance(x, Stream):
            src = (c.x for c in x.batch(batch_size))
        else:
            arr = np.asarray(x) if not isinstance(x, torch.Tensor) else x
            src = (arr[s:s + batch_size] for s in range(0, len(arr), batch_size))
        for bi, xb in enumerate(src):
            out = self._forward(self._prep_x(xb), False).float().cpu().numpy()
            outs.append(out)
            for cb in cbs:
                cb.on_predict_batch_end(bi, {"outputs": out})
        for cb in cbs:
            cb.on_predict_end()
        return np.concatenate(outs) if outs else np.zeros((0, *self.output_shape), np.float32)

    @torch.no_grad()
    def evaluate(self, x, y=None, batch_size: int = 1024, verbose: int = 0) -> Tuple[float, float]:
        if not self.compiled:
            self.compile()
        if self._fused is not None:
            return self._fused.evaluate(x, batch_size=max(batch_size, 65536))
        tot = np.zeros(3)
        xs = np.asarray(x) if not isinstance(x, torch.Tensor) else x
        ys = xs if y is None else (np.asarray(y) if not isinstance(y, torch.Tensor) else y)
        for s in range(0, len(xs), batch_size):
            xb, yb = self._prep_x(xs[s:s + batch_size]), self._prep_y(ys[s:s + batch_size])
            loss, corr = self._loss_and_metric(xb, yb, False)
            tot += [float(loss) * len(xb), float(corr), len(xb)]
        n = max(tot[2], 1)
        return float(tot[0] / n), float(tot[1] / n)

    # ------------------------------------------------------------------ weights / summary
    def get_weights(self) -> List[np.ndarray]:
        self.build()
        if self._fused is not None:
            return self._fused.get_weights()
        return self.fp.get()

    def set_weights(self, weights: Sequence[np.ndarray]) -> None:
        self.build()
        self.fp.set(weights)
        if self._fused is not None:
            self._fused.set_weights(weights)

    def count_params(self) -> int:
        self.build()
        return int(self.fp.n)

    def summary(self, print_fn=print) -> str:
        self.build()
        lines = [f'Model: "{self.name}"', "_" * 65, f"{'Layer (type)':<29}{'Output Shape':<22}{'Param #':>10}",
                 "=" * 65]
        for lyr in self.layers:
            n = sum(int(np.prod(self.fp.shapes[s])) for s in lyr.param_slots)
            lines.append(f"{lyr.name + ' (' + lyr.class_name + ')':<29}{str((None, *lyr.out_shape)):<22}{n:>10}")
        lines += ["=" * 65, f"Total params: {self.count_params():,}", f"Trainable params: {self.count_params():,}",
                  "Non-trainable params: 0", "_" * 65]
        text = "\n".join(lines)
        if print_fn:
            print_fn(text)
        return text

    # ------------------------------------------------------------------ persistence
    def model_config(self) -> dict:
        if self.functional:
            out, prev = [], None
            for lyr in self.layers:
                # node nesting exactly as stored in the reference models/*.h5
                entry = {"name": lyr.name, "class_name": lyr.class_name, "config": lyr.get_config(),
                         "inbound_nodes": [] if prev is None else [[prev, 0, 0, {}]]}
                if isinstance(lyr, Dense):
                    entry["config"].pop("batch_input_shape", None)
                out.append(entry)
                prev = lyr.name
            return {"class_name": "Model", "config": {"name": self.name, "layers": out,
                                                      "input_layers": [self.layers[0].name, 0, 0],
                                                      "output_layers": [self.layers[-1].name, 0, 0]}}
        return kc.sequential(self.name, [{"class_name": l.class_name, "config": l.get_config()}
                                         for l in self.layers])

    def save(self, path: str, include_optimizer: bool = True) -> None:
        if self._fused is not None:
            self._sync_from_fused()
        arrays = self.fp.get()
        layers, flat_names = [], []
        for lyr in self.layers:
            names = [f"{lyr.name}/{n}:0" for n, _ in
                     (lyr.weight_specs(self._in_shape_of(lyr)) if lyr.param_slots else [])]
            ws = [(nm, arrays[s]) for nm, s in zip(names, lyr.param_slots)]
            flat_names += names
            layers.append((lyr.name, ws))
        opt = None
        if include_optimizer and self.opt is not None:
            it, m, v = self.opt.state()
            opt = list(zip(ckh5.adam_weight_names(flat_names), [np.array(it, np.int64)] + m + v))
        tc = kc.training_config(self.hp["lr"], self.hp["beta_1"], self.hp["beta_2"], self.hp["epsilon"],
                                loss=self.loss, metrics=self.metrics)
        ckh5.save_keras_h5(path, self.model_config(), layers, tc, opt)

    def _in_shape_of(self, lyr: Layer):
        prev = tuple(self._input_shape())
        for l in self.layers:
            if l is lyr:
                return prev
            prev = l.out_shape
        return prev


class Sequential(Model):
    def __init__(self, layers: Optional[Sequence[Layer]] = None, name: str = "sequential", device="auto",
                 seed: int = 0):
        super().__init__(layers=list(layers or []), name=name, device=device, seed=seed)
        self.functional = False


def load_model(path: str, device="auto", compile: bool = True, fused: Optional[bool] = None) -> Model:
    """Rebuild a model from a Keras ``.h5`` (written here or by Keras 2.2.4-tf)."""
    ck = ckh5.load_keras_h5(path)
    mc = ck.model_config
    cfg = mc["config"]
    layers = [layer_from_config(l["class_name"], l["config"]) for l in cfg["layers"]]
    if mc["class_name"] == "Sequential":
        model: Model = Sequential(layers, name=cfg.get("name", "sequential"), device=device)
    else:
        for a, b in zip(layers[:-1], layers[1:]):
            b.inbound = [a]
        model = Model(inputs=layers[0], outputs=layers[-1], name=cfg.get("name", "model"), device=device)
    model.build()
    model.fp.set(ck.flat_weights())
    hp = kc.optimizer_hparams(ck.training_config)
    model.hp.update(hp)
    if ck.optimizer_weights and len(ck.optimizer_weights) == 1 + 2 * len(model.fp.shapes):
        arr = [a for _, a in ck.optimizer_weights]
        k = len(model.fp.shapes)
        model._pending_opt_state = (int(np.asarray(arr[0]).reshape(-1)[0]), arr[1:1 + k], arr[1 + k:])
    if compile:
        tc = ck.training_config or {}
        model.compile(optimizer=Adam(**{("learning_rate" if k == "lr" else k): v for k, v in model.hp.items()}),
                      loss=tc.get("loss", "mean_squared_error"), metrics=tc.get("metrics") or [], fused=fused)
    return model
