"""MNIST MLP classifier.

Reference models:

* python-scripts/tensorflow-kafka-mnist.py:39-47 and confluent-tensorflow-io-kafka.py:40-50 ::

      Flatten(input_shape=(28, 28)) -> Dense(128, relu) -> Dense(10, softmax)
      compile(optimizer='adam', loss='sparse_categorical_crossentropy', metrics=['accuracy'])
      fit(zip(xx, yy).batch(1), epochs=5, steps_per_epoch=12000)

* confluent-tensorflow-io-kafka-simplified.py:10-29 -- Dense(512, relu) + Dropout(0.2),
  ``fit(x_train, y_train, epochs=5, validation_data=(x_test, y_test))`` (Keras default batch 32).

Device path (every GEMM on the in-tree fp32-MFMA kernels of ``csrc/kernels/mlp.hip``):
inputs travel as ``uint8`` and are scaled by 1/255 as the GEMM stages them
(``convert_image_dtype``); layer 1 = one launch with bias + relu + Dropout fused in
the epilogue (the mask is a counter hash of (seed, step, row, col), no torch.rand);
layer 2 = one launch; softmax + sparse-CE forward/backward + the accuracy count are
ONE fused HIP kernel (``softmax_xent``, K13); the backward is three launches (dW2|db2
as one [h ; 1]^T . dz product written straight into the flat gradient buffer, dH =
dz . W2^T gated by [h > 0] / keep, dW1|db1 = [x ; 1]^T . dH) and the optimizer step is
one flat HIP Adam launch.  Metrics stay on the device until the epoch ends.
"""
from __future__ import annotations

import math
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ckpt import h5 as ckh5
from ..nn import keras_config as kc
from ..nn.callbacks import Callback, History
from ..ops.adam import FlatAdam, FlatParams
from ..ops._ext import load_c


def _resolve_device(device) -> torch.device:
    if device in (None, "auto"):
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(device)


def softmax_xent_reference(logits: torch.Tensor, labels: torch.Tensor):
    """fp32 torch oracle: (loss_sum, correct, dlogits for a unit loss scale)."""
    lsm = torch.log_softmax(logits.float(), dim=1)
    y = labels.long()
    loss = -lsm.gather(1, y[:, None]).sum()
    correct = (logits.argmax(dim=1) == y).sum()
    d = lsm.exp()
    d[torch.arange(len(y)), y] -= 1.0
    return loss, correct, d


class MLPClassifier:
    def __init__(self, hidden: int = 128, classes: int = 10, input_shape=(28, 28), dropout: float = 0.0,
                 device="auto", seed: int = 0, lr: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, name: str = "sequential"):
        self.device = _resolve_device(device)
        self.input_shape = tuple(input_shape)
        self.in_features = int(np.prod(self.input_shape))
        self.hidden, self.classes, self.dropout = int(hidden), int(classes), float(dropout)
        self.name = name
        self.hp = dict(lr=lr, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon)
        rng = np.random.default_rng(seed)

        def glorot(fi, fo):
            lim = math.sqrt(6.0 / (fi + fo))
            return rng.uniform(-lim, lim, size=(fi, fo)).astype(np.float32)

        init = [glorot(self.in_features, self.hidden), np.zeros(self.hidden, np.float32),
                glorot(self.hidden, self.classes), np.zeros(self.classes, np.float32)]
        self.fp = FlatParams([a.shape for a in init], self.device, init)
        self.opt = FlatAdam(self.fp, **self.hp)
        self.on_gpu = self.device.type == "cuda"
        self.C = load_c() if self.on_gpu else None
        self._acc = torch.zeros(2, device=self.device)
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(seed)
        self._seed, self._step = int(seed) & 0xffffffff, 0   # in-kernel dropout RNG key
        self.stop_training = False

    # ------------------------------------------------------------------ core
    @property
    def weights(self):
        return self.fp.params

    def count_params(self) -> int:
        return self.fp.n

    def _prep(self, x) -> torch.Tensor:
        """uint8 / float images -> [B, 784] float on the device (uint8 is scaled by 1/255)."""
        t = torch.as_tensor(x)
        if t.device != self.device:
            t = t.to(self.device, non_blocking=True)
        t = t.reshape(len(t), -1)
        if t.dtype == torch.uint8:
            # the device GEMM scales uint8 by 1/255 while staging it (no fp32 copy)
            return t.contiguous() if self.on_gpu else t.float().mul_(1.0 / 255.0)
        return t.float()

    def logits(self, x: torch.Tensor, training: bool = False):
        W1, b1, W2, b2 = self.fp.params
        if self.on_gpu:
            keep = 1.0 - self.dropout if (training and self.dropout > 0) else 1.0
            h = self.C.mlp_fwd(x, W1, b1, True, keep, self._seed, self._step)
            return self.C.mlp_fwd(h, W2, b2, False), h, None
        # CPU path / fp32 oracle: plain torch ops
        x = x.float() / 255.0 if x.dtype == torch.uint8 else x
        h = (x @ W1 + b1).relu_()
        mask = None
        if training and self.dropout > 0:
            keep = 1.0 - self.dropout
            mask = (torch.rand(h.shape, device=h.device, generator=self._gen) < keep).float().mul_(1.0 / keep)
            h = h * mask
        return h @ W2 + b2, h, mask

    @torch.no_grad()
    def train_step(self, x, y, global_batch: Optional[int] = None, allreduce=None) -> None:
        """One Adam step on a batch; loss / correct accumulate into the device-side metric buffer."""
        xb = self._prep(x)
        yb = torch.as_tensor(y).to(self.device, non_blocking=True).reshape(-1).long()
        B = xb.shape[0]
        scale = 1.0 / float(global_batch or B)
        W1, b1, W2, b2 = self.fp.params
        z, h, mask = self.logits(xb, training=True)
        if self.on_gpu:
            dz = torch.empty_like(z)
            self.C.softmax_xent(z.contiguous(), yb.contiguous(), scale, dz, None, self._acc)
            fp = self.fp
            o = fp.offsets
            keep = 1.0 - self.dropout if self.dropout > 0 else 1.0
            self.C.mlp_wgrad(h, dz, fp.grad[o[2]:o[4]])                # dW2 | db2
            dh = self.C.mlp_bwd_data(dz, W2, h, keep)                   # dz . W2^T * [h > 0] / keep
            self.C.mlp_wgrad(xb, dh, fp.grad[o[0]:o[2]])               # dW1 | db1
            self._step += 1
            self.opt.step(allreduce=allreduce)
            return
        else:
            loss, corr, dz = softmax_xent_reference(z, yb)
            dz.mul_(scale)
            self._acc[0] += loss
            self._acc[1] += corr
        gW1, gb1, gW2, gb2 = (p.grad for p in self.fp.params)
        gW2.copy_(h.t() @ dz)
        torch.sum(dz, 0, out=gb2)
        dh = dz @ W2.t()
        dh.mul_(h > 0)
        if mask is not None:
            dh.mul_(mask)
        gW1.copy_(xb.t() @ dh)
        torch.sum(dh, 0, out=gb1)
        self.opt.step(allreduce=allreduce)

    @torch.no_grad()
    def predict(self, x, batch_size: int = 4096, callbacks: Optional[Sequence[Callback]] = None) -> np.ndarray:
        """Softmax probabilities [n, classes]."""
        outs = []
        arr = x
        for bi, s in enumerate(range(0, len(arr), batch_size)):
            z, _, _ = self.logits(self._prep(arr[s:s + batch_size]))
            if self.on_gpu:
                p = torch.empty_like(z)
                lab = torch.zeros(len(z), dtype=torch.long, device=self.device)
                self.C.softmax_xent(z.contiguous(), lab, 0.0, None, p, None)
            else:
                p = torch.softmax(z, dim=1)
            out = p.cpu().numpy()
            outs.append(out)
            for cb in callbacks or []:
                cb.set_model(self)
                cb.on_predict_batch_end(bi, {"outputs": out})
        for cb in callbacks or []:
            cb.on_predict_end()
        return np.concatenate(outs) if outs else np.zeros((0, self.classes), np.float32)

    @torch.no_grad()
    def evaluate(self, x, y, batch_size: int = 8192) -> Tuple[float, float]:
        acc = torch.zeros(2, device=self.device)
        n = len(x)
        for s in range(0, n, batch_size):
            z, _, _ = self.logits(self._prep(x[s:s + batch_size]))
            yb = torch.as_tensor(y[s:s + batch_size]).to(self.device).reshape(-1).long()
            if self.on_gpu:
                self.C.softmax_xent(z.contiguous(), yb, 0.0, None, None, acc)
            else:
                loss, corr, _ = softmax_xent_reference(z, yb)
                acc[0] += loss
                acc[1] += corr
        a = acc.cpu().numpy()
        return float(a[0] / max(n, 1)), float(a[1] / max(n, 1))

    # ------------------------------------------------------------------ training
    def fit(self, x=None, y=None, epochs: int = 1, batch_size: int = 32, steps_per_epoch: Optional[int] = None,
            validation_data=None, callbacks: Optional[Sequence[Callback]] = None, shuffle: bool = True,
            verbose: int = 1, seed: int = 0, stream=None) -> History:
        """Arrays (``x`` uint8/float images, ``y`` int labels) or ``stream`` = a callable returning an
        iterator of ``(images, labels)`` chunks (e.g. :func:`streamml.data.mnist.kafka_mnist`), re-read
        every epoch like a tf.data pipeline."""
        import torch.distributed as dist
        from ..parallel.dp import allreduce_sum_, shard_range

        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        rank = dist.get_rank() if world > 1 else 0
        allreduce = allreduce_sum_ if world > 1 else None
        hist = History()
        cbs = [hist] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
            cb.on_train_begin()
        if x is not None:
            xs = np.asarray(x)
            ys = np.asarray(y)
            if world > 1:
                s0, s1 = shard_range(len(xs), rank, world)
                xs, ys = xs[s0:s1], ys[s0:s1]
            xd = torch.as_tensor(xs).to(self.device)
            yd = torch.as_tensor(ys.astype(np.int64)).to(self.device)
        rng = np.random.default_rng(seed + rank)
        self.stop_training = False
        for epoch in range(epochs):
            t0 = time.perf_counter()
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            self._acc.zero_()
            rows = steps = 0
            if x is not None:
                n = len(xd)
                order = torch.as_tensor(rng.permutation(n), device=self.device) if shuffle else None
                nb = math.ceil(n / batch_size)
                if steps_per_epoch is not None:
                    nb = min(nb, steps_per_epoch)
                for b in range(nb):
                    idx = order[b * batch_size:(b + 1) * batch_size] if order is not None else \
                        slice(b * batch_size, (b + 1) * batch_size)
                    xb, yb = xd[idx], yd[idx]
                    self.train_step(xb, yb, global_batch=len(xb) * world, allreduce=allreduce)
                    rows += len(xb)
                    steps += 1
            else:
                done = False
                for cx, cy in stream():
                    for s in range(0, len(cx), batch_size):
                        if steps_per_epoch is not None and steps >= steps_per_epoch:
                            done = True
                            break
                        xb, yb = cx[s:s + batch_size], cy[s:s + batch_size]
                        self.train_step(xb, yb.astype(np.int64), global_batch=len(xb) * world, allreduce=allreduce)
                        rows += len(xb)
                        steps += 1
                    if done:
                        break
            a = self._acc.clone()
            if world > 1:
                allreduce(a)
                tot = torch.tensor([float(rows)], device=self.device)
                allreduce(tot)
                rows_all = float(tot.item())
            else:
                rows_all = float(rows)
            a = a.cpu().numpy()
            logs = {"loss": float(a[0] / max(rows_all, 1)), "accuracy": float(a[1] / max(rows_all, 1))}
            if validation_data is not None:
                vl, va = self.evaluate(*validation_data)
                logs["val_loss"], logs["val_accuracy"] = vl, va
            logs["_seconds"] = time.perf_counter() - t0
            logs["_rows"] = rows
            if verbose and rank == 0:
                shown = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items() if not k.startswith("_"))
                print(f"Epoch {epoch + 1}/{epochs}\n{steps}/{steps} - {logs['_seconds']:.2f}s - {shown}", flush=True)
            for cb in cbs:
                cb.on_epoch_end(epoch, dict(logs))
            if self.stop_training:
                break
        for cb in cbs:
            cb.on_train_end()
        return hist

    # ------------------------------------------------------------------ persistence
    def _layer_names(self) -> List[str]:
        return ["dense", "dense_1"]

    def model_config(self) -> dict:
        layers = [{"class_name": "Flatten", "config": {"name": "flatten", "trainable": True, "dtype": "float32",
                                                       "batch_input_shape": [None, *self.input_shape],
                                                       "data_format": "channels_last"}},
                  {"class_name": "Dense", "config": kc.dense_config("dense", self.hidden, "relu")}]
        if self.dropout > 0:
            layers.append({"class_name": "Dropout", "config": {"name": "dropout", "trainable": True,
                                                               "dtype": "float32", "rate": self.dropout,
                                                               "noise_shape": None, "seed": None}})
        layers.append({"class_name": "Dense", "config": kc.dense_config("dense_1", self.classes, "softmax")})
        return kc.sequential(self.name, layers)

    def save(self, path: str, include_optimizer: bool = True) -> None:
        W1, b1, W2, b2 = self.fp.get()
        names = ["dense/kernel:0", "dense/bias:0", "dense_1/kernel:0", "dense_1/bias:0"]
        layers = [("flatten", []), ("dense", [(names[0], W1), (names[1], b1)])]
        if self.dropout > 0:
            layers.append(("dropout", []))
        layers.append(("dense_1", [(names[2], W2), (names[3], b2)]))
        opt = None
        if include_optimizer:
            it, m, v = self.opt.state()
            opt = list(zip(ckh5.adam_weight_names(names), [np.array(it, np.int64)] + m + v))
        tc = kc.training_config(self.hp["lr"], self.hp["beta_1"], self.hp["beta_2"], self.hp["epsilon"])
        tc["loss"] = "sparse_categorical_crossentropy"
        ckh5.save_keras_h5(path, self.model_config(), layers, tc, opt)

    @classmethod
    def load(cls, path: str, device="auto") -> "MLPClassifier":
        ck = ckh5.load_keras_h5(path)
        cfg = ck.model_config["config"]
        shape, dense, dropout = (28, 28), [], 0.0
        for lyr in cfg["layers"]:
            c = lyr["config"]
            if lyr["class_name"] == "Flatten" and "batch_input_shape" in c:
                shape = tuple(int(d) for d in c["batch_input_shape"][1:])
            elif lyr["class_name"] == "Dense":
                dense.append(int(c["units"]))
            elif lyr["class_name"] == "Dropout":
                dropout = float(c["rate"])
        if len(dense) != 2:
            raise ValueError("MLPClassifier.load expects Flatten -> Dense -> [Dropout] -> Dense")
        m = cls(hidden=dense[0], classes=dense[1], input_shape=shape, dropout=dropout, device=device,
                name=cfg.get("name", "sequential"), **kc.optimizer_hparams(ck.training_config))
        m.fp.set(ck.flat_weights())
        if ck.optimizer_weights and len(ck.optimizer_weights) == 9:
            arr = [a for _, a in ck.optimizer_weights]
            m.opt.load_state(int(np.asarray(arr[0]).reshape(-1)[0]), arr[1:5], arr[5:])
        return m
