"""Keras-semantics reference implementations in plain PyTorch (fp32 / fp64).

These are the numerics oracles for the HIP kernels and the execution path for
the CPU-only plumbing configuration (BASELINE config 1).  Semantics recovered
from the reference's TF profile trace and ``.h5`` training_config (SURVEY.md
sec. 2.1 C11/C12, sec. 7.5 item 5):

* loss = mean over (batch, features) of (y - x)^2  (Keras ``mean_squared_error``
  then ``SUM_OVER_BATCH_SIZE``)
* activity regulariser on layer 1 output: ``l1 * sum|h1| / batch``
* metric ``'accuracy'`` with MSE resolves to categorical accuracy
  (argmax(y_true) == argmax(y_pred))
* Adam: ``lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)``;
  ``w -= lr_t * m / (sqrt(v) + eps)`` with eps = 1e-7
* GlorotUniform kernels (limit ``sqrt(6 / (fan_in + fan_out))``), zero biases.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

_ACT = {
    "linear": lambda z: z, None: lambda z: z,
    "relu": torch.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid,
}


def glorot_uniform(fan_in: int, fan_out: int, rng: np.random.Generator, shape=None) -> np.ndarray:
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-limit, limit, size=shape or (fan_in, fan_out)).astype(np.float32)


def init_dense_weights(layer_sizes: Sequence[Tuple[int, int]], seed: int = 0) -> List[np.ndarray]:
    rng = np.random.default_rng(seed)
    out: List[np.ndarray] = []
    for i, o in layer_sizes:
        out.append(glorot_uniform(i, o, rng))
        out.append(np.zeros(o, dtype=np.float32))
    return out


def ae_forward_torch(x: torch.Tensor, weights: Sequence[torch.Tensor], activations: Sequence[str]):
    """Returns (y, [h1, h2, h3])."""
    h = x
    hs = []
    for li in range(4):
        k, b = weights[2 * li], weights[2 * li + 1]
        h = _ACT[activations[li]](h @ k + b)
        hs.append(h)
    return hs[-1], hs[:-1]


def ae_loss_torch(x: torch.Tensor, weights: Sequence[torch.Tensor], activations: Sequence[str], l1: float):
    """Keras total loss, MSE part, and categorical accuracy of one batch."""
    y, hs = ae_forward_torch(x, weights, activations)
    mse = ((y - x) ** 2).mean()
    reg = l1 * hs[0].abs().sum() / x.shape[0]
    acc = (torch.argmax(y, dim=1) == torch.argmax(x, dim=1)).float().mean()
    return mse + reg, mse, acc


class KerasAdam:
    """TF-2.0 ``ResourceApplyAdam`` (non-nesterov, no amsgrad)."""

    def __init__(self, params: Sequence[torch.Tensor], lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.params = list(params)
        self.lr, self.b1, self.b2, self.eps = lr, beta_1, beta_2, epsilon
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.iterations = 0

    @torch.no_grad()
    def apply(self, grads: Sequence[torch.Tensor]) -> None:
        self.iterations += 1
        t = self.iterations
        lr_t = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
        for p, g, m, v in zip(self.params, grads, self.m, self.v):
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            p.sub_(lr_t * m / (v.sqrt() + self.eps))


class TorchAE:
    """Autoencoder trainer on torch ops (CPU plumbing path / oracle)."""

    def __init__(self, layer_sizes, activations, l1: float, weights: Sequence[np.ndarray],
                 device="cpu", dtype=torch.float32, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.layer_sizes = list(layer_sizes)
        self.activations = list(activations)
        self.l1 = l1
        self.device = torch.device(device)
        self.dtype = dtype
        self.w = [torch.tensor(np.asarray(a), dtype=dtype, device=self.device).requires_grad_(True) for a in weights]
        self.opt = KerasAdam(self.w, lr, beta_1, beta_2, epsilon)
        self._acc = [0.0, 0.0, 0.0, 0.0]   # loss*n, mse*n, acc*n, n

    def grads(self, x: torch.Tensor):
        loss, mse, acc = ae_loss_torch(x, self.w, self.activations, self.l1)
        g = torch.autograd.grad(loss, self.w)
        return g, loss.detach(), mse.detach(), acc.detach()

    def step(self, x: torch.Tensor, global_batch: Optional[int] = None, allreduce=None) -> None:
        """One Adam step; under DP the local mean gradient is rescaled to this shard's share of the
        global-batch mean and summed over replicas in ONE flat all-reduce (same contract as FusedAE)."""
        x = x.to(self.device, self.dtype)
        g, loss, mse, acc = self.grads(x)
        n = x.shape[0]
        if allreduce is not None:
            flat = torch.cat([gi.reshape(-1) for gi in g]) * (n / float(global_batch or n))
            allreduce(flat)
            g = [c.view_as(w) for c, w in zip(torch.split(flat, [w.numel() for w in self.w]), self.w)]
        self.opt.apply(g)
        self._acc[0] += float(loss) * n
        self._acc[1] += float(mse) * n
        self._acc[2] += float(acc) * n
        self._acc[3] += n

    def step_empty(self, global_batch: int, allreduce) -> None:
        """This replica has no rows in a data-parallel step: contribute a zero gradient to the
        all-reduce and apply the same Adam update as every other replica."""
        flat = torch.zeros(sum(w.numel() for w in self.w), dtype=self.dtype, device=self.device)
        allreduce(flat)
        self.opt.apply([c.view_as(w) for c, w in zip(torch.split(flat, [w.numel() for w in self.w]), self.w)])

    def reset_metrics(self) -> None:
        self._acc = [0.0, 0.0, 0.0, 0.0]

    def read_metrics(self) -> dict:
        n = max(self._acc[3], 1.0)
        return {"loss": self._acc[0] / n, "mse": self._acc[1] / n, "accuracy": self._acc[2] / n, "rows": self._acc[3]}

    @torch.no_grad()
    def forward(self, x: torch.Tensor):
        y, _ = ae_forward_torch(x.to(self.device, self.dtype), self.w, self.activations)
        return y

    def get_weights(self) -> List[np.ndarray]:
        return [w.detach().cpu().numpy().astype(np.float32) for w in self.w]

    def set_weights(self, weights: Sequence[np.ndarray]) -> None:
        with torch.no_grad():
            for w, a in zip(self.w, weights):
                w.copy_(torch.as_tensor(np.asarray(a), dtype=self.dtype))

    def get_optimizer_state(self):
        return (self.opt.iterations, [m.cpu().numpy() for m in self.opt.m], [v.cpu().numpy() for v in self.opt.v])

    def set_optimizer_state(self, it: int, m, v) -> None:
        self.opt.iterations = int(it)
        for dst, src in zip(self.opt.m, m):
            dst.copy_(torch.as_tensor(np.asarray(src), dtype=self.dtype))
        for dst, src in zip(self.opt.v, v):
            dst.copy_(torch.as_tensor(np.asarray(src), dtype=self.dtype))
