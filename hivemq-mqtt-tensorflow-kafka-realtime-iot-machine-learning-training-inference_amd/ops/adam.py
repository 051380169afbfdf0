"""Multi-tensor Adam on one flat fp32 buffer.

All parameters of a model are views into one contiguous buffer and their
``.grad`` are views into one flat gradient buffer, so an optimizer step is ONE
launch of the ``reduce_adam`` HIP kernel (G = 1) over the whole model, and a
data-parallel step is ONE RCCL all-reduce of the flat gradient bucket.  Keras /
TF ResourceApplyAdam semantics (bias-corrected lr_t, epsilon outside the sqrt).
On CPU the same math runs in torch.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from ._ext import load_c

RA_ADAM = 2


class FlatParams:
    """Owns the flat parameter / gradient / moment buffers of a list of shapes."""

    def __init__(self, shapes: Sequence[Sequence[int]], device, init: Optional[Sequence[np.ndarray]] = None):
        self.device = torch.device(device)
        self.shapes = [tuple(s) for s in shapes]
        sizes = [int(np.prod(s)) if len(s) else 1 for s in self.shapes]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
        n = int(self.offsets[-1])
        self.n = n
        self.n_pad = (n + 3) // 4 * 4   # the Adam kernel works on float4 quads
        self.flat = torch.zeros(self.n_pad, device=self.device)
        self.grad = torch.zeros(self.n_pad, device=self.device)
        self.m = torch.zeros(self.n_pad, device=self.device)
        self.v = torch.zeros(self.n_pad, device=self.device)
        self.iter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.params: List[torch.nn.Parameter] = []
        for i, s in enumerate(self.shapes):
            view = self.flat[self.offsets[i]:self.offsets[i + 1]].view(s)
            p = torch.nn.Parameter(view)
            p.grad = self.grad[self.offsets[i]:self.offsets[i + 1]].view(s)
            self.params.append(p)
        if init is not None:
            self.set([np.asarray(a, np.float32) for a in init])

    def set(self, arrays: Sequence[np.ndarray]) -> None:
        with torch.no_grad():
            for p, a in zip(self.params, arrays):
                p.copy_(torch.as_tensor(np.asarray(a, np.float32).reshape(p.shape)))

    def get(self) -> List[np.ndarray]:
        return [p.detach().cpu().numpy().copy() for p in self.params]

    def split(self, flat: torch.Tensor) -> List[np.ndarray]:
        a = flat.detach().cpu().numpy()
        return [a[self.offsets[i]:self.offsets[i + 1]].reshape(s).copy() for i, s in enumerate(self.shapes)]

    def join(self, arrays: Sequence[np.ndarray], out: torch.Tensor) -> None:
        buf = np.zeros(self.n_pad, np.float32)
        for i, a in enumerate(arrays):
            buf[self.offsets[i]:self.offsets[i + 1]] = np.asarray(a, np.float32).ravel()
        out.copy_(torch.from_numpy(buf))

    def zero_grad(self) -> None:
        self.grad.zero_()


class FlatAdam:
    def __init__(self, fp: FlatParams, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.fp = fp
        self.lr, self.b1, self.b2, self.eps = lr, beta_1, beta_2, epsilon
        self.on_gpu = fp.device.type == "cuda"
        if self.on_gpu:
            self.C = load_c()

    def step(self, grad_scale: float = 1.0, allreduce=None, counted: bool = False) -> None:
        """``counted``: the step count was already advanced on the device this step (a fused
        train step folds the increment into its loss kernel: one launch fewer)."""
        fp = self.fp
        if allreduce is not None:
            allreduce(fp.grad)
        if not counted:
            fp.iter.add_(1)
        if self.on_gpu:
            self.C.reduce_adam(fp.grad, 1, fp.n_pad, fp.n_pad, None, fp.flat, fp.m, fp.v, fp.iter, self.lr, self.b1,
                               self.b2, self.eps, float(grad_scale), None, RA_ADAM)
            return
        t = float(fp.iter.item())
        lr_t = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
        with torch.no_grad():
            g = fp.grad * grad_scale
            fp.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            fp.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            fp.flat.sub_(lr_t * fp.m / (fp.v.sqrt() + self.eps))

    def state(self):
        return int(self.fp.iter.item()), self.fp.split(self.fp.m), self.fp.split(self.fp.v)

    def load_state(self, it: int, m, v) -> None:
        self.fp.iter.fill_(int(it))
        self.fp.join(m, self.fp.m)
        self.fp.join(v, self.fp.v)
