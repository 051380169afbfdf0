"""Tall-skinny dense layers on the K1/K2 HIP kernels (``csrc/kernels/dense.hip``).

``dense(x, W, b, act)`` is a differentiable Dense layer: forward = one
``dense_fwd`` launch (bias + activation fused in the epilogue); backward = the
activation derivative, one ``dense_wgrad`` launch (dW and db in one pass over the
rows) and one ``dense_fwd`` launch against W^T for dX.  Layers whose weight does
not fit the register-resident tile (K or N beyond 128..256, e.g. MNIST's 784 x
128) run on the general LDS-tiled MFMA GEMM (``ops/gemm.py``, ``csrc/kernels/gemm.hip``):
forward with bias + activation in its epilogue, dW = x^T . dz split over the rows,
dX = dz . W^T from transposed views; on CPU the reference torch ops run.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import gemm as gm
from ._ext import load_c

ACT = {"linear": 0, None: 0, "relu": 1, "tanh": 2, "sigmoid": 3}


def _act_torch(name, z):
    if name == "relu":
        return torch.relu(z)
    if name == "tanh":
        return torch.tanh(z)
    if name == "sigmoid":
        return torch.sigmoid(z)
    return z


def _act_grad(name, y, dy):
    if name == "relu":
        return dy * (y > 0)
    if name == "tanh":
        return dy * (1 - y * y)
    if name == "sigmoid":
        return dy * y * (1 - y)
    return dy


def supported(K: int, N: int) -> bool:
    return bool(load_c().dense_supported(int(K), int(N)))


def rowgemm(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None, act: str = "linear",
            out_bf16: bool = False) -> torch.Tensor:
    """act(x . W + b) for 2-D ``x`` on the device (K1)."""
    return load_c().dense_fwd(x, W.contiguous(), None if b is None else b.contiguous(), ACT[act], out_bf16)


def wgrad(x: torch.Tensor, dy: torch.Tensor, shift_T: int = 0, want_db: bool = True
          ) -> Tuple[torch.Tensor, torch.Tensor]:
    """(x^T . dy, colsum(dy)) over all rows (K2); ``shift_T`` reads x one row earlier within each
    length-``shift_T`` sequence (zero at sequence starts)."""
    return tuple(load_c().dense_wgrad(x, dy, int(shift_T), bool(want_db)))


class DenseFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, W, b, act: str):
        y = rowgemm(x2, W, b, act)
        ctx.save_for_backward(x2, W, y)
        ctx.act = act
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, W, y = ctx.saved_tensors
        dz = _act_grad(ctx.act, y, dy.contiguous()).contiguous()
        dW = db = dx = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dW, db = wgrad(x2, dz, 0, ctx.has_b)
        if ctx.needs_input_grad[0]:
            dx = rowgemm(dz, W.t().contiguous())
        return dx, dW, (db if ctx.has_b else None), None


class GemmDenseFunction(torch.autograd.Function):
    """Dense layer on the general MFMA GEMM (layers wider than the K1/K2 register tile)."""

    @staticmethod
    def forward(ctx, x2, W, b, act: str):
        y = gm.matmul(x2, W, b, act)
        ctx.save_for_backward(x2, W, y)
        ctx.act = act
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, W, y = ctx.saved_tensors
        dz = _act_grad(ctx.act, y, dy.contiguous()).contiguous()
        dW = db = dx = None
        if ctx.needs_input_grad[1]:
            dW = gm.matmul(x2.t(), dz)           # split over the rows, deterministic
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = dz.sum(0)
        if ctx.needs_input_grad[0]:
            dx = gm.matmul(dz, W.t())            # W^T read in place
            if x2.dtype != dx.dtype:
                dx = dx.to(x2.dtype)
        return dx, dW, db, None


def dense(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None, act: str = "linear") -> torch.Tensor:
    """Dense layer over the last axis of ``x`` (any leading shape)."""
    K, N = W.shape
    lead = x.shape[:-1]
    if x.is_cuda and supported(K, N) and N >= 1:
        x2 = x.reshape(-1, K)
        if x2.dtype not in (torch.float32, torch.bfloat16):
            x2 = x2.float()
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        return DenseFunction.apply(x2, W, b, act).reshape(*lead, N)
    if x.is_cuda:   # wider layers: general MFMA GEMM (bias + activation in its epilogue)
        x2 = x.reshape(-1, K)
        if x2.dtype not in (torch.float32, torch.bfloat16):
            x2 = x2.float()
        return GemmDenseFunction.apply(x2, W, b, act).reshape(*lead, N)
    z = x @ W
    if b is not None:
        z = z + b
    return _act_torch(act, z)
