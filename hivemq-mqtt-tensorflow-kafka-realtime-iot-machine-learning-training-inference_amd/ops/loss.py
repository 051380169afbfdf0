"""Fused MSE loss + categorical accuracy (K3 + K6, ``csrc/kernels/loss.hip``).

``mse_accuracy(y_pred, y)`` returns ``(loss, correct)`` where ``loss`` is the
Keras ``mean_squared_error`` (differentiable; its backward is the gradient the
forward pass already wrote) and ``correct`` the number of rows whose argmax
matches (per-sample mean over broadcast steps, summed) -- one kernel instead of
the ~10 elementwise / reduction launches the torch expression costs per step.
"""
from __future__ import annotations

import torch

from ._ext import load_c


class MSEAccuracy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y_pred, y, bcast: int):
        yp = y_pred.contiguous()
        n = yp.numel()
        grad = torch.empty_like(yp)
        acc = torch.empty(2, device=yp.device)
        load_c().mse_acc(yp, y.contiguous(), int(bcast), 2.0 / n, grad, acc, reset=True)
        ctx.save_for_backward(grad)
        correct = acc[1] / float(bcast)
        ctx.mark_non_differentiable(correct)
        return acc[0] / n, correct

    @staticmethod
    def backward(ctx, g_loss, g_correct):
        (grad,) = ctx.saved_tensors
        return grad * g_loss, None, None


def supported(F: int) -> bool:
    return bool(load_c().mse_acc_supported(int(F)))


def torch_mse_accuracy(y_pred: torch.Tensor, y: torch.Tensor):
    """Reference / CPU path with identical semantics."""
    if y_pred.dim() == 3 and y.dim() == 2:
        y = y.unsqueeze(1)
    yb = torch.broadcast_to(y, y_pred.shape)
    loss = ((y_pred - yb) ** 2).mean()
    correct = (torch.argmax(y_pred, -1) == torch.argmax(yb, -1)).float()
    if correct.dim() > 1:
        return loss, correct.mean(dim=tuple(range(1, correct.dim()))).sum()
    return loss, correct.sum()


def mse_accuracy(y_pred: torch.Tensor, y: torch.Tensor):
    F = y_pred.shape[-1]
    if y_pred.is_cuda and y_pred.dtype == torch.float32 and supported(F):
        if y_pred.dim() == 3 and y.dim() == 2:
            bcast = y_pred.shape[1]
        elif y_pred.shape == y.shape:
            bcast = 1
        else:
            return torch_mse_accuracy(y_pred, y)
        return MSEAccuracy.apply(y_pred, y.float(), bcast)
    return torch_mse_accuracy(y_pred, y)
