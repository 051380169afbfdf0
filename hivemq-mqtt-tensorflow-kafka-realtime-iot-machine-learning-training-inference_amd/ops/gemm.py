"""General GEMM on the hand-written LDS-tiled MFMA kernel (``csrc/kernels/gemm.hip``).

``matmul(a, b, bias, act)`` computes ``act(a @ b + bias)`` for 2-D device tensors of any
shape: fp32 or bf16 operands (bf16 MFMA, fp32 accumulation), either orientation --
transposed views such as ``x.t()`` are read in place, no copy.  Small outputs with a long
contraction (weight gradients ``x.t() @ dy`` over many rows) are split over K and reduced
deterministically.  This is the path for every GEMM wider than the register-resident K1/K2
tiles of ``dense.hip`` (ops/dense.py, ops/lstm.py); on CPU it is ``torch`` matmul.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import load_c

ACT = {"linear": 0, None: 0, "relu": 1, "tanh": 2, "sigmoid": 3}


def matmul(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, act: str = "linear",
           out_bf16: bool = False, splits: int = -1) -> torch.Tensor:
    """act(a @ b + bias): a [M, K], b [K, N]; fp32 result unless ``out_bf16``."""
    if not a.is_cuda:
        z = a.float() @ b.float()
        if bias is not None:
            z = z + bias
        if act == "relu":
            z = torch.relu(z)
        elif act == "tanh":
            z = torch.tanh(z)
        elif act == "sigmoid":
            z = torch.sigmoid(z)
        return z.to(torch.bfloat16) if out_bf16 else z
    if a.dtype not in (torch.float32, torch.bfloat16):
        a = a.float()
    if b.dtype not in (torch.float32, torch.bfloat16):
        b = b.float()
    return load_c().gemm(a, b, None if bias is None else bias.float().contiguous(), ACT[act], bool(out_bf16),
                         int(splits))
