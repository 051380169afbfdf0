"""LSTM layer on HIP: fully fused layer kernels (default) or projection + recurrence.

Default path (:class:`FusedLSTMFunction`, ``csrc/kernels/lstm_fused.hip``): one
kernel for the forward pass (input projection, recurrence, bf16 gate save) and one
for the backward pass (BPTT, weight gradients accumulated in registers, dX).  U = 64
layers keep the one-launch forward; their backward stores dz (bf16) and a second
hand-written kernel (``lstm_dz_wgrad_kernel``, split over gate groups) contracts it,
since 4U x (16 KT + U) weight-gradient accumulators do not fit one wave's registers.
Fallback for shapes without a fused instance (:class:`LSTMFunction`): K1/K2
projection kernels (the general MFMA GEMM for wide layers) + the recurrence-only kernels
described below (U = 128: four waves share each 16-sequence tile).  Widths other than
16 / 32 / 64 / 128 are zero-padded to the next of them (:func:`pad_lstm_weights`: exact).

Fallback forward: Zx = X.W + b over all B*T rows (K1 ``dense_fwd``), then the
``lstm_fwd`` kernel runs the recurrence (U.h MFMAs + gates + state update per
step, h/c in registers).  Fallback backward: the ``lstm_bwd`` kernel walks time
backwards producing the pre-activation gate gradients dz for every step; dW, dU,
db and dX are then K2 ``dense_wgrad`` / K1 passes over the B*T rows.

Keras LSTM semantics (recurrent_activation sigmoid, gate order i,f,c,o,
``activation`` for the candidate and the cell output), reference
LSTM-TensorFlow-IO-Kafka/cardata-v2.py:177-183.  ``lstm_reference`` is the plain
torch oracle / CPU path.
"""
from __future__ import annotations

import torch

from . import dense as dn
from . import gemm as gm
from ._ext import load_c

ACT = {"relu": 1, "tanh": 2}


def _act(name: str):
    return torch.relu if name == "relu" else torch.tanh


def lstm_reference(x: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor, activation: str = "relu",
                   h0=None, c0=None) -> torch.Tensor:
    """[B, T, in] -> h sequence [B, T, u] (differentiable torch ops)."""
    B, T, _ = x.shape
    u = U.shape[0]
    h = x.new_zeros(B, u) if h0 is None else h0
    c = x.new_zeros(B, u) if c0 is None else c0
    act = _act(activation)
    zx = x @ W + b
    hs = []
    for t in range(T):
        z = zx[:, t] + h @ U
        i, f, g, o = z.split(u, dim=-1)
        i, f, o = torch.sigmoid(i), torch.sigmoid(f), torch.sigmoid(o)
        c = f * c + i * act(g)
        h = o * act(c)
        hs.append(h)
    return torch.stack(hs, dim=1)


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 MFMA GEMM, fp32 result, on the general LDS-tiled kernel (``ops/gemm.py``) for
    shapes beyond the K1/K2 register tile; transposed views are read in place."""
    return gm.matmul(a, b)


class LSTMFunction(torch.autograd.Function):
    """Input projection / weight gradients / dX on the K1/K2 tall-skinny kernels
    (the general MFMA GEMM when a layer is too wide for them), recurrence on lstm_fwd/lstm_bwd."""

    @staticmethod
    def forward(ctx, x, W, U, b, act_code: int):
        B, T, inp = x.shape
        u = U.shape[0]
        x2 = x.reshape(B * T, inp)
        fast = dn.supported(inp, 4 * u) and dn.supported(4 * u, inp)
        if fast:
            zx = dn.rowgemm(x2, W, b).reshape(B, T, 4 * u)
        else:
            zx = gm.matmul(x2, W, b).reshape(B, T, 4 * u)
        h, c, gates = load_c().lstm_fwd(zx, U.contiguous(), None, None, act_code)
        ctx.save_for_backward(x, W, U, h, c, gates)
        ctx.act = act_code
        ctx.fast = fast
        return h

    @staticmethod
    def backward(ctx, dh):
        x, W, U, h, c, gates = ctx.saved_tensors
        B, T, inp = x.shape
        u = U.shape[0]
        (dz,) = load_c().lstm_bwd(dh.contiguous().float(), gates, c, None, U.contiguous(), ctx.act, False)
        dz2 = dz.reshape(B * T, 4 * u)
        x2 = x.reshape(B * T, inp)
        h2 = h.reshape(B * T, u)
        dW = dU = db = dx = None
        if ctx.fast:
            if ctx.needs_input_grad[1] or ctx.needs_input_grad[3]:
                dW, db = dn.wgrad(x2, dz2)                       # one pass: X^T.dz and colsum(dz)
            if ctx.needs_input_grad[2]:
                dU, _ = dn.wgrad(h2, dz2, shift_T=T, want_db=False)   # h_{t-1}^T . dz, no copy of h
            if ctx.needs_input_grad[0]:
                dx = dn.rowgemm(dz2, W.t().contiguous()).reshape(B, T, inp)
            return dx, dW, dU, db, None
        dW = _mm(x2.t(), dz2) if ctx.needs_input_grad[1] else None
        if ctx.needs_input_grad[2]:
            hprev = torch.cat([h.new_zeros(B, 1, u), h[:, :-1]], dim=1).reshape(B * T, u)
            dU = _mm(hprev.t(), dz2)
        db = dz2.sum(0) if ctx.needs_input_grad[3] else None
        dx = _mm(dz2, W.t()).reshape(B, T, inp) if ctx.needs_input_grad[0] else None
        return dx, dW, dU, db, None


class FusedLSTMFunction(torch.autograd.Function):
    """Whole layer in two launches: ``lstm_fused_fwd`` (x.W + recurrence, bf16 cell
    state saved) and ``lstm_fused_bwd`` (gate recompute + BPTT + dW/dU/db accumulated
    in registers + dX).  ``x`` may be fp32 (model input) or bf16 (a lower layer's h);
    the h sequence comes back in bf16 -- every consumer feeds it to bf16 MFMAs -- and
    ``dx`` in x's dtype.  ``last_only`` (Keras ``return_sequences=False``) returns h_T
    [B, U] in fp32; its backward reads only that [B, U] gradient instead of a
    [B, T, U] tensor of zeros."""

    @staticmethod
    def forward(ctx, x, W, U, b, act_code: int, last_only: bool = False):
        h, c = load_c().lstm_fused_fwd(x, W.contiguous(), U.contiguous(), b.contiguous(), None, None, act_code)
        ctx.save_for_backward(x, W, U, b, h, c)
        ctx.act = act_code
        ctx.last_only = bool(last_only)
        return h[:, -1].float() if last_only else h

    @staticmethod
    def backward(ctx, dh):
        x, W, U, b, h, c = ctx.saved_tensors
        dx, dW, dU, db, _, _ = load_c().lstm_fused_bwd(dh.contiguous().to(torch.bfloat16), c, h, x, None, None,
                                                       W.contiguous(), U.contiguous(), b.contiguous(), ctx.act,
                                                       bool(ctx.needs_input_grad[0]), False, ctx.last_only)
        return (dx if ctx.needs_input_grad[0] else None), dW, dU, db, None, None


def fused_supported(units: int, in_features: int) -> bool:
    return bool(load_c().lstm_fused_supported(int(units), int(in_features)))


KERNEL_UNITS = (16, 32, 64, 128)   # widths the recurrence kernels are built for


def padded_units(units: int):
    """Smallest kernel width >= ``units`` (None beyond 128)."""
    for p in KERNEL_UNITS:
        if units <= p:
            return p
    return None


def _pad_gates(t: torch.Tensor, u: int, up: int) -> torch.Tensor:
    """[..., 4u] Keras gate columns (i | f | c~ | o) -> [..., 4up], gate block k at
    columns [k up, k up + u), zeros elsewhere (differentiable)."""
    lead = t.shape[:-1]
    return torch.nn.functional.pad(t.reshape(*lead, 4, u), (0, up - u)).reshape(*lead, 4 * up)


def pad_lstm_weights(W: torch.Tensor, U: torch.Tensor, b: torch.Tensor, up: int):
    """Zero-pad a u-unit layer to ``up`` units.  The padded units have zero weights and
    bias, so from zero state their gates are i = f = o = 1/2, g~ = act(0) = 0: c and h
    stay exactly 0 and feed nothing into the real units -- the real units' outputs and
    gradients are those of the unpadded layer."""
    u = U.shape[0]
    Wp = _pad_gates(W, u, up)
    Up = torch.nn.functional.pad(_pad_gates(U, u, up), (0, 0, 0, up - u))
    return Wp, Up, _pad_gates(b, u, up)


def lstm(x: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor, activation: str = "relu",
         fused: bool = True, return_sequences: bool = True) -> torch.Tensor:
    """Device-dispatching LSTM layer: fused HIP kernels on ROCm, torch reference on CPU.
    ``return_sequences=False`` returns h_T [B, U] (Keras semantics)."""
    if x.is_cuda:
        u = U.shape[0]
        if u not in KERNEL_UNITS:
            up = padded_units(u)
            if up is None:   # wider than any kernel: torch ops (counted; SML_STRICT_KERNELS=1 refuses)
                from ._ext import note_fallback
                note_fallback(f"lstm[{u} units]")
                hs = lstm_reference(x.float(), W, U, b, activation)
                return hs if return_sequences else hs[:, -1]
            Wp, Upad, bp = pad_lstm_weights(W, U, b, up)
            hs = lstm(x, Wp, Upad, bp, activation, fused, return_sequences)
            return hs[..., :u]
        if fused and fused_supported(U.shape[0], x.shape[-1]):
            # sliding windows (consecutive rows per step, any sequence stride) are read
            # in place by the fused kernels: no [B, T, F] materialisation
            windowed = x.dim() == 3 and x.stride(2) == 1 and x.stride(1) == x.shape[2] and x.stride(0) >= 0
            xc = x if windowed else x.contiguous()
            if xc.dtype not in (torch.float32, torch.bfloat16):
                xc = xc.float().contiguous()
            return FusedLSTMFunction.apply(xc, W, U, b, ACT[activation], not return_sequences)
        hs = LSTMFunction.apply(x.contiguous().float(), W, U, b, ACT[activation])
    else:
        hs = lstm_reference(x, W, U, b, activation)
    return hs if return_sequences else hs[:, -1]
