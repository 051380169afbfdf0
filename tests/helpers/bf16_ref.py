"""Torch references that round operands to bf16 at exactly the points the HIP kernels do,
and compute everything else in float64.

The fp32 oracles (``lstm_reference``, ``ae_loss_torch``, ``x @ W``) bound a bf16-MFMA
kernel only to the bf16 floor (a few %).  These references reproduce the kernels'
rounding points -- bf16 MFMA operands, fp32 (here fp64) accumulation, bf16-stored
inter-step tensors -- so what remains between kernel and reference is accumulation
order and the hardware transcendental approximations: relative errors of 1e-4..1e-3.
"""
import math

import torch


def bf(t: torch.Tensor) -> torch.Tensor:
    """round to bf16, continue in float64"""
    return t.to(torch.bfloat16).to(torch.float64)


def _act(name, z):
    return torch.relu(z) if name == "relu" else torch.tanh(z)


def _act_d(name, z, y):
    return (z > 0).double() if name == "relu" else 1.0 - y * y


def lstm_fused_bf16_reference(x, W, U, b, act="relu", dh=None, last_only=False, want_dx=True, db_bf16=False):
    """lstm_fused_fwd.hip + lstm_fused.hip.

    Forward: z = b + bf16(x_t) . bf16(W) + bf16(h_{t-1}) . bf16(U); c in fp32, h and c
    stored bf16 (h feeds the next step as the stored bf16 value).
    Backward: gates recomputed from the same operands; the cell state read back as its
    bf16 copy; dh_t = bf16(dh_in) + U . bf16(dz_{t+1}); dz rounded to bf16 for every
    MFMA consumer (dh recurrence, dx, dW, dU); db = fp32 column sums of dz, or with
    ``db_bf16`` (the kernels' bias-column mode, lstm_fused_impl.h bias_in_x: db is the dW^T
    column of a constant-1 input) of bf16(dz), as dW and dU.
    Returns (h_seq [B, T, u] (bf16 values), dx, dW, dU, db) in float64."""
    B, T, IN = x.shape
    u = U.shape[0]
    xb, Wb, Ub = bf(x), bf(W), bf(U)
    bb = b.double()
    h = torch.zeros(B, u, dtype=torch.float64)
    c = torch.zeros(B, u, dtype=torch.float64)
    hs, cs = [], []
    for t in range(T):
        z = bb + xb[:, t] @ Wb + bf(h) @ Ub
        i, f, g, o = z.split(u, dim=1)
        i, f, o = torch.sigmoid(i), torch.sigmoid(f), torch.sigmoid(o)
        c = f * c + i * _act(act, g)
        h = o * _act(act, c)
        hs.append(bf(h))
        cs.append(bf(c))
    hseq = torch.stack(hs, 1)
    if dh is None:
        return hseq
    dhin = bf(dh.double())
    dW = torch.zeros_like(Wb)
    dU = torch.zeros_like(Ub)
    db = torch.zeros_like(bb)
    dx = torch.zeros(B, T, IN, dtype=torch.float64)
    dhr = torch.zeros(B, u, dtype=torch.float64)
    dcn = torch.zeros(B, u, dtype=torch.float64)
    zero = torch.zeros(B, u, dtype=torch.float64)
    for t in range(T - 1, -1, -1):
        hp = hs[t - 1] if t > 0 else zero
        cp = cs[t - 1] if t > 0 else zero
        z = bb + xb[:, t] @ Wb + hp @ Ub
        zi, zf, zg, zo = z.split(u, dim=1)
        gi, gf, go = torch.sigmoid(zi), torch.sigmoid(zf), torch.sigmoid(zo)
        gc = _act(act, zg)
        if last_only:
            d_in = dhin if t == T - 1 else zero
        else:
            d_in = dhin[:, t]
        dht = d_in + dhr
        ct = cs[t]
        ac = _act(act, ct)
        dc = dcn + dht * go * _act_d(act, ct, ac)
        dz = torch.cat([dc * gc * gi * (1 - gi), dc * cp * gf * (1 - gf),
                        dc * gi * _act_d(act, zg, gc), dht * ac * go * (1 - go)], 1)
        dcn = dc * gf
        dzb = bf(dz)
        db += (dzb if db_bf16 else dz).sum(0)
        dhr = dzb @ Ub.t()
        if want_dx:
            dx[:, t] = dzb @ Wb.t()
        dW += xb[:, t].t() @ dzb
        dU += hp.t() @ dzb
    return hseq, dx, dW, dU, db


def ae_bf16_reference(x, w, l1=1e-7):
    """ae_fused.hip train_tile (the reference 18-14-7-7-18 model: tanh, relu, tanh, relu).

    Weights and biases enter the MFMAs as bf16 (the tanh layers' as bf16(2 log2(e) * w),
    tanh evaluated as 1 - 2 / (2^z' + 1)); every activation is rounded to bf16 before the
    next MFMA; the backward W4 operand is bf16(2/D * W4) against the unscaled bf16(dz4);
    the W4 / b4 gradient sums are scaled by 2/D at the end.  Returns the batch-mean
    gradients [W1, b1, ..., W4, b4] and (sum sq err, sum |h1|) in float64."""
    k1 = 2.0 * math.log2(math.e)
    n, D = x.shape
    W1, b1, W2, b2, W3, b3, W4, b4 = [torch.as_tensor(a).double() for a in w]
    xb = bf(torch.as_tensor(x).double())
    xf = torch.as_tensor(x).double()
    z1s = xb @ bf(k1 * W1) + bf(k1 * b1)
    h1 = 1.0 - 2.0 / (torch.exp2(z1s) + 1.0)
    z2 = bf(h1) @ bf(W2) + bf(b2)
    h2 = torch.relu(z2)
    z3s = bf(h2) @ bf(k1 * W3) + bf(k1 * b3)
    h3 = 1.0 - 2.0 / (torch.exp2(z3s) + 1.0)
    z4 = bf(h3) @ bf(W4) + bf(b4)
    y = torch.relu(z4)
    e = y - xf
    dz4b = bf((y > 0).double() * e)
    dh3 = dz4b @ bf((2.0 / D) * W4).t()
    dz3b = bf((1 - h3 * h3) * dh3)
    dh2 = dz3b @ bf(W3).t()
    dz2b = bf((h2 > 0).double() * dh2)
    dh1 = dz2b @ bf(W2).t()
    dz1b = bf((1 - h1 * h1) * (dh1 + l1 * torch.sign(h1)))
    g = [xb.t() @ dz1b, dz1b.sum(0), bf(h1).t() @ dz2b, dz2b.sum(0), bf(h2).t() @ dz3b, dz3b.sum(0),
         (bf(h3).t() @ dz4b) * (2.0 / D), dz4b.sum(0) * (2.0 / D)]
    return [a / n for a in g], (float((e * e).sum()), float(h1.abs().sum()))


def relerr(a, b) -> float:
    a = torch.as_tensor(a).double().reshape(-1)
    b = torch.as_tensor(b).double().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-30))
