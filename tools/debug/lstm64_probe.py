"""U=64 fused LSTM: per-output relative error vs the bf16-rounding oracle at several B (probe)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from helpers.bf16_ref import lstm_fused_bf16_reference, relerr  # noqa: E402
from streamml.ops.lstm import FusedLSTMFunction  # noqa: E402

dev = torch.device("cuda", 0)
cus = torch.cuda.get_device_properties(dev).multi_processor_count
for u, inp in ((64, 18), (32, 18)):
    for B in (70, 1000, 64 * cus + 5, 64 * cus * 2 + 37):
        T = 3
        rng = np.random.default_rng(u + B)
        x = torch.tensor(rng.uniform(-1, 1, (B, T, inp)), dtype=torch.float32)
        W = torch.tensor(rng.standard_normal((inp, 4 * u)) * 0.25, dtype=torch.float32)
        U = torch.tensor(rng.standard_normal((u, 4 * u)) * 0.25, dtype=torch.float32)
        b = torch.tensor(rng.standard_normal(4 * u) * 0.1, dtype=torch.float32)
        gy = torch.tensor(rng.standard_normal((B, T, u)), dtype=torch.float32)
        d = [t.to(dev).requires_grad_(True) for t in (x, W, U, b)]
        y = FusedLSTMFunction.apply(*d, 1, False)
        (y.float() * gy.to(dev)).sum().backward()
        hseq, dx, dW, dU, db = lstm_fused_bf16_reference(x, W, U, b, "relu", dh=gy, last_only=False, db_bf16=True)
        e = {n: relerr(a.cpu(), r) for n, a, r in (("y", y.detach(), hseq), ("dx", d[0].grad, dx), ("dW", d[1].grad, dW),
                                                      ("dU", d[2].grad, dU), ("db", d[3].grad, db))}
        # per-tile split of dW: contribution differences per 16-sequence tile are not observable
        # directly; report the max abs diff location
        diff = (d[1].grad.cpu().double() - dW).abs()
        print(u, B, " ".join("%s=%.2e" % kv for kv in e.items()), "dW maxdiff %.3e at %s" % (
            diff.max().item(), np.unravel_index(diff.argmax().item(), diff.shape)), flush=True)
