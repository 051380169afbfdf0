"""U=64 fused LSTM at B = 64 x CUs x 2 + 37: which sequences' dx deviate from the bf16 oracle (probe)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from helpers.bf16_ref import lstm_fused_bf16_reference  # noqa: E402
from streamml.ops.lstm import FusedLSTMFunction  # noqa: E402

dev = torch.device("cuda", 0)
cus = torch.cuda.get_device_properties(dev).multi_processor_count
u, inp, T = 64, 18, 3
B = 64 * cus * 2 + 37
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
e = (d[0].grad.cpu().double() - dx).abs().amax(dim=(1, 2))
s = (dx.abs().amax(dim=(1, 2)))
bad = torch.nonzero(e > 0.05 * s.clamp(min=1e-3)).flatten().tolist()
print("B", B, "bad sequences", len(bad), bad[:40], flush=True)
print("tiles", sorted(set(i // 16 for i in bad))[:40], flush=True)
ey = (y.detach().float().cpu().double() - hseq).abs().amax(dim=(1, 2))
print("y bad", torch.nonzero(ey > 0.05).flatten().tolist()[:20], flush=True)
