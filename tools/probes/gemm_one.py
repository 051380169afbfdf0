"""One GEMM shape, a few iterations (for rocprofv3 counter passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from streamml.ops import gemm as gm  # noqa: E402

M, K, N = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 4096, 4096)))
dt = torch.bfloat16 if (len(sys.argv) < 5 or sys.argv[4] == "bf16") else torch.float32
a = torch.randn(M, K, device="cuda", dtype=torch.float32).to(dt)
b = torch.randn(K, N, device="cuda", dtype=torch.float32).to(dt)
for _ in range(5):
    gm.matmul(a, b)
torch.cuda.synchronize()
print("ok")
