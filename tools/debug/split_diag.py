"""Split LSTM backward vs the one-wave kernel over shapes: per-output relative errors (diagnosis)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_lstm_split_gpu import _case, _relerr  # noqa: E402

dev = torch.device("cuda", 0)
for (B, T, IN, windows) in [(16, 1, 18, False), (16, 2, 18, False), (16, 3, 18, False), (16, 5, 18, False),
                            (16, 1, 17, False), (16, 2, 17, False), (16, 1, 12, False), (16, 1, 13, False),
                            (16, 1, 24, False), (32, 1, 18, False), (1007, 1, 18, True), (1007, 50, 18, True),
                            (16, 5, 17, False)]:
    for act in (1,):
        C, x, W, U, b, h0, c0, h, c, rng = _case(dev, B, T, IN, act, False, windows, 1)
        dh = torch.tensor(rng.standard_normal((B, T, 32)), dtype=torch.float32, device=dev).to(torch.bfloat16)
        out = {}
        for v in ("1", "0"):
            os.environ["SML_LSTM_SPLIT"] = v
            out[v] = C.lstm_fused_bwd(dh, c, h, x, h0, c0, W, U, b, act, False, True, False)
        torch.cuda.synchronize()
        errs = {n: round(_relerr(g, r), 5) for n, g, r in zip(("dW", "dU", "db", "dh0", "dc0"), out["1"][1:], out["0"][1:])}
        print(B, T, IN, windows, errs, flush=True)
        if T == 1 and IN == 18 and B == 16:
            g, r = out["1"][1], out["0"][1]
            print("dW split row0", g[:, 0].cpu().numpy().round(3))
            print("dW ref   row0", r[:, 0].cpu().numpy().round(3))
            print("dh0 split", out["1"][4][0].cpu().numpy().round(3))
            print("dh0 ref  ", out["0"][4][0].cpu().numpy().round(3))
