"""Per-op device time of the two-layer LSTM step's head and loss (B = 65 536): the Dense
head GEMM, the fused MSE + accuracy kernel with and without its atomic accumulator, the head
weight gradient, dh = dy . K^T and the accumulator reset -- which of the ~110 us of small
kernels per step (profiles/r04 SUMMARY section 3) is worth fusing.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch


def timed(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3   # us per call


def main():
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops._ext import load_c
    C = load_c()
    dev = torch.device("cuda", 0)
    B, T = 65536, 50
    m = LSTMPredictor.two_layer(look_back=T, device=dev, seed=0)
    plan = m._fused_plan()
    hd = plan["head"]
    K, bh = (t.detach() for t in m.fp.params[hd["params"]:hd["params"] + 2])
    h = torch.randn(B, T, 16, device=dev).to(torch.bfloat16)
    hin = h[:, -1]
    y = torch.randn(B, 18, device=dev)
    acc = torch.zeros(2, device=dev)
    yp = C.dense_fwd(hin, K, bh, 0, False, 1024, False)
    dy = torch.empty_like(yp)
    out = {
        "dense_fwd_us": timed(lambda: C.dense_fwd(hin, K, bh, 0, False, 1024, False)),
        "mse_acc_us": timed(lambda: C.mse_acc(yp, y, 1, 1e-5, dy, acc)),
        "mse_noacc_us": timed(lambda: C.mse_acc(yp, y, 1, 1e-5, dy, None)),
        "dense_wgrad_us": timed(lambda: C.dense_wgrad(hin, dy, 0, True, 1024, m.fp.grad, plan["head_map"])),
        "dense_dh_us": timed(lambda: C.dense_fwd(dy, K, None, 0, True, 1024, True)),
        "acc_zero_us": timed(lambda: acc.zero_()),
        "y_to_contig_us": timed(lambda: y[:, :].to(device=dev, dtype=torch.float32).contiguous()),
    }
    print(json.dumps({k: round(v, 2) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
