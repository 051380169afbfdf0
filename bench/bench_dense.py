#!/usr/bin/env python3
"""Microbenchmark of the K1/K2 tall-skinny dense kernels at the LSTM training shapes.

Reports achieved HBM bandwidth (bytes read + written / kernel time) per kernel,
dtype and grid size -- the roofline for these shapes is HBM (~8 TB/s).

    python bench/bench_dense.py [--rows 409600]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=409600)
    args = ap.parse_args()
    from streamml.ops import load_c
    C = load_c()
    dev = torch.device("cuda", 0)
    M = args.rows
    out = []
    shapes = [("proj1", 18, 128), ("proj2", 32, 64), ("dU1", 32, 128), ("dU2", 16, 64), ("dx2", 64, 32),
              ("head", 16, 18)]
    for name, K, N in shapes:
        for dt in (torch.float32, torch.bfloat16):
            x = torch.randn(M, K, device=dev).to(dt)
            W = torch.randn(K, N, device=dev)
            b = torch.randn(N, device=dev)
            dy = torch.randn(M, N, device=dev).to(dt)
            for ob in (False, True):
                t = timeit(lambda: C.dense_fwd(x, W, b, 0, ob))
                byt = M * K * x.element_size() + M * N * (2 if ob else 4)
                out.append({"kernel": "rowgemm", "shape": name, "K": K, "N": N, "in": str(dt)[6:],
                            "out": "bf16" if ob else "fp32", "us": round(t, 1), "TB/s": round(byt / t / 1e6, 2)})
            for mb in (256, 512, 1024, 2048, 4096):
                t = timeit(lambda: C.dense_wgrad(x, dy, 0, True, mb))
                byt = M * K * x.element_size() + M * N * dy.element_size()
                out.append({"kernel": "wgrad", "shape": name, "K": K, "N": N, "in": str(dt)[6:], "max_blocks": mb,
                            "us": round(t, 1), "TB/s": round(byt / t / 1e6, 2)})
            t = timeit(lambda: (x.float() @ W).sum() if False else torch.mm(x, W.to(dt)))
            out.append({"kernel": "hipblaslt_fwd", "shape": name, "K": K, "N": N, "in": str(dt)[6:], "us": round(t, 1),
                        "TB/s": round((M * K + M * N) * x.element_size() / t / 1e6, 2)})
            t = timeit(lambda: torch.mm(x.t(), dy))
            out.append({"kernel": "hipblaslt_wgrad", "shape": name, "K": K, "N": N, "in": str(dt)[6:],
                        "us": round(t, 1), "TB/s": round((M * K + M * N) * x.element_size() / t / 1e6, 2)})
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
