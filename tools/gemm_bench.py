"""Time the general MFMA GEMM (ops/gemm.py, csrc/kernels/gemm.hip) against torch.matmul
(hipBLASLt) on the shapes it serves: wide Dense forward / dX / split-K dW over many rows,
and square products for the compute ceiling.  One JSON line per shape.

    python tools/gemm_bench.py [--iters 20] [--out gpurun_out/gemm_bench.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamml.ops import gemm as gm  # noqa: E402

SHAPES = [
    # name, M, K, N, a transposed view, operand dtype
    ("dense_fwd_784x128", 65536, 784, 128, False, torch.float32),
    ("dense_dx_128x784", 65536, 128, 784, False, torch.float32),
    ("dense_dw_xT_dz", 784, 65536, 128, True, torch.float32),
    ("wide_fwd_512x512_bf16", 262144, 512, 512, False, torch.bfloat16),
    ("lstm_proj_300x512", 200000, 300, 512, False, torch.float32),
    ("square_4096_bf16", 4096, 4096, 4096, False, torch.bfloat16),
    ("square_8192_bf16", 8192, 8192, 8192, False, torch.bfloat16),
]


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    lines = []
    for name, M, K, N, a_t, dt in SHAPES:
        if a_t:   # x^T . dy: x stored [K_contract, M] row-major, used transposed
            a = torch.randn(K, M, device=dev, generator=g, dtype=torch.float32).to(dt).t()
        else:
            a = torch.randn(M, K, device=dev, generator=g, dtype=torch.float32).to(dt)
        b = torch.randn(K, N, device=dev, generator=g, dtype=torch.float32).to(dt)
        ours = _time(lambda: gm.matmul(a, b), args.iters)
        # the vendor reference on the same bf16 operands (hipBLASLt bf16 GEMM, fp32 out)
        ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
        lib = _time(lambda: torch.matmul(ab, bb).float(), args.iters)
        lib_conv = _time(lambda: torch.matmul(a.to(torch.bfloat16), b.to(torch.bfloat16)).float(), args.iters)
        flop = 2.0 * M * K * N
        rec = {"shape": name, "M": M, "K": K, "N": N, "a_transposed": a_t, "dtype": str(dt).split(".")[-1],
               "ours_ms": round(ours, 4), "ours_tflops": round(flop / ours / 1e9, 1),
               "hipblaslt_bf16_ms": round(lib, 4), "hipblaslt_incl_cast_ms": round(lib_conv, 4),
               "ours_vs_hipblaslt": round(lib / ours, 3),
               "ours_vs_hipblaslt_incl_cast": round(lib_conv / ours, 3)}
        print(json.dumps(rec), flush=True)
        lines.append(rec)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
