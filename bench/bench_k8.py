#!/usr/bin/env python3
"""K8 ingest-transform kernels (csrc/kernels/preprocess.hip) at the headline's step size.

Times, on ``--rows`` raw [n, 18] fp32 car-sensor rows resident in HBM:
  pack     -- pack_tiles_argmax: normalize_fn + argmax(x) + 16-row tile packing (bench.py's ring)
  argmax   -- row_argmax_u8: one byte per row
  filter   -- normalize_filter: label predicate + order-preserving compaction (cardata-v3.py:212)
Each as ms per call and effective HBM TB/s (bytes read + written once).  One JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 25)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import numpy as np
    import torch
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.ops._ext import load_c

    C = load_c()
    dev = torch.device("cuda", 0)
    n, D = args.rows, 18
    x = synthetic_device_tensor(n, dev, seed=0)
    sc, sh = normalize_affine()
    tsc = torch.tensor(sc, dtype=torch.float32, device=dev)
    tsh = torch.tensor(sh, dtype=torch.float32, device=dev)
    labels = (torch.rand(n, device=dev) < 0.01).to(torch.uint8)
    out = {"rows": n, "features": D}
    t = _time(lambda: C.pack_tiles_argmax(x, D, tsc, tsh), args.iters)
    byts = n * D * 4 + n // 16 * (64 * D + 16)
    out["pack_ms"] = t * 1e3
    out["pack_tb_s"] = byts / t / 1e12
    t = _time(lambda: C.row_argmax_u8(x, D, tsc, tsh), args.iters)
    out["argmax_ms"] = t * 1e3
    out["argmax_tb_s"] = (n * D * 4 + n) / t / 1e12
    kept = int((labels == 0).sum().item())
    t = _time(lambda: C.normalize_filter(x, D, labels, 0, tsc, tsh, False), args.iters)
    out["filter_ms"] = t * 1e3
    out["filter_tb_s"] = (n * D * 4 + n + kept * D * 4) / t / 1e12
    out["filter_kept"] = kept
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
