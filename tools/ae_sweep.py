"""Kernel-level sweep of the fused AE train step (one process, interleaved rounds).

Times kernel-1 + reduce/Adam with HIP events for several (batch, max_blocks)
configurations so variants are compared on the same device in the same process.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from streamml.data.cardata import normalize_affine, synthetic_device_tensor
from streamml.models.reference import init_dense_weights
from streamml.ops.ae import AESpec, FusedAE


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="65536,262144,1048576,4194304")
    ap.add_argument("--blocks", default="256,512,1024,2048")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = AESpec()
    scale, shift = normalize_affine()
    batches = [int(b) for b in args.batches.split(",")]
    blocks = [int(b) for b in args.blocks.split(",")]
    rows = max(batches) * 4
    data = synthetic_device_tensor(rows, dev, seed=0)
    w = init_dense_weights(spec.layer_sizes, 0)
    fused = {mb: FusedAE(spec, w, dev, max_blocks=mb, scale=scale, shift=shift) for mb in blocks}
    res = {}
    for r in range(args.rounds):
        for B in batches:
            for mb in blocks:
                f = fused[mb]
                for i in range(3):
                    f.step(data[(i % 4) * B:(i % 4 + 1) * B])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(args.iters):
                    f.step(data[(i % 4) * B:(i % 4 + 1) * B])
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                res.setdefault((B, mb), []).append(us)
    out = []
    for (B, mb), v in sorted(res.items()):
        us = float(np.median(v))
        out.append({"batch": B, "max_blocks": mb, "us_per_step": us, "grows_per_s": B / us / 1e3})
        print(f"B={B:>8} blocks={mb:>5}  {us:9.1f} us/step  {B / us / 1e3:7.2f} G rows/s", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/ae_sweep.json", "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
