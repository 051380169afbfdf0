"""Same-box A/B of the direct fused step on fresh rows (33.5 M-row batches, every row trained
once): SML_AE_DIRECT_PAIRS=0 (one-tile loop, in-kernel normalise + argmax) vs 1 (packed pairs
on raw rows), alternated in one process (the launcher reads the switch per launch).  Also the
headline step (K8 pack once + packed-pair kernel) for reference.  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch


def main():
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.models.reference import init_dense_weights
    from streamml.ops.ae import AESpec, FusedAE
    dev = torch.device("cuda", 0)
    B = 1 << 25
    steps = int(os.environ.get("AB_STEPS", "20"))
    data = synthetic_device_tensor(2 * B, dev, seed=0)
    spec = AESpec()
    sc, sh = normalize_affine()
    ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), dev, scale=sc, shift=sh)
    for k in range(150):   # DPM clock settle
        ae.step(data[(k % 2) * B:(k % 2 + 1) * B])
    torch.cuda.synchronize()
    res = {"0": [], "1": []}
    for rep in range(3):
        for v in ("0", "1"):
            os.environ["SML_AE_DIRECT_PAIRS"] = v
            for k in range(4):
                ae.step(data[(k % 2) * B:(k % 2 + 1) * B])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                ae.step(data[(k % 2) * B:(k % 2 + 1) * B])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            res[v].append(round(B / dt / 1e9, 3))
    ae.attach_ring(data[:B], B)
    for _ in range(20):
        ae.step_ring()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ae.step_ring()
    torch.cuda.synchronize()
    packed = B / ((time.perf_counter() - t0) / steps) / 1e9
    print(json.dumps({"direct_one_tile_G_rows_s": res["0"], "direct_pairs_G_rows_s": res["1"],
                      "packed_ring_G_rows_s": round(packed, 3), "batch": B, "steps": steps}), flush=True)


if __name__ == "__main__":
    main()
