"""Fresh rows (each trained once): K8 pack + packed-pair kernel vs the direct fused step
(normalize_fn and argmax inside the unpacked train kernel), 33.5 M-row batches."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.models.reference import init_dense_weights
    from streamml.ops.ae import AESpec, FusedAE
    dev = torch.device("cuda", 0)
    B = 1 << 25
    data = synthetic_device_tensor(2 * B, dev, seed=0)
    spec = AESpec()
    sc, sh = normalize_affine()
    ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), dev, scale=sc, shift=sh)
    out = {}
    for name, fn in (("pack+packed_kernel", lambda k: (ae.pack_ring(data[(k % 2) * B:(k % 2 + 1) * B], B),
                                                       ae.step_ring())),
                     ("direct_step", lambda k: ae.step(data[(k % 2) * B:(k % 2 + 1) * B]))):
        for k in range(60):   # settle + warm
            fn(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(20):
            fn(k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        out[name] = {"ms_per_step": dt * 1e3, "G_rows_per_s": B / dt / 1e9}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
