"""A/B of the small-batch trainer's phase A precision (SML_MB_BF16, read per launch): fp32
(Keras-exact) vs bf16 MFMA contractions.  Rates for Autoencoder.fit(batch_size=100) (the bench's
fit_batch100), keras_batch32 (D = 18) and the BASELINE model (D = 30, batch 32); numerics: the
same 400 steps from one init, parameter / loss differences between the two precisions."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from streamml.data.cardata import normalize_affine, synthetic_device_tensor  # noqa: E402
from streamml.models.reference import init_dense_weights  # noqa: E402
from streamml.ops.ae import AESpec, FusedAE  # noqa: E402

dev = torch.device("cuda", 0)


def numerics(D, B, steps=400):
    spec = AESpec(D, 14, 7)
    if D == 18:
        sc, sh = normalize_affine()
        ring = synthetic_device_tensor(B * 64, dev, seed=3)
    else:
        sc = sh = None
        ring = torch.randn(B * 64, D, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    out = {}
    for bf in ("0", "1"):
        os.environ["SML_MB_BF16"] = bf
        ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=1), dev, scale=sc, shift=sh)
        ae.attach_ring(ring.contiguous(), B)
        ae.train_minibatches(steps)
        torch.cuda.synchronize()
        out[bf] = (ae.params.clone(), ae.read_metrics())
    p0, m0 = out["0"]
    p1, m1 = out["1"]
    rel = float((p1 - p0).norm() / p0.norm())
    return {"D": D, "batch": B, "steps": steps, "param_rel_diff": rel, "loss_fp32": m0["loss"], "loss_bf16": m1["loss"]}


res = {"numerics": [numerics(18, 100), numerics(18, 32), numerics(30, 32)]}
for bf in ("0", "1"):
    os.environ["SML_MB_BF16"] = bf
    r = {"fit_batch100": bench.measure_fit(dev, 2_000_000)["rows_per_s"]}
    spec = AESpec()
    sc, sh = normalize_affine()
    data = synthetic_device_tensor(1 << 20, dev, seed=0)
    r["keras_batch32"] = bench.measure_batch32(spec, data, dev, 20000, sc, sh, 0)["rows_per_s"]
    r["keras_batch32_d30"] = bench.measure_batch32_d30(dev, 20000, 0)["rows_per_s"]
    res["bf16" if bf == "1" else "fp32"] = r
print(json.dumps(res))
