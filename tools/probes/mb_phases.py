"""Per-phase shader cycles of the small-batch trainer (wave 0, model 0; the kernel's prof
counters): phase A, barrier 1, phase B, barrier 2, total -- fp32 vs bf16 contractions."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from streamml.data.cardata import normalize_affine, synthetic_device_tensor  # noqa: E402
from streamml.models.reference import init_dense_weights  # noqa: E402
from streamml.ops.ae import AESpec, FusedAE  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for B in (100, 32):
    for bf in ("0", "1"):
        os.environ["SML_MB_BF16"] = bf
        spec = AESpec()
        sc, sh = normalize_affine()
        ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=1), dev, scale=sc, shift=sh)
        ae.attach_ring(synthetic_device_tensor(B * 256, dev, seed=3).contiguous(), B)
        prof = torch.zeros(11, dtype=torch.int64, device=dev)
        n = 4000
        ae.train_minibatches(n, prof=prof)
        torch.cuda.synchronize()
        p = [int(v) / n for v in prof.cpu().tolist()]
        out[f"b{B}_{'bf16' if bf == '1' else 'fp32'}"] = {"phase_a": p[0], "barrier1": p[1], "phase_b": p[2],
                                                          "barrier2": p[3], "total": p[8]}
print(json.dumps(out))
