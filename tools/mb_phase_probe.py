"""Cycle split of the persistent batch-32 trainer (csrc/kernels/ae_minibatch.hip), one launch of
20 000 steps per build: the pipelined build reports wave 0's W1 wait and wave 4's W1 tile time
(prof[4], prof[5]); the two-barrier build its phase split (prof[0..3]).  Shader-clock cycles
per step (s_memtime / readcyclecounter)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamml.data.cardata import normalize_affine  # noqa: E402
from streamml.models.reference import init_dense_weights  # noqa: E402
from streamml.ops.ae import AESpec, FusedAE  # noqa: E402

dev = torch.device("cuda", 0)
spec = AESpec()
scale, shift = normalize_affine()
raw = torch.rand((32 * 4096, 18), device=dev) * 40.0
steps = 20000
for pipe in ("1", "0"):
    os.environ["SML_MB_PIPE"] = pipe
    ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), dev, scale=scale, shift=shift)
    ae.attach_ring(raw, 32)
    ae.train_minibatches(2000)   # warm
    prof = torch.zeros(11, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ae.train_minibatches(steps, prof=prof)
    torch.cuda.synchronize()
    p = (prof.double() / steps).tolist()
    if pipe == "1":
        out = {"build": "pipelined", "total": p[8], "wave0_wait_w1": p[4], "wave0_chain": p[8] - p[4],
               "w1_tile_wait_to_bump": p[5]}
    else:
        out = {"build": "two-barrier", "total": p[8], "phase_a": p[0], "barrier1": p[1], "phase_b": p[2], "barrier2": p[3]}
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
