"""Determinism probe for the headline AE step variants (SML_AE_PAIR_OCC / SML_AE_PAIR_XP): the same
ring, the same weights, full-chip grid, N steps twice per variant; prints whether the gradient
images of the two runs are bit-identical and the relative difference to variant 3:0."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from streamml.data.cardata import normalize_affine  # noqa: E402
from streamml.models.reference import init_dense_weights  # noqa: E402
from streamml.ops.ae import AESpec, FusedAE  # noqa: E402


def run(variant, raw, B, steps):
    o, x = variant.split(":")
    os.environ["SML_AE_PAIR_OCC"] = o
    os.environ["SML_AE_PAIR_XP"] = x
    spec = AESpec()
    scale, shift = normalize_affine()
    f = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=3), raw.device, scale=scale, shift=shift)
    f.attach_ring(raw, B)
    imgs = []
    for _ in range(steps):
        f.step_ring(allreduce=lambda g: imgs.append(g.detach().cpu().numpy().copy()))
    torch.cuda.synchronize()
    return np.stack(imgs)


def main():
    dev = torch.device("cuda", 0)
    B = 1 << int(os.environ.get("LOGB", "22"))
    rng = np.random.default_rng(1)
    raw = torch.from_numpy((rng.uniform(0, 1, size=(2 * B, 18)) * 40).astype(np.float32)).to(dev)
    base = run("3:0", raw, B, 3)
    for v in sys.argv[1:] or ["3:0", "3:2", "4:1"]:
        a = run(v, raw, B, 3)
        b = run(v, raw, B, 3)
        rel = float(np.abs(a - base).max() / np.abs(base).max())
        print(f"{v}: repeat bit-identical {np.array_equal(a, b)}  max|a-b| {np.abs(a - b).max():.3e}  rel vs 3:0 {rel:.3e}",
              flush=True)


if __name__ == "__main__":
    main()
