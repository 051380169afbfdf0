import os, sys, numpy as np, torch
sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
from streamml.data.cardata import normalize_affine
from streamml.models.reference import init_dense_weights
from streamml.ops.ae import AESpec, FusedAE, NPARAM
dev = torch.device("cuda", 0)
spec = AESpec()
w = init_dense_weights(spec.layer_sizes, seed=7)
rng = np.random.default_rng(8)
for i in range(1, 8, 2): w[i] = rng.uniform(-0.2, 0.2, size=w[i].shape).astype(np.float32)
scale, shift = normalize_affine()
for ntiles, blocks in [(64 * 5, 16), (4096, 48), (100, 16)]:
    B = 16 * ntiles
    raw = torch.from_numpy((np.random.default_rng(17).uniform(0, 1, size=(2 * B, 18)) * 40).astype(np.float32)).to(dev)
    out = {}
    for v in ("1", "3"):
        os.environ["SML_AE_ILP"] = v
        f = FusedAE(spec, w, dev, max_blocks=blocks, scale=scale, shift=shift)
        f.attach_ring(raw, B)
        imgs = []
        f.step_ring(allreduce=lambda g: imgs.append(g.detach().cpu().numpy().copy()))
        torch.cuda.synchronize()
        out[v] = imgs[0]
    a, b = out["1"].astype(np.float64), out["3"].astype(np.float64)
    d = np.abs(a[:NPARAM] - b[:NPARAM])
    print(ntiles, "relerr", np.linalg.norm(d) / np.linalg.norm(a[:NPARAM]), "max abs", d.max(),
          "max rel (|a|>1e-3)", (d / np.maximum(np.abs(a[:NPARAM]), 1e-3)).max(), "metrics", a[NPARAM:], b[NPARAM:])
    # per-layer breakdown
    for name, lo, hi in [("L1", 0, 512), ("L2", 512, 768), ("L3", 768, 1024), ("L4", 1024, 1536)]:
        print("   ", name, np.linalg.norm(d[lo:hi]) / max(np.linalg.norm(a[lo:hi]), 1e-30))
