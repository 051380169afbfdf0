"""The wide-grid AE step's reduction in one launch (slab_adam_kernel: level sum + Adam joined by
per-column arrival counters) against the two launches it replaces (slab_sum_kernel level, then
reduce_adam_kernel).  The final sum is done by whichever workgroup of a column arrives last, in
reduce_adam_kernel's fixed order, so every output must be BIT-identical, step after step (the
counters re-arm themselves).  The one-launch kernel is opt-in (SML_AE_FUSED_REDUCE=1): its
agent-scope release fences write back the L2 and made it slower (profiles/r06/SUMMARY.md §10)."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.reference import init_dense_weights
from streamml.ops.ae import AESpec, FusedAE

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("max_blocks,n", [(None, 1 << 20), (100, 200_000), (2000, 1 << 19)])
def test_one_launch_reduction_is_bit_identical(cuda_device, monkeypatch, max_blocks, n):
    spec = AESpec()
    w = init_dense_weights(spec.layer_sizes, seed=2)
    sc, sh = normalize_affine()
    rng = np.random.default_rng(4)
    steps = 3
    x = torch.from_numpy((rng.uniform(0, 1, size=(steps * n, 18)) * 40).astype(np.float32)).to(cuda_device)
    runs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("SML_AE_FUSED_REDUCE", mode)
        ae = FusedAE(spec, w, cuda_device, max_blocks=max_blocks, scale=sc, shift=sh)
        for s in range(steps):
            ae.step(x[s * n:(s + 1) * n])
        ae.pack_ring(x, n)                 # the headline's path: tile-packed ring, device cursor
        for s in range(steps + 1):
            ae.step_ring()
        ae.gradients(x[:n])                # the gradient-only flags (grad written, no update)
        torch.cuda.synchronize()
        runs[mode] = ae
    a, b = runs["0"], runs["1"]
    G = a.grad_partials(x[:n], bump_iter=False)
    assert G > 64, G                      # the wide-grid path (the one-launch kernel applies)
    assert int(b.cursor.item()) == ((steps + 1) * n) % (steps * n)
    for name in ("params", "m", "v", "grad", "metrics", "iter", "cursor"):
        ta, tb = getattr(a, name), getattr(b, name)
        assert torch.equal(ta, tb), (name, (ta - tb).abs().max().item() if ta.is_floating_point() else None)
    assert int(b.iter.item()) == 2 * steps + 1
    assert int(b.reduce_counters.abs().sum().item()) == 0   # re-armed for the next step
