"""K13 fused softmax-xent HIP kernel vs fp32 torch; MLP device step vs CPU reference."""
import numpy as np
import pytest
import torch

from streamml.data import mnist as mn
from streamml.models.mlp import MLPClassifier, softmax_xent_reference

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C", [2, 10, 16, 32])
@pytest.mark.parametrize("B", [1, 255, 4099])
def test_softmax_xent_kernel(cuda_device, B, C):
    from streamml.ops import load_c
    g = torch.Generator().manual_seed(B * 7 + C)
    z = (torch.randn(B, C, generator=g) * 4).to(cuda_device)
    y = torch.randint(0, C, (B,), generator=g)
    y[0] = -1 if B > 1 else y[0]            # an ignored (invalid-label) row
    yd = y.to(cuda_device)
    d = torch.empty_like(z)
    p = torch.empty_like(z)
    acc = torch.zeros(2, device=cuda_device)
    load_c().softmax_xent(z, yd, 0.5, d, p, acc)
    torch.cuda.synchronize()
    valid = y >= 0
    zc = z.cpu()
    loss, corr, dref = softmax_xent_reference(zc[valid], y[valid])
    torch.testing.assert_close(p.cpu(), torch.softmax(zc, 1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(d.cpu()[valid], dref * 0.5, rtol=1e-5, atol=1e-6)
    assert (d.cpu()[~valid] == 0).all()
    a = acc.cpu()
    assert float(a[0]) == pytest.approx(float(loss), rel=1e-4)
    assert float(a[1]) == float(corr)


def test_mlp_gpu_matches_cpu(cuda_device):
    x, y = mn.synthetic_mnist(512, seed=2)
    mg = MLPClassifier(hidden=128, device=cuda_device, seed=4)
    mc = MLPClassifier(hidden=128, device="cpu", seed=4)
    for s in range(0, 256, 32):
        mg.train_step(x[s:s + 32], y[s:s + 32].astype(np.int64))
        mc.train_step(x[s:s + 32], y[s:s + 32].astype(np.int64))
    for a, b in zip(mg.fp.get(), mc.fp.get()):
        np.testing.assert_allclose(a, b, rtol=0, atol=2e-4)
    lg, ag = mg.evaluate(x, y)
    lc, ac = mc.evaluate(x, y)
    assert lg == pytest.approx(lc, rel=1e-3) and ag == pytest.approx(ac, abs=2 / 512)
    np.testing.assert_allclose(mg.predict(x[:64]), mc.predict(x[:64]), atol=1e-4)
