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


@pytest.mark.parametrize("B,N,u8", [(1, 128, True), (32, 512, True), (33, 128, False), (4099, 128, True)])
def test_mlp_kernels_vs_fp32_torch(cuda_device, B, N, u8):
    """mlp.hip GEMMs (fp32 MFMA, LDS K loop) vs fp32 torch: forward with fused bias +
    relu, dH gated by [h > 0], [x ; 1]^T . dy weight+bias gradient."""
    from streamml.ops import load_c
    C = load_c()
    g = torch.Generator().manual_seed(B + N)
    xu = torch.randint(0, 256, (B, 784), generator=g, dtype=torch.uint8)
    xf = xu.float() / 255.0
    W1 = torch.randn(784, N, generator=g) * 0.05
    b1 = torch.randn(N, generator=g) * 0.1
    W2 = torch.randn(N, 10, generator=g) * 0.1
    dz = torch.randn(B, 10, generator=g)
    xin = (xu if u8 else xf).to(cuda_device)
    h = C.mlp_fwd(xin, W1.to(cuda_device), b1.to(cuda_device), True)
    href = (xf.double() @ W1.double() + b1.double()).relu()
    torch.testing.assert_close(h.cpu().double(), href, rtol=1e-5, atol=1e-5)
    z = C.mlp_fwd(h, W2.to(cuda_device))
    torch.testing.assert_close(z.cpu().double(), h.cpu().double() @ W2.double(), rtol=1e-5, atol=1e-5)
    dh = C.mlp_bwd_data(dz.to(cuda_device), W2.to(cuda_device), h)
    dhref = (dz.double() @ W2.double().t()) * (h.cpu() > 0)
    torch.testing.assert_close(dh.cpu().double(), dhref, rtol=1e-5, atol=1e-5)
    out = torch.empty((785, N), device=cuda_device)
    C.mlp_wgrad(xin, dh, out)
    ref = torch.cat([xf.double(), torch.ones(B, 1, dtype=torch.float64)], 1).t() @ dh.cpu().double()
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-5, atol=1e-4)


def test_mlp_dropout_step_vs_oracle(cuda_device):
    """Dense(512) + Dropout(0.2) (confluent-tensorflow-io-kafka-simplified.py): one device
    train step == an fp32 torch step that applies the kernel's own dropout multipliers."""
    from streamml.ops import load_c
    x, y = mn.synthetic_mnist(32, seed=3)
    m = MLPClassifier(hidden=512, dropout=0.2, device=cuda_device, seed=9)
    W1, b1, W2, b2 = [torch.from_numpy(a).double() for a in m.fp.get()]
    mask = load_c().mlp_dropout_mask(m.fp.flat, 32, 512, 0.8, m._seed, m._step).cpu().double()
    assert 0.7 < float((mask > 0).double().mean()) < 0.9
    m.train_step(x, y.astype(np.int64))
    grads = [gr.double() for gr in (m.fp.grad[m.fp.offsets[i]:m.fp.offsets[i + 1]].cpu() for i in range(4))]
    xf = torch.from_numpy(x.reshape(32, -1)).double() / 255.0
    h = (xf @ W1 + b1).relu() * mask
    z = h @ W2 + b2
    p = torch.softmax(z, 1)
    p[torch.arange(32), torch.from_numpy(y.astype(np.int64))] -= 1.0
    dz = p / 32.0
    dh = (dz @ W2.t()) * (h > 0) * 1.25
    ref = [xf.t() @ dh, dh.sum(0), h.t() @ dz, dz.sum(0)]
    for a, b in zip(grads, ref):
        torch.testing.assert_close(a.reshape(b.shape), b, rtol=1e-4, atol=1e-6)
