"""K1/K2 tall-skinny dense kernels vs plain fp32 torch (bf16 MFMA tolerance)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _tol(ref, k):
    # bf16 operands: relative rounding 2^-8 per product term, accumulation in fp32
    return 2e-2 * (ref.abs().max().item() + 1e-3) + 1e-4 * k


@pytest.mark.parametrize("M,K,N", [(1, 18, 128), (1000, 18, 128), (40961, 32, 64), (777, 7, 18),
                                   (5000, 128, 18), (300, 32, 256), (16, 16, 16), (4099, 30, 14)])
@pytest.mark.parametrize("act", ["linear", "relu", "tanh", "sigmoid"])
def test_rowgemm(cuda_device, M, K, N, act):
    from streamml.ops import dense as dn
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(K, N, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    ref = dn._act_torch(act, x @ W + b)
    out = dn.rowgemm(x.to(cuda_device), W.to(cuda_device), b.to(cuda_device), act).cpu()
    assert out.shape == (M, N)
    assert (out - ref).abs().max().item() < _tol(ref, K)
    # bf16 in / bf16 out
    out2 = dn.rowgemm(x.to(cuda_device).bfloat16(), W.to(cuda_device), b.to(cuda_device), act, out_bf16=True)
    assert out2.dtype == torch.bfloat16
    assert (out2.float().cpu() - ref).abs().max().item() < 2 * _tol(ref, K)


def test_rowgemm_strided_rows(cuda_device):
    from streamml.ops import dense as dn
    x = torch.randn(512, 40)
    W = torch.randn(18, 32)
    xs = x.to(cuda_device)[:, 3:21]          # ld = 40, unaligned start
    out = dn.rowgemm(xs, W.to(cuda_device)).cpu()
    ref = x[:, 3:21] @ W
    assert (out - ref).abs().max().item() < _tol(ref, 18)


@pytest.mark.parametrize("M,K,N", [(1, 18, 128), (4097, 18, 128), (409600, 32, 128), (1000, 128, 18),
                                   (333, 7, 7), (20000, 64, 64), (5000, 16, 256)])
def test_wgrad(cuda_device, M, K, N):
    from streamml.ops import dense as dn
    g = torch.Generator().manual_seed(M * 3 + N)
    x = torch.randn(M, K, generator=g)
    dy = torch.randn(M, N, generator=g)
    dW, db = dn.wgrad(x.to(cuda_device), dy.to(cuda_device))
    rW = x.double().t() @ dy.double()
    rb = dy.double().sum(0)
    # error of a bf16-rounded sum over M terms grows like sqrt(M)
    tol = 1e-2 * (M ** 0.5) * 2 + 1e-2 * rW.abs().max().item()
    assert (dW.cpu().double() - rW).abs().max().item() < tol
    assert (db.cpu().double() - rb).abs().max().item() < tol


def test_wgrad_shifted(cuda_device):
    from streamml.ops import dense as dn
    B, T, K, N = 300, 7, 32, 128
    h = torch.randn(B, T, K)
    dz = torch.randn(B, T, N)
    dU, _ = dn.wgrad(h.reshape(-1, K).to(cuda_device), dz.reshape(-1, N).to(cuda_device), shift_T=T, want_db=False)
    hprev = torch.cat([torch.zeros(B, 1, K), h[:, :-1]], 1).reshape(-1, K)
    ref = hprev.double().t() @ dz.reshape(-1, N).double()
    assert (dU.cpu().double() - ref).abs().max().item() < 2e-2 * (B * T) ** 0.5


def test_dense_autograd(cuda_device):
    from streamml.ops import dense as dn
    g = torch.Generator().manual_seed(7)
    x = torch.randn(64, 5, 18, generator=g)
    W = (torch.randn(18, 32, generator=g) * 0.3)
    b = torch.randn(32, generator=g) * 0.1
    outs = []
    for dev in ("cpu", cuda_device):
        xx = x.detach().clone().to(dev).requires_grad_(True)
        WW = W.detach().clone().to(dev).requires_grad_(True)
        bb = b.detach().clone().to(dev).requires_grad_(True)
        y = dn.dense(xx, WW, bb, "tanh")
        (y * y).sum().backward()
        outs.append([t.detach().cpu() for t in (y, xx.grad, WW.grad, bb.grad)])
    for a, r in zip(outs[1], outs[0]):
        assert (a - r).abs().max().item() < 3e-2 * (r.abs().max().item() + 1e-3) + 0.05


@pytest.mark.parametrize("M,K,N", [(1000, 18, 128), (40961, 32, 64), (777, 7, 18), (5000, 128, 18)])
@pytest.mark.parametrize("act", ["linear", "relu", "tanh", "sigmoid"])
def test_rowgemm_wgrad_vs_bf16_rounded_reference(cuda_device, M, K, N, act):
    """K1 / K2 against references that round the MFMA operands to bf16 (fp64 elsewhere):
    <= 1e-3 relative, where the fp32-oracle tests above need the bf16 floor."""
    from helpers.bf16_ref import bf, relerr
    from streamml.ops import dense as dn
    g = torch.Generator().manual_seed(M * 3 + K + N)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(K, N, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    out = dn.rowgemm(x.to(cuda_device), W.to(cuda_device), b.to(cuda_device), act).cpu()
    ref = dn._act_torch(act, bf(x) @ bf(W) + b.double())
    assert relerr(out, ref) < 1e-3
    dW, db = dn.wgrad(x.to(cuda_device), dy.to(cuda_device))
    assert relerr(dW.cpu(), bf(x).t() @ bf(dy)) < 1e-3
    assert relerr(db.cpu(), dy.double().sum(0)) < 1e-5
