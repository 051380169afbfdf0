"""General LDS-tiled MFMA GEMM (csrc/kernels/gemm.hip) vs torch references.

Every operand orientation (row-major, transposed view), fp32 / bf16 operands, fp32 / bf16
output, bias + activation epilogue, edge tiles (M, N, K not multiples of the 128 x 128 x 64
tile, unaligned leading dims) and the split-K weight-gradient path.  References round the
operands to bf16 and accumulate in fp64 (``helpers.bf16_ref``), so what remains is fp32
accumulation order: relative error <= 1e-3 (bf16 output: the bf16 floor)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ACTS = {"linear": lambda z: z, "relu": torch.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid}


def _ops(M, K, N, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(K, N, generator=g) / K ** 0.5
    return a, b


def _view(t, transposed, dev, dt):
    """t [R, C] on the device as a row-major tensor, or as the transposed view of a
    row-major [C, R] tensor (unit stride along the rows)."""
    if transposed:
        return t.t().contiguous().to(dev, dt).t()
    return t.to(dev, dt)


@pytest.mark.parametrize("M,K,N", [(1, 7, 1), (128, 64, 128), (300, 784, 128), (1000, 129, 257),
                                   (2048, 512, 640), (77, 1000, 33), (4099, 96, 200)])
@pytest.mark.parametrize("a_t", [False, True])
@pytest.mark.parametrize("b_t", [False, True])
def test_gemm_orientations_vs_bf16_reference(cuda_device, M, K, N, a_t, b_t):
    from helpers.bf16_ref import bf, relerr
    from streamml.ops import gemm as gm
    a, b = _ops(M, K, N, M * 7 + K * 3 + N + a_t * 2 + b_t)
    ref = bf(a) @ bf(b)
    for dt in (torch.float32, torch.bfloat16):
        out = gm.matmul(_view(a, a_t, cuda_device, dt), _view(b, b_t, cuda_device, dt), splits=1).cpu()
        assert out.shape == (M, N) and out.dtype == torch.float32
        assert relerr(out, ref) < 1e-3, (dt, relerr(out, ref))


@pytest.mark.parametrize("act", ["linear", "relu", "tanh", "sigmoid"])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_gemm_bias_act_epilogue(cuda_device, act, out_bf16):
    from helpers.bf16_ref import bf, relerr
    from streamml.ops import gemm as gm
    M, K, N = 1500, 784, 130
    a, b = _ops(M, K, N, 11)
    bias = torch.randn(N)
    ref = ACTS[act](bf(a) @ bf(b) + bias.double())
    out = gm.matmul(a.to(cuda_device), b.to(cuda_device), bias.to(cuda_device), act, out_bf16=out_bf16)
    assert out.dtype == (torch.bfloat16 if out_bf16 else torch.float32)
    assert relerr(out.float().cpu(), ref) < (5e-3 if out_bf16 else 1e-3)


@pytest.mark.parametrize("M,K,N,splits", [(60000, 784, 128, -1), (100000, 64, 512, -1), (5000, 300, 10, 7),
                                          (3001, 129, 1, -1)])
def test_gemm_split_k_weight_gradient(cuda_device, M, K, N, splits):
    """dW = x^T . dy over many rows: x^T is a transposed view (no copy), split over the rows
    and reduced deterministically (two runs bit-identical)."""
    from helpers.bf16_ref import bf, relerr
    from streamml.ops import gemm as gm
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g)
    dy = torch.randn(M, N, generator=g)
    xd, dyd = x.to(cuda_device), dy.to(cuda_device)
    dW = gm.matmul(xd.t(), dyd, splits=splits)
    assert dW.shape == (K, N)
    assert relerr(dW.cpu(), bf(x).t() @ bf(dy)) < 1e-3
    assert torch.equal(dW, gm.matmul(xd.t(), dyd, splits=splits))


def test_gemm_unaligned_and_strided_views(cuda_device):
    """leading dims that rule out 16-byte loads, column slices with an odd start"""
    from helpers.bf16_ref import bf, relerr
    from streamml.ops import gemm as gm
    g = torch.Generator().manual_seed(5)
    big = torch.randn(700, 301, generator=g)
    w = torch.randn(299, 150, generator=g)
    a = big[:, 1:300]                       # ld 301, start offset 1 element
    dev_a = big.to(cuda_device)[:, 1:300]
    out = gm.matmul(dev_a, w.to(cuda_device)[:, 3:140]).cpu()
    assert relerr(out, bf(a) @ bf(w[:, 3:140])) < 1e-3
    # bf16 with an odd leading dim
    bb = big.to(cuda_device, torch.bfloat16)[:, :299]
    out2 = gm.matmul(bb, w.to(cuda_device, torch.bfloat16)).cpu()
    assert relerr(out2, bf(big[:, :299]) @ bf(w)) < 1e-3


def test_gemm_matches_torch_matmul_large(cuda_device):
    """a big square product vs torch's bf16 matmul (the same bf16 rounding of the operands)"""
    from streamml.ops import gemm as gm
    g = torch.Generator().manual_seed(9)
    a = torch.randn(2048, 2048, generator=g).to(cuda_device, torch.bfloat16)
    b = torch.randn(2048, 2048, generator=g).to(cuda_device, torch.bfloat16)
    out = gm.matmul(a, b)
    ref = a.float() @ b.float()
    assert ((out - ref).norm() / ref.norm()).item() < 1e-4


def test_wide_dense_layer_autograd_on_gemm(cuda_device):
    """a Dense layer wider than the K1/K2 register tile runs forward and backward on the
    general GEMM (no vendor fallback) and matches torch autograd"""
    from streamml.ops import _ext
    from streamml.ops import dense as dn
    assert not dn.supported(784, 300)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3000, 784, generator=g)
    W = torch.randn(784, 300, generator=g) * 0.03
    b = torch.randn(300, generator=g) * 0.1
    _ext.FALLBACKS.clear()
    outs = []
    for dev in ("cpu", cuda_device):
        xx = x.clone().to(dev).requires_grad_(True)
        WW = W.clone().to(dev).requires_grad_(True)
        bb = b.clone().to(dev).requires_grad_(True)
        y = dn.dense(xx, WW, bb, "relu")
        (y * y).mean().backward()
        outs.append([t.detach().cpu() for t in (y, xx.grad, WW.grad, bb.grad)])
    assert not _ext.FALLBACKS
    for got, ref in zip(outs[1], outs[0]):
        assert ((got - ref).norm() / ref.norm()).item() < 1e-2
