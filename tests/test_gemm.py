"""ops.gemm.matmul on CPU (the torch path the CPU plumbing uses): act(a @ b + bias) with the
same argument contract as the MFMA kernel (tests/test_gemm_gpu.py checks the device)."""
import pytest
import torch

from streamml.ops import gemm as gm


@pytest.mark.parametrize("act", ["linear", "relu", "tanh", "sigmoid"])
def test_cpu_matmul_bias_act(act):
    g = torch.Generator().manual_seed(1)
    a, b, bias = torch.randn(37, 19, generator=g), torch.randn(19, 23, generator=g), torch.randn(23, generator=g)
    ref = {"linear": lambda z: z, "relu": torch.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid}[act](a @ b + bias)
    out = gm.matmul(a, b, bias, act)
    assert out.dtype == torch.float32 and torch.allclose(out, ref, atol=1e-6)
    out16 = gm.matmul(a.t().contiguous().t(), b, bias, act, out_bf16=True)
    assert out16.dtype == torch.bfloat16 and torch.allclose(out16.float(), ref, atol=3e-2, rtol=1e-2)
