"""K3 + K6 fused MSE / accuracy kernel vs the torch fp32 expression (values and gradients)."""
import pytest
import torch

from streamml.ops.loss import MSEAccuracy, torch_mse_accuracy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,tshape", [((1000, 18), (1000, 18)), ((77, 5, 18), (77, 18)), ((4097, 10), (4097, 10)),
                                          ((33, 1, 30), (33, 30)), ((65537, 18), (65537, 18)),
                                          ((300, 64), (300, 64)), ((129, 4, 16), (129, 16))])
def test_mse_accuracy_matches_torch(cuda_device, shape, tshape):
    g = torch.Generator().manual_seed(sum(shape))
    yp = torch.randn(*shape, generator=g)
    y = torch.randn(*tshape, generator=g)
    y[:3] = yp.reshape(-1, shape[-1])[:3] if len(shape) == 2 else y[:3]     # some exact argmax hits
    a = yp.clone().requires_grad_(True)
    l_ref, c_ref = torch_mse_accuracy(a, y)
    l_ref.backward()
    b = yp.to(cuda_device).requires_grad_(True)
    bcast = shape[1] if len(shape) == 3 else 1
    l, c = MSEAccuracy.apply(b, y.to(cuda_device), bcast)
    (l * 3.0).backward()
    assert float(l) == pytest.approx(float(l_ref), rel=1e-5)
    assert float(c) == pytest.approx(float(c_ref), abs=1e-4)
    torch.testing.assert_close(b.grad.cpu(), a.grad * 3.0, rtol=1e-5, atol=1e-7)
