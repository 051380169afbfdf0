"""Persistent reference-stack LSTM trainer (lstm_ref_train.hip) vs the fp32 PyTorch oracle.

The oracle is the same LSTMPredictor on the CPU: plain torch LSTM math (ops/lstm.py
lstm_reference), torch MSE, the torch Keras-Adam of ops/adam.py -- all fp32."""
import numpy as np
import pytest
import torch

from streamml.models.lstm import LSTMPredictor
from streamml.ops import lstm_persistent as lp

pytestmark = pytest.mark.gpu


def _data(n, seed=0):
    rows = np.random.default_rng(seed).uniform(-1, 1, (n + 1, 18)).astype(np.float32)
    return rows[:-1, None, :].copy(), rows[1:].copy()


def test_64_batch1_steps_match_fp32_oracle(cuda_device):
    X, Y = _data(64)
    cpu = LSTMPredictor.reference(look_back=1, device="cpu", seed=3)
    gpu = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=3)
    assert lp.supported(gpu) and lp.check_inactive(gpu)
    p0 = cpu.fp.flat.clone()
    ref_loss = []
    for i in range(64):
        loss, _ = cpu.train_step(torch.from_numpy(X[i:i + 1]), torch.from_numpy(Y[i:i + 1]))
        ref_loss.append(float(loss))
    out = lp.train_steps(gpu, torch.from_numpy(X).to(cuda_device), torch.from_numpy(Y).to(cuda_device), 1, 64)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out[:, 0].cpu().numpy(), ref_loss, rtol=2e-4, atol=1e-7)
    assert int(gpu.fp.iter.item()) == 64
    d_gpu = (gpu.fp.flat.cpu() - p0).double()
    d_cpu = (cpu.fp.flat - p0).double()
    assert (d_gpu - d_cpu).norm() / d_cpu.norm() < 2e-4
    torch.testing.assert_close(gpu.fp.m.cpu(), cpu.fp.m, rtol=2e-3, atol=1e-7)
    torch.testing.assert_close(gpu.fp.v.cpu(), cpu.fp.v, rtol=2e-3, atol=1e-10)


def test_chunked_launches_are_bit_identical_to_one(cuda_device):
    X, Y = _data(100, seed=1)
    Xd, Yd = torch.from_numpy(X).to(cuda_device), torch.from_numpy(Y).to(cuda_device)
    a = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=5)
    b = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=5)
    oa = lp.train_steps(a, Xd, Yd, 4, 25)
    ob = torch.cat([lp.train_steps(b, Xd, Yd, 4, 10), lp.train_steps(b, Xd, Yd, 4, 15, row0=40)])
    torch.testing.assert_close(oa, ob, rtol=0, atol=0)
    torch.testing.assert_close(a.fp.flat, b.fp.flat, rtol=0, atol=0)
    torch.testing.assert_close(a.fp.v, b.fp.v, rtol=0, atol=0)


def test_fit_persistent_matches_cpu_fit_shuffled_partial_batch(cuda_device):
    """fit(batch_size=8, shuffle=True) over 203 samples (last batch of 3), 2 epochs."""
    X, Y = _data(203, seed=2)
    cpu = LSTMPredictor.reference(look_back=1, device="cpu", seed=7)
    gpu = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=7)
    hc = cpu.fit(X, Y, epochs=2, batch_size=8, shuffle=True, verbose=0, normalize=False)
    hg = gpu.fit(X, Y, epochs=2, batch_size=8, shuffle=True, verbose=0, normalize=False)
    assert gpu.last_fit_engine == "persistent"
    np.testing.assert_allclose(hg.history["loss"], hc.history["loss"], rtol=1e-4)
    np.testing.assert_allclose(hg.history["accuracy"], hc.history["accuracy"], atol=1e-9)
    torch.testing.assert_close(gpu.fp.flat.cpu(), cpu.fp.flat, rtol=1e-3, atol=2e-5)


def test_batch1_chunked_launches_bit_identical_across_row_blocks(cuda_device):
    """The batch-1 path (one-wave chain, rows prefetched 32 steps ahead into LDS): 100 steps
    in one launch == 37 + 63 steps in two (block boundaries fall at different steps)."""
    X, Y = _data(100, seed=4)
    Xd, Yd = torch.from_numpy(X).to(cuda_device), torch.from_numpy(Y).to(cuda_device)
    a = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=9)
    b = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=9)
    oa = lp.train_steps(a, Xd, Yd, 1, 100)
    ob = torch.cat([lp.train_steps(b, Xd, Yd, 1, 37), lp.train_steps(b, Xd, Yd, 1, 63, row0=37)])
    torch.testing.assert_close(oa, ob, rtol=0, atol=0)
    torch.testing.assert_close(a.fp.flat, b.fp.flat, rtol=0, atol=0)
    torch.testing.assert_close(a.fp.m, b.fp.m, rtol=0, atol=0)
    assert int(a.fp.iter.item()) == int(b.fp.iter.item()) == 100


def test_batch1_rows_running_out_mid_block(cuda_device):
    """nsteps beyond the rows: the launch stops at the last row (45 of 80 requested)."""
    X, Y = _data(45, seed=6)
    cpu = LSTMPredictor.reference(look_back=1, device="cpu", seed=11)
    gpu = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=11)
    ref = [float(cpu.train_step(torch.from_numpy(X[i:i + 1]), torch.from_numpy(Y[i:i + 1]))[0]) for i in range(45)]
    out = lp.train_steps(gpu, torch.from_numpy(X).to(cuda_device), torch.from_numpy(Y).to(cuda_device), 1, 80)
    torch.cuda.synchronize()
    assert int(gpu.fp.iter.item()) == 45
    np.testing.assert_allclose(out[:45, 0].cpu().numpy(), ref, rtol=2e-4, atol=1e-7)


def test_fit_batch1_shuffled_matches_cpu_fit(cuda_device):
    """fit(batch_size=1, shuffle=True): the permutation is read by the row prefetch."""
    X, Y = _data(70, seed=8)
    cpu = LSTMPredictor.reference(look_back=1, device="cpu", seed=13)
    gpu = LSTMPredictor.reference(look_back=1, device=cuda_device, seed=13)
    hc = cpu.fit(X, Y, epochs=2, batch_size=1, shuffle=True, verbose=0, normalize=False)
    hg = gpu.fit(X, Y, epochs=2, batch_size=1, shuffle=True, verbose=0, normalize=False)
    assert gpu.last_fit_engine == "persistent"
    np.testing.assert_allclose(hg.history["loss"], hc.history["loss"], rtol=2e-4)
    np.testing.assert_allclose(hg.history["accuracy"], hc.history["accuracy"], atol=1e-9)
    torch.testing.assert_close(gpu.fp.flat.cpu(), cpu.fp.flat, rtol=1e-3, atol=2e-5)
