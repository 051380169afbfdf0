"""Unit-block split backward (csrc/kernels/lstm_fused_split.hip, opt-in: SML_LSTM_SPLIT=1) against the
one-wave kernel.

The split kernel runs a U = 32 layer without dX (layer 1 of the seq-50 stack) with two waves per
16-sequence tile that exchange dz through LDS.  Its gates are recomputed exactly as the one-wave
kernel's, but dh_{t-1} = U . dz_t sums the gate tiles in another K order, so the two agree to fp32
rounding carried through BPTT (bf16-rounded dz may flip in the last place); measured bit-identical on
every shape here.  It is off by default (slower than the one-wave kernel on the seq-50 layer,
profiles/r06/SUMMARY.md section 6).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _relerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _case(dev, B, T, IN, act, x_bf16, windows, seed):
    from streamml.data.stream import sliding_windows
    from streamml.ops import load_c
    C = load_c()
    rng = np.random.default_rng(seed)
    if windows:
        base = torch.tensor(rng.uniform(-1, 1, (B + T, IN)), dtype=torch.float32, device=dev)
        x, _ = sliding_windows(base, T)
        x = x[:B]
    else:
        x = torch.tensor(rng.uniform(-1, 1, (B, T, IN)), dtype=torch.float32, device=dev)
    if x_bf16:
        x = x.contiguous().to(torch.bfloat16)

    def w(*shape, s=0.25):
        return torch.tensor(rng.standard_normal(shape) * s, dtype=torch.float32, device=dev)
    W, U, b = w(IN, 128), w(32, 128), w(128, s=0.1)
    h0, c0 = w(B, 32, s=0.5), w(B, 32, s=0.5)
    h, c = C.lstm_fused_fwd(x, W, U, b, h0, c0, act)
    return C, x, W, U, b, h0, c0, h, c, rng


@pytest.mark.parametrize("act", [1, 2])
@pytest.mark.parametrize("B,T,IN,x_bf16,windows,last_only", [
    (1000 + 7, 50, 18, False, True, False),     # the seq-50 layer-1 shape, ragged last tile
    (37, 1, 18, False, False, False),           # one step
    (50, 2, 18, False, False, False),
    (33, 3, 18, False, False, False),
    (16, 4, 18, False, False, False),
    (130, 5, 31, False, False, False),          # DB bias mode (one spare column)
    (100, 7, 12, False, False, False),          # KT = 1
    (100, 9, 13, False, False, False),          # KT = 1, dword x pieces (IN % 3 != 0)
    (90, 11, 17, False, True, False),           # odd IN: b32 ring reads of x
    (70, 8, 24, False, False, False),           # BX, IN % 3 == 0: 12-byte x pieces, 3 per row-group
    (0, 6, 18, False, True, False),             # persistent grid: several 32-sequence groups per workgroup
])
def test_split_backward_matches_one_wave_kernel(cuda_device, monkeypatch, act, B, T, IN, x_bf16, windows, last_only):
    if B == 0:
        B = 32 * 2 * torch.cuda.get_device_properties(cuda_device).multi_processor_count * 3 + 21
    C, x, W, U, b, h0, c0, h, c, rng = _case(cuda_device, B, T, IN, act, x_bf16, windows, B + T + IN + act)
    monkeypatch.setenv("SML_LSTM_SPLIT", "1")
    assert C.lstm_split_applies(32, IN, False) and not C.lstm_split_applies(32, IN, False, True)
    assert not C.lstm_split_applies(32, IN, False, False, True)
    dh = torch.tensor(rng.standard_normal((B, 32) if last_only else (B, T, 32)), dtype=torch.float32,
                      device=cuda_device).to(torch.bfloat16)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SML_LSTM_SPLIT", v)
        assert C.lstm_split_applies(32, IN, False) == (v == "1")
        out[v] = C.lstm_fused_bwd(dh, c, h, x, h0, c0, W, U, b, act, False, True, last_only)
    torch.cuda.synchronize()
    for name, g, r in zip(("dW", "dU", "db", "dh0", "dc0"), out["1"][1:], out["0"][1:]):
        assert g.shape == r.shape, name
        assert torch.isfinite(g).all(), name
        assert _relerr(g, r) < 2e-3, (name, _relerr(g, r))


@pytest.mark.parametrize("act", [1, 2])
def test_split_backward_fragment_mode_equals_row_mode(cuda_device, monkeypatch, act):
    """Fragment-native h / dh (the stacked model's layout) and rows go through the same split
    kernel: every gradient bit for bit."""
    from streamml.data.stream import sliding_windows
    from streamml.ops import load_c
    C = load_c()
    monkeypatch.setenv("SML_LSTM_SPLIT", "1")
    B, T = 1000 + 7, 50
    rng = np.random.default_rng(11 + act)
    base = torch.tensor(rng.uniform(-1, 1, (B + T, 18)), dtype=torch.float32, device=cuda_device)
    x, _ = sliding_windows(base, T)
    x = x[:B]

    def w(*shape, s=0.25):
        return torch.tensor(rng.standard_normal(shape) * s, dtype=torch.float32, device=cuda_device)
    W1, U1, b1 = w(18, 128), w(32, 128), w(128, s=0.1)
    W2, U2, b2 = w(32, 64), w(16, 64), w(64, s=0.1)
    h1, c1, h2, c2, _ = C.lstm_fused_fwd2(x, W1, U1, b1, W2, U2, b2, act, act, False)
    f1, fc1, f2, fc2, _ = C.lstm_fused_fwd2(x, W1, U1, b1, W2, U2, b2, act, act, True)
    dh2 = torch.tensor(rng.standard_normal((B, 16)), dtype=torch.float32, device=cuda_device).to(torch.bfloat16)
    dx2, *_ = C.lstm_fused_bwd(dh2, c2, h2, h1, None, None, W2, U2, b2, act, True, False, True)
    fx2, *_ = C.lstm_fused_bwd(dh2, fc2, f2, f1, None, None, W2, U2, b2, act, True, False, True, frag=True)
    _, dW1, dU1, db1, _, _ = C.lstm_fused_bwd(dx2, c1, h1, x, None, None, W1, U1, b1, act, False, False, False)
    _, gW1, gU1, gb1, _, _ = C.lstm_fused_bwd(fx2, fc1, f1, x, None, None, W1, U1, b1, act, False, False, False,
                                              frag=True)
    torch.cuda.synchronize()
    for name, g, r in (("dW1", gW1, dW1), ("dU1", gU1, dU1), ("db1", gb1, db1)):
        assert torch.equal(g, r), name


def test_split_grid_is_the_slab_count(cuda_device):
    """The partials buffer the binding allocates has one slab per split-kernel workgroup: two per
    CU (four with SML_LSTM_SPLIT_NTW=1), never more than the tile groups."""
    from streamml.ops import load_c
    C = load_c()
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    assert C.lstm_split_grid(65536) == (4 if os.environ.get("SML_LSTM_SPLIT_NTW") == "1" else 2) * cus
    assert C.lstm_split_grid(33) == (3 if os.environ.get("SML_LSTM_SPLIT_NTW") == "1" else 2)
    assert C.lstm_split_grid(1) == 1
