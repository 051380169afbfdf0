"""Numerics of the fused AE HIP kernels vs a plain PyTorch fp32 reference."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.reference import KerasAdam, ae_forward_torch, ae_loss_torch, init_dense_weights
from streamml.ops.ae import AESpec, FusedAE, pack_image, unpack_image

pytestmark = pytest.mark.gpu


def _weights(spec, seed=0, bias=True):
    w = init_dense_weights(spec.layer_sizes, seed=seed)
    if bias:
        rng = np.random.default_rng(seed + 1)
        for i in range(1, 8, 2):
            w[i] = rng.uniform(-0.2, 0.2, size=w[i].shape).astype(np.float32)
    return w


def _relerr(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)


@pytest.mark.parametrize("D,n", [(18, 1000), (18, 4096), (30, 777)])
def test_gradients_match_torch(cuda_device, D, n):
    spec = AESpec(input_dim=D)
    w = _weights(spec)
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, size=(n, D)).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device, max_blocks=64)
    g_fused, metr = fused.gradients(torch.from_numpy(x).to(cuda_device))
    wt = [torch.tensor(a, dtype=torch.float32, requires_grad=True) for a in w]
    xt = torch.from_numpy(x)
    loss, mse, acc = ae_loss_torch(xt, wt, spec.activations, spec.activity_l1)
    g_ref = torch.autograd.grad(loss, wt)
    for gf, gr in zip(g_fused, g_ref):
        assert gf.shape == tuple(gr.shape)
        assert _relerr(gf, gr.numpy()) < 3e-2, (gf, gr)
    sq, ab, corr, rows = metr
    assert rows == n
    assert abs(sq / (n * D) - float(mse)) / float(mse) < 2e-2
    assert abs(corr / n - float(acc)) < 0.03


def test_training_trajectory_matches_torch(cuda_device):
    """Adam after a few steps: bf16 MFMA run vs fp32 torch run of the same stream.

    Adam's early steps are ~lr*sign(g) per parameter, so parameters whose
    gradient is ~0 can legitimately differ by up to 2*lr*steps between a bf16
    and an fp32 run; we bound the bulk (99th percentile) tightly, the max by
    that envelope, and the loss trajectory.
    """
    spec = AESpec()
    w = _weights(spec, seed=3)
    scale, shift = normalize_affine()
    rng = np.random.default_rng(7)
    steps, bs = 8, 512
    raw = (rng.uniform(0, 1, size=(steps * bs, 18)) * 40).astype(np.float32)
    xn = (raw * scale + shift).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device, max_blocks=32, scale=scale, shift=shift)
    ref_w = [torch.tensor(a, requires_grad=True) for a in w]
    opt = KerasAdam(ref_w)
    xr_dev = torch.from_numpy(raw).to(cuda_device)
    ref_losses = []
    for s in range(steps):
        fused.step(xr_dev[s * bs:(s + 1) * bs])
        xb = torch.from_numpy(xn[s * bs:(s + 1) * bs])
        loss, _, _ = ae_loss_torch(xb, ref_w, spec.activations, spec.activity_l1)
        ref_losses.append(float(loss) * bs)
        opt.apply(torch.autograd.grad(loss, ref_w))
    torch.cuda.synchronize()
    got = fused.get_weights()
    assert int(fused.iter.item()) == steps
    diffs = np.concatenate([np.abs(a - b.detach().numpy()).ravel() for a, b in zip(got, ref_w)])
    assert np.median(diffs) < 1e-4, np.median(diffs)
    assert np.percentile(diffs, 99) < 1e-3, np.percentile(diffs, 99)
    assert diffs.max() <= 2 * 1e-3 * steps
    m = fused.read_metrics()
    assert m["rows"] == steps * bs
    ref_loss = sum(ref_losses) / (steps * bs)
    assert abs(m["loss"] - ref_loss) / ref_loss < 2e-2, (m["loss"], ref_loss)


def test_forward_and_score(cuda_device):
    spec = AESpec()
    w = _weights(spec, seed=11)
    rng = np.random.default_rng(2)
    n = 333
    x = rng.uniform(-1, 1, size=(n, 18)).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device)
    r, s, f = fused.forward(torch.from_numpy(x).to(cuda_device), threshold=0.3)
    y, _ = ae_forward_torch(torch.from_numpy(x), [torch.from_numpy(a) for a in w], spec.activations)
    y = y.numpy()
    assert _relerr(r.cpu().numpy(), y) < 2e-2
    score_ref = ((y - x) ** 2).mean(axis=1)
    np.testing.assert_allclose(s.cpu().numpy(), score_ref, rtol=3e-2, atol=3e-3)
    agree = (f.cpu().numpy() == (score_ref > 0.3)).mean()
    assert agree > 0.97


def test_pack_roundtrip_on_device(cuda_device):
    spec = AESpec(input_dim=30)
    w = _weights(spec, seed=4)
    fused = FusedAE(spec, w, cuda_device)
    for a, b in zip(fused.get_weights(), w):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(unpack_image(pack_image(w), spec)[0], w[0])


def test_lane_exchange_helpers(cuda_device):
    from streamml.ops import load_c
    out = load_c().lane_xor_probe(torch.empty(1, device=cuda_device)).cpu().numpy()
    lanes = np.arange(64)
    np.testing.assert_array_equal(out[:64], lanes ^ 16)
    np.testing.assert_array_equal(out[64:], lanes ^ 32)


def test_accuracy_metric_exact(cuda_device):
    """Rows with a clear argmax: categorical accuracy must match exactly."""
    spec = AESpec()
    w = _weights(spec, seed=21)
    n = 512
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, size=(n, 18)).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device)
    _, metr = fused.gradients(torch.from_numpy(x).to(cuda_device))
    y, _ = ae_forward_torch(torch.from_numpy(x), [torch.from_numpy(a) for a in w], spec.activations)
    y = y.numpy()
    ysorted = np.sort(y, axis=1)
    clear = (ysorted[:, -1] - ysorted[:, -2]) > 2e-2
    ref = (np.argmax(y, 1) == np.argmax(x, 1))
    # rows without a clear winner may legitimately flip under bf16
    assert abs(metr[2] - ref.sum()) <= (~clear).sum()


@pytest.mark.parametrize("xpack", ["0", "1"])
def test_ring_cursor_and_graph_replay(cuda_device, xpack, monkeypatch):
    """Device-cursor ring steps == explicit-slice steps; a captured graph replays them.
    xpack=1: the tile-packed ring (rows + ingest-time argmax bytes per 16-row tile)."""
    monkeypatch.setenv("SML_AE_XPACK", xpack)
    # the one-tile loop, so the packed ring's steps are bit-comparable with the slice path
    # (the default packed-pair loop is checked against it in test_tile_pair_loop_matches_one_tile_loop)
    monkeypatch.setenv("SML_AE_ILP", "1")
    spec = AESpec()
    w = _weights(spec, seed=5)
    scale, shift = normalize_affine()
    rng = np.random.default_rng(3)
    B, nsl = 1024, 3
    raw = torch.from_numpy((rng.uniform(0, 1, size=(B * nsl, 18)) * 40).astype(np.float32)).to(cuda_device)
    a = FusedAE(spec, w, cuda_device, max_blocks=16, scale=scale, shift=shift)
    b = FusedAE(spec, w, cuda_device, max_blocks=16, scale=scale, shift=shift)
    b.attach_ring(raw, B)
    for s in range(4):  # wraps around the 3-slice ring
        i = s % nsl
        a.step(raw[i * B:(i + 1) * B])
        b.step_ring()
    torch.cuda.synchronize()
    assert int(b.cursor.item()) == (4 % nsl) * B
    torch.testing.assert_close(a.params, b.params, rtol=0, atol=0)
    # the ring path reads x's argmax from the ingest-time byte array (row_argmax_u8);
    # the accuracy counts equal the in-kernel argmax of the slice path exactly
    assert (b.ring_xpack is not None) == (xpack == "1")
    torch.testing.assert_close(a.metrics, b.metrics, rtol=0, atol=0)
    # hipGraph capture of one ring step, replayed
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        b.step_ring()
        a.step(raw[(4 % nsl) * B:(4 % nsl + 1) * B])
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.step_ring()
    # capture itself does not execute; replay 2 steps and mirror them eagerly
    for s in range(5, 7):
        g.replay()
        i = s % nsl
        a.step(raw[i * B:(i + 1) * B])
    torch.cuda.synchronize()
    torch.testing.assert_close(a.params, b.params, rtol=0, atol=0)
    assert int(b.iter.item()) == int(a.iter.item()) == 7


@pytest.mark.parametrize("D,n,blocks", [(18, 16 * 1000 + 5, 7), (18, 4096, 768), (30, 16 * 333, 5), (18, 40, 64)])
def test_lds_dma_ring_matches_register_path(cuda_device, monkeypatch, D, n, blocks):
    """The LDS-DMA input ring (contiguous rows) and the register-prefetch path
    (rows with a wider stride) run the same tile math in the same order: their
    gradient slabs must agree bit for bit, including ragged tails, waves with no
    tiles and rings clamped past the last tile.  (The one-tile ring loop: the direct
    packed-pair loop is checked against it in test_direct_pair_loop_matches_one_tile_direct.)"""
    monkeypatch.setenv("SML_AE_DIRECT_PAIRS", "0")
    spec = AESpec(input_dim=D)
    w = _weights(spec, seed=11)
    rng = np.random.default_rng(13)
    x = rng.uniform(-1, 1, size=(n, D)).astype(np.float32)
    wide = np.zeros((n, D + 2), np.float32)
    wide[:, :D] = x
    fused = FusedAE(spec, w, cuda_device, max_blocks=blocks)
    g_ring, m_ring = fused.gradients(torch.from_numpy(x).to(cuda_device))
    xw = torch.from_numpy(wide).to(cuda_device)[:, :D]
    assert xw.stride(0) == D + 2
    g_reg, m_reg = fused.gradients(xw)
    for a, b in zip(g_ring, g_reg):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(m_ring, m_reg)


def test_row_argmax_u8_matches_numpy(cuda_device):
    """Ingest-time argmax of the normalised rows (ties -> lowest index, as tf.argmax)."""
    from streamml.ops._ext import load_c
    scale, shift = normalize_affine()
    rng = np.random.default_rng(11)
    raw = (rng.uniform(0, 1, size=(5000, 18)) * 40).astype(np.float32)
    raw[::7, 3] = raw[::7, 9]                     # ties between two features
    raw[::11] = 0.0                               # all-equal normalised rows (zeroed columns tie)
    out = load_c().row_argmax_u8(torch.from_numpy(raw).to(cuda_device), 18,
                                 torch.tensor(scale, dtype=torch.float32, device=cuda_device),
                                 torch.tensor(shift, dtype=torch.float32, device=cuda_device))
    xn = (raw.astype(np.float64) * np.float32(scale) + np.float32(shift)).astype(np.float32)  # = fmaf
    ref = np.argmax(xn, axis=1)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_pack_tiles_argmax_layout(cuda_device):
    """Tile-packed ring: per 16-row tile the normalised rows then their argmax bytes."""
    from streamml.ops._ext import load_c
    scale, shift = normalize_affine()
    rng = np.random.default_rng(12)
    raw = (rng.uniform(0, 1, size=(64, 18)) * 40).astype(np.float32)
    sc = torch.tensor(scale, dtype=torch.float32, device=cuda_device)
    sh = torch.tensor(shift, dtype=torch.float32, device=cuda_device)
    p = load_c().pack_tiles_argmax(torch.from_numpy(raw).to(cuda_device), 18, sc, sh).cpu().numpy()
    tiles = p.reshape(4, 64 * 18 + 16)
    rows = tiles[:, :64 * 18].copy().view(np.float32).reshape(64, 18)
    xn = (raw.astype(np.float64) * np.float32(scale) + np.float32(shift)).astype(np.float32)   # = fmaf
    np.testing.assert_array_equal(rows, xn)
    np.testing.assert_array_equal(tiles[:, 64 * 18:].reshape(64), np.argmax(xn, axis=1))


@pytest.mark.parametrize("D,n", [(18, 1000), (18, 4096), (30, 777)])
def test_gradients_vs_bf16_rounded_reference(cuda_device, D, n):
    """The fused AE step against a torch reference with the kernel's bf16 rounding points
    (tests/helpers/bf16_ref.py): every gradient and the loss sum to <= 1e-3 relative."""
    from helpers.bf16_ref import ae_bf16_reference, relerr
    spec = AESpec(input_dim=D)
    w = _weights(spec)
    x = np.random.default_rng(5).uniform(-1, 1, size=(n, D)).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device, max_blocks=64)
    g_fused, metr = fused.gradients(torch.from_numpy(x).to(cuda_device))
    g_ref, (sq, ab) = ae_bf16_reference(torch.from_numpy(x), w, spec.activity_l1)
    for i, (gf, gr) in enumerate(zip(g_fused, g_ref)):
        assert relerr(gf, gr) < 1e-3, i
    assert abs(metr[0] - sq) / sq < 1e-4
    assert abs(metr[1] - ab) / ab < 1e-4


@pytest.mark.parametrize("ntiles,blocks", [(64 * 4, 16), (2 * 4096, 48), (30, 16), (2, 16), (64 * 2, 64)])
def test_direct_pair_loop_matches_one_tile_direct(cuda_device, monkeypatch, ntiles, blocks):
    """Rows trained once (the direct step, no tile-packed ring): the packed-pair loop on raw
    rows -- normalize_fn and argmax(x) of BOTH tiles in registers (signed-key butterfly) --
    against the one-tile direct loop (SML_AE_DIRECT_PAIRS=0), three steps on raw car-sensor
    rows whose normalised values take both signs.  Same tiles per wave on the same grid: the
    gradient image agrees to the packed MFMAs' K-order rounding, sq / |h1| / rows exactly as
    before, the correct count up to argmax near-ties."""
    from streamml.ops.ae import NPARAM
    spec = AESpec()
    w = _weights(spec, seed=9)
    scale, shift = normalize_affine()
    B = 16 * ntiles
    rng = np.random.default_rng(23)
    raw = torch.from_numpy((rng.uniform(-0.3, 1.2, size=(B, 18)) * 40).astype(np.float32)).to(cuda_device)
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("SML_AE_DIRECT_PAIRS", v)
        f = FusedAE(spec, w, cuda_device, max_blocks=blocks, scale=scale, shift=shift)
        imgs = []
        for _ in range(3):
            f.step(raw, allreduce=lambda g: imgs.append(g.detach().cpu().numpy().copy()))
        torch.cuda.synchronize()
        out[v] = (imgs, f.params.detach().cpu().numpy())
    one, two = out["0"][0], out["1"][0]
    for k in range(3):
        np.testing.assert_allclose(two[k][NPARAM:NPARAM + 2], one[k][NPARAM:NPARAM + 2], rtol=1e-6)
        assert abs(two[k][NPARAM + 2] - one[k][NPARAM + 2]) <= max(2, 1e-3 * B)
        assert two[k][NPARAM + 3] == one[k][NPARAM + 3] == B
        assert _relerr(two[k][:NPARAM], one[k][:NPARAM]) < 1e-6
    assert _relerr(out["1"][1], out["0"][1]) < 1e-6


def test_direct_pair_accuracy_vs_numpy_argmax(cuda_device, monkeypatch):
    """argmax(x) of the direct pair loop (signed keys over normalised inputs of both signs)
    against numpy on rows with a clear input argmax: the correct count matches exactly."""
    monkeypatch.setenv("SML_AE_DIRECT_PAIRS", "1")
    spec = AESpec()
    w = _weights(spec, seed=21)
    scale, shift = normalize_affine()
    n = 16 * 64
    rng = np.random.default_rng(31)
    xn = rng.uniform(-1.5, 1.0, size=(n, 18)).astype(np.float32)
    xn[:, [1, 8]] = -1.4     # zeroed / constant columns stay in the race as negatives
    k = rng.integers(0, 18, n)
    xn[np.arange(n), k] = 1.3 + rng.uniform(0, 0.5, n).astype(np.float32)   # clear winner per row
    live = np.asarray(scale) != 0
    raw = np.where(live, (xn - np.asarray(shift)) / np.where(live, scale, 1), 0).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device, max_blocks=16, scale=scale, shift=shift)
    _, metr = fused.gradients(torch.from_numpy(raw).to(cuda_device))
    xin = (raw * scale + shift).astype(np.float32)
    y, _ = ae_forward_torch(torch.from_numpy(xin), [torch.from_numpy(a) for a in w], spec.activations)
    y = y.numpy()
    ys = np.sort(y, axis=1)
    clear = (ys[:, -1] - ys[:, -2]) > 2e-2
    ref = np.argmax(y, 1) == np.argmax(xin, 1)
    assert abs(metr[2] - ref.sum()) <= (~clear).sum()
    assert metr[3] == n


@pytest.mark.parametrize("ilp", ["2", "3"])
@pytest.mark.parametrize("ntiles,blocks", [(64 * 5, 16), (64 * 4, 16), (100, 16), (30, 16), (4096, 48), (101, 16)])
def test_tile_pair_loop_matches_one_tile_loop(cuda_device, monkeypatch, ntiles, blocks, ilp):
    """SML_AE_ILP=2 (two tiles per wave interleaved, K = 32-row weight-gradient MFMAs) and
    SML_AE_ILP=3 (two tiles packed into one fragment in the 7-wide layers, block-diagonal
    weights, accumulators folded into the image per launch) against the one-tile loop on the
    headline ring (tile-packed, D = 18).  On the same grid every wave visits the same tiles in
    the same order: ILP 2's metric sums are bit-identical, ILP 3's differ only where the
    packed MFMAs sum the same products in another K order.  Tile counts per wave cover odd
    (a last unpaired tile), even, one and zero; ILP 3 pairs contiguous tiles, so an odd total
    (101 tiles) takes the one-tile loop."""
    from streamml.ops.ae import NPARAM
    spec = AESpec()
    w = _weights(spec, seed=7)
    scale, shift = normalize_affine()
    B = 16 * ntiles
    rng = np.random.default_rng(17)
    raw = torch.from_numpy((rng.uniform(0, 1, size=(2 * B, 18)) * 40).astype(np.float32)).to(cuda_device)
    out = {}
    for v in ("1", ilp):
        monkeypatch.setenv("SML_AE_ILP", v)
        f = FusedAE(spec, w, cuda_device, max_blocks=blocks, scale=scale, shift=shift)
        f.attach_ring(raw, B)
        assert f.ring_xpack is not None
        imgs = []
        for _ in range(3):
            f.step_ring(allreduce=lambda g: imgs.append(g.detach().cpu().numpy().copy()))
        torch.cuda.synchronize()
        out[v] = (imgs, f.params.detach().cpu().numpy())
    one, two = out["1"][0], out[ilp][0]
    if ilp == "2":
        np.testing.assert_array_equal(one[0][NPARAM:], two[0][NPARAM:])   # sq, |h1|, correct, rows
    else:
        np.testing.assert_allclose(two[0][NPARAM:NPARAM + 2], one[0][NPARAM:NPARAM + 2], rtol=1e-6)
        assert abs(two[0][NPARAM + 2] - one[0][NPARAM + 2]) <= max(2, 1e-3 * B)   # argmax near-ties
        assert two[0][NPARAM + 3] == one[0][NPARAM + 3]
    assert one[0][NPARAM + 3] == B
    # measured: ~5e-8 for ILP 3 (tools/ilp_err_probe.py) -- a fold that dropped or misplaced any
    # accumulator entry would be off by orders of magnitude more
    assert _relerr(two[0][:NPARAM], one[0][:NPARAM]) < 1e-6
    for a, b in zip(one[1:], two[1:]):
        assert _relerr(b[:NPARAM], a[:NPARAM]) < 1e-4
        assert abs(a[NPARAM] - b[NPARAM]) <= 1e-4 * abs(a[NPARAM])
    assert _relerr(out[ilp][1], out["1"][1]) < 1e-4


@pytest.mark.parametrize("occ", ["2", "4", "3x2", "3x3", "4x3"])
@pytest.mark.parametrize("ntiles,blocks", [(64 * 5, 16), (64 * 4, 16), (4096, 48), (2 * 4096 + 6, 48), (2, 16)])
def test_pair_occupancy_variants_bit_identical(cuda_device, monkeypatch, ntiles, blocks, occ):
    """SML_AE_PAIR_OCC=2 (TWO packed pairs per loop iteration, one interleaved stream, 2 waves per
    SIMD, a deeper ring) and =4 (one pair, 4 waves per SIMD, two ring pair slots, the gradient slabs
    aliasing the loop's LDS, early transposed writes, merged tile-half accumulators) against the
    default one-pair loop at 3 waves per SIMD, on the headline tile-packed ring.  The grid is capped
    by max_blocks, so every wave trains the same pairs in the same order: occ 2 folds them into the
    same accumulators (gradient image, metric sums and parameters after three steps bit-identical),
    occ 4 sums the same products in another K order.  Pair counts per wave cover odd (a lone
    last pair for the two-pair loop), even, one and zero."""
    spec = AESpec()
    w = _weights(spec, seed=5)
    scale, shift = normalize_affine()
    B = 16 * ntiles
    rng = np.random.default_rng(29)
    raw = torch.from_numpy((rng.uniform(0, 1, size=(2 * B, 18)) * 40).astype(np.float32)).to(cuda_device)
    out = {}
    for v in ("3", occ):
        monkeypatch.setenv("SML_AE_PAIR_OCC", v[0])
        monkeypatch.setenv("SML_AE_PAIR_XP", v[2:] or "0")   # "3x2": MFMA transposes (XP 2)
        f = FusedAE(spec, w, cuda_device, max_blocks=blocks, scale=scale, shift=shift)
        f.attach_ring(raw, B)
        assert f.ring_xpack is not None
        imgs = []
        for _ in range(3):
            f.step_ring(allreduce=lambda g: imgs.append(g.detach().cpu().numpy().copy()))
        torch.cuda.synchronize()
        out[v] = (imgs, f.params.detach().cpu().numpy())
    from streamml.ops.ae import NPARAM
    if occ == "2":
        for a, b in zip(out["3"][0], out[occ][0]):
            np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(out["3"][1], out[occ][1])
        return
    # occ 4 sums each tile's dW2 / dW4 half in one 16x16x32 against lane-masked operands (the
    # other tile's products are exact zeros): the same sums in another K order
    one, two = out["3"][0], out[occ][0]
    np.testing.assert_array_equal(one[0][NPARAM + 2:], two[0][NPARAM + 2:])   # correct, rows
    np.testing.assert_allclose(two[0][NPARAM:NPARAM + 2], one[0][NPARAM:NPARAM + 2], rtol=1e-6)
    assert _relerr(two[0][:NPARAM], one[0][:NPARAM]) < 1e-6
    for a, b in zip(one[1:], two[1:]):
        assert _relerr(b[:NPARAM], a[:NPARAM]) < 1e-4
    assert _relerr(out[occ][1], out["3"][1]) < 1e-4
