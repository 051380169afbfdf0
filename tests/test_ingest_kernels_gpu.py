"""K8 ingest transforms (csrc/kernels/preprocess.hip) vs numpy fp32 oracles, on the shapes
that take every code path: the D=18 float4 path, the generic-D float4 path, the strided
(ld != D) path, partial wave groups, scale-less rows, unaligned label arrays and enough
rows that the count scan carries across several 1024-count rounds."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.ops._ext import load_c
from streamml.ops.preprocess import normalize_filter, normalize_filter_reference

pytestmark = pytest.mark.gpu


def _norm(raw, scale, shift):
    if scale is None:
        return raw.astype(np.float32)
    return (raw.astype(np.float64) * np.float32(scale) + np.float32(shift)).astype(np.float32)   # = fmaf


def _tables(D, dev, seed):
    if D == 18:
        scale, shift = normalize_affine()
    else:
        rng = np.random.default_rng(seed)
        scale, shift = rng.uniform(0.5, 2, D).astype(np.float32), rng.uniform(-1, 1, D).astype(np.float32)
    return (np.asarray(scale, np.float32), np.asarray(shift, np.float32),
            torch.tensor(scale, dtype=torch.float32, device=dev), torch.tensor(shift, dtype=torch.float32, device=dev))


@pytest.mark.parametrize("D,n,ld,use_scale", [(18, 16 * 8 * 37 + 48, 18, True), (18, 16, 18, True),
                                              (30, 16 * 8 * 5 + 32, 30, True), (18, 16 * 8 * 3 + 16, 21, True),
                                              (18, 4096, 18, False), (7, 16 * 8 * 2 + 112, 7, True)])
def test_pack_tiles_argmax(cuda_device, D, n, ld, use_scale):
    rng = np.random.default_rng(n + D)
    wide = (rng.uniform(0, 1, size=(n, ld)) * 40).astype(np.float32)
    wide[::9, 1] = wide[::9, 2]              # ties -> lowest index
    sc, sh, tsc, tsh = _tables(D, cuda_device, 1)
    x = torch.from_numpy(wide).to(cuda_device)[:, :D]
    p = load_c().pack_tiles_argmax(x, D, tsc if use_scale else None, tsh if use_scale else None).cpu().numpy()
    tiles = p.reshape(n // 16, 64 * D + 16)
    rows = tiles[:, :64 * D].copy().view(np.float32).reshape(n, D)
    xn = _norm(wide[:, :D], sc if use_scale else None, sh)
    np.testing.assert_array_equal(rows, xn)
    np.testing.assert_array_equal(tiles[:, 64 * D:].reshape(n), np.argmax(xn, axis=1))


@pytest.mark.parametrize("D,n,ld", [(18, 1, 18), (18, 129, 18), (18, 100_001, 18), (30, 5003, 30), (18, 777, 19)])
def test_row_argmax(cuda_device, D, n, ld):
    rng = np.random.default_rng(n)
    wide = (rng.uniform(0, 1, size=(n, ld)) * 40).astype(np.float32)
    wide[::5] = 0.0
    sc, sh, tsc, tsh = _tables(D, cuda_device, 2)
    x = torch.from_numpy(wide).to(cuda_device)[:, :D]
    out = load_c().row_argmax_u8(x, D, tsc, tsh).cpu().numpy()
    np.testing.assert_array_equal(out, np.argmax(_norm(wide[:, :D], sc, sh), axis=1))


@pytest.mark.parametrize("D,n,ld,keep,frac,label_off", [(18, 4096 * 1100 + 77, 18, 0, 0.3, 0),
                                                        (18, 50_000, 18, 0, 0.5, 1), (30, 9000, 30, 1, 0.4, 3),
                                                        (18, 9000, 23, 0, 0.2, 0), (18, 64, 18, -1, 0.5, 0),
                                                        (64, 5000, 64, 0, 0.5, 0)])
def test_normalize_filter_paths(cuda_device, D, n, ld, keep, frac, label_off):
    rng = np.random.default_rng(n + D + label_off)
    wide = (rng.uniform(0, 1, size=(n, ld)) * 100).astype(np.float32)
    lab_all = (rng.uniform(size=n + label_off) < frac).astype(np.uint8)
    labels = lab_all[label_off:]
    sc, sh, _, _ = _tables(D, cuda_device, 3)
    x = torch.from_numpy(wide).to(cuda_device)[:, :D]
    lab_dev = torch.from_numpy(lab_all).to(cuda_device)[label_off:]        # possibly 16-byte unaligned
    got, idx = normalize_filter(x, lab_dev, keep, sc, sh, want_index=True)
    want, widx = normalize_filter_reference(wide[:, :D], labels, keep, sc, sh)
    assert got.shape == want.shape
    np.testing.assert_array_equal(idx.cpu().numpy(), widx)
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-6, atol=1e-6)
