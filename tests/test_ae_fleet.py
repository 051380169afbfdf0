"""CPU side of fleet training (ops/ae_fleet.py, cli/fleet.py): the key -> model ring router."""
import os

import numpy as np
import pytest

from streamml.data.cardata import load_csv
from streamml.ops.ae_fleet import rings_by_key
from streamml.parallel.dp import shard_by_key

CSV = os.path.join(os.path.dirname(__file__), "fixtures", "car-sensor-data.csv")


def test_rings_one_model_per_car_on_reference_csv():
    raw, _, cars = load_csv(CSV)
    rings, members = rings_by_key(raw, cars, batch=32)
    distinct = list(dict.fromkeys(cars.tolist()))            # order of first appearance
    assert [m[0] for m in members] == distinct
    assert rings.shape[0] == len(distinct) and rings.shape[1] % 32 == 0 and rings.shape[2] == raw.shape[1]
    for b, (car,) in enumerate(members):
        own = raw[cars == car]
        n = len(own)
        np.testing.assert_array_equal(rings[b, :n], own)      # stream order kept
        reps = np.resize(np.arange(n), rings.shape[1])         # then cyclic repeat
        np.testing.assert_array_equal(rings[b], own[reps])


def test_rings_hashed_models_follow_shard_by_key():
    rng = np.random.default_rng(0)
    keys = np.array([f"electric-vehicle-{i:05d}" for i in rng.integers(0, 200, size=5000)])
    raw = rng.normal(size=(5000, 18)).astype(np.float32)
    N = 7
    rings, members = rings_by_key(raw, keys, batch=16, n_models=N)
    assert rings.shape[0] == N and rings.shape[1] % 16 == 0
    for b in range(N):
        mask = shard_by_key(keys, b, N)
        assert set(members[b]) == set(keys[mask].tolist())
        np.testing.assert_array_equal(rings[b, :mask.sum()], raw[mask])


def test_rings_rejects_empty_models_and_bad_shapes():
    raw = np.zeros((10, 18), np.float32)
    keys = np.array(["a"] * 10)
    with pytest.raises(ValueError, match="receive no keys"):
        rings_by_key(raw, keys, n_models=4)
    with pytest.raises(ValueError):
        rings_by_key(raw, keys[:5])


def test_fleet_cli_args_and_names():
    from streamml.cli.fleet import model_name, parse_args

    ns = parse_args(["synthetic", "--models", "64", "--epochs", "2"])
    assert ns.models == 64 and ns.epochs == 2 and ns.batch == 32
    assert model_name([["car/1"], ["a", "b"]], 0) == "car_1"
    assert model_name([["car/1"], ["a", "b"]], 1) == "model00001"
