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


def test_fleet_trains_on_normal_rows_only():
    """failure rows must never reach a per-car anomaly model's ring."""
    from streamml.cli.fleet import parse_args, training_rows
    from streamml.data.cardata import SyntheticCarSource
    ns = parse_args(["synthetic", "--synthetic-rows", "20000", "--synthetic-devices", "50", "--seed", "3"])
    raw, keys = training_rows(ns)
    all_raw, fail, _, _ = SyntheticCarSource(seed=3, n_devices=50).generate(20000)
    assert fail.any() and len(raw) == int((~fail).sum()) == len(keys)
    np.testing.assert_array_equal(raw, all_raw[~fail])


def test_fleet_model_names_never_collide():
    from streamml.cli.fleet import model_name
    members = [["car/1"], ["car_1"], ["model00003"], ["a", "b"], ["car:1"]]
    used = set()
    names = [model_name(members, i, used) for i in range(len(members))]
    assert len(set(names)) == len(names)
    assert names[0] == "car_1" and names[1] == "car_1-1" and names[3] == "model00003-3"


def test_ragged_rings_no_padding_to_the_largest_group():
    from streamml.ops.ae_fleet import ragged_rings_by_key
    raw = np.arange(10 * 2, dtype=np.float32).reshape(10, 2)
    keys = np.array(["a"] * 7 + ["b"] * 3)
    flat, table, members = ragged_rings_by_key(raw, keys, batch=4)
    assert members == [["a"], ["b"]]
    np.testing.assert_array_equal(table, [[0, 8], [8, 4]])   # 7 -> 8 rows, 3 -> 4 rows
    np.testing.assert_array_equal(flat[:7], raw[:7])
    np.testing.assert_array_equal(flat[7], raw[0])            # one cyclic pad row
    np.testing.assert_array_equal(flat[8:11], raw[7:])
