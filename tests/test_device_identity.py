"""Refusal logic of a multi-GPU bench record (bench.py): ``n_gpus = N`` needs N distinct devices
(host + UUID / PCI bus id) unless the run is a labelled one-GPU rehearsal (SML_SHARE_GPU0=1)."""
import torch

from streamml.parallel import dp


def _id(host, uuid, bus="0000:05:00.0"):
    return {"host": host, "uuid": uuid, "pci_bus_id": bus, "device": "cuda:0", "pid": 1}


def test_distinct_devices_accepted():
    ids = [_id("h", f"GPU-{k}", f"0000:{k:02x}:00.0") for k in range(8)]
    r = dp.check_distinct_devices(ids, 8, rehearsal=False)
    assert r["ok"] and r["n_distinct_devices"] == 8 and not r["rehearsal"]


def test_shared_device_refused_unless_rehearsal():
    ids = [_id("h", "GPU-0")] * 4
    r = dp.check_distinct_devices(ids, 4, rehearsal=False)
    assert not r["ok"] and r["n_distinct_devices"] == 1 and "distinct" in r["reason"]
    r = dp.check_distinct_devices(ids, 4, rehearsal=True)
    assert r["ok"] and r["n_distinct_devices"] == 1 and r["rehearsal"]


def test_partial_overlap_refused():
    ids = [_id("h", "GPU-0"), _id("h", "GPU-1"), _id("h", "GPU-1"), _id("h", "GPU-3")]
    r = dp.check_distinct_devices(ids, 4, rehearsal=False)
    assert not r["ok"] and r["n_distinct_devices"] == 3


def test_same_uuid_on_two_hosts_is_two_devices():
    ids = [_id("a", "GPU-0"), _id("b", "GPU-0")]
    assert dp.check_distinct_devices(ids, 2, rehearsal=False)["ok"]


def test_bus_id_used_without_uuid():
    ids = [_id("h", "", "0000:05:00.0"), _id("h", "", "0000:06:00.0")]
    assert dp.check_distinct_devices(ids, 2, rehearsal=False)["ok"]
    ids = [_id("h", "", "0000:05:00.0"), _id("h", "", "0000:05:00.0")]
    assert not dp.check_distinct_devices(ids, 2, rehearsal=False)["ok"]


def test_missing_identity_refused():
    r = dp.check_distinct_devices([_id("h", "GPU-0")], 2, rehearsal=True)
    assert not r["ok"] and "identities" in r["reason"]


def test_cpu_identity_and_world1():
    me = dp.device_identity(torch.device("cpu"))
    assert me["host"] and me["pid"] > 0 and me["device"] == "cpu"
    assert dp.check_distinct_devices([me], 1, rehearsal=False)["ok"]
    assert dp.peer_access(torch.device("cpu"), [0, 1]) == {}
