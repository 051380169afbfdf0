"""Why is the scoring leg inside the Kafka loop (~4.8 us, profiles/r03) slower than the
standalone scorer (~3.9 us)?  The loop runs in a Python worker thread, the standalone
measurement in the main thread that allocated the host-mapped rings.  This probe times the
SAME persistent scorer's per-event round trip (ScoringServer.latency_us, C++ loop, GIL
released) from the main thread, from a fresh worker thread, and from worker threads pinned
to the CPUs of the GPU's NUMA node and of another node, 3 x 20 000 events at 10 000 events/s
each, and prints one JSON line per case."""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np


def gpu_numa_node(index: int = 0) -> int:
    import glob
    for card in sorted(glob.glob("/sys/class/drm/card*/device/numa_node")):
        try:
            with open(card) as f:
                return int(f.read().strip())
        except (OSError, ValueError):
            continue
    return -1


def node_cpus(node: int):
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
    except OSError:
        return []
    out = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return [c for c in out if c in os.sched_getaffinity(0)]


def run_case(srv, ev, label, cpu=None, in_thread=True):
    res = {}

    def body():
        if cpu is not None:
            os.sched_setaffinity(0, {cpu})
        srv.latency_us(ev[:1000], qps=10000.0)
        p50s = []
        for _ in range(3):
            lat = srv.latency_us(ev[1000:], qps=10000.0)
            p50s.append(float(np.percentile(lat, 50)))
        res.update({"case": label, "cpu": cpu, "p50_us": float(np.median(p50s)), "p50_runs": p50s})

    if in_thread:
        th = threading.Thread(target=body)
        th.start()
        th.join()
    else:
        body()
    print(json.dumps(res), flush=True)


def main():
    import torch

    from streamml.data.cardata import synthetic_device_tensor
    from streamml.models.autoencoder import Autoencoder
    from streamml.ops.serve import ScoringServer
    dev = torch.device("cuda", 0)
    m = Autoencoder(device=dev, input_normalizer="cardata")
    m.compile()
    ev = synthetic_device_tensor(21000, dev, seed=3).cpu().numpy()
    node = gpu_numa_node()
    near = node_cpus(node) if node >= 0 else []
    far = [c for n in range(8) if n != node for c in node_cpus(n)]
    print(json.dumps({"gpu_numa_node": node, "near_cpus": near[:8], "far_cpus": far[:8],
                      "main_affinity": sorted(os.sched_getaffinity(0))[:16]}), flush=True)
    with ScoringServer(m, slots=4096) as srv:
        run_case(srv, ev, "main thread", in_thread=False)
        run_case(srv, ev, "worker thread")
        if near:
            run_case(srv, ev, "worker pinned near the GPU", cpu=near[len(near) // 2])
        if far:
            run_case(srv, ev, "worker pinned on another NUMA node", cpu=far[len(far) // 2])
        run_case(srv, ev, "main thread again", in_thread=False)


if __name__ == "__main__":
    main()
