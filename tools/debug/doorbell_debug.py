"""Doorbell streaming-epoch diagnosis: which configurations stall (kernel waiting for rows
that the copy stream never lands)?  Each case runs train_stream with a short timeout and
reports (steps, pushed, consumed, status, seconds)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from streamml.data import stream as S
from streamml.models.autoencoder import Autoencoder


def case(name, fn):
    t0 = time.perf_counter()
    try:
        r = fn()
        print(f"{name}: ok {r} {time.perf_counter() - t0:.2f}s", flush=True)
    except Exception as e:
        print(f"{name}: FAIL {type(e).__name__}: {e} {time.perf_counter() - t0:.2f}s", flush=True)


def main():
    dev = torch.device("cuda", 0)
    raw = torch.from_numpy(np.random.default_rng(0).uniform(0, 40, size=(200_000, 18)).astype(np.float32)).to(dev)

    def direct(extra_streams=0, ring=1 << 20, chunk=5000):
        keep = []
        for _ in range(extra_streams):   # busy normal-priority streams (queue sharing?)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                keep.append(raw.sum())
            keep.append(s)
        m = Autoencoder(device=dev, input_normalizer="cardata", seed=1)
        m.compile()
        chunks = [raw[i:i + chunk] for i in range(0, raw.size(0), chunk)]
        r = m.backend.train_stream(chunks, 100, ring_rows=ring, timeout_s=5.0)
        sr = m.backend._sring
        return r, sr.pushed, sr.consumed, sr.status

    def via_loader(ring=1 << 20):
        m = Autoencoder(device=dev, input_normalizer="cardata", seed=1)
        m.compile()
        src = S.synthetic(60_000, chunk=6_001, seed=4, failure_rate=0.05)
        r = m.backend.train_stream(m._stream_device_chunks(src.filter_normal(device=True)), 100, ring_rows=ring,
                                   timeout_s=5.0)
        sr = m.backend._sring
        return r, sr.pushed, sr.consumed, sr.status

    def via_loader_cloned(ring=1 << 20):
        m = Autoencoder(device=dev, input_normalizer="cardata", seed=1)
        m.compile()
        src = S.synthetic(60_000, chunk=6_001, seed=4, failure_rate=0.05)
        chunks = [c.clone() for c in m._stream_device_chunks(src.filter_normal(device=True))]
        torch.cuda.synchronize()
        r = m.backend.train_stream(chunks, 100, ring_rows=ring, timeout_s=5.0)
        sr = m.backend._sring
        return r, sr.pushed, sr.consumed, sr.status

    case("direct", lambda: direct())
    case("direct_small_ring", lambda: direct(ring=4000))
    case("direct_8_streams", lambda: direct(extra_streams=8))
    case("loader_cloned", via_loader_cloned)
    case("loader", via_loader)
    case("direct_after", lambda: direct())
    print("done", flush=True)


if __name__ == "__main__":
    main()
