#!/usr/bin/env python3
"""End-to-end streaming ingest: Kafka (in-process broker over TCP) -> native fetch +
Avro decode -> pinned ring -> H2D -> fused AE train steps.  Reports rows/s of the
whole pipeline and of each host stage in isolation."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--fetch-bytes", type=int, default=4 << 20)
    ap.add_argument("--partitions", type=int, default=8, help="sensor-data has 10 in the reference")
    ap.add_argument("--workers", type=int, default=8, help="partition-parallel fetch+decode threads")
    args = ap.parse_args()
    import numpy as np
    import torch
    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    from streamml.models.autoencoder import Autoencoder

    b = fake_broker("ingest")
    P = args.partitions
    b.create_topic("SENSOR_DATA_S_AVRO", P)
    codec = AvroCodec("cardata-v1")
    t0 = time.perf_counter()
    for i, c in enumerate(S.synthetic(args.rows, chunk=250_000, seed=0, failure_rate=0.0)):
        buf, offs = encode_chunk(codec, c.x, c.label)
        b.append_buffer("SENSOR_DATA_S_AVRO", i % P, buf, offs)
    t_produce = time.perf_counter() - t0
    src = S.kafka("fake://ingest", [f"SENSOR_DATA_S_AVRO:{p}:0" for p in range(P)], max_bytes=args.fetch_bytes,
                  workers=args.workers)
    t0 = time.perf_counter()
    n = sum(len(c) for c in src)
    t_decode = time.perf_counter() - t0
    dev = torch.device("cuda", 0)
    m = Autoencoder(device=dev, input_normalizer="cardata")
    m.compile()
    m.fit(src, epochs=1, batch_size=args.batch, verbose=0)   # warm-up epoch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = m.fit(src, epochs=1, batch_size=args.batch, verbose=0)
    torch.cuda.synchronize()
    t_e2e = time.perf_counter() - t0
    print(json.dumps({"metric": "streaming ingest+train rows/s (Kafka->Avro->ring->H2D->fused AE)",
                      "value": n / t_e2e, "unit": "rows/s", "rows": n, "fetch_decode_rows_per_s": n / t_decode,
                      "produce_rows_per_s": args.rows / t_produce, "batch": args.batch,
                      "partitions": P, "workers": args.workers,
                      "loss": h.history["loss"][-1], "data": "synthetic"}))


if __name__ == "__main__":
    main()
