"""torchrun worker for tests/test_stream_dp.py (CPU, gloo) and tests/test_stream_dp_gpu.py
(every rank on GPU 0, SML_SHARE_GPU0=1): data-parallel ``Autoencoder.fit`` over this rank's
share of a partitioned Kafka topic served by the parent test's in-process broker.

argv: out_dir broker_addr topic batch epochs device assign native engine dp

Per rank it writes ``rank<R>.npz``: the (partition, offset) of every record its share held
(the Python reader, one pass), the shares themselves, the final weights, the Adam iteration
count and the per-epoch history."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from streamml.parallel.dp import init_from_env, shutdown, sync_model_from_rank0  # noqa: E402


def main(out_dir, addr, topic, batch, epochs, device, assign, native, engine, dp):
    env = init_from_env(device)
    rank = env.rank
    from streamml.data import stream as st
    from streamml.models.autoencoder import Autoencoder
    native = native == "1" and env.device.type == "cuda"
    # pass 1: which records did this rank's share hold (Python reader: partitions + offsets)
    probe = st.kafka(addr, [f"{topic}:*:0"], shard="auto", assign=assign)
    parts, offs, labels = [], [], []
    for c in probe:
        parts.append(np.full(len(c), int(c.meta["partition"]), np.int64))
        offs.append(np.asarray(c.offsets, np.int64))
        labels.append(c.label)
    shares = np.array([[s.partition, s.start, s.end] for s in probe.plan.last], np.int64).reshape(-1, 3)
    parts = np.concatenate(parts) if parts else np.zeros(0, np.int64)
    offs = np.concatenate(offs) if offs else np.zeros(0, np.int64)
    labels = np.concatenate(labels) if labels else np.zeros(0, np.uint8)
    # pass 2: train on the share, straight from the stream (native feed on the GPU)
    src = st.kafka(addr, [f"{topic}:*:0"], shard="auto", assign=assign, native=native, workers=2)
    ae = Autoencoder(device=env.device, input_normalizer="cardata", seed=7)
    ae.compile()
    sync_model_from_rank0(ae)
    h = ae.fit(src.filter_normal(device=True), epochs=int(epochs), batch_size=int(batch), verbose=0,
               engine=engine, dp=dp)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), *ae.get_weights(), parts=parts, offs=offs, labels=labels,
             shares=shares, iterations=np.array(ae.iterations), loss=np.array(h.history["loss"]),
             rows=np.array(h.history["_rows"]), engine=np.array(ae.last_fit_engine))
    shutdown()


if __name__ == "__main__":
    torch.set_num_threads(2)
    main(*sys.argv[1:11])
