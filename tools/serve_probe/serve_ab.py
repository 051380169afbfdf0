"""Per-event scorer latency, one configuration per process (env decides, e.g.
SML_SERVE_STORES=nt): prints p50/p99 of 3 x 20 000 events at 10 000 events/s, the AE
scorer and the LSTM forecaster (look_back 1 reference stack)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch


def main():
    from streamml.data.cardata import synthetic_device_tensor
    from streamml.models.autoencoder import Autoencoder
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops.serve import LSTMScoringServer, ScoringServer
    dev = torch.device("cuda", 0)
    ev = synthetic_device_tensor(21000, dev, seed=5).cpu().numpy()
    m = Autoencoder(device=dev, input_normalizer="cardata")
    m.compile()
    out = {"stores": os.environ.get("SML_SERVE_STORES", "cached")}
    with ScoringServer(m, slots=4096) as srv:
        srv.latency_us(ev[:1000], qps=10000)
        p = []
        for _ in range(3):
            host, devt, _, _ = srv.latency_us(ev[1000:], qps=10000, device_breakdown=True)
            p.append((float(np.percentile(host, 50)), float(np.percentile(host, 99)), float(np.percentile(devt, 50))))
        out["ae"] = p
    lm = LSTMPredictor.reference(look_back=1, device=dev)
    keys = np.arange(21000) % 100
    with LSTMScoringServer(lm, nkeys=100) as srv:
        srv.latency_us(ev[:1000], keys[:1000], qps=10000)
        p = []
        for _ in range(3):
            host = srv.latency_us(ev[1000:], keys[1000:], qps=10000)
            p.append((float(np.percentile(host, 50)), float(np.percentile(host, 99))))
        out["lstm_ref"] = p
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
