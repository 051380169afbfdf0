"""LSTM forecaster (look_back 1 reference stack) per-event latency legs: host p50/p99, the
device's pick-up -> results-stored time and its compute part (3 x 20 000 events at
10 000 events/s)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch


def main():
    from streamml.data.cardata import synthetic_device_tensor
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops.serve import LSTMScoringServer
    dev = torch.device("cuda", 0)
    ev = synthetic_device_tensor(21000, dev, seed=5).cpu().numpy()
    nkeys = int(os.environ.get("SML_KEYS", "100"))
    keys = np.arange(21000) % nkeys
    lm = LSTMPredictor.reference(look_back=1, device=dev)
    out = {"keys": nkeys, "runs": []}
    with LSTMScoringServer(lm, nkeys=nkeys) as srv:
        srv.latency_us(ev[:1000], keys[:1000], qps=10000)
        for _ in range(3):
            host, done, comp = srv.latency_us(ev[1000:], keys[1000:], qps=10000, device_breakdown=True)
            out["runs"].append({"p50_us": float(np.percentile(host, 50)), "p99_us": float(np.percentile(host, 99)),
                                "device_done_p50_us": float(np.percentile(done, 50)),
                                "device_compute_p50_us": float(np.percentile(comp, 50))})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
