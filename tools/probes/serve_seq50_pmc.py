"""Pipelined seq-50 forecaster under a counter pass: 3000 events at full speed (qps 0)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from streamml.data.cardata import synthetic_device_tensor  # noqa: E402
from streamml.models.lstm import LSTMPredictor  # noqa: E402
from streamml.ops.serve import LSTMScoringServer  # noqa: E402

dev = torch.device("cuda", 0)
ev = synthetic_device_tensor(8000, dev, seed=9).cpu().numpy()
keys = np.arange(8000) % 100
m = LSTMPredictor.two_layer(look_back=50, device=dev)
with LSTMScoringServer(m, nkeys=100) as srv:
    srv.latency_us(ev[:5000], keys[:5000], qps=0)
    lat = srv.latency_us(ev[5000:], keys[5000:], qps=0)
print("p50_us", float(np.percentile(lat, 50)))
