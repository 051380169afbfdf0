"""A/B of the seq-50 per-event LSTM forecaster: pipelined stack kernel vs the
barrier-per-step kernel (SML_LSTM_SERVE_GENERIC=1), same process, same events.
Prints one JSON line per variant (bench.measure_lstm_seq50_infer's record)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    dev = torch.device("cuda", 0)
    for generic in ("1", "0"):
        os.environ["SML_LSTM_SERVE_GENERIC"] = generic
        r = bench.measure_lstm_seq50_infer(dev, n, 3)
        r["variant"] = "generic (barrier per step)" if generic == "1" else "pipelined (wave per layer)"
        print(json.dumps(r), flush=True)
