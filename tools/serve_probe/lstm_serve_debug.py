"""Debug print of the LSTM forecaster's per-event outputs (flags, scores, forecast[0])."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops.serve import LSTMScoringServer
    dev = torch.device("cuda", 0)
    m = LSTMPredictor.two_layer(look_back=5, device=dev, seed=4)
    rng = np.random.default_rng(5)
    for nkeys, n, batch in ((1, 12, None), (3, 30, None), (3, 30, 1)):
        keys = rng.integers(0, nkeys, size=n)
        raw = rng.uniform(0, 40, size=(n, 18)).astype(np.float32)
        with LSTMScoringServer(m, nkeys=nkeys) as srv:
            if batch:
                outs = [srv.forecast(raw[i:i + 1], keys[i:i + 1]) for i in range(n)]
                pred = np.concatenate([o[0] for o in outs]); s = np.concatenate([o[1] for o in outs])
                f = np.concatenate([o[2] for o in outs])
            else:
                pred, s, f = srv.forecast(raw, keys)
        cnt = {}
        print(f"== nkeys={nkeys} batch={batch}")
        for i in range(n):
            k = int(keys[i])
            c = cnt.get(k, 0)
            print(i, "key", k, "host_cnt", c, "flag", int(f[i]), "score", float(s[i]), "pred0", float(pred[i, 0]))
            cnt[k] = c + 1


if __name__ == "__main__":
    main()
