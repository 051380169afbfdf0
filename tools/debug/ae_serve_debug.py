"""One-event AE scorer diagnosis: submit one row, and if no result arrives dump the ring
state (head, done, stop, alive, launches, stream idle) and the slot's raw words."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch


def dump(srv, seq, tag):
    v = list(srv._s.debug_state(seq))
    print(tag, "head/done/stop/alive/launches/idle:", v[:6], flush=True)
    res = v[6:6 + 40]
    req = v[6 + 40:]
    print("  result words 34..39 (timing fields, padding):",
          [hex(w) for w in res[34:40]], flush=True)
    print("  res tags:", [w >> 32 for w in res], flush=True)
    print("  req tags:", [w >> 32 for w in req], flush=True)


def main():
    from streamml.models.autoencoder import Autoencoder
    from streamml.ops.serve import ScoringServer
    dev = torch.device("cuda", 0)
    m = Autoencoder(device=dev, input_normalizer="cardata")
    m.compile()
    rows = np.random.default_rng(0).uniform(0, 40, size=(300, 18)).astype(np.float32)
    with ScoringServer(m, slots=256, idle_seconds=2.0) as srv:
        time.sleep(0.2)
        dump(srv, 0, "before")
        for i in range(3):
            try:
                s, f = srv.score(rows[i:i + 1]) if hasattr(srv, "score") else (None, None)
                print("event", i, "ok", s, f, flush=True)
            except Exception as e:
                print("event", i, "FAILED", e, flush=True)
                dump(srv, i, "after")
                break
        try:
            s, f = srv.score(rows[10:200])
            print("batch of 190 ok", float(s.mean()), flush=True)
        except Exception as e:
            print("batch FAILED", e, flush=True)


if __name__ == "__main__":
    main()
