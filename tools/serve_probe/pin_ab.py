"""A/B of the Kafka e2e thread placement (bench/bench_infer.kafka_e2e ``pin``): unpinned vs
the scoring loop, producer and broker connection threads on one L3 domain, alternating, for
the autoencoder and the per-car LSTM scorers.  10 000 events at 10 000 events/s per run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def main():
    import torch
    from bench_infer import _l3_cpus, kafka_e2e
    from streamml.data.cardata import synthetic_device_tensor
    from streamml.models.autoencoder import Autoencoder
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops.serve import LSTMScoringServer
    print(json.dumps({"affinity": len(os.sched_getaffinity(0)), "l3_cpus": _l3_cpus(5)}), flush=True)
    dev = torch.device("cuda", 0)
    m = Autoencoder(device=dev, input_normalizer="cardata")
    m.compile()
    lm = LSTMPredictor.reference(look_back=1, device=dev)
    ev = synthetic_device_tensor(10200, dev, seed=3).cpu().numpy()
    reps = int(os.environ.get("PIN_AB_REPS", "3"))
    for rep in range(reps):
        for pin in (False, "l3"):
            for name, kw in (("ae", {}), ("lstm", {"make_scorer": lambda: LSTMScoringServer(lm, nkeys=1000,
                                                                                           threshold=5.0)})):
                r = kafka_e2e(m if name == "ae" else None, ev, 10000.0, 5.0, 10000, warm=200, pin=pin, **kw)
                r = {k: r[k] for k in ("p50_us", "p99_us", "legs_p50_us", "pinned_cpus", "pin")}
                r.update(scorer=name, rep=rep, mode=str(pin))
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
