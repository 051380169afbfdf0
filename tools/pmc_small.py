#!/usr/bin/env python3
"""Driver for counter passes on the persistent small-batch trainers (one mode per run):

    mb32    -- ae_minibatch.hip, Keras fit(batch_size=32)   (BASELINE's 62.7 k rows/s job)
    mb100   -- ae_minibatch.hip, cardata-v3's fit(batch_size=100)
    lstmref -- lstm_ref_train.hip, the reference LSTM stack at look_back 1, batch 1
Each runs 3 launches of ``--steps`` sequential optimizer steps (plus a warm-up launch)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["mb32", "mb100", "lstmref"])
    ap.add_argument("--steps", type=int, default=20000)
    a = ap.parse_args()
    import torch
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    dev = torch.device("cuda", 0)
    sc, sh = normalize_affine()
    if a.mode.startswith("mb"):
        from streamml.models.reference import init_dense_weights
        from streamml.ops.ae import AESpec, FusedAE
        B = 32 if a.mode == "mb32" else 100
        spec = AESpec()
        data = synthetic_device_tensor(B * 32768, dev, seed=0)
        ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), dev, scale=sc, shift=sh)
        ae.attach_ring(data, B)
        if os.environ.get("SML_PMC_NOACC") == "1":   # A/B: the accuracy's cost on the step
            ae.want_acc = False
        for _ in range(3):
            ae.train_minibatches(a.steps)
        import time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ae.train_minibatches(a.steps)
        torch.cuda.synchronize()
        print(f"{a.mode}: {(time.perf_counter() - t0) / a.steps * 1e6:.3f} us/step", flush=True)
    else:
        from streamml.data.stream import sliding_windows
        from streamml.models.lstm import LSTMPredictor
        from streamml.ops import lstm_persistent as lp
        n = a.steps + 1
        raw = synthetic_device_tensor(n + 1, dev, seed=0)
        xn = (raw * torch.tensor(sc, device=dev) + torch.tensor(sh, device=dev)).contiguous()
        X, Y = sliding_windows(xn, 1)
        m = LSTMPredictor.reference(look_back=1, device=dev)
        for _ in range(4):
            lp.train_steps(m, X, Y, 1, a.steps)
    torch.cuda.synchronize()
    print("ok", a.mode)


if __name__ == "__main__":
    main()
