#!/usr/bin/env python3
"""AE training at the reference's own batch size (Keras ``fit(batch_size=32)``).

The headline bench (``bench.py``) runs one optimizer step per 32 M rows.  The
reference steps Adam every 32 rows (cardata-v3.py:187-203; the creditcard notebook's
Keras log, BASELINE.md: 62.5-66.7 k rows/s).  This bench measures the same
per-32-row semantics on one MI355X, three ways:

* ``persistent``: ``FusedAE.train_minibatches`` -- ONE launch runs ``--steps-per-launch``
  sequential Keras steps (csrc/kernels/ae_minibatch.hip, fp32);
* ``launch``: ``FusedAE.step_ring`` per step (train kernel + reduce/Adam kernel, bf16 MFMA);
* the numbers are rows/s and us per optimizer step.
Data: synthetic raw car-sensor rows resident in HBM; weights: random Glorot init.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def measure(device, batch=32, steps_per_launch=20000, launches=5, launch_steps=2000):
    import torch

    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.models.reference import init_dense_weights
    from streamml.ops.ae import AESpec, FusedAE

    spec = AESpec()
    scale, shift = normalize_affine()
    rows = batch * 32768                      # 1 M rows for batch 32: a ring, not one pass
    data = synthetic_device_tensor(rows, device, seed=0, n_devices=100_000)
    out = {}

    ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), device, scale=scale, shift=shift)
    ae.attach_ring(data, batch)
    ae.train_minibatches(steps_per_launch)    # warm-up launch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(launches):
        ae.train_minibatches(steps_per_launch)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = launches * steps_per_launch
    out["persistent_rows_per_s"] = n * batch / dt
    out["persistent_us_per_step"] = dt / n * 1e6
    out["persistent_final_loss"] = ae.read_metrics()["loss"]
    # one profiled launch: per-phase shader cycles of wave 0 (phase A = register fwd/bwd
    # chain of its 16 rows, barrier, phase B = weight-gradient MFMAs + Adam, barrier)
    prof = torch.zeros(11, dtype=torch.int64, device=device)
    ae.train_minibatches(steps_per_launch, prof=prof)
    torch.cuda.synchronize()
    pc = prof.cpu().tolist()
    names = ["phaseA_fwd_bwd", "barrier1", "phaseB_wgrad_adam", "barrier2"]
    out["phase_cycles_per_step"] = {n: pc[i] / steps_per_launch for i, n in enumerate(names)}
    out["cycles_per_step"] = pc[8] / steps_per_launch

    ae2 = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), device, scale=scale, shift=shift)
    ae2.attach_ring(data, batch)
    for _ in range(200):
        ae2.step_ring()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(launch_steps):
        ae2.step_ring()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["launch_rows_per_s"] = launch_steps * batch / dt
    out["launch_us_per_step"] = dt / launch_steps * 1e6
    return out


def measure_fleet(device, n_models, batch=32, steps_per_launch=2000, launches=3):
    """Fleet mode: ``n_models`` independent models, one workgroup each (ops/ae_fleet.py)."""
    import torch

    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.ops.ae import AESpec
    from streamml.ops.ae_fleet import AEFleet

    spec = AESpec()
    scale, shift = normalize_affine()
    rows = batch * 32768
    data = synthetic_device_tensor(rows, device, seed=0, n_devices=100_000)
    fleet = AEFleet.from_seeds(spec, range(n_models), device, scale=scale, shift=shift)
    stride = (rows // n_models // batch) * batch
    fleet.attach_rings(data, batch, offsets=[i * stride for i in range(n_models)])
    fleet.train_minibatches(steps_per_launch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(launches):
        fleet.train_minibatches(steps_per_launch)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = launches * steps_per_launch
    return {"models": n_models, "rows_per_s": n_models * n * batch / dt, "us_per_step_per_model": dt / n * 1e6,
            "mean_final_loss": sum(m["loss"] for m in fleet.read_metrics()) / n_models}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps-per-launch", type=int, default=20000)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--fleet", default="256,512,768,1024,1536",
                    help="comma-separated fleet sizes for the multi-model sweep ('' = skip)")
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    r = measure(dev, args.batch, args.steps_per_launch, args.launches)
    if args.fleet:
        r["fleet"] = [measure_fleet(dev, int(m), args.batch) for m in args.fleet.split(",")]
    base = 62661.0
    print(json.dumps({"metric": "AE train rows/s at Keras batch 32 (one Adam step per batch)",
                      "value": r["persistent_rows_per_s"], "unit": "rows/s", "vs_baseline": r["persistent_rows_per_s"] / base,
                      "batch": args.batch, "dtype": "fp32", "n_gpus": 1, "data": "synthetic", **r}), flush=True)


if __name__ == "__main__":
    main()
