#!/usr/bin/env python3
"""BASELINE config 3: LSTM sensor predictor (seq_len=50, 2-layer) bf16, synthetic stream, 1x MI355X.

Model: LSTM(32, relu, return_sequences) -> LSTM(16, relu) -> Dense(18) predicting
the next car event from a 50-event window (LSTM-.../cardata-v2.py task with
look_back=50).  Each timed step = forward (bf16 input-projection GEMMs + fused HIP
recurrence) + backward (fused HIP BPTT + weight-gradient GEMMs) + HIP Adam.
Prints one JSON line: windows/s and events/s (= windows/s * seq_len).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=None, help="default 65536 (two_layer) / 1 (reference)")
    ap.add_argument("--seq-len", type=int, default=None, help="default 50 (two_layer) / 1 (reference)")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--stack", default="two_layer", choices=["two_layer", "reference"])
    ap.add_argument("--materialize", action="store_true", help="copy every window ([n, T, F]) instead of views")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay each train step (fwd + bwd + Adam) as a captured HIP graph "
                         "(measured: 54.1 vs 55.1 M windows/s eager -- the step is GPU-bound, not launch-bound)")
    args = ap.parse_args()
    ref = args.stack == "reference"
    args.batch = args.batch or (1 if ref else 65536)
    args.seq_len = args.seq_len or (1 if ref else 50)
    if ref and args.seq_len == 1 and args.batch <= 32:
        print(json.dumps(measure_reference(batch=args.batch)))
        return
    print(json.dumps(measure_seq(batch=args.batch, seq_len=args.seq_len, steps=args.steps, warmup=args.warmup,
                                 stack=args.stack, materialize=args.materialize, graph=bool(args.graph))))


def measure_seq(batch: int = 65536, seq_len: int = 50, steps: int = 30, warmup: int = 5, stack: str = "two_layer",
                materialize: bool = False, graph: bool = False, device=None, settle_ms: float = 100.0,
                windows: int = 3) -> dict:
    """Train windows/s of an LSTM stack on sliding windows of synthetic car events.

    Before the ``warmup`` steps, full train steps run untimed until ``settle_ms`` of GPU time
    has passed: the same DPM clock settle as the headline (bench.py docstring) -- a 20-step
    timed region (~20 ms) is otherwise inside the ~30 ms power-management transient."""
    import torch
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.models.lstm import LSTMPredictor

    dev = torch.device(device) if device is not None else torch.device("cuda", 0)
    T, B = seq_len, batch
    ctor = LSTMPredictor.two_layer if stack == "two_layer" else LSTMPredictor.reference
    m = ctor(look_back=T, device=dev)
    sc, sh = normalize_affine()
    raw = synthetic_device_tensor(B * 4 + T + 1, dev, seed=0)
    xn = raw * torch.tensor(sc, dtype=torch.float32, device=dev) + torch.tensor(sh, dtype=torch.float32, device=dev)
    # sliding windows [n, T, 18] -> next row targets, read IN PLACE from the event rows
    # (strided views; cardata-v2.py:199-206's window(look_back, shift=1) + skip(look_back))
    from streamml.data.stream import sliding_windows
    n = B * 4
    X, Y = sliding_windows(xn[:n + T].contiguous(), T)
    if materialize:   # the round-1 layout: every window copied (T x the input bytes)
        X, Y = X.contiguous(), Y.contiguous()
    settle_steps = 0
    ts = time.perf_counter()
    while True:
        i = settle_steps % 4
        m.train_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B])
        settle_steps += 1
        if settle_steps % 4 == 0:
            torch.cuda.synchronize()
            if (time.perf_counter() - ts) * 1e3 >= settle_ms:
                break
    for s in range(warmup):
        i = s % 4
        m.train_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B])
    torch.cuda.synchronize()
    step = lambda s: m.train_step(X[(s % 4) * B:(s % 4 + 1) * B], Y[(s % 4) * B:(s % 4 + 1) * B])
    if graph:
        from streamml.utils.graphs import capture_steps
        step = capture_steps([lambda i=i: m.train_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B])
                              for i in range(4)])
    # `windows` back-to-back timed windows of `steps` steps each; the value is the median window's
    # (a one-off DPM / thermal dip inside one ~13 ms window -- seen once at -14 % in a full
    # bench.py run, profiles/r06/SUMMARY.md §8 -- does not set the number; every window is kept)
    times = []
    for _ in range(max(1, windows)):
        t0 = time.perf_counter()
        for s in range(steps):
            loss, _ = step(s)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]
    wps = B * steps / dt
    return {"metric": "LSTM train windows/s (seq_len=%d, %s)" % (T, stack), "value": wps,
            "unit": "windows/s", "events_per_s": wps * T, "ms_per_step": dt / steps * 1e3,
            "batch": B, "seq_len": T, "steps": steps, "params": m.count_params(), "dtype": "bf16",
            "final_loss": float(loss), "n_gpus": 1, "data": "synthetic", "hip_graph": bool(graph),
            "windows": "materialized" if materialize else "in-place strided views",
            "clock_settle": {"ms": settle_ms, "steps": settle_steps},
            "timed_windows_ms_per_step": [round(t / steps * 1e3, 4) for t in times]}


def measure_seq_dp(batch: int = 65536, seq_len: int = 50, steps: int = 10, warmup: int = 3, device=None,
                   settle_ms: float = 100.0, rank: int = 0, world: int = 1) -> dict:
    """BASELINE config 3 under data parallelism (weak scaling): every rank trains the two-layer stack on
    its OWN ``batch`` windows per step (synthetic events seeded by rank), and the gradient of the
    global batch is one flat fp32 bucket all-reduced per step (RCCL over xGMI on the 8-GPU node;
    ``parallel.dp.allreduce_sum_``), after rank 0's initial parameters and Adam state are broadcast.
    Collective: every rank calls it with the same arguments.  The elapsed time is the max over ranks;
    the replicas' parameters are compared at the end (they must stay bit-identical)."""
    import torch
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.data.stream import sliding_windows
    from streamml.models.lstm import LSTMPredictor
    from streamml.parallel import dp

    dev = torch.device(device) if device is not None else torch.device("cuda", 0)
    T, B = seq_len, batch
    m = LSTMPredictor.two_layer(look_back=T, device=dev, seed=0)
    dp.sync_model_from_rank0(m)
    sc, sh = normalize_affine()
    raw = synthetic_device_tensor(B * 2 + T + 1, dev, seed=1 + rank)
    xn = raw * torch.tensor(sc, dtype=torch.float32, device=dev) + torch.tensor(sh, dtype=torch.float32, device=dev)
    X, Y = sliding_windows(xn[:2 * B + T].contiguous(), T)
    gb = B * world

    def step(s):
        i = s % 2
        return m.train_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B], global_batch=gb, allreduce=dp.allreduce_sum_)

    settle_steps = 0
    ts = time.perf_counter()
    while True:   # clock settle, one decision for all ranks (collectives stay paired)
        for _ in range(2):
            step(settle_steps)
            settle_steps += 1
        torch.cuda.synchronize()
        if dp.allreduce_max((time.perf_counter() - ts) * 1e3, dev) >= settle_ms:
            break
    for s in range(warmup):
        step(s)
    dp.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        loss, _ = step(s)
    torch.cuda.synchronize()
    dp.barrier(dev)
    el = dp.allreduce_max(time.perf_counter() - t0, dev)
    flat = m.fp.flat.detach()
    ref = flat.clone()
    dp.broadcast_(ref, 0)
    diverged = float((flat - ref).abs().max().item())
    diverged = dp.allreduce_max(diverged, dev)
    wps = gb * steps / el
    return {"metric": "LSTM train windows/s (seq_len=%d, two_layer, data parallel)" % T, "value": wps,
            "unit": "windows/s", "ms_per_step": el / steps * 1e3, "batch_per_rank": B, "global_batch": gb,
            "world": world, "steps": steps, "scaling": "weak", "final_loss": float(loss),
            "allreduce": "one flat fp32 gradient bucket per step (RCCL)", "replica_max_abs_diff": diverged,
            "clock_settle": {"ms": settle_ms, "steps": settle_steps}}


def measure_reference(batch: int = 1, epochs: int = 5, steps_per_epoch: int = 1000, autograd_steps: int = 300,
                      device=None) -> dict:
    """cardata-v2.py:172-209 as the reference runs it: look_back 1, batch 1, 1 000 steps x
    5 epochs, one Adam update per event.  Persistent kernel (one launch per epoch) vs the
    per-step autograd path (fused LSTM kernels, ~10 launches per step)."""
    import numpy as np
    import torch
    from streamml.data.cardata import normalize_affine, synthetic_device_tensor
    from streamml.data.stream import sliding_windows
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops import lstm_persistent as lp

    dev = torch.device(device) if device is not None else torch.device("cuda", 0)
    B = batch
    n = max(steps_per_epoch, autograd_steps + 20) * B
    sc, sh = normalize_affine()
    raw = synthetic_device_tensor(n + 1, dev, seed=0)
    xn = (raw * torch.tensor(sc, dtype=torch.float32, device=dev)
          + torch.tensor(sh, dtype=torch.float32, device=dev)).contiguous()
    X, Y = sliding_windows(xn, 1)
    m = LSTMPredictor.reference(look_back=1, device=dev)
    lp.train_steps(m, X, Y, B, 50)          # warm-up (module load, LDS opt-in)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in range(epochs):                  # one launch per epoch, as fit() does
        out = lp.train_steps(m, X, Y, B, steps_per_epoch)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = epochs * steps_per_epoch
    # the same steps through the autograd path (per-step launches), fewer of them
    ma = LSTMPredictor.reference(look_back=1, device=dev)
    for i in range(20):
        ma.train_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B])
    torch.cuda.synchronize()
    na = autograd_steps
    t1 = time.perf_counter()
    for i in range(na):
        ma.train_step(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B])
    torch.cuda.synchronize()
    da = time.perf_counter() - t1
    return {"metric": "LSTM reference stack Keras step time (look_back=1, batch=%d)" % B,
            "value": dt / steps * 1e6, "unit": "us/step", "higher_is_better": False,
            "steps_per_s": steps / dt, "events_per_s": steps * B / dt, "steps": steps,
            "epochs": epochs, "steps_per_epoch": steps_per_epoch, "launches": epochs,
            "autograd_us_per_step": da / na * 1e6, "speedup_vs_autograd": (da / na) / (dt / steps),
            "final_loss": float(out[-1, 0]), "params": m.count_params(), "dtype": "fp32",
            "n_gpus": 1, "data": "synthetic", "engine": "persistent (lstm_ref_train.hip)"}


if __name__ == "__main__":
    main()
