"""torchrun worker for tests/test_p2p_gpu.py: one rank of a P2P (IPC / xGMI) data-parallel
group.  Trains the autoencoder at Keras batch 32 with the gradient exchange inside the
persistent kernel, runs the host-callable P2P all-reduce, and dumps what the test checks."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    out = sys.argv[1]
    from streamml.data.cardata import normalize_affine
    from streamml.models.reference import init_dense_weights
    from streamml.ops.ae import AESpec, FusedAE
    from streamml.parallel import dp
    from streamml.parallel.p2p import P2PGroup

    env = dp.init_from_env("cuda")
    rank, world, dev = env.rank, env.world_size, env.device
    group = P2PGroup(dev, timeout_s=20.0)
    # host-callable all-reduce: rank r contributes 1000 r + i (exact in fp32)
    x = (torch.arange(1540, device=dev, dtype=torch.float32) + 1000.0 * rank).contiguous()
    group.allreduce_(x)
    group.check()
    want = sum(torch.arange(1540, dtype=torch.float32) + 1000.0 * r for r in range(world))
    ar_ok = bool(torch.equal(x.cpu(), want))
    # latency of the one-launch all-reduce on the 6 KB bucket (both ranks share one GPU here)
    import time
    for _ in range(20):
        group.allreduce_(x)
    torch.cuda.synchronize()
    dp.barrier(dev)
    t0 = time.perf_counter()
    for _ in range(200):
        group.allreduce_(x)
    torch.cuda.synchronize()
    ar_us = (time.perf_counter() - t0) / 200 * 1e6
    group.check()
    # DP training: every rank starts from the same weights, trains on its own rows
    spec = AESpec()
    sc, sh = normalize_affine()
    ae = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=5), dev, scale=sc, shift=sh)
    rng = np.random.default_rng(100 + rank)
    raw = torch.from_numpy(rng.uniform(0, 40, (32 * 40, 18)).astype(np.float32)).to(dev)
    steps, _ = ae.train_rows(raw, 32, dp=group)
    steps2, _ = ae.train_rows(raw, 32, dp=group, chunk_steps=7)   # several launches, tags continue
    torch.cuda.synchronize()
    np.save(f"{out}.rank{rank}.npy", ae.params.cpu().numpy())
    # the user-facing entry point: Autoencoder.fit under DP (array shards, a rank-sharded
    # stream, and the local-SGD mode)
    from streamml.data import stream as S
    from streamml.models.autoencoder import Autoencoder
    full = np.random.default_rng(7).uniform(0, 40, (32 * 60 + 17, 18)).astype(np.float32)
    engines = {}
    for mode in ("p2p", "local_sgd:5"):
        m = Autoencoder(device=dev, input_normalizer="cardata", seed=3)
        m.compile()
        m.fit(full, epochs=2, batch_size=32, shuffle=False, verbose=0, dp=mode)
        engines[mode] = m.last_fit_engine
        np.save(f"{out}.fit_{mode.replace(':', '')}.rank{rank}.npy", m.backend.params.cpu().numpy())
    m = Autoencoder(device=dev, input_normalizer="cardata", seed=3)
    m.compile()
    st = S.synthetic(20_000 + 3_000 * rank, chunk=4_096, seed=rank).filter_normal(device=True)
    m.fit(st, epochs=1, batch_size=100, verbose=0, dp="p2p")
    np.save(f"{out}.fit_stream.rank{rank}.npy", m.backend.params.cpu().numpy())
    engines["stream"] = m.last_fit_engine
    engines["stream_iters"] = m.iterations
    if rank == 0:
        with open(out + ".json", "w") as f:
            json.dump({"allreduce_ok": ar_ok, "allreduce_us": ar_us, "steps": steps + steps2,
                       "iter": int(ae.iter.item()), "engines": engines}, f)
    dp.barrier(dev)
    dp.shutdown()


if __name__ == "__main__":
    main()
