"""torchrun worker for tests/test_dp.py: trains each model family data-parallel over gloo
and dumps the final weights per rank (compared by the parent test)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from streamml.parallel.dp import init_from_env, shutdown  # noqa: E402


def main(out_dir: str) -> None:
    env = init_from_env("cpu")
    rank = env.rank
    rng = np.random.default_rng(0)
    # --- autoencoder: 2 epochs, local batch 16 -> global batch 32
    from streamml.models.autoencoder import Autoencoder
    x = rng.uniform(-1, 1, size=(256, 18)).astype(np.float32)
    ae = Autoencoder(device="cpu", seed=3)
    h = ae.fit(x, epochs=2, batch_size=16, shuffle=False, verbose=0)
    np.savez(os.path.join(out_dir, f"ae_{rank}.npz"), *ae.get_weights(), loss=np.array(h.history["loss"]))
    # --- LSTM (reference stack, look_back 4): local batch 8
    from streamml.models.lstm import LSTMPredictor
    xs = rng.uniform(-1, 1, size=(64, 4, 18)).astype(np.float32)
    ys = rng.uniform(-1, 1, size=(64, 18)).astype(np.float32)
    m = LSTMPredictor.reference(look_back=4, device="cpu", seed=1)
    m.fit(xs, ys, epochs=1, batch_size=8, verbose=0)   # fit shards by rank itself
    np.savez(os.path.join(out_dir, f"lstm_{rank}.npz"), *m.fp.get())
    # --- LSTM with uneven shards (61 windows: 31 / 30) and a short last batch (7 + 6 rows)
    xu = rng.uniform(-1, 1, size=(61, 4, 18)).astype(np.float32)
    yu = rng.uniform(-1, 1, size=(61, 18)).astype(np.float32)
    mu = LSTMPredictor.reference(look_back=4, device="cpu", seed=2)
    mu.fit(xu, yu, epochs=1, batch_size=8, verbose=0, shuffle=False)
    np.savez(os.path.join(out_dir, f"lstm_uneven_{rank}.npz"), *mu.fp.get())
    # --- MNIST MLP: local batch 16
    from streamml.data.mnist import synthetic_mnist
    from streamml.models.mlp import MLPClassifier
    xi, yi = synthetic_mnist(128, seed=2)
    mlp = MLPClassifier(hidden=32, device="cpu", seed=5)
    mlp.fit(xi, yi, epochs=1, batch_size=16, shuffle=False, verbose=0)
    np.savez(os.path.join(out_dir, f"mlp_{rank}.npz"), *mlp.fp.get())
    # --- a one-rank measurement inside the group (bench.py's fit side fields): rank 0 fits
    # alone with dp="none" while rank 1 has already left -- no collective may be called
    if rank == 0:
        solo = Autoencoder(device="cpu", seed=4)
        hs = solo.fit(x, epochs=1, batch_size=32, shuffle=False, verbose=0, dp="none")
        np.savez(os.path.join(out_dir, "ae_solo.npz"), *solo.get_weights(), loss=np.array(hs.history["loss"]))
    shutdown()


if __name__ == "__main__":
    torch.set_num_threads(2)
    main(sys.argv[1])
