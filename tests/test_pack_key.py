"""The throughput engine's pack-reuse key: an in-place update of the same
device array changes the key, so ``fit`` re-packs instead of training on stale rows."""
import torch

from streamml.models.autoencoder import Autoencoder


def test_pack_key_changes_on_in_place_update():
    x = torch.zeros(64, 18)
    k0 = Autoencoder.pack_key(x, 16, 4)
    assert Autoencoder.pack_key(x, 16, 4) == k0            # unchanged rows: reuse
    x.add_(1.0)
    assert Autoencoder.pack_key(x, 16, 4) != k0            # in-place update: re-pack
    k1 = Autoencoder.pack_key(x, 16, 4)
    x[3:5].mul_(2.0)                                       # a write through a view bumps it too
    assert Autoencoder.pack_key(x, 16, 4) != k1
    assert Autoencoder.pack_key(x, 32, 2) != Autoencoder.pack_key(x, 16, 4)
