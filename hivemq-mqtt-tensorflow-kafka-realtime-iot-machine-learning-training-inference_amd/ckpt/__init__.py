"""Checkpoints: Keras-compatible HDF5 (native codec) and model stores."""
from .h5 import (Dataset, Group, KerasCheckpoint, adam_weight_names, load_keras_h5, read,  # noqa: F401
                 save_keras_h5, write)
