"""Data sources, schema facts and tf.data-style transforms for streamml."""
from .cardata import (FEATURES, LABEL, NUM_FEATURES, SyntheticCarSource, load_csv,  # noqa: F401
                      normalize_affine, normalize_np)
