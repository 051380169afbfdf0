"""Keras-like building blocks: callbacks and Keras config (de)serialisation."""
from .callbacks import (Callback, EarlyStopping, History, JSONLogger, KafkaPredictionSink,  # noqa: F401
                        ModelCheckpoint, TensorBoard)
