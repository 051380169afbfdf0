"""Keras-like building blocks: callbacks and Keras config (de)serialisation."""
from .callbacks import (Callback, EarlyStopping, History, JSONLogger, KafkaPredictionSink,  # noqa: F401
                        ModelCheckpoint, TensorBoard)
from .layers import (LSTM, Dense, Dropout, Flatten, Input, InputLayer, L1L2, Layer,  # noqa: F401,E402
                     RepeatVector, TimeDistributed, regularizers)
from .model import Adam, Model, Sequential, load_model, optimizers  # noqa: F401,E402
