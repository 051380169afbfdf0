"""Import shim: ``import streamml`` loads the framework package.

The framework's source tree lives in
``hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd/``
(a directory name that is not a valid Python identifier).  This shim points the
``streamml`` package's search path at that directory and executes its
``__init__`` so every submodule (``streamml.ops``, ``streamml.models`` ...)
resolves there.
"""
import os as _os

_PKG_DIR = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd",
)
__path__ = [_PKG_DIR]
__file__ = _os.path.join(_PKG_DIR, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
