"""Loader for the native extensions (``_C`` HIP kernels, ``_io`` host codecs).

The extensions are built in-tree by :mod:`streamml._build`.  On a machine with a
ROCm GPU a missing ``_C`` is a hard error (we never silently fall back to
PyTorch eager ops on the GPU path); on CPU-only machines callers can ask
:func:`has_c` first and use the torch-CPU reference path.
"""
from __future__ import annotations

import collections
import importlib
import os
import threading

_lock = threading.Lock()
_C = None
_IO = None
_C_ERR = None
_IO_ERR = None


def _try_build(which: str) -> None:
    if os.environ.get("SML_NO_AUTOBUILD"):
        return
    from .. import _build
    if which == "c":
        _build.build_c(checked=kernel_checks())
    else:
        _build.build_io()


# Calls that left the in-tree HIP kernels for a vendor library (hipBLASLt GEMMs for shapes
# beyond the tall-skinny register tiles).  The reference models never should: the tests
# assert this stays empty, and SML_STRICT_KERNELS=1 turns any such call into an error.
FALLBACKS: "collections.Counter[str]" = collections.Counter()


def note_fallback(what: str) -> None:
    FALLBACKS[what] += 1
    if os.environ.get("SML_STRICT_KERNELS") == "1":
        raise RuntimeError(f"vendor-library fallback '{what}' with SML_STRICT_KERNELS=1")


def kernel_checks() -> bool:
    """``SML_KERNEL_CHECKS=1``: load ``_C_dbg`` (kernels with device-side SML_DCHECK
    asserts, ``python -m streamml._build --checked``) instead of ``_C``."""
    return os.environ.get("SML_KERNEL_CHECKS", "0") not in ("", "0")


def load_c():
    """Return the ``streamml._C`` module (or ``_C_dbg``), building it in-tree if absent."""
    global _C, _C_ERR
    with _lock:
        if _C is not None:
            return _C
        mod = "streamml._C_dbg" if kernel_checks() else "streamml._C"
        try:
            _C = importlib.import_module(mod)
        except ImportError as e:  # pragma: no cover - exercised only without a build
            _C_ERR = e
            try:
                _try_build("c")
                _C = importlib.import_module(mod)
            except Exception as e2:
                raise RuntimeError(
                    "streamml._C (gfx950 HIP kernels) is not built and could not be built: "
                    f"{e2!r}. Run `python -m streamml._build`.") from e2
        return _C


def load_io():
    """Return the ``streamml._io`` module (host C++ codecs)."""
    global _IO, _IO_ERR
    with _lock:
        if _IO is not None:
            return _IO
        try:
            _IO = importlib.import_module("streamml._io")
        except ImportError as e:
            _IO_ERR = e
            try:
                _try_build("io")
                _IO = importlib.import_module("streamml._io")
            except Exception as e2:
                raise RuntimeError(f"streamml._io (host codecs) unavailable: {e2!r}") from e2
        return _IO


def has_c() -> bool:
    try:
        load_c()
        return True
    except Exception:
        return False


def gpu_available() -> bool:
    import torch
    return torch.cuda.is_available()
