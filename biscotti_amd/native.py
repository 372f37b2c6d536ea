"""Loaders for the native parts of biscotti_amd.

``rt()``  -> the pybind11 host runtime ``_biscotti_rt`` (crypto, ledger, protocol FSM).
``hip()`` -> the gfx950 kernel library ``libbiscotti_hip.so`` (ctypes handle).

Both are built in-tree by :mod:`biscotti_amd._build`.  On a machine with a GPU the HIP library is
mandatory: :func:`hip` raises instead of letting callers fall back to a slow eager path.
"""
from __future__ import annotations

import ctypes
import importlib
import os
import threading
from pathlib import Path

_PKG = Path(__file__).resolve().parent
_lock = threading.Lock()
_rt = None
_hip = None


def rt():
    """Return the host runtime module, building it on first use if it is missing."""
    global _rt
    if _rt is None:
        with _lock:
            if _rt is None:
                try:
                    _rt = importlib.import_module("biscotti_amd._biscotti_rt")
                except ImportError:
                    from . import _build

                    _build.build_runtime()
                    _rt = importlib.import_module("biscotti_amd._biscotti_rt")
    return _rt


def hip_library_path() -> Path:
    return _PKG / "libbiscotti_hip.so"


def hip():
    """Return the ctypes handle of the HIP kernel library (fails loudly if absent)."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                path = hip_library_path()
                if not path.exists():
                    if os.environ.get("BISCOTTI_AUTOBUILD", "1") == "1":
                        from . import _build

                        _build.build_kernels()
                    if not path.exists():
                        raise RuntimeError(
                            f"{path} is missing: run `python -m biscotti_amd._build --kernels` (gfx950)")
                lib = ctypes.CDLL(str(path))
                from .ops import _abi

                _abi.declare(lib)
                _hip = lib
    return _hip


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False
