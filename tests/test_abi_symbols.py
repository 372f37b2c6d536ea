"""The ctypes ABI table matches the built HIP library and the Python call sites.

A renamed or removed ``extern "C"`` entry point would otherwise be skipped silently by
``_abi.declare`` and only fail as an AttributeError on the GPU box.  Loading the library needs
no GPU (the HIP runtime initialises lazily), so this runs in the CPU suite.
"""
import ctypes
import pathlib
import re

import pytest

from biscotti_amd import native
from biscotti_amd.ops import _abi

_ROOT = pathlib.Path(__file__).resolve().parent.parent


def _python_call_sites():
    names = set()
    files = list((_ROOT / "biscotti_amd").rglob("*.py")) + [_ROOT / "bench.py"]
    for p in files:
        names |= set(re.findall(r"\b(bsc_[a-z0-9_]+)\b", p.read_text()))
    return names


def test_every_python_call_site_is_declared():
    undeclared = sorted(_python_call_sites() - set(_abi.SIGNATURES))
    assert not undeclared, f"bsc_* symbols used from Python without a ctypes signature: {undeclared}"


def test_every_declared_symbol_is_exported():
    path = native.hip_library_path()
    if not path.exists():
        pytest.skip("libbiscotti_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(str(path))
    missing = sorted(n for n in _abi.SIGNATURES if not hasattr(lib, n))
    assert not missing, f"declared in _abi.SIGNATURES but not exported by {path.name}: {missing}"


def test_no_static_device_variables_in_kernels():
    """A `static __device__`/`__constant__` variable that the host addresses is externalised with default
    visibility and read through the GOT (two dependent scalar loads per kernel entry, measured ~0.04 ms/round on
    the wave-priority flags); kernel files use externally linked, per-file names instead (wave_prio.h)."""
    bad = []
    for p in sorted((_ROOT / "biscotti_amd" / "csrc" / "kernels").glob("*")):
        if p.suffix in (".hip", ".h", ".hpp"):
            for i, line in enumerate(p.read_text().splitlines(), 1):
                if re.search(r"\bstatic\s+__(device|constant)__\s+(?!__forceinline__|inline)[\w:<>]+\s+\w+\s*[=;\[]",
                             line):
                    bad.append(f"{p.name}:{i}: {line.strip()}")
    assert not bad, bad
