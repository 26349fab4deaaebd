"""CPU-side checks of the C-ABI boundary: libnsgpu.so loads and exports every symbol
include/nsgpu.h declares (no compute calls — there is no GPU here)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in ("nsgpu.h",):
        txt = open(os.path.join(REPO, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        syms |= set(re.findall(r"\b(nsgpu_[a-z0-9_]+)\s*\(", txt))
    return syms


def test_library_exports_all_declared_symbols():
    import nsgpu
    if not os.path.exists(nsgpu.LIB_PATH):
        pytest.skip("libnsgpu.so not built (run __graft_entry__.build())")
    so = ctypes.CDLL(nsgpu.LIB_PATH)
    missing = [s for s in sorted(declared_symbols()) if not hasattr(so, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    import nsgpu
    assert declared_symbols() <= set(nsgpu.SIGNATURES), declared_symbols() - set(nsgpu.SIGNATURES)


def test_no_oracle_in_product():
    """The product library must not link the oracle; the product binding must not import it."""
    import nsgpu
    src = open(nsgpu.__file__).read()
    assert "nsref" not in src
    if os.path.exists(nsgpu.LIB_PATH):
        data = open(nsgpu.LIB_PATH, "rb").read()
        assert b"nsref_" not in data
