"""libgzero.so loads without a GPU and exports every entry point declared in
include/gzero.h (no compute call is made here)."""
import ctypes
import re

from conftest import REPO
from gzero import _lib


def test_header_symbols_exported():
    hdr = open(f"{REPO}/include/gzero.h").read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(gz_[a-z_0-9]+)\(", hdr, re.M))
    assert "gz_search" in declared and "gz_pv_forward" in declared
    L = _lib.load()
    for name in declared:
        assert hasattr(L, name), name
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_struct_sizes_match_header():
    assert ctypes.sizeof(_lib.BoardState) == 80
    assert ctypes.sizeof(_lib.Record) == 80
    L = _lib.load()
    assert L.gz_version() == 1
    from gzero import weights
    assert L.gz_pv_weight_floats() == weights.TOTAL
    assert L.gz_tree_bytes(200) >= 201 * 26


def test_argument_errors_without_gpu():
    L = _lib.load()
    p = _lib.SearchParams(200, 100, 1.6, 0.05, 0.0, 0, 5, 0)
    rc = L.gz_search(None, None, 1, ctypes.byref(p), None, None, None, None, 0, None, None)
    assert rc == -3 and b"planner" in L.gz_last_error()
    p.planner_steps = 0
    p.num_simulations = 100000
    assert L.gz_search(None, None, 1, ctypes.byref(p), None, None, None, None, 0, None, None) == -1
