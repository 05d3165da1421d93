"""CPU tests of the drop-in boundary: libANN.so exists, exports exactly what include/tiler_ann.h declares
(including the five reference ANN.dll symbols of extern.pas:63-67), and fails loudly without a GPU."""
import ctypes
import os
import subprocess

import pytest

import tiler_amd
from tiler_amd import _lib

REFERENCE_ANN = ["ann_kdtree_create", "ann_kdtree_destroy", "ann_kdtree_search", "ann_kdtree_pri_search",
                 "ann_kdtree_search_multi"]


def test_header_declares_reference_surface():
    syms = _lib.header_symbols()
    for s in REFERENCE_ANN:
        assert s in syms
    assert set(syms) == set(_lib._SIGS), "ctypes signatures must cover exactly the header"


def test_library_exports_every_header_symbol():
    assert os.path.exists(_lib.LIB_PATH), "build libANN.so first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if line.strip()}
    missing = [s for s in _lib.header_symbols() if s not in exported]
    assert not missing, missing
    lib = tiler_amd.load()
    for s in _lib.header_symbols():
        assert getattr(lib, s) is not None


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob  # gfx950 only, no multi-target dispatch


def test_no_cpu_fallback_without_gpu():
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present: this checks the no-GPU behaviour")
    lib = tiler_amd.load()
    assert lib.tiler_init(0) == -1
    assert "HIP device" in tiler_amd.last_error() or "gfx950" in tiler_amd.last_error()
    # every compute entry point refuses instead of computing on the CPU
    rows = (ctypes.POINTER(ctypes.c_float) * 1)()
    assert lib.ann_kdtree_create(rows, 0, 4, 1, 0) is None
    assert lib.tiler_kmodes_compute(None, 0, 80, 1, 0, 16, None, None, None, None) == -1
