"""ctypes binding of libANN.so (include/tiler_ann.h).

The shared library is built in-tree (tiler_amd/lib/libANN.so, `python -c "import __graft_entry__ as g; g.build()"`).
There is no CPU fallback: if the library or a gfx950 device is missing, calls raise TilerError.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libANN.so")
_DEFAULT_LIB_PATH = LIB_PATH
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tiler_ann.h")

c_int = ctypes.c_int
c_long = ctypes.c_long
c_float = ctypes.c_float
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p
c_size_t = ctypes.c_size_t
c_uint32 = ctypes.c_uint32
P = ctypes.POINTER


class TilerError(RuntimeError):
    pass


class SearchStats(ctypes.Structure):
    _fields_ = [("queries", ctypes.c_int64), ("fallback_queries", ctypes.c_int64),
                ("exhaustive_queries", ctypes.c_int64), ("exact_integer", ctypes.c_int32), ("splits", ctypes.c_int32),
                ("orbit_groups", ctypes.c_int64), ("orbit_search", ctypes.c_int32), ("orbit_ksteps", ctypes.c_int32),
                ("orbit_expansions", ctypes.c_int64), ("orbit_rescored", ctypes.c_int64),
                ("tie_order", ctypes.c_int32), ("kd_levels", ctypes.c_int32), ("kd_build_ms", ctypes.c_double),
                ("kd_replayed", ctypes.c_int64), ("flat_queries", ctypes.c_int64)]


class PrepareInfo(ctypes.Structure):
    _fields_ = [("items", ctypes.c_int64), ("candidates", ctypes.c_int64)]


_SIGS = {
    "ann_kdtree_create": (c_void_p, [P(P(c_float)), c_int, c_int, c_int, c_int]),
    "ann_kdtree_create_dev": (c_void_p, [c_void_p, c_int, c_int, c_void_p]),
    "ann_kdtree_create_dev_ex": (c_void_p, [c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "tiler_kdtree_positions": (c_int, [c_void_p, c_void_p]),
    "ann_kdtree_destroy": (None, [c_void_p]),
    "ann_kdtree_search": (c_int, [c_void_p, c_void_p, c_float, c_void_p]),
    "ann_kdtree_pri_search": (c_int, [c_void_p, c_void_p, c_float, c_void_p]),
    "ann_kdtree_search_multi": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_float]),
    "ann_kdtree_search_batch": (c_int, [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p]),
    "ann_kdtree_search_multi_batch": (c_int, [c_void_p, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p]),
    "ann_kdtree_pri_search_batch": (c_int, [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p]),
    "ann_kdtree_search_batch_dev": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "ann_kdtree_get_stats": (c_int, [c_void_p, P(SearchStats)]),
    "tiler_set_scan_limits": (c_int, [c_int, c_int]),
    "tiler_debug_percall_bench": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, P(c_double),
                                          P(c_double)]),
    "tiler_debug_force_replay": (c_int, [c_int]),
    "tiler_debug_shortlist_gate": (c_int, [c_int]),
    "tiler_combine_stats": (c_int, [c_void_p, P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_int32)]),
    "tiler_init": (c_int, [c_int]),
    "tiler_device_count": (c_int, []),
    "tiler_kdtree_device": (c_int, [c_void_p]),
    "tiler_kdtree_replicate": (c_int, [c_void_p, c_int]),
    "tiler_placement_plan": (c_int, [c_int, c_void_p, c_int, c_void_p]),
    "tiler_debug_force_replicas": (c_int, [c_int]),
    "tiler_shutdown": (c_int, []),
    "tiler_last_error": (c_char_p, []),
    "tiler_set_gamma": (c_int, [c_double, c_double]),
    "tiler_timing_enable": (c_int, [c_int]),
    "tiler_timing_get": (c_double, [c_char_p, P(c_int)]),
    "tiler_timing_reset": (c_int, []),
    "tiler_psyv_batch": (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                 c_int, c_int, c_void_p, c_void_p]),
    "tiler_psyv_batch_dev": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p]),
    "tiler_ft_set_maps": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "tiler_ft_get_maps": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "tiler_prepare_frame_tiling_dev": (c_void_p, [c_void_p, c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p,
                                                  c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int,
                                                  c_void_p, P(PrepareInfo)]),
    "tiler_frame_tiling": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "tiler_frame_tiling_dev": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    "tiler_smooth_keyframe": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                      c_void_p, c_int, c_void_p, c_double]),
    "tiler_smooth_keyframe_dev": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_double, c_void_p]),
    "tiler_kmodes_medoids": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "tiler_kmodes_batch": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "tiler_kmodes_batch_dev": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    "tiler_kmodes_medoids_batch": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
    "tiler_debug_kmodes_ff_fallback": (c_int, [c_int]),
    "tiler_debug_dl3": (c_int, [c_int]),
    "tiler_kmodes_last_stats": (c_int, [P(ctypes.c_int64), P(ctypes.c_int64)]),
    "tiler_kmodes_compute": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "tiler_dither_tiles": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "tiler_dither_tiles_yliluoma": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                            c_void_p]),
    "tiler_dither_tiles_yliluoma_dev": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                                c_void_p, c_void_p, c_void_p]),
    "tiler_dither_tiles_dev": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                       c_void_p]),
    "tiler_quantize_palettes": (c_int, [c_long, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                        c_void_p]),
    "tiler_quantize_palettes_dev": (c_int, [c_long, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                            c_void_p, c_void_p, c_void_p]),
    "tiler_prepare_dither_tiles": (c_int, [c_long, c_void_p, c_int, c_int, c_int, c_int, c_uint32, c_void_p, c_void_p,
                                           c_void_p]),
    "tiler_prepare_dither_tiles_dev": (c_int, [c_long, c_void_p, c_int, c_int, c_int, c_int, c_uint32, c_void_p,
                                               c_void_p, c_void_p, c_void_p]),
    "tiler_kmeans": (c_int, [c_void_p, c_long, c_int, c_int, c_int, c_uint32, c_void_p, c_void_p, c_void_p]),
    "tiler_finish_quantize_order": (c_int, [c_int, c_void_p, c_void_p]),
    "tiler_interframe_correlation": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "tiler_interframe_correlation_dev": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "tiler_find_keyframes": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "tiler_lzma_encode": (c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_uint32, c_int, c_void_p, c_size_t,
                                  c_void_p]),
}

_lib = None


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function name declared in include/tiler_ann.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b((?:ann|tiler)_[a-z_0-9]+)\s*\(", txt)))


def load() -> ctypes.CDLL:
    """Load the in-tree libANN.so; raise TilerError when it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TilerError(f"{LIB_PATH} missing: build it with __graft_entry__.build() (no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if LIB_PATH == _DEFAULT_LIB_PATH:
                raise  # the shipped library exports every entry point (tests/test_abi.py)
            continue  # an older build selected for an A/B study (tools/*_probe.py --lib)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().tiler_last_error()
    return msg.decode() if msg else ""


def check(rc, what: str):
    if rc is None or (isinstance(rc, int) and rc < 0):
        raise TilerError(f"{what} failed: {last_error()}")
    return rc
