"""Regenerate the committed fixtures in tests/golden/ (run here, where /root/reference is mounted).

kmodes_asm_kat.npz  -- K-Modes dissimilarity / argmin / min-distance vectors computed by the
                       REFERENCE's own x86-64 asm (kmodes.pas:316-596, assembled by
                       oracle/build_ref_asm.sh into oracle/_ref/).  Pins the oracle on the GPU box,
                       where the reference is absent.
psyv_kat.npz        -- descriptor known-answer vectors from the oracle (regression pin; the formulas
                       themselves are checked analytically in tests/test_oracle_kats.py).
Data only: inputs and expected outputs.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import pyoracle  # noqa: E402


def kmodes_asm_kat():
    ref = pyoracle.ref_kmodes_lib()
    if ref is None:
        raise SystemExit("oracle/_ref/libkmodes_ref.so missing: run `make -C oracle` with /root/reference mounted")
    rng = np.random.default_rng(4242)
    rows_all, items, counts, best_idx, best_dis, md_in, md_out = [], [], [], [], [], [], []
    for trial in range(96):
        n = int(rng.integers(1, 40))
        mode = trial % 6
        if mode == 0:
            rows = rng.integers(0, 16, (n, 80), dtype=np.uint8)
            rows[:, 64:] = rng.integers(0, 2, (n, 16))
        elif mode == 1:
            rows = rng.integers(0, 256, (n, 80), dtype=np.uint8)
        elif mode == 2:
            rows = rng.choice(np.array([0, 1, 127, 128, 129, 255], np.uint8), (n, 80))
        elif mode == 3:
            rows = np.repeat(rng.integers(0, 16, (1, 80), dtype=np.uint8), n, 0)
        elif mode == 4:
            rows = np.full((n, 80), 255, np.uint8)
            rows[:, 1] = rng.integers(0, 256, n)
            rows[:, 9] = rng.integers(0, 256, n)
        else:
            rows = rng.integers(0, 256, (n, 80), dtype=np.uint8)
        item = rows[rng.integers(0, n)].copy() if trial % 3 == 0 else rng.integers(0, 256, 80, dtype=np.uint8)
        ptrs = (ctypes.c_void_p * n)(*[rows[i].ctypes.data for i in range(n)])
        best = ctypes.c_uint64()
        bi = ref.ref_get_min(item.ctypes.data_as(ctypes.c_void_p), ptrs, ctypes.c_uint64(n), ctypes.byref(best))
        md = np.full(n, np.iinfo(np.uint64).max, np.uint64)
        md[::2] = rng.integers(0, 70000, md[::2].size)
        md0 = md.copy()
        used = rng.integers(0, 2, n).astype(np.uint8)
        ref.ref_update_min_distance(item.ctypes.data_as(ctypes.c_void_p), ptrs, used.ctypes.data_as(ctypes.c_void_p),
                                    md.ctypes.data_as(ctypes.c_void_p), n)
        pad = np.zeros((40, 80), np.uint8)
        pad[:n] = rows
        rows_all.append(pad)
        items.append(item)
        counts.append(n)
        best_idx.append(bi)
        best_dis.append(best.value)
        m_in = np.zeros(40, np.uint64)
        m_out = np.zeros(40, np.uint64)
        m_in[:n] = md0
        m_out[:n] = md
        md_in.append(m_in)
        md_out.append(m_out)
    np.savez_compressed(os.path.join(HERE, "kmodes_asm_kat.npz"), rows=np.stack(rows_all), items=np.stack(items),
                        counts=np.array(counts, np.int32), best_idx=np.array(best_idx, np.int64),
                        best_dis=np.array(best_dis, np.uint64), md_in=np.stack(md_in), md_out=np.stack(md_out))


def psyv_kat():
    rng = np.random.default_rng(777)
    from tiler_amd import synth
    rgb = synth.frame_tiles(rng, 24)
    pp = rng.integers(0, 16, (8, 64)).astype(np.uint8)
    pal = synth.palettes(rng, 1)[0]
    flags_rgb = np.array([2, 0, 8, 2 | 16 | 32], np.int32)
    flags_pal = np.array([1 | 2, 1 | 8 | 16, 1 | 32], np.int32)
    out_rgb = np.stack([[pyoracle.psyv(rgb=t, flags=int(f)) for t in rgb] for f in flags_rgb])
    out_pal = np.stack([[pyoracle.psyv(palpix=t, pal=pal, flags=int(f)) for t in pp] for f in flags_pal])
    np.savez_compressed(os.path.join(HERE, "psyv_kat.npz"), rgb=rgb, palpix=pp, pal=pal, flags_rgb=flags_rgb,
                        flags_pal=flags_pal, out_rgb=out_rgb, out_pal=out_pal)


if __name__ == "__main__":
    kmodes_asm_kat()
    psyv_kat()
    print("fixtures written to", HERE)
