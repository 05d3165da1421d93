"""Writes tests/golden/gtm_demo.json: structural facts of the reference's own demo streams
(/root/reference/docs/demo/{football,city}_cif.gtm, written by the reference encoder through lzma.exe -lc8)
as decoded by oracle/lzma_dec.c + tests/gtm_read.py.  The demo files stay in the reference tree; only
these numbers and digests are committed.  Run from the repo root: python tests/golden/make_gtm_golden.py"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import pyoracle  # noqa: E402
from gtm_read import read_gtm, render  # noqa: E402

DEMO = "/root/reference/docs/demo"


def facts(path):
    data = open(path, "rb").read()
    g = read_gtm(pyoracle, data)
    items = np.concatenate([f[0] for f in g.frames])
    frames = render(g)
    return {
        "file_bytes": len(data), "file_sha256": hashlib.sha256(data).hexdigest(),
        "lzma_props": [data[0], int.from_bytes(data[1:5], "little")],
        "streams_raw_bytes": [len(s) for s in g.streams],
        "streams_compressed_bytes": g.stream_comp,
        "streams_sha256": [hashlib.sha256(s).hexdigest() for s in g.streams],
        "width": g.width, "height": g.height, "frame_ns": g.frame_ns, "tiles": int(g.tiles.shape[0]),
        "palsize": g.palsize, "frames": len(g.frames), "keyframe_ends": int(sum(f[2] for f in g.frames)),
        "skipped_items": int((items[:, 0] < 0).sum()),
        "rendered_sha256": hashlib.sha256(frames.tobytes()).hexdigest(),
    }


if __name__ == "__main__":
    out = {n: facts(os.path.join(DEMO, n)) for n in ("football_cif.gtm", "city_cif.gtm")}
    with open(os.path.join(HERE, "gtm_demo.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
