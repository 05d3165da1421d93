#!/usr/bin/env python3
"""Debug script: k = 8 small batches on a plain index of 600,000 rows (several rows per scan thread) whose rows come
in groups of 4 identical copies at scattered positions, against the oracle (both tie orders via tests/nncheck)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # the checker (test infrastructure)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import tiler_amd
    import pyoracle
    from nncheck import check_nn
    pyoracle.lib()
    rng = np.random.default_rng(78)
    base = rng.standard_normal((150000, 192)).astype(np.float32)
    rows = np.concatenate([base, np.repeat(base[:150000], 3, axis=0)])[rng.permutation(600000)]
    picks = base[rng.choice(150000, 16, replace=False)]
    qs = np.concatenate([picks[:8], picks[8:] + rng.standard_normal((8, 192)).astype(np.float32) * 0.05])
    for nq in (1, 4, 16):
        check_nn(tiler_amd, pyoracle, rows, qs[:nq], k=8)
        print("nq", nq, "ok", flush=True)


if __name__ == "__main__":
    main()
