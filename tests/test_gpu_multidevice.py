"""libANN.so driving every GPU of the node from ONE process (tiler_init(TILER_ALL_DEVICES)): the unmodified
FreePascal encoder's shape (main.pas:972, 3779, 3961, 4005-4011).  The worker runs in its own process (the library
binding is process-wide); on a one-GPU box it exercises the N = 1 placement, the per-tile calls over several
keyframe handles from 16 threads, and the replication path forced onto the handle's own device."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_placement_plan_least_loaded():
    """The create-time placement rule on the host (no device needed): least loaded by live bytes, ties lowest."""
    import ctypes
    import tiler_amd
    lib = tiler_amd.load()
    vp = ctypes.c_void_p

    def plan(ndev, sizes):
        b = np.asarray(sizes, np.int64)
        out = np.full(b.size, -1, np.int32)
        assert lib.tiler_placement_plan(ndev, b.ctypes.data_as(vp), b.size, out.ctypes.data_as(vp)) == 0
        return out.tolist()

    assert plan(1, [5, 6, 7]) == [0, 0, 0]
    assert plan(8, [10] * 10) == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]  # equal keyframes: round robin
    assert plan(2, [100, 10, 10, 10, 10]) == [0, 1, 1, 1, 1]     # by bytes, not by count
    assert plan(3, [30, 20, 10, 5]) == [0, 1, 2, 2]
    assert plan(4, []) == []
    assert lib.tiler_placement_plan(0, None, 0, None) == -1


@pytest.mark.gpu
def test_all_devices_one_process():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "multidev_worker.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["devices"] >= 1
    assert res["placement"] == res["plan"]
    assert res["per_tile_queries"] == 2400 and res["per_tile_mismatches"] == 0
    assert res["k8_mismatches"] == 0
    assert res["replica_search_mismatches"] == 0
    assert res["prepare_same"] and res["ft_dev_same"] and res["ft_host_same"]
    assert res["replica_ft_mismatches"] == 0
    assert res["stream_replica_mismatches"] == 0
