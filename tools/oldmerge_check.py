"""Runs the tie tests against a library build given by --lib (study tool, not a test).

Used to show that tests/test_gpu_list_ties.py catches the round-4 one-wave merge: build the round-5 source with the
wide-merge gate forced off (`if (nsplit <= 1024)` -> `if (false)` in scan_small's merge lambda) into
tools/_build/libANN_r05oldmerge.so and run

    python3 tools/oldmerge_check.py --lib tools/_build/libANN_r05oldmerge.so

One line per test: passed, or the assertion it failed with.
"""
import argparse
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    import tiler_amd._lib as L
    L.LIB_PATH = os.path.abspath(args.lib)
    import pyoracle
    import tiler_amd
    pyoracle.lib()
    assert tiler_amd.load().tiler_init(0) == 0, tiler_amd.last_error()
    import test_gpu_list_ties as T
    import test_gpu_scan_small as S
    cases = [("merge_ties_across_one_lanes_splits k=1", lambda: T.test_merge_ties_across_one_lanes_splits(tiler_amd, pyoracle, 1)),
             ("merge_ties_across_one_lanes_splits k=8", lambda: T.test_merge_ties_across_one_lanes_splits(tiler_amd, pyoracle, 8)),
             ("scan_thread_list_ties k=8", lambda: T.test_scan_thread_list_ties(tiler_amd, pyoracle, 8)),
             ("scan_small_k8_ties", lambda: S.test_scan_small_k8_ties(tiler_amd, pyoracle))]
    for name, fn in cases:
        try:
            fn()
            print(f"{name}: passed", flush=True)
        except AssertionError as e:
            print(f"{name}: FAILED: {e}", flush=True)
        except Exception:
            print(f"{name}: ERROR: {traceback.format_exc().splitlines()[-1]}", flush=True)


if __name__ == "__main__":
    main()
