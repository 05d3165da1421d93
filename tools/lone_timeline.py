#!/usr/bin/env python3
"""Study script: the timeline of lone per-tile calls from a rocprofv3 runtime + kernel + copy trace
(profiles/r05y2.sh).  Finds the lone-call phase of tiler_debug_percall_bench (one thread, one search at a time) by
the first nn_scan kernels, and prints, for a median call, every HIP API call / copy / kernel with its start offset
and duration relative to the call's first HIP API call."""
import csv
import os
import statistics
import sys


def rows(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main():
    d = sys.argv[1]
    api = rows(os.path.join(d, "hip_api_trace.csv"))
    ker = rows(os.path.join(d, "kernel_trace.csv"))
    cpy = rows(os.path.join(d, "memory_copy_trace.csv"))
    ev = []
    for r in api:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r.get("Function", r.get("Operation", "?")),
                   r.get("Thread_Id", "")))
    for r in ker:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kern", r["Kernel_Name"].split("(")[0][-48:], ""))
    for r in cpy:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", r.get("Direction", "copy"), ""))
    ev.sort()
    # lone calls: each begins with the H2D copy of a 1-query batch; take the scan kernels and group by the API thread
    scans = [e for e in ev if e[2] == "kern" and ("nn_scan_orbit" in e[3] or "nn_scan_small" in e[3] or "nn_scan_rows" in e[3])]
    if not scans:
        print("no scan kernels")
        return
    # the lone phase: the first 64 scans of the C3 handle (percall bench runs lone calls first)
    lone = scans[:64]
    gaps = []
    windows = []
    for k in lone:
        # the call's window: from the last hipMemcpyAsync (H2D) before the scan to the next hipStreamSynchronize end
        before = [e for e in ev if e[2] == "api" and "Memcpy" in e[3] and e[0] <= k[0]]
        after = [e for e in ev if e[2] == "api" and "Synchronize" in e[3] and e[1] >= k[1]]
        if not before or not after:
            continue
        t0, t1 = before[-1][0], after[0][1]
        windows.append((t1 - t0, t0, t1))
    windows.sort()
    if not windows:
        print("no windows")
        return
    med = windows[len(windows) // 2]
    print(f"lone calls: {len(windows)}, window median {med[0] / 1e3:.1f} us (min {windows[0][0] / 1e3:.1f})")
    t0, t1 = med[1], med[2]
    for e in ev:
        if e[1] >= t0 and e[0] <= t1:
            print(f"  {(e[0] - t0) / 1e3:8.1f} us  +{(e[1] - e[0]) / 1e3:7.1f} us  {e[2]:5s} {e[3]} {e[4]}")


if __name__ == "__main__":
    main()
