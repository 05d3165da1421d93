#!/usr/bin/env python3
"""Study script: from a rocprofv3 kernel trace (+ optional HIP API trace) of bench_encoder.py, how much of the
per-keyframe Prepare's kernel time runs beside FrameTiling's kernels, and which host calls of the Prepare thread
block longest.  Usage: overlap_trace.py <dir with *_kernel_trace.csv [and *_hip_api_trace.csv]>"""
import csv
import glob
import os
import sys
from collections import defaultdict

FT = ("nn_shortlist16", "nn_rescore", "nn_pairs", "nn_collect", "ft_", "orbit_ft", "smooth", "kd_verify",
      "kd_replay", "nn_exact", "psyv")


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not f:
        return []
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main():
    d = sys.argv[1]
    ks = load(d, "*kernel_trace.csv")
    rows = []
    for r in ks:
        nm = r["Kernel_Name"]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm, r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    # the timed clip: the last 60 % of the trace's shortlist launches
    sl = [r for r in rows if "nn_shortlist16" in r[2]]
    t_lo = sl[len(sl) * 2 // 5][0] if sl else rows[0][0]
    rows = [r for r in rows if r[0] >= t_lo]
    ft = [(s, e) for s, e, n, q in rows if n.startswith(FT) or any(x in n for x in ("shortlist16", "smooth"))]
    ft_iv = sorted(ft)
    merged = []
    for s, e in ft_iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    import bisect
    starts = [m[0] for m in merged]

    def overlap(s, e):
        i = max(0, bisect.bisect_right(starts, s) - 1)
        tot = 0
        while i < len(merged) and merged[i][0] < e:
            tot += max(0, min(e, merged[i][1]) - max(s, merged[i][0]))
            i += 1
        return tot

    by = defaultdict(lambda: [0, 0, 0])
    prep_tot = prep_ov = 0
    ftset = set(id(x) for x in ft)
    for s, e, n, q in rows:
        is_ft = n.startswith(FT) or "shortlist16" in n or "smooth" in n
        if is_ft:
            continue
        key = n.split("(")[0].split("<")[0][:48]
        ov = overlap(s, e)
        by[key][0] += 1
        by[key][1] += e - s
        by[key][2] += ov
        prep_tot += e - s
        prep_ov += ov
    span = rows[-1][1] - rows[0][0]
    ft_busy = sum(e - s for s, e in merged)
    print(f"window {span / 1e6:.1f} ms, FT-kernel busy {ft_busy / 1e6:.1f} ms, other kernels {prep_tot / 1e6:.1f} ms "
          f"of which beside FT {prep_ov / 1e6:.1f} ms")
    for k, v in sorted(by.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {k:50s} n={v[0]:6d} {v[1] / 1e6:8.2f} ms  beside FT {v[2] / 1e6:8.2f} ms")
    api = load(d, "*hip_api_trace.csv")
    if api:
        agg = defaultdict(lambda: [0, 0, 0])
        for r in api:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s < t_lo:
                continue
            a = agg[r["Function"]]
            a[0] += 1
            a[1] += e - s
            a[2] = max(a[2], e - s)
        print("HIP API (timed window): calls, total ms, max us")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
            print(f"  {k:32s} {v[0]:7d} {v[1] / 1e6:9.2f} {v[2] / 1e3:9.1f}")


if __name__ == "__main__":
    main()
