"""Per-iteration host bubbles and per-step launch timeline of one K-Modes call from a rocprofv3 kernel trace (study tool).

Usage: km_gaps.py <kernel_trace.csv> [call index, default 1 = bench_globaltiling's timed call]
A call starts with kmb_prep_points; an iteration with kmb_iter_reset.  Prints, per iteration, the GPU idle time
between the previous kernel's end and the reset's start (the host's convergence check + work-list upload), and the
median duration / gap of the assignment, decision and attribute launches in the iteration.
"""
import csv
import json
import statistics
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    call = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    starts = [i for i, r in enumerate(rows) if "kmb_prep_points" in r[2]]
    lo = starts[call]
    hi = starts[call + 1] if call + 1 < len(starts) else len(rows)
    ks = rows[lo:hi]
    out = {"kernels": len(ks), "span_ms": (ks[-1][1] - ks[0][0]) / 1e6, "iterations": []}
    its = [i for i, r in enumerate(ks) if "kmb_iter_reset" in r[2]]
    busy = sum(e - s for s, e, _ in ks)
    out["busy_ms"] = busy / 1e6
    out["idle_ms"] = out["span_ms"] - out["busy_ms"]
    tot_bubble = 0
    for j, i in enumerate(its):
        end = its[j + 1] if j + 1 < len(its) else len(ks)
        bubble = ks[i][0] - ks[i - 1][1]
        tot_bubble += bubble
        seg = ks[i + 1:end]
        d = {"bubble_us": bubble / 1e3, "launches": len(seg), "span_ms": (seg[-1][1] - ks[i][0]) / 1e6 if seg else 0}
        for name, key in (("kmb_assign", "assign"), ("kmb_seq_strided", "decide"), ("kmb_seq_apply", "apply")):
            dur = [e - s for s, e, n in seg if name in n]
            gaps = [seg[k][0] - seg[k - 1][1] for k in range(1, len(seg)) if name in seg[k][2]]
            if dur:
                d[key] = {"n": len(dur), "med_us": statistics.median(dur) / 1e3, "sum_ms": sum(dur) / 1e6,
                          "gap_med_us": statistics.median(gaps) / 1e3 if gaps else None, "gap_sum_ms": sum(gaps) / 1e6}
        out["iterations"].append(d)
    out["bubbles_ms"] = tot_bubble / 1e6
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
