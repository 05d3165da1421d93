"""Summarise a profiles/run_profile.sh output directory into one JSON per round (committed under profiles/).

    python profiles/summarize.py gpurun_out/r01 > profiles/r01_summary.json

Per kernel: rocprofv3 --kernel-trace --stats durations, then the PMC passes averaged per dispatch:
  * HBM traffic = FETCH_SIZE + WRITE_SIZE (KiB units as rocprofv3 reports them on gfx950; FETCH_SIZE
    undercounts 64-B requests by 2x on gfx950 per MI355X_MICROARCH.md, so the corrected read figure
    is reported next to the raw one);
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall; MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES /
    (clock cycles x 1024 SIMDs);
  * wave-cycle split SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY (quad-cycles).
"""
from __future__ import annotations

import collections
import csv
import json
import os
import sys


def _short(name: str) -> str:
    for key in ("orbit_ft_query2_kernel", "orbit_ft_query_kernel", "smooth_chain_coop_kernel", "smooth_hash_insert",
                "smooth_hash_number", "smooth_hash_lookup", "nn_orbit_pairs_kernel", "kd_verify_kernel", "kd_replay_kernel", "kd_rootbox_kernel",
                "nn_orbit_shortlist_pipe_kernel", "nn_orbit_shortlist_kernel", "nn_orbit_rescore_kernel", "orbit_prep_kernel", "orbit_eq_kernel", "nn_shortlist16_kernel", "nn_shortlist2_kernel", "nn_shortlist4_kernel", "nn_shortlist_kernel", "nn_collect_kernel",
                "nn_rescore2_kernel", "nn_rescore_kernel", "nn_exact_kernel", "prep_rows_kernel", "psyv_kernel",
                "maxabs_kernel", "smooth_kernel"):
        if key in name:
            return key
    return name[:48]


def _pmc(path: str):
    rows = list(csv.DictReader(open(path)))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in rows:
        k = _short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return ({k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()},
            {k: sum(v) / len(v) for k, v in dur.items()})


def summarize(d: str) -> dict:
    out: dict = {"source": os.path.basename(os.path.normpath(d)), "kernels": {}}
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            k = _short(r["Name"])
            out["kernels"].setdefault(k, {})["trace"] = {
                "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6, "pct": float(r["Percentage"])}
    merged = collections.defaultdict(dict)
    walls = collections.defaultdict(list)
    for p in ("pmc_sq", "pmc_fetch", "pmc_write", "pmc_inst"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        vals, dur = _pmc(f)
        for k, v in vals.items():
            merged[k].update(v)
            walls[k].append(dur[k])
    for k, c in merged.items():
        e = out["kernels"].setdefault(k, {})
        wall_ns = sum(walls[k]) / len(walls[k])
        pm = {"counters": {n: round(v, 1) for n, v in sorted(c.items())}, "profiled_wall_ms": wall_ns / 1e6}
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            fetch = c.get("FETCH_SIZE", 0.0) * 1024
            write = c.get("WRITE_SIZE", 0.0) * 1024
            pm["hbm_read_bytes_raw"] = fetch
            pm["hbm_read_bytes_corrected"] = 2 * fetch
            pm["hbm_write_bytes"] = write
            pm["hbm_traffic_bytes"] = 2 * fetch + write
        if "GRBM_GUI_ACTIVE" in c and wall_ns > 0:
            clk = c["GRBM_GUI_ACTIVE"] / 8 / (wall_ns * 1e-9)
            pm["effective_clock_ghz"] = clk / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                pm["mfma_util"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * wall_ns * 1e-9 * 1024)
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
            wc = c["SQ_WAVE_CYCLES"]
            pm["wave_split"] = {n: c.get(n, 0.0) / wc for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        e["pmc"] = pm
    return out


def traffic_table(summary: dict) -> dict:
    """Per-launch HBM bytes by kernel (read by bench.py for roofline.traffic)."""
    t = {"source": summary["source"], "kernels": {}}
    for k, v in summary["kernels"].items():
        pm = v.get("pmc", {})
        if "hbm_traffic_bytes" in pm:
            t["kernels"][k] = {"hbm_traffic_bytes": pm["hbm_traffic_bytes"], "hbm_read_bytes_raw": pm["hbm_read_bytes_raw"],
                               "hbm_write_bytes": pm["hbm_write_bytes"],
                               "avg_ms_trace": v.get("trace", {}).get("avg_ms")}
    return t


if __name__ == "__main__":
    summ = summarize(sys.argv[1])
    print(json.dumps(summ, indent=1))
    if len(sys.argv) > 2:  # also write the per-launch traffic table
        with open(sys.argv[2], "w") as f:
            json.dump(traffic_table(summ), f, indent=1)
