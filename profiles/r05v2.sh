#!/usr/bin/env bash
# Round 5 pass v2: PMC counters of the orbit small-batch scan (C3 handle, 1 / 4 / 16-query batches), one counter set per pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05v2}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" "SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 $R/tools/percall_probe.py --scan-only > "$OUT/p$i.log" 2>&1 || echo "pass $i failed"
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 - "$f" "$OUT/pmc_$i.txt" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    n = r.get("Kernel_Name", "")
    if "nn_scan_orbit_kernel" not in n and "nn_scan_merge" not in n:
        continue
    key = n.split("(")[0]
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(key, r["Counter_Name"])] += 1
with open(sys.argv[2], "w") as o:
    for k, d in agg.items():
        o.write(k + "\n")
        for c, v in sorted(d.items()):
            o.write(f"  {c:32s} {v / max(1, cnt[(k, c)]):16.1f} per dispatch ({cnt[(k, c)]} dispatches)\n")
PY
  rm -rf "$OUT/p$i"
done
cat "$OUT"/pmc_*.txt
