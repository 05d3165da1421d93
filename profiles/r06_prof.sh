#!/usr/bin/env bash
# r06 final build: rocprofv3 kernel trace + stats and the separate PMC passes of bench.py's C3 step (run_profile.sh),
# summarised (profiles/summarize.py, refreshes pmc_traffic.json as gpurun_out/<tag>/pmc_traffic.json)
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06prof}
OUT=$R/gpurun_out/$TAG
cd "$R"
STEPS=3 bash profiles/run_profile.sh "$TAG"
python3 profiles/summarize.py "$OUT" "$OUT/pmc_traffic.json" > "$OUT/summary.json"
echo "summary done"
