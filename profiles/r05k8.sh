#!/usr/bin/env bash
# Round 5 pass k8 (debug record): the k = 8 small-batch scan's per-split lists for a failing query of
# tools/k8_plain_check.py, from a study build that dumped them (TILER_DEBUG_DUMP_SCAN, not in the shipped source);
# output kept in profiles/r05k8/partials_dump.txt.  The fix: the wide cross-lane merge (nn_scan_merge_kernel<8, true>).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 400 python3 tools/k8_plain_check.py
