#!/usr/bin/env bash
# Round-3 pass zf: do the shortlist's bound adds cost because they read fresh MFMA results?  Timing modes (experiment
# build, results invalid, lists empty): 12 MFMA chains + LDS reads; 11 = 12 + the same number of VALU adds on registers
# no MFMA writes; 1 = 12 + the real bound adds (reading the accumulators).  Same box, one call.
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
MODES="12 11 1 12 11 1" STEPS=6 bash profiles/pmode_ab.sh
