#!/usr/bin/env bash
# Round-3 pass v: what the A-fragment LDS reads cost the shortlist -- timing modes of the experiment build (results
# invalid, lists empty): 1 bound VALU without list updates, 15 = 1 without the per-k-step A-fragment LDS reads,
# 12 MFMA chains only, 14 = 12 without the A-fragment LDS reads; 0 the shipped kernel.  Same box, one call.
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
MODES="0 1 15 12 14 0" STEPS=6 bash profiles/pmode_ab.sh
