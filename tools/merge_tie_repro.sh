#!/usr/bin/env bash
# Builds (here, no GPU needed) or runs (GPU box) tools/merge_tie_repro.hip in its four variants.
#   bash tools/merge_tie_repro.sh build     -> tools/_build/merge_tie_repro{,_inline_walk,_no_call,_fixed} (+ .s ISA)
#   bash tools/merge_tie_repro.sh run       -> one line per variant and seed
#   bash tools/merge_tie_repro.sh detail    -> the base variant's first differing lanes
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/tools/_build
VARS="base: INLINE_WALK:_inline_walk NO_CALL:_no_call FIXED:_fixed"
if [ "${1:-run}" = build ]; then
  mkdir -p "$B"
  for v in $VARS; do
    def=${v%%:*}; suf=${v#*:}; D=""; [ "$def" != base ] && D="-D$def"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I "$R/tiler_amd/csrc" $D \
      "$R/tools/merge_tie_repro.hip" -o "$B/merge_tie_repro$suf" 2>/dev/null
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I "$R/tiler_amd/csrc" $D \
      --cuda-device-only -S "$R/tools/merge_tie_repro.hip" -o "$B/merge_tie_repro$suf.s" 2>/dev/null
  done
  exit 0
fi
if [ "${1:-run}" = detail ]; then  # the base variant's first differing lanes, host list against GPU list
  timeout -k 5 60 "$B/merge_tie_repro" 1024 6 1 || true
  exit 0
fi
for v in $VARS; do
  suf=${v#*:}
  for s in 1 2 3; do
    printf '%-28s ' "merge_tie_repro$suf"
    timeout -k 5 60 "$B/merge_tie_repro$suf" 1024 6 $s | tail -1 || true
  done
done
