#!/usr/bin/env bash
# TEST INFRASTRUCTURE: build the reference's OWN K-Modes inner loops (kmodes.pas:316-596,
# x86-64 SSE2/SSSE3/POPCNT, MS x64 calling convention) into oracle/_ref/libkmodes_ref.so.
#
# The asm bodies are extracted at build time from /root/reference/kmodes.pas where they lie and
# rewritten mechanically into GNU-as Intel syntax (FPC operand names -> registers, $hex -> 0x,
# 'oword' -> 'xmmword', labels made unique, FPC's stack frame for UpdateMinDistance_Asm's 5th
# argument recreated).  Nothing of the reference is copied into the repository: the generated
# .S and the .so live only in oracle/_ref/ (git-ignored).  No reference build system is run.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
SRC="${TILER_REFERENCE:-/root/reference}/kmodes.pas"
OUT="$HERE/_ref"
if [ ! -f "$SRC" ]; then
  echo "build_ref_asm: $SRC not present (GPU box): skipping reference asm build" >&2
  exit 0
fi
mkdir -p "$OUT"

body() { # $1 = first line of the Pascal declaration; prints the lines between 'asm' and 'end;'
  awk -v start="$1" 'NR>start && /^asm[[:space:]]*$/ {on=1; next} on && /^end;/ {exit} on {print}' "$SRC"
}

L1=$(grep -n '^function GetMinMatchingDissim_Asm' "$SRC" | cut -d: -f1)
L2=$(grep -n '^procedure UpdateMinDistance_Asm' "$SRC" | cut -d: -f1)

xform() { # $1 = label prefix
  sed -E \
    -e 's/\boword ptr\b/xmmword ptr/g' \
    -e 's/\$([0-9a-fA-F]+)/0x\1/g' \
    -e 's/\bitem_rcx\b/rcx/g; s/\blist_rdx\b/rdx/g; s/\bcount_r8\b/r8/g; s/\bpbest_r9\b/r9/g' \
    -e 's/\bused_r8\b/r8/g; s/\bmindist_r9\b/r9/g' \
    -e 's/\bcDissimSubMatchingSize\b/11/g' \
    -e 's/\bmov eax, count\b/mov eax, dword ptr [rbp + 48]/' \
    -e "s/^([[:space:]]*)(loop|worst|used|start):/\1.L$1_\2:/" \
    -e "s/\b(jne|ja|jmp|jb|je)[[:space:]]+(loop|worst|used|start)\b/\1 .L$1_\2/" \
    -e 's/\/\/.*$//'
}

{
  echo '.intel_syntax noprefix'
  echo '.text'
  echo '.globl ref_GetMinMatchingDissim_Asm'
  echo '.type ref_GetMinMatchingDissim_Asm,@function'
  echo 'ref_GetMinMatchingDissim_Asm:'
  body "$L1" | xform gmm
  echo '  ret'
  echo '.globl ref_UpdateMinDistance_Asm'
  echo '.type ref_UpdateMinDistance_Asm,@function'
  echo 'ref_UpdateMinDistance_Asm:'
  echo '  push rbp'          # FPC 'assembler' (no nostackframe) frame: count = [rbp + 48]
  echo '  mov rbp, rsp'
  body "$L2" | xform umd
  echo '  pop rbp'
  echo '  ret'
  echo '.section .note.GNU-stack,"",@progbits'
} > "$OUT/kmodes_ref.S"

gcc -c -o "$OUT/kmodes_ref.o" "$OUT/kmodes_ref.S"
gcc -O2 -fPIC -shared -o "$OUT/libkmodes_ref.so" "$HERE/ref_kmodes_wrap.c" "$OUT/kmodes_ref.o"
echo "built $OUT/libkmodes_ref.so"
