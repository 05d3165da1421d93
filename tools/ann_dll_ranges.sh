#!/usr/bin/env bash
# Static reading of the reference's ANN.dll ("Static cross-check"): prints the disassembly of every
# routine ann_kdtree_create / ann_kdtree_search reach, by the VA ranges recorded in DESIGN.md.  Reads the PE as
# data with objdump; the DLL is never loaded or executed.  Usage: tools/ann_dll_ranges.sh [/root/reference/ANN.dll]
set -eu
DLL=${1:-/root/reference/ANN.dll}
dis() { echo "== $1 ($2..$3)"; objdump -d -M intel --no-show-raw-insn --start-address=$2 --stop-address=$3 "$DLL" | grep -E '^ +1800' | grep -v 'int3'; }
dis ann_kdtree_create 0x180003e10 0x180003e6d
dis "ANNkd_tree ctor" 0x180014bc0 0x180014dd0
echo "== split-rule jump table (RVA offsets of the cases 0..5)"; objdump -s --start-address=0x180014dd0 --stop-address=0x180014de8 "$DLL" | tail -2
dis annEnclRect 0x180014f80 0x180015110
dis rkd_tree 0x1800149c0 0x180014bb6
dis kd_split 0x180012f60 0x180012fc9
dis annMaxSpread 0x1800158e0 0x180015cf0
dis annMedianSplit 0x180015cf0 0x180015fd4
echo "== cut-value constant"; objdump -s --start-address=0x1800b90b4 --stop-address=0x1800b90b8 "$DLL" | tail -1
dis annkSearch 0x1800128e0 0x180012b16
dis annBoxDistance 0x180015490 0x180015620
dis "ANNkd_split::ann_search" 0x180012b60 0x180012ced
dis "ANNkd_leaf::ann_search" 0x180012cf0 0x180012f5a
echo "== vtables: ANNkd_leaf 0x1800b8be0, ANNkd_split 0x1800b8c20 (slot 1 = ann_search, slot 2 = ann_pri_search)"
objdump -s --start-address=0x1800b8be0 --stop-address=0x1800b8c58 "$DLL" | tail -8
