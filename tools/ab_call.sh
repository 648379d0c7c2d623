#!/bin/bash
# One GPU call of an A/B comparison of kernel variants (tools/ab.py: one
# process, interleaved rounds, every variant's image bit-identical to the
# first's).  Variants are built on the CPU beforehand with
#   make variant NAME=<name> DEFS="-D..."       (kernels only)
#   make fullvariant NAME=<name> DEFS="-D..."   (kernels + host side)
# usage: tools/ab_call.sh [--sets d8,d9,4k,sec,r8,d6,tr] NAME1 NAME2 ...
#        (build/ab/libvrt_NAME.so; "head" = the in-tree libvrt.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
sets="d8,4k,sec"
if [ "$1" = "--sets" ]; then sets=$2; shift 2; fi
L=""
for n in "$@"; do
  if [ "$n" = head ]; then L="$L voxelraytrace20190722_amd/libvrt.so"; else L="$L build/ab/libvrt_$n.so"; fi
done
steps=()
for s in ${sets//,/ }; do
  case $s in
    d8)  steps+=("ab_d8|300|python -u tools/ab.py $L --rounds 6") ;;
    d9)  steps+=("ab_d9|300|python -u tools/ab.py $L --depth 9 --rounds 4") ;;
    4k)  steps+=("ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4") ;;
    sec) steps+=("ab_sec|400|python -u tools/ab.py $L --mode secondary --poses 8 --rounds 3") ;;
    r8)  steps+=("ab_r8|300|python -u tools/ab.py $L --ranks 8 --rounds 4") ;;
    tr)  steps+=("ab_tr|300|python -u tools/ab.py $L --mode trace --rounds 4") ;;
    s8)  steps+=("ab_s8|400|python -u tools/ab.py $L --share-ranks 8 --share-of 0,1,4 --rounds 5 --steps 64") ;;
    d6)  steps+=("ab_d6|300|python -u tools/ab.py $L --depth 6 --rounds 4") ;;
    *) echo "unknown set $s"; exit 2 ;;
  esac
done
bash tools/gpu_steps.sh "${steps[@]}"
