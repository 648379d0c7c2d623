#!/bin/bash
# Headline and 8-rank-rehearsal bench lines of several library variants in
# one GPU call, alternating (each variant's libvrt.so swapped into the
# package in turn, the in-tree one restored at the end).
# usage: tools/swap_bench.sh NAME1 NAME2 ...   ("head" = the in-tree libvrt.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=voxelraytrace20190722_amd/libvrt.so
cp $P build/libvrt_head.so
B="python -u bench.py --no-cpu --no-pmc --no-d9 --steps 64 --warmup 8"
steps=()
for round in 1 2; do
  for n in "$@"; do
    src=build/variants/libvrt_$n.so; [ "$n" = head ] && src=build/libvrt_head.so
    steps+=("cp_${n}_$round|20|cp $src $P")
    steps+=("one_${n}_$round|200|$B")
    steps+=("reh8_${n}_$round|200|$B --rehearse-ranks 8 --steps 256")
  done
done
steps+=("restore|20|cp build/libvrt_head.so $P")
bash tools/gpu_steps.sh "${steps[@]}"
