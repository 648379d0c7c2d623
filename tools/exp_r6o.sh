#!/bin/bash
# Round-6 experiment set O: config 5 bench lines (the metric, 32 frames, two
# runs each) with 1 / 2 / 4 / 8 pixels per dequeue (swapped in as the box
# copy's libvrt.so; 1 = r6d).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
cp $L build/ab/libvrt_take2.so
cp build/ab/libvrt_r6d.so build/ab/libvrt_take1.so
steps=()
for r in a b; do
  for t in 1 2 4 8; do
    steps+=("sec$t$r|200|cp build/ab/libvrt_take$t.so $L && python -u bench.py --mode secondary --no-cpu --no-pmc")
  done
done
bash tools/gpu_steps.sh "${steps[@]}"
