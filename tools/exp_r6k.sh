#!/bin/bash
# Round-6 experiment set K: config 5's stop threshold 18 / 30 / 34 / 40 / 48:
# per build (swapped in as the box copy's libvrt.so) the compaction counts
# (tools/sec_diag.py) and the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
cp $L build/ab/libvrt_st18.so
steps=()
for t in 18 30 34 40 48; do
  steps+=("diag$t|200|cp build/ab/libvrt_st$t.so $L && python -u tools/sec_diag.py --poses 4")
  steps+=("sec$t|200|python -u bench.py --mode secondary --no-cpu --no-pmc")
done
bash tools/gpu_steps.sh "${steps[@]}"
