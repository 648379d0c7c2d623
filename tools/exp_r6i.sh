#!/bin/bash
# Round-6 experiment set I: config 5's phase-A stop threshold (walking lanes)
# re-measured with the fast-only walk kernel: 14 / 22 / 26 against 18.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "ab_st|500|python -u tools/ab.py voxelraytrace20190722_amd/libvrt.so build/ab/libvrt_st14.so build/ab/libvrt_st22.so build/ab/libvrt_st26.so --mode secondary --rounds 4"
