#!/bin/bash
# Round-6 experiment set J: config 5's phase-A stop threshold 24 / 26 / 30 /
# 34 against 18 (6 rounds), (A/B only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "ab_st|600|python -u tools/ab.py voxelraytrace20190722_amd/libvrt.so build/ab/libvrt_st24.so build/ab/libvrt_st26.so build/ab/libvrt_st30.so build/ab/libvrt_st34.so --mode secondary --rounds 6"
