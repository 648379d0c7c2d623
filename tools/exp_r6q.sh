#!/bin/bash
# Round-6 experiment set Q: one rank's tile index split by a magic divisor
# (RenderParams::ntx_magic, rank_tile) in the primary render, the light and
# trace-primary passes and the cone shading, against r6f (a division per
# unit): GPU tests of those paths, A/B at 1080p, 4K and on the trace frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
bash tools/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -v -k 'c1 or c2 or c3 or 4k or frames_in_flight or trace or lightmap or band or host_output or defer or ray_march' --timeout 300 --timeout-method thread" \
  "ab_d8|300|python -u tools/ab.py build/ab/libvrt_r6f.so $L --rounds 6" \
  "ab_4k|300|python -u tools/ab.py build/ab/libvrt_r6f.so $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_tr|300|python -u tools/ab.py build/ab/libvrt_r6f.so $L --mode trace --rounds 6"
