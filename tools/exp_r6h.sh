#!/bin/bash
# Round-6 experiment set H: config 5's pixel-centre primary pass with a wave
# per 8x8 tile (k_primary1) on top of the side-stream deferred walk: config-5
# tests, A/B against r6a and the side-stream-only build, bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "tests_c5|600|python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction or defer or dist' --timeout 300 --timeout-method thread" \
  "ab_sec|400|python -u tools/ab.py build/ab/libvrt_r6a.so build/ab/libvrt_side.so voxelraytrace20190722_amd/libvrt.so --mode secondary --rounds 4" \
  "sec|300|python -u bench.py --mode secondary --no-cpu --no-pmc"
