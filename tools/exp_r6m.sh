#!/bin/bash
# Round-6 experiment set M: config 5 with the one-rank deal fast path (no
# tile_deal / deal_count divisions per pixel) against the previous build
# (r6c): config-5 tests, A/B, bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "tests_c5|600|python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction' --timeout 300 --timeout-method thread" \
  "ab_sec|400|python -u tools/ab.py build/ab/libvrt_r6c.so voxelraytrace20190722_amd/libvrt.so --mode secondary --rounds 4" \
  "sec|300|python -u bench.py --mode secondary --no-cpu --no-pmc"
