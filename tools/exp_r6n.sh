#!/bin/bash
# Round-6 experiment set N: config 5's walk kernel taking 2 (HEAD) / 4 pixels
# per dequeue against 1 (r6d, which has the one-rank deal fast path) and r6c
# (before it): config-5 tests, A/B, bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "tests_c5|600|python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction or build_flags' --timeout 300 --timeout-method thread" \
  "ab_sec|500|python -u tools/ab.py build/ab/libvrt_r6c.so build/ab/libvrt_r6d.so voxelraytrace20190722_amd/libvrt.so build/ab/libvrt_take4.so --mode secondary --rounds 4" \
  "sec|300|python -u bench.py --mode secondary --no-cpu --no-pmc"
