#!/bin/bash
# Round-6 experiment set L: config 5 with the lane-staggered PCG start states
# from a compile-time table (c_pcg_jump3) against the previous build (r6b):
# config-5 tests, A/B, bench line; then the primary kernel's vector-memory
# path counters (tools/pmc_ta.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "tests_c5|600|python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction' --timeout 300 --timeout-method thread" \
  "ab_sec|400|python -u tools/ab.py build/ab/libvrt_r6b.so voxelraytrace20190722_amd/libvrt.so --mode secondary --rounds 4" \
  "sec|300|python -u bench.py --mode secondary --no-cpu --no-pmc" \
  "ta|400|bash tools/pmc_ta.sh"
