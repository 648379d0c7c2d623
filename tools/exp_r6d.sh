#!/bin/bash
# Round-6 experiment set D: the walk's event counts (VRT_PHASE_STAMPS build),
# the cone march with one divergent region per step (trace tests, A/B, bench
# line with the SALU fraction), the streaming resume holding leaves until
# VRT_STREAM_LEAF_T lanes have one (config-5 tests, A/B of thresholds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
bash tools/gpu_steps.sh \
  "diag|200|python -u tools/diag_phases.py build/ab/libvrt_diag.so" \
  "tests_d|900|python -u -m pytest tests -m gpu -k 'trace or compaction or secondary or c5' -v --timeout 300 --timeout-method thread" \
  "ab_tr|400|python -u tools/ab.py build/ab/libvrt_base.so $L --mode trace --rounds 6" \
  "ab_st|500|python -u tools/ab.py $L build/ab/libvrt_t0.so build/ab/libvrt_t24.so build/ab/libvrt_t48.so build/ab/libvrt_base.so --mode secondary --rounds 4" \
  "trace|400|python -u bench.py --mode trace --no-cpu --steps 32"
