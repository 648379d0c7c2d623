#!/bin/bash
# Round-6 experiment set E (the set D of commit 6777541, first run): full GPU
# tests and smoke of HEAD, the walk's event counts (VRT_PHASE_STAMPS build),
# A/B of the trace frame against the previous commit's library (base), A/B of
# the streaming resume's leaf-hold threshold (t0 = test every turn), and the
# trace and config-5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
bash tools/check_call.sh \
  "diag|200|python -u tools/diag_phases.py build/ab/libvrt_diag.so" \
  "ab_tr|400|python -u tools/ab.py build/ab/libvrt_base.so $L --mode trace --rounds 6" \
  "ab_st|500|python -u tools/ab.py $L build/ab/libvrt_t0.so build/ab/libvrt_t24.so build/ab/libvrt_t48.so build/ab/libvrt_base.so --mode secondary --rounds 4" \
  "trace|400|python -u bench.py --mode trace --no-cpu --steps 32" \
  "sec|400|python -u bench.py --mode secondary --no-cpu --no-pmc"
