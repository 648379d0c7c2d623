#!/bin/bash
# Round-6 experiment set B: the fast-only config-5 walk kernel (no scratch)
# with its deferred-pixel launch: GPU tests of config 5, the write-request
# pass, the compaction stats, the A/B against the previous build; and the
# full-grid frames-in-flight variant of the primary render, A/B'd on the
# bench's own schedule (3 frames in flight, 20 and 64 frames).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum"
bash tools/gpu_steps.sh \
  "tests_c5|600|python -u -m pytest tests -m gpu -k 'secondary or c5 or compaction' -v --timeout 300 --timeout-method thread" \
  "secw_new|250|bash tools/pmc_pass.sh secw_new \"$W\" --mode secondary" \
  "secdiag|200|python -u tools/sec_diag.py --poses 16" \
  "ab_sec|400|python -u tools/ab.py build/ab/libvrt_base.so voxelraytrace20190722_amd/libvrt.so --mode secondary --rounds 4" \
  "ab_gd1_64|300|python -u tools/ab.py build/ab/libvrt_base.so build/ab/libvrt_gd1.so --share-ranks 1 --share-of 0 --fl 3 --steps 64 --rounds 6" \
  "ab_gd1_20|300|python -u tools/ab.py build/ab/libvrt_base.so build/ab/libvrt_gd1.so --share-ranks 1 --share-of 0 --fl 3 --steps 20 --rounds 8"
