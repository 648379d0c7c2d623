#!/bin/bash
# Round-6 experiment set G: config 5's deferred-pixel walk on the compaction
# set's side stream beside the streaming resume (fork / join events) against
# the previous build (r6a): config-5 tests, A/B, bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "tests_c5|600|python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction or defer or dist' --timeout 300 --timeout-method thread" \
  "ab_sec|400|python -u tools/ab.py build/ab/libvrt_r6a.so voxelraytrace20190722_amd/libvrt.so --mode secondary --rounds 4" \
  "sec|300|python -u bench.py --mode secondary --no-cpu --no-pmc" \
  "ktr|300|rocprofv3 --kernel-trace --stats -d gpurun_out/ktr_sec -o ktr -- python -u bench.py --mode secondary --no-cpu --no-pmc --steps 8"
