#!/bin/bash
# Round-6 experiment set R: config 5's pixel-centre primary pass compiled
# fast-only (a wave with a ray off the fast march lists its tile for
# k_primary1_defer) at 6 / 5 / 4 waves per SIMD (p1w6 / p1w5 / p1w4) against
# the general pass (r6g): config-5 tests of p1w6 (swapped in as the box
# copy's libvrt.so), A/B, and a kernel trace of its bench (k_primary1's time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
bash tools/gpu_steps.sh \
  "ab_sec|500|python -u tools/ab.py build/ab/libvrt_r6g.so build/ab/libvrt_p1w6.so build/ab/libvrt_p1w5.so build/ab/libvrt_p1w4.so --mode secondary --rounds 4" \
  "tests_c5|600|cp build/ab/libvrt_p1w6.so $L && python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction' --timeout 300 --timeout-method thread" \
  "ktr|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktr_sec -o ktr -- python -u bench.py --mode secondary --no-cpu --no-pmc --steps 8"
