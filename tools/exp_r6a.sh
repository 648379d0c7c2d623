#!/bin/bash
# Round-6 experiment set A: config-5 walk write split (WRREQ passes on the
# head build and on a 5-waves/SIMD build without scratch), their timing A/B,
# the full-grid frames-in-flight variant, and the bench step-count scan that
# separates the frames-in-flight pipeline fill from the per-frame time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
W="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum"
cp $L build/libvrt_head.so
bash tools/gpu_steps.sh \
  "secw_head|250|bash tools/pmc_pass.sh secw_head \"$W\" --mode secondary" \
  "cp_w5|20|cp build/ab/libvrt_w5.so $L" \
  "secw_w5|250|bash tools/pmc_pass.sh secw_w5 \"$W\" --mode secondary" \
  "restore1|20|cp build/libvrt_head.so $L" \
  "ab_sec_w5|400|python -u tools/ab.py build/libvrt_head.so build/ab/libvrt_w5.so --mode secondary --rounds 4" \
  "ab_gd1|300|python -u tools/ab.py build/libvrt_head.so build/ab/libvrt_gd1.so --share-ranks 1 --fl 3 --steps 64 --rounds 6" \
  "steps20|200|python -u bench.py --no-cpu --no-pmc --no-d9 --steps 20 --warmup 5" \
  "steps32|200|python -u bench.py --no-cpu --no-pmc --no-d9 --steps 32 --warmup 5" \
  "steps64|200|python -u bench.py --no-cpu --no-pmc --no-d9 --steps 64 --warmup 5" \
  "steps128|200|python -u bench.py --no-cpu --no-pmc --no-d9 --steps 128 --warmup 5" \
  "steps16|200|python -u bench.py --no-cpu --no-pmc --no-d9 --steps 16 --warmup 5"
