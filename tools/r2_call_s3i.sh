#!/bin/bash
# Session-3 GPU call I: leaf-record LDS-DMA prefetch A/B (bit-identical images checked by ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=build/variants
L="$V/libvrt_pf0.so $V/libvrt_pf1.so"
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $L --rounds 6" \
  "ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_d9|300|python -u tools/ab.py $L --depth 9 --rounds 4" \
  "ab_r8|300|python -u tools/ab.py $L --ranks 8 --rounds 4"
