#!/bin/bash
# Session-3 GPU call K: leaf triangle-box skip A/B (bit-identical images checked by ab.py),
# primary 1080p d8 / d9 / 4K d9 and config 5; then the GPU tests with it on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=build/variants
L="$V/libvrt_lb0.so $V/libvrt_lb1.so"
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $L --rounds 6" \
  "ab_d9|300|python -u tools/ab.py $L --depth 9 --rounds 4" \
  "ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_sec|400|python -u tools/ab.py $L --mode secondary --poses 8 --rounds 3" \
  "tests|900|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread"
