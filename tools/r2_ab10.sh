#!/bin/bash
# A/B of the node triangle-box skip (VRT_NODE_BOX 0 = leaves only, 1 = every
# node) + the GPU tests of the default build (node boxes on).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
L="$V/libvrt_nb0.so $V/libvrt_nb1.so"
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $L" \
  "ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_d9|300|python -u tools/ab.py $L --depth 9 --rounds 4" \
  "ab_sec|400|python -u tools/ab.py $L --mode secondary --poses 8 --rounds 3" \
  "tests|900|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread"
