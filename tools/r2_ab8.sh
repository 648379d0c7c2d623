#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
bash tools/gpu_steps.sh \
  "ab_sec|400|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_pv1.so $V/libvrt_pv2.so --mode secondary --poses 8 --rounds 3" \
  "tests|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread"
