#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_fin.so $V/libvrt_finw6.so $V/libvrt_rc2.so $V/libvrt_rc2w6.so" \
  "ab_4k|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_fin.so $V/libvrt_finw6.so $V/libvrt_rc2.so $V/libvrt_rc2w6.so --width 3840 --height 2160 --depth 9 --rounds 4" \
  "tests|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread"
