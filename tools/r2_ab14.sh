#!/bin/bash
# A/B: texel bytes from two aligned dwords (VRT_TEXEL_DW).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
L="$V/libvrt_head.so $V/libvrt_tdw.so"
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $L" \
  "ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_sec|400|python -u tools/ab.py $L --mode secondary --poses 8 --rounds 3"
