#!/bin/bash
# A/B: HEAD (node boxes) vs the fma line test (VRT_NB_FMA) vs 6 waves/SIMD;
# phase breakdown of the fast march at HEAD (diagnostic build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
L="$V/libvrt_nb1.so $V/libvrt_nbf.so $V/libvrt_w6.so"
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $L" \
  "ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_sec|400|python -u tools/ab.py $L --mode secondary --poses 8 --rounds 3" \
  "diag|300|python -u tools/diag_phases.py $V/libvrt_diag.so"
