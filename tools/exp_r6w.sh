#!/bin/bash
# Round-6 experiment set W: the primary render's 4-sample film sum by DPP
# quad broadcasts instead of ds_bpermute (build dpp; HEAD = r6i): A/B at
# 1080p, 4K and on the 8-rank share (images bit-identical), then the GPU
# tests of the primary images with the working tree's (dpp) library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
A=build/ab
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $A/libvrt_r6i.so $A/libvrt_dpp.so --rounds 6" \
  "ab_4k|300|python -u tools/ab.py $A/libvrt_r6i.so $A/libvrt_dpp.so --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_s8|300|python -u tools/ab.py $A/libvrt_r6i.so $A/libvrt_dpp.so --share-ranks 8 --share-of 0,1,4 --rounds 5 --steps 64" \
  "tests|700|python -u -m pytest tests -m gpu -v -k 'c1 or c2 or c3 or 4k or frames_in_flight or defer or band or host_output or tiles or multi or selftest or golden' --timeout 300 --timeout-method thread"
