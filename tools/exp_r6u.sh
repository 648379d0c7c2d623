#!/bin/bash
# Round-6 experiment set U: config 5's per-pixel primary record as one
# scalar load before the hit flag's branch (prec), the root node record
# through the scalar cache in every walk (root), both (both), against r6h
# (HEAD): A/B of config 5 and of the 1080p primary frame, then config-5
# tests + bench lines of prec and of root (each swapped in as the box
# copy's libvrt.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
A=build/ab
B="python -u bench.py --no-cpu --no-pmc"
T="python -u -m pytest tests -m gpu -v -k 'secondary or c5 or compaction or dist or c2 or frames_in_flight' --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "ab_sec|500|python -u tools/ab.py $A/libvrt_r6h.so $A/libvrt_prec.so $A/libvrt_root.so $A/libvrt_both.so --mode secondary --rounds 4" \
  "ab_d8|300|python -u tools/ab.py $A/libvrt_r6h.so $A/libvrt_root.so --rounds 6" \
  "tests_prec|600|cp $A/libvrt_prec.so $L && $T" \
  "sec_prec|200|$B --mode secondary" \
  "tests_root|600|cp $A/libvrt_root.so $L && $T" \
  "sec_root|200|$B --mode secondary"
