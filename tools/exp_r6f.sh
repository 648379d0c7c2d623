#!/bin/bash
# Round-6 experiment set F: the persistent render's per-unit phase split
# (dequeue / setup / march / shading, VRT_PHASE_STAMPS build) and the
# shading-chain change (TriPos beside TriAttr, texture record inline in the
# material) against the previous build (head6): A/B on the 1080p, 4K,
# config-5 and trace frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "diag|200|python -u tools/diag_phases.py build/ab/libvrt_diag.so" \
  "ab_d8|300|python -u tools/ab.py build/ab/libvrt_head6.so voxelraytrace20190722_amd/libvrt.so --rounds 6" \
  "ab_4k|300|python -u tools/ab.py build/ab/libvrt_head6.so voxelraytrace20190722_amd/libvrt.so --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_tr|300|python -u tools/ab.py build/ab/libvrt_head6.so voxelraytrace20190722_amd/libvrt.so --mode trace --rounds 4" \
  "sel|600|python -u -m pytest tests -m gpu -v -k 'c2_1080p or frames_in_flight or obj_ingest or trace_main or lightmap_and_trace or c5_1080p' --timeout 300 --timeout-method thread"
