#!/bin/bash
# Round-6 experiment set C: full-grid frames in flight (VRT_INFLIGHT_GRID_DIV=1)
# against the half-grid default, on bench.py's own schedule (the driver's
# 20 / 5 command and 64 frames) and on the 8-rank rehearsal; the config-5
# multi-rank rehearsal (pack + gather); the GPU tests of the changed paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
B="python -u bench.py --no-cpu --no-pmc --no-d9"
cp $L build/libvrt_head.so
bash tools/gpu_steps.sh \
  "tests_sel|600|python -u -m pytest tests -m gpu -k 'compaction or dist or secondary_rank or tile_partition' -v --timeout 300 --timeout-method thread" \
  "head20a|200|$B --steps 20 --warmup 5" \
  "head64a|200|$B --steps 64 --warmup 5" \
  "cp_gd1|20|cp build/ab/libvrt_gd1.so $L" \
  "gd1_20a|200|$B --steps 20 --warmup 5" \
  "gd1_64a|200|$B --steps 64 --warmup 5" \
  "gd1_reh8|300|$B --rehearse-ranks 8 --steps 256" \
  "restore|20|cp build/libvrt_head.so $L" \
  "head20b|200|$B --steps 20 --warmup 5" \
  "head64b|200|$B --steps 64 --warmup 5" \
  "head_reh8|300|$B --rehearse-ranks 8 --steps 256" \
  "cp_gd1b|20|cp build/ab/libvrt_gd1.so $L" \
  "gd1_20b|200|$B --steps 20 --warmup 5" \
  "gd1_64b|200|$B --steps 64 --warmup 5" \
  "restore2|20|cp build/libvrt_head.so $L" \
  "sec_reh8|400|$B --mode secondary --rehearse-ranks 8 --steps 16 --rehearse-repeats 1"
