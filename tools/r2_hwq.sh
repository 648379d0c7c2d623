#!/bin/bash
# Frames in flight x hardware queues x grid share: 8-rank rehearsal step and
# the one-GPU frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python -u bench.py --no-cpu --no-pmc --no-d9 --steps 128 --warmup 8"
bash tools/gpu_steps.sh \
  "q4f3|200|$B --rehearse-ranks 8" \
  "q8f3|200|GPU_MAX_HW_QUEUES=8 $B --rehearse-ranks 8" \
  "q8f4|200|GPU_MAX_HW_QUEUES=8 $B --rehearse-ranks 8 --frames-in-flight 4" \
  "q8f4d3|200|GPU_MAX_HW_QUEUES=8 VRT_GRID_DIV=3 $B --rehearse-ranks 8 --frames-in-flight 4" \
  "q8f6d3|200|GPU_MAX_HW_QUEUES=8 VRT_GRID_DIV=3 $B --rehearse-ranks 8 --frames-in-flight 6" \
  "q8f6d4|200|GPU_MAX_HW_QUEUES=8 VRT_GRID_DIV=4 $B --rehearse-ranks 8 --frames-in-flight 6" \
  "q4f4d3|200|VRT_GRID_DIV=3 $B --rehearse-ranks 8 --frames-in-flight 4" \
  "one_q4f3|200|$B" \
  "one_q8f4|200|GPU_MAX_HW_QUEUES=8 $B --frames-in-flight 4" \
  "one_q8f4d3|200|GPU_MAX_HW_QUEUES=8 VRT_GRID_DIV=3 $B --frames-in-flight 4"
