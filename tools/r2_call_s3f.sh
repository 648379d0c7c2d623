#!/bin/bash
# Session-3 GPU call F: persistent grid size per frame with frames in flight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R="python -u bench.py --no-cpu --no-pmc --no-d9"
bash tools/gpu_steps.sh \
  "r8d1|200|VRT_PERSIST_GRID_DIV=1 $R --rehearse-ranks 8 --steps 128 --warmup 8" \
  "r8d2|200|VRT_PERSIST_GRID_DIV=2 $R --rehearse-ranks 8 --steps 128 --warmup 8" \
  "r8d2f4|200|VRT_PERSIST_GRID_DIV=2 $R --rehearse-ranks 8 --frames-in-flight 4 --steps 128 --warmup 8" \
  "r8d3|200|VRT_PERSIST_GRID_DIV=3 $R --rehearse-ranks 8 --steps 128 --warmup 8" \
  "n1d1|200|VRT_PERSIST_GRID_DIV=1 $R --steps 64 --warmup 4" \
  "n1d2|200|VRT_PERSIST_GRID_DIV=2 $R --steps 64 --warmup 4" \
  "n1d2f2|200|VRT_PERSIST_GRID_DIV=2 $R --frames-in-flight 2 --steps 64 --warmup 4" \
  "r4d1|200|VRT_PERSIST_GRID_DIV=1 $R --rehearse-ranks 4 --steps 128 --warmup 8" \
  "r4d2|200|VRT_PERSIST_GRID_DIV=2 $R --rehearse-ranks 4 --steps 128 --warmup 8" \
  "r2d1|200|VRT_PERSIST_GRID_DIV=1 $R --rehearse-ranks 2 --steps 128 --warmup 8" \
  "r2d2|200|VRT_PERSIST_GRID_DIV=2 $R --rehearse-ranks 2 --steps 128 --warmup 8"
