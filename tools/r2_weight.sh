#!/bin/bash
# Weighted tile deal (rank 0 lighter from 4 ranks on): the multi-rank GPU
# tests, then the 8- and 4-rank rehearsals of rank 0's whole step (share +
# gather + unpack) and of rank 1's renders (the largest share).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python -u bench.py --no-cpu --no-pmc --steps 256 --warmup 8"
bash tools/gpu_steps.sh \
  "tests|500|python -u -m pytest tests/test_gpu.py tests/test_gpu_frames.py -m gpu -v -k 'partition or c4 or C4 or rank or tiles or in_flight' --timeout 300 --timeout-method thread" \
  "r8_0|200|$B --rehearse-ranks 8" \
  "r8_1r|200|$B --rehearse-ranks 8 --rehearse-rank 1 --rehearse-render-only" \
  "r8_1|200|$B --rehearse-ranks 8 --rehearse-rank 1" \
  "r4_0|200|$B --rehearse-ranks 4" \
  "r4_1r|200|$B --rehearse-ranks 4 --rehearse-rank 1 --rehearse-render-only" \
  "r2_0|200|$B --rehearse-ranks 2" \
  "r8_0b|200|$B --rehearse-ranks 8" \
  "r8_1rb|200|$B --rehearse-ranks 8 --rehearse-rank 1 --rehearse-render-only"
