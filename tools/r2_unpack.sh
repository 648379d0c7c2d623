#!/bin/bash
# k_unpack4: the partition/C4 GPU tests and the 8/4/2-rank rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest tests/test_gpu.py tests/test_gpu_frames.py -m gpu -v -k 'partition or c4 or C4 or rank' --timeout 300 --timeout-method thread" \
  "reh8|200|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 256 --warmup 8" \
  "reh4|200|python -u bench.py --rehearse-ranks 4 --no-cpu --no-pmc --steps 256 --warmup 8" \
  "reh2|200|python -u bench.py --rehearse-ranks 2 --no-cpu --no-pmc --steps 256 --warmup 8" \
  "reh8b|200|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 256 --warmup 8"
