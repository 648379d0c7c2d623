#!/bin/bash
# Session-3 GPU call D: host enqueue time per step of the multi-rank path
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "reh8f2|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh8f3|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --frames-in-flight 3 --steps 128 --warmup 8" \
  "reh4f2|240|python -u bench.py --rehearse-ranks 4 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh2f2|240|python -u bench.py --rehearse-ranks 2 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "fif3|240|python -u bench.py --no-cpu --no-pmc --no-d9 --frames-in-flight 3 --steps 64 --warmup 4" \
  "fif2|240|python -u bench.py --no-cpu --no-pmc --no-d9 --steps 64 --warmup 4"
