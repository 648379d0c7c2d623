#!/bin/bash
# 8/4-rank rehearsal: the whole per-rank step vs the share's renders alone,
# 1-3 frames in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "reh8|200|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh8r|200|python -u bench.py --rehearse-ranks 8 --rehearse-render-only --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh8r1|200|python -u bench.py --rehearse-ranks 8 --rehearse-render-only --frames-in-flight 1 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh8_1|200|python -u bench.py --rehearse-ranks 8 --frames-in-flight 1 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "one1|200|python -u bench.py --frames-in-flight 1 --no-cpu --no-pmc --no-d9 --steps 128 --warmup 8"
