#!/bin/bash
# Every rank's share of the N-rank step rehearsed on one GPU (bench.py
# --rehearse-ranks N --rehearse-rank r), plus render-only spans of ranks 0/1.
# usage: tools/reh_all.sh [steps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=${1:-256}
steps=()
for r in 0 1 2 3 4 5 6 7; do
  steps+=("reh8_r$r|120|python -u bench.py --no-cpu --no-pmc --rehearse-ranks 8 --rehearse-rank $r --steps $S")
done
for r in 0 1; do
  steps+=("reh8ro_r$r|120|python -u bench.py --no-cpu --no-pmc --rehearse-ranks 8 --rehearse-rank $r --rehearse-render-only --steps $S")
done
for r in 0 1 2 3; do
  steps+=("reh4_r$r|120|python -u bench.py --no-cpu --no-pmc --rehearse-ranks 4 --rehearse-rank $r --steps $S")
done
bash tools/gpu_steps.sh "${steps[@]}"
