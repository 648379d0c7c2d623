#!/bin/bash
# Session-3 GPU call J: composition of the 8-rank share step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R="python -u bench.py --no-cpu --no-pmc --no-d9"
TR="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv"
bash tools/gpu_steps.sh \
  "r8|200|$R --rehearse-ranks 8 --steps 256 --warmup 8" \
  "r8ro|200|$R --rehearse-ranks 8 --rehearse-render-only --steps 256 --warmup 8" \
  "r8ro1|200|$R --rehearse-ranks 8 --rehearse-render-only --frames-in-flight 1 --steps 256 --warmup 8" \
  "r8tr|300|$TR -d $(pwd)/gpurun_out/tr_r8 -o tr -- python3 $(pwd)/bench.py --no-cpu --no-pmc --no-d9 --rehearse-ranks 8 --steps 64 --warmup 4"
