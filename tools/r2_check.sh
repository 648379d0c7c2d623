#!/bin/bash
# Round-2 GPU check: GPU tests, smoke, default bench (each step time-limited,
# stops after a fault/timeout).  Output under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "tests|1000|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python -u bench.py"
