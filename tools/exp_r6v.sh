#!/bin/bash
# Final round-6 check of HEAD: GPU tests + smoke, the driver's bench command
# and the config-5 / trace bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python -u bench.py --no-cpu --no-pmc"
bash tools/check_call.sh \
  "drv|300|python -u bench.py --gpus 1 --steps 20 --warmup 5" \
  "sec|200|$B --mode secondary" \
  "trace|200|$B --mode trace"
