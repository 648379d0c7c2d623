#!/bin/bash
# Round-6 check of HEAD: GPU tests + smoke (tools/check_call.sh), config 5's
# bench line with 1 / 2 frames in flight (two runs each), the driver's
# command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python -u bench.py --no-cpu --no-pmc"
bash tools/check_call.sh \
  "sec_f1a|200|$B --mode secondary" \
  "sec_f2a|200|$B --mode secondary --frames-in-flight-secondary 2" \
  "sec_f1b|200|$B --mode secondary" \
  "sec_f2b|200|$B --mode secondary --frames-in-flight-secondary 2" \
  "drv|300|python -u bench.py --gpus 1 --steps 20 --warmup 5"
