#!/bin/bash
# One GPU check of HEAD: GPU tests, smoke, then optional extra steps given as
# "name|timeout|command" arguments (tools/gpu_steps.sh stops at the first
# fault / abort / timeout).  usage: tools/check_call.sh [--no-tests] [steps...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
steps=()
if [ "$1" = "--no-tests" ]; then shift; else
  steps+=("tests|900|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread")
  steps+=("smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'")
fi
bash tools/gpu_steps.sh "${steps[@]}" "$@"
