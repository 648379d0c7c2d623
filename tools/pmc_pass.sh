#!/bin/bash
# One rocprofv3 PMC pass (no tracing combined) over bench.py, one frame in
# flight so counters are per launch.  Counters must fit one pass (see
# MI355X_MICROARCH.md: <= 8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_, 2 GRBM_).
# usage: tools/pmc_pass.sh TAG "COUNTER ..." [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; counters=$2; shift 2
O=$R/gpurun_out/pmc_$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc $counters --output-format csv -d "$O" -o "$tag" -- \
  python3 "$R/bench.py" --no-cpu --no-counters --no-pmc --no-d9 --frames-in-flight 1 --steps 16 --warmup 2 "$@" \
  > "$O/$tag.log" 2>&1
rc=$?
echo "pmc $tag rc=$rc"
exit $rc
