#!/bin/bash
# Kernel trace of the 8-rank rehearsal (renders only, and the whole step).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/reh8r -o t -- python3 $R/bench.py --rehearse-ranks 8 --rehearse-render-only --no-cpu --no-pmc --steps 64 --warmup 8 > $R/gpurun_out/reh8r.log 2>&1
echo "reh8r rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/reh8 -o t -- python3 $R/bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 64 --warmup 8 > $R/gpurun_out/reh8.log 2>&1
echo "reh8 rc=$?"
