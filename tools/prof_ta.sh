#!/bin/bash
# Counter list of the box + SQ stall/activity pass over the default bench
# (k_render_p, one frame in flight so counters are per launch).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_ta
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > $O/list_avail.txt 2>&1
echo "list rc=$?"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD --output-format csv -d $O/stall -o stall -- python3 $R/bench.py --no-cpu --no-counters --no-pmc --no-d9 --frames-in-flight 1 --steps 16 --warmup 2 > $O/stall.log 2>&1
echo "stall rc=$?"
