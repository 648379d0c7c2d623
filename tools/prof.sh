#!/bin/bash
# rocprofv3 passes over bench.py (kernel trace + stats, then one PMC group per
# pass, never combined with tracing).  usage: tools/prof.sh TAG [bench args]
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $O/$name -o $name -- python3 $R/bench.py --no-cpu --no-counters "${ARGS[@]}" > $O/$name.log 2>&1; }
ARGS=("$@")
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run tcc --pmc TCC_HIT_sum TCC_MISS_sum
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS
run grbm --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES
echo done
