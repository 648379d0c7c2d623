#!/bin/bash
# VALU mix (fp64 share) and TA/TCP activity of k_render_p, one frame in flight.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_ta2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-counters --no-pmc --no-d9 --frames-in-flight 1 --steps 16 --warmup 2"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES --output-format csv -d $O/mix -o mix -- $B > $O/mix.log 2>&1
echo "mix rc=$?"
timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 --output-format csv -d $O/ta -o ta -- $B > $O/ta.log 2>&1
echo "ta rc=$?"
