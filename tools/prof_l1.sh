#!/bin/bash
# vL1D (TCP) hit rate of k_render_p, one frame in flight.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_l1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-counters --no-pmc --no-d9 --frames-in-flight 1 --steps 16 --warmup 2"
timeout -s KILL 200 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/a -o a -- $B > $O/a.log 2>&1
echo "a rc=$?"
timeout -s KILL 200 rocprofv3 --pmc TCP_PERF_SEL_TOTAL_HIT_LRU_READ TCP_PERF_SEL_TOTAL_MISS_LRU_READ TCP_PERF_SEL_TOTAL_MISS_EVICT_READ TCP_PERF_SEL_TOTAL_READ --output-format csv -d $O/b -o b -- $B > $O/b.log 2>&1
echo "b rc=$?"
