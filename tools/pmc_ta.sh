#!/bin/bash
# Vector-memory-path counters of the primary kernel: the counter list of the
# box (TA/TD/TCP blocks), then one PMC pass per group over the bench's timed
# frames (one frame in flight), each under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ta
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/ta/avail.txt 2>&1
grep -E "^\s*(TA|TD|TCP)_" gpurun_out/ta/avail.txt | head -80 > gpurun_out/ta/avail_tatd.txt
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pmc --no-counters --no-d9 --frames-in-flight 1 --warmup 0 --steps 16"
i=0
for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TD_BUSY_avr TD_BUSY_max GRBM_GUI_ACTIVE" "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ta/p$i -o p$i -- $B) > gpurun_out/ta/p$i.log 2>&1
  echo "pass $i ($grp) rc=$?"
done
