#!/bin/bash
# A/B of primary-render variants + the default bench with its PMC CSVs kept
# + a rocprofv3 kernel-trace/stats pass of the same bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
R=$(pwd)
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nofast.so $V/libvrt_nohelp.so $V/libvrt_lds320.so $V/libvrt_w4.so $V/libvrt_w6.so" \
  "ab_4k|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nofast.so $V/libvrt_nohelp.so $V/libvrt_lds320.so --width 3840 --height 2160 --depth 9 --rounds 4" \
  "bench|400|python -u bench.py --pmc-save $R/gpurun_out/pmc_bench" \
  "trace|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_bench -o trace -- python3 $R/bench.py --no-cpu --no-pmc --no-counters --no-d9"
