#!/bin/bash
# Copy a tools/r2_check2.sh run (gpurun_out/) into profiles/TAG: bench JSON
# lines, PMC CSVs (+ summary.json re-deriving each roofline), kernel-trace
# stats, the GPU test list and the smoke output.  usage: tools/save_profiles.sh TAG
set -e
T=profiles/$1
rm -rf "$T"; mkdir -p "$T"
for x in pmc_bench:pmc_primary pmc_sec:pmc_secondary pmc_4k:pmc_4k; do
  [ -d gpurun_out/${x%%:*} ] && cp -r gpurun_out/${x%%:*} "$T/${x#*:}" && rm -f "$T/${x#*:}"/*agent_info.csv
done
for f in bench:primary bench_sec:secondary bench_4k:4k bench_trace:trace gloo2:gloo2_rehearsal reh8:rccl_rehearsal8 reh4:rccl_rehearsal4 reh2:rccl_rehearsal2; do
  [ -f gpurun_out/${f%%:*}.log ] && grep '^{' gpurun_out/${f%%:*}.log > "$T/bench_${f#*:}.json" || true
done
cp gpurun_out/trace_bench/trace_kernel_stats.csv "$T/primary_kernel_stats.csv"
cp gpurun_out/trace_sec/trace_kernel_stats.csv "$T/secondary_kernel_stats.csv"
[ -f gpurun_out/trace_bench1/trace_kernel_stats.csv ] && cp gpurun_out/trace_bench1/trace_kernel_stats.csv "$T/primary_1frame_kernel_stats.csv"
grep -E "PASSED|FAILED|ERROR" gpurun_out/tests.log | sed 's/ *\[ *[0-9]*%\]$//' > "$T/gpu_tests.txt"
tail -1 gpurun_out/tests.log >> "$T/gpu_tests.txt"
cp gpurun_out/smoke.log "$T/smoke.txt"
for x in primary:pmc_primary secondary:pmc_secondary 4k:pmc_4k; do
  python3 tools/pmc_summary.py "$T/bench_${x%%:*}.json" "$T/${x#*:}" | cut -c1-100
done
