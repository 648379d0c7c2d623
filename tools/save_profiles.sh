#!/bin/bash
# Copy a tools/collect.sh run (gpurun_out/) into profiles/TAG: bench JSON
# lines, PMC CSVs and kernel-trace stats (+ summary.json re-deriving each
# roofline from them), the GPU test list and the smoke output.
# usage: tools/save_profiles.sh TAG
set -e
T=profiles/$1
rm -rf "$T"; mkdir -p "$T"
for x in pmc_bench:pmc_primary pmc_sec:pmc_secondary pmc_4k:pmc_4k pmc_trace:pmc_trace; do
  [ -d gpurun_out/${x%%:*} ] && cp -r gpurun_out/${x%%:*} "$T/${x#*:}"
done
for f in drv:driver_cmd bench:primary bench_sec:secondary bench_4k:4k bench_trace:trace gloo2:gloo2 abim8:abi_multi_rehearsal8 reh8:rccl_rehearsal8 reh4:rccl_rehearsal4 reh2:rccl_rehearsal2; do
  [ -f gpurun_out/${f%%:*}.log ] && grep '^{' gpurun_out/${f%%:*}.log > "$T/bench_${f#*:}.json" || true
done
grep -E "PASSED|FAILED|ERROR" gpurun_out/tests.log | sed 's/ *\[ *[0-9]*%\]$//' > "$T/gpu_tests.txt"
tail -1 gpurun_out/tests.log >> "$T/gpu_tests.txt"
cp gpurun_out/smoke.log "$T/smoke.txt"
for x in primary:pmc_primary secondary:pmc_secondary 4k:pmc_4k trace:pmc_trace; do
  python3 tools/pmc_summary.py "$T/bench_${x%%:*}.json" "$T/${x#*:}" | cut -c1-160
done
