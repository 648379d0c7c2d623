#!/bin/bash
# The measurement set of a round in one GPU call: GPU tests, smoke, the
# driver's own bench command (bench.py --gpus 1 --steps 20 --warmup 5), the C2 /
# C3 / config-5 / trace bench lines with their PMC passes and kernel-trace
# stats saved (bench.py --pmc-save), the 8/4/2-rank RCCL rehearsals and a
# 2-rank gloo run of the spawning launcher.  tools/save_profiles.sh TAG then
# copies the results into profiles/TAG.
# usage: tools/collect.sh [--no-tests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmc_bench gpurun_out/pmc_4k gpurun_out/pmc_sec gpurun_out/pmc_trace
B="python -u bench.py"
exec bash tools/check_call.sh "$@" \
  "drv|500|$B --gpus 1 --steps 20 --warmup 5" \
  "bench|500|$B --pmc-save gpurun_out/pmc_bench" \
  "bench_4k|500|$B --width 3840 --height 2160 --depth 9 --pmc-save gpurun_out/pmc_4k" \
  "bench_sec|700|$B --mode secondary --pmc-save gpurun_out/pmc_sec" \
  "bench_trace|500|$B --mode trace --pmc-save gpurun_out/pmc_trace" \
  "reh8|200|$B --no-cpu --no-pmc --rehearse-ranks 8 --steps 256" \
  "reh4|200|$B --no-cpu --no-pmc --rehearse-ranks 4 --steps 256" \
  "reh2|200|$B --no-cpu --no-pmc --rehearse-ranks 2 --steps 256" \
  "gloo2|300|$B --no-cpu --no-pmc --gpus 2 --dist-backend gloo" \
  "abim8|200|$B --abi-multi --abi-multi-virtual 8 --steps 64"
