#!/bin/bash
# Round-2 GPU check of HEAD (session 3): tests, smoke, the benches (PMC CSVs
# kept), kernel-trace stats of the primary bench as run (3 frames in flight)
# and with one frame in flight, of config 5, the 8/4/2-rank RCCL rehearsals
# and a 2-rank gloo rehearsal of bench.py on the one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TR="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv"
bash tools/gpu_steps.sh \
  "tests|900|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|400|python -u bench.py --pmc-save $R/gpurun_out/pmc_bench" \
  "bench_sec|400|python -u bench.py --mode secondary --pmc-save $R/gpurun_out/pmc_sec" \
  "bench_4k|400|python -u bench.py --width 3840 --height 2160 --depth 9 --no-d9 --pmc-save $R/gpurun_out/pmc_4k" \
  "bench_trace|300|python -u bench.py --mode trace" \
  "reh8|200|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh4|200|python -u bench.py --rehearse-ranks 4 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "reh2|200|python -u bench.py --rehearse-ranks 2 --no-cpu --no-pmc --steps 128 --warmup 8" \
  "trace_p|300|$TR -d $R/gpurun_out/trace_bench -o trace -- python3 $R/bench.py --no-cpu --no-pmc --no-counters --no-d9" \
  "trace_p1|300|$TR -d $R/gpurun_out/trace_bench1 -o trace -- python3 $R/bench.py --no-cpu --no-pmc --no-counters --no-d9 --frames-in-flight 1" \
  "trace_s|300|$TR -d $R/gpurun_out/trace_sec -o trace -- python3 $R/bench.py --mode secondary --no-cpu --no-pmc" \
  "gloo2|300|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 2 --dist-backend gloo"
