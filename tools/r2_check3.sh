#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
bash tools/gpu_steps.sh \
  "tests|900|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "bench_trace|300|python -u bench.py --mode trace --steps 16 --warmup 2 --no-cpu" \
  "ab_sec|400|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_secfin.so build/variants/libvrt_cur.so --mode secondary --poses 8 --rounds 3"
