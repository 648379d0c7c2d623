#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
R=$(pwd)
bash tools/gpu_steps.sh \
  "tests|900|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread" \
  "ab_d8|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nostrips.so $V/libvrt_w6.so" \
  "ab_4k|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nostrips.so $V/libvrt_w6.so --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_sec|400|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nostrips.so $V/libvrt_secw5.so $V/libvrt_secw7.so --mode secondary --poses 8 --rounds 3" \
  "bench|400|python -u bench.py --pmc-save $R/gpurun_out/pmc_bench" \
  "bench_sec|400|python -u bench.py --mode secondary --steps 16 --pmc-save $R/gpurun_out/pmc_sec"
