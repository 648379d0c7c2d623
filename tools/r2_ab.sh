#!/bin/bash
# Round-2 A/B: GPU tests, then interleaved in-process A/B of kernel variants
# (tools/ab.py: every variant's images bit-identical to the first's), then the
# default bench (live PMC roofline).  Output under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=build/variants
bash tools/gpu_steps.sh "dbg|90|python -u tools/dbg_sec.py" \
  "tests|900|python -u -m pytest tests -m gpu -v --maxfail 5 --timeout 300 --timeout-method thread" \
  "ab_d8|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nofast.so $V/libvrt_nohelp.so $V/libvrt_lds320.so $V/libvrt_w4.so $V/libvrt_w6.so" \
  "ab_4k|300|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_nofast.so $V/libvrt_nohelp.so $V/libvrt_lds320.so --width 3840 --height 2160 --depth 9 --rounds 4" \
  "ab_sec|400|python -u tools/ab.py $V/libvrt_head.so $V/libvrt_base.so $V/libvrt_secold.so $V/libvrt_secw5.so $V/libvrt_secw8.so --mode secondary --poses 8 --rounds 3" \
  "bench|400|python -u bench.py"
