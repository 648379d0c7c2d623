#!/bin/bash
# Session-3 GPU call E: LDS material/texture tables A/B; frames in flight 3/4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=build/variants
L="$V/libvrt_tabs0.so $V/libvrt_tabs1.so"
bash tools/gpu_steps.sh \
  "ab_d8|300|python -u tools/ab.py $L --rounds 6" \
  "ab_4k|300|python -u tools/ab.py $L --width 3840 --height 2160 --depth 9 --rounds 4" \
  "reh8f4|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --frames-in-flight 4 --steps 128 --warmup 8" \
  "reh8f3|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --frames-in-flight 3 --steps 128 --warmup 8" \
  "fif4|240|python -u bench.py --no-cpu --no-pmc --no-d9 --frames-in-flight 4 --steps 64 --warmup 4" \
  "fif3|240|python -u bench.py --no-cpu --no-pmc --no-d9 --frames-in-flight 3 --steps 64 --warmup 4"
