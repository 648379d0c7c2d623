#!/bin/bash
# Session-3 GPU call A: GPU tests at HEAD, the single-GPU RCCL rehearsal of
# the N-rank step, the phase-stamp breakdown and an SQ stall pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "tests|600|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "reh8|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 64 --warmup 8" \
  "reh4|240|python -u bench.py --rehearse-ranks 4 --no-cpu --no-pmc --steps 64 --warmup 8" \
  "reh2|240|python -u bench.py --rehearse-ranks 2 --no-cpu --no-pmc --steps 64 --warmup 8" \
  "diag|240|python -u tools/diag_phases.py build/variants/libvrt_diag.so" \
  "stall|300|bash tools/prof_stall.sh p --no-pmc --no-d9 --steps 16 --warmup 2"
