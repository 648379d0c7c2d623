#!/bin/bash
# Session-3 GPU call B: where the per-rank share of a multi-GPU frame loses
# time -- PMC of rank 0's share of 8 (rehearsal) vs a full 1080p frame, a
# 680x384 film (1/8 the rays over the same view) and a 1920x136 film (1/8
# the rays, compact), all on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "reh8p|400|python -u bench.py --rehearse-ranks 8 --no-cpu --steps 32 --warmup 4 --pmc-save gpurun_out/pmc_reh8" \
  "full|400|python -u bench.py --no-cpu --no-d9 --steps 32 --warmup 4" \
  "f680|400|python -u bench.py --no-cpu --no-d9 --width 680 --height 384 --steps 32 --warmup 4" \
  "f136|400|python -u bench.py --no-cpu --no-d9 --width 1920 --height 136 --steps 32 --warmup 4" \
  "reh8new|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 64 --warmup 8"
