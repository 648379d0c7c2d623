#!/bin/bash
# Session-3 GPU call B: where the per-rank share of a multi-GPU frame loses
# time, and the tile-deal block size A/B (G = 1, 2, 4, 8; every rank's share
# timed, slowest rank per pose) at 1080p depth 8 and 4K depth 9, 8 and 2
# ranks; PMC of rank 0's share of 8 (rehearsal) and of full frames at
# reduced resolution (1/8 of the rays over the same view / compact).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=build/variants
L="$V/libvrt_g1.so $V/libvrt_g2.so $V/libvrt_g4.so $V/libvrt_g8.so"
bash tools/gpu_steps.sh \
  "ab8|300|python -u tools/ab.py $L --ranks 8 --rounds 4" \
  "ab2|300|python -u tools/ab.py $L --ranks 2 --rounds 4" \
  "ab8_4k|400|python -u tools/ab.py $L --ranks 8 --rounds 3 --width 3840 --height 2160 --depth 9" \
  "reh8p|400|python -u bench.py --rehearse-ranks 8 --no-cpu --steps 32 --warmup 4 --pmc-save gpurun_out/pmc_reh8" \
  "full|400|python -u bench.py --no-cpu --no-d9 --steps 32 --warmup 4" \
  "f680|400|python -u bench.py --no-cpu --no-d9 --width 680 --height 384 --steps 32 --warmup 4" \
  "f136|400|python -u bench.py --no-cpu --no-d9 --width 1920 --height 136 --steps 32 --warmup 4"
