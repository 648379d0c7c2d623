#!/bin/bash
# Session-3 GPU call C: frames in flight (2 streams) vs one stream, N=1 and
# the 8-rank rehearsal; GPU tests after the tile-deal change; gloo 2-rank
# rehearsal of the multi-rank bench path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "fif2|400|python -u bench.py --no-cpu --steps 32 --warmup 4" \
  "fif1|300|python -u bench.py --no-cpu --no-pmc --no-d9 --frames-in-flight 1 --steps 32 --warmup 4" \
  "reh8f2|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --steps 64 --warmup 8" \
  "reh8f1|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --frames-in-flight 1 --steps 64 --warmup 8" \
  "reh8f3|240|python -u bench.py --rehearse-ranks 8 --no-cpu --no-pmc --frames-in-flight 3 --steps 64 --warmup 8" \
  "sec2|400|python -u bench.py --mode secondary --no-cpu --no-pmc --steps 16 --warmup 2" \
  "k4|300|python -u bench.py --width 3840 --height 2160 --depth 9 --no-cpu --no-pmc --no-d9 --steps 16 --warmup 2" \
  "gloo2|300|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 8 --warmup 2" \
  "tests|600|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread"
