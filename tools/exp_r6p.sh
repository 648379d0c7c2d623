#!/bin/bash
# Round-6 experiment set P: the multi-rank tile deal tabled on the device
# (RenderParams::tile_xy, one scalar load per unit / pixel) against r6e (the
# deal computed per unit): multi-rank GPU tests, the 8-rank primary shares
# (A/B, every 3rd rank), the 8-rank rehearsals of both modes per build
# (swapped in as the box copy's libvrt.so); then config 5's bench line with
# 1 / 2 / 4 / 8 pixels per dequeue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
cp $L build/ab/libvrt_map.so
B="python -u bench.py --no-cpu --no-pmc"
bash tools/gpu_steps.sh \
  "tests|600|python -u -m pytest tests -m gpu -v -k 'dist or rank or partition or multi or tiles or unpack or c5 or compaction' --timeout 300 --timeout-method thread" \
  "ab_s8|400|python -u tools/ab.py build/ab/libvrt_r6e.so $L --share-ranks 8 --share-of 0,1,4 --rounds 5 --steps 64" \
  "reh8_map|200|$B --rehearse-ranks 8 --steps 256" \
  "sreh8_map|300|$B --mode secondary --rehearse-ranks 8" \
  "reh8_old|200|cp build/ab/libvrt_r6e.so $L && $B --rehearse-ranks 8 --steps 256" \
  "sreh8_old|300|$B --mode secondary --rehearse-ranks 8" \
  "sec1|200|cp build/ab/libvrt_r6d.so $L && $B --mode secondary" \
  "sec2|200|cp build/ab/libvrt_map.so $L && $B --mode secondary" \
  "sec4|200|cp build/ab/libvrt_take4.so $L && $B --mode secondary" \
  "sec8|200|cp build/ab/libvrt_take8.so $L && $B --mode secondary" \
  "sec2b|200|cp build/ab/libvrt_map.so $L && $B --mode secondary" \
  "sec4b|200|cp build/ab/libvrt_take4.so $L && $B --mode secondary"
