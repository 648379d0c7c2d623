#!/bin/bash
# Upper bound of dropping the per-frame k_render_defer launch (timing only):
# the 8-rank rehearsal and the one-GPU frame, head vs a build without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python -u bench.py --no-cpu --no-pmc --no-d9 --steps 256 --warmup 8"
cp voxelraytrace20190722_amd/libvrt.so build/libvrt_head.so
bash tools/gpu_steps.sh \
  "h_reh8|200|$B --rehearse-ranks 8" \
  "h_one|200|$B" \
  "swap|20|cp build/variants/libvrt_nodefer.so voxelraytrace20190722_amd/libvrt.so" \
  "n_reh8|200|$B --rehearse-ranks 8" \
  "n_one|200|$B" \
  "back|20|cp build/libvrt_head.so voxelraytrace20190722_amd/libvrt.so" \
  "h_reh8b|200|$B --rehearse-ranks 8" \
  "h_oneb|200|$B"
