#!/bin/bash
# Cone-march path cache (VRT_CONE_PATH = cached levels, 0 = off): the
# reference main() frame per variant, then the trace parity tests on each
# caching variant; the head library is restored at the end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cp voxelraytrace20190722_amd/libvrt.so build/libvrt_head.so
B="python -u bench.py --mode trace --no-cpu --steps 64 --warmup 4"
T="python -u -m pytest tests/test_gpu.py -m gpu -q -k 'lightmap_and_trace or trace_device' --timeout 300 --timeout-method thread"
steps=()
for r in 1 2; do
  for n in 0 3 5 6; do
    steps+=("sw_${n}_$r|20|cp build/variants/libvrt_cp$n.so voxelraytrace20190722_amd/libvrt.so")
    steps+=("tr_${n}_$r|200|$B")
  done
done
for n in 3 5 6; do
  steps+=("swt_$n|20|cp build/variants/libvrt_cp$n.so voxelraytrace20190722_amd/libvrt.so")
  steps+=("test_$n|300|$T")
done
steps+=("back|20|cp build/libvrt_head.so voxelraytrace20190722_amd/libvrt.so")
bash tools/gpu_steps.sh "${steps[@]}"
