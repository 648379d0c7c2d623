#!/bin/bash
# Round-6 call: experiment set R (the fast-only pixel-centre primary pass,
# tools/exp_r6r.sh), the in-tree library restored, then the round's
# measurement set of HEAD (tools/collect.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=voxelraytrace20190722_amd/libvrt.so
cp $L build/ab/libvrt_head.so
bash tools/exp_r6r.sh
rc=$?
cp build/ab/libvrt_head.so $L
[ $rc -ge 124 ] && exit $rc
bash tools/collect.sh
