cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=voxelraytrace20190722_amd/libvrt.so
bash tools/gpu_steps.sh \
 "ab_s8g|400|python -u tools/ab.py $L build/ab/libvrt_g8.so build/ab/libvrt_g16.so build/ab/libvrt_g2.so --share-ranks 8 --share-of 0,1,2,3,4,5,6,7 --rounds 5 --steps 64"
