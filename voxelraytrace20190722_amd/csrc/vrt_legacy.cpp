// vrt_legacy.cpp -- the reference's two geometric primitives with the
// reference's own (C++) linkage.
//
// VRT/raytri.h:5-7 and VRT/tribox2.h:6 declare
//     int intersect_triangle3(double[3], double[3], double[3], double[3],
//                             double[3], double*, double*, double*);
//     int triBoxOverlap(float[3], float[3], float[3][3]);
// as plain C++ functions (no extern "C"), so the reference's caller
// VRT/voxel_octree.cc:446,490 imports the mangled names
//     _Z19intersect_triangle3PdS_S_S_S_S_S_S_
//     _Z13triBoxOverlapPfS_PA3_f
// This translation unit defines exactly those, forwarding to the code the
// kernels inline (vrt_math.h).  It must not include include/vrt.h: that
// header declares the same names with C linkage (the unmangled exports a C
// or ctypes caller binds, defined in vrt_host.cpp), and C++ forbids both
// linkages for one signature in one translation unit.  C++ callers who want
// a header use include/vrt_legacy.hpp (the reference's two declarations).
//
// VRT/x = /root/reference/VoxelRayTrace20190722/x
#include "vrt_math.h"

#define VRT_EXPORT __attribute__((visibility("default")))

VRT_EXPORT int intersect_triangle3(double orig[3], double dir[3],
                                   double vert0[3], double vert1[3],
                                   double vert2[3], double *t, double *u,
                                   double *v)
{
        return vrt::mt_isect(orig, dir, vert0, vert1, vert2, t, u, v);
}

VRT_EXPORT int triBoxOverlap(float boxcenter[3], float boxhalfsize[3],
                             float triverts[3][3])
{
        return vrt::tri_box_overlap(boxcenter, boxhalfsize, &triverts[0][0]);
}
