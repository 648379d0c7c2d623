/* vrt_legacy.hpp -- the reference's two primitive declarations, C++ linkage.
 *
 * Identical to VRT/raytri.h:5-7 and VRT/tribox2.h:6 (which a reference
 * build may keep including instead): libvrt.so defines these two functions
 * under their C++ (mangled) names, so VRT/voxel_octree.cc:446,490 link
 * against the library unchanged once raytri.cc / tribox2.cc are dropped.
 *
 * The same functions are also exported with C linkage, declared in vrt.h
 * (for C and ctypes callers).  A C++ translation unit includes one of the
 * two headers, not both: C++ does not allow one signature under both
 * linkages in the same scope.
 */
#ifndef VRT_LEGACY_HPP
#define VRT_LEGACY_HPP

#ifndef __cplusplus
#error "vrt_legacy.hpp declares C++-linkage functions; C callers include vrt.h"
#endif

int intersect_triangle3(double orig[3], double dir[3], double vert0[3],
                        double vert1[3], double vert2[3], double *t, double *u,
                        double *v);

int triBoxOverlap(float boxcenter[3], float boxhalfsize[3], float triverts[3][3]);

#endif /* VRT_LEGACY_HPP */
