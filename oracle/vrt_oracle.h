/*
 * vrt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, gcc -O2 -ffp-contract=off, x86-64 SSE, no FMA)
 * of jqly/VoxelRayTrace20190722's primary-ray hot path, used as the parity
 * checker for the HIP product path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library
 * (libvrt.so) never links, loads or calls anything in oracle/.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - ora_intersect_triangle3 / ora_tri_box_overlap are pinned bit-exactly
 *     against the reference's own raytri.cc / tribox2.cc compiled unmodified
 *     from /root/reference into oracle/_ref (tests/golden/kat_*.npz).
 *   - The HDR writer is checked against the reference's stb_image_write.h
 *     compiled unmodified into oracle/_ref (tests/golden/hdr_*.npz).
 *   - Camera / AABB / octree build / traversal / shading depend on
 *     graphics_math.h, which this image's g++/libstdc++ cannot compile without
 *     editing the reference source (MSVC-only token pasting,
 *     graphics_math.h:264-319) and supplying C++17 std:: math names
 *     libstdc++ 11 lacks (graphics_math.h:579,1037).  Those functions are
 *     therefore a cited restatement whose end-to-end parity is
 *     "parity unpinned" against a running reference; their floating-point
 *     leaves (MT, SAT) are pinned as above.
 *
 * Citations: VRT/x = /root/reference/VoxelRayTrace20190722/x
 */
#ifndef VRT_ORACLE_H
#define VRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_scene ora_scene;

/* VRT/raytri.cc:197-249 */
int ora_intersect_triangle3(const double orig[3], const double dir[3],
                            const double vert0[3], const double vert1[3],
                            const double vert2[3], double *t, double *u,
                            double *v);
/* VRT/tribox2.cc:122-196 */
int ora_tri_box_overlap(const float boxcenter[3], const float boxhalfsize[3],
                        const float triverts[9]);

/* Camera: VRT/camera.cc:65-75.  cam_out[16] = column-major C_ (4x4),
 * cam_out[16] = near, cam_out[17] = far, cam_out[18] = fov. */
void ora_camera_init(float fov, const float eye[3], const float spot[3],
                     const float up[3], float near_, float far_,
                     float cam_out[19]);
/* VRT/camera.cc:95-112 (gen_rays4) / :77-93 (gen_rays1).
 * rays_out: n x {ox,oy,oz,dx,dy,dz,tmin,tmax}.  Returns ray count. */
int ora_gen_rays4(const float cam[19], float film_w, float film_h, int nx,
                  int ny, int px, int py, float rays_out[32]);
int ora_gen_rays1(const float cam[19], float film_w, float film_h, int nx,
                  int ny, int px, int py, float rays_out[8]);
/* jql::Ray ctor: VRT/graphics_math.h:1159-1166 (normalises d). */
void ora_make_ray(const float o[3], const float d[3], float tmin, float tmax,
                  float ray_out[8]);
/* AABB3D::isect(ray, nullptr): VRT/graphics_math.h:1312-1332 */
int ora_aabb_isect(const float box[6], const float ray[8]);

/* travorder's std::sort of the 8 (ci, dist) Items and ray_march_isect's
 * std::min_element, on arbitrary inputs (VRT/voxel_octree.cc:91-93,122-125) */
void ora_sort8(const float dist[8], int ord[8]);
int ora_first_min(const float *depth, int n);

/* Scene: triangles as built by Triangle::Triangle (VRT/voxel_octree.cc:423-431).
 * pos: ntri*9, nrm: ntri*9 (raw, normalised here like the ctor), uv: ntri*6,
 * mat: ntri material ids.  Materials: mat_tex[m] = texture id or -1 (then
 * mat_kd[3m..] is used, VRT/voxel_octree.cc:474-477).  Textures: tex_dims
 * ntex*3 {w,h,channels}, tex_off byte offsets into tex_data. */
ora_scene *ora_scene_create(const float *pos, const float *nrm,
                            const float *uv, const int32_t *mat, int ntri,
                            int max_depth);
void ora_scene_set_materials(ora_scene *s, int nmat, const int32_t *mat_tex,
                             const float *mat_kd, int ntex,
                             const int32_t *tex_dims, const int64_t *tex_off,
                             const uint8_t *tex_data, int64_t tex_bytes);
void ora_scene_destroy(ora_scene *s);
/* info[0]=nodes [1]=internal [2]=leaves(all) [3]=nonempty leaves [4]=refs */
void ora_scene_info(const ora_scene *s, int64_t info[5], float root_box[6]);
/* Non-empty leaves sorted by voxel key (ix | iy<<10 | iz<<20 at max depth):
 * vox[nl], cnt[nl], tris[refs] (concatenated lists, input order). */
void ora_scene_leaves(const ora_scene *s, uint32_t *vox, uint32_t *cnt,
                      int32_t *tris);

/* gi::ray_march (VRT/voxel_octree.cc:131-188) over n rays {o,d,tmin,tmax}.
 * Outputs (any may be NULL): hit[n], tri[n], vox[n], hitp[3n], nrm[3n],
 * cnt[4n] = {A aabb tests, L leaves entered, T tri tests, H hit}. */
void ora_ray_march(const ora_scene *s, const float *rays, int n, int32_t *hit,
                   int32_t *tri, uint32_t *vox, float *hitp, float *nrm,
                   uint32_t *cnt);
/* One primary sample's colour: hit -> Triangle::get_diffuse(isect, ray,
 * (1,1,1)) (VRT/voxel_octree.cc:462-484); miss -> sky (VRT/main.cc:18-20). */
void ora_shade(const ora_scene *s, const float *rays, int n, float *rgb_out);

/* Primary render (VRT/main.cc:112-123 with the light-map-pass shading of
 * VRT/main.cc:86-90): render_mt tiles (VRT/camera.h:42-68), gen_rays4, per
 * sample ray_march + get_diffuse / sky, Film::add(c*.25f).
 * film_index: 0 = reference index y*ny+x (VRT/camera.cc:17-20; only valid
 * when in bounds), 1 = y*nx+x.  rgb: nx*ny*3 (zero-initialised here).
 * Per-sample outputs (may be NULL), indexed ((py*nx+px)*4+s):
 * s_hit, s_tri, s_vox, s_rgb[3], s_cnt[4].  nthreads>=1. */
void ora_render(const ora_scene *s, const float cam[19], float film_w,
                float film_h, int nx, int ny, int film_index, int nthreads,
                float *rgb, int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox,
                float *s_rgb, uint32_t *s_cnt);
/* Same (film index y*nx+x), restricted to the rows py % row_stride ==
 * row_phase and without per-sample outputs: the bounded CPU-baseline sample.
 * Returns wall seconds. rgb is accumulated into (caller zeroes it). */
double ora_render_rows(const ora_scene *s, const float cam[19], float film_w,
                       float film_h, int nx, int ny, int row_stride,
                       int row_phase, int nthreads, float *rgb);

/* One render_mt task (VRT/camera.h:50-60): pixels [x0,x1) x [y0,y1), rows
 * then columns, film index y*nx+x, accumulated into rgb (nx*ny*3). */
void ora_render_tile(const ora_scene *s, const float cam[19], float film_w,
                     float film_h, int nx, int ny, int x0, int y0, int x1,
                     int y1, float *rgb);

/* jql::PCG (VRT/graphics_math.h:821-857): one operator() call. */
uint32_t ora_pcg_next(uint64_t *state);
/* std::uniform_real_distribution<float>{-1, 1}(pcg) as libstdc++ 11 does it
 * (generate_canonical<float,24>: one draw, float(g)/2^32 clamped below 1,
 * then u*(b-a)+a; /usr/include/c++/11/bits/random.tcc:3348-3380,
 * random.h:1868-1870). */
float ora_uniform_m11(uint64_t *state);
/* jql::random_point_in_unit_sphere (VRT/graphics_math.h:1208-1216). */
void ora_random_point_in_unit_sphere(uint64_t *state, float p[3]);
/* SURVEY §8(d) config 5 ("64 spp stochastic secondary rays"), over the
 * 8*(n/8) render area: primary = gen_rays1 (pixel centre); on a hit, PCG
 * seeded 0xc01dbeef ^ (py*nx+px) draws `spp` points p, secondary ray =
 * Ray{isect.hit, isect.normal + p, res, FLT_MAX} (the ctor normalises; the
 * pattern of VRT/voxel_octree.cc:600-603); vis[py*nx+px] = misses / spp
 * (1 for a primary miss, 0 outside the render area).  res = min component
 * of root.size() / 2^max_depth (VRT/main.cc:69-70).  Optional per-ray
 * outputs (index (py*nx+px)*spp + s): s_hit, s_tri, s_vox (unused slots
 * -1 / 0xFFFFFFFF).  Returns the number of rays traced. */
int64_t ora_render_secondary(const ora_scene *s, const float cam[19],
                             float film_w, float film_h, int nx, int ny,
                             int spp, int nthreads, float *vis,
                             int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox);

/* ---- full trace() ------------------------------------
 * Light pass (VRT/main.cc:79-97): render_mt over the light film with
 * gen_rays4; every hit adds clamp(dot(illum_d[i], n), 0, 1) * get_diffuse
 * to leaf_ptr->illum[i].  The reference's += is racy across its thread
 * pool; here the sums run in the canonical single-threaded order (task
 * t = tx*8+ty, pixels row-major, samples 0..3).  Returns the hit count. */
int64_t ora_lightmap(ora_scene *s, const float cam[19], float film_w,
                     float film_h, int nx, int ny, int nthreads);
/* cone_trace_init_filter (VRT/voxel_octree.cc:190-214). */
void ora_lightmap_filter(ora_scene *s);
/* Per node (oracle order): key = depth<<32 | ix | iy<<10 | iz<<20 at its
 * depth, coverage, illum[6][3]. */
void ora_lightmap_nodes(const ora_scene *s, uint64_t *key, float *cov,
                        float *illum);
/* min component of root.size() / powf(2, levels) (VRT/main.cc:69-70). */
float ora_min_voxel(const ora_scene *s, int levels);
/* trace(root, ray, 5, true) per ray (VRT/main.cc:10-30): sky on a miss,
 * else get_albedo * (cone_trace(root, isect, res) + leaf compute_illum(-d)). */
void ora_shade_trace(const ora_scene *s, const float *rays, int n, float res,
                     float *rgb);
/* The cone-tracing render (VRT/main.cc:114-123): rgb nx*ny*3 (index
 * y*nx+x), optional per-sample s_hit / s_rgb ((py*nx+px)*4+s). */
void ora_render_trace(const ora_scene *s, const float cam[19], float film_w,
                      float film_h, int nx, int ny, float res, int nthreads,
                      float *rgb, int32_t *s_hit, float *s_rgb);

/* stbiw__linear_to_rgbe (VRT/stb_image_write.h:601-616) for one pixel. */
void ora_linear_to_rgbe(const float linear[3], uint8_t rgbe[4]);

#ifdef __cplusplus
}
#endif
#endif
