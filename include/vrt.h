/*
 * vrt.h -- C ABI of the MI355X-native voxel-octree ray-march hot path
 * (drop-in for jqly/VoxelRayTrace20190722's per-pixel primary-ray loop).
 *
 * libvrt.so (voxelraytrace20190722_amd/libvrt.so) exports exactly the symbols
 * below.  Conventions: plain pointers and sizes, caller-owned outputs, opaque
 * handles, int status codes (VRT_OK = 0, negative = error; the legacy
 * symbols keep the reference's 1/0 returns), no exceptions or exit() across
 * the ABI.  Reference citations: VRT/x = VoxelRayTrace20190722/x.
 */
#ifndef VRT_H
#define VRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

#define VRT_OK 0
#define VRT_E_INVALID (-1)  /* bad argument (NULL, size, depth, id range) */
#define VRT_E_NOMEM (-2)    /* host allocation failed */
#define VRT_E_DEVICE (-3)   /* HIP runtime error (see vrt_last_error) */
#define VRT_E_NODEVICE (-4) /* no usable gfx950 device */
#define VRT_E_IO (-5)       /* file could not be opened / written */

#define VRT_MAX_DEPTH 11    /* voxel ids pack 10 bits per axis */

typedef struct vrt_scene vrt_scene;

/* Triangle soup in obj2voxel's output order (VRT/voxel_octree.cc:305-371);
 * triangle i is gi::Triangle{p0,p1,p2,n0,n1,n2,t0,t1,t2,mtl}
 * (VRT/voxel_octree.h:94-113).  Normals are normalised by the build exactly
 * like Triangle::Triangle (VRT/voxel_octree.cc:426). */
typedef struct {
        int32_t ntri;
        const float *pos;      /* ntri*9 */
        const float *nrm;      /* ntri*9 */
        const float *uv;       /* ntri*6, NULL = all zero (texcoord_index -1) */
        const int32_t *mat;    /* ntri,   NULL = all material 0 */
        int32_t nmat;          /* >= 1 */
        const int32_t *mat_tex;/* nmat texture ids, -1 = untextured (Kd) */
        const float *mat_kd;   /* nmat*3 tinyobj material_t::diffuse */
        int32_t ntex;
        const int32_t *tex_dims;  /* ntex*3 {width, height, channels 1..4} */
        const int64_t *tex_off;   /* ntex byte offsets into tex_data */
        const uint8_t *tex_data;  /* stbi_load(...,0) bytes, row 0 = top */
        int64_t tex_bytes;
} vrt_scene_desc;

/* jql::Ray after construction (VRT/graphics_math.h:1150-1167): d is already
 * normalised; tmin/tmax bound AABB3D::isect (VRT/graphics_math.h:1312). */
typedef struct {
        float o[3];
        float d[3];
        float tmin, tmax;
} vrt_ray;

/* Camera (VRT/camera.h:70-84): C = affine_transform(Mat3{s,up_,-fwd}, eye),
 * column-major.  `origin` = point_transform(C,{}) is cached; the film plane
 * z = -(film.h / (2*tanf(fov/2))) is evaluated on the host per film. */
typedef struct {
        float C[16];
        float fov, near_, far_;
        float origin[3];
} vrt_camera;

/* Film (VRT/camera.h:24-39): physical w,h and pixel counts nx,ny. */
typedef struct {
        float w, h;
        int32_t nx, ny;
} vrt_film;

/* One gi::ray_march result (VRT/voxel_octree.h:87-89). */
typedef struct {
        int32_t hit;      /* 1 = ray_march returned true */
        int32_t tri;      /* index of *voxel_ptr in the input soup, -1 */
        uint32_t voxel;   /* *leaf_ptr's integer coords at max depth:
                             ix | iy<<10 | iz<<20, 0xFFFFFFFF on a miss */
        float hit_p[3];   /* ISect::hit */
        float normal[3];  /* ISect::normal */
} vrt_hit;

typedef struct {
        int64_t nodes, internal, leaves, nonempty_leaves, tri_refs;
        int32_t max_depth, device;
        float root_min[3], root_max[3];
        int64_t device_bytes;
        double build_ms, upload_ms;
        double build_device_ms;  /* GPU part of a VRT_BUILD_DEVICE build, else 0 */
} vrt_scene_info_t;

/* Optional per-sample outputs of vrt_render (host arrays, index
 * ((py*nx+px)*4 + s), s = gen_rays4 sample order).  Any pointer may be NULL.
 * counters = {A aabb tests, L leaves entered, T triangle tests, H hit} as
 * the reference's ray_march performs them; requesting them
 * selects the instrumented kernel variant. */
typedef struct {
        int32_t *hit;
        int32_t *tri;
        uint32_t *voxel;
        float *rgb;       /* 3 per sample: get_diffuse / sky colour */
        uint32_t *counters;
} vrt_samples;

/* Aggregate counters of one instrumented render (sums over all samples). */
typedef struct {
        uint64_t rays, aabb_tests, leaves, tri_tests, hits;
        double kernel_ms;
} vrt_stats;

/* ---- device / scene ------------------------------------------------- */
int vrt_device_count(int *n);
/* gi::ray_march_init (VRT/voxel_octree.cc:67-75) on the host, then upload
 * of the flattened octree + triangles + textures to `device`.  device < 0
 * builds a host-only scene (info / leaves only; device calls then return
 * VRT_E_NODEVICE). */
int vrt_scene_create(const vrt_scene_desc *desc, int max_depth, int device,
                     vrt_scene **out);
/* Same, with build flags: VRT_BUILD_DEVICE runs the octree build on the GPU
 * (level-synchronous SAT descent + hipCUB sorts + BFS flatten, SURVEY §8
 * f3); the octree is identical to the host build.  Needs device >= 0. */
#define VRT_BUILD_DEVICE 1
int vrt_scene_create_ex(const vrt_scene_desc *desc, int max_depth, int device,
                        int flags, vrt_scene **out);
void vrt_scene_destroy(vrt_scene *s);
int vrt_scene_info(const vrt_scene *s, vrt_scene_info_t *info);
/* Non-empty leaves sorted by voxel id; tris = concatenated leaf lists in
 * insertion (input) order.  Sizes from vrt_scene_info. */
int vrt_scene_leaves(const vrt_scene *s, uint32_t *voxel, uint32_t *count,
                     int32_t *tris);
/* The flattened octree, nodes entries each: box (min xyz,
 * max xyz), word a (first child | 0x80000000 + count for leaves), word b
 * (content mask | first leaf record).  Any output may be NULL. */
int vrt_scene_nodes(const vrt_scene *s, float *box, uint32_t *a, uint32_t *b);

/* ---- camera (host, VRT/camera.cc) ------------------------------------ */
int vrt_camera_init(float fov, const float eye[3], const float spot[3],
                    const float up[3], float near_, float far_,
                    vrt_camera *out);
int vrt_gen_rays4(const vrt_camera *cam, const vrt_film *film, int px, int py,
                  vrt_ray out[4]);
int vrt_gen_rays1(const vrt_camera *cam, const vrt_film *film, int px, int py,
                  vrt_ray out[1]);
/* jql::Ray::Ray(o, d, tmin, tmax): normalises d. */
int vrt_make_ray(const float o[3], const float d[3], float tmin, float tmax,
                 vrt_ray *out);
/* AABB3D::isect(ray, nullptr) on the host (box = min xyz, max xyz). */
int vrt_aabb_isect(const float box[6], const vrt_ray *ray);
/* *bound = an upper bound on the gen_rays4 rays of the film with a direction
 * component |d_q| < 2^-64 (an exact zero included): the rays the fast-only
 * persistent render defers to its exact pass.  0 certifies that the frame
 * needs no deferred pass (it is then not launched); INT64_MAX when a camera
 * term is not finite.  Never below the true count. */
int vrt_camera_defer_bound(const vrt_camera *cam, const vrt_film *film, int64_t *bound);

/* ---- the hot path ------------------------------------------------------ */
/* Primary render = the per-pixel loop of VRT/main.cc:118-123 with the
 * primary shading contract (hit: Triangle::get_diffuse(isect, ray, (1,1,1));
 * miss: sky lerp, VRT/main.cc:18-20), 4 gen_rays4 samples accumulated with
 * Film::add(c * .25f).  Pixels outside render_mt's 8x8 tile grid
 * (px >= 8*(nx/8) or py >= 8*(ny/8), VRT/camera.h:45-61) stay 0.
 * Film index is y*nx+x (the reference's y*ny+x, VRT/camera.cc:19, agrees for
 * square films).  rgb: host nx*ny*3 floats.  samples / stats may be NULL. */
int vrt_render(vrt_scene *s, const vrt_camera *cam, const vrt_film *film,
               float *rgb, const vrt_samples *samples, vrt_stats *stats);

/* Device-resident variant (inputs/outputs in HBM, enqueued on `stream`, a
 * hipStream_t or NULL for the null stream; no host synchronisation).
 * Screen = the ntx x nty grid of 8x8-pixel tiles (ntx = nx/8, nty = ny/8).
 * The tile deal (one rule for every multi-rank entry point): with
 * G = vrt_tile_deal_block() (G = 1 when nranks == 1), the whole G x G blocks
 * of tiles are dealt round-robin in block raster order (block j -> rank
 * j % nranks; from 2 ranks on rank 0, which also gathers and re-assembles,
 * is dealt (m-1)/m of a share, m = max(2, 48/nranks): block j -> rank
 * nranks-1 - (j % V) % nranks with V = m*nranks - 1, a rank's blocks in
 * raster order); the tiles outside the whole-block region -- the right strip
 * (rows ty < G*(nty/G), columns tx >= G*(ntx/G)), then the bottom strip, each
 * in raster order -- continue the deal one tile at a time (leftover i ->
 * rank (F + i) % nranks, F = number of whole blocks).  A rank's k-th tile:
 * its blocks' tiles first (block order, row-major inside a block), then its
 * leftover tiles.  This call renders this rank's tiles into d_out packed
 * tile-major: d_out[(k*64 + (y%8)*8 + x%8)*3 + c], sized
 * vrt_tiles_per_rank()*192 floats (the largest share).  rank=0, nranks=1
 * with image_layout=1 writes the nx*ny*3 image directly instead. */
int vrt_tiles_per_rank(const vrt_film *film, int nranks);
/* Launch hint: the caller keeps `n` frames in flight on different streams
 * (n >= 2) or renders one at a time (n = 1, the default).  With n >= 2 a
 * persistent render grid takes half of the resident workgroup slots, so
 * consecutive frames share the chip and one frame's latency-bound ramp-down
 * runs beside the next frame; results are identical either way.  Applies to
 * the device entry points (vrt_render_tiles_device); the synchronous
 * vrt_render always uses the whole chip. */
int vrt_scene_set_frames_in_flight(vrt_scene *s, int n);
int vrt_tile_deal_block(void);
/* The deal as tables (host, no device): for every tile ty*ntx+tx, its rank
 * and its index k in that rank's buffer. */
int vrt_tile_deal_map(const vrt_film *film, int nranks, int32_t *rank_of_tile, int32_t *slot_of_tile);
int vrt_render_tiles_device(vrt_scene *s, const vrt_camera *cam,
                            const vrt_film *film, int rank, int nranks,
                            int image_layout, float *d_out, void *stream);
/* Rank 0 after the gather: d_gathered = nranks * tiles_per_rank * 192 floats
 * (rank-major) -> d_image nx*ny*3 (pixels outside the tile grid zeroed). */
int vrt_unpack_tiles_device(const vrt_film *film, int nranks,
                            const float *d_gathered, float *d_image,
                            void *stream);
/* The same deal for images of `comps` floats per pixel (config 5's
 * visibility image: comps = 1).  Pack: rank `rank`'s tiles of d_image
 * (ny, nx, comps) -> d_packed, tile k at k * 64 * comps, pixels row-major in
 * the tile (tiles_per_rank * 64 * comps floats hold any rank's share).
 * Unpack (rank 0 after the gather): d_gathered = nranks * tiles_per_rank *
 * 64 * comps floats, rank-major -> d_image (zero outside the tile grid). */
int vrt_pack_tiles_c_device(const vrt_film *film, int rank, int nranks, int comps, const float *d_image,
                            float *d_packed, void *stream);
int vrt_unpack_tiles_c_device(const vrt_film *film, int nranks, int comps, const float *d_gathered, float *d_image,
                              void *stream);
/* Device time of the last render kernel enqueued by this thread on `s`
 * (HIP events around the launch, on its stream). */
int vrt_last_kernel_ms(vrt_scene *s, float *ms);

/* SURVEY §8(d) config 5 (stochastic secondary rays, divergent traversal):
 * per pixel of the 8*(n/8) render area a pixel-centre primary ray
 * (gen_rays1); on a hit, jql::PCG seeded 0xc01dbeef ^ (py*nx+px) draws `spp`
 * (1..64) points with jql::random_point_in_unit_sphere (libstdc++'s
 * uniform_real_distribution<float>{-1,1} mapping) and each traces
 * Ray{isect.hit, isect.normal + p, res, FLT_MAX} (VRT/voxel_octree.cc:
 * 600-603 pattern; res = min(root.size()/2^max_depth), VRT/main.cc:69-70).
 * vis[py*nx+px] = misses/spp (1 on a primary miss, 0 outside the area).
 * Per-ray ids (index (py*nx+px)*spp + s) may be NULL; *rays (may be NULL)
 * = rays traced (primary + secondary). */
int vrt_render_secondary(vrt_scene *s, const vrt_camera *cam,
                         const vrt_film *film, int spp, float *vis,
                         int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox,
                         int64_t *rays);
/* Device-resident variant: rank `rank` of `nranks` writes its pixels (its
 * 8x8-pixel tiles of the tile deal, vrt_render_tiles_device) into d_vis (nx*ny floats, caller-zeroed:
 * a sum-reduce over ranks assembles the image exactly); d_prim = scratch of
 * 8*(nx/8)*8*(ny/8)*8 floats. */
int vrt_render_secondary_device(vrt_scene *s, const vrt_camera *cam,
                                const vrt_film *film, int spp, int rank,
                                int nranks, float *d_prim, float *d_vis,
                                void *stream);

/* Batched gi::ray_march (VRT/voxel_octree.cc:131-188) on host arrays. */
int vrt_ray_march_batch(vrt_scene *s, const vrt_ray *rays, int64_t n,
                        vrt_hit *hits);
/* Device-resident variant (d_rays / d_hits in HBM). */
int vrt_ray_march_batch_device(vrt_scene *s, const vrt_ray *d_rays, int64_t n,
                               vrt_hit *d_hits, void *stream);

/* Device copies of the fp64 Moller-Trumbore and fp32 SAT leaves (the exact
 * code the kernels inline), run on n host-array cases for parity tests.
 * mt_in: n*15 doubles {orig,dir,v0,v1,v2}; mt_out: n*4 doubles
 * {ret, t, u, v} (t,u,v = 0 unless ret == 1).  sat_in: n*15 floats
 * {center, half, tri[9]}; sat_out: n ints. */
int vrt_device_selftest(int device, const double *mt_in, double *mt_out,
                        const float *sat_in, int32_t *sat_out, int64_t n);

/* Test hook: process-wide flags read by every later render launch.
 * VRT_TEST_FORCE_DEFER makes the persistent fast-path kernel defer every
 * unit to its exact fallback pass (k_render_defer), so tests can pin that
 * rarely taken path against the oracle.  0 = normal operation. */
#define VRT_TEST_FORCE_DEFER 1
/* VRT_TEST_FAIL_LAUNCH makes every fast-path render launch report a launch
 * failure after its first kernel is enqueued (the error path that must
 * leave the scene's work-queue slot usable by later launches). */
#define VRT_TEST_FAIL_LAUNCH 2
/* VRT_TEST_SPILL_ALL makes config-5's ray compaction stop a wave's rays as
 * soon as one of them has ended (every resume round but the last likewise),
 * so that nearly every secondary ray is saved and resumed at least once. */
#define VRT_TEST_SPILL_ALL 4
/* VRT_TEST_VIRTUAL_RANKS_N(n) (2 <= n <= 16), read by vrt_scene_create_multi:
 * a one-device mask creates n *virtual* ranks on that device -- n scene
 * replicas, n streams, the same per-rank send buffers, gather buffer, tile
 * deal and unpack as n devices -- with the RCCL gather replaced by
 * device-to-device copies of each rank's buffer into its slot of rank 0's
 * receive buffer (ordered like the collective: after the rank's render on
 * its stream, before rank 0's unpack).  RCCL refuses duplicate devices; this
 * runs the n-rank frame on a one-GPU box.  Handles created without it are
 * unaffected. */
#define VRT_TEST_VIRTUAL_RANKS 8
/* VRT_TEST_STREAM_LEFTOVER makes config-5's streaming resume round leave
 * every odd chunk of saved rays to its batch-pool launch (the path a chunk
 * with a degenerate ray takes). */
#define VRT_TEST_STREAM_LEFTOVER 16
/* VRT_TEST_LIGHT_TAIL makes the light pass hand every sample to its tail
 * launch (8 lanes per sample; the path of samples whose walk passes the
 * light pass's triangle-test budget). */
#define VRT_TEST_LIGHT_TAIL 32
/* VRT_TEST_PRIM_TAIL does the same for the primary pass of the cone-traced
 * render (vrt_render_trace*, vrt_trace_frame_device). */
#define VRT_TEST_PRIM_TAIL 64
/* VRT_TEST_SEC_DEFER: config 5's fast-only walk kernel defers every odd
 * pixel of its rank to the exact-walk launch after it (k_secondary_defer),
 * as it does a pixel with a ray off the fast walk. */
#define VRT_TEST_SEC_DEFER 128
#define VRT_TEST_VIRTUAL_RANKS_N(n) (VRT_TEST_VIRTUAL_RANKS | ((n) << 8))
int vrt_set_test_flags(int flags);
/* The current vrt_set_test_flags value (so a caller can restore it). */
int vrt_test_flags(void);

/* Diagnostic: the records appended to each compaction queue (phase A, then
 * resume rounds 1..3; with the one streaming resume round only queue 0 is
 * used) by the scene's last config-5 launch; waits for it.  All 0 when that
 * launch used no compaction. */
int vrt_secondary_spill_counts(vrt_scene *s, int64_t counts[4]);
/* Diagnostic: the scene's last config-5 launch's compaction, waits for it:
 * stats[0] records queued, [1] stopped rays finished in place because the
 * queue was full, [2] queue chunks taken, [3] chunks allocated, [4] chunks
 * left to the batch-pool launch after the streaming round, [5] bytes per
 * record, [6] pixels deferred from the fast-only walk kernel to the exact
 * walk (a ray with a zero or tiny direction component).  All 0 when that
 * launch used no compaction. */
int vrt_secondary_spill_stats(vrt_scene *s, int64_t stats[7]);
/* Device bytes the scene holds beyond its octree, triangles and textures
 * (vrt_scene_info().device_bytes): per-call scratch kept between calls --
 * config 5's compaction queues (*spill_bytes, may be NULL), the light-map
 * build's scratch and light-map sets, the trace records, the host-output
 * image, the tabled tile deals of multi-rank calls (4 B per tile of the
 * rank). */
int vrt_scene_scratch_bytes(vrt_scene *s, int64_t *bytes, int64_t *spill_bytes);

/* The kernels' own travorder sort (std::sort of the 8 Items by dist,
 * VRT/voxel_octree.cc:77-97) and ray_march_isect min_element
 * (VRT/voxel_octree.cc:122-125) on arbitrary inputs, for the pin against
 * the real libstdc++ (tests/golden/travorder_std.cpp).  Per case i:
 * dist[8i..8i+7] and hit_mask[i] (bit ci = child ci's slab test passed) ->
 * orders[6i..6i+5] = {full insertion-sort order (3-bit fields), exact-path
 * hit order | count << 24, rank order | count << 24, two-slot order,
 * 4-slot network order, full-position word} (the last four are the
 * NaN-free fast paths).  Per record list j: depth[j*stride .. +len[j]) ->
 * argmin[j] (the first minimum, -1 when empty). */
int vrt_device_selftest_order(int device, const float *dist,
                              const uint32_t *hit_mask, int64_t n,
                              uint32_t *orders, const float *depth,
                              const int32_t *len, int64_t m, int32_t stride,
                              int32_t *argmin);

/* ---- multi-device frame (render_mt, VRT/camera.h:42-68,
 * over the GPUs of one node) --------------------------------------------------
 * One handle for the scene replicated on every device of `device_mask` (bit d
 * = HIP device d; rank i = the i-th set bit, rank 0 = the lowest device, which
 * receives and re-assembles the frame) and an RCCL communicator over them
 * (ncclCommInitAll; RCCL is linked into libvrt.so).  The octree is built once
 * on the host (or on the first device with VRT_BUILD_DEVICE) and uploaded to
 * every device.  A frame: rank i renders its tiles of the tile deal
 * (vrt_render_tiles_device with rank i of n) on its device's stream, one
 * ncclGather of the packed tile buffers to rank 0 over xGMI (rank 0's share
 * rendered in place into the receive buffer), then vrt_unpack_tiles_device
 * on rank 0.  Pixels are the single-device render's, bit for bit. */
typedef struct vrt_multi vrt_multi;
int vrt_scene_create_multi(const vrt_scene_desc *desc, int max_depth,
                           uint32_t device_mask, int flags, vrt_multi **out);
void vrt_multi_destroy(vrt_multi *m);
/* devices[i] = rank i's HIP device (n entries, n = set bits of the mask). */
int vrt_multi_devices(const vrt_multi *m, int *n, int32_t *devices);
/* Rank i's scene (borrowed, owned by m): info, single-device entry points. */
int vrt_multi_scene(vrt_multi *m, int rank, vrt_scene **out);
/* The whole frame into a host nx*ny*3 array (index y*nx+x, as vrt_render). */
int vrt_render_multi(vrt_multi *m, const vrt_camera *cam,
                     const vrt_film *film, float *rgb);
/* The whole frame into d_image (nx*ny*3 floats on rank 0's device), ordered
 * after the work already queued on `stream` (a hipStream_t of rank 0's
 * device); work queued on `stream` afterwards sees the image.  stream = NULL:
 * the call returns when the image is complete.  The ranks' renders and the
 * gather run on streams owned by m. */
int vrt_render_multi_device(vrt_multi *m, const vrt_camera *cam,
                            const vrt_film *film, float *d_image,
                            void *stream);
/* The deal of a frame over the devices of a mask (host, no device): per
 * tile ty*ntx+tx, its device and its index in that device's buffer. */
int vrt_multi_tile_map(const vrt_film *film, uint32_t device_mask,
                       int32_t *device_of_tile, int32_t *slot_of_tile);

/* ---- full trace() (VRT/main.cc:10-30, 79-123) -------
 * The reference's actual image: a light pass from a light camera
 * (render_mt + gen_rays4; every hit adds clamp(dot(illum_d[i], n), 0, 1) *
 * get_diffuse to leaf->illum[i]), cone_trace_init_filter, then per camera
 * sample trace(root, ray, 5, true) = sky on a miss, else get_albedo *
 * (6-cone cone_trace + leaf compute_illum(-d)), accumulated with
 * Film::add(c * .25f).  The reference's light-map += races across threads;
 * here the per-leaf sums run in the canonical single-threaded order (task
 * t = tx*8+ty, pixels row-major, samples 0..3), so results are
 * deterministic and bit-identical to the oracle's single-threaded order.
 *
 * vrt_lightmap_build: light pass + filter on the scene's device (blocking);
 * hits (may be NULL) = light samples that hit.  A new build replaces the
 * previous light map. */
int vrt_lightmap_build(vrt_scene *s, const vrt_camera *light_cam,
                       const vrt_film *light_film, int64_t *hits);
/* Per node (vrt_scene_info().nodes entries, BFS order): key = depth << 32 |
 * ix | iy<<10 | iz<<20 (coords at that depth), VoxelOctree::coverage and
 * illum[6][3].  coverage / illum may be NULL. */
int vrt_lightmap_nodes(vrt_scene *s, uint64_t *key, float *coverage,
                       float *illum);
/* min component of root.size() / powf(2, levels) -- the reference's Res
 * (VRT/main.cc:69-70); levels <= 0 uses the scene's max_depth. */
int vrt_scene_min_voxel(const vrt_scene *s, int levels, float *res);
/* Cone-tracing render with min_voxel_size = min_voxel (<= 0: the scene's
 * Res).  rgb: host nx*ny*3 (index y*nx+x); s_hit / s_rgb optional
 * per-sample outputs ((py*nx+px)*4+s). */
int vrt_render_trace(vrt_scene *s, const vrt_camera *cam, const vrt_film *film,
                     float min_voxel, float *rgb, int32_t *s_hit,
                     float *s_rgb);
/* Device-resident variant with the tile partition of
 * vrt_render_tiles_device. */
int vrt_render_trace_device(vrt_scene *s, const vrt_camera *cam,
                            const vrt_film *film, float min_voxel, int rank,
                            int nranks, int image_layout, float *d_out,
                            void *stream);

/* The whole reference main() frame (VRT/main.cc:75-126) in one call: the
 * light pass + cone_trace_init_filter (as vrt_lightmap_build, on the scene's
 * stream) and, beside them on `stream`, the view's primary march, which reads
 * no light map; the cone-traced shading then waits for the filter.  Values
 * equal vrt_lightmap_build followed by vrt_render_trace_device (same tile
 * deal / layout arguments).  Returns after one host sync (the light pass's
 * hit count, *hits, may be NULL); the image is complete in stream order. */
int vrt_trace_frame_device(vrt_scene *s, const vrt_camera *light_cam,
                           const vrt_film *light_film, const vrt_camera *cam,
                           const vrt_film *film, float min_voxel, int rank,
                           int nranks, int image_layout, float *d_out,
                           void *stream, int64_t *hits);

/* ---- output (VRT/stb_image_write.h:178,723-757) ------------------------- */
/* Byte-identical to stbi_write_hdr: returns 1 on success, 0 on failure. */
int vrt_write_hdr(const char *filename, int w, int h, int comp,
                  const float *data);
/* Same bytes into memory: returns the byte count, or -(needed) if cap is
 * too small, or 0 on invalid input. */
int64_t vrt_write_hdr_mem(int w, int h, int comp, const float *data,
                          uint8_t *out, int64_t cap);

/* Device half of the writer: stbiw__linear_to_rgbe for every pixel of a
 * device image (w*h*comp floats) into w*h*4 device bytes on `stream`; then
 * vrt_write_hdr_rgbe[_mem] RLE-encodes those bytes on the host.  The file is
 * byte-identical to vrt_write_hdr / stbi_write_hdr on the same pixels. */
int vrt_rgbe_device(const float *d_img, int w, int h, int comp,
                    uint8_t *d_rgbe, void *stream);
int vrt_write_hdr_rgbe(const char *filename, int w, int h,
                       const uint8_t *rgbe);
int64_t vrt_write_hdr_rgbe_mem(int w, int h, const uint8_t *rgbe,
                               uint8_t *out, int64_t cap);

/* ---- legacy reference symbols (identical signatures and results) ------- */
/* C linkage here; the library also defines the same two functions with the
 * reference headers' C++ linkage (declared in vrt_legacy.hpp), the names
 * VRT/voxel_octree.cc:446,490 import. */
/* VRT/raytri.h:5-7 */
int intersect_triangle3(double orig[3], double dir[3], double vert0[3],
                        double vert1[3], double vert2[3], double *t,
                        double *u, double *v);
/* VRT/tribox2.h:6 */
int triBoxOverlap(float boxcenter[3], float boxhalfsize[3],
                  float triverts[3][3]);
/* VRT/stb_image_write.h:178 (stb_image_write v1.13, called at VRT/main.cc:126):
 * the same function as vrt_write_hdr, under the reference's name, so a
 * caller of the reference's writer relinks without renaming the call. */
int stbi_write_hdr(char const *filename, int w, int h, int comp,
                   const float *data);

/* ---- build identity ---------------------------------------------------- */
/* Source hash this library was built from (tools/build_id.py: sha256 of
 * csrc/, include/vrt.h and the Makefile, 16 hex digits). */
const char *vrt_build_id(void);
/* The value of one path-selecting compile-time switch of this build (e.g.
 * "VRT_SEC_SPILL_T": config 5's compaction threshold, 0 = no compaction;
 * "VRT_SEC_SLICE_CHUNK", "VRT_SLICE_CHUNK": the persistent kernels' slice
 * chunks; "VRT_SEC_TAKE": config-5 pixels per dequeue; "VRT_DEAL_BLOCK" / "VRT_DEAL_WEIGHT" / "VRT_DEAL_SPAN": the tile
 * deal; "VRT_LIGHT_BUDGET" / "VRT_PRIM_BUDGET": the trace walks' budgets);
 * VRT_E_INVALID for a name the build does not know.  Lets a test assert which
 * path a build takes. */
int vrt_build_flag(const char *name, int64_t *value);

/* ---- scene ingest (VRT/voxel_octree.cc:305-388) -------------------------
 * vrt_obj_load = obj2voxel(path) + load_image for every texture a face
 * uses: tinyobjloader v1.4.0 LoadObj(.., path, mtldir = dir(path) + "/",
 * triangulate = true) restated bit-exactly (its non-correctly-rounded float
 * parser and ear-clipping triangulation included), then one triangle per
 * (shape, face) in shape order.  Textures are decoded like stbi_load(path,
 * .., 0) (TGA only).  Faces without normals or with out-of-range indices
 * are errors; faces without a material get an extra default material (Kd
 * 0) appended after the file's materials.  VRT_OBJ_PARSE_ONLY stops after
 * LoadObj (no soup, no textures; no normal requirement). */
#define VRT_OBJ_PARSE_ONLY 1

typedef struct vrt_obj vrt_obj;
typedef struct {
        int64_t nvert, nnormal, ntexcoord; /* attrib_t sizes / 3, / 3, / 2 */
        int32_t nshape;                    /* shapes.size() */
        int64_t nface;                     /* triangles over all shapes */
        int32_t nmat;                      /* materials.size() (MTL order) */
        int32_t has_soup;                  /* 0 with VRT_OBJ_PARSE_ONLY */
        int32_t nsoup_mat;                 /* nmat (+1 if a default was added) */
        int32_t ntex;
        int64_t tex_bytes;
} vrt_obj_info_t;

int vrt_obj_load(const char *obj_path, int flags, vrt_obj **out);
void vrt_obj_free(vrt_obj *o);
int vrt_obj_info(const vrt_obj *o, vrt_obj_info_t *info);
/* Borrowed views, valid until vrt_obj_free: attrib_t::vertices / normals /
 * texcoords. */
int vrt_obj_attrib(const vrt_obj *o, const float **v, const float **vn,
                   const float **vt);
/* Per triangle (shape order): idx[9] = {v, vn, vt} x 3 (0-based, -1 =
 * absent), tinyobj material id (-1 = none) and shape index.  Any output may
 * be NULL; sizes from vrt_obj_info().nface. */
int vrt_obj_faces(const vrt_obj *o, int32_t *idx, int32_t *mat,
                  int32_t *shape);
/* material_t i: name, diffuse (Kd), diffuse_texname (as in the MTL). */
int vrt_obj_material(const vrt_obj *o, int i, const char **name, float kd[3],
                     const char **texname);
/* Resolved file of soup texture i (mtldir + diffuse_texname). */
int vrt_obj_texture_path(const vrt_obj *o, int i, const char **path);
const char *vrt_obj_warnings(const vrt_obj *o);
/* The soup as a scene descriptor for vrt_scene_create (borrowed pointers). */
int vrt_obj_scene_desc(const vrt_obj *o, vrt_scene_desc *desc);

/* stbi_load(path, &w, &h, &comp, 0) for TGA files (VRT/stb_image.h:
 * 5404-5640): 8-bit interleaved, row 0 = top; free with vrt_image_free. */
int vrt_tga_load(const char *path, int *w, int *h, int *comp, uint8_t **out);
int vrt_tga_decode(const uint8_t *buf, int64_t len, int *w, int *h, int *comp,
                   uint8_t **out);
void vrt_image_free(uint8_t *p);

/* ---- synthetic inputs ----------------------------------------------------
 * Deterministic "sponza-proxy" atrium (no Sponza asset ships): floor, walls,
 * two storeys of colonnades and arches, curtains, details; every material
 * textured with procedural 8-bit textures.  `detail` scales tessellation
 * (1.0 ~ 262k triangles).  Two-call protocol: call with NULL arrays to get
 * counts in *ntri / *nmat / *ntex / *tex_bytes, then with arrays sized to
 * them.  Bounds match the scaled Sponza frame the reference cameras use
 * (VRT/main.cc:76-78,112-115). */
int vrt_proxy_scene(double detail, uint32_t seed, int32_t *ntri, float *pos,
                    float *nrm, float *uv, int32_t *mat, int32_t *nmat,
                    int32_t *mat_tex, float *mat_kd, int32_t *ntex,
                    int32_t *tex_dims, int64_t *tex_off, uint8_t *tex_data,
                    int64_t *tex_bytes);
/* Camera-sweep pose i of n: ellipse at 0.4 * AABB height around the AABB
 * centre, looking at the centre, fov 90 degrees. */
int vrt_sweep_pose(const float root_min[3], const float root_max[3], int i,
                   int n, float eye[3], float spot[3], float up[3],
                   float *fov);

const char *vrt_status_string(int status);
const char *vrt_last_error(void);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
