// vrt_host.cpp -- host side of libvrt.so: the C ABI of include/vrt.h.
//
//  * octree build (gi::ray_march_init, VRT/voxel_octree.cc:27-75) as a
//    parallel per-triangle descent + sort, flattened to the BFS child-block
//    layout the kernels read (DESIGN.md "Data layout in HBM");
//  * scene upload, render / ray-march orchestration on a HIP stream;
//  * camera (VRT/camera.cc:65-112) and the legacy intersect_triangle3 /
//    triBoxOverlap symbols, all through vrt_math.h (the kernels' own code).
//
// VRT/x = /root/reference/VoxelRayTrace20190722/x
#include "../../include/vrt.h"
#include "vrt_error.h"
#include "vrt_internal.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using namespace vrt;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

static int vfail(int code, const char *fmt, va_list ap)
{
        char buf[512];
        vsnprintf(buf, sizeof buf, fmt, ap);
        g_err = buf;
        return code;
}

static int fail(int code, const char *fmt, ...)
{
        va_list ap;
        va_start(ap, fmt);
        vfail(code, fmt, ap);
        va_end(ap);
        return code;
}

// shared with the ingest sources (vrt_obj.cpp, vrt_tga.cpp); hidden symbol
int vrt::set_error(int code, const char *fmt, ...)
{
        va_list ap;
        va_start(ap, fmt);
        vfail(code, fmt, ap);
        va_end(ap);
        return code;
}

#define HIPCHK(expr)                                                             \
        do {                                                                     \
                hipError_t e_ = (expr);                                          \
                if (e_ != hipSuccess)                                            \
                        return fail(VRT_E_DEVICE, "%s failed: %s", #expr,       \
                                    hipGetErrorString(e_));                      \
        } while (0)

extern "C" const char *vrt_last_error(void) { return g_err.c_str(); }

extern "C" const char *vrt_status_string(int s)
{
        switch (s) {
        case VRT_OK: return "ok";
        case VRT_E_INVALID: return "invalid argument";
        case VRT_E_NOMEM: return "out of host memory";
        case VRT_E_DEVICE: return "HIP runtime error";
        case VRT_E_NODEVICE: return "no usable gfx950 device";
        case VRT_E_IO: return "i/o error";
        default: return "unknown status";
        }
}

static double now_ms()
{
        using namespace std::chrono;
        return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------------------
// legacy reference symbols
// ---------------------------------------------------------------------------
extern "C" int intersect_triangle3(double orig[3], double dir[3],
                                   double vert0[3], double vert1[3],
                                   double vert2[3], double *t, double *u,
                                   double *v)
{
        return mt_isect(orig, dir, vert0, vert1, vert2, t, u, v);
}

extern "C" int triBoxOverlap(float boxcenter[3], float boxhalfsize[3],
                             float triverts[3][3])
{
        return tri_box_overlap(boxcenter, boxhalfsize, &triverts[0][0]);
}

// ---------------------------------------------------------------------------
// camera (VRT/camera.cc:65-112)
// ---------------------------------------------------------------------------
extern "C" int vrt_camera_init(float fov, const float eye[3],
                               const float spot[3], const float up[3],
                               float near_, float far_, vrt_camera *out)
{
        if (!eye || !spot || !up || !out)
                return fail(VRT_E_INVALID, "vrt_camera_init: null argument");
        const f3 e = mk3(eye[0], eye[1], eye[2]);
        const f3 fwd = normalize(mk3(spot[0], spot[1], spot[2]) - e);
        const f3 s = normalize(cross(fwd, mk3(up[0], up[1], up[2])));
        const f3 u = normalize(cross(s, fwd));
        const f3 nf = -fwd;
        const float C[16] = { s.x, s.y, s.z, 0.f, u.x, u.y, u.z, 0.f,
                              nf.x, nf.y, nf.z, 0.f, e.x, e.y, e.z, 1.f };
        std::memcpy(out->C, C, sizeof C);
        out->fov = fov;
        out->near_ = near_;
        out->far_ = far_;
        // point_transform(C_, {}): dot(C, (0,0,0,1)) then /= w
        // (VRT/graphics_math.h:1063-1070)
        float r[4];
        for (int k = 0; k < 4; ++k) {
                float acc = 0.0f;
                acc += C[k] * 0.0f;
                acc += C[4 + k] * 0.0f;
                acc += C[8 + k] * 0.0f;
                acc += C[12 + k] * 1.0f;
                r[k] = acc;
        }
        const float w = r[3];
        for (int k = 0; k < 3; ++k)
                out->origin[k] = r[k] / w;
        return VRT_OK;
}

static float cam_zplane(const vrt_camera *cam, const vrt_film *film)
{
        // -(film.h / (2 * std::tanf(fov / 2)))  (VRT/camera.cc:100)
        return -(film->h / (2.0f * tanf(cam->fov / 2.0f)));
}

static void fill_cam_params(const vrt_camera *cam, const vrt_film *film,
                            CamParams *cp)
{
        for (int k = 0; k < 3; ++k) {
                cp->s[k] = cam->C[k];
                cp->u[k] = cam->C[4 + k];
                cp->nf[k] = cam->C[8 + k];
                cp->e[k] = cam->C[12 + k];
                cp->origin[k] = cam->origin[k];
        }
        cp->z = cam_zplane(cam, film);
        cp->tmin = cam->near_;
        cp->tmax = cam->far_;
        cp->nx = film->nx;
        cp->ny = film->ny;
}

static int gen_rays(const vrt_camera *cam, const vrt_film *film, int px,
                    int py, vrt_ray *out, int n)
{
        if (!cam || !film || !out)
                return fail(VRT_E_INVALID, "gen_rays: null argument");
        if (px < 0 || px >= film->nx || py < 0 || py >= film->ny)
                return fail(VRT_E_INVALID, "gen_rays: pixel (%d,%d) outside film", px, py);
        CamParams cp;
        fill_cam_params(cam, film, &cp);
        for (int s = 0; s < n; ++s) {
                const float sx = n == 4 ? sample_x(s) : 0.5f;
                const float sy = n == 4 ? sample_y(s) : 0.5f;
                const f3 d = camera_dir(cp.s, cp.u, cp.nf, cp.e, cp.z, cp.nx, cp.ny,
                                        px, py, sx, sy);
                for (int k = 0; k < 3; ++k)
                        out[s].o[k] = cp.origin[k];
                out[s].d[0] = d.x;
                out[s].d[1] = d.y;
                out[s].d[2] = d.z;
                out[s].tmin = cp.tmin;
                out[s].tmax = cp.tmax;
        }
        return VRT_OK;
}

extern "C" int vrt_camera_defer_bound(const vrt_camera *cam, const vrt_film *film, int64_t *bound)
{
        if (!cam || !film || !bound || film->nx < 1 || film->ny < 1)
                return fail(VRT_E_INVALID, "vrt_camera_defer_bound: bad argument");
        CamParams cp;
        fill_cam_params(cam, film, &cp);
        *bound = camera_defer_bound(cp);
        return VRT_OK;
}

extern "C" int vrt_gen_rays4(const vrt_camera *cam, const vrt_film *film,
                             int px, int py, vrt_ray out[4])
{
        return gen_rays(cam, film, px, py, out, 4);
}

extern "C" int vrt_gen_rays1(const vrt_camera *cam, const vrt_film *film,
                             int px, int py, vrt_ray out[1])
{
        return gen_rays(cam, film, px, py, out, 1);
}

extern "C" int vrt_make_ray(const float o[3], const float d[3], float tmin,
                            float tmax, vrt_ray *out)
{
        if (!o || !d || !out)
                return fail(VRT_E_INVALID, "vrt_make_ray: null argument");
        const f3 dn = normalize(mk3(d[0], d[1], d[2]));
        for (int k = 0; k < 3; ++k)
                out->o[k] = o[k];
        out->d[0] = dn.x;
        out->d[1] = dn.y;
        out->d[2] = dn.z;
        out->tmin = tmin;
        out->tmax = tmax;
        return VRT_OK;
}

extern "C" int vrt_aabb_isect(const float box[6], const vrt_ray *ray)
{
        if (!box || !ray)
                return 0;
        const f3 o = mk3(ray->o[0], ray->o[1], ray->o[2]);
        const f3 di = mk3(dinv_of(ray->d[0]), dinv_of(ray->d[1]), dinv_of(ray->d[2]));
        return aabb_isect(box, box + 3, o, di, ray->tmin, ray->tmax) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// octree build
// ---------------------------------------------------------------------------
namespace {

struct Box {
        float mn[3], mx[3];
};

// split() child box (VRT/voxel_octree.cc:30-35)
inline Box child_box(const Box &p, int i)
{
        Box c;
        const int m[3] = { (i & 4) ? 1 : 0, (i & 2) ? 1 : 0, (i & 1) ? 1 : 0 };
        for (int k = 0; k < 3; ++k) {
                const float half = (p.mx[k] - p.mn[k]) / 2.0f;
                c.mn[k] = p.mn[k] + (float)m[k] * half;
                c.mx[k] = c.mn[k] + half;
        }
        return c;
}

// Triangle::is_overlap (VRT/voxel_octree.cc:486-492)
inline bool overlaps(const float *tri9, const Box &b)
{
        float c[3], h[3];
        for (int k = 0; k < 3; ++k) {
                c[k] = (b.mn[k] + b.mx[k]) * .5f;
                h[k] = (b.mx[k] - b.mn[k]) / 2.f;
        }
        return tri_box_overlap(c, h, tri9) == 1;
}

struct BuildOut {
        // internal node keys per depth (path code, 3 bits per level)
        std::vector<std::vector<uint32_t>> internal;
        // (leaf code << 32 | tri) at max depth
        std::vector<uint64_t> refs;
};

// Descend one triangle: the set of nodes insert() reaches for it.  A node is
// split iff some triangle overlaps it (and all its ancestors) above
// max_depth; a max-depth leaf lists exactly those triangles.
void descend(const float *tri9, uint32_t tri, const Box &b, int depth,
             int max_depth, uint32_t code, BuildOut &o)
{
        if (!overlaps(tri9, b))
                return;
        if (depth == max_depth) {
                o.refs.push_back(((uint64_t)code << 32) | tri);
                return;
        }
        o.internal[depth].push_back(code);
        for (int i = 0; i < 8; ++i)
                descend(tri9, tri, child_box(b, i), depth + 1, max_depth,
                        (code << 3) | (uint32_t)i, o);
}

uint32_t vox_of(uint32_t code, int depth)
{
        uint32_t ix = 0, iy = 0, iz = 0;
        for (int l = depth - 2; l >= 0; --l) {
                const uint32_t ci = (code >> (3 * l)) & 7u;
                ix = (ix << 1) | ((ci >> 2) & 1u);
                iy = (iy << 1) | ((ci >> 1) & 1u);
                iz = (iz << 1) | (ci & 1u);
        }
        return ix | (iy << 10) | (iz << 20);
}

}  // namespace

// Bands of vrt_render's host-output path: tile-row bands rendered
// alternately on two streams (each a half-chip persistent grid, as with
// frames in flight), each band's D2H copy queued as soon as it is rendered,
// so the copies of the first bands run beside the renders of the last.
constexpr int kOutBands = 4;
struct HostOut {
        float *d_img = nullptr;   // nx*ny*3 floats; pixels outside the tile grid stay 0
        float *h_pin = nullptr;   // pinned staging of d_img
        size_t bytes = 0;
        int nx = 0, ny = 0;
        hipStream_t st2 = nullptr, cp = nullptr;
        hipEvent_t ev_r[kOutBands] = {}, ev_c[kOutBands] = {};
        hipEvent_t ev_j = nullptr;  // second render stream joined back
};

// One set of the full trace's scene scratch (vrt_scene::ts).
struct TraceSet {
        LMRec *lm = nullptr;  // nodes x (LMRec + float4 cone record) + the finiteness flag
        void *rec = nullptr;  // split-trace records (64 B per sample), the cone step table
        size_t rec_bytes = 0;
        float steps_key[2] = { -1.f, -1.f };  // (mindist, maxdist) the step table holds
        hipEvent_t ev = nullptr;  // its last user's work
        bool live = false;
};

struct vrt_scene {
        int device = 0;
        int max_depth = 0;
        int ntri = 0;
        std::vector<NodeRec> nodes;
        std::vector<uint32_t> node_vox;
        std::vector<RefRec48> refs48;   // one of the two leaf-record formats
        std::vector<RefRec64> refs64;   // (wide_leaves: RefRec64)
        bool wide_leaves = false;
        std::vector<uint32_t> ref_tri;  // triangle id per leaf-list entry
        std::vector<TriPos> tri_pos;
        std::vector<TriAttr> tri_attr;
        std::vector<MatRec> mats;
        std::vector<TexRec> texs;
        int64_t tex_bytes = 0;
        vrt_scene_info_t info{};
        std::vector<int64_t> level_begin;  // BFS level l (1-based) = [lb[l-1], lb[l])
        // full trace: two sets of {light-map block (LMRec + cone-descent
        // records + finiteness flag), split-trace records}, taken by
        // alternate light-map builds so that one frame's cone-traced shading
        // runs beside the next frame's light pass; each with the event of its
        // last user.  lm_cur = the set with the latest light map (-1: none).
        // The light pass's own scratch (keys, sort) is used on the scene
        // stream only.
        TraceSet ts[2];
        int ts_next = 0;
        int lm_cur = -1;
        void *d_light = nullptr;
        size_t light_bytes = 0;
        // config-5 ray compaction (SpillQueues): round counters + two record
        // queues of spill_cap chunks each; two sets, used by alternate
        // frames (two config-5 frames in flight on two streams), each with
        // the event of its last launch
        void *d_spill[2] = {};
        uint32_t spill_cap[2] = {};  // chunks per queue
        int64_t spill_px[2] = {};    // deferred-pixel list capacity (pixels)
        hipEvent_t spill_ev[2] = {};
        bool spill_live[2] = {};
        hipStream_t spill_stream[2] = {};  // the set's last user (a stream keeps its set)
        // per set: the side stream of its deferred-pixel walk, fork / join
        SideLaunch spill_side[2] = {};
        // multi-rank tile deals tabled on the device (RenderParams::tile_xy),
        // one per (tiles, ranks, rank) used, built on first use by a kernel
        // on that call's stream (ev), kept until the scene is destroyed
        struct DealMap {
                int ntx, nty, nranks, rank;
                uint32_t *d;
                hipEvent_t ev;
        };
        std::vector<DealMap> dmaps;
        uint32_t *h_spill = nullptr;       // pinned: per set, its last launch's round counters (ctr[0..7])
        uint32_t spill_want = 0;           // queue-0 chunks the next launch sizes for (0: first estimate)
        int spill_next = 0;
        int spill_last = -1;  // the set the last config-5 launch compacted with (vrt_secondary_spill_counts)
        // device
        void *d_mem = nullptr;
        DevScene dev{};
        hipStream_t stream = nullptr;
        hipEvent_t ev0 = nullptr, ev1 = nullptr;
        bool timed = false;
        // persistent-render work queues (WorkQueue, vrt_internal.h): a ring
        // of kQueueSlots counter sets, each with its bases and the event of
        // its last launch
        uint32_t *d_queue = nullptr;
        uint32_t q_base[kQueueSlots][8] = {};
        hipEvent_t q_ev[kQueueSlots] = {};
        bool q_live[kQueueSlots] = {};
        int q_next = 0;
        hipEvent_t lm_ev = nullptr;  // vrt_trace_frame_device: the light map is filtered
        // vrt_render's host-output path (render_to_host): a device image kept
        // between calls, its pinned host staging copy, a second render stream
        // and a copy stream, and an event per band
        HostOut ho;
        // vrt_ray_march_batch: device ray / hit buffers and pinned staging
        // kept between calls (grown as needed)
        void *d_rays = nullptr, *d_hits = nullptr, *h_rays = nullptr, *h_hits = nullptr;
        int64_t rays_cap = 0;
        // every entry point that launches work on the scene holds mu (one
        // host thread at a time; device work on several streams is ordered
        // by the events above)
        std::mutex mu;
};

static int finish_tree(vrt_scene *s, const vrt_scene_desc *d, const Box &root, const std::vector<uint64_t> &refs,
                       int64_t ninternal);
static int check_device(int device);

static int build_tree(vrt_scene *s, const vrt_scene_desc *d, bool on_device)
{
        const int D = s->max_depth;
        const int n = d->ntri;
        // root = AABB{} merged with every triangle AABB, in input order
        // (VRT/voxel_octree.cc:70-72; AABB(Iter,Iter) graphics_math.h:1240-1251)
        Box root;
        for (int k = 0; k < 3; ++k) {
                root.mn[k] = kFltMax;
                root.mx[k] = -kFltMax;
        }
        for (int i = 0; i < n; ++i) {
                const float *p = d->pos + 9 * (size_t)i;
                float tmn[3] = { kFltMax, kFltMax, kFltMax };
                float tmx[3] = { -kFltMax, -kFltMax, -kFltMax };
                for (int v = 0; v < 3; ++v)
                        for (int k = 0; k < 3; ++k) {
                                tmn[k] = std_min(tmn[k], p[3 * v + k]);
                                tmx[k] = std_max(tmx[k], p[3 * v + k]);
                        }
                for (int k = 0; k < 3; ++k) {
                        root.mn[k] = std_min(root.mn[k], tmn[k]);
                        root.mx[k] = std_max(root.mx[k], tmx[k]);
                }
        }

        if (on_device) {
                // level-synchronous descent, sorts, flatten and masks on the GPU
                DeviceBuild db;
                std::string err;
                int rc = check_device(s->device);
                if (rc)
                        return rc;
                if (build_tree_device(s->device, d->pos, n, root.mn, root.mx, D, &db, &err) != hipSuccess)
                        return fail(VRT_E_DEVICE, "device octree build: %s", err.c_str());
                s->nodes.swap(db.nodes);
                s->node_vox.swap(db.node_vox);
                s->level_begin.swap(db.level_begin);
                s->info.build_device_ms = db.device_ms;
                return finish_tree(s, d, root, db.refs, db.ninternal);
        }
        // parallel per-triangle descent
        unsigned nth = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
        if (n < 4096)
                nth = 1;
        std::vector<BuildOut> outs(nth);
        for (auto &o : outs)
                o.internal.resize(D + 1);
        {
                std::atomic<int> next{ 0 };
                auto work = [&](unsigned t) {
                        BuildOut &o = outs[t];
                        for (;;) {
                                const int i0 = next.fetch_add(1024);
                                if (i0 >= n)
                                        break;
                                const int i1 = std::min(n, i0 + 1024);
                                for (int i = i0; i < i1; ++i)
                                        descend(d->pos + 9 * (size_t)i, (uint32_t)i, root, 1, D, 0u, o);
                        }
                };
                std::vector<std::thread> th;
                for (unsigned t = 1; t < nth; ++t)
                        th.emplace_back(work, t);
                work(0);
                for (auto &x : th)
                        x.join();
        }
        // merge
        std::vector<std::vector<uint32_t>> internal(D + 1);
        for (int l = 1; l < D; ++l) {
                size_t tot = 0;
                for (auto &o : outs)
                        tot += o.internal[l].size();
                internal[l].reserve(tot);
                for (auto &o : outs) {
                        internal[l].insert(internal[l].end(), o.internal[l].begin(), o.internal[l].end());
                        std::vector<uint32_t>().swap(o.internal[l]);
                }
                std::sort(internal[l].begin(), internal[l].end());
                internal[l].erase(std::unique(internal[l].begin(), internal[l].end()), internal[l].end());
        }
        std::vector<uint64_t> refs;
        {
                size_t tot = 0;
                for (auto &o : outs)
                        tot += o.refs.size();
                refs.reserve(tot);
                for (auto &o : outs) {
                        refs.insert(refs.end(), o.refs.begin(), o.refs.end());
                        std::vector<uint64_t>().swap(o.refs);
                }
                // (leaf code, tri index): leaf lists in insertion = input order
                std::sort(refs.begin(), refs.end());
        }

        // flatten: root = node 0; level by level, internal nodes in code
        // order each own the next block of 8 children.
        int64_t ninternal = 0;
        for (int l = 1; l < D; ++l)
                ninternal += (int64_t)internal[l].size();
        const int64_t nnodes = 1 + 8 * ninternal;
        if (nnodes > 0x7FFFFFFF)
                return fail(VRT_E_INVALID, "octree too large (%lld nodes)", (long long)nnodes);
        s->nodes.assign((size_t)nnodes, NodeRec{});
        s->node_vox.assign((size_t)nnodes, 0u);
        std::vector<Box> boxes((size_t)nnodes);
        std::vector<uint32_t> codes((size_t)nnodes);
        std::vector<int32_t> depth_of((size_t)nnodes);
        boxes[0] = root;
        codes[0] = 0;
        depth_of[0] = 1;
        // first node index of each level and the block base of each internal
        // node: internal node j (global order) owns children 1 + 8j ...
        int64_t j_base = 0;  // global index of first internal node at level l
        // level l's nodes occupy a contiguous index range [lv_begin, lv_end)
        int64_t lv_begin = 0, lv_end = 1;
        size_t ref_pos = 0;
        s->level_begin.clear();
        for (int l = 1; l <= D; ++l) {
                s->level_begin.push_back(lv_begin);
                const std::vector<uint32_t> &I = internal[l];  // empty at l == D
                // nodes of this level are in code order (children blocks of
                // the previous level's code-ordered internal nodes)
                size_t ii = 0;
                for (int64_t ni = lv_begin; ni < lv_end; ++ni) {
                        const uint32_t code = codes[ni];
                        NodeRec &nr = s->nodes[ni];
                        for (int k = 0; k < 3; ++k) {
                                nr.bmin[k] = boxes[ni].mn[k];
                                nr.bmax[k] = boxes[ni].mx[k];
                        }
                        s->node_vox[ni] = vox_of(code, l);
                        while (ii < I.size() && I[ii] < code)
                                ++ii;
                        if (l < D && ii < I.size() && I[ii] == code) {
                                const int64_t jg = j_base + (int64_t)ii;
                                const int64_t first = 1 + 8 * jg;
                                nr.a = (uint32_t)first;
                                nr.b = 0;
                                for (int c = 0; c < 8; ++c) {
                                        boxes[first + c] = child_box(boxes[ni], c);
                                        codes[first + c] = (code << 3) | (uint32_t)c;
                                        depth_of[first + c] = l + 1;
                                }
                        } else if (l == D) {
                                // max-depth leaf: its list in refs
                                const uint64_t key = (uint64_t)code << 32;
                                while (ref_pos < refs.size() && refs[ref_pos] < key)
                                        ++ref_pos;
                                const size_t r0 = ref_pos;
                                while (ref_pos < refs.size() && (refs[ref_pos] >> 32) == code)
                                        ++ref_pos;
                                nr.a = kLeafBit | (uint32_t)(ref_pos - r0);
                                nr.b = (uint32_t)r0;
                        } else {
                                nr.a = kLeafBit;  // empty leaf above max depth
                                nr.b = 0;
                        }
                }
                // next level: children of this level's internal nodes, in
                // the same (code) order
                const int64_t next_begin = lv_end;
                const int64_t next_end = next_begin + 8 * (int64_t)I.size();
                j_base += (int64_t)I.size();
                lv_begin = next_begin;
                lv_end = next_end;
                if (l < D && lv_begin == lv_end)
                        break;
        }
        s->level_begin.push_back(nnodes);
        // content masks, bottom-up (children always follow their parent):
        // an internal node's b = the children that hold triangles somewhere
        // below.  The kernels never push a child outside this mask: a
        // subtree without triangles cannot hit, so the DFS result is
        // unchanged (the instrumented kernel ignores it to count exactly the
        // reference's visits).
        {
                std::vector<uint8_t> has((size_t)nnodes, 0);
                for (int64_t ni = nnodes - 1; ni >= 0; --ni) {
                        NodeRec &nr = s->nodes[ni];
                        if (nr.a & kLeafBit) {
                                has[ni] = (nr.a & ~kLeafBit) ? 1 : 0;
                        } else {
                                uint32_t m = 0;
                                for (int c = 0; c < 8; ++c)
                                        m |= (uint32_t)has[nr.a + c] << c;
                                nr.b = m;
                                has[ni] = m ? 1 : 0;
                        }
                }
        }
        return finish_tree(s, d, root, refs, ninternal);
}

// leaf records with inlined vertices + scene info (both build paths)
static int finish_tree(vrt_scene *s, const vrt_scene_desc *d, const Box &root, const std::vector<uint64_t> &refs,
                       int64_t ninternal)
{
        const int64_t nnodes = (int64_t)s->nodes.size();
        int64_t leaves = 0, nonempty = 0;
        for (const NodeRec &nr : s->nodes) {
                if (nr.a & kLeafBit) {
                        ++leaves;
                        if (nr.a & ~kLeafBit)
                                ++nonempty;
                }
        }
        s->wide_leaves = refs.size() >= 8 * (size_t)std::max<int64_t>(1, nonempty);
        s->ref_tri.resize(refs.size());
        if (s->wide_leaves)
                s->refs64.resize(refs.size());
        else
                s->refs48.resize(refs.size());
        for (size_t i = 0; i < refs.size(); ++i) {
                const uint32_t t = (uint32_t)(refs[i] & 0xFFFFFFFFu);
                s->ref_tri[i] = t;
                const float *p = d->pos + 9 * (size_t)t;
                if (s->wide_leaves) {
                        RefRec64 &rr = s->refs64[i];
                        for (int k = 0; k < 3; ++k) {
                                rr.v0[k] = p[k];
                                rr.e1[k] = (double)p[3 + k] - (double)p[k];  // SUB(edge1, vert1, vert0)
                                rr.e2[k] = (double)p[6 + k] - (double)p[k];  // SUB(edge2, vert2, vert0)
                        }
                        rr.tri = t;
                } else {
                        RefRec48 &rr = s->refs48[i];
                        std::memcpy(rr.p, p, sizeof rr.p);
                        rr.tri = t;
                        rr.pad[0] = rr.pad[1] = 0;
                }
        }
        s->info.nodes = nnodes;
        s->info.internal = ninternal;
        s->info.leaves = leaves;
        s->info.nonempty_leaves = nonempty;
        s->info.tri_refs = (int64_t)refs.size();
        for (int k = 0; k < 3; ++k) {
                s->info.root_min[k] = root.mn[k];
                s->info.root_max[k] = root.mx[k];
        }
        return VRT_OK;
}

static int check_device(int device)
{
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
                return fail(VRT_E_NODEVICE, "no HIP device visible");
        if (device < 0 || device >= n)
                return fail(VRT_E_NODEVICE, "device %d out of range (%d visible)", device, n);
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
                return fail(VRT_E_NODEVICE, "device %d is %s, kernels are built for gfx950",
                            device, prop.gcnArchName);
        return VRT_OK;
}

extern "C" int vrt_device_count(int *n)
{
        if (!n)
                return fail(VRT_E_INVALID, "null");
        *n = 0;
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess)
                return VRT_OK;
        *n = c;
        return VRT_OK;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// DevScene::xnodes: every node's own record followed by the union box of all
// triangles below it (a leaf: its own), enlarged by eps = 2^-16 * the root's
// largest extent and rounded outward to float.  Sets lb_center and
// lb_reach = 16 * that extent: for a ray origin within lb_reach of the
// centre (per axis) and a point of a leaf's triangles, every slab distance
// |p - o| / |d| is below 17 * extent / |d|, the three fp32 roundings of
// (p - o) * (1/d) move it by less than 3 * 2^-24 * 17 * extent / |d| <
// eps / |d|, so the fp32 line test on the enlarged box passes whenever the
// exact line meets the unenlarged one -- and intersect_triangle3 accepts a
// triangle only where the line meets it (up to its fp64 rounding, far below
// eps); an internal node's box bounds the triangles of its leaves, which all
// lie in the root box, so the same bound holds.  Nodes with no triangle below
// them (never visited by the content-masked walk), and every node of a scene
// whose extent is not finite and positive (no skip), carry their voxel box.
static void march_nodes(vrt_scene *s, const vrt_scene_desc *d, std::vector<XNodeRec> &xn)
{
        const size_t nn = s->nodes.size();
        xn.resize(nn);
        for (size_t i = 0; i < nn; ++i) {
                xn[i] = XNodeRec{};
                xn[i].n = s->nodes[i];
                for (int k = 0; k < 3; ++k) {
                        xn[i].tmin[k] = s->nodes[i].bmin[k];
                        xn[i].tmax[k] = s->nodes[i].bmax[k];
                }
        }
        float ext = 0.f;
        for (int k = 0; k < 3; ++k) {
                ext = std::max(ext, s->info.root_max[k] - s->info.root_min[k]);
                s->dev.lb_center[k] = 0.5f * (s->info.root_min[k] + s->info.root_max[k]);
        }
        s->dev.lb_reach = 16.f * ext;
        if (!(ext > 0.f) || !std::isfinite(ext)) {
                s->dev.lb_reach = -1.f;  // never skip
                return;
        }
        const double eps = std::ldexp((double)ext, -16);
        // unenlarged triangle boxes, bottom-up (children follow their parent
        // in the BFS array)
        std::vector<double> lo(3 * nn, HUGE_VAL), hi(3 * nn, -HUGE_VAL);
        for (size_t i = nn; i-- > 0;) {
                const NodeRec &nr = s->nodes[i];
                double *l = &lo[3 * i], *h = &hi[3 * i];
                if (nr.a & kLeafBit) {
                        const uint32_t n = nr.a & ~kLeafBit;
                        for (uint32_t j = 0; j < n; ++j) {
                                const float *p = d->pos + 9 * (size_t)s->ref_tri[nr.b + j];
                                for (int v = 0; v < 3; ++v)
                                        for (int k = 0; k < 3; ++k) {
                                                l[k] = std::min(l[k], (double)p[3 * v + k]);
                                                h[k] = std::max(h[k], (double)p[3 * v + k]);
                                        }
                        }
                } else {
                        for (uint32_t c = 0; c < 8; ++c)
                                for (int k = 0; k < 3; ++k) {
                                        l[k] = std::min(l[k], lo[3 * (nr.a + c) + k]);
                                        h[k] = std::max(h[k], hi[3 * (nr.a + c) + k]);
                                }
                }
        }
        for (size_t i = 1; i < nn; ++i) {
                const double *l = &lo[3 * i], *h = &hi[3 * i];
                if (!(l[0] <= h[0]))
                        continue;  // no triangle below this node
                float bl[3], bh[3];
                for (int k = 0; k < 3; ++k) {
                        float fl = (float)(l[k] - eps), fh = (float)(h[k] + eps);
                        if ((double)fl > l[k] - eps)
                                fl = std::nextafter(fl, -HUGE_VALF);
                        if ((double)fh < h[k] + eps)
                                fh = std::nextafter(fh, HUGE_VALF);
                        bl[k] = fl;
                        bh[k] = fh;
                }
                for (int k = 0; k < 3; ++k) {
                        xn[i].tmin[k] = bl[k];
                        xn[i].tmax[k] = bh[k];
                }
        }
}

static int upload(vrt_scene *s, const vrt_scene_desc *d)
{
        int rc = check_device(s->device);
        if (rc)
                return rc;
        HIPCHK(hipSetDevice(s->device));
        const size_t sz_nodes = s->nodes.size() * sizeof(NodeRec);
        const size_t sz_vox = s->node_vox.size() * sizeof(uint32_t);
        const void *refs_host = s->wide_leaves ? (const void *)s->refs64.data() : (const void *)s->refs48.data();
        const size_t refs_bytes = s->wide_leaves ? s->refs64.size() * sizeof(RefRec64)
                                                 : s->refs48.size() * sizeof(RefRec48);
        const size_t sz_refs = std::max<size_t>(64, refs_bytes);
        const size_t sz_pos = std::max<size_t>(1, s->tri_pos.size()) * sizeof(TriPos);
        const size_t sz_attr = std::max<size_t>(1, s->tri_attr.size()) * sizeof(TriAttr);
        const size_t sz_mats = s->mats.size() * sizeof(MatRec);
        const size_t sz_texs = std::max<size_t>(1, s->texs.size()) * sizeof(TexRec);
        const size_t sz_tex = (size_t)std::max<int64_t>(16, s->tex_bytes);
        size_t off[11];
        size_t tot = 0;
        const size_t sz_xnodes = s->nodes.size() * sizeof(XNodeRec);
        const size_t sizes[10] = { sz_nodes, sz_vox, sz_refs, sz_pos, sz_attr, sz_mats, sz_texs, sz_tex,
                                   kQueueSlots * kQueueBytes, sz_xnodes };
        for (int i = 0; i < 10; ++i) {
                off[i] = tot;
                tot += align_up(sizes[i]);
        }
        off[10] = tot;
        HIPCHK(hipMalloc(&s->d_mem, tot));
        char *base = static_cast<char *>(s->d_mem);
        HIPCHK(hipMemset(base + off[8], 0, kQueueSlots * kQueueBytes));
        HIPCHK(hipMemcpy(base + off[0], s->nodes.data(), sz_nodes, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(base + off[1], s->node_vox.data(), sz_vox, hipMemcpyHostToDevice));
        if (refs_bytes)
                HIPCHK(hipMemcpy(base + off[2], refs_host, refs_bytes, hipMemcpyHostToDevice));
        if (!s->tri_pos.empty())
                HIPCHK(hipMemcpy(base + off[3], s->tri_pos.data(), s->tri_pos.size() * sizeof(TriPos), hipMemcpyHostToDevice));
        if (!s->tri_attr.empty())
                HIPCHK(hipMemcpy(base + off[4], s->tri_attr.data(), s->tri_attr.size() * sizeof(TriAttr), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(base + off[5], s->mats.data(), sz_mats, hipMemcpyHostToDevice));
        if (!s->texs.empty())
                HIPCHK(hipMemcpy(base + off[6], s->texs.data(), s->texs.size() * sizeof(TexRec), hipMemcpyHostToDevice));
        if (s->tex_bytes > 0)
                HIPCHK(hipMemcpy(base + off[7], d->tex_data, (size_t)s->tex_bytes, hipMemcpyHostToDevice));
        s->dev.nodes = reinterpret_cast<const NodeRec *>(base + off[0]);
        s->dev.node_vox = reinterpret_cast<const uint32_t *>(base + off[1]);
        s->dev.refs = base + off[2];
        s->dev.tri_pos = reinterpret_cast<const TriPos *>(base + off[3]);
        s->dev.tri_attr = reinterpret_cast<const TriAttr *>(base + off[4]);
        s->dev.mats = reinterpret_cast<const MatRec *>(base + off[5]);
        s->dev.texs = reinterpret_cast<const TexRec *>(base + off[6]);
        s->dev.tex_data = reinterpret_cast<const uint8_t *>(base + off[7]);
        s->d_queue = reinterpret_cast<uint32_t *>(base + off[8]);
        {
                // the march records of the nodes (DevScene::xnodes)
                std::vector<XNodeRec> xn;
                march_nodes(s, d, xn);
                if (sz_xnodes)
                        HIPCHK(hipMemcpy(base + off[9], xn.data(), sz_xnodes, hipMemcpyHostToDevice));
                s->dev.xnodes = reinterpret_cast<const XNodeRec *>(base + off[9]);
        }
        HIPCHK(persistent_blocks(&s->dev.persist_blocks, &s->dev.sec_blocks));
        s->dev.grid_div = 1;
        s->dev.max_depth = s->max_depth;
        s->dev.nmat = (int32_t)s->mats.size();
        s->dev.ntex = (int32_t)s->texs.size();
        {
                bool ok = true;
                for (int k = 0; k < 3; ++k) {
                        const float lo = s->info.root_min[k], hi = s->info.root_max[k];
                        ok = ok && std::fabs(lo) < 0x1p60f && std::fabs(hi) < 0x1p60f;  // see fast_ok()
                }
                s->dev.fast_ok = ok ? 1 : 0;
                s->dev.wide_leaves = s->wide_leaves ? 1 : 0;
        }
        s->info.device_bytes = (int64_t)tot;
        HIPCHK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreate(&s->ev0));
        HIPCHK(hipEventCreate(&s->ev1));
        for (int k = 0; k < kQueueSlots; ++k)
                HIPCHK(hipEventCreateWithFlags(&s->q_ev[k], hipEventDisableTiming));
        for (TraceSet &t : s->ts)
                HIPCHK(hipEventCreateWithFlags(&t.ev, hipEventDisableTiming));
        return VRT_OK;
}

static int validate_desc(const vrt_scene_desc *d, int max_depth)
{
        if (!d)
                return fail(VRT_E_INVALID, "null scene descriptor");
        if (max_depth < 1 || max_depth > VRT_MAX_DEPTH)
                return fail(VRT_E_INVALID, "max_depth %d outside [1,%d]", max_depth, VRT_MAX_DEPTH);
        if (d->ntri < 0 || (d->ntri > 0 && (!d->pos || !d->nrm)))
                return fail(VRT_E_INVALID, "bad triangle arrays");
        if (d->nmat < 1 || !d->mat_tex || !d->mat_kd)
                return fail(VRT_E_INVALID, "need >= 1 material (mat_tex, mat_kd)");
        if (d->ntex < 0 || (d->ntex > 0 && (!d->tex_dims || !d->tex_off || !d->tex_data)))
                return fail(VRT_E_INVALID, "bad texture arrays");
        for (int m = 0; m < d->nmat; ++m)
                if (d->mat_tex[m] < -1 || d->mat_tex[m] >= d->ntex)
                        return fail(VRT_E_INVALID, "material %d: texture id %d out of range", m, d->mat_tex[m]);
        for (int t = 0; t < d->ntex; ++t) {
                const int w = d->tex_dims[3 * t], h = d->tex_dims[3 * t + 1], c = d->tex_dims[3 * t + 2];
                if (w < 1 || h < 1 || c < 1 || c > 4 || d->tex_off[t] < 0 ||
                    d->tex_off[t] + (int64_t)w * h * c > d->tex_bytes)
                        return fail(VRT_E_INVALID, "texture %d: bad dims/offset", t);
        }
        if (d->mat)
                for (int i = 0; i < d->ntri; ++i)
                        if (d->mat[i] < 0 || d->mat[i] >= d->nmat)
                                return fail(VRT_E_INVALID, "triangle %d: material %d out of range", i, d->mat[i]);
        return VRT_OK;
}

extern "C" int vrt_scene_create(const vrt_scene_desc *d, int max_depth,
                                int device, vrt_scene **out)
{
        return vrt_scene_create_ex(d, max_depth, device, 0, out);
}

extern "C" int vrt_scene_create_ex(const vrt_scene_desc *d, int max_depth,
                                   int device, int flags, vrt_scene **out)
{
        if (!out)
                return fail(VRT_E_INVALID, "null out");
        *out = nullptr;
        int rc = validate_desc(d, max_depth);
        if (rc)
                return rc;
        if (flags & ~VRT_BUILD_DEVICE)
                return fail(VRT_E_INVALID, "unknown flags %#x", flags);
        if ((flags & VRT_BUILD_DEVICE) && device < 0)
                return fail(VRT_E_INVALID, "VRT_BUILD_DEVICE needs a device (device >= 0)");
        std::unique_ptr<vrt_scene> s(new (std::nothrow) vrt_scene);
        if (!s)
                return fail(VRT_E_NOMEM, "scene alloc");
        s->device = device;
        s->max_depth = max_depth;
        s->ntri = d->ntri;
        const double t0 = now_ms();
        try {
                rc = build_tree(s.get(), d, (flags & VRT_BUILD_DEVICE) != 0);
                if (rc)
                        return rc;
                const int n = d->ntri;
                s->tri_pos.resize((size_t)n);
                s->tri_attr.resize((size_t)n);
                for (int i = 0; i < n; ++i) {
                        TriPos &tp = s->tri_pos[i];
                        std::memcpy(tp.p, d->pos + 9 * (size_t)i, sizeof tp.p);
                        tp.pad[0] = tp.pad[1] = tp.pad[2] = 0.f;
                        TriAttr &ta = s->tri_attr[i];
                        for (int v = 0; v < 3; ++v) {
                                const float *nn = d->nrm + 9 * (size_t)i + 3 * v;
                                const f3 q = normalize(mk3(nn[0], nn[1], nn[2]));
                                ta.n[3 * v + 0] = q.x;
                                ta.n[3 * v + 1] = q.y;
                                ta.n[3 * v + 2] = q.z;
                        }
                        for (int k = 0; k < 6; ++k)
                                ta.t[k] = d->uv ? d->uv[6 * (size_t)i + k] : 0.f;
                        ta.mat = d->mat ? d->mat[i] : 0;
                }
                s->mats.resize((size_t)d->nmat);
                for (int m = 0; m < d->nmat; ++m) {
                        s->mats[m].tex = d->mat_tex[m];
                        for (int k = 0; k < 3; ++k)
                                s->mats[m].kd[k] = d->mat_kd[3 * m + k];
                }
                s->texs.resize((size_t)d->ntex);
                for (int t = 0; t < d->ntex; ++t) {
                        s->texs[t].off = d->tex_off[t];
                        s->texs[t].w = d->tex_dims[3 * t];
                        s->texs[t].h = d->tex_dims[3 * t + 1];
                        s->texs[t].c = d->tex_dims[3 * t + 2];
                        s->texs[t].pad = 0;
                }
                for (auto &mr : s->mats)
                        mr.tx = (mr.tex >= 0 && mr.tex < d->ntex) ? s->texs[(size_t)mr.tex] : TexRec{};
                s->tex_bytes = d->ntex ? d->tex_bytes : 0;
        } catch (const std::bad_alloc &) {
                return fail(VRT_E_NOMEM, "octree build: out of host memory");
        }
        s->info.build_ms = now_ms() - t0;
        s->info.max_depth = max_depth;
        s->info.device = device;
        const double t1 = now_ms();
        if (device < 0) {  // host-only scene: build and inspect, no device
                *out = s.release();
                return VRT_OK;
        }
        rc = upload(s.get(), d);
        if (rc) {
                vrt_scene_destroy(s.release());
                return rc;
        }
        s->info.upload_ms = now_ms() - t1;
        *out = s.release();
        return VRT_OK;
}

// The same scene on another device (vrt_scene_create_multi): the host-side
// octree, leaf records and shading tables of `src` are copied, not rebuilt,
// and uploaded to `device` exactly as vrt_scene_create uploads them.
int vrt::scene_replicate(const vrt_scene *src, const vrt_scene_desc *d, int device, vrt_scene **out)
{
        *out = nullptr;
        std::unique_ptr<vrt_scene> s(new (std::nothrow) vrt_scene);
        if (!s)
                return fail(VRT_E_NOMEM, "scene alloc");
        const double t0 = now_ms();
        try {
                s->device = device;
                s->max_depth = src->max_depth;
                s->ntri = src->ntri;
                s->nodes = src->nodes;
                s->node_vox = src->node_vox;
                s->refs48 = src->refs48;
                s->refs64 = src->refs64;
                s->wide_leaves = src->wide_leaves;
                s->ref_tri = src->ref_tri;
                s->tri_pos = src->tri_pos;
                s->tri_attr = src->tri_attr;
                s->mats = src->mats;
                s->texs = src->texs;
                s->tex_bytes = src->tex_bytes;
                s->info = src->info;
                s->level_begin = src->level_begin;
        } catch (const std::bad_alloc &) {
                return fail(VRT_E_NOMEM, "scene replica: out of host memory");
        }
        s->info.device = device;
        s->info.build_ms = 0;
        if (int rc = upload(s.get(), d)) {
                vrt_scene_destroy(s.release());
                return rc;
        }
        s->info.upload_ms = now_ms() - t0;
        *out = s.release();
        return VRT_OK;
}

extern "C" void vrt_scene_destroy(vrt_scene *s)
{
        if (!s)
                return;
        if (s->d_mem || s->ts[0].lm || s->ts[1].lm || s->d_light || s->ts[0].rec || s->ts[1].rec || s->d_spill[0] ||
            s->d_spill[1] || s->stream || s->ev0 || s->ev1 || s->ts[0].ev || s->ts[1].ev) {
                (void)hipSetDevice(s->device);
                if (s->stream)
                        (void)hipStreamSynchronize(s->stream);
                // launches on callers' streams: every work-queue slot, trace
                // set and compaction set records its last user's event
                for (int k = 0; k < kQueueSlots; ++k)
                        if (s->q_live[k])
                                (void)hipEventSynchronize(s->q_ev[k]);
                for (TraceSet &t : s->ts)
                        if (t.live)
                                (void)hipEventSynchronize(t.ev);
                for (int k = 0; k < 2; ++k)
                        if (s->spill_live[k])
                                (void)hipEventSynchronize(s->spill_ev[k]);
                if (s->d_mem)
                        (void)hipFree(s->d_mem);
                for (TraceSet &t : s->ts) {
                        if (t.lm)
                                (void)hipFree(t.lm);
                        if (t.rec)
                                (void)hipFree(t.rec);
                        if (t.ev)
                                (void)hipEventDestroy(t.ev);
                }
                if (s->d_light)
                        (void)hipFree(s->d_light);
                if (s->h_spill)
                        (void)hipHostFree(s->h_spill);
                for (int k = 0; k < 2; ++k) {
                        if (s->d_spill[k])
                                (void)hipFree(s->d_spill[k]);
                        if (s->spill_ev[k])
                                (void)hipEventDestroy(s->spill_ev[k]);
                        if (s->spill_side[k].st)
                                (void)hipStreamDestroy(s->spill_side[k].st);
                        if (s->spill_side[k].fork)
                                (void)hipEventDestroy(s->spill_side[k].fork);
                        if (s->spill_side[k].join)
                                (void)hipEventDestroy(s->spill_side[k].join);
                }
                for (auto &m : s->dmaps) {
                        (void)hipEventSynchronize(m.ev);
                        (void)hipEventDestroy(m.ev);
                        (void)hipFree(m.d);
                }
                if (s->ev0)
                        (void)hipEventDestroy(s->ev0);
                if (s->ev1)
                        (void)hipEventDestroy(s->ev1);
                for (int k = 0; k < kQueueSlots; ++k)
                        if (s->q_ev[k])
                                (void)hipEventDestroy(s->q_ev[k]);
                if (s->lm_ev)
                        (void)hipEventDestroy(s->lm_ev);
                HostOut &ho = s->ho;
                if (ho.st2)
                        (void)hipStreamSynchronize(ho.st2);
                if (ho.cp)
                        (void)hipStreamSynchronize(ho.cp);
                if (ho.d_img)
                        (void)hipFree(ho.d_img);
                if (ho.h_pin)
                        (void)hipHostFree(ho.h_pin);
                for (int b = 0; b < kOutBands; ++b) {
                        if (ho.ev_r[b])
                                (void)hipEventDestroy(ho.ev_r[b]);
                        if (ho.ev_c[b])
                                (void)hipEventDestroy(ho.ev_c[b]);
                }
                if (ho.ev_j)
                        (void)hipEventDestroy(ho.ev_j);
                if (ho.st2)
                        (void)hipStreamDestroy(ho.st2);
                if (ho.cp)
                        (void)hipStreamDestroy(ho.cp);
                if (s->d_rays)
                        (void)hipFree(s->d_rays);
                if (s->d_hits)
                        (void)hipFree(s->d_hits);
                if (s->h_rays)
                        (void)hipHostFree(s->h_rays);
                if (s->h_hits)
                        (void)hipHostFree(s->h_hits);
                if (s->stream)
                        (void)hipStreamDestroy(s->stream);
        }
        delete s;
}

extern "C" int vrt_scene_info(const vrt_scene *s, vrt_scene_info_t *info)
{
        if (!s || !info)
                return fail(VRT_E_INVALID, "null argument");
        *info = s->info;
        return VRT_OK;
}

extern "C" int vrt_scene_nodes(const vrt_scene *s, float *box, uint32_t *a, uint32_t *b)
{
        if (!s)
                return fail(VRT_E_INVALID, "null argument");
        for (size_t i = 0; i < s->nodes.size(); ++i) {
                const NodeRec &nr = s->nodes[i];
                if (box) {
                        std::memcpy(box + 6 * i, nr.bmin, 12);
                        std::memcpy(box + 6 * i + 3, nr.bmax, 12);
                }
                if (a)
                        a[i] = nr.a;
                if (b)
                        b[i] = nr.b;
        }
        return VRT_OK;
}

extern "C" int vrt_scene_leaves(const vrt_scene *s, uint32_t *voxel,
                                uint32_t *count, int32_t *tris)
{
        if (!s || !voxel || !count || !tris)
                return fail(VRT_E_INVALID, "null argument");
        std::vector<std::pair<uint32_t, size_t>> lv;
        for (size_t i = 0; i < s->nodes.size(); ++i) {
                const NodeRec &nr = s->nodes[i];
                if ((nr.a & kLeafBit) && (nr.a & ~kLeafBit))
                        lv.emplace_back(s->node_vox[i], i);
        }
        std::sort(lv.begin(), lv.end());
        size_t o = 0;
        for (size_t j = 0; j < lv.size(); ++j) {
                const NodeRec &nr = s->nodes[lv[j].second];
                const uint32_t n = nr.a & ~kLeafBit;
                voxel[j] = lv[j].first;
                count[j] = n;
                for (uint32_t k = 0; k < n; ++k)
                        tris[o++] = (int32_t)s->ref_tri[nr.b + k];
        }
        return VRT_OK;
}

// ---------------------------------------------------------------------------
// render
// ---------------------------------------------------------------------------
static int need_device(const vrt_scene *s)
{
        if (!s->d_mem)
                return fail(VRT_E_NODEVICE, "scene was created host-only (device < 0)");
        return VRT_OK;
}

static int film_ok(const vrt_film *f)
{
        if (!f || f->nx < 1 || f->ny < 1 || f->nx > 32768 || f->ny > 32768)
                return fail(VRT_E_INVALID, "bad film");
        return VRT_OK;
}

extern "C" int vrt_tiles_per_rank(const vrt_film *film, int nranks)
{
        if (film_ok(film) || nranks < 1)
                return 0;
        // the largest share of the tile deal (tile_deal, vrt_internal.h)
        const TileDeal d = tile_deal(film->nx / 8, film->ny / 8, nranks);
        int m = 0;
        for (int r = 0; r < nranks; ++r)
                m = std::max(m, deal_count(d, r));
        return m;
}

extern "C" int vrt_scene_set_frames_in_flight(vrt_scene *s, int n)
{
        if (!s || n < 1)
                return fail(VRT_E_INVALID, "bad argument");
        std::lock_guard<std::mutex> lk(s->mu);
        // measured: half the slots per frame with 2-3 frames
        // in flight; a third is slower, the whole chip per frame the same
        // (round 6, bench's own schedule)
        s->dev.grid_div = n >= 2 ? 2 : 1;
        return VRT_OK;
}

extern "C" int vrt_tile_deal_block(void)
{
        return VRT_DEAL_BLOCK;
}

extern "C" int vrt_tile_deal_map(const vrt_film *film, int nranks, int32_t *rank_of_tile, int32_t *slot_of_tile)
{
        if (int rc = film_ok(film))
                return rc;
        if (nranks < 1 || !rank_of_tile || !slot_of_tile)
                return fail(VRT_E_INVALID, "bad argument");
        const int ntx = film->nx / 8, nty = film->ny / 8;
        const TileDeal d = tile_deal(ntx, nty, nranks);
        for (int ty = 0; ty < nty; ++ty)
                for (int tx = 0; tx < ntx; ++tx) {
                        int r, k;
                        deal_slot(d, tx, ty, r, k);
                        rank_of_tile[ty * ntx + tx] = r;
                        slot_of_tile[ty * ntx + tx] = k;
                        // the forward map must invert it
                        int bx = -1, by = -1;
                        if (k < deal_count(d, r))
                                deal_tile(d, r, k, bx, by);
                        if (bx != tx || by != ty)
                                return fail(VRT_E_INVALID, "tile deal does not invert at (%d, %d)", tx, ty);
                }
        return VRT_OK;
}

static std::atomic<int> g_test_flags{0};

extern "C" int vrt_set_test_flags(int flags)
{
        g_test_flags.store(flags);
        return VRT_OK;
}

int vrt::test_flags() { return g_test_flags.load(); }

extern "C" int vrt_test_flags(void) { return g_test_flags.load(); }

extern "C" int vrt_build_flag(const char *name, int64_t *value)
{
        if (!name || !value)
                return fail(VRT_E_INVALID, "null argument");
        if (!build_flag(name, value))
                return fail(VRT_E_INVALID, "unknown build flag %s", name);
        return VRT_OK;
}

static void fill_render_params(vrt_scene *s, const vrt_camera *cam,
                               const vrt_film *film, int rank, int nranks,
                               RenderParams *p)
{
        std::memset(p, 0, sizeof *p);
        p->sc = s->dev;
        fill_cam_params(cam, film, &p->cam);
        p->ntx = film->nx / 8;
        p->nty = film->ny / 8;
        p->rank = rank;
        p->nranks = nranks;
        p->tiles_this_rank = deal_count(tile_deal(p->ntx, p->nty, nranks), rank);
        // k * ceil(2^40 / ntx) >> 40 == k / ntx for k < 2^40 / ntx, which
        // k < 2^24 and ntx < 2^16 guarantee
        if (p->ntx > 0 && p->ntx < (1 << 16) && (int64_t)p->ntx * p->nty < ((int64_t)1 << 24))
                p->ntx_magic = (((uint64_t)1 << 40) + (uint64_t)p->ntx - 1) / (uint64_t)p->ntx;
        p->test_flags = g_test_flags.load();
}

static float scene_res(const vrt_scene *s);

// Work-queue ring (WorkQueue, vrt_internal.h; caller holds s->mu).  A
// persistent launch takes the next slot: its stream first waits for the
// slot's previous launch (on whatever stream it ran), the kernel takes its
// units from base[] on, and the slot's bases advance by exactly the adds the
// launch makes.
static int queue_take(vrt_scene *s, hipStream_t st, WorkQueue *q, int *slot)
{
        *slot = s->q_next;
        s->q_next = (*slot + 1) % kQueueSlots;
        if (s->q_live[*slot])
                HIPCHK(hipStreamWaitEvent(st, s->q_ev[*slot], 0));
        q->ctr = s->d_queue + (size_t)*slot * kQueueWords;
        q->defer = q->ctr + 8 * kQueueStride;
        std::memcpy(q->base, s->q_base[*slot], sizeof q->base);
        return VRT_OK;
}

static int queue_release(vrt_scene *s, int slot, hipStream_t st, const int slice_units[8], int waves)
{
        for (int x = 0; x < 8; ++x)
                if (slice_units[x] > 0)
                        s->q_base[slot][x] += (uint32_t)slice_units[x] + (uint32_t)waves;
        HIPCHK(hipEventRecord(s->q_ev[slot], st));
        s->q_live[slot] = true;
        return VRT_OK;
}

// A launch failed after taking `slot`: whatever part of it was enqueued runs
// before this memset (same stream), then the slot restarts from zero
// counters, zero bases and an empty deferred list -- so a failed launch
// never leaves a slot whose bases disagree with its counters (every later
// launch on it would otherwise find its queue already drained).
static void queue_reset(vrt_scene *s, int slot, hipStream_t st)
{
        (void)hipMemsetAsync(s->d_queue + (size_t)slot * kQueueWords, 0, kQueueBytes, st);
        std::memset(s->q_base[slot], 0, sizeof s->q_base[slot]);
        if (hipEventRecord(s->q_ev[slot], st) == hipSuccess)
                s->q_live[slot] = true;
}

// One render launch on stream st (caller holds s->mu).
static int render_launch(vrt_scene *s, RenderParams &p, bool instrumented, hipStream_t st)
{
        int slot = -1;
        (void)hipGetLastError();  // a leftover error of an earlier call is not this launch's
        if (render_kind(p, instrumented) != kRenderGrid) {
                if (int rc = queue_take(s, st, &p.q, &slot))
                        return rc;
        }
        int waves = 0, units[8];
        const hipError_t e = launch_render(p, instrumented, st, &waves, units);
        if (e != hipSuccess) {
                if (slot >= 0)
                        queue_reset(s, slot, st);
                return fail(VRT_E_DEVICE, "render launch failed: %s", hipGetErrorString(e));
        }
        if (slot >= 0)
                return queue_release(s, slot, st, units, waves);
        return VRT_OK;
}

static int ts_acquire(vrt_scene *s, int i, hipStream_t st);
static int ts_release(vrt_scene *s, int i, hipStream_t st);

// Compaction queue of one config-5 launch (SpillQueues).  Its
// size is an estimate: when the queue is full, the rays that stop finish
// their walks in place (spill_room), so any size gives the same images.  The
// first launch sizes queue 0 for 1/32 of the rank's secondary rays (1080p:
// 4.1 M 64-B records, 0.26 GB) plus one partly filled chunk per resident
// wave; after every launch its counters are copied to pinned memory, and a
// later launch sizes for 1.25 x the records its phase A stopped (queued +
// finished in place), growing, never shrinking, and never past 1 GiB per set.
// Only queue 0's records are allocated: the one pooled resume round walks
// every saved ray to its end (queue 1's fill words list the streaming round's
// leftover chunks).  The scene keeps two sets; a stream keeps using the set
// it used last (stream order protects it), an idle set is shared, and a
// second set is allocated only for frames in flight on two streams (the new
// stream waits for the set's last user's event).  sq->nchunks stays 0 (no
// compaction) when the build disables it, the film has 2^26 pixels or more,
// the octree 2^24 nodes or more (SpillRec's packed words), or the allocation
// fails.
// chunks: the records, their two fill words, the counters and the deferred-
// pixel list (dpb bytes) within 1 GiB
static uint32_t spill_cap_max(size_t dpb)
{
        return (uint32_t)((((size_t)1 << 30) - 4096 - dpb) / ((size_t)kSpillChunk * sizeof(SpillRec) + 8));
}
static size_t spill_dpix_bytes(int64_t pixels)
{
        return ((size_t)pixels * 4 + 255) & ~(size_t)255;
}
static size_t spill_set_bytes(uint32_t nch, int64_t pixels)
{
        const size_t fb = ((size_t)nch * 4 + 255) & ~(size_t)255;
        return (size_t)kSpillMaxRounds * kSpillCtrStride * 4 + 2 * fb + (size_t)nch * kSpillChunk * sizeof(SpillRec) +
               spill_dpix_bytes(pixels);
}
static int spill_setup(vrt_scene *s, int64_t rays, int64_t pixels, hipStream_t st, SpillQueues *sq, int *set)
{
        *sq = spill_defaults();
        *set = -1;
        // SpillRec packs the pixel in 26 bits and a stack entry's block in 24
        if (sq->t_first == 0 || rays <= 0 || pixels >= (int64_t)1 << 26 || s->nodes.size() >= ((size_t)1 << 24))
                return VRT_OK;
        // this stream's own set; else an allocated set whose last launch has
        // finished (a second set is allocated only for frames in flight on
        // two streams); else the next one
        int k = -1;
        for (int i = 0; i < 2 && k < 0; ++i)
                if (s->spill_live[i] && s->spill_stream[i] == st)
                        k = i;
        for (int i = 0; i < 2 && k < 0; ++i)
                if (s->d_spill[i] && (!s->spill_live[i] || hipEventQuery(s->spill_ev[i]) == hipSuccess))
                        k = i;
        if (k < 0) {
                k = s->spill_next;
                s->spill_next ^= 1;
        }
        if (!s->spill_ev[k])
                HIPCHK(hipEventCreateWithFlags(&s->spill_ev[k], hipEventDisableTiming));
        if (!s->spill_side[k].st) {
                // all three or none (a set without a side stream runs the
                // deferred walk on the launch's stream)
                SideLaunch sl{};
                if (hipEventCreateWithFlags(&sl.fork, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&sl.join, hipEventDisableTiming) == hipSuccess &&
                    hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking) == hipSuccess) {
                        s->spill_side[k] = sl;
                } else {
                        (void)hipGetLastError();
                        if (sl.fork)
                                (void)hipEventDestroy(sl.fork);
                        if (sl.join)
                                (void)hipEventDestroy(sl.join);
                }
        }
        if (!s->h_spill) {
                HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&s->h_spill), 16 * sizeof(uint32_t),
                                     hipHostMallocDefault));
                std::memset(s->h_spill, 0, 16 * sizeof(uint32_t));
        }
        // the deferred-pixel list holds one entry per pixel of the film
        const int64_t px = std::max<int64_t>(pixels, s->spill_px[k]);
        const uint32_t cap_max = spill_cap_max(spill_dpix_bytes(px));
        // what the finished launches of either set stopped: records queued
        // (ctr[2]) + records finished in place for want of room (ctr[5])
        for (int i = 0; i < 2; ++i)
                if (s->spill_live[i] && s->spill_cap[i] && hipEventQuery(s->spill_ev[i]) == hipSuccess) {
                        const uint64_t need = (uint64_t)s->h_spill[8 * i + 2] + s->h_spill[8 * i + 5];
                        const uint64_t w = (need * 5 / 4 + kSpillChunk - 1) / kSpillChunk;
                        s->spill_want = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(s->spill_want, w), cap_max);
                }
        if (s->spill_live[k] && s->spill_stream[k] != st)
                HIPCHK(hipStreamWaitEvent(st, s->spill_ev[k], 0));
        // + one partly filled chunk per wave of a resident grid
        const int64_t partial = (int64_t)std::max(1, s->dev.sec_blocks) * 4;
        const int64_t est = s->spill_want ? (int64_t)s->spill_want : (rays / 32 + kSpillChunk - 1) / kSpillChunk;
        const uint32_t nch = (uint32_t)std::min<int64_t>(std::min<int64_t>(est, (rays + kSpillChunk - 1) / kSpillChunk) +
                                                                 partial, cap_max);
        const size_t ctr_bytes = (size_t)kSpillMaxRounds * kSpillCtrStride * 4;
        if (s->spill_cap[k] < nch || s->spill_px[k] < pixels) {
                // a regrowth for a larger film keeps the chunks it had
                const uint32_t c = std::min(std::max(nch, s->spill_cap[k]), cap_max);
                if (s->d_spill[k]) {
                        // the set's users on any stream are ordered by its event
                        // (spill_done after each, a stream wait when a set
                        // changes stream): the last one's event covers them all
                        if (s->spill_live[k])
                                HIPCHK(hipEventSynchronize(s->spill_ev[k]));
                        (void)hipFree(s->d_spill[k]);
                        s->d_spill[k] = nullptr;
                        s->spill_cap[k] = 0;
                        s->spill_px[k] = 0;
                }
                if (hipMalloc(&s->d_spill[k], spill_set_bytes(c, px)) != hipSuccess) {
                        (void)hipGetLastError();
                        s->d_spill[k] = nullptr;
                        return VRT_OK;  // no compaction
                }
                s->spill_cap[k] = c;
                s->spill_px[k] = px;
        }
        const size_t fb = ((size_t)s->spill_cap[k] * 4 + 255) & ~(size_t)255;
        char *b = static_cast<char *>(s->d_spill[k]);
        sq->ctr = reinterpret_cast<uint32_t *>(b);
        sq->fill[0] = reinterpret_cast<uint32_t *>(b + ctr_bytes);
        sq->fill[1] = reinterpret_cast<uint32_t *>(b + ctr_bytes + fb);
        sq->rec[0] = reinterpret_cast<SpillRec *>(b + ctr_bytes + 2 * fb);
        sq->rec[1] = nullptr;  // the pooled resume round stops no ray
        sq->nchunks = s->spill_cap[k];
        sq->dpix = reinterpret_cast<uint32_t *>(b + ctr_bytes + 2 * fb +
                                                (size_t)s->spill_cap[k] * kSpillChunk * sizeof(SpillRec));
        HIPCHK(hipMemsetAsync(sq->ctr, 0, ctr_bytes, st));
        *set = k;
        return VRT_OK;
}

// After a config-5 launch with compaction set k on st: its counters to
// pinned memory (spill_setup reads them once the set's event has passed) and
// the set's event.
static int spill_done(vrt_scene *s, int k, const SpillQueues &sq, hipStream_t st)
{
        HIPCHK(hipMemcpyAsync(s->h_spill + 8 * k, sq.ctr, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(s->spill_ev[k], st));
        s->spill_live[k] = true;
        s->spill_stream[k] = st;
        return VRT_OK;
}

// One config-5 launch (k_primary1 + secondary rays) on stream st (caller
// holds s->mu).
static int secondary_launch(vrt_scene *s, const RenderParams &p, int spp, int rank, int nranks, float *d_prim,
                            float *d_vis, int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox, hipStream_t st)
{
        int slot = -1;
        WorkQueue q;
        std::memset(&q, 0, sizeof q);
        (void)hipGetLastError();  // a leftover error of an earlier call is not this launch's
        SpillQueues sq;
        std::memset(&sq, 0, sizeof sq);
        int set = -1;
        if (secondary_uses_queue(p.sc)) {
                if (int rc = queue_take(s, st, &q, &slot))
                        return rc;
                if (!s_tri && !s_vox) {  // the occlusion walk: compaction
                        const int64_t rays = deal_count(tile_deal(p.ntx, p.nty, nranks), rank) * 64 * (int64_t)spp;
                        if (int rc = spill_setup(s, rays, (int64_t)p.ntx * 8 * p.nty * 8, st, &sq, &set))
                                return rc;
                }
        }
        int waves = 0, units[8];
        s->spill_last = sq.nchunks > 0 ? set : -1;
        const hipError_t e = launch_secondary(p, spp, rank, nranks, scene_res(s), d_prim, d_vis, s_hit, s_tri,
                                              s_vox, slot >= 0 ? &q : nullptr, st, &waves, units, &sq,
                                              set >= 0 && s->spill_side[set].st ? &s->spill_side[set] : nullptr);
        if (set >= 0)
                if (int rc = spill_done(s, set, sq, st))
                        return rc;
        if (e != hipSuccess) {
                if (slot >= 0)
                        queue_reset(s, slot, st);
                return fail(VRT_E_DEVICE, "secondary launch failed: %s", hipGetErrorString(e));
        }
        if (slot >= 0)
                return queue_release(s, slot, st, units, waves);
        return VRT_OK;
}

// A trace scratch set (vrt_scene::ts) serves one user at a time: the next
// user's stream waits for the previous user's (caller holds s->mu).
static int ts_acquire(vrt_scene *s, int i, hipStream_t st)
{
        if (s->ts[i].live)
                HIPCHK(hipStreamWaitEvent(st, s->ts[i].ev, 0));
        return VRT_OK;
}

static int ts_release(vrt_scene *s, int i, hipStream_t st)
{
        HIPCHK(hipEventRecord(s->ts[i].ev, st));
        s->ts[i].live = true;
        return VRT_OK;
}

// set i's light-map block (nodes x (LMRec + float4) + the flag word)
// Per node, the cell a cone march's descent to it implies (TraceParams::
// cells): the root's is all of space; a child's is its parent's cut at the
// parent's box centre (AABB3D::center, as k_lm_aux computes it) on the side
// of the child's octant -- per axis the tightest (lo, hi] the descent's
// `pt > centre` choices establish.
static std::vector<float4> cone_cells(const std::vector<NodeRec> &nodes)
{
        const float inf = std::numeric_limits<float>::infinity();
        std::vector<float4> c(2 * nodes.size());
        if (nodes.empty())
                return c;
        c[0] = make_float4(-inf, -inf, -inf, 0.f);
        c[1] = make_float4(inf, inf, inf, 0.f);
        for (size_t i = 0; i < nodes.size(); ++i) {  // BFS order: parents first
                const NodeRec &nr = nodes[i];
                if (nr.a & kLeafBit)
                        continue;
                const float cx = (nr.bmin[0] + nr.bmax[0]) * .5f, cy = (nr.bmin[1] + nr.bmax[1]) * .5f,
                            cz = (nr.bmin[2] + nr.bmax[2]) * .5f;
                for (uint32_t o = 0; o < 8; ++o) {
                        float4 lo = c[2 * i], hi = c[2 * i + 1];
                        if (o & 4) lo.x = std::max(lo.x, cx); else hi.x = std::min(hi.x, cx);
                        if (o & 2) lo.y = std::max(lo.y, cy); else hi.y = std::min(hi.y, cy);
                        if (o & 1) lo.z = std::max(lo.z, cz); else hi.z = std::min(hi.z, cz);
                        c[2 * (size_t)(nr.a + o)] = lo;
                        c[2 * (size_t)(nr.a + o) + 1] = hi;
                }
        }
        return c;
}

// Trace set i's block: light map, cone-descent records, finiteness flag
// (256 B), then the nodes' cone cells (static, filled on allocation).
// One trace set's light-map block: the light map (LMRec per node), the
// cone-descent records (float4 per node), the non-finite flag (256 B) and the
// per-node cells (2 float4 per node)
static size_t lm_set_bytes(size_t n)
{
        return n * (sizeof(LMRec) + sizeof(float4)) + 256 + n * 2 * sizeof(float4);
}

static int ensure_lm(vrt_scene *s, int i)
{
        if (!s->ts[i].lm) {
                const size_t n = s->nodes.size();
                HIPCHK(hipMalloc(reinterpret_cast<void **>(&s->ts[i].lm), lm_set_bytes(n)));
                const std::vector<float4> cells = cone_cells(s->nodes);
                HIPCHK(hipMemcpy(reinterpret_cast<char *>(s->ts[i].lm) + n * (sizeof(LMRec) + sizeof(float4)) + 256,
                                 cells.data(), cells.size() * sizeof(float4), hipMemcpyHostToDevice));
        }
        return VRT_OK;
}

// The rank's tabled deal (RenderParams::tile_xy) for nranks > 1, built on
// first use on stream st; a stream other than the builder's waits for the
// build.  nullptr (the kernels then compute the deal): one rank, tile grids
// of 2^16 or more, more than kDealMaps deals in use, or no memory.
constexpr size_t kDealMaps = 32;
static const uint32_t *deal_map(vrt_scene *s, int ntx, int nty, int nranks, int rank, hipStream_t st)
{
        if (nranks <= 1 || ntx >= 65536 || nty >= 65536)
                return nullptr;
        for (auto &m : s->dmaps)
                if (m.ntx == ntx && m.nty == nty && m.nranks == nranks && m.rank == rank) {
                        if (hipEventQuery(m.ev) != hipSuccess && hipStreamWaitEvent(st, m.ev, 0) != hipSuccess) {
                                (void)hipGetLastError();
                                return nullptr;
                        }
                        return m.d;
                }
        const int n = deal_count(tile_deal(ntx, nty, nranks), rank);
        if (n <= 0 || s->dmaps.size() >= kDealMaps)
                return nullptr;
        vrt_scene::DealMap m{ ntx, nty, nranks, rank, nullptr, nullptr };
        if (hipMalloc(reinterpret_cast<void **>(&m.d), (size_t)n * sizeof(uint32_t)) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
        }
        if (hipEventCreateWithFlags(&m.ev, hipEventDisableTiming) != hipSuccess ||
            launch_deal_map(ntx, nty, nranks, rank, m.d, st) != hipSuccess || hipEventRecord(m.ev, st) != hipSuccess) {
                (void)hipGetLastError();
                // a launch that got as far as the stream finishes before the free
                (void)hipStreamSynchronize(st);
                if (m.ev)
                        (void)hipEventDestroy(m.ev);
                (void)hipFree(m.d);
                return nullptr;
        }
        try {
                s->dmaps.push_back(m);
        } catch (const std::bad_alloc &) {
                (void)hipEventSynchronize(m.ev);
                (void)hipEventDestroy(m.ev);
                (void)hipFree(m.d);
                return nullptr;
        }
        return m.d;
}

extern "C" int vrt_render_tiles_device(vrt_scene *s, const vrt_camera *cam,
                                       const vrt_film *film, int rank,
                                       int nranks, int image_layout,
                                       float *d_out, void *stream)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !cam || !d_out)
                return fail(VRT_E_INVALID, "null argument");
        if (int rc = film_ok(film))
                return rc;
        if (nranks < 1 || rank < 0 || rank >= nranks)
                return fail(VRT_E_INVALID, "rank %d of %d", rank, nranks);
        if (image_layout && nranks != 1)
                return fail(VRT_E_INVALID, "image_layout requires nranks == 1");
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        RenderParams p;
        fill_render_params(s, cam, film, rank, nranks, &p);
        p.image_layout = image_layout;
        p.out = d_out;
        hipStream_t st = static_cast<hipStream_t>(stream);
        p.tile_xy = deal_map(s, p.ntx, p.nty, nranks, rank, st);
        HIPCHK(hipEventRecord(s->ev0, st));
        if (int rc = render_launch(s, p, false, st))
                return rc;
        HIPCHK(hipEventRecord(s->ev1, st));
        s->timed = true;
        return VRT_OK;
}

extern "C" int vrt_last_kernel_ms(vrt_scene *s, float *ms)
{
        if (!s || !ms)
                return fail(VRT_E_INVALID, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        if (!s->timed)
                return fail(VRT_E_INVALID, "no timed launch yet");
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipEventSynchronize(s->ev1));
        HIPCHK(hipEventElapsedTime(ms, s->ev0, s->ev1));
        return VRT_OK;
}

extern "C" int vrt_unpack_tiles_device(const vrt_film *film, int nranks,
                                       const float *d_gathered, float *d_image,
                                       void *stream)
{
        if (!d_gathered || !d_image || nranks < 1)
                return fail(VRT_E_INVALID, "bad argument");
        if (int rc = film_ok(film))
                return rc;
        const int tpr = vrt_tiles_per_rank(film, nranks);
        HIPCHK(launch_unpack(film->nx, film->ny, film->nx / 8, film->ny / 8, nranks, tpr,
                             d_gathered, d_image, static_cast<hipStream_t>(stream)));
        return VRT_OK;
}

extern "C" int vrt_pack_tiles_c_device(const vrt_film *film, int rank, int nranks, int comps, const float *d_image,
                                       float *d_packed, void *stream)
{
        if (!d_image || !d_packed || nranks < 1 || rank < 0 || rank >= nranks || comps < 1 || comps > 4)
                return fail(VRT_E_INVALID, "bad argument");
        if (int rc = film_ok(film))
                return rc;
        HIPCHK(launch_pack_c(film->nx, film->ny, rank, nranks, comps, d_image, d_packed,
                             static_cast<hipStream_t>(stream)));
        return VRT_OK;
}

extern "C" int vrt_unpack_tiles_c_device(const vrt_film *film, int nranks, int comps, const float *d_gathered,
                                         float *d_image, void *stream)
{
        if (!d_gathered || !d_image || nranks < 1 || comps < 1 || comps > 4)
                return fail(VRT_E_INVALID, "bad argument");
        if (int rc = film_ok(film))
                return rc;
        HIPCHK(launch_unpack_c(film->nx, film->ny, nranks, vrt_tiles_per_rank(film, nranks), comps, d_gathered,
                               d_image, static_cast<hipStream_t>(stream)));
        return VRT_OK;
}

extern "C" int vrt_rgbe_device(const float *d_img, int w, int h, int comp, uint8_t *d_rgbe, void *stream)
{
        if (!d_img || !d_rgbe || w <= 0 || h <= 0 || comp < 1 || comp > 4)
                return fail(VRT_E_INVALID, "vrt_rgbe_device: bad argument");
        HIPCHK(launch_rgbe(d_img, (int64_t)w * h, comp, d_rgbe, static_cast<hipStream_t>(stream)));
        return VRT_OK;
}

namespace {
struct DevBuf {
        void *p = nullptr;
        ~DevBuf()
        {
                if (p)
                        (void)hipFree(p);
        }
};
}  // namespace

// memcpy of a large host range split over up to 4 threads (pinned staging
// <-> the caller's pageable arrays: one core's memcpy is well below PCIe)
void vrt::par_memcpy(void *dst, const void *src, size_t bytes)
{
        const int nth = bytes >= ((size_t)4 << 20) ? 4 : 1;
        if (nth == 1) {
                std::memcpy(dst, src, bytes);
                return;
        }
        auto part = [&](int j) {
                const size_t a = (bytes * j / nth) & ~(size_t)63, b = j + 1 == nth ? bytes : (bytes * (j + 1) / nth) & ~(size_t)63;
                std::memcpy(static_cast<char *>(dst) + a, static_cast<const char *>(src) + a, b - a);
        };
        std::vector<std::thread> th;
        for (int j = 1; j < nth; ++j)
                th.emplace_back(part, j);
        part(0);
        for (auto &t : th)
                t.join();
}

// vrt_render into a host array (no per-sample outputs): the device image and
// a pinned staging copy are kept in the scene; the frame is rendered as
// kOutBands tile-row bands alternating over two streams (half-chip grids, so
// a band's ramp-down runs beside the next band), each band copied D2H into
// the pinned buffer on a copy stream as soon as it is rendered, and copied
// on to `rgb` by up to 4 host threads as its copy lands.  The same kernels
// and pixels as the one-launch render (a pixel's value does not depend on
// the launch it belongs to).  Caller holds s->mu, device set.
static int render_to_host(vrt_scene *s, const vrt_camera *cam, const vrt_film *film, float *rgb)
{
        HostOut &ho = s->ho;
        const int nx = film->nx, ny = film->ny, ntx = nx / 8, nty = ny / 8;
        const size_t bytes = (size_t)nx * ny * 12;
        if (ntx == 0 || nty == 0) {  // no 8x8 tile: render_mt renders nothing
                std::memset(rgb, 0, bytes);
                return VRT_OK;
        }
        if (!ho.st2) {
                HIPCHK(hipStreamCreateWithFlags(&ho.st2, hipStreamNonBlocking));
                HIPCHK(hipStreamCreateWithFlags(&ho.cp, hipStreamNonBlocking));
                for (int b = 0; b < kOutBands; ++b) {
                        HIPCHK(hipEventCreateWithFlags(&ho.ev_r[b], hipEventDisableTiming));
                        HIPCHK(hipEventCreateWithFlags(&ho.ev_c[b], hipEventDisableTiming));
                }
                HIPCHK(hipEventCreateWithFlags(&ho.ev_j, hipEventDisableTiming));
        }
        if (ho.nx != nx || ho.ny != ny) {
                if (ho.bytes < bytes) {
                        HIPCHK(hipStreamSynchronize(ho.cp));
                        if (ho.d_img)
                                (void)hipFree(ho.d_img);
                        if (ho.h_pin)
                                (void)hipHostFree(ho.h_pin);
                        ho.d_img = nullptr;
                        ho.h_pin = nullptr;
                        ho.bytes = 0;
                        HIPCHK(hipMalloc(&ho.d_img, bytes));
                        HIPCHK(hipHostMalloc(&ho.h_pin, bytes, hipHostMallocDefault));
                        ho.bytes = bytes;
                }
                // pixels outside the tile grid are never written: zero once per film shape
                HIPCHK(hipMemsetAsync(ho.d_img, 0, bytes, s->stream));
                ho.nx = nx;
                ho.ny = ny;
        }
        const int nb = std::min(kOutBands, nty);
        HIPCHK(hipEventRecord(s->ev0, s->stream));
        HIPCHK(hipEventRecord(ho.ev_j, s->stream));
        HIPCHK(hipStreamWaitEvent(ho.st2, ho.ev_j, 0));
        size_t off[kOutBands + 1];
        for (int b = 0; b < nb; ++b) {
                const int r0 = b * nty / nb, r1 = (b + 1) * nty / nb;
                hipStream_t st = (b & 1) ? ho.st2 : s->stream;
                RenderParams p;
                fill_render_params(s, cam, film, 0, 1, &p);
                p.nty = r1 - r0;
                p.ty0 = r0;
                p.tiles_this_rank = ntx * (r1 - r0);
                p.sc.grid_div = nb > 1 ? 2 : 1;
                p.image_layout = 1;
                p.out = ho.d_img;
                if (int rc = render_launch(s, p, false, st))
                        return rc;
                HIPCHK(hipEventRecord(ho.ev_r[b], st));
                HIPCHK(hipStreamWaitEvent(ho.cp, ho.ev_r[b], 0));
                // band b's rows (the last band also carries the rows below the grid)
                off[b] = b == 0 ? 0 : (size_t)8 * r0 * nx * 12;
                off[b + 1] = b + 1 == nb ? bytes : (size_t)8 * r1 * nx * 12;
                HIPCHK(hipMemcpyAsync(reinterpret_cast<char *>(ho.h_pin) + off[b],
                                      reinterpret_cast<const char *>(ho.d_img) + off[b], off[b + 1] - off[b],
                                      hipMemcpyDeviceToHost, ho.cp));
                HIPCHK(hipEventRecord(ho.ev_c[b], ho.cp));
        }
        HIPCHK(hipEventRecord(ho.ev_j, ho.st2));
        HIPCHK(hipStreamWaitEvent(s->stream, ho.ev_j, 0));
        HIPCHK(hipEventRecord(s->ev1, s->stream));
        s->timed = true;
        // copy-out: band b as soon as its D2H copy has landed
        std::atomic<bool> bad{ false };
        const int nth = bytes >= ((size_t)4 << 20) ? 4 : 1;
        auto work = [&](int j) {
                for (int b = 0; b < nb; ++b) {
                        if (hipEventSynchronize(ho.ev_c[b]) != hipSuccess) {
                                bad = true;
                                return;
                        }
                        const size_t n = off[b + 1] - off[b];
                        const size_t a = off[b] + ((n * j / nth) & ~(size_t)63);
                        const size_t e = j + 1 == nth ? off[b + 1] : off[b] + ((n * (j + 1) / nth) & ~(size_t)63);
                        std::memcpy(reinterpret_cast<char *>(rgb) + a, reinterpret_cast<const char *>(ho.h_pin) + a,
                                    e - a);
                }
        };
        std::vector<std::thread> th;
        for (int j = 1; j < nth; ++j)
                th.emplace_back(work, j);
        work(0);
        for (auto &t : th)
                t.join();
        HIPCHK(hipStreamSynchronize(s->stream));
        if (bad)
                return fail(VRT_E_DEVICE, "vrt_render: device-to-host copy failed");
        return VRT_OK;
}

extern "C" int vrt_render(vrt_scene *s, const vrt_camera *cam,
                          const vrt_film *film, float *rgb,
                          const vrt_samples *samples, vrt_stats *stats)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !cam || !rgb)
                return fail(VRT_E_INVALID, "null argument");
        if (int rc = film_ok(film))
                return rc;
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        const bool no_samples = !samples || !(samples->hit || samples->tri || samples->voxel || samples->rgb ||
                                              samples->counters);
        if (no_samples && !stats)
                return render_to_host(s, cam, film, rgb);
        const size_t npix = (size_t)film->nx * film->ny;
        const size_t ns = npix * 4;
        const bool want_cnt = (samples && samples->counters) || stats;
        DevBuf img, shit, stri, svox, srgb, scnt;
        HIPCHK(hipMalloc(&img.p, npix * 3 * sizeof(float)));
        HIPCHK(hipMemsetAsync(img.p, 0, npix * 3 * sizeof(float), s->stream));
        RenderParams p;
        fill_render_params(s, cam, film, 0, 1, &p);
        p.sc.grid_div = 1;  // synchronous: one frame at a time, the whole chip
        p.image_layout = 1;
        p.out = static_cast<float *>(img.p);
        auto alloc_fill = [&](DevBuf &b, size_t bytes, int byte) -> hipError_t {
                hipError_t e = hipMalloc(&b.p, bytes);
                if (e != hipSuccess)
                        return e;
                return hipMemsetAsync(b.p, byte, bytes, s->stream);
        };
        if (samples && samples->hit) {
                HIPCHK(alloc_fill(shit, ns * 4, 0));
                p.so.hit = static_cast<int32_t *>(shit.p);
        }
        if (samples && samples->tri) {
                HIPCHK(alloc_fill(stri, ns * 4, 0xFF));
                p.so.tri = static_cast<int32_t *>(stri.p);
        }
        if (samples && samples->voxel) {
                HIPCHK(alloc_fill(svox, ns * 4, 0xFF));
                p.so.vox = static_cast<uint32_t *>(svox.p);
        }
        if (samples && samples->rgb) {
                HIPCHK(alloc_fill(srgb, ns * 12, 0));
                p.so.rgb = static_cast<float *>(srgb.p);
        }
        if (want_cnt) {
                HIPCHK(alloc_fill(scnt, ns * 16, 0));
                p.so.cnt = static_cast<uint32_t *>(scnt.p);
        }
        HIPCHK(hipEventRecord(s->ev0, s->stream));
        if (int rc = render_launch(s, p, want_cnt, s->stream))
                return rc;
        HIPCHK(hipEventRecord(s->ev1, s->stream));
        s->timed = true;
        HIPCHK(hipStreamSynchronize(s->stream));
        HIPCHK(hipMemcpy(rgb, img.p, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
        if (p.so.hit)
                HIPCHK(hipMemcpy(samples->hit, shit.p, ns * 4, hipMemcpyDeviceToHost));
        if (p.so.tri)
                HIPCHK(hipMemcpy(samples->tri, stri.p, ns * 4, hipMemcpyDeviceToHost));
        if (p.so.vox)
                HIPCHK(hipMemcpy(samples->voxel, svox.p, ns * 4, hipMemcpyDeviceToHost));
        if (p.so.rgb)
                HIPCHK(hipMemcpy(samples->rgb, srgb.p, ns * 12, hipMemcpyDeviceToHost));
        std::vector<uint32_t> cnt;
        if (want_cnt) {
                cnt.resize(ns * 4);
                HIPCHK(hipMemcpy(cnt.data(), scnt.p, ns * 16, hipMemcpyDeviceToHost));
                if (samples && samples->counters)
                        std::memcpy(samples->counters, cnt.data(), ns * 16);
        }
        if (stats) {
                std::memset(stats, 0, sizeof *stats);
                const int W8 = 8 * (film->nx / 8), H8 = 8 * (film->ny / 8);
                for (int py = 0; py < H8; ++py)
                        for (int px = 0; px < W8; ++px)
                                for (int q = 0; q < 4; ++q) {
                                        const uint32_t *c = &cnt[(((size_t)py * film->nx + px) * 4 + q) * 4];
                                        stats->rays++;
                                        stats->aabb_tests += c[0];
                                        stats->leaves += c[1];
                                        stats->tri_tests += c[2];
                                        stats->hits += c[3];
                                }
                float ms = 0.f;
                HIPCHK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
                stats->kernel_ms = ms;
        }
        return VRT_OK;
}

// Res = *min_element(root.aabb.size() / powf(2, max_depth)) (VRT/main.cc:69-70)
static float scene_res(const vrt_scene *s)
{
        const float p2 = std::pow(2.f, (float)s->max_depth);
        float res = 0.f;
        for (int k = 0; k < 3; ++k) {
                const float v = (s->info.root_max[k] - s->info.root_min[k]) / p2;
                if (k == 0 || v < res)
                        res = v;
        }
        return res;
}

extern "C" int vrt_render_secondary_device(vrt_scene *s, const vrt_camera *cam,
                                           const vrt_film *film, int spp,
                                           int rank, int nranks, float *d_prim,
                                           float *d_vis, void *stream)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !cam || !d_prim || !d_vis || spp < 1 || spp > 64)
                return fail(VRT_E_INVALID, "bad argument (spp must be 1..64)");
        if (int rc = film_ok(film))
                return rc;
        if (nranks < 1 || rank < 0 || rank >= nranks)
                return fail(VRT_E_INVALID, "rank %d of %d", rank, nranks);
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        RenderParams p;
        fill_render_params(s, cam, film, 0, 1, &p);
        hipStream_t st = static_cast<hipStream_t>(stream);
        // the secondary rays' share (the primary pass covers every pixel)
        p.tile_xy = deal_map(s, p.ntx, p.nty, nranks, rank, st);
        HIPCHK(hipEventRecord(s->ev0, st));
        if (int rc = secondary_launch(s, p, spp, rank, nranks, d_prim, d_vis, nullptr, nullptr, nullptr, st))
                return rc;
        HIPCHK(hipEventRecord(s->ev1, st));
        s->timed = true;
        return VRT_OK;
}

extern "C" int vrt_scene_scratch_bytes(vrt_scene *s, int64_t *bytes, int64_t *spill_bytes)
{
        if (!s || !bytes)
                return fail(VRT_E_INVALID, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        int64_t sp = 0;
        for (int k = 0; k < 2; ++k)
                if (s->d_spill[k])
                        sp += (int64_t)spill_set_bytes(s->spill_cap[k], s->spill_px[k]);
        int64_t t = sp + (int64_t)s->light_bytes + (int64_t)s->ho.bytes;
        for (const TraceSet &ts : s->ts) {
                if (ts.lm)
                        t += (int64_t)lm_set_bytes(s->nodes.size());
                t += (int64_t)ts.rec_bytes;
        }
        for (const auto &m : s->dmaps)  // the tabled multi-rank deals
                t += (int64_t)deal_count(tile_deal(m.ntx, m.nty, m.nranks), m.rank) * (int64_t)sizeof(uint32_t);
        *bytes = t;
        if (spill_bytes)
                *spill_bytes = sp;
        return VRT_OK;
}

extern "C" int vrt_secondary_spill_counts(vrt_scene *s, int64_t counts[4])
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !counts)
                return fail(VRT_E_INVALID, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        for (int r = 0; r < 4; ++r)
                counts[r] = 0;
        if (s->spill_last < 0 || !s->d_spill[s->spill_last])
                return VRT_OK;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipEventSynchronize(s->spill_ev[s->spill_last]));  // the set's last launch
        std::vector<uint32_t> c((size_t)kSpillMaxRounds * kSpillCtrStride);
        HIPCHK(hipMemcpy(c.data(), s->d_spill[s->spill_last], c.size() * 4, hipMemcpyDeviceToHost));
        for (int r = 0; r < 4 && r < kSpillMaxRounds; ++r)
                counts[r] = c[(size_t)r * kSpillCtrStride + 2];  // records (spill_close)
        return VRT_OK;
}

extern "C" int vrt_secondary_spill_stats(vrt_scene *s, int64_t stats[7])
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !stats)
                return fail(VRT_E_INVALID, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        for (int r = 0; r < 7; ++r)
                stats[r] = 0;
        if (s->spill_last < 0 || !s->d_spill[s->spill_last])
                return VRT_OK;
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipEventSynchronize(s->spill_ev[s->spill_last]));
        uint32_t c[8];
        HIPCHK(hipMemcpy(c, s->d_spill[s->spill_last], sizeof c, hipMemcpyDeviceToHost));
        stats[0] = c[2];                     // records queued (spill_close)
        stats[1] = c[5];                     // rays finished in place, queue full (spill_room)
        stats[2] = std::min(c[0], s->spill_cap[s->spill_last]);  // chunks taken
        stats[3] = s->spill_cap[s->spill_last];                  // chunks allocated
        stats[4] = c[3];                     // chunks left to the batch-pool launch
        stats[5] = (int64_t)sizeof(SpillRec);
        stats[6] = c[6];                     // pixels deferred to k_secondary_defer (exact walk)
        return VRT_OK;
}

extern "C" int vrt_render_secondary(vrt_scene *s, const vrt_camera *cam,
                                    const vrt_film *film, int spp, float *vis,
                                    int32_t *s_hit, int32_t *s_tri,
                                    uint32_t *s_vox, int64_t *rays)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !cam || !vis || spp < 1 || spp > 64)
                return fail(VRT_E_INVALID, "bad argument (spp must be 1..64)");
        if (int rc = film_ok(film))
                return rc;
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        const size_t npix = (size_t)film->nx * film->ny;
        const size_t ns = npix * (size_t)spp;
        const size_t narea = (size_t)(8 * (film->nx / 8)) * (8 * (film->ny / 8));
        DevBuf dvis, dprim, dh, dt, dv;
        HIPCHK(hipMalloc(&dvis.p, npix * 4));
        HIPCHK(hipMemsetAsync(dvis.p, 0, npix * 4, s->stream));
        HIPCHK(hipMalloc(&dprim.p, std::max<size_t>(1, narea) * 32));
        if (s_hit) {
                HIPCHK(hipMalloc(&dh.p, ns * 4));
                HIPCHK(hipMemsetAsync(dh.p, 0, ns * 4, s->stream));
        }
        if (s_tri) {
                HIPCHK(hipMalloc(&dt.p, ns * 4));
                HIPCHK(hipMemsetAsync(dt.p, 0xFF, ns * 4, s->stream));
        }
        if (s_vox) {
                HIPCHK(hipMalloc(&dv.p, ns * 4));
                HIPCHK(hipMemsetAsync(dv.p, 0xFF, ns * 4, s->stream));
        }
        RenderParams p;
        fill_render_params(s, cam, film, 0, 1, &p);
        HIPCHK(hipEventRecord(s->ev0, s->stream));
        if (int rc = secondary_launch(s, p, spp, 0, 1, static_cast<float *>(dprim.p), static_cast<float *>(dvis.p),
                                      static_cast<int32_t *>(dh.p), static_cast<int32_t *>(dt.p),
                                      static_cast<uint32_t *>(dv.p), s->stream))
                return rc;
        HIPCHK(hipEventRecord(s->ev1, s->stream));
        s->timed = true;
        HIPCHK(hipStreamSynchronize(s->stream));
        HIPCHK(hipMemcpy(vis, dvis.p, npix * 4, hipMemcpyDeviceToHost));
        if (s_hit)
                HIPCHK(hipMemcpy(s_hit, dh.p, ns * 4, hipMemcpyDeviceToHost));
        if (s_tri)
                HIPCHK(hipMemcpy(s_tri, dt.p, ns * 4, hipMemcpyDeviceToHost));
        if (s_vox)
                HIPCHK(hipMemcpy(s_vox, dv.p, ns * 4, hipMemcpyDeviceToHost));
        if (rays) {
                std::vector<float> prim(narea * 8);
                if (narea)
                        HIPCHK(hipMemcpy(prim.data(), dprim.p, narea * 32, hipMemcpyDeviceToHost));
                int64_t hits = 0;
                for (size_t i = 0; i < narea; ++i)
                        hits += prim[8 * i] != 0.f;
                *rays = (int64_t)narea + hits * spp;
        }
        return VRT_OK;
}

// ---------------------------------------------------------------------------
// full trace(): light map, filter, cone-tracing render
// ---------------------------------------------------------------------------
// (int)log2f(x) thresholds of the host libm: split_up[e] = smallest float in
// [2^e, 2^(e+1)) whose log2f rounds up to e+1 (+inf if none).  The cone
// march (VRT/voxel_octree.cc:286) truncates log2f; the device evaluates the
// same integer from x's exponent and this table.
static const float *split_table()
{
        static float tab[64];
        static std::once_flag once;
        std::call_once(once, [] {
                for (int e = 0; e < 64; ++e) {
                        const float lo = std::ldexp(1.0f, e), top = std::ldexp(1.0f, e + 1);
                        float t = INFINITY;
                        for (float x = std::nextafter(top, 0.0f); x >= lo; x = std::nextafter(x, 0.0f)) {
                                volatile float xv = x;
                                if ((int)log2f(xv) != e + 1)
                                        break;
                                t = x;
                        }
                        tab[e] = t;
                }
        });
        return tab;
}

extern "C" int vrt_scene_min_voxel(const vrt_scene *s, int levels, float *res)
{
        if (!s || !res)
                return fail(VRT_E_INVALID, "null argument");
        const float p2 = std::pow(2.f, (float)(levels > 0 ? levels : s->max_depth));
        for (int k = 0; k < 3; ++k) {
                const float v = (s->info.root_max[k] - s->info.root_min[k]) / p2;
                if (k == 0 || v < *res)
                        *res = v;
        }
        return VRT_OK;
}

static hipError_t ensure_light_scratch(vrt_scene *s, size_t bytes)
{
        if (s->light_bytes >= bytes)
                return hipSuccess;
        if (s->d_light) {
                hipError_t e = hipStreamSynchronize(s->stream);
                if (e != hipSuccess)
                        return e;
                (void)hipFree(s->d_light);
                s->d_light = nullptr;
                s->light_bytes = 0;
        }
        hipError_t e = hipMalloc(&s->d_light, bytes);
        if (e == hipSuccess)
                s->light_bytes = bytes;
        return e;
}

// The light pass + filter of VRT/main.cc:75-100 on the scene's stream
// (caller holds s->mu).  `overlap` (may be empty) is called right after the
// light pass is enqueued, before the one mid-build host sync, so work it
// enqueues on another stream runs beside the light pass; on return the
// filter is enqueued and *lm_done (if given) recorded after it.
static int lightmap_enqueue(vrt_scene *s, int set, const vrt_camera *light_cam, const vrt_film *light_film,
                            unsigned int *hits, const std::function<int()> &overlap, hipEvent_t lm_done)
{
        const int64_t nnodes = (int64_t)s->nodes.size();
        const int ptx = light_film->nx / 8, pty = light_film->ny / 8;
        const int64_t ns = (int64_t)64 * ptx * pty * 4;
        if (ns > 0x7FFFFFFF)
                return fail(VRT_E_INVALID, "light film too large (%lld samples)", (long long)ns);
        // one block: light map, cone-descent records, finiteness flag
        if (int rc = ensure_lm(s, set))
                return rc;
        LMRec *d_lm = s->ts[set].lm;
        float4 *d_cc = reinterpret_cast<float4 *>(d_lm + nnodes);
        uint32_t *d_bad = reinterpret_cast<uint32_t *>(d_cc + nnodes);
        if (int rc = ts_acquire(s, set, s->stream))  // a trace render may still read this set
                return rc;
        // scratch (sized for every sample hitting): 64-bit keys and 32-bit
        // slots in + out, the per-hit (illum, normal) records and their copy
        // in sorted order, the sort's temp, the counters, the leaf runs
        size_t sort_bytes = 0;
        int kbits = 1, lbits = 1;
        while (kbits < 40 && (ns - 1) >> kbits)
                ++kbits;
        while (lbits < 32 && ((uint64_t)nnodes >> lbits) != 0)
                ++lbits;
        HIPCHK(sort_pairs_u64(nullptr, &sort_bytes, nullptr, nullptr, nullptr, nullptr, ns, kbits + lbits, s->stream));
        const size_t b4 = align_up((size_t)ns * 4), b8 = align_up((size_t)ns * 8), b24 = align_up((size_t)ns * 48);
        const int64_t max_seg = std::max<int64_t>(1, s->info.nonempty_leaves);
        const size_t bseg = align_up((size_t)max_seg * 4);
        const size_t bend = align_up((size_t)nnodes * 4);
        const size_t need = 2 * b8 + 2 * b4 + b24 + align_up(sort_bytes) + 256 + bseg + bend;
        HIPCHK(ensure_light_scratch(s, need));
        char *base = static_cast<char *>(s->d_light);
        uint64_t *k_in = reinterpret_cast<uint64_t *>(base);
        uint64_t *k_out = reinterpret_cast<uint64_t *>(base + b8);
        uint32_t *v_in = reinterpret_cast<uint32_t *>(base + 2 * b8);
        uint32_t *v_out = reinterpret_cast<uint32_t *>(base + 2 * b8 + b4);
        float *samp = reinterpret_cast<float *>(base + 2 * b8 + 2 * b4);
        void *temp = base + 2 * b8 + 2 * b4 + b24;
        char *ctr = base + 2 * b8 + 2 * b4 + b24 + align_up(sort_bytes);
        unsigned int *d_count = reinterpret_cast<unsigned int *>(ctr);
        unsigned int *d_nseg = reinterpret_cast<unsigned int *>(ctr + 64);
        unsigned int *d_tail_n = reinterpret_cast<unsigned int *>(ctr + 128);
        uint32_t *d_seg = reinterpret_cast<uint32_t *>(ctr + 256);
        uint32_t *d_seg_end = reinterpret_cast<uint32_t *>(ctr + 256 + bseg);
        LightParams lp;
        std::memset(&lp, 0, sizeof lp);
        fill_render_params(s, light_cam, light_film, 0, 1, &lp.r);
        lp.ptx = ptx;
        lp.pty = pty;
        lp.kbits = kbits;
        lp.count = d_count;
        lp.keys = k_in;
        lp.vals = v_in;
        lp.samp = samp;
        lp.tail_n = d_tail_n;
        lp.tail = v_out;  // free until the sort
        HIPCHK(hipEventRecord(s->ev0, s->stream));
        // cone_trace_init_filter's leaf case first: it also zeroes the
        // counters the passes below add to (no memsets)
        HIPCHK(launch_lm_leaves(s->dev.nodes, nnodes, d_lm, d_bad, d_count, d_tail_n, d_nseg, s->stream));
        HIPCHK(launch_light(lp, s->stream));
        if (overlap)
                if (int rc = overlap())
                        return rc;
        // the sort takes its length on the host: the one mid-build sync
        unsigned int nhit = 0;
        HIPCHK(hipMemcpyAsync(&nhit, d_count, sizeof nhit, hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
#ifdef VRT_LIGHT_DIAG
        {
                static int ndump = 0;
                const size_t nw = (size_t)std::min<int64_t>(ns / 64, 1 << 20);
                std::vector<uint32_t> d(nw * 8);
                HIPCHK(light_diag_copy(d.data(), d.size() * 4));
                char name[64];
                std::snprintf(name, sizeof name, "gpurun_out/light_diag_%d.bin", ndump++);
                if (FILE *f = std::fopen(name, "wb")) {
                        std::fwrite(d.data(), 4, d.size(), f);
                        std::fclose(f);
                }
        }
#endif
#ifdef VRT_LIGHT_TAIL_REPORT
        {
                unsigned int ntail = 0;
                HIPCHK(hipMemcpy(&ntail, d_tail_n, sizeof ntail, hipMemcpyDeviceToHost));
                std::fprintf(stderr, "light pass: %u of %lld samples deferred, %u hits\n", ntail, (long long)ns, nhit);
        }
#endif
        if (nhit > 0)
                HIPCHK(sort_pairs_u64(temp, &sort_bytes, k_in, k_out, v_in, v_out, nhit, kbits + lbits, s->stream));
        HIPCHK(launch_lm_accum(nhit, k_out, v_out, kbits, samp, d_seg, d_nseg, max_seg, d_seg_end, d_lm,
                               s->stream));
        // cone_trace_init_filter: internal levels bottom-up
        const int nlev = (int)s->level_begin.size() - 1;
        for (int l = nlev; l >= 1; --l)
                HIPCHK(launch_lm_level(s->dev.nodes, s->level_begin[l - 1], s->level_begin[l], d_lm, s->stream));
        HIPCHK(launch_lm_aux(s->dev.nodes, d_lm, nnodes, d_cc, d_bad, s->stream));
        HIPCHK(hipEventRecord(s->ev1, s->stream));
        if (lm_done)
                HIPCHK(hipEventRecord(lm_done, s->stream));
        s->timed = true;
        s->lm_cur = set;
        *hits = nhit;
        return VRT_OK;
}

extern "C" int vrt_lightmap_build(vrt_scene *s, const vrt_camera *light_cam,
                                  const vrt_film *light_film, int64_t *hits)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !light_cam)
                return fail(VRT_E_INVALID, "null argument");
        if (int rc = film_ok(light_film))
                return rc;
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        unsigned int nhit = 0;
        const int set = s->ts_next;
        s->ts_next ^= 1;
        if (int rc = lightmap_enqueue(s, set, light_cam, light_film, &nhit, {}, nullptr))
                return rc;
        if (int rc = ts_release(s, set, s->stream))
                return rc;
        HIPCHK(hipStreamSynchronize(s->stream));
        if (hits)
                *hits = (int64_t)nhit;
        return VRT_OK;
}

extern "C" int vrt_lightmap_nodes(vrt_scene *s, uint64_t *key, float *coverage, float *illum)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !key)
                return fail(VRT_E_INVALID, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->lm_cur < 0)
                return fail(VRT_E_INVALID, "no light map: call vrt_lightmap_build first");
        HIPCHK(hipSetDevice(s->device));
        const size_t n = s->nodes.size();
        std::vector<LMRec> lm(n);
        // the set may be filled on the scene stream and read on callers'
        // streams (trace frames): its last user's event covers both
        HIPCHK(hipStreamSynchronize(s->stream));
        if (s->ts[s->lm_cur].live)
                HIPCHK(hipEventSynchronize(s->ts[s->lm_cur].ev));
        HIPCHK(hipMemcpy(lm.data(), s->ts[s->lm_cur].lm, n * sizeof(LMRec), hipMemcpyDeviceToHost));
        for (size_t l = 0; l + 1 < s->level_begin.size(); ++l)
                for (int64_t i = s->level_begin[l]; i < s->level_begin[l + 1]; ++i) {
                        key[i] = ((uint64_t)(l + 1) << 32) | s->node_vox[(size_t)i];
                        if (coverage)
                                coverage[i] = lm[(size_t)i].cov;
                        if (illum)
                                std::memcpy(illum + 18 * (size_t)i, lm[(size_t)i].illum, 18 * sizeof(float));
                }
        return VRT_OK;
}

static int trace_ok(vrt_scene *s, float min_voxel)
{
        if (!(min_voxel > 0.f))
                vrt_scene_min_voxel(s, 0, &min_voxel);
        const float mindist = 1.414f * min_voxel;
        if (!(mindist > 0.f) || !std::isfinite(mindist))
                return fail(VRT_E_INVALID, "degenerate cone step: min voxel %g (flat scene?)", (double)min_voxel);
        for (int k = 0; k < 3; ++k)
                if (!std::isfinite(s->info.root_max[k] - s->info.root_min[k]))
                        return fail(VRT_E_INVALID, "scene bounds not finite");
        return VRT_OK;
}

static int trace_scratch(vrt_scene *s, int set, const TraceParams &tp, TraceParams *out)
{
        *out = tp;
        TraceSet &t = s->ts[set];
        const size_t nslots = (size_t)tp.r.tiles_this_rank * 256;
        // the cone step table and its length (at fixed offsets: the table
        // outlives calls with other tile counts), the primary pass's 64-B
        // records, its deferred-sample count (512 B) and list
        const size_t head = (size_t)kConeSteps * 16 + 256;
        const size_t need = head + nslots * 64 + 512 + nslots * 4;
        if (t.rec_bytes < need) {
                if (t.rec) {
                        // every user of the set's scratch is ordered by its event
                        // (ts_acquire waits for it, ts_release records it)
                        if (t.live)
                                HIPCHK(hipEventSynchronize(t.ev));
                        (void)hipFree(t.rec);
                        t.rec = nullptr;
                        t.rec_bytes = 0;
                }
                HIPCHK(hipMalloc(&t.rec, need));
                t.rec_bytes = need;
                t.steps_key[0] = t.steps_key[1] = -1.f;
        }
        // the step table depends on mindist and maxdist only: rebuilt when
        // they change (the set's users are ordered by its event); the key is
        // committed only once k_cone_steps is enqueued (steps_commit)
        out->build_steps = !(t.steps_key[0] == tp.mindist && t.steps_key[1] == tp.maxdist);
        char *b = static_cast<char *>(t.rec);
        out->steps = reinterpret_cast<float4 *>(b);
        out->nsteps = reinterpret_cast<int *>(b + (size_t)kConeSteps * 16);
        out->rec = reinterpret_cast<float4 *>(b + head);
        out->tail_n = reinterpret_cast<unsigned int *>(b + head + nslots * 64);
        out->tail = reinterpret_cast<uint32_t *>(b + head + nslots * 64 + 512);
        return VRT_OK;
}

// After launch_trace_prim returned success: the step table it was asked to
// build (k_cone_steps) is enqueued, so the set's key may say so.  Every error
// return before that leaves the key as it was, and the next call rebuilds.
static void steps_commit(vrt_scene *s, int set, const TraceParams &tp)
{
        if (!tp.build_steps || tp.r.tiles_this_rank <= 0)
                return;
        s->ts[set].steps_key[0] = tp.mindist;
        s->ts[set].steps_key[1] = tp.maxdist;
}

// The cone march's split level as a function of the diameter
// (TraceParams::split_bound): S(diam) = split_level_of(fl(maxdist / diam))
// -- the kernels' own rule on the correctly rounded quotient, which the host
// division reproduces -- is non-increasing in diam, so bound[k] = the
// largest float diam with S(diam) >= k, found by bisection over the float
// bit patterns (monotone in value for positive floats).
static int split_level_host(float x, const float *up)
{
        uint32_t u;
        std::memcpy(&u, &x, 4);
        const int e = (int)(u >> 23) - 127;
        if (e >= 63)
                return e;
        return x >= up[e] ? e + 1 : e;
}

static void split_bounds(float maxdist, const float *up, float *bound)
{
        static thread_local float last_max = -1.f;
        static thread_local float last[64];
        if (maxdist == last_max) {
                std::memcpy(bound, last, sizeof last);
                return;
        }
        bound[0] = maxdist;
        auto S = [&](uint32_t bits) {
                float d;
                std::memcpy(&d, &bits, 4);
                volatile float q = maxdist / d;  // one correctly rounded division, as on the device
                return split_level_host(q, up);
        };
        uint32_t top;
        std::memcpy(&top, &maxdist, 4);
        for (int k = 1; k < 64; ++k) {
                if (!(maxdist > 0.f) || !std::isfinite(maxdist) || S(1u) < k) {  // not even the least diameter
                        bound[k] = 0.f;
                        continue;
                }
                uint32_t lo = 1u, hi = top;  // S(lo) >= k; find the largest bits with S >= k
                while (lo < hi) {
                        const uint32_t mid = lo + (hi - lo + 1) / 2;
                        if (S(mid) >= k)
                                lo = mid;
                        else
                                hi = mid - 1;
                }
                std::memcpy(&bound[k], &lo, 4);
        }
        last_max = maxdist;
        std::memcpy(last, bound, sizeof last);
}

static void fill_trace_params(vrt_scene *s, int set, const vrt_camera *cam, const vrt_film *film, float min_voxel,
                              int rank, int nranks, TraceParams *tp)
{
        std::memset(tp, 0, sizeof *tp);
        fill_render_params(s, cam, film, rank, nranks, &tp->r);
        if (!(min_voxel > 0.f))
                vrt_scene_min_voxel(s, 0, &min_voxel);
        tp->lm = s->ts[set].lm;
        tp->cc = reinterpret_cast<const float4 *>(s->ts[set].lm + s->nodes.size());
        tp->lm_bad = reinterpret_cast<const uint32_t *>(tp->cc + s->nodes.size());
        tp->cells = reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(tp->lm_bad) + 256);
        // float mindist = 1.414f * min_voxel_size; maxdist = length(root.aabb.size())
        tp->mindist = 1.414f * min_voxel;
        const f3 sz = mk3(s->info.root_max[0] - s->info.root_min[0], s->info.root_max[1] - s->info.root_min[1],
                          s->info.root_max[2] - s->info.root_min[2]);
        tp->maxdist = length(sz);
        std::memcpy(tp->split_up, split_table(), sizeof tp->split_up);
        split_bounds(tp->maxdist, tp->split_up, tp->split_bound);
}

extern "C" int vrt_render_trace_device(vrt_scene *s, const vrt_camera *cam, const vrt_film *film,
                                       float min_voxel, int rank, int nranks, int image_layout,
                                       float *d_out, void *stream)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !cam || !d_out)
                return fail(VRT_E_INVALID, "null argument");
        if (int rc = film_ok(film))
                return rc;
        if (nranks < 1 || rank < 0 || rank >= nranks)
                return fail(VRT_E_INVALID, "rank %d of %d", rank, nranks);
        if (image_layout && nranks != 1)
                return fail(VRT_E_INVALID, "image_layout requires nranks == 1");
        if (int rc = trace_ok(s, min_voxel))
                return rc;
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->lm_cur < 0)
                return fail(VRT_E_INVALID, "no light map: call vrt_lightmap_build first");
        HIPCHK(hipSetDevice(s->device));
        const int set = s->lm_cur;  // the latest light map
        TraceParams tp0, tp;
        fill_trace_params(s, set, cam, film, min_voxel, rank, nranks, &tp0);
        tp0.r.image_layout = image_layout;
        tp0.r.out = d_out;
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (int rc = trace_scratch(s, set, tp0, &tp))
                return rc;
        if (int rc = ts_acquire(s, set, st))
                return rc;
        HIPCHK(hipEventRecord(s->ev0, st));
        HIPCHK(launch_trace(tp, st));
        steps_commit(s, set, tp);
        HIPCHK(hipEventRecord(s->ev1, st));
        if (int rc = ts_release(s, set, st))
                return rc;
        s->timed = true;
        return VRT_OK;
}

// The reference main() frame in one call (VRT/main.cc:75-126): light pass
// + filter on the scene's stream and, beside them on `stream`, the view's
// primary march (k_trace_prim reads no light map); the cones + film pass
// waits for the filter.  Same values as vrt_lightmap_build followed by
// vrt_render_trace_device.  Returns once the filter is enqueued (the light
// pass's hit count needs one host sync); the image is ordered on `stream`.
extern "C" int vrt_trace_frame_device(vrt_scene *s, const vrt_camera *light_cam, const vrt_film *light_film,
                                      const vrt_camera *cam, const vrt_film *film, float min_voxel, int rank,
                                      int nranks, int image_layout, float *d_out, void *stream, int64_t *hits)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !light_cam || !cam || !d_out)
                return fail(VRT_E_INVALID, "null argument");
        if (int rc = film_ok(light_film))
                return rc;
        if (int rc = film_ok(film))
                return rc;
        if (nranks < 1 || rank < 0 || rank >= nranks)
                return fail(VRT_E_INVALID, "rank %d of %d", rank, nranks);
        if (image_layout && nranks != 1)
                return fail(VRT_E_INVALID, "image_layout requires nranks == 1");
        if (int rc = trace_ok(s, min_voxel))
                return rc;
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (!s->lm_ev)
                HIPCHK(hipEventCreateWithFlags(&s->lm_ev, hipEventDisableTiming));
        // alternate sets: this frame's light pass waits only for the frame
        // before last (the set's previous user), so it runs beside the
        // previous frame's cone-traced shading
        const int set = s->ts_next;
        s->ts_next ^= 1;
        if (int rc = ensure_lm(s, set))  // the trace parameters point into it
                return rc;
        TraceParams tp0, tp;
        fill_trace_params(s, set, cam, film, min_voxel, rank, nranks, &tp0);
        tp0.r.image_layout = image_layout;
        tp0.r.out = d_out;
        if (int rc = trace_scratch(s, set, tp0, &tp))
                return rc;
        unsigned int nhit = 0;
        auto overlap = [&]() -> int {
                // the view's primary march beside the light pass (its records
                // wait only for the previous frame's users of the scratch)
                if (int rc = ts_acquire(s, set, st))
                        return rc;
                HIPCHK(launch_trace_prim(tp, st));
                steps_commit(s, set, tp);
                return VRT_OK;
        };
        if (int rc = lightmap_enqueue(s, set, light_cam, light_film, &nhit, overlap, s->lm_ev)) {
                // whatever was enqueued on either stream (the light pass on
                // the scene's, the primary march on the caller's) finishes
                // before the set's next user starts
                if (hipEventRecord(s->lm_ev, s->stream) == hipSuccess)
                        (void)hipStreamWaitEvent(st, s->lm_ev, 0);
                (void)ts_release(s, set, st);
                return rc;
        }
        HIPCHK(hipStreamWaitEvent(st, s->lm_ev, 0));
        if (hipError_t e = launch_cones(tp, st)) {
                (void)ts_release(s, set, st);
                return fail(VRT_E_DEVICE, "cone pass launch failed: %s", hipGetErrorString(e));
        }
        if (int rc = ts_release(s, set, st))
                return rc;
        if (hits)
                *hits = (int64_t)nhit;
        return VRT_OK;
}

extern "C" int vrt_render_trace(vrt_scene *s, const vrt_camera *cam, const vrt_film *film, float min_voxel,
                                float *rgb, int32_t *s_hit, float *s_rgb)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || !cam || !rgb)
                return fail(VRT_E_INVALID, "null argument");
        if (int rc = film_ok(film))
                return rc;
        if (int rc = trace_ok(s, min_voxel))
                return rc;
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->lm_cur < 0)
                return fail(VRT_E_INVALID, "no light map: call vrt_lightmap_build first");
        HIPCHK(hipSetDevice(s->device));
        const int set = s->lm_cur;
        const size_t npix = (size_t)film->nx * film->ny, ns = npix * 4;
        DevBuf img, dh, dr;
        HIPCHK(hipMalloc(&img.p, npix * 12));
        HIPCHK(hipMemsetAsync(img.p, 0, npix * 12, s->stream));
        TraceParams tp0, tp;
        fill_trace_params(s, set, cam, film, min_voxel, 0, 1, &tp0);
        tp0.r.image_layout = 1;
        tp0.r.out = static_cast<float *>(img.p);
        if (int rc = trace_scratch(s, set, tp0, &tp))
                return rc;
        if (s_hit) {
                HIPCHK(hipMalloc(&dh.p, ns * 4));
                HIPCHK(hipMemsetAsync(dh.p, 0, ns * 4, s->stream));
                tp.r.so.hit = static_cast<int32_t *>(dh.p);
        }
        if (s_rgb) {
                HIPCHK(hipMalloc(&dr.p, ns * 12));
                HIPCHK(hipMemsetAsync(dr.p, 0, ns * 12, s->stream));
                tp.r.so.rgb = static_cast<float *>(dr.p);
        }
        if (int rc = ts_acquire(s, set, s->stream))
                return rc;
        HIPCHK(hipEventRecord(s->ev0, s->stream));
        HIPCHK(launch_trace(tp, s->stream));
        steps_commit(s, set, tp);
        HIPCHK(hipEventRecord(s->ev1, s->stream));
        if (int rc = ts_release(s, set, s->stream))
                return rc;
        s->timed = true;
        HIPCHK(hipStreamSynchronize(s->stream));
        HIPCHK(hipMemcpy(rgb, img.p, npix * 12, hipMemcpyDeviceToHost));
        if (s_hit)
                HIPCHK(hipMemcpy(s_hit, dh.p, ns * 4, hipMemcpyDeviceToHost));
        if (s_rgb)
                HIPCHK(hipMemcpy(s_rgb, dr.p, ns * 12, hipMemcpyDeviceToHost));
        return VRT_OK;
}

extern "C" int vrt_ray_march_batch_device(vrt_scene *s, const vrt_ray *d_rays,
                                          int64_t n, vrt_hit *d_hits,
                                          void *stream)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        if (!s || (n > 0 && (!d_rays || !d_hits)) || n < 0)
                return fail(VRT_E_INVALID, "bad argument");
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(launch_ray_march(s->dev, d_rays, n, d_hits, static_cast<hipStream_t>(stream)));
        return VRT_OK;
}

extern "C" int vrt_ray_march_batch(vrt_scene *s, const vrt_ray *rays,
                                   int64_t n, vrt_hit *hits)
{
        if (s && need_device(s))
                return VRT_E_NODEVICE;
        static_assert(sizeof(vrt_ray) == 32, "vrt_ray layout");
        static_assert(sizeof(vrt_hit) == 36, "vrt_hit layout");
        if (!s || n < 0 || (n > 0 && (!rays || !hits)))
                return fail(VRT_E_INVALID, "bad argument");
        if (n == 0)
                return VRT_OK;
        std::lock_guard<std::mutex> lk(s->mu);
        HIPCHK(hipSetDevice(s->device));
        // device buffers and pinned staging kept in the scene (grown as needed)
        if (n > s->rays_cap) {
                HIPCHK(hipStreamSynchronize(s->stream));
                for (void **p : { &s->d_rays, &s->d_hits })
                        if (*p) {
                                (void)hipFree(*p);
                                *p = nullptr;
                        }
                for (void **p : { &s->h_rays, &s->h_hits })
                        if (*p) {
                                (void)hipHostFree(*p);
                                *p = nullptr;
                        }
                s->rays_cap = 0;
                HIPCHK(hipMalloc(&s->d_rays, (size_t)n * sizeof(vrt_ray)));
                HIPCHK(hipMalloc(&s->d_hits, (size_t)n * sizeof(vrt_hit)));
                HIPCHK(hipHostMalloc(&s->h_rays, (size_t)n * sizeof(vrt_ray), hipHostMallocDefault));
                HIPCHK(hipHostMalloc(&s->h_hits, (size_t)n * sizeof(vrt_hit), hipHostMallocDefault));
                s->rays_cap = n;
        }
        par_memcpy(s->h_rays, rays, (size_t)n * sizeof(vrt_ray));
        HIPCHK(hipMemcpyAsync(s->d_rays, s->h_rays, (size_t)n * sizeof(vrt_ray), hipMemcpyHostToDevice, s->stream));
        HIPCHK(launch_ray_march(s->dev, s->d_rays, n, s->d_hits, s->stream));
        HIPCHK(hipMemcpyAsync(s->h_hits, s->d_hits, (size_t)n * sizeof(vrt_hit), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        par_memcpy(hits, s->h_hits, (size_t)n * sizeof(vrt_hit));
        return VRT_OK;
}

extern "C" int vrt_device_selftest(int device, const double *mt_in,
                                   double *mt_out, const float *sat_in,
                                   int32_t *sat_out, int64_t n)
{
        if (n < 0 || (mt_in && !mt_out) || (sat_in && !sat_out))
                return fail(VRT_E_INVALID, "bad argument");
        if (int rc = check_device(device))
                return rc;
        HIPCHK(hipSetDevice(device));
        DevBuf a, b, c, d;
        if (mt_in) {
                HIPCHK(hipMalloc(&a.p, (size_t)n * 15 * 8));
                HIPCHK(hipMalloc(&b.p, (size_t)n * 4 * 8));
                HIPCHK(hipMemcpy(a.p, mt_in, (size_t)n * 15 * 8, hipMemcpyHostToDevice));
        }
        if (sat_in) {
                HIPCHK(hipMalloc(&c.p, (size_t)n * 15 * 4));
                HIPCHK(hipMalloc(&d.p, (size_t)n * 4));
                HIPCHK(hipMemcpy(c.p, sat_in, (size_t)n * 15 * 4, hipMemcpyHostToDevice));
        }
        HIPCHK(launch_selftest(static_cast<double *>(a.p), static_cast<double *>(b.p),
                               static_cast<float *>(c.p), static_cast<int32_t *>(d.p), n, nullptr));
        HIPCHK(hipDeviceSynchronize());
        if (mt_in)
                HIPCHK(hipMemcpy(mt_out, b.p, (size_t)n * 4 * 8, hipMemcpyDeviceToHost));
        if (sat_in)
                HIPCHK(hipMemcpy(sat_out, d.p, (size_t)n * 4, hipMemcpyDeviceToHost));
        return VRT_OK;
}

extern "C" int vrt_device_selftest_order(int device, const float *dist, const uint32_t *hit_mask, int64_t n,
                                         uint32_t *orders, const float *depth, const int32_t *len, int64_t m,
                                         int32_t stride, int32_t *argmin)
{
        if (n < 0 || m < 0 || (n > 0 && (!dist || !hit_mask || !orders)) ||
            (m > 0 && (!depth || !len || !argmin || stride < 0)))
                return fail(VRT_E_INVALID, "bad argument");
        for (int64_t j = 0; j < m; ++j)
                if (len[j] < 0 || len[j] > stride)
                        return fail(VRT_E_INVALID, "record list %lld: length %d outside [0, %d]", (long long)j,
                                    len[j], stride);
        if (int rc = check_device(device))
                return rc;
        HIPCHK(hipSetDevice(device));
        DevBuf dd, dh, dout, ddep, dlen, darg;
        if (n > 0) {
                HIPCHK(hipMalloc(&dd.p, (size_t)n * 8 * sizeof(float)));
                HIPCHK(hipMalloc(&dh.p, (size_t)n * sizeof(uint32_t)));
                HIPCHK(hipMalloc(&dout.p, (size_t)n * 6 * sizeof(uint32_t)));
                HIPCHK(hipMemcpy(dd.p, dist, (size_t)n * 8 * sizeof(float), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(dh.p, hit_mask, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
        if (m > 0) {
                HIPCHK(hipMalloc(&ddep.p, std::max<size_t>(1, (size_t)m * stride) * sizeof(float)));
                HIPCHK(hipMalloc(&dlen.p, (size_t)m * sizeof(int32_t)));
                HIPCHK(hipMalloc(&darg.p, (size_t)m * sizeof(int32_t)));
                if (stride > 0)
                        HIPCHK(hipMemcpy(ddep.p, depth, (size_t)m * stride * sizeof(float), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(dlen.p, len, (size_t)m * sizeof(int32_t), hipMemcpyHostToDevice));
        }
        HIPCHK(launch_selftest_order(static_cast<float *>(dd.p), static_cast<uint32_t *>(dh.p), n,
                                     static_cast<uint32_t *>(dout.p), static_cast<float *>(ddep.p),
                                     static_cast<int32_t *>(dlen.p), m, stride, static_cast<int32_t *>(darg.p),
                                     nullptr));
        HIPCHK(hipDeviceSynchronize());
        if (n > 0)
                HIPCHK(hipMemcpy(orders, dout.p, (size_t)n * 6 * sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (m > 0)
                HIPCHK(hipMemcpy(argmin, darg.p, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost));
        return VRT_OK;
}
