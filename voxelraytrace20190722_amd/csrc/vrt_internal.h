// vrt_internal.h -- device data layout shared by the host library and the
// gfx950 kernels.  See DESIGN.md "Data layout in HBM".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "vrt.h"
#include "vrt_math.h"

namespace vrt {

// One octree node, 32 B (two dwordx4 loads).  The 8 children of an internal
// node are contiguous.  Boxes are the exact float boxes split() produces
// (VRT/voxel_octree.cc:27-39).
//   internal:        a = index of first child      (bit 31 clear)
//   leaf:            a = kLeafBit | triangle count, b = first ref record
struct alignas(16) NodeRec {
        float bmin[3];
        float bmax[3];
        uint32_t a;
        uint32_t b;
};
static_assert(sizeof(NodeRec) == 32, "NodeRec must be 32 B");
constexpr uint32_t kLeafBit = 0x80000000u;

// March record of the node triangle-box walk (DevScene::xnodes): the node's
// own record (voxel box, a, b) followed by the union box of every triangle
// below it (a leaf: its own triangles), enlarged by lb_eps -- one 64-B
// record, so the walk fetches both halves with one address.
struct alignas(16) XNodeRec {
        NodeRec n;
        float tmin[3];
        float tmax[3];
        uint32_t pad[2];
};
static_assert(sizeof(XNodeRec) == 64, "XNodeRec must be 64 B");


// Leaf-list records, in leaf order with the vertices inlined (no dependent
// index load in the leaf loop).  Two formats, chosen per scene:
// RefRec48 for small leaves (fewer bytes per gather), RefRec64 for scenes
// with >= 8 records per non-empty leaf (DevScene::wide_leaves), where the
// leaf loop dominates and a wave often tests one leaf together.
struct alignas(16) RefRec48 {
        float p[9];
        uint32_t tri;
        uint32_t pad[2];
};
static_assert(sizeof(RefRec48) == 48, "RefRec48 must be 48 B");
// 64 B (one cache line): vert0 as float (widened in the kernel), the
// triangle id, and Moller-Trumbore's edge1 = vert1 - vert0, edge2 = vert2 -
// vert0 already in double -- the same IEEE subtractions of widened floats
// intersect_triangle3 makes (VRT/raytri.cc:209-210), done once per record.
struct alignas(16) RefRec64 {
        float v0[3];
        uint32_t tri;
        double e1[3];
        double e2[3];
};
static_assert(sizeof(RefRec64) == 64, "RefRec64 must be 64 B");

// Shading attributes of one triangle (64 B): normalised vertex normals
// (Triangle::Triangle, VRT/voxel_octree.cc:426), uvs, material id.
struct alignas(16) TriAttr {
        float n[9];
        float t[6];
        int32_t mat;
};
static_assert(sizeof(TriAttr) == 64, "TriAttr must be 64 B");

struct alignas(16) TriPos {
        float p[9];
        float pad[3];
};

struct alignas(16) TexRec {
        int64_t off;
        int32_t w, h, c, pad;
};

// A material with its texture's record inline (a copy of texs[tex]), so a
// textured hit's shading is TriAttr (beside TriPos) -> MatRec -> texel: one
// dependent load fewer than MatRec -> TexRec.
struct alignas(16) MatRec {
        int32_t tex;  // -1 = untextured: Kd
        float kd[3];
        TexRec tx;    // texs[tex] when tex >= 0, else zero
};
static_assert(sizeof(MatRec) == 48, "MatRec must be 48 B");

// Device-side scene view passed by value to kernels.
struct DevScene {
        const NodeRec *nodes;
        const uint32_t *node_vox;
        const void *refs;  // RefRec64 if wide_leaves, else RefRec48
        const TriPos *tri_pos;
        const TriAttr *tri_attr;
        const MatRec *mats;
        const TexRec *texs;
        const uint8_t *tex_data;
        int32_t max_depth;
        int32_t nmat, ntex;
        int32_t fast_ok;  // root box finite and |coords| < 2^60 (expand_v1, fast_ok())
        int32_t wide_leaves;  // >= 8 records per non-empty leaf on average: RefRec64 records,
                              // wave-uniform leaf loads (leaf_isect)
        int32_t persist_blocks;  // resident 256-thread blocks of the persistent render on this
                                 // device (a multiple of 8), 0 = no persistent launches
        int32_t sec_blocks;      // the same for the persistent secondary-ray kernel
        int32_t grid_div;        // persistent render grid = resident slots / grid_div
                                 // (vrt_scene_set_frames_in_flight)
        // March records of the nodes (XNodeRec): the node record and the
        // union box of every triangle below it enlarged by lb_eps
        // (leaf_box_ok).  A ray whose line misses that box cannot pass
        // intersect_triangle3 (which accepts a hit at any t) on any triangle
        // below the node, so the finite-slab walks skip the subtree (a leaf:
        // its triangle loop); results are unchanged.  The skip is used for
        // rays with every |o - lb_center| <= lb_reach, where lb_eps exceeds
        // the fp32 rounding of the line test.
        const XNodeRec *xnodes;
        float lb_center[3];
        float lb_reach;
};

// Work queue of one persistent launch (k_render_p, k_secondary_p): 8
// counters, one per XCD slice of the units, one 128-B line each.  The
// kernel never resets them: unit j of slice x is taken by the atomicAdd that
// returns base[x] + j, and every wave makes exactly one more (failing) add
// per non-empty slice, so after a launch of `waves` waves counter x has
// advanced by (hi - lo of queue_range(units, x)) + waves -- the host keeps
// base[] from that, per ring slot (vrt_host.cpp: queue_take /
// queue_release).  Launches on different streams use different slots; a
// slot is reused only after its previous launch has finished (an event), so
// no two launches share counters and no memset is needed.
// After the counters: the deferred-unit lists of k_render_p<true>, one per
// XCD slice (a wave appends a unit to the list of the slice it took it
// from; 8 counters instead of one keep the appends as spread as the takes):
// slice x's count at defer[x * kQueueStride + kDeferCount], its list at
// defer[kDeferList + x * kDeferSliceCap ...].  A slice with more than
// kDeferSliceCap deferred units is re-rendered whole.  k_render_defer,
// launched behind it on the same stream, renders them (its waves take
// entries from the slice's defer[x * kQueueStride + kDeferTake] and count
// themselves out on defer[kDeferDoneWord]); its last wave zeroes every count,
// take counter and the done counter.
constexpr int kQueueStride = 32;
constexpr int kQueueSlots = 8;
constexpr int kDeferCount = 0;
constexpr int kDeferTake = 1;
constexpr int kDeferDoneWord = 8 * kQueueStride;
constexpr int kDeferList = kDeferDoneWord + kQueueStride;
constexpr int kDeferSliceCap = 512;
constexpr size_t kQueueWords = 8 * kQueueStride + kDeferList + 8 * kDeferSliceCap;
constexpr size_t kQueueBytes = kQueueWords * sizeof(uint32_t);
struct WorkQueue {
        uint32_t *ctr;
        uint32_t *defer;
        uint32_t base[8];
};
// units of slice x: a contiguous range [lo, hi) of the unit order
__host__ __device__ inline void queue_range(int units, int x, int &lo, int &hi)
{
        const int per = (units + 7) >> 3;
        lo = x * per;
        hi = lo + per < units ? lo + per : units;
        if (hi < lo)
                hi = lo;
}

// XCD slices of a persistent launch's units (the kernels and the host's
// queue bases agree through these two functions).  ch = 0: slice x is
// queue_range's contiguous eighth of the units; ch > 0: the unit order is cut
// into chunks of ch units dealt to the slices round-robin (chunk c -> slice c
// % 8), so every XCD's share is spread over the whole frame and the XCDs run
// out of work together (a contiguous eighth of a frame can cost far more
// than another); each chunk is still a compact run of tiles for the XCD's L2.
// Measured (tools/ab.py): primary 1080p single launch +4.1 %, 4K +4.9 %.
#ifndef VRT_SLICE_CHUNK
#define VRT_SLICE_CHUNK 512       // primary render: 128 tiles x 4 quadrant units
#endif
#ifndef VRT_SEC_SLICE_CHUNK
#define VRT_SEC_SLICE_CHUNK 8192  // config 5: pixels (128 tiles x 64); +2.3 % per frame
#endif
__host__ __device__ inline int slice_size(int units, int x, int ch)
{
        if (ch == 0) {
                int lo, hi;
                queue_range(units, x, lo, hi);
                return hi - lo;
        }
        const int nc = units / ch, rem = units % ch;
        return (nc / 8 + (x < nc % 8 ? 1 : 0)) * ch + (nc % 8 == x ? rem : 0);
}
// the u-th unit of slice x (u < slice_size(units, x, ch))
__host__ __device__ inline int slice_unit(int units, int x, int u, int ch)
{
        if (ch == 0) {
                int lo, hi;
                queue_range(units, x, lo, hi);
                return lo + u;
        }
        return ((u / ch) * 8 + x) * ch + u % ch;
}

// Config-5 ray compaction (k_secondary_p + k_sec_resume).  A
// wave walks one pixel's secondary rays until fewer than `t_first` of them
// are still walking; it then stops, and each of those rays writes its walk
// state -- the ray, the node it was about to visit next and its DFS stack --
// to queue 0.  The resume round (k_sec_stream, or k_sec_resume for films of
// 2^26 pixels or more) continues their walks from the saved states, 64 rays
// to a wave as one pool, to their ends.  The walk after a resume is the walk
// that would have run, so every ray's hit boolean is unchanged.  The pixel's count of hits and of
// rays still out lives in its unused primary-record word (prim[8*pix+7]);
// the ray that brings the outstanding count to zero writes the pixel.
// A queue is cut into chunks of kSpillChunk records: a wave takes a whole
// chunk with one atomic and fills it itself (one atomic per chunk, not per
// stopped pixel, on the queue's counter), and writes the chunk's fill count
// when it moves on; a resume wave takes one chunk at a time.
constexpr int kSpillStack = 10;  // >= the DFS stack (kStack, vrt_kernels.hip)
constexpr uint32_t kSpillChunk = 256;
// 64 B.  The compaction runs only for films under 2^26 pixels and octrees
// under 2^24 nodes (spill_setup), so a pixel and a DFS stack entry each fit a
// word.
struct alignas(16) SpillRec {
        uint32_t pix_smp;  // primary record index (y * W8 + x) | secondary ray index << 26
        uint32_t base;     // the child block the walk was in
        uint32_t mask_sp;  // its children left to visit (8 bits) | stack entries << 8
        float d[3];        // normalised direction (the ray's origin is the pixel's hit point)
        uint32_t stk[kSpillStack];  // DFS stack, bottom first: block << 8 | children left
};
static_assert(sizeof(SpillRec) == 64, "SpillRec layout");
constexpr int kSpillCtrStride = 32;  // one 128-B line per round's counters
constexpr int kSpillMaxRounds = 4;
struct SpillQueues {
        uint32_t *ctr;       // zeroed per frame: [0] chunks taken by phase A, [1] chunks taken by the
                             // stream, [2] records written, [3] chunks the stream left to k_sec_resume,
                             // [4] their pieces taken, [5] stopped rays finished in place (queue full),
                             // [6] pixels deferred to k_secondary_defer, [7] of them taken;
                             // the words of rounds 1..3 ([r * kSpillCtrStride + 2]) stay 0
        uint32_t *dpix;      // the deferred pixels (this rank's pixel indices), one per pixel of the
                             // film at most; NULL: no fast-only kernel
        uint32_t *fill[2];   // [0] records in each chunk of queue 0, written by the chunk's writer;
                             // [1] the chunks the stream left
        SpillRec *rec[2];    // queue 0's records: rec[0] + chunk * kSpillChunk ([1] unused)
        uint32_t nchunks;    // chunks in queue 0; 0 = no compaction
        uint32_t t_first;    // phase-A threshold (walking lanes)
        int32_t stream;      // 1: the resume round streams queue 0 (the only mode)
};

// Tile deal of a multi-rank frame.  The ntx x nty grid of
// 8x8-pixel tiles is cut into G x G blocks of tiles (G = VRT_DEAL_BLOCK);
// the whole blocks are dealt round-robin in block raster order (block j ->
// rank j % nranks), then the tiles outside the whole-block region -- the
// right strip (rows above the bottom strip), then the bottom strip, each in
// raster order -- continue the round robin one tile at a time (leftover i ->
// rank (F + i) % nranks, F = whole blocks).  A rank's tiles are numbered k =
// 0, 1, ...: its blocks' tiles (block order, row-major inside a block), then
// its leftover tiles.  A rank's share is so made of compact G x G regions
// (rays of one region walk the same part of the octree), and every rank gets
// the same number of blocks +-1.  G = 1 is tile t -> rank t % nranks.
//
// Rank 0 lighter (VRT_DEAL_WEIGHT, nranks >= 2): rank 0 also gathers and
// re-assembles the frame, so it is dealt (m-1)/m of another rank's blocks,
// m = max(2, VRT_DEAL_SPAN / nranks) (5/6 at 8 ranks, 11/12 at 4, 23/24 at 2:
// round 5, from every rank's rehearsed step; 7/8 and 15/16 with span 64, and
// no weighting below 4 ranks, left rank 0 the slowest once the collective
// no longer delayed the other ranks).  The whole blocks
// then run in periods of V = m*nranks - 1: position pos = j % V of block j
// goes to rank nranks-1 - pos % nranks (ranks in descending order, rank 0's
// last turn of the period left out); a rank's blocks keep raster order.
#ifndef VRT_DEAL_BLOCK
#define VRT_DEAL_BLOCK 4
#endif
#ifndef VRT_DEAL_WEIGHT
#define VRT_DEAL_WEIGHT 1
#endif
#ifndef VRT_DEAL_SPAN
#define VRT_DEAL_SPAN 48
#endif
struct TileDeal {
        int ntx, nty, nranks, G;
        int bx, by;  // whole blocks per block row / per block column
        int F;       // whole blocks
        int rw;      // width of the right strip (ntx - bx*G)
        int nA;      // tiles of the right strip
        int L;       // leftover tiles (right strip + bottom strip)
        int m, V;    // weighted deal: turns per period of ranks >= 1, period (V = 0: plain round robin)
};
__host__ __device__ inline TileDeal tile_deal(int ntx, int nty, int nranks)
{
        TileDeal d;
        d.ntx = ntx;
        d.nty = nty;
        d.nranks = nranks;
        d.G = nranks > 1 ? VRT_DEAL_BLOCK : 1;  // one rank: raster order
        d.bx = ntx / d.G;
        d.by = nty / d.G;
        d.F = d.bx * d.by;
        d.rw = ntx - d.bx * d.G;
        d.nA = d.by * d.G * d.rw;
        d.L = ntx * nty - d.F * d.G * d.G;
        d.m = VRT_DEAL_WEIGHT && nranks >= 2 ? (VRT_DEAL_SPAN / nranks > 2 ? VRT_DEAL_SPAN / nranks : 2) : 0;
        d.V = d.m ? d.m * nranks - 1 : 0;
        return d;
}
// blocks of rank r in one period of the weighted deal
__host__ __device__ inline int deal_turns(const TileDeal &d, int r)
{
        return r == 0 ? d.m - 1 : d.m;
}
// whole blocks of rank r, and the first leftover index it owns
__host__ __device__ inline int deal_blocks(const TileDeal &d, int r)
{
        if (d.V) {
                const int q = d.nranks - 1 - r, rem = d.F % d.V;
                return (d.F / d.V) * deal_turns(d, r) + (rem > q ? (rem - 1 - q) / d.nranks + 1 : 0);
        }
        return r < d.F ? (d.F - r + d.nranks - 1) / d.nranks : 0;
}
__host__ __device__ inline int deal_l0(const TileDeal &d, int r)
{
        return ((r - d.F) % d.nranks + d.nranks) % d.nranks;
}
// tiles of rank r
__host__ __device__ inline int deal_count(const TileDeal &d, int r)
{
        const int l0 = deal_l0(d, r);
        return deal_blocks(d, r) * d.G * d.G + (l0 < d.L ? (d.L - l0 + d.nranks - 1) / d.nranks : 0);
}
// rank r's k-th tile -> (tx, ty)
__host__ __device__ inline void deal_tile(const TileDeal &d, int r, int k, int &tx, int &ty)
{
        if (d.nranks == 1) {  // raster order (the general form with G = 1, fewer divisions)
                tx = k % d.ntx;
                ty = k / d.ntx;
                return;
        }
        const int G2 = d.G * d.G, nb = deal_blocks(d, r);
        if (k < nb * G2) {
                const int kb = k / G2, w = k % G2;
                int j = r + kb * d.nranks;
                if (d.V) {
                        const int c = deal_turns(d, r);
                        j = (kb / c) * d.V + (d.nranks - 1 - r) + (kb % c) * d.nranks;
                }
                tx = (j % d.bx) * d.G + w % d.G;
                ty = (j / d.bx) * d.G + w / d.G;
                return;
        }
        int li = deal_l0(d, r) + (k - nb * G2) * d.nranks;
        if (li < d.nA) {
                ty = li / d.rw;
                tx = d.bx * d.G + li % d.rw;
        } else {
                li -= d.nA;
                ty = d.by * d.G + li / d.ntx;
                tx = li % d.ntx;
        }
}
// tile (tx, ty) -> its rank r and index k there
__host__ __device__ inline void deal_slot(const TileDeal &d, int tx, int ty, int &r, int &k)
{
        if (tx < d.bx * d.G && ty < d.by * d.G) {
                const int j = (ty / d.G) * d.bx + tx / d.G, w = (ty % d.G) * d.G + tx % d.G;
                if (d.V) {
                        const int pos = j % d.V;
                        r = d.nranks - 1 - pos % d.nranks;
                        k = ((j / d.V) * deal_turns(d, r) + pos / d.nranks) * d.G * d.G + w;
                } else {
                        r = j % d.nranks;
                        k = (j / d.nranks) * d.G * d.G + w;
                }
                return;
        }
        const int li = ty < d.by * d.G ? ty * d.rw + (tx - d.bx * d.G) : d.nA + (ty - d.by * d.G) * d.ntx + tx;
        r = (d.F + li) % d.nranks;
        k = deal_blocks(d, r) * d.G * d.G + li / d.nranks;
}

// Camera + film constants for ray generation (T1), computed on the host.
struct CamParams {
        float s[3], u[3], nf[3], e[3];  // columns of C_
        float origin[3];                // point_transform(C_, {})
        float z;                        // -(film.h / (2*tanf(fov/2)))
        float tmin, tmax;               // near, far
        int32_t nx, ny;
};

// Per-sample outputs (device pointers, any may be null).
struct SampleOut {
        int32_t *hit;
        int32_t *tri;
        uint32_t *vox;
        float *rgb;
        uint32_t *cnt;
};

struct RenderParams {
        DevScene sc;
        CamParams cam;
        int32_t ntx, nty;      // 8x8 tiles in the render area
        int32_t rank, nranks;  // this rank's tiles: tile_deal / deal_tile
        int32_t tiles_this_rank;
        int32_t image_layout;  // 1: out is nx*ny*3 image; 0: packed tiles
        int32_t test_flags;    // vrt_set_test_flags (VRT_TEST_FORCE_DEFER)
        int32_t ty0;           // primary render: first tile row of the band rendered (the tile grid
                               // is rows [ty0, ty0 + nty) of the film; 0 = the whole film)
        float *out;
        SampleOut so;
        WorkQueue q;           // persistent launches only
        // nranks > 1: this rank's tiles in deal order, tx | ty << 16 each
        // (k_deal_map, cached per scene), read with a scalar load instead of
        // tile_deal / deal_tile's divisions per unit; nullptr: computed
        const uint32_t *tile_xy;
        // one rank: ceil(2^40 / ntx), so a tile index k < 2^24 splits into
        // (k % ntx, k / ntx) with one multiply (rank_tile); 0: divide
        uint64_t ntx_magic;
};

// ---- full trace() -------------------------------------
// Per-node cone-tracing state (80 B): VoxelOctree::coverage and illum[6]
// (VRT/voxel_octree.h:64-70), indexed like NodeRec.
struct alignas(16) LMRec {
        float cov;
        float illum[18];
        float pad;
};
static_assert(sizeof(LMRec) == 80, "LMRec must be 80 B");

// Light pass (VRT/main.cc:79-97) over r's film: every sample of the
// canonical single-threaded order k (render_mt task t = tx*8+ty of
// ptx x pty pixels, row-major, samples 0..3) that hits takes the next slot
// j of a compact list (one atomic add per wave) and writes keys[j] = hit leaf
// << kbits | k, vals[j] = j and samp[6j..6j+5] = get_diffuse rgb, isect
// normal; *count ends as the number of hits.  Sorting the pairs by key puts
// each leaf's samples together in canonical order.
struct LightParams {
        RenderParams r;
        int32_t ptx, pty;
        int32_t kbits;       // bits of the canonical index k
        unsigned int *count;
        uint64_t *keys;
        uint32_t *vals;
        float *samp;
        unsigned int *tail_n;  // deferred samples (k_light_tail): count, then work unit << 6 | lane
        uint32_t *tail;
};

// Cone-tracing render (trace(), VRT/main.cc:10-30 + cone_trace,
// VRT/voxel_octree.cc:276-330).  split_up[e]: smallest float x in
// [2^e, 2^(e+1)) with (int)log2f(x) == e+1 under the host libm (the same
// log2f the oracle and the reference's float path call), +inf if none.
struct TraceParams {
        RenderParams r;
        const LMRec *lm;
        const float4 *cc;          // per node: box centre xyz, word a (cone descent)
        const uint32_t *lm_bad;    // != 0: some illum is not finite (exact slow path)
        const float4 *cells;       // per node: the cell (lo.xyz, hi.xyz) of the descent to it
        float mindist, maxdist;
        float split_up[64];
        // split_bound[k] (k = 1..63) = the largest cone diameter whose split
        // level (int)log2f(maxdist / diam) -- split_level_of(fl(maxdist /
        // diam)) -- is >= k (0 if none): the level is non-increasing in diam,
        // so it is the count of bounds >= diam, kept by a cursor as a cone's
        // diameter grows instead of a division per step
        float split_bound[64];
        // split path (rec != nullptr): per-sample records of the primary
        // pass (4 x float4: hit point | hit flag, normal, albedo or sky,
        // the hit leaf and -d), tiles_this_rank*256 slots, read by k_cones_film
        float4 *rec;
        // the primary pass's deferred samples (k_trace_prim_tail): count, slots
        unsigned int *tail_n;
        uint32_t *tail;
        // the cone march's step table (kConeSteps entries) and its length,
        // written by k_cone_steps (launched after k_trace_prim)
        float4 *steps;
        int *nsteps;
        int32_t build_steps;  // launch_trace_prim rebuilds the table (k_cone_steps)
};
// Capacity of TraceParams::steps.  A cone's distance grows by >= 11.5 % a
// step (diam >= 2 * aperture * dist), so even maxdist / mindist = 2^128
// takes < 820 steps; a longer sequence (not reachable for finite scenes)
// is flagged (-1) and the march computes its steps inline.
constexpr int kConeSteps = 1024;

// GPU octree build (vrt_build.hip): the host build's
// arrays, produced on `device` and copied back.
struct DeviceBuild {
        std::vector<NodeRec> nodes;        // content masks included
        std::vector<uint32_t> node_vox;
        std::vector<uint64_t> refs;        // sorted (leaf code << 32 | tri)
        std::vector<int64_t> level_begin;  // BFS level ranges (+ end)
        int64_t ninternal = 0;
        double device_ms = 0;              // descent + sorts + flatten + masks
};
hipError_t build_tree_device(int device, const float *pos, int ntri, const float root_mn[3],
                             const float root_mx[3], int max_depth, DeviceBuild *out, std::string *err);

// Host helpers shared by vrt_host.cpp and vrt_multi.cpp (hidden symbols).
// scene_replicate: src's host-side build uploaded to another device.
int scene_replicate(const vrt_scene *src, const vrt_scene_desc *d, int device, vrt_scene **out);
// memcpy of a large host range over up to 4 threads.
void par_memcpy(void *dst, const void *src, size_t bytes);
// the process-wide vrt_set_test_flags value
int test_flags();

// Kernel launchers (vrt_kernels.hip)
// Which primary-render kernel launch_render runs: the one-wave grid
// (k_render: instrumented, per-sample outputs, large-leaf scenes), the
// persistent kernel (k_render_p<false>) or the persistent fast-only kernel
// + its deferred-unit pass (k_render_p<true> + k_render_defer).  The
// persistent kinds take their units from p.q.
enum RenderKind { kRenderGrid = 0, kRenderPersist = 1, kRenderPersistFast = 2 };
RenderKind render_kind(const RenderParams &p, bool instrumented);
// upper bound on the camera rays of the film that fail the fast-only
// kernel's per-wave check (vrt_kernels.hip; cached for the last 32 cameras)
int64_t camera_defer_bound(const CamParams &c);
// *q_waves = the failing adds each slice counter receives (the waves
// launched that visit it), slice_units[x] = the units of slice x (all 0 when
// no work queue was used), for the queue bases
hipError_t launch_render(const RenderParams &p, bool instrumented,
                         hipStream_t st, int *q_waves, int slice_units[8]);
// resident blocks of the persistent render / secondary kernels on the
// current device
hipError_t persistent_blocks(int *render_blocks, int *sec_blocks);
bool secondary_uses_queue(const DevScene &sc);
hipError_t launch_ray_march(const DevScene &sc, const void *d_rays,
                            int64_t n, void *d_hits, hipStream_t st);
hipError_t launch_unpack(int nx, int ny, int ntx, int nty, int nranks,
                         int tiles_per_rank, const float *src, float *dst,
                         hipStream_t st);
hipError_t launch_pack_c(int nx, int ny, int rank, int nranks, int comps, const float *img, float *dst,
                         hipStream_t st);
hipError_t launch_unpack_c(int nx, int ny, int nranks, int tiles_per_rank, int comps, const float *src, float *dst,
                           hipStream_t st);
// A side stream of a compaction set and its fork / join events: the
// deferred pixels' exact walk (k_secondary_defer) runs there beside the
// streaming resume instead of after it on the launch's stream.
struct SideLaunch {
        hipStream_t st;
        hipEvent_t fork, join;
};
// q: the launch's work queue (persistent kernel) or nullptr (one wave per
// pixel); side: nullptr = every kernel on st
hipError_t launch_secondary(const RenderParams &rp, int spp, int rank,
                            int nranks, float res, float *prim, float *vis,
                            int32_t *s_hit, int32_t *s_tri, uint32_t *s_vox,
                            const WorkQueue *q, hipStream_t st, int *q_waves, int slice_units[8],
                            const SpillQueues *sq = nullptr, const SideLaunch *side = nullptr);
// the compaction settings of this build (VRT_SEC_SPILL*), cap left 0
SpillQueues spill_defaults();
// a path-selecting compile-time switch of the kernel build by name (false:
// unknown name) -- vrt_build_flag
bool build_flag(const char *name, int64_t *value);
hipError_t launch_light(const LightParams &p, hipStream_t st);
// out[k] = rank's k-th tile of the deal (deal_tile), tx | ty << 16, for k <
// deal_count (ntx, nty < 2^16)
hipError_t launch_deal_map(int ntx, int nty, int nranks, int rank, uint32_t *out, hipStream_t st);
hipError_t light_diag_copy(void *host, size_t bytes);  // VRT_LIGHT_DIAG builds
// samp: n x 6 floats followed by room for their sorted copy (n x 6);
// seg_start: max_seg entries (>= non-empty leaves), nseg zeroed (by
// launch_lm_leaves); seg_end: one entry per node (each hit leaf's run end is
// written)
hipError_t launch_lm_accum(int64_t n, const uint64_t *keys_sorted, const uint32_t *vals_sorted, int kbits,
                           const float *samp, uint32_t *seg_start, unsigned int *nseg,
                           int64_t max_seg, uint32_t *seg_end, LMRec *lm, hipStream_t st);
// every leaf's coverage and (zero) illum; also zeroes the light map's
// counters (the finiteness flag, the hit, deferred-sample and run counts) --
// the first kernel of a light-map build, so nothing is cleared by a memset
hipError_t launch_lm_leaves(const NodeRec *nodes, int64_t nnodes, LMRec *lm, uint32_t *bad, unsigned int *count,
                            unsigned int *tail_n, unsigned int *nseg, hipStream_t st);
hipError_t launch_lm_level(const NodeRec *nodes, int64_t begin, int64_t end, LMRec *lm, hipStream_t st);
hipError_t launch_trace(const TraceParams &p, hipStream_t st);
hipError_t launch_trace_prim(const TraceParams &p, hipStream_t st);
hipError_t launch_cones(const TraceParams &p, hipStream_t st);
// per-node cone-descent records and the light map's finiteness flag
hipError_t launch_lm_aux(const NodeRec *nodes, const LMRec *lm, int64_t n, float4 *cc, uint32_t *bad,
                         hipStream_t st);
// stable radix sort of (key, value) pairs on the low `bits` key bits
// (vrt_build.hip); temp == nullptr queries *temp_bytes
hipError_t sort_pairs_u64(void *temp, size_t *temp_bytes, const uint64_t *keys_in, uint64_t *keys_out,
                          const uint32_t *vals_in, uint32_t *vals_out, int64_t n, int bits, hipStream_t st);
hipError_t launch_rgbe(const float *img, int64_t npx, int comp, uint8_t *out, hipStream_t st);
hipError_t launch_selftest_order(const float *dist, const uint32_t *hm, int64_t n, uint32_t *out,
                                 const float *depth, const int32_t *len, int64_t m, int32_t stride,
                                 int32_t *argmin, hipStream_t st);
hipError_t launch_selftest(const double *mt_in, double *mt_out,
                           const float *sat_in, int32_t *sat_out, int64_t n,
                           hipStream_t st);

}  // namespace vrt
